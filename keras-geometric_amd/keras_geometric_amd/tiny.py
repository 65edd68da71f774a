"""Packed records of a schedule's tail of rows of degree <= 2.

The fused aggregate->transform launch (kgx_spmm_gemm_ex2) reads the rows of
degree <= 2 at the end of the degree-descending schedule (on R-MAT about
two thirds of all rows; the self loop alone is half) from one record each
instead of an item plus index and weight loads: {row, degree, col0, col1}
(col1 = col0 for degree 1, 0 and 0 for degree 0) and {w0, w1}.  Built once
per graph on the device (kgx_tiny_pack; the torch restatement below builds
the same records from host tensors and defines the layout the host tests
check) and cached on the graph.
Reference semantics are unchanged: the kernel folds exactly the row's CSR
edges in order (gcn_conv.py:233-272, aggregators.py:56-167).
"""

from __future__ import annotations

import os
from typing import Optional

import torch

TINY_MAX = 2       # the kernel gathers two edges per row
_MIN_ROWS = 4096   # below this the tail stays on the short-row kernel


def tiny_suffix_start(items: torch.Tensor) -> int:
    """Index of the first item of the suffix of unsplit rows of degree <= 2
    (device items: one kgx_schedule_suffixes pass)."""
    n = items.shape[0]
    if n == 0:
        return 0
    if items.is_cuda:
        from .graph import schedule_suffixes

        return schedule_suffixes(items, TINY_MAX, TINY_MAX)[1]
    lens = items[:, 2] - items[:, 1]
    big = (lens > TINY_MAX) | (items[:, 3] >= 0)
    nz = torch.nonzero(big)
    return int(nz[-1]) + 1 if nz.numel() else 0


def pack_numel(n: int, n2: int) -> int:
    """int32 entries of the packed tail of n rows (n2 of them of degree 2)."""
    return 4 * n


def records(pack: torch.Tensor, tw: Optional[torch.Tensor], n: int, n2: int):
    """The packed tail as {row, degree, col0, col1} [n, 4] and {w0, w1} [n, 2]
    (or None) per row: what tests and tools compare."""
    return pack[:n].long(), (tw[:n] if tw is not None else None)


def _tiny_pack_device(g, its: torch.Tensor, start: int, n: int):
    """The records of items [start, start + n) in one kgx_tiny_pack pass (the
    layout of the host restatement in tiny_pack below, bit for bit)."""
    import ctypes

    from . import _native as nat

    dev = its.device
    pack = torch.empty((n, 4), dtype=torch.int32, device=dev)
    w = getattr(g, "w", None)
    tw = torch.empty((n, 2), dtype=torch.float32, device=dev) if w is not None else None
    ws = torch.empty(16, dtype=torch.uint8, device=dev)
    out = (ctypes.c_int64 * 2)()
    nat.check(nat.lib().kgx_tiny_pack(nat.ptr(its.contiguous()), start, n, nat.ptr(g.col), nat.ptr(w),
                                      int(g.col.numel()), nat.ptr(pack), nat.ptr(tw), nat.ptr(ws), out,
                                      nat.stream(dev)), "kgx_tiny_pack")
    n2, last2 = int(out[0]), int(out[1])
    if n2 and last2 != n2:  # not degree-descending: every record takes the two-edge kernel
        n2 = n
    return pack, tw, start, n2


def tiny_pack(g, refresh: bool = False) -> tuple[Optional[torch.Tensor], Optional[torch.Tensor], int, int]:
    """(pack [n, 4] int32, weights [n, 2] float32 or None, n_short_end, n_deg2)
    for graph g's schedule, or (None, None, -1, 0) when the tail is too short
    or disabled (KGX_TINY=0).  The first n_deg2 records have degree 2 (the
    kernel gathers one edge per row for the rest).  Cached on g; built when
    the schedule is (graph._build_schedule, refresh=True), where the graph
    build syncs anyway, so a fused launch never syncs and can be captured
    into a HIP graph whatever ran on the graph first."""
    cached = getattr(g, "_kgx_tiny", None)
    w_now = getattr(g, "w", None)
    # the records carry the edge weights: a weight tensor assigned after the
    # schedule was built (sharded / transposed graphs) makes them stale
    if cached is not None and not refresh and getattr(g, "_kgx_tiny_w", None) is w_now:
        return cached
    res = (None, None, -1, 0)
    items = getattr(g, "items", None)
    if items is not None and os.environ.get("KGX_TINY", "1") not in ("0", "false", "False"):
        n_items = int(getattr(g, "n_items", items.shape[0]))
        its = items[:n_items]
        start = tiny_suffix_start(its)
        n_long = getattr(g, "n_long", -1)
        start = max(start, n_long if 0 <= n_long <= n_items else 0)
        if n_items - start >= _MIN_ROWS and its.is_cuda and g.col.numel() > 0:
            res = _tiny_pack_device(g, its, start, n_items - start)
        elif n_items - start >= _MIN_ROWS:
            t = its[start:]
            beg = t[:, 1].long()
            deg = (t[:, 2] - t[:, 1]).long()
            last = max(int(g.col.numel()) - 1, 0)
            i0 = beg.clamp(max=last)
            i1 = (beg + (deg > 1).long()).clamp(max=last)
            if g.col.numel() == 0:  # no edges: no source row to gather; the short-row kernel masks them all
                res = (None, None, -1, 0)
                g._kgx_tiny, g._kgx_tiny_w = res, w_now
                return res
            c0 = torch.where(deg > 0, g.col[i0].long(), torch.zeros_like(deg))
            c1 = torch.where(deg > 0, g.col[i1].long(), torch.zeros_like(deg))
            pack = torch.stack([t[:, 0].long(), deg, c0, c1], 1).to(torch.int32).contiguous()
            tw = None
            if getattr(g, "w", None) is not None:
                w0 = torch.where(deg > 0, g.w[i0], torch.zeros_like(g.w[i0]))
                w1 = torch.where(deg > 1, g.w[i1], torch.zeros_like(g.w[i1]))
                tw = torch.stack([w0, w1], 1).to(torch.float32).contiguous()
            # degree-descending schedule: the degree-2 rows come first; if not
            # (another item order), every record takes the two-edge kernel
            n2 = int((deg == 2).sum())
            if n2 and not bool((deg[:n2] == 2).all()):
                n2 = pack.shape[0]
            res = (pack, tw, start, n2)
    try:
        g._kgx_tiny = res
        g._kgx_tiny_w = w_now
    except AttributeError:
        pass
    return res
