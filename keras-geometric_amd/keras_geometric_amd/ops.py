"""PyTorch-ROCm operator registration of the kgx C-ABI (torch.ops.kgx.*).

Each op is a `torch.library.custom_op` whose implementation calls straight into
libkgx.so on torch's current HIP stream, with a fake (meta) kernel so that
torch.compile / symbolic tracing sees shapes without running the GPU.

  kgx::spmm   fused gather -> message -> segment {sum,mean,max,min,std} -> epilogue
  kgx::gatv2  fused GATv2 attention aggregation
  kgx::gather_rows, kgx::scatter_f32   row movement helpers
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

from . import _native as nat
from .graph import CSRGraph


def _f32c(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if t is None:
        return None
    if t.dtype != torch.float32:
        raise TypeError(f"kgx kernels compute in fp32; got {t.dtype}")
    return t.contiguous()


_EXACT_DYN = __import__("os").environ.get("KGX_EXACT_DYN", "1") != "0"


@torch.library.custom_op("kgx::spmm", mutates_args=())
def spmm(
    table: torch.Tensor,
    rowptr: torch.Tensor,
    rows: torch.Tensor,
    items: Optional[torch.Tensor],
    split: Optional[torch.Tensor],
    idx: torch.Tensor,
    w: Optional[torch.Tensor],
    n_slots: int,
    reduce: int,
    epilogue: int,
    bias: Optional[torch.Tensor],
    xroot: Optional[torch.Tensor],
    gin_scale: float,
    drop_key: Optional[torch.Tensor] = None,
    drop_p: float = 0.0,
    drop_seed: int = 0,
    n_long: int = -1,
) -> torch.Tensor:
    table = _f32c(table)
    w, bias, xroot = _f32c(w), _f32c(bias), _f32c(xroot)
    dev = nat.require_device(table, rowptr, rows, idx, w, bias, xroot, items, split)
    n_dst = rowptr.numel() - 1
    F = table.shape[1]
    out = torch.empty((n_dst, F), dtype=torch.float32, device=dev)
    if n_dst == 0 or F == 0:
        return out
    n_items = 0 if items is None else items.shape[0]
    n_split = 0 if split is None else split.shape[0]
    partials = None
    if items is not None and n_split > 0 and reduce != nat.STD:
        partials = torch.empty((n_slots, F), dtype=torch.float32, device=dev)
    if items is not None:  # EXACT mode (no items): n_long names the short suffix of the row list (or -1)
        n_long = n_items if n_long < 0 or n_long > n_items else n_long
    # EXACT mode: the hub-row kernel hands its items out dynamically (KGX_EXACT_DYN=0: static, A/B only)
    counters = (torch.zeros(2, dtype=torch.int32, device=dev)
                if items is None and reduce != nat.STD and _EXACT_DYN else None)
    nat.check(
        nat.lib().kgx_spmm_ex2(
            reduce, epilogue, nat.ptr(rowptr), nat.ptr(rows), n_dst,
            nat.ptr(items), n_items, n_long, nat.ptr(split), n_split,
            nat.ptr(idx), nat.ptr(w), nat.ptr(table), table.stride(0), None, 0, F,
            nat.ptr(out), out.stride(0),
            nat.ptr(bias), nat.ptr(xroot), xroot.stride(0) if xroot is not None else 0, float(gin_scale),
            nat.ptr(drop_key) if drop_p > 0 else None, float(drop_p), int(drop_seed) & (2**64 - 1),
            nat.ptr(partials), nat.ptr(counters), nat.stream(dev),
        ),
        "kgx_spmm",
    )
    return out


@spmm.register_fake
def _spmm_fake(table, rowptr, rows, items, split, idx, w, n_slots, reduce, epilogue, bias, xroot, gin_scale,
               drop_key=None, drop_p=0.0, drop_seed=0, n_long=-1):
    return table.new_empty((rowptr.shape[0] - 1, table.shape[1]))


@torch.library.custom_op("kgx::spmm_acc_", mutates_args=("out",))
def spmm_acc_(
    out: torch.Tensor,
    table: torch.Tensor,
    rowptr: torch.Tensor,
    rows: torch.Tensor,
    items: Optional[torch.Tensor],
    split: Optional[torch.Tensor],
    idx: torch.Tensor,
    w: Optional[torch.Tensor],
    n_slots: int,
    n_long: int = -1,
    epilogue: int = 4,
    bias: Optional[torch.Tensor] = None,
    xroot: Optional[torch.Tensor] = None,
    gin_scale: float = 1.0,
    table2: Optional[torch.Tensor] = None,
) -> None:
    """out[i] += SUM_{e in row i} table[idx[e]] (* w[e]) in place (KGX_EPI_ACCUM,
    the default epilogue); any other epilogue overwrites the scheduled rows of
    out (and leaves the rest untouched).  table2: sources >= table.shape[0]
    are rows of table2 (kgx_spmm_ex2)."""
    table, w, bias, xroot, table2 = _f32c(table), _f32c(w), _f32c(bias), _f32c(xroot), _f32c(table2)
    dev = nat.require_device(out, table, rowptr, rows, idx, w, items, split, bias, xroot, table2)
    if table2 is not None and (table2.dim() != 2 or table2.shape[1] != table.shape[1]
                               or (table2.shape[0] and table2.stride(0) != table.stride(0))):
        raise ValueError("spmm_acc_: table2 must have table's row width and leading dimension")
    n_dst = rowptr.numel() - 1
    F = table.shape[1]
    if out.dtype != torch.float32 or out.shape != (n_dst, F) or out.stride(1) != 1:
        raise ValueError(f"spmm_acc_: out must be float32 [{n_dst}, {F}] with unit column stride")
    if n_dst == 0 or F == 0:
        return
    n_items = 0 if items is None else items.shape[0]
    n_split = 0 if split is None else split.shape[0]
    partials = None
    if items is not None and n_split > 0:
        partials = torch.empty((n_slots, F), dtype=torch.float32, device=dev)
    n_long = n_items if n_long < 0 or n_long > n_items else n_long
    nat.check(
        nat.lib().kgx_spmm_ex2(
            nat.SUM, int(epilogue), nat.ptr(rowptr), nat.ptr(rows), n_dst,
            nat.ptr(items), n_items, n_long, nat.ptr(split), n_split,
            nat.ptr(idx), nat.ptr(w), nat.ptr(table), table.stride(0), nat.ptr(table2),
            table.shape[0] if table2 is not None else 0, F,
            nat.ptr(out), out.stride(0), nat.ptr(bias), nat.ptr(xroot), xroot.stride(0) if xroot is not None else 0,
            float(gin_scale), None, 0.0, 0, nat.ptr(partials), None, nat.stream(dev),
        ),
        "kgx_spmm",
    )


@spmm_acc_.register_fake
def _spmm_acc_fake(out, table, rowptr, rows, items, split, idx, w, n_slots, n_long=-1, epilogue=4, bias=None,
                   xroot=None, gin_scale=1.0, table2=None):
    return None


def aggregate_accumulate(g: CSRGraph, table: torch.Tensor, out: torch.Tensor, *, weighted: bool = False,
                         epilogue: int = nat.EPI_ACCUM, bias: torch.Tensor | None = None,
                         xroot: torch.Tensor | None = None, gin_scale: float = 1.0,
                         table2: torch.Tensor | None = None) -> torch.Tensor:
    """out += (weighted) row sums of table rows over g, in place; forward only.
    Meant for accumulate-only graphs (graph.split_by_part), whose schedules skip
    the rows they add nothing to.  Another epilogue (NONE / BIAS / GIN)
    overwrites g's scheduled rows of out instead; table2 = second table for
    sources >= table.shape[0] (the sharded layers' merged halo pass)."""
    if _needs_grad(table, out, table2):
        raise NotImplementedError("aggregate_accumulate is a forward-only (no_grad) path")
    items, _, split, _, n_slots = g.work(False)
    w = g.w if weighted else None
    if weighted and w is None:
        raise ValueError("graph was built without edge weights")
    _timed(lambda: torch.ops.kgx.spmm_acc_(out, table, g.rowptr, g.rows, items, split, g.col, w, n_slots,
                                           g.n_long if items is not None else -1, int(epilogue), bias, xroot,
                                           float(gin_scale), table2))
    return out


# Launch hint (results unchanged): while set, fused launches leave 1/8 of the
# block slots free for a concurrent collective (distributed.py's own-source pass).
# Per host thread: ranks driven by threads of one process (tests, rehearsals)
# each enter and leave their own passes' contexts; a process-wide flag was left
# set by interleaved exits.
_SHARE = threading.local()


def _share_gpu() -> bool:
    return getattr(_SHARE, "on", False)


class sharing_gpu:
    def __enter__(self):
        self._old = _share_gpu()
        _SHARE.on = True

    def __exit__(self, *exc):
        _SHARE.on = self._old


_NOSPLIT = threading.local()


class _unsplit:
    """CU-split launches off inside (per host thread): the training backward's
    transposed pass.  There the split measured slower -- NS training step 21.40-21.62
    ms split against 20.69-20.79 one-stream, the dx pass 9.12-9.18 against 8.79-8.82
    (profiles/r06/train/split_ab/) -- while the inference forward gains from it.
    KGX_BWD_CU_SPLIT=1 keeps the split (measurement)."""

    def __enter__(self):
        self._old = getattr(_NOSPLIT, "on", False)
        _NOSPLIT.on = os.environ.get("KGX_BWD_CU_SPLIT") != "1"

    def __exit__(self, *exc):
        _NOSPLIT.on = self._old


def _tiny_abi(items, n_items, n_long, tpack, tw, n_short_end, n_tiny2):
    """(n_short_end, tpack, tw, n_tiny2) arguments of kgx_spmm_gemm_ex2."""
    if items is None or tpack is None or not (n_long <= n_short_end <= n_items):
        return n_items, None, None, 0
    from . import tiny

    if tpack.numel() != tiny.pack_numel(n_items - n_short_end, n_tiny2):
        raise ValueError(f"tiny records: {tpack.numel()} ints for a tail of {n_items - n_short_end} rows "
                         f"({n_tiny2} of degree 2) -- stale or foreign pack (tiny.py)")
    return n_short_end, tpack, tw, n_tiny2


def _x2_args(x, x2):
    """(x2 pointer, n_x1) of kgx_spmm_gemm_ex3: sources >= x.shape[0] are rows of x2."""
    if x2 is None:
        return None, 0
    if x2.dim() != 2 or x2.shape[1] != x.shape[1] or (x2.shape[0] and x2.stride(0) != x.stride(0)):
        raise ValueError(f"spmm_gemm: x2 {tuple(x2.shape)} must have x's row width and leading dimension")
    return nat.ptr(x2), x.shape[0]


F256 = 256  # F_in of kgx_spmm_gemm_f256 (GINConv C4: 256 -> 256)
# layers take the 256-wide fused kernels by default: at C4 they beat the unfused
# pair (kgx_spmm + kgx_dense), 22.0 vs 24.5 ms; KGX_FUSED256=0 turns them off
_F256_DEFAULT = "1"


def _f256_call(reduce, rowptr, rows, n_dst, items, n_items, split, n_split, idx, w, x, x2, W, bias, flags, gin_scale,
               out, partials, agg, dev, tpack=None, tw=None, n_short_end=-1, n_long=-1):
    """kgx_spmm_gemm_f256_ex: the 256-wide fused kernels (main + the degree <= 2
    tail from the packed records); x2: second feature table for sources >=
    x.shape[0] (the sharded GIN layer's merged halo pass; sum only)."""
    n_se, tpack, tw, _ = _tiny_abi(items, n_items, 0, tpack, tw if w is not None else None, n_short_end, 0)
    x2p, n_x1 = _x2_args(x, x2)
    nat.check(
        nat.lib().kgx_spmm_gemm_f256_ex(
            reduce, nat.ptr(rowptr), nat.ptr(rows), n_dst, nat.ptr(items), n_items,
            n_long if items is not None and 0 <= n_long <= n_se else -1, n_se, nat.ptr(tpack), nat.ptr(tw),
            nat.ptr(split), n_split,
            nat.ptr(idx), nat.ptr(w), nat.ptr(x), x.stride(0), x2p, n_x1, x.shape[1], nat.ptr(W), W.shape[1],
            nat.ptr(bias),
            flags, float(gin_scale), nat.ptr(out), out.stride(0), nat.ptr(partials),
            nat.ptr(agg), agg.stride(0) if agg is not None else 0, nat.stream(dev),
        ),
        "kgx_spmm_gemm_f256",
    )


def _f256_cu_split(n_edges: int, n_tiny: int) -> bool:
    """Whether a 256-wide launch runs its degree <= 2 tail on 64 CUs beside the
    rest on the other 192 (KGX_FUSED_CU_SPLIT): when the modelled split time,
    max(head on 192 CUs, tail on 64) plus the measured 10 % interference, beats
    the one-stream sum by 3 %.  Per-unit costs from the C4 graph
    (profiles/r05/c4_cupart*.json: head 15.7 ms / 97M edges on 256 CUs, 17.9 on
    192; tail 5.63 ms / 7.46M rows on 256, 16.0 on 64).  Large launches only
    (>= 1M tail rows): the fork / join and the smaller grids cost more than they
    hide on small ones.  KGX_F256_CU_SPLIT: unset = this model (8 of every 32
    CUs for the tail), "0" = never, t > 0 = always, with t of every 32 CUs."""
    per32 = _per32_override("KGX_F256_CU_SPLIT")
    if per32 is not None:
        return n_tiny > 0 and per32 > 0
    if n_tiny < 1_000_000:
        return False
    head_e = max(n_edges - 2 * n_tiny, 0)
    t_seq = 1.62e-7 * head_e + 7.55e-7 * n_tiny
    t_split = 1.1 * max(1.85e-7 * head_e, 2.14e-6 * n_tiny)
    return t_split < 0.97 * t_seq


CU_SPLIT_LAUNCHES = 0  # launches that ran CU-split (KGX_FUSED_CU_SPLIT): bench.py reports it


def _per32_override(name: str):
    """A KGX_*_CU_SPLIT override parsed as the library parses it: None when
    unset, else the tail CUs per 32 -- an integer in 1..31, anything else 0
    (the library then runs unsplit)."""
    env = os.environ.get(name)
    if env is None:
        return None
    try:
        v = int(env.strip())
    except ValueError:
        return 0
    return v if 0 < v < 32 else 0


_DEVICE_SPLIT_OK: dict = {}


def _device_split_ok(dev: torch.device | None) -> bool:
    """The device has the layout the CU split was validated on (kgx_cu_split_supported:
    gfx950, 256 CUs, 8 XCDs); else its launches run unsplit and are not counted."""
    if dev is None:
        return True
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    ok = _DEVICE_SPLIT_OK.get(idx)
    if ok is None:
        ok = _DEVICE_SPLIT_OK[idx] = nat.lib().kgx_cu_split_supported(int(idx)) == 1
    return ok


def _split_allowed(dev: torch.device | None = None) -> bool:
    """CU-split launches stay off while a launch shares the GPU with an exchange
    (sharing_gpu: the sharded layers' passes beside RCCL and the packing), unless
    KGX_CU_SPLIT_SHARED=1 (measurement); off on a device whose layout is not the
    validated one, and for a tensor on another device than the current one (the
    library would run it unsplit)."""
    if _share_gpu() and os.environ.get("KGX_CU_SPLIT_SHARED") != "1":
        return False
    if getattr(_NOSPLIT, "on", False):
        return False
    if dev is not None and dev.type == "cuda" and dev.index is not None and dev.index != torch.cuda.current_device():
        return False
    return _device_split_ok(dev)


def _count_cu_split() -> None:
    global CU_SPLIT_LAUNCHES
    CU_SPLIT_LAUNCHES += 1


def _fused_cu_split(n_edges: int, n_tail_rows: int) -> bool:
    """Whether a 128-wide fused launch runs its short-row and tiny-record
    launches on 64 CUs beside spmm_gemm_kernel on the other 192
    (KGX_FUSED_CU_SPLIT): large schedules with a large tail only -- fitted on
    the north-star graph (profiles/r05/ns_cusplit*/: 8.62-8.69 against
    8.92-8.94 ms one-stream; main 8.29 ms on 192 CUs beside the tails' 8.61 on
    64).  KGX_FUSED_CU_SPLIT: unset = this rule, "0" = never, t > 0 = always,
    with t of every 32 CUs (only 8 measured well: see DESIGN.md §4)."""
    per32 = _per32_override("KGX_FUSED_CU_SPLIT")
    if per32 is not None:
        return n_tail_rows > 0 and per32 > 0
    return n_edges >= 50_000_000 and n_tail_rows >= 2_000_000


def _partial_width(x: torch.Tensor) -> int:
    """Floats per hub-chunk partial: the 256-wide kernels 256, kgx_spmm_gemm 128 (any F_in <= 128)."""
    return F256 if x.shape[1] == F256 else 128


def _spmm_gemm_impl(x, rowptr, rows, items, split, idx, w, n_slots, reduce, W, bias, pre_gin, gin_scale, save_agg,
                    relu=False, n_long=-1, tpack=None, tw=None, n_short_end=-1, n_tiny2=0, x2=None):
    x, w, W, bias, x2 = _f32c(x), _f32c(w), _f32c(W), _f32c(bias), _f32c(x2)
    dev = nat.require_device(x, rowptr, rows, idx, w, W, bias, items, split, x2)
    n_dst = rowptr.numel() - 1
    F_out = W.shape[1]
    out = torch.empty((n_dst, F_out), dtype=torch.float32, device=dev)
    agg = torch.empty((n_dst if save_agg else 0, x.shape[1]), dtype=torch.float32, device=dev)
    if n_dst == 0:
        return out, agg
    n_items = 0 if items is None else items.shape[0]
    n_split = 0 if split is None else split.shape[0]
    partials = None
    if items is not None and n_split > 0:
        partials = torch.empty((n_slots, _partial_width(x)), dtype=torch.float32, device=dev)
    flags = int(pre_gin) | (nat.FUSED_SHARE_GPU if _share_gpu() else 0) | (nat.FUSED_RELU if relu else 0)
    if x.shape[1] == F256:
        if tpack is not None and items is not None and not save_agg and _split_allowed(dev) and \
                _f256_cu_split(idx.numel(), n_items - (n_short_end if n_short_end >= 0 else n_items)):
            flags |= nat.FUSED_CU_SPLIT
            _count_cu_split()
        _f256_call(reduce, rowptr, rows, n_dst, items, n_items, split, n_split, idx, w, x, x2, W, bias, flags,
                   gin_scale, out, partials, agg if save_agg else None, dev, tpack, tw, n_short_end, n_long)
        return out, agg
    n_long = n_items if n_long < 0 or n_long > n_items else n_long
    n_se, tpack, tw, n_tiny2 = _tiny_abi(items, n_items, n_long, tpack, tw if w is not None else None, n_short_end,
                                         n_tiny2)
    # not for the training forward's saved-aggregate launch: its tail launches also store the
    # aggregated rows (the EXTRA instantiations), and split it measured slower (NS training step
    # 23.1 -> 25.0 ms, profiles/r05/train/)
    if items is not None and not save_agg and _split_allowed(dev) and _fused_cu_split(idx.numel(), n_items - n_long):
        flags |= nat.FUSED_CU_SPLIT
        _count_cu_split()
    x2p, n_x1 = _x2_args(x, x2)
    nat.check(
        nat.lib().kgx_spmm_gemm_ex3(
            reduce, nat.ptr(rowptr), nat.ptr(rows), n_dst, nat.ptr(items), n_items, n_long, n_se, nat.ptr(tpack),
            nat.ptr(tw), n_tiny2, nat.ptr(split), n_split,
            nat.ptr(idx), nat.ptr(w), nat.ptr(x), x.stride(0), x2p, n_x1, x.shape[1], nat.ptr(W), F_out, nat.ptr(bias),
            flags, float(gin_scale), nat.ptr(out), out.stride(0),
            nat.ptr(partials),
            nat.ptr(agg) if save_agg else None, agg.stride(0) if save_agg else 0, nat.stream(dev),
        ),
        "kgx_spmm_gemm",
    )
    return out, agg


@torch.library.custom_op("kgx::spmm_gemm", mutates_args=())
def spmm_gemm(
    x: torch.Tensor,
    rowptr: torch.Tensor,
    rows: torch.Tensor,
    items: Optional[torch.Tensor],
    split: Optional[torch.Tensor],
    idx: torch.Tensor,
    w: Optional[torch.Tensor],
    n_slots: int,
    reduce: int,
    W: torch.Tensor,
    bias: Optional[torch.Tensor],
    pre_gin: bool,
    gin_scale: float,
    relu: bool = False,
    n_long: int = -1,
    tpack: Optional[torch.Tensor] = None,
    tw: Optional[torch.Tensor] = None,
    n_short_end: int = -1,
    n_tiny2: int = 0,
    x2: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """x2 (two-table gathers, kgx_spmm_gemm_ex3): sources >= x.shape[0] are rows of x2."""
    return _spmm_gemm_impl(x, rowptr, rows, items, split, idx, w, n_slots, reduce, W, bias, pre_gin, gin_scale,
                           False, relu, n_long, tpack, tw, n_short_end, n_tiny2, x2)[0]


@spmm_gemm.register_fake
def _spmm_gemm_fake(x, rowptr, rows, items, split, idx, w, n_slots, reduce, W, bias, pre_gin, gin_scale, relu=False,
                    n_long=-1, tpack=None, tw=None, n_short_end=-1, n_tiny2=0, x2=None):
    return x.new_empty((rowptr.shape[0] - 1, W.shape[1]))


@torch.library.custom_op("kgx::spmm_gemm_save", mutates_args=())
def spmm_gemm_save(
    x: torch.Tensor,
    rowptr: torch.Tensor,
    rows: torch.Tensor,
    items: Optional[torch.Tensor],
    split: Optional[torch.Tensor],
    idx: torch.Tensor,
    w: Optional[torch.Tensor],
    n_slots: int,
    reduce: int,
    W: torch.Tensor,
    bias: Optional[torch.Tensor],
    pre_gin: bool,
    gin_scale: float,
    n_long: int = -1,
    tpack: Optional[torch.Tensor] = None,
    tw: Optional[torch.Tensor] = None,
    n_short_end: int = -1,
    n_tiny2: int = 0,
) -> tuple[torch.Tensor, torch.Tensor]:
    """kgx::spmm_gemm that also returns the aggregated rows before the transform."""
    return _spmm_gemm_impl(x, rowptr, rows, items, split, idx, w, n_slots, reduce, W, bias, pre_gin, gin_scale, True,
                           False, n_long, tpack, tw, n_short_end, n_tiny2)


@spmm_gemm_save.register_fake
def _spmm_gemm_save_fake(x, rowptr, rows, items, split, idx, w, n_slots, reduce, W, bias, pre_gin, gin_scale,
                         n_long=-1, tpack=None, tw=None, n_short_end=-1, n_tiny2=0):
    n = rowptr.shape[0] - 1
    return x.new_empty((n, W.shape[1])), x.new_empty((n, x.shape[1]))


@torch.library.custom_op("kgx::spmm_gemm_acc_", mutates_args=("out",))
def spmm_gemm_acc_(
    out: torch.Tensor,
    x: torch.Tensor,
    rowptr: torch.Tensor,
    rows: torch.Tensor,
    items: Optional[torch.Tensor],
    split: Optional[torch.Tensor],
    idx: torch.Tensor,
    w: Optional[torch.Tensor],
    n_slots: int,
    reduce: int,
    W: torch.Tensor,
    bias: Optional[torch.Tensor],
    n_long: int = -1,
    tpack: Optional[torch.Tensor] = None,
    tw: Optional[torch.Tensor] = None,
    n_short_end: int = -1,
    n_tiny2: int = 0,
    x2: Optional[torch.Tensor] = None,
    accumulate: bool = True,
    flags: int = 0,
    gin_scale: float = 1.0,
) -> None:
    """out += bias + REDUCE(...) @ W (KGX_FUSED_ACCUMULATE), in place; with
    accumulate=False the scheduled rows of out are overwritten instead (and the
    rest left untouched): two launches over disjoint row sets fill one output.
    flags: KGX_FUSED_PRE_GIN / KGX_FUSED_RELU for an overwriting launch (the
    sharded GIN layer's passes: (1+eps) x_i + aggr -> Dense)."""
    x, w, W, bias, x2 = _f32c(x), _f32c(w), _f32c(W), _f32c(bias), _f32c(x2)
    dev = nat.require_device(out, x, rowptr, rows, idx, w, W, bias, items, split, x2)
    n_dst = rowptr.numel() - 1
    if out.dtype != torch.float32 or out.shape != (n_dst, W.shape[1]) or out.stride(1) != 1:
        raise ValueError(f"spmm_gemm_acc_: out must be float32 [{n_dst}, {W.shape[1]}] with unit column stride")
    if n_dst == 0:
        return
    n_items = 0 if items is None else items.shape[0]
    n_split = 0 if split is None else split.shape[0]
    partials = None
    if items is not None and n_split > 0:
        partials = torch.empty((n_slots, _partial_width(x)), dtype=torch.float32, device=dev)
    if x.shape[1] == F256:
        if tpack is not None and items is not None and _split_allowed(dev) and \
                _f256_cu_split(idx.numel(), n_items - (n_short_end if n_short_end >= 0 else n_items)):
            flags |= nat.FUSED_CU_SPLIT
            _count_cu_split()
        _f256_call(reduce, rowptr, rows, n_dst, items, n_items, split, n_split, idx, w, x, x2, W, bias,
                   (nat.FUSED_ACCUMULATE if accumulate else 0) | (nat.FUSED_SHARE_GPU if _share_gpu() else 0) | flags,
                   gin_scale, out, partials, None, dev, tpack, tw, n_short_end, n_long)
        return
    n_long = n_items if n_long < 0 or n_long > n_items else n_long
    n_se, tpack, tw, n_tiny2 = _tiny_abi(items, n_items, n_long, tpack, tw if w is not None else None, n_short_end,
                                         n_tiny2)
    if items is not None and _split_allowed(dev) and _fused_cu_split(idx.numel(), n_items - n_long):
        flags |= nat.FUSED_CU_SPLIT
        _count_cu_split()
    x2p, n_x1 = _x2_args(x, x2)
    nat.check(
        nat.lib().kgx_spmm_gemm_ex3(
            reduce, nat.ptr(rowptr), nat.ptr(rows), n_dst, nat.ptr(items), n_items, n_long, n_se, nat.ptr(tpack),
            nat.ptr(tw), n_tiny2, nat.ptr(split), n_split,
            nat.ptr(idx), nat.ptr(w), nat.ptr(x), x.stride(0), x2p, n_x1, x.shape[1], nat.ptr(W), W.shape[1],
            nat.ptr(bias), (nat.FUSED_ACCUMULATE if accumulate else 0) | (nat.FUSED_SHARE_GPU if _share_gpu() else 0) | flags,
            float(gin_scale), nat.ptr(out), out.stride(0), nat.ptr(partials), None, 0, nat.stream(dev),
        ),
        "kgx_spmm_gemm",
    )


@spmm_gemm_acc_.register_fake
def _spmm_gemm_acc_fake(out, x, rowptr, rows, items, split, idx, w, n_slots, reduce, W, bias, n_long=-1, tpack=None,
                        tw=None, n_short_end=-1, n_tiny2=0, x2=None, accumulate=True, flags=0, gin_scale=1.0):
    return None


def fused_transform_supported(f_in: int, f_out: int, two_table: bool = False) -> bool:
    """Shapes kgx_spmm_gemm (F_in 128) and kgx_spmm_gemm_f256 (F_in 256)
    implement, with one feature table or two (two_table: the sharded layers'
    merged halo passes, sum only; aggregate-then-transform is also only worth
    it when F_in <= F_out)."""
    import os

    if os.environ.get("KGX_FUSED", "1") in ("0", "false", "False"):
        return False
    if f_in == F256:
        return f_out == F256 and os.environ.get("KGX_FUSED256", _F256_DEFAULT) not in ("0", "false", "False")
    return f_in == 128 and f_out % 16 == 0 and 0 < f_out <= 128 and f_in <= f_out


def fused_sage_supported(f_in: int, f_out: int) -> bool:
    """SAGEConv's update through kgx_spmm_gemm (any F_in, F_out <= 128, multiples
    of 4): out = x W_self + b by kgx_dense, then out = relu?(out + REDUCE(x) W_neigh)
    in the fused aggregation's store, so the [N, F_in] aggregate is never
    written (C5: 2.45M x 100).  Opt-in (KGX_FUSED_SAGE=1): at C5 it measured
    slower than the two-step path -- the fused main kernel's W registers hold
    it at 4 waves per SIMD, and C5's 50-edge rows want spmm_kernel's gather
    depth.  KGX_FUSED=0 turns it off too."""
    import os

    if os.environ.get("KGX_FUSED", "1") in ("0", "false", "False"):
        return False
    if os.environ.get("KGX_FUSED_SAGE", "0") not in ("1", "true", "True"):
        return False
    return 0 < f_in <= 128 and f_in % 4 == 0 and 0 < f_out <= 128 and f_out % 4 == 0


def _gatv2_impl(h_src, h_dst, rowptr, rows, items, split, col, att, heads, channels, negative_slope, bias,
                n_slots, save_stats, drop_key=None, drop_p=0.0, drop_seed=0):
    h_src, h_dst, att, bias = _f32c(h_src), _f32c(h_dst), _f32c(att), _f32c(bias)
    dev = nat.require_device(h_src, h_dst, rowptr, rows, col, att, bias, items, split)
    n_dst = rowptr.numel() - 1
    HC = heads * channels
    out = torch.empty((n_dst, HC), dtype=torch.float32, device=dev)
    stats = torch.empty((n_dst if save_stats else 0, 2 * heads), dtype=torch.float32, device=dev)
    if n_dst == 0:
        return out, stats
    n_items = 0 if items is None else items.shape[0]
    n_split = 0 if split is None else split.shape[0]
    partials = None
    if items is not None and n_split > 0:
        partials = torch.empty((n_slots, HC + 2 * heads), dtype=torch.float32, device=dev)
    nat.check(
        nat.lib().kgx_gatv2(
            nat.ptr(rowptr), nat.ptr(rows), n_dst, nat.ptr(items), n_items, nat.ptr(split), n_split,
            nat.ptr(col), nat.ptr(h_src), nat.ptr(h_dst), h_src.stride(0), nat.ptr(att), heads, channels,
            float(negative_slope), nat.ptr(out), out.stride(0), nat.ptr(bias), nat.ptr(partials),
            nat.ptr(stats) if save_stats else None, nat.ptr(drop_key) if drop_p > 0 else None, float(drop_p),
            int(drop_seed) & (2**64 - 1), nat.stream(dev),
        ),
        "kgx_gatv2",
    )
    return out, stats


@torch.library.custom_op("kgx::gatv2_save", mutates_args=())
def gatv2_save(
    h_src: torch.Tensor,
    h_dst: torch.Tensor,
    rowptr: torch.Tensor,
    rows: torch.Tensor,
    items: Optional[torch.Tensor],
    split: Optional[torch.Tensor],
    col: torch.Tensor,
    att: torch.Tensor,
    heads: int,
    channels: int,
    negative_slope: float,
    bias: Optional[torch.Tensor],
    n_slots: int,
    drop_key: Optional[torch.Tensor] = None,
    drop_p: float = 0.0,
    drop_seed: int = 0,
) -> tuple[torch.Tensor, torch.Tensor]:
    """kgx::gatv2 that also returns the per-row softmax statistics [n, 2*heads]."""
    return _gatv2_impl(h_src, h_dst, rowptr, rows, items, split, col, att, heads, channels, negative_slope, bias,
                       n_slots, True, drop_key, drop_p, drop_seed)


@gatv2_save.register_fake
def _gatv2_save_fake(h_src, h_dst, rowptr, rows, items, split, col, att, heads, channels, negative_slope, bias,
                     n_slots, drop_key=None, drop_p=0.0, drop_seed=0):
    n = rowptr.shape[0] - 1
    return h_src.new_empty((n, heads * channels)), h_src.new_empty((n, 2 * heads))


@torch.library.custom_op("kgx::gatv2", mutates_args=())
def gatv2(
    h_src: torch.Tensor,
    h_dst: torch.Tensor,
    rowptr: torch.Tensor,
    rows: torch.Tensor,
    items: Optional[torch.Tensor],
    split: Optional[torch.Tensor],
    col: torch.Tensor,
    att: torch.Tensor,
    heads: int,
    channels: int,
    negative_slope: float,
    bias: Optional[torch.Tensor],
    n_slots: int,
    drop_key: Optional[torch.Tensor] = None,
    drop_p: float = 0.0,
    drop_seed: int = 0,
) -> torch.Tensor:
    return _gatv2_impl(h_src, h_dst, rowptr, rows, items, split, col, att, heads, channels, negative_slope, bias,
                       n_slots, False, drop_key, drop_p, drop_seed)[0]


@gatv2.register_fake
def _gatv2_fake(h_src, h_dst, rowptr, rows, items, split, col, att, heads, channels, negative_slope, bias, n_slots,
                drop_key=None, drop_p=0.0, drop_seed=0):
    return h_src.new_empty((rowptr.shape[0] - 1, heads * channels))


@torch.library.custom_op("kgx::gather_rows", mutates_args=())
def gather_rows(table: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
    table = _f32c(table)
    dev = nat.require_device(table, rows)
    n, F = rows.numel(), table.shape[1]
    out = torch.empty((n, F), dtype=torch.float32, device=dev)
    nat.check(
        nat.lib().kgx_gather_rows(
            nat.ptr(table), table.stride(0), nat.ptr(rows.contiguous()), n, F, nat.ptr(out), out.stride(0),
            nat.stream(dev),
        ),
        "kgx_gather_rows",
    )
    return out


@gather_rows.register_fake
def _gather_rows_fake(table, rows):
    return table.new_empty((rows.shape[0], table.shape[1]))


@torch.library.custom_op("kgx::scatter_f32", mutates_args=())
def scatter_f32(values: torch.Tensor, perm: torch.Tensor, n_out: int) -> torch.Tensor:
    """out[perm[i]] = values[i]; positions not hit are zero."""
    values = _f32c(values)
    dev = nat.require_device(values, perm)
    out = torch.zeros(n_out, dtype=torch.float32, device=dev)
    nat.check(
        nat.lib().kgx_scatter_f32(nat.ptr(values), nat.ptr(perm.contiguous()), values.numel(), nat.ptr(out),
                                  nat.stream(dev)),
        "kgx_scatter_f32",
    )
    return out


@scatter_f32.register_fake
def _scatter_fake(values, perm, n_out):
    return values.new_empty((n_out,))


# ---------------------------------------------------------------------------
# graph-level helpers used by the layers
# ---------------------------------------------------------------------------
# When a list is installed here, every aggregation launch is bracketed by a
# pair of torch.cuda.Events recorded on the current stream — the stream the
# kernels are launched on — so a harness can time the kernels alone.
EVENT_SINK: list | None = None


def _timed(fn):
    if EVENT_SINK is None:
        return fn()
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    start.record()
    out = fn()
    end.record()
    EVENT_SINK.append((start, end))
    return out

def _reduce_id(reduce) -> int:
    return nat.REDUCE_IDS[reduce] if isinstance(reduce, str) else int(reduce)


def _needs_grad(*ts) -> bool:
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)


def _exact_short(g, red) -> int:
    """EXACT mode's short-row suffix for kgx_spmm's n_long_items (graph.exact_short_start)."""
    from . import graph as G

    return -1 if red == nat.STD else G.exact_short_start(g)


def _aggregate_raw(g, table, red, weighted, by_edge, epilogue, bias, xroot, gin_scale, exact, drop_p=0.0,
                   drop_seed=0):
    items, _, split, _, n_slots = g.work(exact or red == nat.STD)
    idx = g.eid if by_edge else g.col
    w = g.w if weighted else None
    if weighted and w is None:
        raise ValueError("graph was built without GCN normalisation weights")
    if drop_p > 0 and red != nat.SUM:
        raise ValueError("message dropout is implemented for sum aggregation (GCNConv) only")
    return _timed(lambda: torch.ops.kgx.spmm(
        table, g.rowptr, g.rows, items, split, idx, w, n_slots, red, epilogue, bias, xroot, float(gin_scale),
        g.eid if drop_p > 0 else None, float(drop_p), int(drop_seed),
        g.n_long if items is not None else _exact_short(g, red),
    ))


def _reduce_backward(g: CSRGraph, red: int, weighted: bool, by_edge: bool, table: torch.Tensor | None,
                     grad_out: torch.Tensor, exact: bool, table_rows: int, raw: bool = False, drop_p: float = 0.0,
                     drop_seed: int = 0) -> torch.Tensor:
    """d loss / d table of REDUCE_{e in row} table[idx_e] (* w_e), given d loss / d out.

    sum / mean: the transposed aggregation (graph.transpose: each source row
    gathers the gradient rows of its edges' destinations, in input-edge order);
    max / min: kgx_spmm_max_backward (ties share evenly, +-inf rows pass
    nothing — torch scatter_reduce amax/amin under the reference's isinf guard);
    by_edge (message tensors): each message receives its row's gradient."""
    from . import graph as G

    grad_out = grad_out.contiguous()
    if red == nat.STD:
        # std_i = sqrt(ssd_i / n_i) (0 where n_i <= 1), aggregators.py:182-228:
        #   d std_i / d m_e = (m_e - mean_i) / (n_i std_i)   (the mean's own path sums to 0)
        # so with A_i = g_i / (n_i std_i) (0 where n_i <= 1):
        #   grad m_e = A_i (m_e - mean_i);  grad x_j = x_j * (A^T A)_j - (A^T (A * mean))_j
        std = _aggregate_raw(g, table, nat.STD, False, by_edge, nat.EPI_NONE, None, None, 1.0, True)
        mean = _aggregate_raw(g, table, nat.MEAN, False, by_edge, nat.EPI_NONE, None, None, 1.0, True)
        # As torch autograd of the reference: the count <= 1 guard's where() sends 0 into
        # sqrt'(0) = inf, so rows with one message (and zero-variance rows) yield NaN.
        count = torch.clamp(g.deg, max=1 << 24).float().unsqueeze(1)
        A = grad_out / (torch.clamp(count, min=1e-8) * std)
        A = torch.where(count > 1, A, torch.full_like(A, float("nan")))
        if by_edge:
            rows = G.row_of_slot(g).long()
            gt = grad_out.new_zeros((table_rows, grad_out.shape[1]))
            gt.index_copy_(0, g.eid.long(), A.index_select(0, rows) * (table.index_select(0, g.eid.long())
                                                                       - mean.index_select(0, rows)))
            return gt
        t = G.transpose(g)
        sa = _aggregate_raw(t, A.contiguous(), nat.SUM, False, False, nat.EPI_NONE, None, None, 1.0, exact)
        sb = _aggregate_raw(t, (A * mean).contiguous(), nat.SUM, False, False, nat.EPI_NONE, None, None, 1.0, exact)
        return table * sa - sb
    if red in (nat.MAX, nat.MIN):
        table = table.contiguous()
        gt = torch.zeros_like(table)
        idx = g.eid if by_edge else g.col
        nat.check(
            nat.lib().kgx_spmm_max_backward(
                red, int(raw), nat.ptr(g.rowptr), g.n_dst, nat.ptr(idx), nat.ptr(table), table.stride(0), table.shape[1],
                nat.ptr(grad_out), grad_out.stride(0), nat.ptr(gt), gt.stride(0), nat.stream(table.device),
            ),
            "kgx_spmm_max_backward",
        )
        return gt
    d = grad_out
    if red == nat.MEAN:  # forward: sum / max(count_f32, 1e-8) (aggregators.py:56-85)
        count = torch.clamp(g.deg, max=1 << 24).float()
        d = (grad_out / torch.clamp(count, min=1e-8).unsqueeze(1)).contiguous()
    if by_edge:
        vals = d.index_select(0, G.row_of_slot(g).long())
        if weighted:
            vals = vals * g.w.unsqueeze(1)
        gt = grad_out.new_zeros((table_rows, grad_out.shape[1]))
        gt.index_copy_(0, g.eid.long(), vals)
        return gt
    t = G.transpose(g)  # t.eid = input edge ids: the same dropout mask keys as the forward
    return _aggregate_raw(t, d, nat.SUM, weighted, False, nat.EPI_NONE, None, None, 1.0, exact, drop_p, drop_seed)


def dropout_mask(seed: int, p: float, keys: torch.Tensor, F: int) -> torch.Tensor:
    """The multipliers (0 or 1/(1-p)) kgx's message dropout applies: [len(keys), F]."""
    keys = keys.to(torch.int32).contiguous()
    out = torch.empty((keys.numel(), F), dtype=torch.float32, device=keys.device)
    nat.check(nat.lib().kgx_dropout_mask(int(seed) & (2**64 - 1), float(p), nat.ptr(keys), keys.numel(), F,
                                         nat.ptr(out), nat.stream(keys.device)), "kgx_dropout_mask")
    return out


class _AggregateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, bias, xroot, g, red, weighted, by_edge, epilogue, gin_scale, exact, drop_p, drop_seed):
        ctx.g, ctx.red, ctx.weighted, ctx.by_edge = g, red, weighted, by_edge
        ctx.epilogue, ctx.gin_scale, ctx.exact = epilogue, gin_scale, exact
        ctx.drop_p, ctx.drop_seed = drop_p, drop_seed
        ctx.table_rows = table.shape[0]
        ctx.save_for_backward(table if red in (nat.MAX, nat.MIN, nat.STD) else None)
        return _aggregate_raw(g, table, red, weighted, by_edge, epilogue, bias, xroot, gin_scale, exact, drop_p,
                              drop_seed)

    @staticmethod
    def backward(ctx, grad_out):
        (table,) = ctx.saved_tensors
        g_table = g_bias = g_xroot = None
        if ctx.needs_input_grad[0]:
            g_table = _reduce_backward(ctx.g, ctx.red, ctx.weighted, ctx.by_edge, table, grad_out, ctx.exact,
                                       ctx.table_rows, raw=ctx.epilogue == nat.EPI_RAW, drop_p=ctx.drop_p,
                                       drop_seed=ctx.drop_seed)
        if ctx.needs_input_grad[1] and ctx.epilogue == nat.EPI_BIAS:
            g_bias = grad_out.sum(0)
        if ctx.needs_input_grad[2] and ctx.epilogue == nat.EPI_GIN:
            g_xroot = grad_out * ctx.gin_scale
        return g_table, g_bias, g_xroot, None, None, None, None, None, None, None, None, None


def aggregate(
    g: CSRGraph,
    table: torch.Tensor,
    reduce: str | int = "sum",
    *,
    weighted: bool = False,
    by_edge: bool = False,
    epilogue: int = nat.EPI_NONE,
    bias: torch.Tensor | None = None,
    xroot: torch.Tensor | None = None,
    gin_scale: float = 1.0,
    exact: bool = False,
    dropout: float = 0.0,
    seed: int = 0,
) -> torch.Tensor:
    """out[i] = EPI(REDUCE_{e in row i} table[idx[e]] * (w[e] if weighted)).

    by_edge=False gathers node rows through `col` (the fused propagate path);
    by_edge=True gathers rows of a per-edge message tensor through `eid`
    (the reference's Aggregator.aggregate(messages, target_idx, dim_size)).
    Differentiable in table, bias and xroot (sum, mean, max, min).  dropout > 0
    (sum only): every message element is kept with probability 1 - dropout and
    scaled by 1/(1 - dropout), the mask a function of (seed, input edge id,
    column) -- GCNConv's training-time message dropout (gcn_conv.py:237-242).
    """
    red = _reduce_id(reduce)
    if dropout and by_edge:
        raise ValueError("message dropout applies to gathered node rows, not to message tensors")
    if _needs_grad(table, bias, xroot):
        return _AggregateFn.apply(table, bias, xroot, g, red, weighted, by_edge, epilogue, float(gin_scale), exact,
                                  float(dropout), int(seed))
    return _aggregate_raw(g, table, red, weighted, by_edge, epilogue, bias, xroot, gin_scale, exact, float(dropout),
                          int(seed))


def _tiny_of(g, items):
    """(tpack, tw, n_short_end, n_tiny2) for a fused launch over g's schedule
    (tiny.py: packed records of the degree <= 2 tail, built once per graph)."""
    if items is None:
        return None, None, -1, 0
    from . import tiny

    return tiny.tiny_pack(g)


def _aggregate_transform_raw(g, x, W, red, weighted, bias, pre_gin, gin_scale, exact, relu=False, x2=None):
    items, _, split, _, n_slots = g.work(exact)
    w = g.w if weighted else None
    if weighted and w is None:
        raise ValueError("graph was built without GCN normalisation weights")
    return _timed(lambda: torch.ops.kgx.spmm_gemm(
        x, g.rowptr, g.rows, items, split, g.col, w, n_slots, red, W, bias, bool(pre_gin), float(gin_scale),
        bool(relu), g.n_long if items is not None else -1, *_tiny_of(g, items), x2
    ))


def gemm_tn(P: torch.Tensor, D: torch.Tensor, with_db: bool = False):
    """(P^T D, column sums of D or None) in one pass over P and D (kgx_gemm_tn:
    the bf16x3-split MFMA product over the node dimension, split-K over row
    ranges with partials summed in block order) -- the weight and bias
    gradients of a layer out = P W + b.  Device tensors only (the product path
    has no CPU fallback)."""
    P = P if P.stride(-1) == 1 else P.contiguous()
    D = D if D.stride(-1) == 1 else D.contiguous()
    dev = nat.require_device(P, D)
    if P.dtype != torch.float32 or D.dtype != torch.float32 or P.dim() != 2 or D.dim() != 2 or P.shape[0] != D.shape[0]:
        raise ValueError(f"gemm_tn: float32 [N, K] and [N, M] expected (got {tuple(P.shape)}, {tuple(D.shape)})")
    N, K, M = P.shape[0], P.shape[1], D.shape[1]
    dW = torch.empty((K, M), dtype=torch.float32, device=dev)
    db = torch.empty(M, dtype=torch.float32, device=dev) if with_db else None
    if K == 0 or M == 0:
        return dW, (db.zero_() if db is not None else None)
    L = nat.lib()
    nbytes = ctypes.c_size_t(0)
    nat.check(L.kgx_gemm_tn_workspace_bytes(N, K, M, ctypes.byref(nbytes)), "kgx_gemm_tn_workspace_bytes")
    ws = torch.empty(max(nbytes.value, 4), dtype=torch.uint8, device=dev)
    nat.check(L.kgx_gemm_tn(N, nat.ptr(P), P.stride(0), K, nat.ptr(D), D.stride(0), M, nat.ptr(dW), M, nat.ptr(db),
                            nat.ptr(ws), nbytes.value, nat.stream(dev)), "kgx_gemm_tn")
    return dW, db


class _AggregateTransformFn(torch.autograd.Function):
    """out = bias + PRE(A x) W.  Backward: P = PRE(A x) is recomputed (one
    aggregation launch) rather than kept from the forward; dW = P^T dOut,
    db = sum dOut, dx = A^T-backward(dOut W^T) (+ gin_scale dOut W^T)."""

    @staticmethod
    def forward(ctx, x, W, bias, g, red, weighted, pre_gin, gin_scale, exact):
        ctx.g, ctx.red, ctx.weighted, ctx.pre_gin, ctx.gin_scale, ctx.exact = g, red, weighted, pre_gin, gin_scale, exact
        items, _, split, _, n_slots = g.work(exact)
        w = g.w if weighted else None
        if ctx.needs_input_grad[1]:  # keep P = PRE(A x) for dW (one extra row store instead of a recompute)
            out, P = _timed(lambda: torch.ops.kgx.spmm_gemm_save(
                x, g.rowptr, g.rows, items, split, g.col, w, n_slots, red, W, bias, bool(pre_gin), float(gin_scale),
                g.n_long if items is not None else -1, *_tiny_of(g, items)))
        else:
            out = _aggregate_transform_raw(g, x, W, red, weighted, bias, pre_gin, gin_scale, exact)
            P = None
        ctx.save_for_backward(x if red in (nat.MAX, nat.MIN) else None, W, P)
        ctx.x_rows = x.shape[0]
        return out

    @staticmethod
    def backward(ctx, grad_out):
        from . import graph as G

        x, W, P = ctx.saved_tensors
        grad_out = grad_out.contiguous()
        g_x = g_W = g_b = None
        # dW / db (kgx_gemm_tn) beside the dx pass: the side stream waits for an event recorded
        # here, before dx is launched, and is forked after it, so dx's blocks are dispatched first;
        # W^T is copied before the event (queued after it, the small copy waited for the whole
        # dW pass: its waves found no registers free beside kgx_gemm_tn's, profiles/r06/train/)
        overlap = ctx.needs_input_grad[1] and ctx.needs_input_grad[0] and grad_out.is_cuda and _tn_overlap()
        W_t = W.t().contiguous() if ctx.needs_input_grad[0] else None  # before the fork: see above
        start = None
        if overlap:
            start = torch.cuda.Event()
            start.record()
        if not overlap and ctx.needs_input_grad[1]:  # dW = P^T dOut and db = colsum(dOut) in one pass
            g_W, g_b = gemm_tn(P, grad_out, with_db=ctx.needs_input_grad[2])
        elif not ctx.needs_input_grad[1] and ctx.needs_input_grad[2]:
            g_b = grad_out.sum(0)
        if ctx.needs_input_grad[0]:
            with _unsplit():  # the transposed pass one-stream (see _unsplit)
                f_out, f_in = W.shape[1], W.shape[0]
                if ctx.red in (nat.SUM, nat.MEAN) and not ctx.pre_gin and fused_transform_supported(f_out, f_in):
                    # dx = A^T (dOut W^T) = (A^T dOut) W^T: the same fused kernel on the transposed graph
                    d = grad_out
                    if ctx.red == nat.MEAN:
                        count = torch.clamp(ctx.g.deg, max=1 << 24).float()
                        d = (grad_out / torch.clamp(count, min=1e-8).unsqueeze(1)).contiguous()
                    t = G.transpose(ctx.g)
                    g_x = _aggregate_transform_raw(t, d, W_t, nat.SUM, ctx.weighted, None, False, 1.0, ctx.exact)
                else:
                    dP = grad_out @ W_t
                    g_x = _reduce_backward(ctx.g, ctx.red, ctx.weighted, False, x, dP, ctx.exact, ctx.x_rows)
                    if ctx.pre_gin:
                        g_x = g_x + dP * ctx.gin_scale
        if overlap:
            cur = torch.cuda.current_stream(grad_out.device)
            side = _side_stream(grad_out.device)
            side.wait_event(start)
            with torch.cuda.stream(side):
                g_W, g_b = gemm_tn(P, grad_out, with_db=ctx.needs_input_grad[2])
            P.record_stream(side)
            grad_out.record_stream(side)
            cur.wait_stream(side)  # join: dW / db are ready before anything later on this stream
            for t_ in (g_W, g_b):
                if t_ is not None:
                    t_.record_stream(cur)
        return g_x, g_W, g_b, None, None, None, None, None, None


_SIDE_STREAMS: dict = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    """One side stream per device for backward work that runs beside the main pass."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = _SIDE_STREAMS[key] = torch.cuda.Stream(device=dev)
    return s


def _tn_overlap() -> bool:
    """KGX_TN_OVERLAP (default 0): 1 runs the fused layers' dW / db pass (kgx_gemm_tn) on a side
    stream beside the dx pass of the same backward.  Off by default: both passes stream HBM, and
    side by side the dx pass's main kernel went 8.2 -> 13.9 ms for the 2.3 ms of dW it hid (NS
    training step 21.7 ms serial against 21.8-24.4 overlapped, profiles/r06/train/overlap.md)."""
    return os.environ.get("KGX_TN_OVERLAP", "0") not in ("0", "", "false", "False")


def aggregate_transform(
    g: CSRGraph,
    x: torch.Tensor,
    W: torch.Tensor,
    reduce: str | int = "sum",
    *,
    weighted: bool = False,
    bias: torch.Tensor | None = None,
    pre_gin: bool = False,
    gin_scale: float = 1.0,
    exact: bool = False,
    out: torch.Tensor | None = None,
    relu: bool = False,
    x2: torch.Tensor | None = None,
    accumulate: bool = True,
) -> torch.Tensor:
    """out = bias + PRE(REDUCE_{e in row} x[col_e] * w_e) @ W in one fused launch
    (out += ... in place when `out` is given, or, with accumulate=False, the
    graph's scheduled rows of `out` overwritten; relu=True applies max(., 0) in
    the kernel's store).  Differentiable in x, W, bias.  x2 (forward only): a
    second table, sources col >= x.shape[0] gather x2[col - x.shape[0]]
    (the sharded layers' own rows + received halo rows in one pass)."""
    red = _reduce_id(reduce)
    if x2 is not None and _needs_grad(x, x2, W, bias):
        raise NotImplementedError("aggregate_transform(x2=...) is a forward-only (no_grad) path")
    if out is not None:  # into `out`: a sum may be split over launches (the caller splits a row's edges);
        # a mean / max / min launch must cover each row's whole edge list
        if red != nat.SUM and (x2 is not None or x.shape[1] == F256):
            raise ValueError("aggregate_transform(out=...): two-table and 256-wide passes accumulate plain sums only")
        if accumulate and (pre_gin or (relu and x.shape[1] == F256)):
            raise ValueError("aggregate_transform(out=...): pre_gin (and relu at F_in 256) only with "
                             "accumulate=False (overwrite)")
        if _needs_grad(x, W, bias, out):
            raise NotImplementedError("aggregate_transform(out=...) is a forward-only (no_grad) path")
        items, _, split, _, n_slots = g.work(exact)
        w = g.w if weighted else None
        flags = (nat.FUSED_PRE_GIN if pre_gin else 0) | (nat.FUSED_RELU if relu else 0)
        _timed(lambda: torch.ops.kgx.spmm_gemm_acc_(out, x, g.rowptr, g.rows, items, split, g.col, w, n_slots, red,
                                                   W, bias, g.n_long if items is not None else -1,
                                                   *_tiny_of(g, items), x2, bool(accumulate), int(flags),
                                                   float(gin_scale)))
        return out
    if x2 is not None:
        return _aggregate_transform_raw(g, x, W, red, weighted, bias, pre_gin, gin_scale, exact, relu, x2)
    if _needs_grad(x, W, bias):
        y = _AggregateTransformFn.apply(x, W, bias, g, red, weighted, pre_gin, float(gin_scale), exact)
        return torch.relu(y) if relu else y
    return _aggregate_transform_raw(g, x, W, red, weighted, bias, pre_gin, gin_scale, exact, relu)


def _gatv2_raw(g, h_src, h_dst, att, heads, channels, negative_slope, bias, exact, drop_p=0.0, drop_seed=0):
    items, _, split, _, n_slots = g.work(exact)
    return _timed(lambda: torch.ops.kgx.gatv2(
        h_src, h_dst, g.rowptr, g.rows, items, split, g.col, att.reshape(-1), heads, channels,
        float(negative_slope), bias, n_slots, g.eid if drop_p > 0 else None, float(drop_p), int(drop_seed),
    ))


class _GATv2Fn(torch.autograd.Function):
    """Autograd of the fused GATv2 aggregation: the forward keeps its output
    and per-row softmax statistics; kgx_gatv2_backward does one pass over the
    destination CSR (d h_dst, d att, per-edge alpha / ds) and pulls d h_src
    over the transposed CSR, both with hub rows split into chunks."""

    @staticmethod
    def forward(ctx, h_src, h_dst, att, bias, g, heads, channels, negative_slope, exact, drop_p, drop_seed):
        ctx.g, ctx.heads, ctx.channels, ctx.slope, ctx.exact = g, heads, channels, float(negative_slope), exact
        ctx.drop_p, ctx.drop_seed = drop_p, drop_seed
        items, _, split, _, n_slots = g.work(exact)
        out, stats = _timed(lambda: torch.ops.kgx.gatv2_save(
            h_src, h_dst, g.rowptr, g.rows, items, split, g.col, att.reshape(-1), heads, channels,
            float(negative_slope), bias, n_slots, g.eid if drop_p > 0 else None, float(drop_p), int(drop_seed),
        ))
        ctx.save_for_backward(h_src, h_dst, att, bias, out, stats)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        from . import graph as G

        h_src, h_dst, att, bias, out, stats = ctx.saved_tensors
        g, H, C = ctx.g, ctx.heads, ctx.channels
        grad_out = grad_out.contiguous()
        h_src, h_dst = h_src.contiguous(), h_dst.contiguous()
        att_flat = att.reshape(-1).contiguous()
        t = G.transpose(g)
        items, _, split, _, n_slots = g.work(ctx.exact)
        t_items, _, t_split, _, t_slots = t.work(ctx.exact)
        dev = grad_out.device
        g_src = torch.empty((g.n_src, H * C), dtype=torch.float32, device=dev)
        g_dst = torch.empty((g.n_dst, H * C), dtype=torch.float32, device=dev)
        g_att = torch.zeros(H * C, dtype=torch.float32, device=dev)
        alpha = torch.empty((max(g.kept, 1), H), dtype=torch.float32, device=dev)
        ds = torch.empty_like(alpha)
        partials = torch.empty((max(n_slots, t_slots, 1), H * C), dtype=torch.float32, device=dev)
        slot = t.extras.get("fwd_slot32")
        if slot is None:
            slot = t.extras["fwd_slot"].to(torch.int32)
            t.extras["fwd_slot32"] = slot
        n_items = 0 if items is None else items.shape[0]
        n_split = 0 if split is None else split.shape[0]
        t_n_items = 0 if t_items is None else t_items.shape[0]
        t_n_split = 0 if t_split is None else t_split.shape[0]
        nat.check(
            nat.lib().kgx_gatv2_backward(
                nat.ptr(g.rowptr), nat.ptr(g.rows), g.n_dst, nat.ptr(items), n_items, nat.ptr(split), n_split,
                nat.ptr(g.col), nat.ptr(h_src), nat.ptr(h_dst), h_src.stride(0), nat.ptr(att_flat), H, C,
                ctx.slope, nat.ptr(out), out.stride(0), nat.ptr(bias), nat.ptr(stats), nat.ptr(grad_out),
                grad_out.stride(0), nat.ptr(t.rowptr), nat.ptr(t.rows), g.n_src, nat.ptr(t_items), t_n_items,
                nat.ptr(t_split), t_n_split, nat.ptr(t.col), nat.ptr(slot), nat.ptr(g_src), nat.ptr(g_dst),
                g_src.stride(0), nat.ptr(g_att), nat.ptr(alpha), nat.ptr(ds), nat.ptr(partials),
                nat.ptr(g.eid) if ctx.drop_p > 0 else None, float(ctx.drop_p), int(ctx.drop_seed) & (2**64 - 1),
                nat.stream(dev),
            ),
            "kgx_gatv2_backward",
        )
        g_bias = grad_out.sum(0) if ctx.needs_input_grad[3] else None
        return g_src, g_dst, g_att.view(att.shape), g_bias, None, None, None, None, None, None, None


def gatv2_aggregate(
    g: CSRGraph,
    h_src: torch.Tensor,
    h_dst: torch.Tensor,
    att: torch.Tensor,
    heads: int,
    channels: int,
    negative_slope: float,
    bias: torch.Tensor | None = None,
    exact: bool = False,
    dropout: float = 0.0,
    seed: int = 0,
) -> torch.Tensor:
    """Fused GATv2 attention aggregation; differentiable in h_src, h_dst, att, bias.
    dropout > 0: attention dropout of alpha per (edge, head), mask of (seed, input edge id, head)."""
    if _needs_grad(h_src, h_dst, att, bias):
        return _GATv2Fn.apply(h_src, h_dst, att, bias, g, heads, channels, negative_slope, exact, float(dropout),
                              int(seed))
    return _gatv2_raw(g, h_src, h_dst, att, heads, channels, negative_slope, bias, exact, float(dropout), int(seed))


# ---------------------------------------------------------------------------
# Dense node transform: kgx_dense (bf16x3-split MFMA, f32-accurate)
# ---------------------------------------------------------------------------
def _aligned16(t: torch.Tensor) -> torch.Tensor:
    """Contiguous fp32 rows on a 16-byte boundary (what kgx_dense's dwordx4 loads need)."""
    t = _f32c(t)
    return t if t.data_ptr() % 16 == 0 else t.clone()


def dense_supported(x0: torch.Tensor, W0: torch.Tensor, W1: torch.Tensor | None = None) -> bool:
    """Shapes kgx_dense implements: K0 + K1 <= 256, N <= 256, K0, K1 multiples of 4."""
    if not (x0.is_cuda and x0.dim() == 2 and W0.dim() == 2):
        return False
    k0, n = W0.shape
    k1 = 0 if W1 is None else W1.shape[0]
    return (0 < n <= nat.DENSE_MAX_N and k0 + k1 <= nat.DENSE_MAX_K and k0 % 4 == 0 and k1 % 4 == 0
            and (W1 is None or W1.shape[1] == n))


@torch.library.custom_op("kgx::dense", mutates_args=())
def dense_op(
    x0: torch.Tensor,
    W0: torch.Tensor,
    x1: Optional[torch.Tensor],
    W1: Optional[torch.Tensor],
    bias: Optional[torch.Tensor],
    relu: bool,
) -> torch.Tensor:
    x0, W0, bias = _aligned16(x0), _f32c(W0), _f32c(bias)
    x1 = None if x1 is None else _aligned16(x1)
    W1 = None if W1 is None else _f32c(W1)
    dev = nat.require_device(x0, W0, x1, W1, bias)
    M, N = x0.shape[0], W0.shape[1]
    if x1 is not None and x1.shape[0] != M:
        raise ValueError(f"kgx.dense: x1 has {x1.shape[0]} rows, x0 has {M}")
    out = torch.empty((M, N), dtype=torch.float32, device=dev)
    nat.check(
        nat.lib().kgx_dense(
            M, nat.ptr(x0), x0.stride(0), x0.shape[1], nat.ptr(W0),
            nat.ptr(x1), x1.stride(0) if x1 is not None else 0, x1.shape[1] if x1 is not None else 0, nat.ptr(W1),
            N, nat.ptr(bias), nat.DENSE_RELU if relu else 0, nat.ptr(out), out.stride(0), nat.stream(dev),
        ),
        "kgx_dense",
    )
    return out


@dense_op.register_fake
def _dense_fake(x0, W0, x1, W1, bias, relu):
    return x0.new_empty((x0.shape[0], W0.shape[1]))


def _matmul_t(g: torch.Tensor, W: torch.Tensor) -> torch.Tensor:
    """g @ W^T for the backward: the library fp32 GEMM, so gradients keep the
    reference autograd's fp32 GEMM numerics (kgx_dense is f32-accurate too,
    but its re-associated sums moved GIN's d/dx past the 1e-5 gradient bar
    on the toy graph of tests/test_gpu_backward.py)."""
    return g @ W.t()


class _DenseFn(torch.autograd.Function):
    """y = relu?(bias + x0 W0 + x1 W1).  Backward: dz = dy * (y > 0) for ReLU;
    dx_t = dz W_t^T (kgx_dense again), dW_t = x_t^T dz (split-K), db = sum dz."""

    @staticmethod
    def forward(ctx, x0, W0, x1, W1, bias, relu):
        y = torch.ops.kgx.dense(x0, W0, x1, W1, bias, relu)
        ctx.relu = relu
        ctx.save_for_backward(x0, W0, x1, W1, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, grad):
        x0, W0, x1, W1, y = ctx.saved_tensors
        dz = grad.contiguous()
        if ctx.relu:
            dz = dz * (y > 0)
        g = [None] * 6
        if ctx.needs_input_grad[0]:
            g[0] = _matmul_t(dz, W0)
        if ctx.needs_input_grad[1]:  # dW0 = x0^T dz (+ db = colsum(dz) in the same pass, kgx_gemm_tn)
            g[1], g[4] = gemm_tn(x0, dz, with_db=ctx.needs_input_grad[4])
        if x1 is not None and ctx.needs_input_grad[2]:
            g[2] = _matmul_t(dz, W1)
        if x1 is not None and ctx.needs_input_grad[3]:
            g[3], _ = gemm_tn(x1, dz)
        if ctx.needs_input_grad[4] and g[4] is None:
            g[4] = dz.sum(0)
        return tuple(g)


def dense(
    x0: torch.Tensor,
    W0: torch.Tensor,
    bias: torch.Tensor | None = None,
    *,
    x1: torch.Tensor | None = None,
    W1: torch.Tensor | None = None,
    relu: bool = False,
) -> torch.Tensor:
    """relu?(bias + x0 @ W0 (+ x1 @ W1)) -- keras Dense / SAGEConv's two linear
    maps in one kgx_dense launch (differentiable).  Shapes kgx_dense does not
    implement (K > 256, N > 256, K % 4 != 0) run as the library GEMM
    (hipBLASLt) on the same device."""
    if (x1 is None) != (W1 is None):
        raise ValueError("dense: x1 and W1 go together")
    if dense_supported(x0, W0, W1):
        if _needs_grad(x0, W0, x1, W1, bias):
            return _DenseFn.apply(x0, W0, x1, W1, bias, bool(relu))
        return torch.ops.kgx.dense(x0, W0, x1, W1, bias, bool(relu))
    y = torch.addmm(bias, x0, W0) if bias is not None else x0 @ W0
    if x1 is not None:
        y = torch.addmm(y, x1, W1)
    return torch.relu(y) if relu else y
