"""Device-resident graph structure: stable destination CSR + row schedule.

The reference re-derives everything from `edge_index` on every call
(message_passing.py:256-268 casts/caches edge_index by id(); add_self_loops and
compute_gcn_normalization run per call, gcn_conv.py:328-353).  Here one
`CSRGraph` is built on the GPU per (edge_index, node count, flags) and cached
while the edge_index tensor is alive and unmodified (its storage pointer and
version counter are part of the key and the cache holds a reference, so a
freed-and-reused address can never alias a stale entry).
"""

from __future__ import annotations

import ctypes
import os
from collections import OrderedDict
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _native as nat

_ASSUMED_GROUP_SLOTS = 2048 * 256  # resident lanes (256 CUs x 8 blocks x 256 threads)


def _pow2_floor(v: int) -> int:
    return 1 << (max(int(v), 1).bit_length() - 1)


def default_split_len(n_edges: int, n_features: int = 128) -> int:
    """Hub-split chunk length for a graph.

    Static grid-stride scheduling over degree-sorted items bounds the per-group
    imbalance by the largest item, so chunks are sized to about a quarter of a
    group's average share of the edges (power of two, 256..8192).
    """
    lanes = max(1, (max(n_features, 1) + 3) // 4)  # float4 lanes per row
    G = min(64, 1 << (lanes - 1).bit_length())  # lanes per group (pow2)
    groups = _ASSUMED_GROUP_SLOTS // G
    share = max(1, n_edges // groups)
    return int(min(8192, max(256, _pow2_floor(max(share // 4, 1)))))


def exact_mode_default() -> bool:
    return os.environ.get("KGX_EXACT", "0") not in ("", "0", "false", "False")


@dataclass
class CSRGraph:
    n_src: int
    n_dst: int
    n_input_edges: int
    kept: int  # edges kept in the CSR (incl. self loops)
    max_degree: int
    flags: int
    rowptr: torch.Tensor  # int32 [n_dst+1]
    col: torch.Tensor  # int32 [kept]   source node per CSR slot
    eid: torch.Tensor  # int32 [kept]   input edge id per CSR slot (E+i = self loop i)
    deg: torch.Tensor  # int32 [n_dst]
    dinv: torch.Tensor | None = None  # fp32 [n_dst]  (GCN_NORM)
    w: torch.Tensor | None = None  # fp32 [kept]   GCN edge norm in CSR order
    rows: torch.Tensor | None = None  # int32 [n_dst]  rows in schedule order
    items: torch.Tensor | None = None  # int32 [n_items, 4]
    split: torch.Tensor | None = None  # int32 [n_split, 4]
    n_items: int = 0
    n_split: int = 0
    n_slots: int = 0
    split_len: int = 0
    # items [n_long, n_items): the schedule's suffix of unsplit rows of degree <=
    # KGX_SHORT_ROW_MAX, which the fused kernel reduces 32-64 rows per block
    # iteration (kgx_spmm_gemm_ex); -1: none / not computed
    n_long: int = -1
    extras: dict = field(default_factory=dict)

    @property
    def device(self) -> torch.device:
        return self.rowptr.device

    def work(self, exact: bool):
        """(items, n_items, split, n_split, n_slots) for a launch; exact -> none."""
        if exact or self.n_items == 0:
            return None, 0, None, 0, 0
        return self.items, self.n_items, self.split, self.n_split, self.n_slots


# ---------------------------------------------------------------------------
# GCN dinv as the reference evaluates it
# ---------------------------------------------------------------------------
_DINV_TABLES: dict = {}
_DINV_SLICE = 16384  # < ATen's GRAIN_SIZE (one thread) and a multiple of every vector width


def _dinv_values(lo: int, hi: int) -> torch.Tensor:
    """float32 [hi - lo]: (k + 1e-12)^-0.5 for k in [lo, hi) exactly as the
    reference computes dinv (utils/main.py:25: keras.ops.power(keras.ops.add(
    degrees, 1e-12), -0.5) -> torch.pow(Tensor, 0-dim Tensor) on ATen's CPU
    kernel).  ATen evaluates that with its vectorised (Sleef) powf, which is
    not correctly rounded for some degrees; scalar leftovers of a vector loop
    would use libm's powf instead, so the values are made in aligned slices
    that run on one thread and end on a whole vector: every entry takes the
    vectorised path, the one ATen takes for all but the last few elements of
    each thread's chunk of the reference's degree vector."""
    out = []
    exp = torch.tensor(-0.5, dtype=torch.float32)
    for a in range(lo - lo % _DINV_SLICE, hi, _DINV_SLICE):
        k = torch.arange(a, a + _DINV_SLICE, dtype=torch.float32)
        out.append(torch.pow(torch.add(k, torch.tensor(1e-12, dtype=torch.float32)), exp))
    vals = torch.cat(out)
    off = lo - (lo - lo % _DINV_SLICE)
    return vals[off: off + hi - lo]


def gcn_dinv_table(device: torch.device, max_degree: int = 0) -> torch.Tensor:
    """Device table dinv_table[k] = the reference's dinv of a node of fp32 degree
    k, covering k <= min(max_degree, 2^24) (grown in powers of two and cached
    per device).  kgx_csr_build2 / kgx_gcn_dinv_table index it."""
    need = min(max(int(max_degree), 0), 1 << 24) + 1
    key = str(torch.device(device))
    t = _DINV_TABLES.get(key)
    if t is None or t.numel() < need:
        n = max(4096, 1 << (need - 1).bit_length())
        n = min(n, (1 << 24) + 1)
        t = _dinv_values(0, n).to(device)
        _DINV_TABLES[key] = t
    return t


def build_csr(
    src: torch.Tensor,
    dst: torch.Tensor,
    n_src: int,
    n_dst: int,
    *,
    self_loops: bool = False,
    gcn_norm: bool = False,
    segment_only: bool = False,
    split_len: int | None = None,
    n_features: int = 128,
) -> CSRGraph:
    """COO (int32 device tensors) -> CSRGraph via kgx_csr_build + kgx_schedule_build."""
    dev = nat.require_device(src, dst)
    if src.dtype != torch.int32 or dst.dtype != torch.int32:
        raise TypeError("build_csr expects int32 src/dst")
    src = src.contiguous()
    dst = dst.contiguous()
    E = int(src.numel())
    if int(dst.numel()) != E:
        raise ValueError(f"src/dst length mismatch: {E} vs {dst.numel()}")
    flags = (
        (nat.CSR_SELF_LOOPS if self_loops else 0)
        | (nat.CSR_SEGMENT_ONLY if segment_only else 0)
        | (nat.CSR_GCN_NORM if gcn_norm else 0)
    )
    cap = E + (n_dst if self_loops else 0)
    L = nat.lib()
    i32 = dict(dtype=torch.int32, device=dev)
    rowptr = torch.empty(n_dst + 1, **i32)
    col = torch.empty(max(cap, 1), **i32)
    eid = torch.empty(max(cap, 1), **i32)
    deg = torch.empty(max(n_dst, 1), **i32)
    dinv = torch.empty(max(n_dst, 1), dtype=torch.float32, device=dev) if gcn_norm else None
    w = torch.empty(max(cap, 1), dtype=torch.float32, device=dev) if gcn_norm else None
    nbytes = ctypes.c_size_t(0)
    nat.check(L.kgx_csr_workspace_bytes(E, n_dst, flags, ctypes.byref(nbytes)), "kgx_csr_workspace_bytes")
    ws = torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=dev)
    info = (ctypes.c_int64 * 4)()
    table = gcn_dinv_table(dev) if gcn_norm else None
    nat.check(
        L.kgx_csr_build2(
            nat.ptr(src), nat.ptr(dst), E, n_src, n_dst, flags,
            nat.ptr(rowptr), nat.ptr(col), nat.ptr(eid), nat.ptr(deg), nat.ptr(dinv), nat.ptr(w),
            nat.ptr(table), table.numel() if table is not None else 0,
            nat.ptr(ws), nbytes.value, info, nat.stream(dev),
        ),
        "kgx_csr_build2",
    )
    del ws
    kept, max_deg = int(info[0]), int(info[1])
    if gcn_norm and int(info[3]):  # degrees past the table: grow it, redo dinv and w
        table = gcn_dinv_table(dev, max_deg)
        st = nat.stream(dev)
        nat.check(L.kgx_gcn_dinv_table(nat.ptr(deg), n_dst, nat.ptr(table), table.numel(), nat.ptr(dinv), st),
                  "kgx_gcn_dinv_table")
        nat.check(L.kgx_gcn_edge_norm(nat.ptr(rowptr), nat.ptr(col), n_dst, nat.ptr(dinv), nat.ptr(dinv),
                                      nat.ptr(w), st), "kgx_gcn_edge_norm")
    g = CSRGraph(
        n_src=n_src, n_dst=n_dst, n_input_edges=E, kept=kept, max_degree=max_deg, flags=flags,
        rowptr=rowptr, col=col[:kept], eid=eid[:kept], deg=deg[:n_dst],
        dinv=dinv[:n_dst] if dinv is not None else None, w=w[:kept] if w is not None else None,
    )
    _build_schedule(g, split_len if split_len is not None else default_split_len(kept, n_features))
    return g


def _build_schedule(g: CSRGraph, split_len: int) -> None:
    dev = g.device
    n = g.n_dst
    if split_len > 0:
        split_len = _pow2_floor(split_len)
    g.split_len = split_len
    if n == 0:
        g.rows = torch.empty(0, dtype=torch.int32, device=dev)
        return
    L = nat.lib()
    cap_items = n + (g.kept // split_len if split_len > 0 else 0) + 1
    cap_split = min(n, (g.kept // split_len if split_len > 0 else 0) + 1)
    rows = torch.empty(n, dtype=torch.int32, device=dev)
    items = torch.empty((cap_items, 4), dtype=torch.int32, device=dev)
    split = torch.empty((max(cap_split, 1), 4), dtype=torch.int32, device=dev)
    nbytes = ctypes.c_size_t(0)
    nat.check(L.kgx_schedule_workspace_bytes(n, ctypes.byref(nbytes)), "kgx_schedule_workspace_bytes")
    ws = torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=dev)
    info = (ctypes.c_int64 * 4)()
    nat.check(
        L.kgx_schedule_build(
            nat.ptr(g.rowptr), n, split_len, nat.ptr(rows), nat.ptr(items), cap_items, nat.ptr(split),
            nat.ptr(ws), nbytes.value, info, nat.stream(dev),
        ),
        "kgx_schedule_build",
    )
    g.rows = rows
    g.n_items, g.n_split, g.n_slots = int(info[0]), int(info[1]), int(info[2])
    if g.n_split > cap_split:
        raise RuntimeError("kgx schedule: split list overflow")
    g.items = items[: g.n_items]
    g.split = split[: max(g.n_split, 0)]
    g.n_long = short_suffix_start(g.items)
    _refresh_tiny(g)


def _refresh_tiny(g: CSRGraph) -> None:
    """(Re)build the tiny-row records of g's schedule now (tiny.py), so no
    later fused launch has to sync to build them."""
    from . import tiny

    tiny.tiny_pack(g, refresh=True)


SHORT_ROW_MAX = 7  # KGX_SHORT_ROW_MAX (include/kgx.h)


def schedule_suffixes(items: torch.Tensor, short_max: int, tiny_max: int) -> tuple[int, int]:
    """(first item of the suffix of unsplit rows of degree <= short_max, the
    same for tiny_max) of a device item list, in one kgx_schedule_suffixes pass."""
    n = int(items.shape[0])
    if n == 0:
        return 0, 0
    ws = torch.empty(16, dtype=torch.uint8, device=items.device)
    out = (ctypes.c_int64 * 2)()
    nat.check(nat.lib().kgx_schedule_suffixes(nat.ptr(items.contiguous()), n, int(short_max), int(tiny_max),
                                              nat.ptr(ws), out, nat.stream(items.device)), "kgx_schedule_suffixes")
    return int(out[0]), int(out[1])


def short_suffix_start(items: torch.Tensor) -> int:
    """First item of the degree-descending schedule's suffix of unsplit rows of
    degree <= SHORT_ROW_MAX (split rows' chunks are a prefix; rows come in
    exactly descending degree after them).  KGX_SHORT_ROWS=0: no suffix."""
    n = int(items.shape[0])
    if n == 0 or os.environ.get("KGX_SHORT_ROWS", "1") in ("0", "false", "False"):
        return n
    smax = int(os.environ.get("KGX_SHORT_MAX", SHORT_ROW_MAX))  # experiment knob (the kernel takes any degree)
    if items.is_cuda:
        return schedule_suffixes(items, smax, smax)[0]
    short = ((items[:, 2] - items[:, 1]) <= smax) & (items[:, 3] < 0)
    # the suffix starts after the last item that is NOT short
    not_short = torch.nonzero(~short)
    return int(not_short[-1]) + 1 if not_short.numel() else 0


def exact_short_start(g: CSRGraph) -> int:
    """EXACT mode (no schedule): the index in g.rows (degree-descending) where the
    suffix of rows of degree <= SHORT_ROW_MAX starts; kgx_spmm reduces that
    suffix with its short-row kernel (each row still one chain in CSR order).
    -1 when there is no such suffix or KGX_SHORT_ROWS=0 (cached per graph)."""
    hit = g.extras.get("exact_short")
    if hit is not None:
        return hit
    n = -1
    if g.rows is not None and g.n_dst > 0 and os.environ.get("KGX_SHORT_ROWS", "1") not in ("0", "false", "False"):
        smax = int(os.environ.get("KGX_SHORT_MAX", SHORT_ROW_MAX))
        k = int((g.deg[g.rows.long()] > smax).sum())  # rows come in descending degree
        n = k if 0 < k < g.n_dst else -1
    g.extras["exact_short"] = n
    return n


def row_of_slot(g: CSRGraph) -> torch.Tensor:
    """int32 [kept]: the destination row of every CSR slot (cached)."""
    r = g.extras.get("row_of_slot")
    if r is None:
        if g.kept:
            r = torch.repeat_interleave(torch.arange(g.n_dst, device=g.device, dtype=torch.int32),
                                        g.deg.long(), output_size=g.kept)
        else:
            r = torch.empty(0, dtype=torch.int32, device=g.device)
        g.extras["row_of_slot"] = r
    return r


def transpose(g: CSRGraph) -> CSRGraph:
    """The reversed graph as a CSR over SOURCE rows (cached on `g`): row j lists
    the edges leaving source j, in input-edge order (the order the reference's
    autograd accumulates x_j's gradient in), `col` = the edge's destination row,
    `w` = the same edge weight.  Built with the same stable kgx_csr_build, so
    sum / mean / weighted-sum backward is one kgx_spmm over it."""
    t = g.extras.get("T")
    if t is not None:
        return t
    if g.kept:
        order = torch.sort(g.eid, stable=True).indices  # slots in input-edge order
        src_t = row_of_slot(g)[order].contiguous()  # reversed edge: dst row -> source
        dst_t = g.col[order].contiguous()
    else:
        order = torch.empty(0, dtype=torch.int64, device=g.device)
        src_t = dst_t = torch.empty(0, dtype=torch.int32, device=g.device)
    t = build_csr(src_t, dst_t, g.n_dst, g.n_src)
    slot = order[t.eid.long()] if t.kept else order  # forward CSR slot of every transposed slot
    t.eid = g.eid[slot].contiguous() if t.kept else g.eid[:0]
    if g.w is not None:
        t.w = g.w[slot].contiguous()
        _refresh_tiny(t)  # the tiny-row records carry the weights
    t.extras["fwd_slot"] = slot
    g.extras["T"] = t
    return t


def split_by_source(g: CSRGraph, n_own: int) -> tuple[CSRGraph, CSRGraph]:
    """Split every CSR row into its edges from sources < n_own ("own") and the
    rest ("other", sources re-based to col - n_own), each part in CSR order and
    carrying its slice of the edge weights.  Used by the sharded layers to start
    on a row's own-source part while its halo rows are still in flight
    (distributed.py); sum(own) + sum(other) re-associates the row's sum, so the
    split path is tolerance-equal, not bit-equal, to the one-pass row."""
    own, other = split_by_source_ranges(g, [0, n_own, g.n_src], accumulate_from=2)
    return own, other


def split_by_source_ranges(g: CSRGraph, cuts: list[int], accumulate_from: int = 1) -> list[CSRGraph]:
    """Split every CSR row by source range: part k holds the row's edges with
    cuts[k] <= col < cuts[k+1] (CSR order kept, sources re-based to cuts[k],
    edge weights sliced along).  The sharded GCN layer runs part 0 (own
    sources) while the halo rows are in flight and then one accumulating pass
    per arrived halo chunk (distributed.py).

    Parts k >= accumulate_from are meant for accumulate-mode launches
    (out += part): their schedules drop the items of rows with no edges in the
    part (a degree-sorted suffix), so such a pass neither reads nor rewrites
    rows it contributes nothing to -- and adds no 0 * W term, which would turn
    -0 into +0 or an inf/NaN weight into NaN where the one-pass row has none."""
    if len(cuts) < 2 or cuts[0] != 0 or cuts[-1] != g.n_src or any(a > b for a, b in zip(cuts, cuts[1:])):
        raise ValueError(f"split_by_source_ranges: cuts must rise from 0 to n_src={g.n_src} (got {cuts})")
    part_of = torch.bucketize(g.col, torch.tensor(cuts[1:-1], dtype=torch.int32, device=g.device), right=True)
    return split_by_part(g, part_of, [(cuts[k], cuts[k + 1] - cuts[k]) for k in range(len(cuts) - 1)],
                         accumulate_from)


def split_by_part(g: CSRGraph, part_of: torch.Tensor, sources: list, accumulate_from: int = 1) -> list[CSRGraph]:
    """Split every CSR row's edges by part_of[slot] in [0, len(sources)): part k
    keeps its edges in CSR order with sources re-based to sources[k] = (base,
    n_src) and the edge weights sliced along.  Parts k >= accumulate_from are
    accumulate-only (see split_by_source_ranges)."""
    row_of = row_of_slot(g)
    parts = []
    for k, (base, n_src) in enumerate(sources):
        m = part_of == k
        deg = torch.bincount(row_of[m], minlength=g.n_dst).to(torch.int32)[: g.n_dst]
        rowptr = torch.zeros(g.n_dst + 1, dtype=torch.int32, device=g.device)
        rowptr[1:] = torch.cumsum(deg, 0)
        col = g.col[m] - base if base else g.col[m]
        kept = int(col.numel())
        sub = CSRGraph(
            n_src=n_src, n_dst=g.n_dst, n_input_edges=kept, kept=kept,
            max_degree=int(deg.max()) if g.n_dst else 0, flags=g.flags,
            rowptr=rowptr, col=col.contiguous(), eid=g.eid[m].contiguous(), deg=deg,
            dinv=g.dinv, w=g.w[m].contiguous() if g.w is not None else None,
        )
        _build_schedule(sub, default_split_len(kept))
        if k >= accumulate_from and sub.n_items:
            empty = int((deg == 0).sum())  # one item each, last in the degree-descending schedule
            sub.n_items -= empty
            sub.items = sub.items[: sub.n_items]
            sub.n_long = min(sub.n_long, sub.n_items)
            sub.extras["accumulate_only"] = True
            _refresh_tiny(sub)
        parts.append(sub)
    return parts


def restrict_rows(g: CSRGraph, row_mask: torch.Tensor) -> CSRGraph:
    """A view of g whose schedule covers only the rows with row_mask[row] set
    (zero-degree ones included): a launch over it writes exactly those rows and
    leaves every other output row untouched.  CSR arrays are shared; the item
    and split lists are filtered in order (the schedule stays degree-descending,
    so the short-row suffix is recomputed and the tiny-row records rebuilt)."""
    from dataclasses import replace

    if g.n_items == 0:
        return replace(g, extras={})
    keep = row_mask[g.items[:, 0].long()]
    items = g.items[keep].contiguous()
    split = g.split[row_mask[g.split[:, 0].long()]].contiguous() if g.n_split else g.split
    sub = replace(g, items=items, split=split, n_items=int(items.shape[0]), n_split=int(split.shape[0]) if g.n_split
                  else 0, extras={"restricted_of": g})
    sub.n_long = short_suffix_start(items)
    _refresh_tiny(sub)
    return sub


# ---------------------------------------------------------------------------
# cache keyed on the caller's edge_index tensor (kept alive by the entry)
# ---------------------------------------------------------------------------
_CACHE: "OrderedDict[tuple, tuple[torch.Tensor, CSRGraph]]" = OrderedDict()
_CACHE_SIZE = int(os.environ.get("KGX_GRAPH_CACHE", "8"))


def host_array_key(a) -> tuple | None:
    """Key of a host (numpy) edge_index.  The reference casts edge_index once
    and caches the cast by id() (message_passing.py:256-268); here the key is
    the id, the data address, shape, strides and dtype, plus a fingerprint of
    4096 evenly spaced elements, so an array modified in place in the sampled
    positions is not served stale (the reference would).  The cache entry
    holds a reference to the array, so its id cannot be reused while cached.
    None for anything that is not an ndarray (a list becomes a new array on
    every call: nothing to key on)."""
    if not isinstance(a, np.ndarray):
        return None
    n = a.size
    pick = np.linspace(0, n - 1, min(n, 4096)).astype(np.int64) if n else np.zeros(0, np.int64)
    sample = np.ascontiguousarray(a.flat[pick])
    return ("host", id(a), a.__array_interface__["data"][0], a.shape, a.strides, a.dtype.str,
            hash(sample.tobytes()))


def cache_key(edge_index: torch.Tensor, *extra) -> tuple | None:
    if not isinstance(edge_index, torch.Tensor):
        hk = host_array_key(edge_index)
        return (*hk, *extra) if hk is not None else None
    return (
        edge_index.data_ptr(), edge_index._version, tuple(edge_index.shape), tuple(edge_index.stride()),
        edge_index.dtype, str(edge_index.device), *extra,
    )


def cached(key: tuple | None, anchor, builder) -> CSRGraph:
    if key is None or _CACHE_SIZE <= 0:
        return builder()
    hit = _CACHE.get(key)
    if hit is not None:
        _CACHE.move_to_end(key)
        return hit[1]
    g = builder()
    _CACHE[key] = (anchor, g)
    while len(_CACHE) > _CACHE_SIZE:
        _CACHE.popitem(last=False)
    return g


def clear_cache() -> None:
    _CACHE.clear()
    from .layers import _edges

    _edges._HOST_CAST.clear()
