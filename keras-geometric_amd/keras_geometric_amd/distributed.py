"""Multi-GPU message passing: destination-range shards + RCCL halo exchange.

No reference counterpart (the reference is single-device).
Every destination row is independent once its source rows are present
(SURVEY.md §8e), so the graph is cut into contiguous destination ranges, one
per process/GPU.  Rank r owns nodes [lo, hi): their feature rows and all their
in-edges (in the global input order, so each row's accumulation order — and
therefore the result — is bit-identical to the single-GPU EXACT result).
Sources owned by other ranks ("halo" rows) arrive once per layer through
all-to-all-v steps over RCCL (torch.distributed "nccl" = RCCL on ROCm, over
xGMI): the send lists are planned once per graph.

GCN layer, default mode (aggregate-then-transform, push-pull halo exchanged in
K chunks; chunk k = the k-th slice of every owner's pull and push lists):
    side stream:  per chunk k: send_k = owner's pulled rows and pushed partial
                  sums (one weighted-sum pass); RCCL all-to-all -> halo[k]
    main stream:  out  = bias + (A_own x_local) W        fused kgx kernel
                  per chunk k: wait for halo[k];
                  out += (A_k halo[k]) W                  same kernel, accumulate
  (each row's sum is split own-sources-then-chunks: tolerance-equal to one GPU)
EXACT mode (and the generic propagate):
    table[:n_local] = x_local (@ W);  table[n_local:] = halo all-to-all
    out = kgx aggregation over the shard CSR in global input order
  (bit-identical to the single-GPU EXACT result)

The device work goes through a backend object; the default is the HIP engine.
Tests substitute a CPU backend built on the oracle to check the planning and
exchange logic under gloo (tests/test_distributed_gloo.py).
"""

from __future__ import annotations

import contextlib
import os
import sys
import threading
import time
from dataclasses import dataclass

import torch
import torch.distributed as dist

from . import _native as nat
from . import graph as G
from . import ops as kops
from .layers.base import Dropout, Layer, get_initializer


class KgxBackend:
    """HIP implementations of the shard's device work (the product path)."""

    def build_graph(self, src: torch.Tensor, dst: torch.Tensor, n_src: int, n_dst: int, n_features: int):
        return G.build_csr(src, dst, n_src, n_dst, n_features=n_features)

    def dinv(self, deg: torch.Tensor) -> torch.Tensor:
        """The reference's dinv (utils/main.py:25) from the ATen-valued table
        (graph.gcn_dinv_table), bit-identical to the one-GPU build."""
        out = torch.empty(deg.numel(), dtype=torch.float32, device=deg.device)
        if deg.numel() == 0:
            return out
        table = G.gcn_dinv_table(deg.device, int(deg.max()))
        nat.check(nat.lib().kgx_gcn_dinv_table(nat.ptr(deg), deg.numel(), nat.ptr(table), table.numel(),
                                               nat.ptr(out), nat.stream(deg.device)), "kgx_gcn_dinv_table")
        return out

    def edge_norm(self, g, dinv_dst: torch.Tensor, dinv_src: torch.Tensor) -> torch.Tensor:
        w = torch.empty(max(g.kept, 1), dtype=torch.float32, device=g.device)
        nat.check(
            nat.lib().kgx_gcn_edge_norm(nat.ptr(g.rowptr), nat.ptr(g.col), g.n_dst, nat.ptr(dinv_dst),
                                        nat.ptr(dinv_src), nat.ptr(w), nat.stream(g.device)),
            "kgx_gcn_edge_norm",
        )
        return w[: g.kept]

    def gather_rows(self, table: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
        return kops.gather_rows(table, rows)

    def transform(self, x: torch.Tensor, W: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
        """Node-level x W (+ bias) (kgx_dense; the library GEMM past its shapes)."""
        return kops.dense(x, W, bias)

    def split_by_source(self, g, cuts: list):
        """Parts of g by source range [cuts[k], cuts[k+1]); every part after the
        first is accumulate-only (graph.split_by_source_ranges)."""
        return G.split_by_source_ranges(g, cuts, accumulate_from=1)

    def supports_fused(self, f_in: int, f_out: int) -> bool:
        return kops.fused_transform_supported(f_in, f_out, two_table=True)  # the sharded passes' gathers

    def aggregate_transform(self, g, x, W, bias=None, out=None, x2=None, accumulate=True, weighted=True,
                            pre_gin=False, gin_scale=1.0, relu=False):
        """Sum (with the GCN edge weights unless weighted=False), then @ W (+
        bias); out += ... if given (accumulate=False: g's scheduled rows of out
        overwritten).  x2: second table for sources >= x.shape[0] (two-table
        gathers).  pre_gin: GIN's gin_scale * x_i + aggr before the product
        (root rows of x); relu: max(., 0) at the store (overwriting launches)."""
        return kops.aggregate_transform(g, x, W, "sum", weighted=weighted, bias=bias, out=out, x2=x2,
                                        accumulate=accumulate, pre_gin=pre_gin, gin_scale=gin_scale, relu=relu)

    def restrict_rows(self, g, row_mask):
        return G.restrict_rows(g, row_mask)

    def gatv2(self, g, h_src, h_dst, att, heads, channels, negative_slope, bias=None, exact=False):
        """GATv2 attention over g (kgx_gatv2: score, segment softmax, weighted
        sum, + bias); h_src rows index g's sources, h_dst its rows."""
        return kops.gatv2_aggregate(g, h_src, h_dst, att, heads, channels, negative_slope, bias=bias, exact=exact)

    def aggregate(self, g, table, reduce="sum", weighted=False, epilogue=nat.EPI_NONE, bias=None, xroot=None,
                  gin_scale=1.0, exact=False):
        return kops.aggregate(g, table, reduce, weighted=weighted, epilogue=epilogue, bias=bias, xroot=xroot,
                              gin_scale=gin_scale, exact=exact)

    def aggregate_transposed(self, g, t, weighted=True):
        """The backward of a (weighted) row sum over g: for every SOURCE row j of
        g, sum over its out-edges e = (j -> i) of w_e t[i] -- one kgx_spmm over
        g's transpose (graph.transpose: rows = g's sources, each row's edges in
        input order)."""
        gt = G.transpose(g)
        return kops.aggregate(gt, t, "sum", weighted=weighted)

    def aggregate_accumulate(self, g, table, out, weighted=False, epilogue=nat.EPI_ACCUM, bias=None, xroot=None,
                             gin_scale=1.0, table2=None):
        """out += the (weighted) row sums of table over g, in place (KGX_EPI_ACCUM);
        another epilogue overwrites g's scheduled rows; table2: second table for
        sources >= table.shape[0]."""
        return kops.aggregate_accumulate(g, table, out, weighted=weighted, epilogue=epilogue, bias=bias,
                                         xroot=xroot, gin_scale=gin_scale, table2=table2)


class TorchComm:
    """Collectives of the product path: torch.distributed on the process group
    ("nccl" = RCCL over xGMI on ROCm)."""

    def __init__(self, group=None):
        self.group = group

    def rank(self) -> int:
        return dist.get_rank(self.group)

    def world(self) -> int:
        return dist.get_world_size(self.group)

    def all_to_all_single(self, out, inp, out_splits=None, in_splits=None) -> None:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def all_to_all_start(self, out, inp, out_splits=None, in_splits=None):
        """Enqueue the all-to-all behind the CURRENT stream's work and return a
        handle whose wait() makes the then-current stream wait for it (RCCL runs
        it on its own stream, so kernels on other streams overlap it)."""
        return dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group, async_op=True)

    def broadcast(self, t, src: int = 0) -> None:
        dist.broadcast(t, src=src, group=self.group)

    def all_reduce(self, t) -> None:
        """t <- the sum of every rank's t (the sharded backward's dW / db)."""
        dist.all_reduce(t, group=self.group)

    def all_gather(self, out, inp) -> None:
        """out = [rank 0's inp | rank 1's inp | ...] (equal sizes)."""
        dist.all_gather_into_tensor(out, inp, group=self.group)

    def all_gather_start(self, out, inp):
        """all_gather behind the CURRENT stream's work; the handle's wait()
        orders the then-current stream after it (as all_to_all_start)."""
        return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True)


class HostStagedComm(TorchComm):
    """Exchange staged through host memory over a gloo group: for rehearsing the
    multi-rank path where RCCL cannot run (ranks sharing one GPU).  Not a
    product path -- bench.py only uses it under KGX_BENCH_REHEARSAL=1."""

    def all_to_all_single(self, out, inp, out_splits=None, in_splits=None) -> None:
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.group)
        out.copy_(o)

    def all_to_all_start(self, out, inp, out_splits=None, in_splits=None):
        self.all_to_all_single(out, inp, out_splits, in_splits)
        return None

    def broadcast(self, t, src: int = 0) -> None:
        h = t.detach().cpu()
        dist.broadcast(h, src=src, group=self.group)
        t.copy_(h)

    def all_reduce(self, t) -> None:
        h = t.detach().cpu()
        dist.all_reduce(h, group=self.group)
        t.copy_(h)

    def all_gather(self, out, inp) -> None:
        h = inp.detach().cpu()
        parts = [torch.empty_like(h) for _ in range(dist.get_world_size(self.group))]
        dist.all_gather(parts, h, group=self.group)
        out.copy_(torch.cat(parts))

    def all_gather_start(self, out, inp):
        self.all_gather(out, inp)
        return None


def _inference_only(layer: Layer, weights) -> None:
    """The sharded layers are a forward (inference) engine: their kernels run
    under no_grad, so an output would carry no gradient to the weights."""
    if torch.is_grad_enabled() and any(p.requires_grad for p in weights):
        raise NotImplementedError(
            f"{type(layer).__name__} is inference-only here: call it under torch.no_grad() (or freeze its "
            "weights); training runs on the single-GPU layers, ShardedGCNConv, and ShardedGINConv / "
            "ShardedSAGEConv with a sum or mean aggregator")


# where progress and heartbeat lines go (stderr; tests substitute a buffer)
LOG_STREAM = None


def _log_line(rank: int, msg: str) -> None:
    print(f"[kgx r{rank}] {msg}", file=LOG_STREAM or sys.stderr, flush=True)


def _progress(sg, msg: str) -> None:
    """One progress line per rank on stderr when KGX_LOG is set (bench.py sets
    it for N > 1: the shard build, each exchange plan and each tuner
    candidate stay visible, rank by rank, so a stalled rank is named)."""
    if os.environ.get("KGX_LOG"):
        _log_line(sg.rank, msg)


@contextlib.contextmanager
def heartbeat(rank: int, what: str, every_s: float | None = None):
    """While the block runs, a line '[kgx r<rank>] <what>: running, <t> s' every
    KGX_HEARTBEAT_S seconds (default 30) from a daemon thread, plus one when
    it ends: a first forward that stalls (a collective waiting on a peer, a
    long tune) is reported, not silent.  bench.py wraps the N > 1 shard build
    and first forward in it."""
    every = float(os.environ.get("KGX_HEARTBEAT_S", "30")) if every_s is None else float(every_s)
    stop = threading.Event()
    t0 = time.perf_counter()

    def beat():
        while not stop.wait(every):
            _log_line(rank, f"{what}: running, {time.perf_counter() - t0:.0f} s")

    th = threading.Thread(target=beat, name=f"kgx-heartbeat-{rank}", daemon=True)
    th.start()
    try:
        yield
    finally:
        stop.set()
        th.join(timeout=5)
        _log_line(rank, f"{what}: done in {time.perf_counter() - t0:.1f} s")


def equal_bounds(n_global: int, world: int) -> list[int]:
    base, rem = divmod(n_global, world)
    b = [0]
    for r in range(world):
        b.append(b[-1] + base + (1 if r < rem else 0))
    return b


def default_halo_chunks(world: int) -> int:
    """Exchange steps per layer (KGX_HALO_CHUNKS overrides; every rank must use
    the same count).  The halo volume is a property of the graph (DESIGN.md
    §6: ~6 GB per rank per layer at 8 weak-scaled shards), so a single
    all-to-all leaves the halo pass waiting for all of it; in chunks, pass k
    runs while chunk k+1 is on the links, for about one extra read-modify-write
    of the rows each pass touches."""
    v = os.environ.get("KGX_HALO_CHUNKS")
    if v:
        return max(1, int(v))
    # 2: one rank's device work at 8 weak shards (tools/shard_sim.py, exchange
    # free) is 15.5 / 16.4 / 18.0 ms at K = 1 / 2 / 4, and at an all-to-all rate
    # near 400 GB/s per GPU K = 2 hides half of the ~9 ms exchange
    return 2 if world > 1 else 1


def use_push_pull() -> bool:
    """The default GCN path exchanges the push-pull halo (KGX_HALO_PUSH=0: pull only)."""
    return os.environ.get("KGX_HALO_PUSH", "1") not in ("0", "", "false", "False")


def _merge_unit(unit: str) -> str:
    """merged_passes' unit.  The tuner's "group" candidates name group_passes
    (cached as pp.merged["group"]); a layer without group passes
    (propagate_overlapped) sharing the graph merges the same plan's steps."""
    return unit if unit in ("step", "chunk", "none") else "step"


def prune_pulls() -> bool:
    """push_pull_plan drops pulled sources whose rows are all pushed anyway
    (KGX_HALO_PRUNE=0: keep them; read when a plan is built)."""
    return os.environ.get("KGX_HALO_PRUNE", "1") not in ("0", "", "false", "False")


@dataclass
class HaloChunk:
    """One exchange step.  Every rank sends each peer the k-th slice of the
    rows that peer requested from it and receives the k-th slice of each of its
    own requests, into the contiguous halo-table rows [lo, hi) (the halo table
    is chunk-major, then grouped by owner)."""
    lo: int
    hi: int
    recv_splits: list
    send_splits: list
    send_rows: torch.Tensor  # int32 local rows to send, grouped by destination rank
    # push-pull plan: the send rows are one weighted-sum pass over this CSR
    # (pushed partial sums)
    send_graph: object = None
    # a push-pull chunk: its exchange steps (pulled rows, then partials), each
    # landing in its own contiguous slice of [lo, hi)
    steps: list | None = None
    # "a2a": all-to-all-v of send rows; "allgather": every rank contributes its
    # local rows [src_lo, src_hi), padded to `pad` rows, and receives all ranks'
    kind: str = "a2a"
    src_lo: int = 0
    src_hi: int = 0
    pad: int = 0


@dataclass
class PushPullPlan:
    """Halo plan of the default GCN path (ShardedGraph.push_pull_plan)."""
    chunks: list  # HaloChunk per exchange step, send rows packed by send_graph
    parts: list  # receiver CSR per chunk: sources = that chunk's halo rows (accumulate-only)
    n_rows: int  # halo rows received per layer
    n_pull: int  # of which source rows
    n_push: int  # of which partial sums pushed by the owners
    recv_graph: object = None  # receiver CSR over all halo rows (sources = halo buffer rows)
    step_parts: list | None = None  # receiver CSR per exchange step, in issue order (accumulate-only)
    weighted: bool = True  # receiver edges carry the GCN norms (else weight 1, plain partial sums)
    kind: str = "halo"  # "halo" (push-pull all-to-all), "pull" (the same all-to-all, pulled rows only) or "allgather" (every rank's rows, chunked)
    merged: dict | None = None  # unit -> (own pass, first-group pass, later groups, first wait): merged_passes
    row_group: object = None  # kind "group": each local row's destination group (group_passes)


class _Works:
    """The handles of one chunk's exchange steps: wait() orders the current
    stream after all of them."""

    def __init__(self, handles):
        self.handles = handles

    def wait(self):
        for h in self.handles:
            if h is not None:
                h.wait()


def halo_first_frac() -> float | None:
    """KGX_HALO_FIRST (0 < f < 1): the push-pull plan's first exchange chunk
    takes this fraction of every peer list and the other K - 1 chunks split the
    rest evenly -- a small first chunk lands sooner, so the passes that need
    halo rows start earlier while the larger chunks are on the links.  Unset:
    K even chunks."""
    v = os.environ.get("KGX_HALO_FIRST")
    if not v:
        return None
    f = float(v)
    if not 0.0 < f < 1.0:
        raise ValueError(f"KGX_HALO_FIRST must lie in (0, 1), got {v!r}")
    return f


def halo_chunk_weights(K: int) -> tuple | None:
    """KGX_HALO_WEIGHTS (measurement): K comma-separated relative sizes of the
    push-pull plan's slice chunks (e.g. "1,4,1": small first and last chunks).
    Applied only when it names exactly K positive weights; overrides
    KGX_HALO_FIRST.  Unset: None."""
    v = os.environ.get("KGX_HALO_WEIGHTS")
    if not v or K <= 1:
        return None
    w = tuple(float(t) for t in v.split(","))
    if len(w) != K or any(t <= 0 for t in w):
        return None
    return w


def chunk_slice(count: int, k: int, K: int, first: float | tuple | None = None) -> tuple[int, int]:
    """[a, b) of chunk k of a list of `count` rows cut K ways: evenly
    (floor(count k / K)); with chunk 0 holding floor(count * first) rows and
    chunks 1..K-1 splitting the rest evenly; or, `first` a tuple of K weights,
    at the weights' cumulative fractions.  Requester and owner compute it
    from the same count, so both sides agree on every chunk."""
    if first is None or K == 1:
        return count * k // K, count * (k + 1) // K
    if isinstance(first, tuple):
        tot = sum(first)
        return int(count * (sum(first[:k]) / tot)), (count if k == K - 1 else int(count * (sum(first[:k + 1]) / tot)))
    f = int(count * first)
    if k == 0:
        return 0, f
    rest = count - f
    return f + rest * (k - 1) // (K - 1), f + rest * k // (K - 1)


def _prefix(v: list) -> list:
    out = [0]
    for c in v:
        out.append(out[-1] + c)
    return out


def _plan_chunks(requested_local: torch.Tensor, send_counts: list, recv_counts: list, n_chunks: int,
                 dev) -> tuple[list, torch.Tensor]:
    """(chunks, pos): pos[i] = halo-table row of the i-th sorted halo id.  The
    slice bounds floor(count*k/K) are computed identically by the requester and
    the owner from the same count, so both sides agree on every chunk."""
    K = max(1, n_chunks)
    rstart = [0]
    for c in recv_counts:
        rstart.append(rstart[-1] + c)
    sstart = [0]
    for c in send_counts:
        sstart.append(sstart[-1] + c)
    pos = torch.empty(rstart[-1], dtype=torch.long, device=dev)
    chunks, off = [], 0
    for k in range(K):
        recv_splits, send_splits, send_parts = [], [], []
        lo = off
        for p, R in enumerate(recv_counts):
            a, b = rstart[p] + R * k // K, rstart[p] + R * (k + 1) // K
            pos[a:b] = torch.arange(off, off + b - a, device=dev)
            off += b - a
            recv_splits.append(b - a)
        for p, S in enumerate(send_counts):
            a, b = sstart[p] + S * k // K, sstart[p] + S * (k + 1) // K
            send_parts.append(requested_local[a:b])
            send_splits.append(b - a)
        rows = torch.cat(send_parts) if send_parts else requested_local[:0]
        chunks.append(HaloChunk(lo=lo, hi=off, recv_splits=recv_splits, send_splits=send_splits,
                                send_rows=rows.to(torch.int32).contiguous()))
    return chunks, pos


@dataclass
class ShardedGraph:
    rank: int
    world: int
    n_global: int
    bounds: list[int]
    graph: object  # CSRGraph over local rows; sources index [own rows | halo rows]
    send_counts: list[int]  # rows this rank sends to each rank per layer
    recv_counts: list[int]  # halo rows this rank receives from each rank per layer
    halo_ids: torch.Tensor  # global ids of halo rows in table order (chunk-major)
    chunks: list  # one HaloChunk per exchange step
    dinv_table: torch.Tensor | None
    backend: object
    comm: object = None
    exact: bool = False
    _parts: tuple | None = None  # (own-source CSR, [halo-chunk CSRs]), built on first use
    _side: object = None  # HIP stream for the halo exchange
    _halo_buf: dict | None = None
    _pp: PushPullPlan | None = None  # the push-pull plan last used
    _pp_by_k: dict | None = None
    chunks_fixed: bool = False  # K given (halo_chunks= or KGX_HALO_CHUNKS): no tuning
    halo_k: int | None = None  # exchange chunk count chosen by tune_exchange (or fixed)
    tuning: dict | None = None  # K (or "exchange:K") -> slowest rank's forward seconds
    exchange: str | None = None  # "halo" / "pull" / "allgather"; None: not chosen yet (push-pull halo until tuned)
    merge_unit: str | None = None  # merged_passes' unit ("step" / "chunk" / "none"); None: KGX_HALO_MERGE or "step"
    tuning_s: float | None = None  # wall time tune_exchange took on this rank
    tuning_skipped: int = 0  # candidates left untimed once KGX_TUNE_BUDGET_S was spent
    self_loops: bool = True  # the shard graph carries utils/main.py:8-16's self loops (GCN, GATv2)
    link_probe: list | None = None  # a list: time every exchange step's landing (bench.py N > 1; link_report)
    _probe_stream: object = None
    packs_done: object = None  # event: the side stream after every step's packing

    @property
    def lo(self) -> int:
        return self.bounds[self.rank]

    @property
    def n_local(self) -> int:
        return self.bounds[self.rank + 1] - self.bounds[self.rank]

    @property
    def n_halo(self) -> int:
        return int(self.halo_ids.numel())

    # -- construction -------------------------------------------------------
    @classmethod
    def build(cls, src: torch.Tensor, dst: torch.Tensor, bounds: list[int], *, comm=None,
              self_loops: bool = True, gcn_norm: bool = True, backend=None, n_features: int = 128,
              exact: bool = False, halo_chunks: int | None = None) -> "ShardedGraph":
        """src/dst: this rank's edges (global ids, int32) whose dst lies in its range,
        in global input order.  halo_chunks: exchange steps per layer (the same
        on every rank; default `default_halo_chunks`)."""
        backend = backend or KgxBackend()
        comm = comm or TorchComm()
        rank, world = comm.rank(), comm.world()
        n_chunks = default_halo_chunks(world) if halo_chunks is None else max(1, int(halo_chunks))
        chunks_fixed = halo_chunks is not None or bool(os.environ.get("KGX_HALO_CHUNKS"))
        lo, hi = bounds[rank], bounds[rank + 1]
        n_local = hi - lo
        dev = src.device
        src = src.long()
        dst = dst.long()
        if dst.numel() and (int(dst.min()) < lo or int(dst.max()) >= hi):
            raise ValueError("ShardedGraph.build: an edge's destination lies outside this rank's range")
        if src.numel() and (int(src.min()) < 0 or int(src.max()) >= bounds[-1]):
            raise IndexError("ShardedGraph.build: source id outside the global node range")
        log = bool(os.environ.get("KGX_LOG"))
        if log:
            _log_line(rank, f"shard build: rows [{lo}, {hi}), {src.numel()} in-edges; halo request lists")
        local = (src >= lo) & (src < hi)
        halo_ids = torch.unique(src[~local])  # sorted -> grouped by owner
        bt = torch.tensor(bounds[1:-1], dtype=torch.long, device=dev)
        owners = torch.bucketize(halo_ids, bt, right=True)
        recv_counts_t = torch.bincount(owners, minlength=world)
        send_counts_t = torch.empty_like(recv_counts_t)
        comm.all_to_all_single(send_counts_t, recv_counts_t)
        recv_counts = [int(v) for v in recv_counts_t.cpu()]
        send_counts = [int(v) for v in send_counts_t.cpu()]
        requested = torch.empty(sum(send_counts), dtype=torch.long, device=dev)
        comm.all_to_all_single(requested, halo_ids, send_counts, recv_counts)
        chunks, pos = _plan_chunks(requested - lo, send_counts, recv_counts, n_chunks, dev)
        if pos.numel():
            hidx = torch.searchsorted(halo_ids, src).clamp_(max=pos.numel() - 1)
            col = torch.where(local, src - lo, n_local + pos[hidx])
        else:
            col = src - lo
        halo_table_ids = torch.empty_like(halo_ids)
        halo_table_ids[pos] = halo_ids
        row = dst - lo
        if self_loops:  # utils/main.py:8-16 — loop i after all input edges
            ar = torch.arange(n_local, device=dev)
            col = torch.cat([col, ar])
            row = torch.cat([row, ar])
        n_src = n_local + int(halo_ids.numel())
        if log:
            _log_line(rank, f"shard build: {halo_ids.numel()} halo rows; shard CSR + schedule")
        g = backend.build_graph(col.to(torch.int32).contiguous(), row.to(torch.int32).contiguous(), n_src, n_local,
                                n_features)
        sg = cls(rank=rank, world=world, n_global=bounds[-1], bounds=list(bounds), graph=g,
                 send_counts=send_counts, recv_counts=recv_counts, halo_ids=halo_table_ids.to(torch.int32),
                 chunks=chunks, dinv_table=None, backend=backend, comm=comm, exact=exact, chunks_fixed=chunks_fixed,
                 self_loops=self_loops)
        if gcn_norm:
            dinv_local = backend.dinv(g.deg)
            table = torch.empty((n_src, 1), dtype=torch.float32, device=dev)
            table[:n_local, 0] = dinv_local
            sg.halo_exchange(table)
            sg.dinv_table = table[:, 0].contiguous()
            g.dinv = dinv_local
            g.w = backend.edge_norm(g, dinv_local, sg.dinv_table)
        return sg

    @classmethod
    def rmat(cls, n_global: int, e_global: int, seed: int = 0, device=None, comm=None, **kw) -> "ShardedGraph":
        """Shard of the global synthetic R-MAT graph (every rank generates the same
        edge stream and keeps its destination range; no communication)."""
        from . import synthetic

        comm = comm or TorchComm()
        rank, world = comm.rank(), comm.world()
        bounds = equal_bounds(n_global, world)
        ei = synthetic.rmat_dst_shard(n_global, e_global, bounds[rank], bounds[rank + 1], seed=seed, device=device)
        return cls.build(ei[0], ei[1], bounds, comm=comm, **kw)

    # -- per layer ----------------------------------------------------------
    def new_table(self, features: int, like: torch.Tensor) -> torch.Tensor:
        return torch.empty((self.n_local + self.n_halo, features), dtype=torch.float32, device=like.device)

    def _pack(self, x_local: torch.Tensor, c: HaloChunk) -> torch.Tensor:
        if c.kind == "allgather":  # a contiguous slice of the layer input; padded only when short
            rows = x_local[c.src_lo: c.src_hi]
            if rows.shape[0] == c.pad:
                return rows
            buf = x_local.new_zeros((c.pad, x_local.shape[1]))
            buf[: rows.shape[0]] = rows
            return buf
        if c.send_graph is not None:
            return self.backend.aggregate(c.send_graph, x_local, "sum", weighted=True)
        if c.send_rows.numel():
            return self.backend.gather_rows(x_local, c.send_rows)
        return x_local.new_empty((0, x_local.shape[1]))

    def push_pull_plan(self, n_chunks: int | None = None, weighted: bool | None = None,
                       pull_only: bool = False, groups: bool = False) -> PushPullPlan:
        """A smaller halo for the weighted-sum (GCN) path.  Collective: every
        rank calls it once (ShardedGCNConv does, on its first forward).

        Pulling a source row serves all of its edges into this rank; an owner
        pushing the partial sum sum_e w_e x_src of one destination row serves
        all of that row's edges from the owner.  Per peer the rows moved must
        cover every halo edge (a vertex cover of the bipartite halo graph);
        pull-only takes every source, push-only every destination.  Here each
        edge goes to its endpoint of larger degree in that bipartite graph
        (ties: pull), and a destination is pushed only for edges whose source is
        not pulled anyway.  On power-law R-MAT shards that moves ~40 % fewer
        rows than pulling (1/10-scale probe at 8 shards: 0.72M vs 1.26M rows).
        A pushed partial enters the receiver's CSR as one edge of weight 1; the
        owner packs pulled rows and partials in one weighted-sum pass over a
        send CSR (a pulled row = one edge of weight 1, multiplied exactly).
        Row sums are re-associated (partials first), so this is a tolerance
        path like the rest of the overlapped layer; EXACT mode keeps pulling.

        weighted (default: the graph carries edge weights) says whether the
        receiver's pass multiplies by them: an unweighted plan (GIN / SAGE sums
        on a graph that also has GCN norms) pushes plain partial sums and gives
        every receiver edge weight 1, so the plans are kept per (K, weighted).

        pull_only (exchange kind "pull"): every halo edge is served by pulling
        its source -- more rows on the links, but no partial sums for the
        owner to compute and write and the receiver to read back; which wins
        depends on the link rate, so the tuner times both.

        groups (exchange kind "group"): the chunks follow DESTINATION row
        groups instead of slices of the request lists.  The local rows with
        halo edges are cut into K groups of about equal halo-edge counts (the
        first one KGX_HALO_FIRST of them when set); chunk k carries group k's
        pushed partials and the pulled sources group k needs that no earlier
        group needed (a source goes with the first group that reads it).  So
        once chunk k has landed, every halo row of group k's rows is present
        and ONE two-table pass writes each of those rows once
        (ShardedGraph.group_passes) -- no accumulating pass re-reads and
        rewrites a row per chunk.  The bytes moved are the same as the
        slice-chunked plan's."""
        K = n_chunks or self.halo_k or len(self.chunks)
        if weighted is None:
            weighted = self.graph.w is not None
        if weighted and self.graph.w is None:
            raise ValueError("push_pull_plan(weighted=True): the shard graph has no edge weights")
        if self._pp_by_k is None:
            self._pp_by_k = {}
        first = halo_first_frac() if K > 1 else None
        if not groups and halo_chunk_weights(K) is not None:
            first = halo_chunk_weights(K)
        key = ("group" if groups else ("pull" if pull_only else "halo"), K, weighted, first)
        if key in self._pp_by_k:
            self._pp = self._pp_by_k[key]
            return self._pp
        _progress(self, f"{key[0]} plan: K {K}, weighted {weighted}")
        g, comm, world, lo, n_local = self.graph, self.comm, self.world, self.lo, self.n_local
        dev = g.col.device
        rows = torch.repeat_interleave(torch.arange(g.n_dst, device=dev), g.deg.long())
        col = g.col.long()
        halo = col >= n_local
        hs = self.halo_ids.long()[col[halo] - n_local]  # global source id per halo edge
        hd = rows[halo]
        hw = g.w[halo] if weighted else torch.ones(hd.numel(), dtype=torch.float32, device=dev)
        bt = torch.tensor(self.bounds[1:-1], dtype=torch.long, device=dev)
        us, inv_s, cs = torch.unique(hs, return_inverse=True, return_counts=True)
        stride = n_local + 1
        ud, inv_d, cd = torch.unique(torch.bucketize(hs, bt, right=True) * stride + hd, return_inverse=True,
                                     return_counts=True)
        push = cd[inv_d] > cs[inv_s]  # the edge is served from its busier endpoint
        if pull_only:
            push = torch.zeros_like(push)
        pulled = torch.zeros(us.numel(), dtype=torch.bool, device=dev)
        pulled[inv_s[~push]] = True
        via_pull = pulled[inv_s]
        used = torch.zeros(ud.numel(), dtype=torch.bool, device=dev)
        used[inv_d[~via_pull]] = True
        if not pull_only and prune_pulls():
            # a pulled source whose every halo edge lands in a row that is pushed
            # anyway is not pulled: its edges join those partials.  Dropping sources
            # never un-pushes a row, so one pass finds them all.  R-MAT at 8 shards
            # (tools/exp_cover.py): 2.6 % fewer rows moved, against 3.9 % for a
            # minimum vertex cover
            dest_pushed = torch.ones(us.numel(), dtype=torch.int32, device=dev)
            dest_pushed.scatter_reduce_(0, inv_s, used[inv_d].to(torch.int32), "amin")
            pulled &= dest_pushed == 0
            via_pull = pulled[inv_s]
        pull_ids = us[pulled]  # sorted -> grouped by owner
        push_keys = ud[used]  # sorted -> owner-major, then destination row
        push_owner = push_keys // stride
        push_row_of_key = torch.cumsum(used.long(), 0) - 1
        pull_cnt = torch.bincount(torch.bucketize(pull_ids, bt, right=True), minlength=world)
        push_cnt = torch.bincount(push_owner, minlength=world)
        pe = ~via_pull  # edges served by a pushed partial, grouped by push row
        pe_row = push_row_of_key[inv_d[pe]]
        order = torch.argsort(pe_row, stable=True)
        pe_row, pe_src, pe_w = pe_row[order], hs[pe][order], hw[pe][order]
        pe_owner = push_owner[pe_row]
        pe_cnt = torch.bincount(pe_owner, minlength=world)
        pull_owner = torch.bucketize(pull_ids, bt, right=True)
        if groups:
            # destination groups of about equal halo-edge counts, in row order
            hdeg = torch.bincount(hd, minlength=n_local)
            cum = torch.cumsum(hdeg, 0) - hdeg  # halo edges of the rows before each row
            tot = max(int(hdeg.sum()), 1)
            if first is None:
                grp = (cum * K) // tot
            else:  # group 0: the first `first` of the halo edges, the rest in K - 1 even groups
                f = int(tot * first)
                grp = torch.where(cum < f, torch.zeros_like(cum), 1 + ((cum - f) * (K - 1)) // max(tot - f, 1))
            grp = grp.clamp_(max=K - 1)
            # a pulled source travels with the first group that reads it; a partial with its row's group
            ce = grp[hd]
            src_chunk = torch.full((us.numel(),), K, dtype=torch.long, device=dev)
            src_chunk.scatter_reduce_(0, inv_s[via_pull], ce[via_pull], "amin")
            pull_chunk = src_chunk[pulled]
            push_chunk = grp[push_keys % stride]
            # (owner, chunk, id) order for the pull list, (owner, chunk, row) for the push list
            pull_perm = torch.argsort(pull_owner * K + pull_chunk, stable=True)
            push_perm = torch.argsort(push_owner * K + push_chunk, stable=True)
            push_rank = torch.empty_like(push_perm)
            push_rank[push_perm] = torch.arange(push_perm.numel(), device=dev)
            # push row index within its owner, in the new order
            pe_slot = push_rank[pe_row] - (torch.cumsum(push_cnt, 0) - push_cnt)[pe_owner]
            pull_cnt_k = torch.bincount(pull_owner * K + pull_chunk, minlength=world * K).view(world, K)
            push_cnt_k = torch.bincount(push_owner * K + push_chunk, minlength=world * K).view(world, K)
        else:
            pull_perm = push_perm = None
            pe_slot = pe_row - (torch.cumsum(push_cnt, 0) - push_cnt)[pe_owner]  # push row index within its owner
            pull_cnt_k = pull_cnt.view(world, 1)
            push_cnt_k = push_cnt.view(world, 1)
        kk = pull_cnt_k.shape[1]
        counts = torch.cat([pull_cnt_k, push_cnt_k, pe_cnt.view(world, 1)], 1).reshape(-1).contiguous()
        counts_in = torch.empty_like(counts)
        comm.all_to_all_single(counts_in, counts)
        co, ci = counts.view(world, 2 * kk + 1).cpu().tolist(), counts_in.view(world, 2 * kk + 1).cpu().tolist()
        r_pull_k, r_push_k = [c[:kk] for c in co], [c[kk: 2 * kk] for c in co]
        s_pull_k, s_push_k = [c[:kk] for c in ci], [c[kk: 2 * kk] for c in ci]
        r_pull, r_push, r_pe = [sum(v) for v in r_pull_k], [sum(v) for v in r_push_k], [c[2 * kk] for c in co]
        s_pull, s_push, s_pe = [sum(v) for v in s_pull_k], [sum(v) for v in s_push_k], [c[2 * kk] for c in ci]

        def cut(count_k, count, k):
            """[a, b) of chunk k within one peer's list: per-group counts, or chunk_slice."""
            if groups:
                a = sum(count_k[:k])
                return a, a + count_k[k]
            return chunk_slice(count, k, K, first)

        def exchange(t, dtype, s, r):
            out = torch.empty(sum(s), dtype=dtype, device=dev)
            comm.all_to_all_single(out, t.contiguous(), s, r)
            return out

        req_pull = exchange(pull_ids if pull_perm is None else pull_ids[pull_perm], torch.long, s_pull, r_pull) - lo
        req_slot = exchange(pe_slot, torch.long, s_pe, r_pe)
        req_src = exchange(pe_src, torch.long, s_pe, r_pe) - lo
        req_w = exchange(pe_w, torch.float32, s_pe, r_pe)

        # Per chunk k, two exchange steps: the pulled rows (slice k of every
        # requester's pull list; the owner packs them with kgx_gather_rows, a
        # plain copy) and the pushed partial sums (slice k of every push list;
        # one weighted-sum pass over a send CSR).  Packing the pulled rows as
        # one-edge CSR rows made the pack latency-bound: a dependent chain of
        # item, index and row loads per row, 6.4 ms for 12.7 GB at 8 shards
        # (tools/shard_sim.py).  The receiver lands chunk k as [pulled rows from
        # every peer | partials from every peer].
        sp, spe = _prefix(s_pull), _prefix(s_pe)
        rp, ru = _prefix(r_pull), _prefix(r_push)
        pull_pos = torch.empty(rp[-1], dtype=torch.long, device=dev)
        push_pos = torch.empty(ru[-1], dtype=torch.long, device=dev)
        none_i32 = torch.empty(0, dtype=torch.int32, device=dev)
        chunks, off = [], 0
        for k in range(K):
            lo_k = off
            rows, pull_send, pull_recv = [], [], []
            for r in range(world):
                a, b = (sp[r] + v for v in cut(s_pull_k[r], s_pull[r], k))
                rows.append(req_pull[a:b])
                pull_send.append(b - a)
            for p in range(world):  # receiver side: where chunk k's pulled rows from p land
                a, b = cut(r_pull_k[p], r_pull[p], k)
                pull_pos[rp[p] + a: rp[p] + b] = torch.arange(off, off + b - a, device=dev)
                off += b - a
                pull_recv.append(b - a)
            pull_step = HaloChunk(lo=lo_k, hi=off, recv_splits=pull_recv, send_splits=pull_send,
                                  send_rows=torch.cat(rows).to(torch.int32).contiguous() if rows else none_i32)
            cols, slots, ws, push_send, push_recv = [], [], [], [], []
            n_slots, push_lo = 0, off
            for r in range(world):
                j0, j1 = cut(s_push_k[r], s_push[r], k)
                sl = req_slot[spe[r]: spe[r + 1]]
                m = (sl >= j0) & (sl < j1)
                cols.append(req_src[spe[r]: spe[r + 1]][m])
                slots.append(n_slots + sl[m] - j0)
                ws.append(req_w[spe[r]: spe[r + 1]][m])
                n_slots += j1 - j0
                push_send.append(j1 - j0)
            for p in range(world):  # receiver side: where chunk k's partials from p land
                j0, j1 = cut(r_push_k[p], r_push[p], k)
                push_pos[ru[p] + j0: ru[p] + j1] = torch.arange(off, off + j1 - j0, device=dev)
                off += j1 - j0
                push_recv.append(j1 - j0)
            send_graph = None
            if n_slots:
                send_graph = self.backend.build_graph(torch.cat(cols).to(torch.int32), torch.cat(slots).to(torch.int32),
                                                      n_local, n_slots, 128)
                send_graph.w = torch.cat(ws)[send_graph.eid.long()].contiguous()
            push_step = HaloChunk(lo=push_lo, hi=off, recv_splits=push_recv, send_splits=push_send,
                                  send_rows=none_i32, send_graph=send_graph)
            chunks.append(HaloChunk(lo=lo_k, hi=off, recv_splits=[], send_splits=[], send_rows=none_i32,
                                    steps=[pull_step, push_step]))
        if groups:  # positions were assigned in the (owner, chunk, ...) order: back to sorted-id / key order
            pp_sorted = torch.empty_like(pull_pos)
            pp_sorted[pull_perm] = pull_pos
            pull_pos = pp_sorted
            pu_sorted = torch.empty_like(push_pos)
            pu_sorted[push_perm] = push_pos
            push_pos = pu_sorted
        # receiver CSR over the received rows: pulled rows keep their edges and
        # weights; a pushed partial is one edge of weight 1 into its row
        pidx = torch.searchsorted(pull_ids, hs[via_pull])
        rcol = torch.cat([pull_pos[pidx], push_pos])
        rrow = torch.cat([hd[via_pull], push_keys % stride])
        rw = torch.cat([hw[via_pull], torch.ones(push_keys.numel(), dtype=torch.float32, device=dev)])
        parts, step_parts, rg = [], [], None
        if off:
            rg = self.backend.build_graph(rcol.to(torch.int32), rrow.to(torch.int32), off, n_local, 128)
            rg.w = rw[rg.eid.long()].contiguous()
            # a leading empty range makes every chunk part accumulate-only
            parts = list(self.backend.split_by_source(rg, [0, 0] + [c.hi for c in chunks])[1:])
            step_parts = list(self.backend.split_by_source(rg, [0, 0] + [st.hi for c in chunks for st in c.steps])[1:])
        self._pp = PushPullPlan(chunks=chunks, parts=parts, n_rows=off, n_pull=rp[-1], n_push=ru[-1], recv_graph=rg,
                                step_parts=step_parts, weighted=weighted, kind=key[0])
        if groups:
            self._pp.row_group = grp  # [n_local]: the destination group of each row with halo edges
        self._pp_by_k[key] = self._pp
        return self._pp

    def allgather_plan(self, n_chunks: int = 1, weighted: bool | None = None) -> PushPullPlan:
        """Exchange plan that moves EVERY rank's rows: K all-gathers (RCCL over
        xGMI), chunk k = rows [k cs, (k+1) cs) of every rank (cs = ceil(max
        rank rows / K)), landing chunk-major in a [K * world * cs] table.  No
        request lists, no packing kernel (each step sends a contiguous slice of
        the layer input), no partial sums: worth it when the graph's remote
        sources cover most of the other ranks' rows anyway -- SURVEY.md §8(e)
        proposes it for C5, whose X is 0.98 GB.  The receiver CSR maps each
        remote edge to its source's table row."""
        K = max(1, int(n_chunks))
        if weighted is None:
            weighted = self.graph.w is not None
        key = ("allgather", K, weighted)
        if self._pp_by_k is None:
            self._pp_by_k = {}
        if key in self._pp_by_k:
            self._pp = self._pp_by_k[key]
            return self._pp
        g, world, n_local = self.graph, self.world, self.n_local
        dev = g.col.device
        sizes = [b - a for a, b in zip(self.bounds, self.bounds[1:])]
        cs = max(1, -(-max(sizes) // K))
        span = world * cs
        rows = torch.repeat_interleave(torch.arange(g.n_dst, device=dev), g.deg.long(), output_size=g.kept)
        col = g.col.long()
        remote = col >= n_local
        gid = self.halo_ids.long()[col[remote] - n_local]
        bt = torch.tensor(self.bounds[1:-1], dtype=torch.long, device=dev)
        owner = torch.bucketize(gid, bt, right=True)
        i = gid - torch.tensor(self.bounds[:-1], dtype=torch.long, device=dev)[owner]
        k = i // cs
        pos = k * span + owner * cs + (i - k * cs)
        n_rows = K * span
        none_i32 = torch.empty(0, dtype=torch.int32, device=dev)
        chunks = []
        for kk in range(K):
            a, b = min(kk * cs, n_local), min((kk + 1) * cs, n_local)
            st = HaloChunk(lo=kk * span, hi=(kk + 1) * span, recv_splits=[], send_splits=[], send_rows=none_i32,
                           kind="allgather", src_lo=a, src_hi=b, pad=cs)
            chunks.append(HaloChunk(lo=st.lo, hi=st.hi, recv_splits=[], send_splits=[], send_rows=none_i32,
                                    steps=[st], kind="allgather"))
        parts, rg = [], None
        if int(remote.sum()):
            rg = self.backend.build_graph(pos.to(torch.int32), rows[remote].to(torch.int32), n_rows, n_local, 128)
            wr = g.w[remote] if weighted else torch.ones(int(remote.sum()), dtype=torch.float32, device=dev)
            rg.w = wr[rg.eid.long()].contiguous()
            parts = list(self.backend.split_by_source(rg, [0, 0] + [c.hi for c in chunks])[1:])
        self._pp = PushPullPlan(chunks=chunks, parts=parts, n_rows=n_rows, n_pull=n_rows - K * cs, n_push=0,
                                recv_graph=rg, step_parts=list(parts), weighted=weighted, kind="allgather")
        self._pp_by_k[key] = self._pp
        return self._pp

    def exchange_plan(self, n_chunks: int | None = None, weighted: bool | None = None) -> PushPullPlan:
        """The plan of the chosen exchange ("halo": push-pull all-to-all; "allgather";
        not chosen yet: KGX_EXCHANGE, else the halo)."""
        kind = self.exchange or os.environ.get("KGX_EXCHANGE", "halo")
        if kind == "allgather":
            return self.allgather_plan(n_chunks or self.halo_k or len(self.chunks), weighted)
        return self.push_pull_plan(n_chunks, weighted, pull_only=kind == "pull", groups=kind == "group")

    def exchange_candidates(self, halo_ks=(1, 2, 4), gather_ks=(1, 2, 4), units=("step", "chunk", "none"),
                            group_ks=()) -> list:
        """(exchange, K, merge unit) triples worth timing: the push-pull halo at
        each K and merge unit (merged_passes), and the all-gather when its table
        (every rank's rows) is at most 4x the largest pull-only halo over the
        ranks (weak-scaled shards, whose halo is a small part of the global
        graph, skip it without a run).  Collective: the halo size is agreed by
        one all-to-all (its max over ranks), so every rank lists the same
        candidates -- tune_exchange runs their collectives in lock step.
        KGX_EXCHANGE (halo / pull / allgather) / KGX_HALO_MERGE restrict the set."""
        fixed = os.environ.get("KGX_EXCHANGE")
        fixed_unit = os.environ.get("KGX_HALO_MERGE")
        units = (fixed_unit,) if fixed_unit else tuple(units)
        # without merged passes the halo path ignores the unit: time each K once
        halo_units = units if use_merged_halo() else ("none",)
        # the pull-only halo (kind "pull", KGX_EXCHANGE=pull) is not timed: one-rank
        # simulations at NS weak P=8 put it behind push-pull both with the exchange
        # free (11.96-12.78 vs 11.16-11.18 ms) and at 400 GB/s (22.5 vs 12.9 ms)
        halo_kind = "pull" if fixed == "pull" else "halo"
        cands = [(halo_kind, k, u) for k in halo_ks for u in dict.fromkeys(halo_units)]
        # destination-group chunks (the GCN layer's grouped passes; the unit is implied)
        cands += [("group", k, "group") for k in group_ks]
        n = torch.full((self.world,), self.n_halo, dtype=torch.long, device=self.graph.col.device)
        every = torch.empty_like(n)
        self.comm.all_to_all_single(every, n)
        max_halo = int(every.max())
        if fixed == "allgather" or (fixed is None and self.n_global <= 4 * max(max_halo, 1)):
            # one step per all-gather chunk: "step" and "chunk" coincide
            g_units = dict.fromkeys("step" if u == "chunk" else u for u in units)
            cands += [("allgather", k, u) for k in gather_ks for u in g_units]
        if fixed:
            cands = [c for c in cands if c[0] == fixed]
        if not cands:
            raise ValueError(f"exchange_candidates: nothing to time (KGX_EXCHANGE={fixed!r}, "
                             f"KGX_HALO_MERGE={fixed_unit!r})")
        return cands

    def tune_exchange(self, run, candidates) -> tuple:
        """Choose (exchange, K, merge unit) by timing one forward per candidate
        (`run(kind, K)`, with the candidate installed; the plan is built before
        its timed call), best of two; every rank times the same candidates and
        the slowest rank's time counts (one all-to-all of the times).  Like a
        library autotuner: the best choice depends on the links' rate, which
        only the machine knows (tools/shard_sim.py: exchange-free, merging a
        chunk's steps wins; with 400 GB/s links, merging only its pulled rows).
        Bounded: once the agreed (slowest-rank) time spent passes
        KGX_TUNE_BUDGET_S (default 60 s) the remaining candidates are left
        untimed (inf); `tuning_s` / `tuning_skipped` record it."""
        dev = self.graph.col.device
        budget = float(os.environ.get("KGX_TUNE_BUDGET_S", "60"))
        worst, spent, t_start = [], 0.0, time.perf_counter()
        _progress(self, f"tune: {len(candidates)} exchange candidates, budget {budget:.0f} s")
        for kind, K, unit in candidates:
            if spent > budget:  # every rank sees the same agreed times, so all stop at the same candidate
                worst.append(float("inf"))
                continue
            self.exchange, self.halo_k, self.merge_unit = kind, K, unit
            t_plan = time.perf_counter()
            self.exchange_plan(K)
            best, total = float("inf"), time.perf_counter() - t_plan
            _progress(self, f"tune {kind}:{K}:{unit}: plan {total:.1f} s")
            for _ in range(2):
                if dev.type == "cuda":
                    torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                run(kind, K)
                if dev.type == "cuda":
                    torch.cuda.synchronize(dev)
                best = min(best, time.perf_counter() - t0)
                total += time.perf_counter() - t0
            # agree on (best, time spent) now: the slowest rank's counts for both
            t = torch.tensor([best, total], dtype=torch.float64, device=dev)
            every = torch.empty(self.world * 2, dtype=torch.float64, device=dev)
            self.comm.all_to_all_single(every, t.repeat(self.world).contiguous())
            mx = every.view(self.world, 2).max(0).values.cpu()
            worst.append(float(mx[0]))
            spent += float(mx[1])
            _progress(self, f"tune {kind}:{K}:{unit} {1e3 * worst[-1]:.2f} ms (agreed; {spent:.1f} s spent, "
                            f"{len(worst)}/{len(candidates)})")
        i = min(range(len(worst)), key=worst.__getitem__)
        self.exchange, self.halo_k, self.merge_unit = candidates[i]
        self.tuning = {f"{kind}:{K}:{unit}": v for (kind, K, unit), v in zip(candidates, worst)}
        self.tuning_s = time.perf_counter() - t_start
        self.tuning_skipped = sum(1 for v in worst if v == float("inf"))
        self.exchange_plan(self.halo_k)
        return candidates[i]

    def merged_passes(self, pp: PushPullPlan, unit: str | None = None, light: int = 0):
        """(g_a, g_b, later): the default path's passes with the first exchange
        group folded into the rows it touches (cached on the plan per unit).

        Groups: unit "step" (default; KGX_HALO_MERGE=step) -- every exchange
        step on its own (chunk k's pulled rows, then its pushed partials);
        "chunk" -- a chunk's steps together; "none" -- nothing merged: the own
        pass writes every row and each step accumulates (step granularity).  H = the local rows with an edge in
        the first group.  g_a: the own-source CSR restricted to the rows NOT in
        H -- it writes them, while the exchange is in flight.  g_b: for the rows
        in H, their own-source edges followed by their first-group edges
        (sources >= n_local index the halo buffer), written once by ONE
        two-table pass (kgx_spmm_gemm_ex3 / kgx_spmm_ex2) instead of an own pass
        that writes them and a halo pass that reads and rewrites them.  later:
        [(step to wait for, CSR, halo lo, halo hi)] for the remaining groups,
        accumulate-only over the rows each touches.  Each row's sum is own
        edges, then first-group edges, then later groups: a re-association of
        the one-pass order, tolerance-equal like the rest of this path.

        light > 0 (ShardedGCNConv only; KGX_HALO_LIGHT): rows of total degree <=
        light whose edges reach a later group are taken out of g_a / g_b / the
        later passes and written once each, with all their edges, by a
        two-table pass right after the last group they need has landed
        (ShardedGraph.light_passes) -- the short / tiny-row launches then see
        each light row once instead of once per pass it is touched by."""
        unit = unit or self.merge_unit or os.environ.get("KGX_HALO_MERGE", "step")
        unit = _merge_unit(unit)
        if pp.merged is None:
            pp.merged = {}
        key = unit if light <= 0 or unit == "none" else (unit, light)
        if key in pp.merged:
            return pp.merged[key]
        g_own, _ = self.own_halo_parts()
        n_local = self.n_local
        dev = g_own.col.device
        steps = [st for c in pp.chunks for st in c.steps]
        groups, idx = [], 0
        if unit == "none":  # nothing merged: the own pass over every row, then every step accumulates
            for i, g in enumerate(pp.step_parts or []):
                if g.kept:
                    groups.append((i, g, steps[i].lo, steps[i].hi))
            pp.merged[unit] = (g_own, None, groups, -1)
            return pp.merged[unit]
        if unit == "chunk":
            for k, c in enumerate(pp.chunks):
                idx += len(c.steps)
                if k < len(pp.parts):
                    groups.append((idx - 1, pp.parts[k], c.lo, c.hi))
        else:
            for i, g in enumerate(pp.step_parts or []):
                groups.append((i, g, steps[i].lo, steps[i].hi))
        first = groups[0][1] if groups else None
        if first is None or first.kept == 0:
            pp.merged[unit] = (g_own, None, [t for t in groups if t[1].kept], -1)
            return pp.merged[unit]
        lo0 = groups[0][2]
        in_h = first.deg > 0
        ar = torch.arange(n_local, device=dev)
        r_own = torch.repeat_interleave(ar, g_own.deg.long(), output_size=g_own.kept)
        keep = in_h[r_own]
        r_first = torch.repeat_interleave(ar, first.deg.long(), output_size=first.kept)
        rows = torch.cat([r_own[keep], r_first])
        cols = torch.cat([g_own.col[keep].long(), first.col.long() + (n_local + lo0)])
        # own edges first, then the group's: the stable CSR keeps that order inside every row
        g_b = self.backend.build_graph(cols.to(torch.int32), rows.to(torch.int32), n_local + pp.n_rows, n_local, 128)
        if pp.weighted:
            g_b.w = torch.cat([g_own.w[keep], first.w])[g_b.eid.long()].contiguous()
        defer = torch.zeros(n_local, dtype=torch.bool, device=dev)
        if light > 0:
            total = g_own.deg.long().clone()
            need = torch.full((n_local,), -1, dtype=torch.long, device=dev)
            for gi, (_, g, _, _) in enumerate(groups):
                total += g.deg.long()
                need = torch.where(g.deg > 0, torch.full_like(need, gi), need)
            defer = (total <= light) & (need >= 1)
            pp.merged[("light_rows", key)] = (defer, need)
        g_b = self.backend.restrict_rows(g_b, in_h & ~defer)
        g_a = self.backend.restrict_rows(g_own, ~in_h & ~defer)
        later = [t for t in groups[1:] if t[1].kept]
        if light > 0:
            later = [(i, self.backend.restrict_rows(g, ~defer), lo, hi) for (i, g, lo, hi) in later]
            later = [t for t in later if t[1].kept]
            pp.merged[("light_groups", key)] = groups
        pp.merged[key] = (g_a, g_b, later, groups[0][0])
        return pp.merged[key]

    def light_passes(self, pp: PushPullPlan, unit: str, light: int):
        """[(wait step, CSR)] for merged_passes(..., light): per later group j,
        the deferred light rows whose last edge group is j, with their own edges
        then every group's edges up to j (sources >= n_local index the halo
        buffer), for one two-table overwriting pass once group j has landed."""
        unit = _merge_unit(unit)
        key = (unit, light)
        lk = ("light", key)
        if lk in pp.merged:
            return pp.merged[lk]
        self.merged_passes(pp, unit, light)
        groups = pp.merged[("light_groups", key)]
        defer, need = pp.merged[("light_rows", key)]
        g_own, _ = self.own_halo_parts()
        n_local = self.n_local
        dev = g_own.col.device
        ar = torch.arange(n_local, device=dev)
        out = []
        for j in range(1, len(groups)):
            sel = defer & (need == j)
            if not bool(sel.any()):
                continue
            rows, cols, ws = [], [], []
            r_own = torch.repeat_interleave(ar, g_own.deg.long(), output_size=g_own.kept)
            k_own = sel[r_own]
            rows.append(r_own[k_own])
            cols.append(g_own.col[k_own].long())
            if pp.weighted:
                ws.append(g_own.w[k_own])
            for gi in range(j + 1):
                _, g, lo, _ = groups[gi]
                r_g = torch.repeat_interleave(ar, g.deg.long(), output_size=g.kept)
                k_g = sel[r_g]
                rows.append(r_g[k_g])
                cols.append(g.col[k_g].long() + (n_local + lo))
                if pp.weighted:
                    ws.append(g.w[k_g])
            gl = self.backend.build_graph(torch.cat(cols).to(torch.int32), torch.cat(rows).to(torch.int32),
                                          n_local + pp.n_rows, n_local, 128)
            if pp.weighted:
                gl.w = torch.cat(ws)[gl.eid.long()].contiguous()
            out.append((groups[j][0], self.backend.restrict_rows(gl, sel)))
        pp.merged[lk] = out
        return out

    def group_passes(self, pp: PushPullPlan):
        """(g_a, [(wait step, g_k)]) for a destination-group plan (kind "group"):
        g_a = the own-source CSR restricted to the rows with no halo edge (they
        need nothing from the exchange); g_k = group k's rows with their own
        edges, then their halo edges (sources >= n_local index the halo
        buffer, every chunk <= k), for ONE two-table pass that writes each row
        once after chunk k's last step has landed (cached on the plan)."""
        if pp.merged is None:
            pp.merged = {}
        if "group" in pp.merged:
            return pp.merged["group"]
        g_own, _ = self.own_halo_parts()
        n_local = self.n_local
        dev = g_own.col.device
        rg = pp.recv_graph
        has_halo = torch.zeros(n_local, dtype=torch.bool, device=dev)
        if rg is not None:
            has_halo = rg.deg > 0
        g_a = self.backend.restrict_rows(g_own, ~has_halo)
        ar = torch.arange(n_local, device=dev)
        r_own = torch.repeat_interleave(ar, g_own.deg.long(), output_size=g_own.kept)
        passes = []
        if rg is not None:
            r_h = torch.repeat_interleave(ar, rg.deg.long(), output_size=rg.kept)
            grp = pp.row_group
            steps_before = 0
            for k, c in enumerate(pp.chunks):
                steps_before += len(c.steps)
                in_k = has_halo & (grp == k)
                if not bool(in_k.any()):
                    continue
                keep_o, keep_h = in_k[r_own], in_k[r_h]
                rows = torch.cat([r_own[keep_o], r_h[keep_h]])
                cols = torch.cat([g_own.col[keep_o].long(), rg.col[keep_h].long() + n_local])
                g_k = self.backend.build_graph(cols.to(torch.int32), rows.to(torch.int32), n_local + pp.n_rows,
                                               n_local, 128)
                if pp.weighted:
                    g_k.w = torch.cat([g_own.w[keep_o], rg.w[keep_h]])[g_k.eid.long()].contiguous()
                passes.append((steps_before - 1, self.backend.restrict_rows(g_k, in_k)))
        pp.merged["group"] = (g_a, passes)
        return pp.merged["group"]

    def halo_exchange(self, table: torch.Tensor) -> None:
        """table[n_local:] <- rows other ranks own (one all-to-all-v over RCCL
        per chunk, each landing in its contiguous slice of the halo rows)."""
        own, halo = table[: self.n_local], table[self.n_local:]
        for c in self.chunks:
            self.comm.all_to_all_single(halo[c.lo: c.hi], self._pack(own, c), c.recv_splits, c.send_splits)

    def own_halo_parts(self):
        """(own-source CSR, [one CSR per halo chunk]): the shard CSR split by
        source range, CSR order kept inside each part; a chunk part's sources
        index that chunk's halo rows from 0 and its schedule skips the rows the
        chunk does not touch (accumulate-only)."""
        if self._parts is None:
            cuts = [0, self.n_local] + [self.n_local + c.hi for c in self.chunks]
            parts = self.backend.split_by_source(self.graph, cuts)
            self._parts = (parts[0], list(parts[1:]))
        return self._parts

    def halo_buffer(self, features: int, like: torch.Tensor, rows: int | None = None) -> torch.Tensor:
        """Persistent [rows (default n_halo), features] receive buffer (reused every layer call)."""
        if self._halo_buf is None:
            self._halo_buf = {}
        rows = self.n_halo if rows is None else rows
        key = (features, like.device, rows)
        buf = self._halo_buf.get(key)
        if buf is None:
            buf = torch.empty((rows, features), dtype=torch.float32, device=like.device)
            self._halo_buf[key] = buf
        return buf

    def start_halo_exchange(self, x_local: torch.Tensor, halo: torch.Tensor, chunks: list | None = None) -> list:
        """Per chunk: pack the rows other ranks need and start the all-to-all
        into halo[chunk] on a side stream.  Returns one handle per chunk whose
        wait() orders the then-current stream after that chunk's rows (None:
        the comm ran synchronously and the rows are already ordered)."""
        chunks = self.chunks if chunks is None else chunks
        probe = []  # (chunk, step, start event, handle, send bytes, receive bytes) when link_probe is on

        def run():
            start = getattr(self.comm, "all_to_all_start", None)
            works = []
            for k, c in enumerate(chunks):
                handles = []
                for j, st in enumerate(c.steps or [c]):
                    send = self._pack(x_local, st)
                    ev = None
                    if self.link_probe is not None and start is not None and x_local.is_cuda:
                        ev = torch.cuda.Event(enable_timing=True)
                        ev.record()  # the side stream, after this step's packing: the transfer may start
                    if st.kind == "allgather":
                        gstart = getattr(self.comm, "all_gather_start", None) if start is not None else None
                        if gstart is None:
                            self.comm.all_gather(halo[st.lo: st.hi], send)
                            handles.append(None)
                        else:
                            handles.append(gstart(halo[st.lo: st.hi], send))
                    elif start is None:
                        self.comm.all_to_all_single(halo[st.lo: st.hi], send, st.recv_splits, st.send_splits)
                    else:
                        handles.append(start(halo[st.lo: st.hi], send, st.recv_splits, st.send_splits))
                    if ev is not None and handles[-1] is not None:
                        probe.append((k, j, ev, handles[-1], send.numel() * 4, (st.hi - st.lo) * halo.shape[1] * 4))
                works.append(_Works(handles) if start is not None else None)
            return works

        if not x_local.is_cuda:
            return run()
        if self._side is None:
            # high priority: the packing kernels are the exchange's critical path
            # start; at normal priority the resident own-source pass launched
            # right after them holds all but the block slots it leaves free and
            # the packing crawls on those (tools/shard_sim.py: 6.8 ms for 12.7 GB)
            prio = 0 if os.environ.get("KGX_SIDE_PRIORITY", "1") == "0" else -1  # 0: measurement A/B only
            self._side = torch.cuda.Stream(device=x_local.device, priority=prio)
        cur = torch.cuda.current_stream(x_local.device)
        self._side.wait_stream(cur)
        with torch.cuda.stream(self._side):
            works = run()
            # the side stream after its last packing kernel (the transfers run on the
            # comm's own stream): a pass may wait for the packs without the transfers
            self.packs_done = torch.cuda.Event()
            self.packs_done.record()
        if any(w is None for w in works):  # synchronous comm: order the halo rows before later work
            cur.wait_stream(self._side)
        if probe:  # the landing of every step, seen from a stream that waits for nothing else
            if self._probe_stream is None:
                self._probe_stream = torch.cuda.Stream(device=x_local.device)
            self._probe_stream.wait_stream(self._side)
            with torch.cuda.stream(self._probe_stream):
                for k, j, ev0, h, sb, rb in probe:
                    h.wait()
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev1.record()
                    self.link_probe.append({"chunk": k, "step": j, "start": ev0, "land": ev1,
                                            "send_bytes": sb, "recv_bytes": rb})
        return works

    def link_report(self, steps: int, link_gbps: float = 400.0) -> list:
        """Per exchange step (chunk, step), averaged over `steps` layer calls of
        the link_probe log (call after a synchronize): the bytes this rank sent
        and received, the measured time from the end of its packing to its
        landing (the transfer, plus any wait behind the previous steps on the
        comm stream), and the time a modelled link of `link_gbps` would take for
        the received bytes (tools/shard_sim.py's model)."""
        acc = {}
        for r in self.link_probe or []:
            a = acc.setdefault((r["chunk"], r["step"]), {"chunk": r["chunk"], "step": r["step"], "n": 0, "ms": 0.0,
                                                        "send_bytes": r["send_bytes"], "recv_bytes": r["recv_bytes"]})
            a["n"] += 1
            a["ms"] += r["start"].elapsed_time(r["land"])
        out = []
        for key in sorted(acc):
            a = acc[key]
            out.append({"chunk": a["chunk"], "step": a["step"], "send_MB": a["send_bytes"] / 1e6,
                        "recv_MB": a["recv_bytes"] / 1e6, "measured_ms": a["ms"] / max(a["n"], 1),
                        "modelled_ms_at_%dGBps" % int(link_gbps): a["recv_bytes"] / (link_gbps * 1e6),
                        "calls": a["n"]})
        return out

    def propagate_overlapped(self, x_local: torch.Tensor, reduce: str = "sum", *, gin_scale: float | None = None,
                             weighted: bool = False, bias: torch.Tensor | None = None) -> torch.Tensor:
        """Sum / mean propagation (unweighted shard graph: GIN, SAGE) with the
        push-pull halo exchanged in chunks on the side stream, as ShardedGCNConv:
        the own-source pass runs while the halo is in flight, then one
        accumulating pass (KGX_EPI_ACCUM) per landed chunk over the rows it
        touches.  gin_scale: GIN's (1+eps) x_i + aggr (gin_conv.py:216-222).
        Row sums are re-associated (own, then chunks): tolerance-equal to the
        one-pass result; EXACT mode uses `propagate`."""
        if reduce not in ("sum", "mean"):
            raise ValueError(f"propagate_overlapped: sum or mean only (got {reduce!r})")
        if (weighted or bias is not None) and (reduce != "sum" or gin_scale is not None):
            raise ValueError("propagate_overlapped: weights / bias go with a plain sum (the GCN layer)")
        x_local = x_local.contiguous()
        g_own, _ = self.own_halo_parts()
        pp = self.exchange_plan(weighted=weighted)
        halo = self.halo_buffer(x_local.shape[1], x_local, pp.n_rows)
        fold_gin = gin_scale is not None and reduce == "sum"
        epi = nat.EPI_GIN if fold_gin else (nat.EPI_BIAS if bias is not None else nat.EPI_NONE)
        if use_merged_halo() or pp.kind == "allgather":
            out = self._propagate_merged(x_local, pp, halo, weighted, epi, bias, fold_gin, gin_scale)
            if reduce == "mean":  # aggregators.py:56-85: sum / max(count, 1e-8), count in fp32
                count = torch.clamp(self.graph.deg[: self.n_local].to(torch.float32), min=1e-8)
                out = out / count.unsqueeze(1)
                if gin_scale is not None:
                    out = torch.tensor(float(gin_scale), dtype=torch.float32, device=out.device) * x_local + out
            return out
        with torch.no_grad():
            works = self.start_halo_exchange(x_local, halo, pp.chunks)
            epi = nat.EPI_GIN if fold_gin else (nat.EPI_BIAS if bias is not None else nat.EPI_NONE)
            with kops.sharing_gpu():
                out = self.backend.aggregate(g_own, x_local, "sum", weighted=weighted, epilogue=epi, bias=bias,
                                             xroot=x_local if fold_gin else None,
                                             gin_scale=float(gin_scale) if fold_gin else 1.0)
            for k, c in enumerate(pp.chunks):
                if works[k] is not None:
                    works[k].wait()
                g = pp.parts[k] if k < len(pp.parts) else None
                if g is not None and g.kept:
                    self.backend.aggregate_accumulate(g, halo[c.lo: c.hi], out, weighted=weighted)
            if reduce == "mean":  # aggregators.py:56-85: sum / max(count, 1e-8), count in fp32
                count = torch.clamp(self.graph.deg[: self.n_local].to(torch.float32), min=1e-8)
                out = out / count.unsqueeze(1)
                if gin_scale is not None:
                    out = torch.tensor(float(gin_scale), dtype=torch.float32, device=out.device) * x_local + out
        return out

    def _propagate_merged(self, x_local, pp, halo, weighted, epi, bias, fold_gin, gin_scale):
        """propagate_overlapped's passes with the first exchange step merged into
        its rows (merged_passes): the rows without first-step edges (own
        sources, epilogue applied) while the exchange is in flight; the rows
        with them in ONE two-table pass (own then first-step edges, epilogue
        applied) once chunk 0's pulled rows have landed; then out += the later
        steps' row sums as each lands.  Light rows are written once, epilogue
        applied, after the last step they need -- only when KGX_HALO_LIGHT is set
        explicitly: on these plain sum / mean passes the C5 simulation (SAGE mean,
        strong P = 4, 400 GB/s) measured it slower (K 1: 2.57 -> 2.64 ms, K 2:
        3.20 -> 3.53; profiles/r05/sim_light/c5_*)."""
        unit = self.merge_unit or os.environ.get("KGX_HALO_MERGE", "step")
        light = halo_light() if (pp.kind != "allgather" and unit != "none"
                                 and os.environ.get("KGX_HALO_LIGHT") is not None) else 0
        g_a, g_b, later, first_wait = self.merged_passes(pp, unit, light)
        lights = self.light_passes(pp, unit, light) if light > 0 and g_b is not None else []
        steps = [st for c in pp.chunks for st in c.steps]
        kw = dict(weighted=weighted, bias=bias, xroot=x_local if fold_gin else None,
                  gin_scale=float(gin_scale) if fold_gin else 1.0)
        with torch.no_grad():
            works = self.start_halo_exchange(x_local, halo, pp.chunks)
            handles = []
            for w, c in zip(works, pp.chunks):
                handles.extend(w.handles if w is not None else [None] * len(c.steps))
            waited = set()

            def wait_step(i):
                for j in range(i + 1):
                    if j not in waited:
                        waited.add(j)
                        if handles[j] is not None:
                            handles[j].wait()

            with kops.sharing_gpu():
                out = self.backend.aggregate(g_a, x_local, "sum", epilogue=epi, **kw)
            if g_b is not None:
                wait_step(first_wait)
                self.backend.aggregate_accumulate(g_b, x_local, out, epilogue=epi, table2=halo, **kw)
            pending = list(lights)
            for i, g, lo, hi in later:
                wait_step(i)
                self.backend.aggregate_accumulate(g, halo[lo: hi], out, weighted=weighted)
                while pending and pending[0][0] <= i:
                    _, gl = pending.pop(0)
                    self.backend.aggregate_accumulate(gl, x_local, out, epilogue=epi, table2=halo, **kw)
            for i, gl in pending:
                wait_step(i)
                self.backend.aggregate_accumulate(gl, x_local, out, epilogue=epi, table2=halo, **kw)
            wait_step(len(steps) - 1)
        return out

    def reverse_halo_exchange(self, g_src: torch.Tensor) -> torch.Tensor:
        """The backward of halo_exchange: g_src [n_local + n_halo, F] holds
        gradients w.r.t. this rank's table rows; each halo row's gradient goes
        back to the rank that owns the row (the forward all-to-all with the
        splits swapped) and is added to that row's own gradient.  Returns
        [n_local, F].  Within one (chunk, peer) slice the rows are distinct,
        and slices are added in chunk, then rank order: deterministic."""
        n = self.n_local
        dx = g_src[:n].clone()
        halo = g_src[n:]
        F = g_src.shape[1]
        for c in self.chunks:
            recv = g_src.new_empty((int(sum(c.send_splits)), F))
            self.comm.all_to_all_single(recv, halo[c.lo: c.hi].contiguous(), c.send_splits, c.recv_splits)
            off = 0
            for cnt in c.send_splits:
                if cnt:
                    dx.index_add_(0, c.send_rows[off: off + cnt].long(), recv[off: off + cnt])
                off += cnt
        return dx

    def propagate(self, x_local: torch.Tensor, reduce: str = "sum", **kw) -> torch.Tensor:
        """Sharded MessagePassing.propagate with the default message x_j."""
        table = self.new_table(x_local.shape[1], x_local)
        table[: self.n_local] = x_local
        self.halo_exchange(table)
        return self.backend.aggregate(self.graph, table, reduce, exact=self.exact, **kw)


class ShardedGCNConv(Layer):
    """GCNConv over a ShardedGraph (same math as layers.GCNConv; weights are
    broadcast from rank 0 so every shard applies the same layer)."""

    def __init__(self, output_dim: int, sg: ShardedGraph, use_bias: bool = True,
                 kernel_initializer="glorot_uniform", bias_initializer="zeros", **kwargs):
        super().__init__(**kwargs)
        self.output_dim = output_dim
        self.sg = sg
        self.use_bias = use_bias
        self.kernel_initializer = get_initializer(kernel_initializer)
        self.bias_initializer = get_initializer(bias_initializer)
        self.kernel = None
        self.bias = None

    def build(self, input_shape) -> None:
        self.kernel = self.add_weight((input_shape[-1], self.output_dim), self.kernel_initializer, name="kernel")
        if self.use_bias:
            self.bias = self.add_weight((self.output_dim,), self.bias_initializer, name="bias")
        with torch.no_grad():
            for p in self.weights:
                self.sg.comm.broadcast(p.data, src=0)
        self.built = True

    def forward(self, x_local: torch.Tensor) -> torch.Tensor:
        if not self.built:
            self._build_device = x_local.device
            self.build(tuple(x_local.shape))
        if torch.is_grad_enabled() and (x_local.requires_grad or any(p.requires_grad for p in self.weights)):
            # training: the sharded forward + backward (_ShardedGCNFn)
            use_b = self.use_bias and self.bias is not None
            return _ShardedGCNFn.apply(x_local, self.kernel, self.bias if use_b else None, self)
        sg = self.sg
        use_b = self.use_bias and self.bias is not None
        if not sg.exact and sg.backend.supports_fused(x_local.shape[1], self.output_dim):
            return self._forward_overlapped(x_local, self.bias if use_b else None)
        if not sg.exact and use_push_pull() and sg.graph.w is not None:
            # the weighted sum with the push-pull halo pipelined under the own-source
            # pass, over the narrower of X (aggregate, then transform) and X W
            # (transform first): those are the rows exchanged and gathered
            with torch.no_grad():
                x_local = x_local.contiguous()
                if self.output_dim < x_local.shape[1]:
                    h = sg.backend.transform(x_local, self.kernel)
                    return sg.propagate_overlapped(h, "sum", weighted=True, bias=self.bias if use_b else None)
                agg = sg.propagate_overlapped(x_local, "sum", weighted=True)
                return sg.backend.transform(agg, self.kernel, self.bias if use_b else None)
        table = sg.new_table(self.output_dim, x_local)
        with torch.no_grad():  # forward engine: X W written straight into the table's own-rows slice
            torch.matmul(x_local, self.kernel, out=table[: sg.n_local])
        sg.halo_exchange(table)
        return sg.backend.aggregate(sg.graph, table, "sum", weighted=True,
                                    epilogue=nat.EPI_BIAS if use_b else nat.EPI_NONE,
                                    bias=self.bias if use_b else None, exact=sg.exact)

    def tune(self, x_local: torch.Tensor) -> int | None:
        """Time the exchanges once (ShardedGraph.tune_exchange: the push-pull
        halo at K = 1 / 2 / 4 chunks, and the all-gather where its table is
        not far larger); a no-op when K is fixed, on one rank, or off the
        default path."""
        sg = self.sg
        if not self.built:
            self._build_device = x_local.device
            self.build(tuple(x_local.shape))
        use_b = self.use_bias and self.bias is not None
        if (sg.exact or sg.chunks_fixed or sg.world < 2 or sg.halo_k is not None or not use_push_pull()
                or not sg.backend.supports_fused(x_local.shape[1], self.output_dim)):
            return sg.halo_k
        with torch.no_grad():
            sg.tune_exchange(lambda kind, K: self._forward_overlapped(x_local, self.bias if use_b else None, K),
                             sg.exchange_candidates(group_ks=(2, 4)))
        return sg.halo_k

    def _forward_overlapped(self, x_local: torch.Tensor, bias, n_chunks: int | None = None) -> torch.Tensor:
        """Aggregate-then-transform with the halo exchange pipelined in chunks:
        side stream, per chunk k: pack its send rows of X -> RCCL all-to-all
        into halo[k];
        main stream: out = bias + (A_own X_own) W   (fused kernel, own sources),
        then per chunk k, once its rows have landed: out += (A_k X_halo[k]) W
        (same kernel, accumulate mode, only the rows chunk k touches) -- so
        pass k runs while chunk k+1 is on the links.  Each row's sum is split
        own-then-chunks, a re-association of the one-pass order
        (tolerance-equal; EXACT mode keeps the one-pass order and waits for the
        whole halo)."""
        sg = self.sg
        g_own, g_chunks = sg.own_halo_parts()
        chunks, n_rows = sg.chunks, sg.n_halo
        pp = None
        if use_push_pull():
            if n_chunks is None and sg.halo_k is None and not sg.chunks_fixed and sg.world > 1:
                self.tune(x_local)  # first call: time the exchanges (and K) once
            pp = sg.exchange_plan(n_chunks)
            chunks, g_chunks, n_rows = pp.chunks, pp.parts, pp.n_rows
        x_local = x_local.contiguous()
        halo = sg.halo_buffer(x_local.shape[1], x_local, n_rows)
        if pp is not None and pp.kind == "group":
            return self._forward_grouped(x_local, bias, pp, halo)
        if pp is not None and (use_merged_halo() or pp.kind == "allgather"):
            return self._forward_merged(x_local, bias, pp, halo)
        with torch.no_grad():
            works = sg.start_halo_exchange(x_local, halo, chunks)
            with kops.sharing_gpu():  # the exchange's RCCL kernels run beside this pass
                out = sg.backend.aggregate_transform(g_own, x_local, self.kernel, bias=bias)
            last = max((k for k, g in enumerate(g_chunks) if g.kept), default=-1)
            for k, c in enumerate(chunks):
                # wait for every chunk, used or not: it also orders the side stream's
                # reads of x_local (the packing) before anything later on this stream
                if works[k] is not None:
                    works[k].wait()
                g = g_chunks[k] if k < len(g_chunks) else None
                if g is None or not g.kept:
                    continue
                # leave block slots to the chunks still in flight; the last pass takes the whole GPU
                with kops.sharing_gpu() if k < last else contextlib.nullcontext():
                    sg.backend.aggregate_transform(g, halo[c.lo: c.hi], self.kernel, out=out)
        return out


    def _forward_grouped(self, x_local: torch.Tensor, bias, pp: PushPullPlan, halo: torch.Tensor) -> torch.Tensor:
        """Destination-group exchange (kind "group"): side stream as
        _forward_merged; main stream: out[rows with no halo edge] = b + (A_own X) W
        while the exchange is in flight, then per group k, once chunk k has
        landed, out[group k] = b + (A_own X + A_halo halo) W in one two-table
        pass -- every row written once."""
        sg = self.sg
        g_a, passes = sg.group_passes(pp)
        steps = [st for c in pp.chunks for st in c.steps]
        with torch.no_grad():
            works = sg.start_halo_exchange(x_local, halo, pp.chunks)
            handles = []
            for w, c in zip(works, pp.chunks):
                handles.extend(w.handles if w is not None else [None] * len(c.steps))
            waited = set()

            def wait_step(i):
                for j in range(i + 1):  # steps land in issue order on the comm stream
                    if j not in waited:
                        waited.add(j)
                        if handles[j] is not None:
                            handles[j].wait()

            with kops.sharing_gpu():  # the exchange's packing and RCCL kernels run beside this pass
                out = sg.backend.aggregate_transform(g_a, x_local, self.kernel, bias=bias)
            for n, (i, g) in enumerate(passes):
                wait_step(i)
                with kops.sharing_gpu() if n + 1 < len(passes) else contextlib.nullcontext():
                    sg.backend.aggregate_transform(g, x_local, self.kernel, bias=bias, out=out, x2=halo,
                                                   accumulate=False)
            wait_step(len(steps) - 1)  # also orders the side stream's reads of x_local
        return out

    def _forward_merged(self, x_local: torch.Tensor, bias, pp: PushPullPlan, halo: torch.Tensor) -> torch.Tensor:
        """The default path with the first exchange step merged into its rows
        (ShardedGraph.merged_passes): side stream as _forward_overlapped; main
        stream: out[rows not in H] = bias + (A_own X) W while the exchange is in
        flight; once chunk 0's pulled rows have landed, out[H] = bias + (A_own X
        + A_0 halo_0) W in one two-table pass; then out += (A_s halo_s) W per
        later step (pushed partials, later chunks) as each lands."""
        sg = self.sg
        unit = sg.merge_unit or os.environ.get("KGX_HALO_MERGE", "step")
        light = halo_light() if pp.kind != "allgather" else 0
        g_a, g_b, later, first_wait = sg.merged_passes(pp, unit, light)
        lights = sg.light_passes(pp, unit, light) if light > 0 and g_b is not None and unit != "none" else []
        steps = [st for c in pp.chunks for st in c.steps]
        # the own-only rows' pass (g_a) after the merged pass when two or more exchange
        # groups follow the first: then the first pack runs alone and the first transfer
        # starts earlier (tools/shard_sim.py at modelled 400 GB/s, NS weak P=8: K=2 step
        # groups 13.91 -> 12.98 ms, K=4 chunks 14.08 -> 13.81; with one group or none
        # after the first it measured slower: K=1 14.22 -> 15.82, K=2 chunks 13.91 ->
        # 14.47).  KGX_HALO_A_LATE=0 / 1 forces either order (measurement A/B).
        # KGX_HALO_A_LATE=2 (experiment): pass A where it is, but after the packs
        # (the side stream's packing alone on the GPU, then pass A beside the transfers)
        forced = os.environ.get("KGX_HALO_A_LATE")
        a_late = forced == "1" if forced in ("0", "1", "2") else len(later) >= 2
        a_after_pack = forced == "2"
        with torch.no_grad():
            works = sg.start_halo_exchange(x_local, halo, pp.chunks)
            handles = []
            for w, c in zip(works, pp.chunks):
                handles.extend(w.handles if w is not None else [None] * len(c.steps))
            waited = set()

            def wait_step(i):
                for j in range(i + 1):  # steps land in issue order on the comm stream
                    if j not in waited:
                        waited.add(j)
                        if handles[j] is not None:
                            handles[j].wait()

            if a_late and g_b is not None:
                out = torch.empty((x_local.shape[0], self.kernel.shape[1]), dtype=torch.float32,
                                  device=x_local.device)
            else:
                if a_after_pack and getattr(sg, "packs_done", None) is not None and x_local.is_cuda:
                    torch.cuda.current_stream(x_local.device).wait_event(sg.packs_done)
                with kops.sharing_gpu():  # the exchange's packing and RCCL kernels run beside this pass
                    out = sg.backend.aggregate_transform(g_a, x_local, self.kernel, bias=bias)
            if g_b is not None:
                wait_step(first_wait)
                with kops.sharing_gpu() if later else contextlib.nullcontext():
                    sg.backend.aggregate_transform(g_b, x_local, self.kernel, bias=bias, out=out, x2=halo,
                                                   accumulate=False)
                if a_late:  # later groups are still in flight: leave block slots to their RCCL kernels
                    # (pinned by one-rank simulations only until an N > 1 RCCL run measures it)
                    with kops.sharing_gpu() if later else contextlib.nullcontext():
                        sg.backend.aggregate_transform(g_a, x_local, self.kernel, bias=bias, out=out,
                                                       accumulate=False)
            pending = list(lights)  # light rows, each written once after the last group it needs
            for n, (i, g, lo, hi) in enumerate(later):
                wait_step(i)
                last = n + 1 == len(later)
                with kops.sharing_gpu() if not last else contextlib.nullcontext():
                    sg.backend.aggregate_transform(g, halo[lo: hi], self.kernel, out=out)
                while pending and pending[0][0] <= i:
                    _, gl = pending.pop(0)
                    with kops.sharing_gpu() if not last else contextlib.nullcontext():
                        sg.backend.aggregate_transform(gl, x_local, self.kernel, bias=bias, out=out, x2=halo,
                                                       accumulate=False)
            for i, gl in pending:  # groups with light rows but no accumulate pass left
                wait_step(i)
                sg.backend.aggregate_transform(gl, x_local, self.kernel, bias=bias, out=out, x2=halo,
                                               accumulate=False)
            # every step, used or not: also orders the side stream's reads of x_local
            wait_step(len(steps) - 1)
        return out


def halo_light() -> int:
    """KGX_HALO_LIGHT: rows of total degree <= this many edges are written once,
    after the last exchange group they need (ShardedGraph.merged_passes);
    0 = off.  Default 32, from one-rank simulations of NS weak P = 8, halo K 2,
    modelled 400 GB/s (profiles/r05/sim_light/, two rounds each): off
    12.89-12.98 ms, 7: 12.47-12.61, 12: 12.39-12.50, 20: 12.18-12.35, 32:
    12.12-12.25, 48: 12.21-12.26, 64: 12.45-12.53, every row: 15.08 (the
    deferred passes then carry the heavy rows past the last landing)."""
    try:
        return max(0, int(os.environ.get("KGX_HALO_LIGHT", "32")))
    except ValueError:
        return 0


class _ShardedGCNFn(torch.autograd.Function):
    """ShardedGCNConv with gradients (the reference's model.fit path,
    tests/performance/test_large_graphs.py:341-357, on sharded rows).

    forward:  table = [x_local | pulled halo x] (halo_exchange);
              agg = A_shard table (weighted sum over the shard CSR, in each
              row's global input order), y = agg W + b
              (= the reference's sum_e norm_e x_j W + b, gcn_conv.py:233-272).
    backward: dagg = dY W^T;  G = A_shard^T dagg over the shard's sources
              (graph.transpose: own rows and halo rows);  the halo rows' G goes
              back to their owners (reverse_halo_exchange) and is added to
              their own G: dX_local;  dW = sum over ranks of agg^T dY and db =
              sum over ranks of sum_i dY_i (all-reduce)."""

    @staticmethod
    def forward(ctx, x_local, kernel, bias, layer):
        sg = layer.sg
        with torch.no_grad():
            x_local = x_local.contiguous()
            table = sg.new_table(x_local.shape[1], x_local)
            table[: sg.n_local] = x_local
            sg.halo_exchange(table)
            agg = sg.backend.aggregate(sg.graph, table, "sum", weighted=True, exact=sg.exact)
            del table
            y = sg.backend.transform(agg, kernel, bias)
        ctx.layer = layer
        ctx.has_bias = bias is not None
        ctx.save_for_backward(agg, kernel)
        return y

    @staticmethod
    def backward(ctx, dy):
        agg, kernel = ctx.saved_tensors
        sg = ctx.layer.sg
        dy = dy.contiguous()
        dx = dW = db = None
        if ctx.needs_input_grad[0]:
            dagg = sg.backend.transform(dy, kernel.t().contiguous())
            dx = sg.reverse_halo_exchange(sg.backend.aggregate_transposed(sg.graph, dagg))
        if ctx.needs_input_grad[1]:
            dW = torch.matmul(agg.t(), dy)
            sg.comm.all_reduce(dW)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.sum(0)
            sg.comm.all_reduce(db)
        return dx, dW, db, None


class _ShardedAggFn(torch.autograd.Function):
    """AGG_j x_j over a shard, sum or mean of the plain message x_j, with
    gradients: the neighbour reduction of GINConv and SAGEConv on the
    reference's model.fit path (tests/performance/test_large_graphs.py:341-357;
    gin_conv.py:216-225, sage_conv.py:404-439), whose node update then trains
    through torch autograd on the shard's own rows.

    forward:  table = [x_local | pulled halo x] (halo_exchange); agg = the shard
              CSR's row sums in each row's global input order (ShardedGraph.
              propagate), mean = sum / max(fp32 in-degree, 1e-8)
              (aggregators.py:56-85).
    backward: mean: dagg / count; G = A_shard^T dagg over the shard's sources
              (graph.transpose: own rows and halo rows); the halo rows' G goes
              back to their owners (reverse_halo_exchange, the forward
              all-to-all with the splits swapped) and is added to their own G."""

    @staticmethod
    def forward(ctx, x_local, sg, reduce):
        with torch.no_grad():
            agg = sg.propagate(x_local.contiguous(), reduce)
        ctx.sg, ctx.reduce = sg, reduce
        return agg

    @staticmethod
    def backward(ctx, dagg):
        sg = ctx.sg
        d = dagg.contiguous()
        if ctx.reduce == "mean":
            count = torch.clamp(sg.graph.deg[: sg.n_local].to(torch.float32), min=1e-8)
            d = d / count.unsqueeze(1)
        g_src = sg.backend.aggregate_transposed(sg.graph, d.contiguous(), weighted=False)
        return sg.reverse_halo_exchange(g_src), None, None


def _training(weights, x_local: torch.Tensor) -> bool:
    return torch.is_grad_enabled() and (x_local.requires_grad or any(p.requires_grad for p in weights))


def use_merged_halo() -> bool:
    """The default GCN path merges the first halo step into its rows' pass
    (KGX_HALO_MERGED=0: the round-2 own pass + accumulating chunk passes)."""
    return os.environ.get("KGX_HALO_MERGED", "1") not in ("0", "", "false", "False")


class _ShardedWrap(Layer):
    """A single-device conv layer applied to a ShardedGraph: the neighbour
    reduction runs over the shard CSR (own rows + exchanged halo rows), the
    node update runs on the shard's own rows with the wrapped layer's weights
    (broadcast from rank 0 at build)."""

    def __init__(self, conv: Layer, sg: ShardedGraph, **kwargs):
        super().__init__(**kwargs)
        self.conv = conv
        self.sg = sg

    def _ensure_built(self, x_local: torch.Tensor) -> None:
        if self.conv.built:
            return
        self.conv._build_device = x_local.device
        self.conv.build([tuple(x_local.shape), (2, 0)])
        with torch.no_grad():
            for p in self.conv.weights:
                self.sg.comm.broadcast(p.data, src=0)
        if self.sg.world > 1:
            # training: a weight's gradient from this rank's rows is a partial sum; every
            # rank gets the sum over all ranks (as ShardedGCNConv's dW / db), so the same
            # optimizer step keeps the broadcast weights identical everywhere
            for p in self.conv.weights:
                if p.requires_grad:
                    p.register_hook(self._all_reduce_grad)
        self.built = True

    def _all_reduce_grad(self, grad: torch.Tensor) -> torch.Tensor:
        g = grad.detach().clone().contiguous()
        self.sg.comm.all_reduce(g)
        return g

    def _pipelined(self) -> bool:
        """Whether the forward takes the pipelined (exchange-overlapped) sum / mean path."""
        return False

    def _maybe_tune(self, x_local: torch.Tensor) -> None:
        """First forward on the pipelined path: time the exchanges (the push-pull
        halo at K = 1 / 2 / 4, the all-gather where its table is not far
        larger) with this layer's own forward and keep the fastest
        (ShardedGraph.tune_exchange); K fixed (halo_chunks= / KGX_HALO_CHUNKS),
        one rank or EXACT mode: no tuning."""
        sg = self.sg
        if sg.halo_k is not None or sg.chunks_fixed or sg.world < 2 or sg.exact or not self._pipelined():
            return
        with torch.no_grad():
            sg.tune_exchange(lambda kind, K: self._forward_impl(x_local, None),
                             sg.exchange_candidates(group_ks=self._group_ks(x_local)))

    def _group_ks(self, x_local: torch.Tensor) -> tuple:
        """Destination-group chunk counts the tuner also times: only where the
        layer has a grouped forward (the fused GIN path)."""
        return ()


class ShardedGINConv(_ShardedWrap):
    """GINConv over a ShardedGraph: h_i = MLP((1+eps) x_i + AGG_j x_j)
    (gin_conv.py:216-225).  Shard graph: no self loops, no GCN norm
    (ShardedGraph.build(..., self_loops=False, gcn_norm=False)).  The
    (1+eps) x_i + aggr epilogue is fused into the aggregation as on one GPU,
    so EXACT-mode h is bit-identical to the single-GPU layer's."""

    def __init__(self, output_dim: int, sg: ShardedGraph, **gin_kwargs):
        from .layers.gin_conv import GINConv

        super().__init__(GINConv(output_dim, exact=sg.exact, **gin_kwargs), sg)

    def _pipelined(self) -> bool:
        return not self.sg.exact and self.conv.aggregator in ("sum", "mean")

    def forward(self, x_local: torch.Tensor, training=None) -> torch.Tensor:
        self._ensure_built(x_local)
        conv = self.conv
        if _training(conv.weights, x_local) and conv.aggregator in ("sum", "mean"):
            # training (sum / mean): the aggregation through _ShardedAggFn, (1+eps) x_i +
            # aggr and the MLP through torch autograd (gin_conv.py:216-225)
            agg = _ShardedAggFn.apply(x_local, self.sg, conv.aggregator)
            scale = (1 + conv.eps) if conv.train_eps else torch.tensor(float(conv._scale()), dtype=torch.float32,
                                                                        device=x_local.device)
            return conv.mlp(scale * x_local + agg, training=training)
        _inference_only(self, conv.weights)
        self._maybe_tune(x_local.contiguous())
        return self._forward_impl(x_local, training)

    def _group_ks(self, x_local: torch.Tensor) -> tuple:
        return (2, 4) if self._fused(x_local) else ()

    def _fused(self, x_local: torch.Tensor) -> bool:
        """Whether (1+eps) x_i + aggr -> the MLP's first Dense runs fused into the
        pipelined passes (sum, a linear or ReLU first Dense, a shape the fused
        kernels take with two tables: C4's 256 -> 256)."""
        first = self.conv.mlp.layers[0]
        return (self._pipelined() and self.conv.aggregator == "sum" and first.activation in (None, torch.relu)
                and self.sg.backend.supports_fused(x_local.shape[1], first.units))

    def _forward_impl(self, x_local: torch.Tensor, training=None) -> torch.Tensor:
        sg, conv = self.sg, self.conv
        x_local = x_local.contiguous()
        with torch.no_grad():
            if self._fused(x_local):
                h = self._forward_fused(x_local)
                for layer in conv.mlp.layers[1:]:
                    h = layer(h, training=training) if isinstance(layer, Dropout) else layer(h)
                return h
            if self._pipelined():  # halo pipelined under the own-source pass
                h = sg.propagate_overlapped(x_local, conv.aggregator, gin_scale=float(conv._scale()))
            else:
                h = sg.propagate(x_local, conv.aggregator, epilogue=nat.EPI_GIN, xroot=x_local,
                                 gin_scale=conv._scale())
            return conv.mlp(h, training=training)

    def _forward_fused(self, x_local: torch.Tensor) -> torch.Tensor:
        """The pipelined GIN-sum passes with the MLP's first Dense fused in, as
        ShardedGCNConv._forward_merged (gin_conv.py:216-225 per shard):
        side stream: pack + exchange; main stream: out[rows not in H] =
        b + (s x_i + A_own x) W while the exchange is in flight; out[H] =
        b + (s x_i + A_own x + A_0 halo_0) W in one two-table launch once the
        first group has landed; out += (A_k halo_k) W per later group.  No
        [n_local, F_in] aggregate is written or read back.  The first Dense's
        ReLU goes into the overwriting launches when no later group adds to the
        rows, else onto out at the end (max(., 0) after the whole sum)."""
        sg, conv = self.sg, self.conv
        first = conv.mlp.layers[0]
        W, b = first.kernel, (first.bias if first.use_bias else None)
        pp = sg.exchange_plan(weighted=False)
        halo = sg.halo_buffer(x_local.shape[1], x_local, pp.n_rows)
        if pp.kind == "group":
            return self._forward_fused_grouped(x_local, W, b, pp, halo)
        unit = None if (use_merged_halo() or pp.kind == "allgather") else "none"
        unit = unit or sg.merge_unit or os.environ.get("KGX_HALO_MERGE", "step")
        light = halo_light() if pp.kind != "allgather" and unit != "none" else 0
        g_a, g_b, later, first_wait = sg.merged_passes(pp, unit, light)
        lights = sg.light_passes(pp, unit, light) if light > 0 and g_b is not None else []
        steps = [st for c in pp.chunks for st in c.steps]
        relu = first.activation is torch.relu
        kw = dict(weighted=False, pre_gin=True, gin_scale=float(conv._scale()), relu=relu and not later)
        works = sg.start_halo_exchange(x_local, halo, pp.chunks)
        handles = []
        for w, c in zip(works, pp.chunks):
            handles.extend(w.handles if w is not None else [None] * len(c.steps))
        waited = set()

        def wait_step(i):
            for j in range(i + 1):  # steps land in issue order on the comm stream
                if j not in waited:
                    waited.add(j)
                    if handles[j] is not None:
                        handles[j].wait()

        with kops.sharing_gpu():  # the exchange's packing and RCCL kernels run beside this pass
            out = sg.backend.aggregate_transform(g_a, x_local, W, bias=b, **kw)
        if g_b is not None:
            wait_step(first_wait)
            with kops.sharing_gpu() if later else contextlib.nullcontext():
                sg.backend.aggregate_transform(g_b, x_local, W, bias=b, out=out, x2=halo, accumulate=False, **kw)
        kw_light = dict(kw, relu=relu)  # light rows are complete when written: their ReLU goes in
        pending = list(lights)
        for n, (i, g, lo, hi) in enumerate(later):
            wait_step(i)
            last = n + 1 == len(later)
            with kops.sharing_gpu() if not last else contextlib.nullcontext():
                sg.backend.aggregate_transform(g, halo[lo: hi], W, out=out, weighted=False)
            while pending and pending[0][0] <= i:
                _, gl = pending.pop(0)
                with kops.sharing_gpu() if not last else contextlib.nullcontext():
                    sg.backend.aggregate_transform(gl, x_local, W, bias=b, out=out, x2=halo, accumulate=False,
                                                   **kw_light)
        for i, gl in pending:
            wait_step(i)
            sg.backend.aggregate_transform(gl, x_local, W, bias=b, out=out, x2=halo, accumulate=False, **kw_light)
        wait_step(len(steps) - 1)  # also orders the side stream's reads of x_local
        if relu and later:
            out = torch.relu_(out)
        return out


    def _forward_fused_grouped(self, x_local, W, b, pp: PushPullPlan, halo: torch.Tensor) -> torch.Tensor:
        """Destination-group exchange (kind "group", ShardedGraph.group_passes)
        with the first Dense fused: out[rows with no halo edge] = b + (s x_i +
        A_own x) W while the exchange is in flight, then per group k, once chunk
        k has landed, out[group k] = b + (s x_i + A_own x + A_halo halo) W in one
        two-table launch -- every row written once, so the first Dense's ReLU
        goes into every launch."""
        sg, conv = self.sg, self.conv
        first = conv.mlp.layers[0]
        g_a, passes = sg.group_passes(pp)
        steps = [st for c in pp.chunks for st in c.steps]
        kw = dict(weighted=False, pre_gin=True, gin_scale=float(conv._scale()), relu=first.activation is torch.relu)
        works = sg.start_halo_exchange(x_local, halo, pp.chunks)
        handles = []
        for w, c in zip(works, pp.chunks):
            handles.extend(w.handles if w is not None else [None] * len(c.steps))
        waited = set()

        def wait_step(i):
            for j in range(i + 1):  # steps land in issue order on the comm stream
                if j not in waited:
                    waited.add(j)
                    if handles[j] is not None:
                        handles[j].wait()

        with kops.sharing_gpu():  # the exchange's packing and RCCL kernels run beside this pass
            out = sg.backend.aggregate_transform(g_a, x_local, W, bias=b, **kw)
        for n, (i, g) in enumerate(passes):
            wait_step(i)
            with kops.sharing_gpu() if n + 1 < len(passes) else contextlib.nullcontext():
                sg.backend.aggregate_transform(g, x_local, W, bias=b, out=out, x2=halo, accumulate=False, **kw)
        wait_step(len(steps) - 1)  # also orders the side stream's reads of x_local
        return out


class ShardedSAGEConv(_ShardedWrap):
    """SAGEConv over a ShardedGraph: lin_neigh(AGG_j x_j) + lin_self(x_i) + b
    (sage_conv.py:405-439; the 'pooling' aggregator exchanges pool_mlp(x)
    rows and max-reduces them, :300-348).  Shard graph: no self loops, no
    GCN norm."""

    def __init__(self, output_dim: int, sg: ShardedGraph, **sage_kwargs):
        from .layers.sage_conv import SAGEConv

        super().__init__(SAGEConv(output_dim, exact=sg.exact, **sage_kwargs), sg)

    def _pipelined(self) -> bool:
        return not self.sg.exact and self.conv.actual_aggregator in ("sum", "mean")

    def forward(self, x_local: torch.Tensor, training=None) -> torch.Tensor:
        self._ensure_built(x_local)
        conv = self.conv
        if _training(conv.weights, x_local) and conv.actual_aggregator in ("sum", "mean"):
            if training and conv.dropout_rate > 0:
                raise NotImplementedError("ShardedSAGEConv: training with message dropout runs on the single-GPU "
                                          "SAGEConv (sage_conv.py:280-298 masks every message)")
            # training (sum / mean): the aggregation through _ShardedAggFn, lin_neigh(aggr) +
            # lin_self(x) + b, activation and L2 norm through torch autograd (sage_conv.py:404-439)
            agg = _ShardedAggFn.apply(x_local, self.sg, conv.actual_aggregator)
            return conv.update_nodes(x_local, agg)
        _inference_only(self, conv.weights)
        self._maybe_tune(x_local.contiguous())
        return self._forward_impl(x_local, training)

    def _forward_impl(self, x_local: torch.Tensor, training=None) -> torch.Tensor:
        sg, conv = self.sg, self.conv
        x_local = x_local.contiguous()
        with torch.no_grad():
            if conv.actual_aggregator == "pooling":
                aggr = sg.propagate(conv.pool_mlp(x_local).contiguous(), "max")
            elif self._pipelined():
                aggr = sg.propagate_overlapped(x_local, conv.actual_aggregator)
            else:
                aggr = sg.propagate(x_local, conv.actual_aggregator)
            return conv.update_nodes(x_local, aggr)


class ShardedGATv2Conv(_ShardedWrap):
    """GATv2Conv over a ShardedGraph (gatv2_conv.py:176-352 per shard).

    h = x W on the owner's rows (the layer's shared linear map, kgx_dense), the
    halo's h rows pulled over the shard's all-to-all plan, then ONE fused
    attention pass (kgx_gatv2) over [own h | halo h]: every destination's
    scores, segment softmax (gatv2_conv.py:291-311) and alpha-weighted sum run
    on its owner, whose shard CSR holds all of that row's in-edges in global
    input order -- so EXACT mode is bit-identical to the single-GPU layer.  The
    halo moves h, not partial sums: the softmax of a row needs every score
    a . leaky_relu(h_i + h_j), and h_i lives on the owner only.  Shard graph:
    self loops iff the layer adds them (default), no GCN norm
    (ShardedGraph.build(..., gcn_norm=False)).  Inference engine, like the
    other sharded layers."""

    def __init__(self, output_dim: int, sg: ShardedGraph, **gat_kwargs):
        from .layers.gatv2_conv import GATv2Conv

        super().__init__(GATv2Conv(output_dim, exact=sg.exact, **gat_kwargs), sg)
        if self.conv.add_self_loops_flag != sg.self_loops:
            raise ValueError(f"ShardedGATv2Conv: add_self_loops={self.conv.add_self_loops_flag} needs a shard graph "
                             f"built with self_loops={self.conv.add_self_loops_flag}")

    def forward(self, x_local: torch.Tensor, training=None) -> torch.Tensor:
        self._ensure_built(x_local)
        _inference_only(self, self.conv.weights)
        sg, conv = self.sg, self.conv
        H, C = conv.heads, conv.features_per_head
        n = sg.n_local
        use_b = conv.use_bias and conv.bias is not None
        with torch.no_grad():
            h = sg.backend.transform(x_local.contiguous(), conv.linear_transform.kernel)
            table = sg.new_table(H * C, h)
            table[:n] = h
            del h
            sg.halo_exchange(table)
            out = sg.backend.gatv2(sg.graph, table, table[:n], conv.att, H, C, conv.negative_slope,
                                   bias=conv.bias if (use_b and conv.concat) else None, exact=sg.exact)
            if not conv.concat:  # gatv2_conv.py:341-346
                out = out.view(n, H, C).mean(dim=1)
                if use_b:
                    out = out + conv.bias
        return out
