"""Multi-process (world_size 2, gloo, CPU) test of the destination-range
sharding and halo-exchange logic of keras_geometric_amd.distributed.

The device work is done by a CPU backend built on the oracle (sequential
accumulation in CSR order), so the sharded result must be BIT-IDENTICAL to the
same computation on the unsharded graph — the property the HIP backend keeps
on the GPU (each row's edges stay in global input order on its owner)."""

import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from keras_geometric_amd import _native as nat
from keras_geometric_amd import distributed as kd
from oracle import keras_torch as K
from oracle import reference as R
from oracle.rmat import rmat_edges, scale_for


class OracleBackend:
    """CPU stand-in for KgxBackend (test infrastructure)."""

    def build_graph(self, src, dst, n_src, n_dst, n_features):
        rowptr, col, eid, deg = R.csr_by_destination(src.numpy(), dst.numpy(), n_src, n_dst, self_loops=False)
        t = torch.from_numpy
        return SimpleNamespace(rowptr=t(rowptr), col=t(col), eid=t(eid), deg=t(deg), n_dst=n_dst, n_src=n_src,
                               kept=int(rowptr[-1]), dinv=None, w=None, device=torch.device("cpu"))

    def dinv(self, deg):
        d = torch.clamp(deg, max=1 << 24).float() + torch.tensor(1e-12, dtype=torch.float32)
        return (1.0 / torch.from_numpy(np.sqrt(d.numpy()))).float()

    def edge_norm(self, g, dinv_dst, dinv_src):
        rows = torch.repeat_interleave(torch.arange(g.n_dst), g.deg.long())
        return dinv_dst[rows] * dinv_src[g.col.long()]

    def gather_rows(self, table, rows):
        return table[rows.long()]

    def split_by_source(self, g, cuts):
        rows = torch.repeat_interleave(torch.arange(g.n_dst), g.deg.long())
        col = g.col.long()
        parts = []
        for lo, hi in zip(cuts, cuts[1:]):
            m = (col >= lo) & (col < hi)
            deg = torch.bincount(rows[m], minlength=g.n_dst).int()
            rowptr = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(deg.long(), 0)]).int()
            parts.append(SimpleNamespace(rowptr=rowptr, col=(col[m] - lo).int(), eid=g.eid[m], deg=deg,
                                         n_dst=g.n_dst, kept=int(m.sum()), dinv=None, w=g.w[m] if g.w is not None else None,
                                         device=torch.device("cpu")))
        return parts

    def aggregate_accumulate(self, g, table, out, weighted=False, epilogue=nat.EPI_ACCUM, bias=None, xroot=None,
                             gin_scale=1.0, table2=None):
        table = table if table2 is None else torch.cat([table, table2])
        mask = getattr(g, "row_mask", None)
        if mask is None:
            mask = torch.ones(g.n_dst, dtype=torch.bool)
        if epilogue == nat.EPI_ACCUM:
            out[mask] += self.aggregate(g, table, "sum", weighted=weighted)[mask]
        else:
            y = self.aggregate(g, table, "sum", weighted=weighted, epilogue=epilogue, bias=bias, xroot=xroot,
                               gin_scale=gin_scale)
            out[mask] = y[mask]
        return out

    def transform(self, x, W, bias=None):
        y = torch.matmul(x, W)
        return y if bias is None else K.add(y, bias)

    def supports_fused(self, f_in, f_out):
        return True

    def restrict_rows(self, g, row_mask):
        return SimpleNamespace(**vars(g), row_mask=row_mask)

    def aggregate_transform(self, g, x, W, bias=None, out=None, x2=None, accumulate=True, weighted=True,
                            pre_gin=False, gin_scale=1.0, relu=False):
        """sum_e (w_e) x[col_e] in CSR order (pre_gin: gin_scale x_i + that, root
        rows of x), then @ W (+ bias, ReLU); out += ... if given (accumulate=False:
        overwrite); x2: sources >= len(x) are rows of x2.  A row-restricted graph
        (restrict_rows) writes only its rows; the others come out NaN (unwritten)
        so a pass that misses a row fails the test."""
        table = x if x2 is None else torch.cat([x, x2])
        agg = self.aggregate(g, table, "sum", weighted=weighted)
        if pre_gin:  # (1+eps) x_i + aggr (gin_conv.py:216-222)
            agg = torch.tensor(gin_scale, dtype=torch.float32) * x[: g.n_dst] + agg
        y = torch.matmul(agg, W)
        if bias is not None:
            y = K.add(y, bias)
        if relu:
            y = torch.relu(y)
        mask = getattr(g, "row_mask", None)
        if mask is None:
            mask = torch.ones(g.n_dst, dtype=torch.bool)
        if out is None:
            return torch.where(mask.unsqueeze(1), y, torch.full_like(y, float("nan")))
        if accumulate:
            out[mask] += y[mask]
        else:
            out[mask] = y[mask]
        return out

    def aggregate(self, g, table, reduce="sum", weighted=False, epilogue=nat.EPI_NONE, bias=None, **kw):
        rows = torch.repeat_interleave(torch.arange(g.n_dst), g.deg.long())
        msg = table[g.col.long()]
        if weighted:
            msg = msg * g.w.unsqueeze(1)
        out = R.aggregate(reduce, msg, rows, g.n_dst)
        if epilogue == nat.EPI_BIAS:
            out = K.add(out, bias)
        elif epilogue == nat.EPI_GIN:  # (1+eps) x_i + aggr (gin_conv.py:216-222)
            out = torch.tensor(kw["gin_scale"], dtype=torch.float32) * kw["xroot"] + out
        mask = getattr(g, "row_mask", None)
        if mask is not None:  # a row-restricted launch leaves the other rows unwritten
            out = torch.where(mask.unsqueeze(1), out, torch.full_like(out, float("nan")))
        return out


def _oracle_gatv2(g, h_src, h_dst, att, heads, channels, negative_slope, bias=None, exact=False):
    """GATv2 attention over a shard CSR with the oracle's ops in its order
    (oracle/reference.py gatv2_forward, gatv2_conv.py:241-352): per-edge score,
    segment max / exp / segment sum by destination, alpha-weighted sum of h_j."""
    n = g.n_dst
    rows = torch.repeat_interleave(torch.arange(n), g.deg.long())
    hs = h_src.reshape(-1, heads, channels)
    hd = h_dst.reshape(-1, heads, channels)
    h_j = K.take(hs, g.col.long(), axis=0)
    h_i = K.take(hd, rows, axis=0)
    z = K.leaky_relu(K.add(h_i, h_j), negative_slope)
    scores = torch.sum(K.multiply(z, K.convert(att)), dim=-1)
    mx = K.segment_max(scores, rows, n)
    ex = torch.exp(torch.subtract(scores, K.take(mx, rows, axis=0)))
    ssum = K.segment_sum(ex, rows, n)
    alpha = K.divide(ex, K.add(K.take(ssum, rows, axis=0), 1e-10))
    msg = torch.unsqueeze(alpha, -1) * h_j
    out = K.segment_sum(msg.reshape(-1, heads * channels), rows, n)
    return out + K.convert(bias) if bias is not None else out


OracleBackend.gatv2 = staticmethod(_oracle_gatv2)


def _oracle_aggregate_transposed(self, g, t, weighted=True):
    """sum over every source row's out-edges of (w_e) t[dst_e], in CSR slot order."""
    rows = torch.repeat_interleave(torch.arange(g.n_dst), g.deg.long())
    msg = t[rows]
    if weighted:
        msg = msg * g.w.unsqueeze(1)
    return R.aggregate("sum", msg, g.col.long(), g.n_src)


OracleBackend.aggregate_transposed = _oracle_aggregate_transposed


class UnfusedOracleBackend(OracleBackend):
    def supports_fused(self, f_in, f_out):
        return False


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


N, E, F_IN, F_OUT = 1000, 12000, 16, 8


F_WIDE = 24  # F_out > F_in: the unfused sharded GCN aggregates X first


def _wide_weights():
    rng = np.random.default_rng(7)
    return (rng.standard_normal((F_IN, F_WIDE)) * 0.3).astype(np.float32), \
        rng.standard_normal(F_WIDE).astype(np.float32)


def _graph():
    s, d = rmat_edges(21, scale_for(N), N, 0, E)
    rng = np.random.default_rng(0)
    x = rng.standard_normal((N, F_IN)).astype(np.float32)
    W = (rng.standard_normal((F_IN, F_OUT)) * 0.3).astype(np.float32)
    b = rng.standard_normal(F_OUT).astype(np.float32)
    return s, d, x, W, b


def _full_graph_reference(world_size=1):
    """The same backend on the unsharded graph (world of one)."""
    s, d, x, W, b = _graph()
    be = OracleBackend()
    n = N
    src = torch.from_numpy(s).long()
    dst = torch.from_numpy(d).long()
    ar = torch.arange(n)
    g = be.build_graph(torch.cat([src, ar]).int(), torch.cat([dst, ar]).int(), n, n, F_OUT)
    dinv = be.dinv(g.deg)
    g.w = be.edge_norm(g, dinv, dinv)
    h = torch.from_numpy(x) @ torch.from_numpy(W)
    return be.aggregate(g, h, "sum", weighted=True, epilogue=nat.EPI_BIAS, bias=torch.from_numpy(b)), \
        be.aggregate(g, torch.from_numpy(x), "max")


def _worker(rank, world, chunks, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, d, x, W, b = _graph()
        bounds = kd.equal_bounds(N, world)
        lo, hi = bounds[rank], bounds[rank + 1]
        keep = (d >= lo) & (d < hi)  # stable: global input order kept
        sg = kd.ShardedGraph.build(torch.from_numpy(s[keep]), torch.from_numpy(d[keep]), bounds,
                                   backend=OracleBackend(), n_features=F_OUT, halo_chunks=chunks)
        assert len(sg.chunks) == chunks and sg.chunks[-1].hi == sg.n_halo
        h = torch.from_numpy(x[lo:hi]) @ torch.from_numpy(W)
        table = sg.new_table(F_OUT, h)
        table[: sg.n_local] = h
        sg.halo_exchange(table)
        gcn = sg.backend.aggregate(sg.graph, table, "sum", weighted=True, epilogue=nat.EPI_BIAS,
                                   bias=torch.from_numpy(b))
        mx = sg.propagate(torch.from_numpy(x[lo:hi]), "max")
        # the GCN layer's default (overlapped, own-then-halo) path
        layer = kd.ShardedGCNConv(F_OUT, sg)
        layer._build_device = torch.device("cpu")  # host-logic test with the oracle backend
        layer.build((hi - lo, F_IN))
        with torch.no_grad():
            layer.kernel.copy_(torch.from_numpy(W))
            layer.bias.copy_(torch.from_numpy(b))
        with torch.no_grad():
            y = layer(torch.from_numpy(x[lo:hi]))  # push-pull halo (the default)
        pp = sg._pp
        assert pp is not None and pp.n_rows == pp.n_pull + pp.n_push == pp.chunks[-1].hi
        def merged(unit):  # the plan's cached passes (keyed by unit, with the light-row bound when on)
            lt = kd.halo_light()
            return pp.merged[(unit, lt) if lt > 0 else unit]

        assert pp.merged is not None and merged("step")[1] is not None  # the first step folded into its rows' pass
        os.environ["KGX_HALO_MERGE"] = "chunk"  # a chunk's steps (pulled rows + partials) merged together
        try:
            with torch.no_grad():
                y_chunk = layer(torch.from_numpy(x[lo:hi]))
        finally:
            del os.environ["KGX_HALO_MERGE"]
        assert merged("chunk")[1] is not None
        # the own-only rows' pass before / after the merged pass (the default picks by the
        # number of later exchange groups): disjoint rows, so the same bits either way
        for order in ("0", "1"):
            os.environ["KGX_HALO_A_LATE"] = order
            try:
                with torch.no_grad():
                    y_order = layer(torch.from_numpy(x[lo:hi]))
            finally:
                del os.environ["KGX_HALO_A_LATE"]
            assert torch.equal(y_order, y), order
        os.environ["KGX_HALO_MERGED"] = "0"
        try:
            with torch.no_grad():
                y_unmerged = layer(torch.from_numpy(x[lo:hi]))  # own pass + accumulating chunk passes
        finally:
            del os.environ["KGX_HALO_MERGED"]
        os.environ["KGX_HALO_PUSH"] = "0"
        try:
            with torch.no_grad():
                y_pull = layer(torch.from_numpy(x[lo:hi]))  # pull-only halo
        finally:
            del os.environ["KGX_HALO_PUSH"]
        y_first = y
        if chunks > 1:  # a small first chunk (KGX_HALO_FIRST): the same rows, other chunk bounds
            os.environ["KGX_HALO_FIRST"] = "0.2"
            try:
                with torch.no_grad():
                    y_first = layer(torch.from_numpy(x[lo:hi]))
                ppf = sg._pp
                assert ppf is not pp and ppf.n_rows == pp.n_rows and len(ppf.chunks) == chunks
                sizes = [c.hi - c.lo for c in ppf.chunks]
                assert sizes[0] <= 0.25 * pp.n_rows + world, sizes
            finally:
                del os.environ["KGX_HALO_FIRST"]
        # light rows (KGX_HALO_LIGHT): rows of total degree <= L that reach a later exchange
        # group are written once, with all their edges, after the last group they need
        ys_light = []
        for light in ("7", "100000"):
            os.environ["KGX_HALO_LIGHT"] = light
            try:
                with torch.no_grad():
                    ys_light.append(layer(torch.from_numpy(x[lo:hi])).numpy())
            finally:
                del os.environ["KGX_HALO_LIGHT"]
            if chunks > 1:
                unit = sg.merge_unit or "step"
                lp = sg.light_passes(sg._pp, unit, int(light))
                assert lp, light  # some rows were deferred
        # K left open: the first forward times K = 1 / 2 / 4 (collective) and keeps the fastest
        sg2 = kd.ShardedGraph.build(torch.from_numpy(s[keep]), torch.from_numpy(d[keep]), bounds,
                                    backend=OracleBackend(), n_features=F_OUT)
        layer2 = kd.ShardedGCNConv(F_OUT, sg2)
        layer2._build_device = torch.device("cpu")
        layer2.build((hi - lo, F_IN))
        with torch.no_grad():
            layer2.kernel.copy_(torch.from_numpy(W))
            layer2.bias.copy_(torch.from_numpy(b))
        with torch.no_grad():
            y_tuned = layer2(torch.from_numpy(x[lo:hi]))
        # every candidate timed: the push-pull halo at K = 1 / 2 / 4 with each merge unit and
        # (this small graph's remote sources cover most rows) the all-gather at K = 1 / 2 / 4
        units = ("step", "chunk", "none")
        assert sorted(sg2.tuning) == sorted([f"halo:{k}:{u}" for k in (1, 2, 4) for u in units]
                                            + [f"allgather:{k}:{u}" for k in (1, 2, 4) for u in ("step", "none")]
                                            + [f"group:{k}:group" for k in (2, 4)])
        assert sg2.exchange in ("halo", "allgather", "group") and sg2.halo_k in (1, 2, 4)
        assert sg2.merge_unit in units + ("group",)
        assert len(sg2._pp.chunks) == sg2.halo_k and sg2._pp.kind == sg2.exchange
        # the all-gather exchange on its own (K = 1 and 3), within the tolerance of the reference
        ys_gather = []
        for kk in (1, 3):
            sg2.exchange, sg2.halo_k = "allgather", kk
            with torch.no_grad():
                ys_gather.append(layer2(torch.from_numpy(x[lo:hi])).numpy())
            assert sg2._pp.kind == "allgather" and len(sg2._pp.chunks) == kk
        # destination-group chunks: every row with halo edges written once, by its group's pass
        ys_group = []
        for kk in (2, 3):
            sg2.exchange, sg2.halo_k = "group", kk
            with torch.no_grad():
                ys_group.append(layer2(torch.from_numpy(x[lo:hi])).numpy())
            ppg = sg2._pp
            assert ppg.kind == "group" and len(ppg.chunks) == kk and ppg.merged["group"] is not None
            assert ppg.n_rows == ppg.n_pull + ppg.n_push == ppg.chunks[-1].hi
        # the pull-only halo through the merged passes (no partial sums pushed)
        sg2.exchange, sg2.halo_k = "pull", 2
        with torch.no_grad():
            y_pullplan = layer2(torch.from_numpy(x[lo:hi])).numpy()
        assert sg2._pp.kind == "pull" and sg2._pp.n_push == 0 and len(sg2._pp.chunks) == 2
        # shapes the fused kernel does not take: X W first, then the pipelined weighted sum
        sg3 = kd.ShardedGraph.build(torch.from_numpy(s[keep]), torch.from_numpy(d[keep]), bounds,
                                    backend=UnfusedOracleBackend(), n_features=F_OUT, halo_chunks=chunks)
        layer3 = kd.ShardedGCNConv(F_OUT, sg3)
        layer3._build_device = torch.device("cpu")
        layer3.build((hi - lo, F_IN))
        with torch.no_grad():
            layer3.kernel.copy_(torch.from_numpy(W))
            layer3.bias.copy_(torch.from_numpy(b))
        with torch.no_grad():
            y_unfused = layer3(torch.from_numpy(x[lo:hi]))
        assert sg3._pp is not None
        # F_out > F_in on the unfused path: aggregate X first (narrower rows), then X W + b
        W2, b2 = _wide_weights()
        layer4 = kd.ShardedGCNConv(F_WIDE, sg3)
        layer4._build_device = torch.device("cpu")
        layer4.build((hi - lo, F_IN))
        with torch.no_grad():
            layer4.kernel.copy_(torch.from_numpy(W2))
            layer4.bias.copy_(torch.from_numpy(b2))
            y_wide = layer4(torch.from_numpy(x[lo:hi]))
        # an unweighted sum / mean over a GCN-normed shard graph: the push-pull plan
        # must push plain partial sums (plans are kept per (K, weighted))
        xl = torch.from_numpy(x[lo:hi])
        mean_pp = sg.propagate_overlapped(xl, "mean")
        sum_pp = sg.propagate_overlapped(xl, "sum")
        mean_tab, sum_tab = sg.propagate(xl, "mean"), sg.propagate(xl, "sum")
        scale = sg.propagate(xl.abs(), "sum")
        assert (mean_pp - mean_tab).abs().max() <= 1e-5 * max(1.0, float(scale.max()))
        assert ((sum_pp - sum_tab).abs() <= 1e-5 * scale.clamp_min(1)).all()
        with torch.no_grad():
            y_again = layer(xl)  # the weighted plan is still the one the GCN layer uses
        assert torch.equal(y_again, y)
        q.put((rank, gcn.numpy(), mx.numpy(), sg.n_halo, sum(sg.send_counts), y.numpy(), y_pull.numpy(), pp.n_push,
               y_tuned.numpy(), y_unfused.numpy(), y_wide.numpy(), y_unmerged.numpy(), ys_gather[0], ys_gather[1],
               y_chunk.numpy(), y_pullplan, y_first.numpy(), ys_group[0], ys_group[1], ys_light[0], ys_light[1]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world,chunks", [(2, 1), (2, 4), (3, 3), (8, 2)])
def test_sharded_equals_unsharded_bitwise(world, chunks):
    """EXACT table path bit-identical to the unsharded graph for any halo
    chunking (the chunk-major halo table only renames source rows), and the
    chunk-pipelined GCN layer (own part, then one accumulating part per chunk)
    within the north-star tolerance."""
    if torch.cuda.is_initialized():
        pytest.skip("never start processes from a process that has initialised the GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, chunks, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        rank, *res = q.get(timeout=90)
        results[rank] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gcn = np.concatenate([results[r][0] for r in range(world)])
    mx = np.concatenate([results[r][1] for r in range(world)])
    ref_gcn, ref_max = _full_graph_reference()
    np.testing.assert_array_equal(gcn, ref_gcn.numpy())
    np.testing.assert_array_equal(mx, ref_max.numpy())
    assert sum(results[r][2] for r in range(world)) == sum(results[r][3] for r in range(world)) > 0
    # and the oracle GCN layer within the north-star tolerance (1-ulp dinv differences)
    s, d, x, W, b = _graph()
    y = R.gcn_forward(torch.from_numpy(x), torch.from_numpy(np.stack([s, d])), torch.from_numpy(W),
                      torch.from_numpy(b)).numpy()
    err = np.abs(gcn - y) / np.maximum(1, np.abs(y))
    assert err.max() <= 1e-5
    # overlapped layer path, push-pull and pull-only halos: own-source part, then
    # one part per halo chunk per row (re-associated sums)
    assert sum(results[r][6] for r in range(world)) > 0  # partial sums were pushed
    for i in (4, 5, 7, 8, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19):
        y_split = np.concatenate([results[r][i] for r in range(world)])
        err = np.abs(y_split - y) / np.maximum(1, np.abs(y))
        assert err.max() <= 1e-5
    W2, b2 = _wide_weights()
    y2 = R.gcn_forward(torch.from_numpy(x), torch.from_numpy(np.stack([s, d])), torch.from_numpy(W2),
                       torch.from_numpy(b2)).numpy()
    got = np.concatenate([results[r][9] for r in range(world)])
    assert (np.abs(got - y2) / np.maximum(1, np.abs(y2))).max() <= 1e-5



def _conv_worker(rank, world, port, q):
    """ShardedGINConv / ShardedSAGEConv on a shard graph without loops or norms."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, d, x, _, _ = _graph()
        bounds = kd.equal_bounds(N, world)
        lo, hi = bounds[rank], bounds[rank + 1]
        keep = (d >= lo) & (d < hi)
        sg = kd.ShardedGraph.build(torch.from_numpy(s[keep]), torch.from_numpy(d[keep]), bounds,
                                   backend=OracleBackend(), n_features=F_IN, self_loops=False, gcn_norm=False)
        xl = torch.from_numpy(x[lo:hi])
        outs, grouped = [], []
        for layer in (kd.ShardedGINConv(F_OUT, sg, mlp_hidden=[12], aggregator="sum", eps_init=0.25),
                      kd.ShardedGINConv(F_OUT, sg, aggregator="max"),
                      kd.ShardedSAGEConv(F_OUT, sg, aggregator="mean", normalize=True),
                      kd.ShardedSAGEConv(F_OUT, sg, aggregator="pooling", pool_hidden_dim=10)):
            layer._ensure_built(xl)  # weights drawn per rank, then broadcast from rank 0
            if isinstance(layer, kd.ShardedGINConv) and layer.conv.aggregator == "sum":
                assert layer._fused(xl)  # (1+eps) x + aggr -> first Dense (+ReLU) fused into the passes
            with torch.no_grad():
                outs.append((layer(xl).numpy(), list(layer.conv.get_weights())))
                if isinstance(layer, kd.ShardedGINConv) and layer.conv.aggregator == "sum":
                    # destination-group chunks on the fused GIN path: each row written once
                    saved = (sg.exchange, sg.halo_k, sg.merge_unit)
                    for kk in (2, 3):
                        sg.exchange, sg.halo_k = "group", kk
                        grouped.append(layer(xl).numpy())  # checked against the oracle like outs[0]
                        assert sg.exchange_plan(weighted=False).kind == "group"
                    sg.exchange, sg.halo_k, sg.merge_unit = saved
                if isinstance(layer, kd.ShardedSAGEConv) and layer.conv.aggregator == "mean":
                    # light rows on the plain sum / mean passes (off unless KGX_HALO_LIGHT is set)
                    os.environ["KGX_HALO_LIGHT"] = "7"
                    try:
                        grouped.append(layer(xl).numpy())
                    finally:
                        del os.environ["KGX_HALO_LIGHT"]
        q.put((rank, (outs, grouped)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_sharded_gin_sage_layers():
    """Sharded GIN (sum / max) and SAGE (mean + L2 norm / pooling) equal the
    oracle layers on the whole graph (within 1e-5), with rank 0's weights."""
    if torch.cuda.is_initialized():
        pytest.skip("never start processes from a process that has initialised the GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_conv_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res2 = dict(q.get(timeout=90) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = {r: v[0] for r, v in res2.items()}
    s, d, x, _, _ = _graph()
    X, EI = torch.from_numpy(x), torch.from_numpy(np.stack([s, d]))
    for i in range(4):
        for a, b in zip(res[0][i][1], res[1][i][1]):  # broadcast: identical weights on every rank
            np.testing.assert_array_equal(a, b)
    w = [[torch.from_numpy(a) for a in res[0][i][1]] for i in range(4)]
    refs = [
        R.gin_forward(X, EI, [(w[0][0], w[0][1], "relu"), (w[0][2], w[0][3], None)], "sum", eps=0.25),
        R.gin_forward(X, EI, [(w[1][0], w[1][1], None)], "max"),
        # SAGE weights in Layer.weights order: bias, [pool kernel, pool bias,] lin_neigh, lin_self
        R.sage_forward(X, EI, w[2][1], w[2][2], w[2][0], "mean", normalize=True),
        R.sage_forward(X, EI, w[3][3], w[3][4], w[3][0], "pooling", pool=(w[3][1], w[3][2], "relu")),
    ]
    # the sum / mean layers take the pipelined path (own part, then one
    # accumulating part per halo chunk): a re-association of each row's sum,
    # bounded by the same computation on absolute values (|x|, |W|, |b|)
    Xa = X.abs()
    wa = [[a.abs() for a in wl] for wl in w]
    scales = [
        R.gin_forward(Xa, EI, [(wa[0][0], wa[0][1], "relu"), (wa[0][2], wa[0][3], None)], "sum", eps=0.25).numpy(),
        None,
        None,  # L2-normalised rows: |out| <= 1
        None,
    ]
    errs = []
    for i, ref in enumerate(refs):
        got = np.concatenate([res[r][i][0] for r in range(world)])
        ref = ref.numpy()
        scale = np.maximum(1, np.abs(ref) if scales[i] is None else scales[i])
        errs.append(float((np.abs(got - ref) / scale).max()))
    # the fused GIN layer again with destination-group chunks (K 2, 3): each row written once
    for k in range(2):
        got = np.concatenate([res2[r][1][k] for r in range(world)])
        errs.append(float((np.abs(got - refs[0].numpy()) / np.maximum(1, scales[0])).max()))
    got = np.concatenate([res2[r][1][2] for r in range(world)])  # SAGE mean with light rows
    errs.append(float((np.abs(got - refs[2].numpy()) / np.maximum(1, np.abs(refs[2].numpy()))).max()))
    assert max(errs) <= 1e-5, errs


def _local_only_worker(rank, world, port, q):
    """Every edge stays inside its destination's shard: no halo rows at all."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, d, x, W, b = _local_only_graph()
        bounds = kd.equal_bounds(N, world)
        lo, hi = bounds[rank], bounds[rank + 1]
        keep = (d >= lo) & (d < hi)
        sg = kd.ShardedGraph.build(torch.from_numpy(s[keep]), torch.from_numpy(d[keep]), bounds,
                                   backend=OracleBackend(), n_features=F_OUT)
        layer = kd.ShardedGCNConv(F_OUT, sg)
        layer._build_device = torch.device("cpu")
        layer.build((hi - lo, F_IN))
        with torch.no_grad():
            layer.kernel.copy_(torch.from_numpy(W))
            layer.bias.copy_(torch.from_numpy(b))
        with torch.no_grad():
            y = layer(torch.from_numpy(x[lo:hi]))
        gsg = kd.ShardedGraph.build(torch.from_numpy(s[keep]), torch.from_numpy(d[keep]), bounds,
                                    backend=OracleBackend(), n_features=F_IN, self_loops=False, gcn_norm=False)
        gin = kd.ShardedGINConv(F_OUT, gsg, aggregator="sum", eps_init=0.5)
        gin._ensure_built(torch.from_numpy(x[lo:hi]))
        with torch.no_grad():
            h = gin(torch.from_numpy(x[lo:hi]))
        q.put((rank, sg.n_halo, sg._pp.n_rows, y.numpy(), h.numpy(), [a for a in gin.conv.get_weights()]))
    finally:
        dist.destroy_process_group()


def _local_only_graph():
    s, d, x, W, b = _graph()
    half = N // 2
    s = np.where((s < half) == (d < half), s, (s + half) % N).astype(s.dtype)  # source moved into d's half
    return s, d, x, W, b


@pytest.mark.timeout(180)
def test_sharded_no_halo():
    """Shards without any remote source: empty halo plans (no pulled rows, no
    pushed partials, empty chunks), chunk tuning and the pipelined GCN / GIN
    paths still run and equal the oracle layers."""
    if torch.cuda.is_initialized():
        pytest.skip("never start processes from a process that has initialised the GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_local_only_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=90)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(res[r][0] == 0 and res[r][1] == 0 for r in range(world))
    s, d, x, W, b = _local_only_graph()
    X, EI = torch.from_numpy(x), torch.from_numpy(np.stack([s, d]))
    y = R.gcn_forward(X, EI, torch.from_numpy(W), torch.from_numpy(b)).numpy()
    got = np.concatenate([res[r][2] for r in range(world)])
    assert (np.abs(got - y) / np.maximum(1, np.abs(y))).max() <= 1e-5
    w = [torch.from_numpy(a) for a in res[0][4]]
    h = R.gin_forward(X, EI, [(w[0], w[1], None)], "sum", eps=0.5).numpy()
    got = np.concatenate([res[r][3] for r in range(world)])
    assert (np.abs(got - h) / np.maximum(1, np.abs(h))).max() <= 1e-5


def _uneven_graph():
    """Rank 0's rows draw every edge from rank 1's nodes, rank 1's rows only from
    their own: one rank has a large halo, the other none."""
    s, d, x, W, b = _graph()
    half = N // 2
    s = np.where(d < half, half + s % half, half + s % half).astype(s.dtype)
    return s, d, x, W, b


def _uneven_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, d, x, W, b = _uneven_graph()
        bounds = kd.equal_bounds(N, world)
        lo, hi = bounds[rank], bounds[rank + 1]
        keep = (d >= lo) & (d < hi)
        sg = kd.ShardedGraph.build(torch.from_numpy(s[keep]), torch.from_numpy(d[keep]), bounds,
                                   backend=OracleBackend(), n_features=F_OUT)
        os.environ.update(KGX_EXCHANGE="allgather", KGX_HALO_MERGE="chunk")
        try:  # the all-gather's "chunk" unit maps to "step" instead of emptying the list
            fixed = sg.exchange_candidates()
        finally:
            del os.environ["KGX_EXCHANGE"], os.environ["KGX_HALO_MERGE"]
        os.environ["KGX_EXCHANGE"] = "pull"
        try:  # the pull-only halo is not timed by default, but a fixed choice still tunes K and unit
            assert sg.exchange_candidates() == [("pull", k, u) for k in (1, 2, 4) for u in ("step", "chunk", "none")]
        finally:
            del os.environ["KGX_EXCHANGE"]
        layer = kd.ShardedGCNConv(F_OUT, sg)
        layer._build_device = torch.device("cpu")
        layer.build((hi - lo, F_IN))
        with torch.no_grad():
            layer.kernel.copy_(torch.from_numpy(W))
            layer.bias.copy_(torch.from_numpy(b))
            y = layer(torch.from_numpy(x[lo:hi]))  # first forward: the collective tuner
        import bench  # the N > 1 line's per-rank diagnostics (bench.shard_summary)

        info = bench.shard_summary(sg, "gcn", F_IN, F_OUT, False)
        q.put((rank, sg.n_halo, sorted(sg.tuning), (sg.exchange, sg.halo_k, sg.merge_unit), fixed, y.numpy(),
               sg.tuning_s, info))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_sharded_uneven_halo_tuner_agrees():
    """One rank with a large halo, one with none: every rank lists and times the
    same exchange candidates (the all-gather included, decided on the largest
    halo), agrees on the choice, and the layer equals the oracle."""
    if torch.cuda.is_initialized():
        pytest.skip("never start processes from a process that has initialised the GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_uneven_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] > 4 * max(res[1][0], 1)  # very uneven halos
    assert res[0][1] == res[1][1] and any(k.startswith("allgather:") for k in res[0][1])
    assert res[0][2] == res[1][2]
    assert res[0][3] == res[1][3] == [("allgather", k, "step") for k in (1, 2, 4)]
    assert res[0][5] is not None and res[0][5] >= 0
    for r in range(world):  # what the N > 1 bench line reports per rank
        info = res[r][6]
        assert info["backend"] == "gloo" and info["world_size_reported"] == world
        assert (info["exchange"], info["halo_chunks"], info["merge_unit"]) == res[r][2]
        assert sorted(info["exchange_tuning_s"]) == res[r][1]
        assert info["exchange_tuning_total_s"] > 0 and info["exchange_tuning_skipped"] == 0
    s, d, x, W, b = _uneven_graph()
    y = R.gcn_forward(torch.from_numpy(x), torch.from_numpy(np.stack([s, d])), torch.from_numpy(W),
                      torch.from_numpy(b)).numpy()
    got = np.concatenate([res[r][4] for r in range(world)])
    assert (np.abs(got - y) / np.maximum(1, np.abs(y))).max() <= 1e-5


def _gat_worker(rank, world, port, q):
    """ShardedGATv2Conv (concat and mean over heads) on a shard graph with self loops."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, d, x, _, _ = _graph()
        bounds = kd.equal_bounds(N, world)
        lo, hi = bounds[rank], bounds[rank + 1]
        keep = (d >= lo) & (d < hi)
        sg = kd.ShardedGraph.build(torch.from_numpy(s[keep]), torch.from_numpy(d[keep]), bounds,
                                   backend=OracleBackend(), n_features=F_IN, gcn_norm=False, halo_chunks=2)
        assert sg.n_halo > 0
        xl = torch.from_numpy(x[lo:hi])
        outs = []
        for layer in (kd.ShardedGATv2Conv(4, sg, heads=3, bias_initializer="glorot_uniform"),
                      kd.ShardedGATv2Conv(5, sg, heads=2, concat=False, negative_slope=0.1,
                                          bias_initializer="glorot_uniform")):
            layer._ensure_built(xl)
            with pytest.raises(NotImplementedError):  # inference-only
                layer(xl)
            with torch.no_grad():
                outs.append((layer(xl).numpy(), list(layer.conv.get_weights())))
        with pytest.raises(ValueError):  # a shard graph without loops for a layer that adds them
            sg_nl = kd.ShardedGraph.build(torch.from_numpy(s[keep]), torch.from_numpy(d[keep]), bounds,
                                          backend=OracleBackend(), n_features=F_IN, self_loops=False,
                                          gcn_norm=False)
            kd.ShardedGATv2Conv(4, sg_nl)
        q.put((rank, outs))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_sharded_gatv2_layer_bitwise():
    """ShardedGATv2Conv at world 2 (pulled h halo in two chunks, one attention
    pass per owner) equals oracle.reference.gatv2_forward on the whole graph
    with rank 0's weights BIT FOR BIT: every destination's scores, softmax and
    weighted sum run on its owner over its in-edges in global input order
    (gatv2_conv.py:176-352)."""
    if torch.cuda.is_initialized():
        pytest.skip("never start processes from a process that has initialised the GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gat_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=90) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s, d, x, _, _ = _graph()
    X, EI = torch.from_numpy(x), torch.from_numpy(np.stack([s, d]))
    for i, (heads, concat, slope) in enumerate(((3, True, 0.2), (2, False, 0.1))):
        for a, b in zip(res[0][i][1], res[1][i][1]):  # broadcast: identical weights on every rank
            np.testing.assert_array_equal(a, b)
        # Layer.weights order: att, final_bias, then linear_transform's kernel
        att, bias, kernel = (torch.from_numpy(a) for a in res[0][i][1])
        ref = R.gatv2_forward(X, EI, kernel, att, bias, heads=heads, concat=concat, negative_slope=slope).numpy()
        got = np.concatenate([res[r][i][0] for r in range(world)])
        np.testing.assert_array_equal(got, ref)


def _progress_worker(rank, world, port, q):
    """The N > 1 progress reporting: per-rank shard-build and tuner lines, a
    heartbeat while the first forward runs, and the KGX_TUNE_BUDGET_S bound."""
    import io

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KGX_LOG="1", KGX_HEARTBEAT_S="0.02")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf = io.StringIO()
    kd.LOG_STREAM = buf
    try:
        s, d, x, W, b = _graph()
        bounds = kd.equal_bounds(N, world)
        lo, hi = bounds[rank], bounds[rank + 1]
        keep = (d >= lo) & (d < hi)
        sg = kd.ShardedGraph.build(torch.from_numpy(s[keep]), torch.from_numpy(d[keep]), bounds,
                                   backend=OracleBackend(), n_features=F_OUT)
        layer = kd.ShardedGCNConv(F_OUT, sg)
        layer._build_device = torch.device("cpu")
        layer.build((hi - lo, F_IN))
        os.environ["KGX_TUNE_BUDGET_S"] = "0"  # the first candidate is timed, the rest left untimed
        try:
            with kd.heartbeat(rank, "first forward"), torch.no_grad():
                import time as _t

                _t.sleep(0.1)  # a slow first forward: the heartbeat must tick meanwhile
                layer(torch.from_numpy(x[lo:hi]))
        finally:
            del os.environ["KGX_TUNE_BUDGET_S"]
        n_cands = len(sg.tuning)  # the layer's own candidate list (GCN adds group:2 / group:4)
        assert n_cands >= len(sg.exchange_candidates())
        q.put((rank, buf.getvalue(), sg.tuning_skipped, n_cands, sg.tuning_s, sorted(sg.tuning.items())))
    finally:
        kd.LOG_STREAM = None
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_n_gt_1_progress_and_tune_budget():
    """What a stalled N > 1 first forward leaves on stderr: every rank prints its
    shard build, each exchange plan and tuner candidate, and a heartbeat line at
    least every KGX_HEARTBEAT_S while the forward runs (bench.py wraps the
    shard build and the first forward in distributed.heartbeat, 30 s by
    default); KGX_TUNE_BUDGET_S bounds the tune (candidates past it untimed,
    the same on every rank)."""
    if torch.cuda.is_initialized():
        pytest.skip("never start processes from a process that has initialised the GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_progress_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        text, skipped, n_cands, tuning_s, tuning = res[r]
        lines = text.splitlines()
        assert all(ln.startswith(f"[kgx r{r}] ") for ln in lines), lines[:3]
        assert any("shard build:" in ln for ln in lines)
        assert any("tune:" in ln and "budget 0 s" in ln for ln in lines)
        assert sum("first forward: running" in ln for ln in lines) >= 2  # ticks during the forward
        assert any("first forward: done in" in ln for ln in lines)
        assert n_cands > 1 and skipped == n_cands - 1 and tuning_s is not None
        assert sum(v != float("inf") for _, v in tuning) == 1
    assert res[0][4] == res[1][4]  # the same candidates timed / skipped on every rank


def _train_worker(rank, world, port, q):
    """ShardedGCNConv with gradients: forward on the pulled halo table, backward
    through the transposed shard CSR, halo gradients pushed back, dW / db all-reduced."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, d, x, W, b = _graph()
        bounds = kd.equal_bounds(N, world)
        lo, hi = bounds[rank], bounds[rank + 1]
        keep = (d >= lo) & (d < hi)
        sg = kd.ShardedGraph.build(torch.from_numpy(s[keep]), torch.from_numpy(d[keep]), bounds,
                                   backend=OracleBackend(), n_features=F_OUT, halo_chunks=2)
        layer = kd.ShardedGCNConv(F_OUT, sg)
        layer._build_device = torch.device("cpu")
        layer.build((hi - lo, F_IN))
        with torch.no_grad():
            layer.kernel.copy_(torch.from_numpy(W))
            layer.bias.copy_(torch.from_numpy(b))
        xl = torch.from_numpy(x[lo:hi]).clone().requires_grad_(True)
        y = layer(xl)
        r = torch.from_numpy(np.random.default_rng(3).standard_normal((N, F_OUT)).astype(np.float32))[lo:hi]
        (y * r).sum().backward()
        with torch.no_grad():
            y_inf = layer(torch.from_numpy(x[lo:hi]))  # the inference path: the same forward values
        q.put((rank, y.detach().numpy(), xl.grad.numpy(), layer.kernel.grad.numpy(), layer.bias.grad.numpy(),
               y_inf.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_sharded_gcn_backward():
    """Sharded GCNConv training step at world 2 against torch autograd through
    the oracle's whole-graph forward (oracle.reference.gcn_forward): the output,
    dX (every rank's rows), dW and db (all-reduced) within 1e-5 of max(1, |ref|)
    (dW / db: sums over all rows, sqrt(N) * 1e-5 as the single-GPU backward
    tests use)."""
    if torch.cuda.is_initialized():
        pytest.skip("never start processes from a process that has initialised the GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s, d, x, W, b = _graph()
    X = torch.from_numpy(x).clone().requires_grad_(True)
    Wt = torch.from_numpy(W).clone().requires_grad_(True)
    bt = torch.from_numpy(b).clone().requires_grad_(True)
    y = R.gcn_forward(X, torch.from_numpy(np.stack([s, d])), Wt, bt)
    rr = torch.from_numpy(np.random.default_rng(3).standard_normal((N, F_OUT)).astype(np.float32))
    (y * rr).sum().backward()

    def close(got, ref, tol):
        err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= tol, err.max()

    close(np.concatenate([res[r][0] for r in range(world)]), y.detach().numpy(), 1e-5)
    close(np.concatenate([res[r][4] for r in range(world)]), y.detach().numpy(), 1e-5)
    close(np.concatenate([res[r][1] for r in range(world)]), X.grad.numpy(), 1e-5)
    for r in range(world):  # all-reduced: the same on every rank
        np.testing.assert_array_equal(res[r][2], res[0][2])
        np.testing.assert_array_equal(res[r][3], res[0][3])
    close(res[0][2], Wt.grad.numpy(), 1e-5 * np.sqrt(N))
    close(res[0][3], bt.grad.numpy(), 1e-5 * np.sqrt(N))


def test_chunk_slice_bounds():
    """chunk_slice: even cuts, or a first chunk of floor(count * f) rows and the
    rest split evenly; the slices tile [0, count) for any count and K."""
    for count in (0, 1, 7, 100, 12345):
        for K in (1, 2, 3, 4):
            for first in (None, 0.1, 0.5):
                cuts = [kd.chunk_slice(count, k, K, first) for k in range(K)]
                assert cuts[0][0] == 0 and cuts[-1][1] == count
                assert all(a <= b for a, b in cuts) and all(cuts[k][1] == cuts[k + 1][0] for k in range(K - 1))
                if first is not None and K > 1:
                    assert cuts[0][1] == int(count * first)
    assert kd.chunk_slice(10, 1, 4) == (2, 5)
    for count in (0, 1, 7, 100, 12345):  # KGX_HALO_WEIGHTS: K relative sizes
        for w in ((1.0, 4.0, 1.0), (2.0, 1.0), (1.0, 3.0, 3.0, 1.0)):
            cuts = [kd.chunk_slice(count, k, len(w), w) for k in range(len(w))]
            assert cuts[0][0] == 0 and cuts[-1][1] == count
            assert all(a <= b for a, b in cuts) and all(cuts[k][1] == cuts[k + 1][0] for k in range(len(w) - 1))
    assert [kd.chunk_slice(1000, k, 3, (1.0, 4.0, 1.0)) for k in range(3)] == [(0, 166), (166, 833), (833, 1000)]


def test_halo_chunk_weights_env(monkeypatch):
    monkeypatch.setenv("KGX_HALO_WEIGHTS", "1,4,1")
    assert kd.halo_chunk_weights(3) == (1.0, 4.0, 1.0)
    assert kd.halo_chunk_weights(2) is None  # names K weights or is ignored
    monkeypatch.setenv("KGX_HALO_WEIGHTS", "1,0,1")
    assert kd.halo_chunk_weights(3) is None


def _train_gin_sage_worker(rank, world, port, q):
    """ShardedGINConv (sum, trainable eps) and ShardedSAGEConv (mean, L2 norm) with
    gradients: _ShardedAggFn over the pulled halo table, the node update through
    torch autograd, weight gradients all-reduced by the layers' hooks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, d, x, _, _ = _graph()
        bounds = kd.equal_bounds(N, world)
        lo, hi = bounds[rank], bounds[rank + 1]
        keep = (d >= lo) & (d < hi)
        sg = kd.ShardedGraph.build(torch.from_numpy(s[keep]), torch.from_numpy(d[keep]), bounds,
                                   backend=OracleBackend(), n_features=F_IN, self_loops=False, gcn_norm=False,
                                   halo_chunks=2)
        r = torch.from_numpy(np.random.default_rng(5).standard_normal((N, F_OUT)).astype(np.float32))[lo:hi]
        out = []
        for layer in (kd.ShardedGINConv(F_OUT, sg, mlp_hidden=[12], aggregator="sum", eps_init=0.25, train_eps=True),
                      kd.ShardedGINConv(F_OUT, sg, aggregator="mean"),
                      kd.ShardedSAGEConv(F_OUT, sg, aggregator="mean", normalize=True),
                      kd.ShardedSAGEConv(F_OUT, sg, aggregator="sum")):
            xl = torch.from_numpy(x[lo:hi]).clone()
            layer._ensure_built(xl)
            xg = xl.clone().requires_grad_(True)
            y = layer(xg)
            (y * r).sum().backward()
            weights = [p.detach().numpy().copy() for p in layer.conv.weights]
            grads = [p.grad.numpy().copy() for p in layer.conv.weights]
            out.append((y.detach().numpy(), xg.grad.numpy(), weights, grads))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_sharded_gin_sage_backward():
    """Sharded GINConv (sum with trainable eps; mean) and SAGEConv (mean + L2
    norm; sum) training steps at world 2 against torch autograd through the
    oracle's whole-graph forwards (gin_conv.py:216-225, sage_conv.py:404-439):
    output and dX within 1e-5 of max(1, |ref|); every weight gradient (eps
    included) all-reduced -- the same on both ranks -- and within sqrt(N) * 1e-5
    of the reference's (sums over all rows)."""
    if torch.cuda.is_initialized():
        pytest.skip("never start processes from a process that has initialised the GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_gin_sage_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s, d, x, _, _ = _graph()
    EI = torch.from_numpy(np.stack([s, d]))
    rr = torch.from_numpy(np.random.default_rng(5).standard_normal((N, F_OUT)).astype(np.float32))

    def close(got, ref, tol):
        err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= tol, err.max()

    for i in range(4):
        y0, _, w0, g0 = res[0][i]
        for r in range(1, world):
            for a, b in zip(w0, res[r][i][2]):  # broadcast weights
                np.testing.assert_array_equal(a, b)
            for a, b in zip(g0, res[r][i][3]):  # all-reduced gradients
                np.testing.assert_array_equal(a, b)
        X = torch.from_numpy(x).clone().requires_grad_(True)
        w = [torch.from_numpy(a).clone().requires_grad_(True) for a in w0]
        src, dst = EI[0].long(), EI[1].long()
        reduce = "sum" if i in (0, 3) else "mean"
        # the oracle forwards of gin_conv.py:216-225 / sage_conv.py:351-439 written out so the
        # aggregate's gradient (dagg) is visible: dX's error bound needs A^T |dagg|
        agg = R.aggregate(reduce, K.take(X, src, axis=0), dst, N)
        agg.retain_grad()
        if i == 0:  # weights: eps, hidden kernel, bias, output kernel, bias
            h = (1 + w[0]) * X + agg
            ref = K.dense(K.dense(h, w[1], w[2], "relu"), w[3], w[4], None)
        elif i == 1:
            ref = K.dense(1.0 * X + agg, w[0], w[1], None)
        else:  # SAGE weights: bias, lin_neigh, lin_self
            out = K.add(K.add(K.dense(X, w[2]), K.dense(agg, w[1])), w[0])
            out = torch.relu(out)
            ref = K.normalize_l2(out) if i == 2 else out
        (ref * rr).sum().backward()
        cnt = np.maximum(np.bincount(d, minlength=N).astype(np.float64), 1.0) if reduce == "mean" else np.ones(N)
        mag = np.zeros((N, F_IN))
        np.add.at(mag, s, (np.abs(agg.grad.numpy()).astype(np.float64) / cnt[:, None])[d])
        close(np.concatenate([res[r][i][0] for r in range(world)]), ref.detach().numpy(), 1e-5)
        got = np.concatenate([res[r][i][1] for r in range(world)])
        # dX: re-associated sums over each source's out-edges, bounded by the sum of |terms|
        err = np.abs(got - X.grad.numpy()) / np.maximum(1.0, np.abs(X.grad.numpy()) + mag)
        assert err.max() <= 1e-5, (i, err.max())
        for got, wt in zip(g0, w):
            close(got, wt.grad.numpy(), 1e-5 * np.sqrt(N))
