"""Backward of the propagate path against the oracle.

The oracle forwards are ATen CPU restatements of the Keras-torch lowering, so
torch autograd through them IS the reference's gradient (segment_sum ->
scatter_add backward = gather; take -> index_select backward = index_add;
segment_max -> scatter_reduce amax backward: ties share evenly; the isinf
guard's where() passes nothing for +-inf rows).  The kgx side: sum / mean /
weighted sums through kgx_spmm over the transposed graph, max / min through
kgx_spmm_max_backward, the fused GCN transform through recompute + GEMMs.
Float gradients are tolerance-checked (north-star 1e-5, relative to
max(1, |ref|)); the scatter order of the backward is not the CPU's.
"""

import numpy as np
import pytest
import torch

from keras_geometric_amd import graph as G
from keras_geometric_amd import ops as kops
from keras_geometric_amd.layers import GCNConv, GINConv, SAGEConv
from oracle import reference as R
from oracle.rmat import rmat_edges, scale_for

pytestmark = pytest.mark.gpu

T = torch.from_numpy


def assert_tol(a, b, tol=1e-5):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    b = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else b
    assert a.shape == b.shape
    err = np.abs(a.astype(np.float64) - b) / np.maximum(1.0, np.abs(b.astype(np.float64)))
    assert err.max() <= tol, f"max rel err {err.max():.3g}"


def assert_tol_scaled(a, b, scale, tol=1e-5):
    """|a-b| <= tol * max(1, scale): scale = the same sum over |terms| (the error
    bound of a re-associated fp32 sum; used where split hub rows change the order)."""
    a, b, scale = (t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else t for t in (a, b, scale))
    err = np.abs(a.astype(np.float64) - b) / np.maximum(1.0, np.abs(scale.astype(np.float64)))
    assert err.max() <= tol, f"max rel err {err.max():.3g}"


def _graph(N=1500, E=16000, seed=4):
    s, d = rmat_edges(seed, scale_for(N), N, 0, E)
    return np.stack([s, d]).astype(np.int32)


def _x(N, F, seed, ties=False):
    rng = np.random.default_rng(seed)
    if ties:  # few distinct values: max/min ties across different sources
        return rng.integers(-3, 4, (N, F)).astype(np.float32)
    return rng.standard_normal((N, F)).astype(np.float32)


@pytest.mark.parametrize("aggr", ["sum", "mean", "max", "min"])
@pytest.mark.parametrize("ties", [False, True])
@pytest.mark.parametrize("split_len", [0, 64])
def test_aggregate_backward(dev, aggr, ties, split_len):
    N, F = 1500, 24
    ei = _graph(N)
    x = _x(N, F, 1, ties)
    gout = _x(N, F, 2)
    g = G.build_csr(T(ei[0]).to(dev), T(ei[1]).to(dev), N, N, split_len=split_len)
    xd = T(x).to(dev).requires_grad_(True)
    y = kops.aggregate(g, xd, aggr, exact=split_len == 0)
    y.backward(T(gout).to(dev))
    xr = T(x).requires_grad_(True)
    yr = R.propagate(xr, T(ei), aggr)
    yr.backward(T(gout))
    assert_tol(y, yr)
    if split_len == 0:
        assert_tol(xd.grad, xr.grad)
    else:  # hub sources' gradients are summed in split chunks
        xa = T(x).requires_grad_(True)
        R.propagate(xa, T(ei), aggr).backward(T(np.abs(gout)))
        assert_tol_scaled(xd.grad, xr.grad, xa.grad)


@pytest.mark.parametrize("aggr", ["sum", "mean", "max"])
def test_aggregate_backward_by_edge_messages(dev, aggr):
    """Aggregator.aggregate(messages, target_idx, dim_size): gradient per message."""
    N, F, E = 800, 16, 9000
    ei = _graph(N, E, seed=7)
    tgt = ei[1].copy()
    tgt[::97] = -3  # negative targets are dropped (segment semantics): zero gradient
    msg = _x(E, F, 3, ties=aggr == "max")
    gout = _x(N, F, 4)
    g = G.build_csr(T(ei[0]).to(dev), T(tgt).to(dev), N, N, segment_only=True)
    md = T(msg).to(dev).requires_grad_(True)
    kops.aggregate(g, md, aggr, by_edge=True, exact=True).backward(T(gout).to(dev))
    mr = T(msg).requires_grad_(True)
    R.aggregate(aggr, mr, T(tgt), N).backward(T(gout))
    assert_tol(md.grad, mr.grad)


def test_weighted_sum_and_epilogue_backward(dev):
    """GCN-weighted sum with bias epilogue, and the GIN epilogue scale*xroot + aggr."""
    N, F = 1200, 32
    ei = _graph(N, 14000, seed=9)
    x, gout = _x(N, F, 5), _x(N, F, 6)
    b = _x(1, F, 7)[0]
    g = G.build_csr(T(ei[0]).to(dev), T(ei[1]).to(dev), N, N, self_loops=True, gcn_norm=True, split_len=32)
    xd, bd = T(x).to(dev).requires_grad_(True), T(b).to(dev).requires_grad_(True)
    kops.aggregate(g, xd, "sum", weighted=True, epilogue=1, bias=bd).backward(T(gout).to(dev))
    xr, br = T(x).requires_grad_(True), T(b).requires_grad_(True)
    eil = R.add_self_loops(T(ei), N)
    w = R.compute_gcn_normalization(eil, N)
    (R.aggregate("sum", xr[eil[0].long()] * w.unsqueeze(1), eil[1], N) + br).backward(T(gout))
    assert_tol(xd.grad, xr.grad)
    assert_tol(bd.grad, br.grad)
    # GIN epilogue: d/dx of 1.5 x + max_aggr(x) has both paths
    g2 = G.build_csr(T(ei[0]).to(dev), T(ei[1]).to(dev), N, N)
    xd2 = T(x).to(dev).requires_grad_(True)
    kops.aggregate(g2, xd2, "max", epilogue=2, xroot=xd2, gin_scale=1.5).backward(T(gout).to(dev))
    xr2 = T(x).requires_grad_(True)
    (1.5 * xr2 + R.propagate(xr2, T(ei), "max")).backward(T(gout))
    assert_tol(xd2.grad, xr2.grad)


def _layer_grads(layer, x, ei, gout):
    y = layer([x, ei])
    y.backward(gout)
    return y, x.grad, [w.grad for w in layer.weights]


@pytest.mark.parametrize("exact", [False, True])
def test_gcn_layer_backward(dev, exact):
    """Fused aggregate->transform (default) and GEMM+aggregate (exact) layers:
    d/dx, d/dW, d/db vs autograd through the reference forward."""
    N, Fi, Fo = 1500, 128, 64
    ei = _graph(N, 18000, seed=11)
    x, gout = _x(N, Fi, 12), _x(N, Fo, 13)
    torch.manual_seed(0)  # weight init independent of the tests that ran before
    layer = GCNConv(Fo, exact=exact)
    xd = T(x).to(dev).requires_grad_(True)
    layer([xd, T(ei).to(dev)])
    rng = np.random.default_rng(14)
    W = (rng.standard_normal((Fi, Fo)) * 0.1).astype(np.float32)
    b = rng.standard_normal(Fo).astype(np.float32)
    layer.set_weights([W, b])
    y, gx, (gW, gb) = _layer_grads(layer, xd, T(ei).to(dev), T(gout).to(dev))
    xr, Wr, br = T(x).requires_grad_(True), T(W).requires_grad_(True), T(b).requires_grad_(True)
    yr = R.gcn_forward(xr, T(ei), Wr, br)
    yr.backward(T(gout))
    assert_tol(y, yr)
    assert_tol(gx, xr.grad)
    # dW sums over all N rows: relative to the magnitude of the sum's terms
    assert_tol(gW, Wr.grad, tol=2e-5 * max(1.0, float(np.sqrt(N))))
    assert_tol(gb, br.grad, tol=1e-5 * max(1.0, float(np.sqrt(N))))


@pytest.mark.parametrize("aggr", ["sum", "mean", "max"])
@pytest.mark.parametrize("train_eps", [False, True])
def test_gin_layer_backward(dev, aggr, train_eps):
    N, F = 1000, 16
    ei = _graph(N, 9000, seed=15)
    x, gout = _x(N, F, 16, ties=aggr == "max"), _x(N, 12, 17)
    torch.manual_seed(0)  # weight init independent of the tests that ran before
    layer = GINConv(output_dim=12, mlp_hidden=[20], aggregator=aggr, eps_init=0.25, train_eps=train_eps, exact=True)
    xd = T(x).to(dev).requires_grad_(True)
    layer([xd, T(ei).to(dev)])
    ws = [w.detach().cpu() for w in layer.weights]
    y, gx, grads = _layer_grads(layer, xd, T(ei).to(dev), T(gout).to(dev))
    xr = T(x).requires_grad_(True)
    wr = [w.clone().requires_grad_(True) for w in ws]
    if train_eps:
        eps_t, W1, b1, W2, b2 = wr
        yr = R.gin_forward(xr, T(ei), [(W1, b1, "relu"), (W2, b2, None)], aggr, eps_tensor=eps_t)
    else:
        W1, b1, W2, b2 = wr
        yr = R.gin_forward(xr, T(ei), [(W1, b1, "relu"), (W2, b2, None)], aggr, eps=0.25)
    yr.backward(T(gout))
    assert_tol(y, yr)
    assert_tol(gx, xr.grad)
    for a, b in zip(grads, wr):
        assert_tol(a, b.grad, tol=1e-5 * np.sqrt(N))


@pytest.mark.parametrize("aggr", ["sum", "mean", "max"])
@pytest.mark.parametrize("hidden", [[], [64]])
def test_gin_fused_layer(dev, aggr, hidden):
    """F_in = 128: (1+eps)x + aggr and the MLP's first Dense (bias, ReLU when
    hidden) run in the fused kernel (bf16x3 MFMA).  Forward and d/dx, d/dW vs
    autograd through the reference forward, within 1e-5 of the same
    computation on |terms| (a bound on every intermediate's magnitude)."""
    N, F, Fo = 1500, 128, 32
    ei = _graph(N, 18000, seed=40)
    x, gout = _x(N, F, 41), _x(N, Fo, 42)
    torch.manual_seed(0)  # weight init independent of the tests that ran before
    layer = GINConv(output_dim=Fo, mlp_hidden=hidden, aggregator=aggr, eps_init=0.25)
    xd = T(x).to(dev).requires_grad_(True)
    layer([xd, T(ei).to(dev)])
    ws = [w.detach().cpu() for w in layer.weights]
    with torch.no_grad():  # inference path: ReLU in the kernel's store
        y0 = layer([xd, T(ei).to(dev)])
    y, gx, grads = _layer_grads(layer, xd, T(ei).to(dev), T(gout).to(dev))
    acts = ["relu"] * len(hidden) + [None]

    def ref(xx, wl, agg):
        return R.gin_forward(xx, T(ei), [(wl[2 * i], wl[2 * i + 1], a) for i, a in enumerate(acts)], agg, eps=0.25)

    xr = T(x).requires_grad_(True)
    wr = [w.clone().requires_grad_(True) for w in ws]
    yr = ref(xr, wr, aggr)
    yr.backward(T(gout))
    xa = T(np.abs(x)).requires_grad_(True)
    wa = [w.abs().clone().requires_grad_(True) for w in ws]
    ya = ref(xa, wa, "sum")  # sum of |terms| bounds sum, mean and max alike
    ya.backward(T(np.abs(gout)))
    assert_tol_scaled(y0, yr, ya)
    assert_tol_scaled(y, yr, ya)
    assert_tol_scaled(gx, xr.grad, xa.grad)
    for a, r, m in zip(grads, wr, wa):
        assert_tol_scaled(a, r.grad, m.grad)


@pytest.mark.parametrize("aggr", ["mean", "max", "sum", "min"])
def test_sage_layer_backward(dev, aggr):
    N, F = 1100, 20
    ei = _graph(N, 12000, seed=18)
    x, gout = _x(N, F, 19), _x(N, 12, 20)
    torch.manual_seed(0)  # weight init independent of the tests that ran before
    layer = SAGEConv(output_dim=12, aggregator=aggr, exact=True)
    xd = T(x).to(dev).requires_grad_(True)
    layer([xd, T(ei).to(dev)])
    b, Wn, Ws = [w.detach().cpu() for w in layer.weights]
    y, gx, (gb, gWn, gWs) = _layer_grads(layer, xd, T(ei).to(dev), T(gout).to(dev))
    xr = T(x).requires_grad_(True)
    br, Wnr, Wsr = (t.clone().requires_grad_(True) for t in (b, Wn, Ws))
    yr = R.sage_forward(xr, T(ei), Wnr, Wsr, br, aggr, "relu", False)
    yr.backward(T(gout))
    assert_tol(y, yr)
    assert_tol(gx, xr.grad)
    for a, r in ((gb, br), (gWn, Wnr), (gWs, Wsr)):
        assert_tol(a, r.grad, tol=1e-5 * np.sqrt(N))


def test_transpose_graph(dev):
    """The transposed CSR lists each source's out-edges in input-edge order."""
    N = 700
    ei = _graph(N, 6000, seed=21)
    g = G.build_csr(T(ei[0]).to(dev), T(ei[1]).to(dev), N, N, self_loops=True, gcn_norm=True)
    t = G.transpose(g)
    assert t.kept == g.kept and t.n_dst == N
    src = np.concatenate([ei[0], np.arange(N)])
    dst = np.concatenate([ei[1], np.arange(N)])
    order = np.argsort(src, kind="stable")  # by source, input order within
    np.testing.assert_array_equal(t.eid.cpu().numpy(), order)
    np.testing.assert_array_equal(t.col.cpu().numpy(), dst[order])
    w_by_eid = np.empty(g.kept, np.float32)
    w_by_eid[g.eid.cpu().numpy()] = g.w.cpu().numpy()
    np.testing.assert_array_equal(t.w.cpu().numpy(), w_by_eid[order])
    np.testing.assert_array_equal(t.deg.cpu().numpy(), np.bincount(src, minlength=N))


def assert_tol_nan(a, b, tol=1e-5):
    """NaN in the same places, then the tolerance elsewhere."""
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    b = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else b
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    ok = ~np.isnan(b)
    assert_tol(a[ok], b[ok], tol)


@pytest.mark.parametrize("by_edge", [False, True])
def test_std_backward(dev, by_edge):
    """std aggregation (aggregators.py:182-228) gradient vs oracle autograd,
    including the reference's NaNs: its count <= 1 guard is a where() after a
    sqrt, so rows with one message send 0 * inf = NaN to that message."""
    N, F = 600, 8
    ei = _graph(N, 5000, seed=22)
    gout = _x(N, F, 24)
    if by_edge:
        msg = _x(ei.shape[1], F, 23)
        g = G.build_csr(T(ei[0]).to(dev), T(ei[1]).to(dev), N, N, segment_only=True)
        md = T(msg).to(dev).requires_grad_(True)
        kops.aggregate(g, md, "std", by_edge=True).backward(T(gout).to(dev))
        mr = T(msg).requires_grad_(True)
        R.aggregate("std", mr, T(ei[1]), N).backward(T(gout))
        assert_tol_nan(md.grad, mr.grad, tol=1e-4)  # ill-conditioned where std is small
        assert np.isnan(mr.grad.numpy()).any()  # the fixture exercises the single-message rows
        return
    x = _x(N, F, 23)
    g = G.build_csr(T(ei[0]).to(dev), T(ei[1]).to(dev), N, N)
    xd = T(x).to(dev).requires_grad_(True)
    kops.aggregate(g, xd, "std").backward(T(gout).to(dev))
    xr = T(x).requires_grad_(True)
    R.propagate(xr, T(ei), "std").backward(T(gout))
    assert_tol_nan(xd.grad, xr.grad, tol=1e-4)


@pytest.mark.parametrize("heads,C,concat", [(8, 16, True), (2, 5, True), (4, 8, False)])
def test_gatv2_layer_backward(dev, heads, C, concat):
    """GATv2Conv: d/dx, d/d kernel, d/d att, d/d bias through kgx_gatv2_backward
    vs autograd through the reference forward (segment softmax included)."""
    from keras_geometric_amd.layers import GATv2Conv

    N, Fi = 900, 24
    ei = _graph(N, 8000, seed=24)
    x = _x(N, Fi, 25)
    out_dim = heads * C if concat else C
    gout = _x(N, out_dim, 26)
    torch.manual_seed(0)  # weight init independent of the tests that ran before
    layer = GATv2Conv(C, heads=heads, concat=concat, exact=True)
    xd = T(x).to(dev).requires_grad_(True)
    layer([xd, T(ei).to(dev)])
    with torch.no_grad():  # non-trivial bias
        layer.bias.copy_(T(_x(1, out_dim, 27)[0]))
    kern, att, bias = (t.detach().cpu() for t in (layer.linear_transform.kernel, layer.att, layer.bias))
    y = layer([xd, T(ei).to(dev)])
    y.backward(T(gout).to(dev))
    # fp32 reference on the kernel's own leaky-ReLU branches: the gradient jumps at
    # z = 0, and on some draws one z lies within ~1e-8 of it, where any two fp32
    # evaluations may take different sides (tests/test_gatv2_conditioning.py)
    with torch.no_grad():
        h = layer.linear_transform(T(x).to(dev)).cpu().reshape(N, heads, C)
    loops = torch.arange(N, dtype=torch.int64)
    src, dst = torch.cat([T(ei[0]).long(), loops]), torch.cat([T(ei[1]).long(), loops])
    branch = (h[dst] + h[src]) > 0
    xr = T(x).requires_grad_(True)
    kr, ar, br = (t.clone().requires_grad_(True) for t in (kern, att, bias))
    yr = R.gatv2_forward(xr, T(ei), kr, ar, br, heads=heads, concat=concat, lrelu_positive=branch)
    yr.backward(T(gout))
    assert_tol(y, yr)
    assert_tol(xd.grad, xr.grad)
    assert_tol(layer.att.grad, ar.grad, tol=1e-5 * np.sqrt(N))
    assert_tol(layer.bias.grad, br.grad, tol=1e-5 * np.sqrt(N))
    assert_tol(layer.linear_transform.kernel.grad, kr.grad, tol=1e-5 * np.sqrt(N))


@pytest.mark.parametrize("aggr", ["sum", "max"])
def test_backward_bipartite_wide_noncontiguous(dev, aggr):
    """Bipartite propagate (n_src != n_dst), F > 1024 (column-sliced launches)
    and a non-contiguous feature view, through the transposed-graph / max
    backward paths."""
    from keras_geometric_amd.layers import MessagePassing

    n_dst, n_src, F, E = 300, 700, 1100, 5000
    rng = np.random.default_rng(31)
    ei = np.stack([rng.integers(0, n_src, E), rng.integers(0, n_dst, E)]).astype(np.int32)
    xs = rng.standard_normal((F, n_src)).astype(np.float32)  # stored transposed -> non-contiguous view
    xd_dst = rng.standard_normal((n_dst, F)).astype(np.float32)
    gout = rng.standard_normal((n_dst, F)).astype(np.float32)
    src_t = T(xs).to(dev).requires_grad_(True)
    mp = MessagePassing(aggregator=aggr, exact=True)
    y = mp.propagate((T(xd_dst).to(dev), src_t.t()), T(ei).to(dev))
    y.backward(T(gout).to(dev))
    xr = T(xs).requires_grad_(True)
    yr = R.propagate(None, T(ei), aggr, x_pair=(T(xd_dst), xr.t()))
    yr.backward(T(gout))
    assert_tol(y, yr)
    assert_tol(src_t.grad, xr.grad)


@pytest.mark.parametrize("loops,norm", [(False, True), (True, False), (False, False)])
def test_gcn_backward_flags(dev, loops, norm):
    N, F = 500, 128
    ei = _graph(N, 4000, seed=32)
    x, gout = _x(N, F, 33), _x(N, 64, 34)
    # without the symmetric normalisation (or with the 1e6 dinv of zero-in-degree
    # nodes when loops are off) the sums are large and cancel: bound-based check
    torch.manual_seed(0)  # weight init independent of the tests that ran before
    layer = GCNConv(64, add_self_loops=loops, normalize=norm)
    xd = T(x).to(dev).requires_grad_(True)
    layer([xd, T(ei).to(dev)])
    W, b = (t.detach().cpu() for t in layer.weights)
    y = layer([xd, T(ei).to(dev)])
    y.backward(T(gout).to(dev))
    xr, Wr, br = T(x).requires_grad_(True), W.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = R.gcn_forward(xr, T(ei), Wr, br, loops, norm)
    yr.backward(T(gout))
    # error bound of a re-ordered fp32 sum: relative to the same computation on |terms|
    # (the forward and both gradients are linear in x, W with non-negative norms)
    xa, Wa, ba = (t.abs().clone().requires_grad_(True) for t in (T(x), W, b))
    ya = R.gcn_forward(xa, T(ei), Wa, ba, loops, norm)
    ya.backward(T(np.abs(gout)))
    assert_tol_scaled(y, yr, ya)
    assert_tol_scaled(xd.grad, xr.grad, xa.grad)
    assert_tol_scaled(layer.kernel.grad, Wr.grad, Wa.grad)
