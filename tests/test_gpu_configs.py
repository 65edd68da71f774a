"""Parity at BASELINE.json's config sizes (one MI355X), on the layers' default paths.

C2  GCNConv 1M / 10M, F 128 -> 128: the fused aggregate->transform layer
    (`kgx_spmm_gemm`, split hub rows) against the oracle's op-for-op
    Keras-torch forward of gcn_conv.py:275-364 on the WHOLE graph, and the
    EXACT sum / mean / max aggregation bit-identical to the oracle's
    propagate (message_passing.py:147-220) on the whole graph.
C3  GATv2Conv 1M / 10M, 8 heads x 16: the layer against the oracle's
    gatv2_conv.py:176-352 forward on the whole graph.
C4  GINConv sum 10M / 100M, F 256 (one GPU; the oracle's [E, 256] message
    tensor and int64 ids would not fit host memory in test time), through
    size-independent properties: CSR invariants over every slot; EXACT
    sampled rows (the hubs included) == a sequential host fp32 loop with the
    (1+eps) x_i + aggr epilogue (gin_conv.py:216-222), bit for bit; split vs
    EXACT; a float64 linearity checksum; the MLP Dense (gin_conv.py:129-162)
    against a float64 GEMM of the same MLP input.
C5  SAGEConv mean 2,449,029 / 123,718,280, F 100 (the tail path: 100 is not a
    multiple of the 32-lane float4 groups), with the same properties plus
    mean = fp32 sum / fp32 count on sampled rows, bit for bit
    (aggregators.py:56-85), and the two linear maps + bias + ReLU
    (sage_conv.py:405-439) against float64.

Tolerances: the north-star fp32 bar |a - b| <= 1e-5 max(1, |b|); for a dense
map against float64, the forward-error bound of an fp32 K-term dot product,
4e-6 (|a| |W| + |b|) + 1e-6.
"""

import numpy as np
import pytest
import torch

import keras_geometric_amd as kgx
from keras_geometric_amd import _native as nat
from keras_geometric_amd import graph as G
from keras_geometric_amd import ops as kops
from keras_geometric_amd import synthetic
import oracle_sample as OS
from oracle import reference as R

pytestmark = [pytest.mark.gpu, pytest.mark.slow, pytest.mark.timeout(900)]


def _tol(got, ref, tol=1e-5):
    got = got.detach().cpu() if isinstance(got, torch.Tensor) else torch.from_numpy(got)
    ref = ref.detach().cpu() if isinstance(ref, torch.Tensor) else torch.from_numpy(ref)
    err = ((got - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
    assert err <= tol, err
    return err


def _x(n, f, seed):
    return torch.randn(n, f, generator=torch.Generator().manual_seed(seed))


@pytest.fixture(autouse=True)
def _release():
    yield
    G.clear_cache()
    torch.cuda.empty_cache()


def _csr_invariants(g, ei, n, e, self_loops):
    rowptr, col, eid, deg = g.rowptr.long(), g.col.long(), g.eid.long(), g.deg.long()
    loops = n if self_loops else 0
    assert g.kept == e + loops and int(rowptr[0]) == 0 and int(rowptr[-1]) == e + loops
    assert bool((rowptr[1:] >= rowptr[:-1]).all())
    assert torch.equal(deg, torch.bincount(ei[1].long(), minlength=n) + (1 if self_loops else 0))
    assert bool((torch.bincount(eid, minlength=e + loops) == 1).all())  # a permutation
    row_of = torch.repeat_interleave(torch.arange(n, device=deg.device), deg)
    same_row = row_of[1:] == row_of[:-1]
    assert bool((eid[1:] > eid[:-1])[same_row].all())  # input order kept inside every row
    src = ei[0].long()
    if self_loops:
        src = torch.cat([src, torch.arange(n, device=deg.device)])
    assert torch.equal(col, src[eid])
    assert g.max_degree == int(deg.max())


def _sample_rows(g, n, k=120, seed=0):
    hubs = torch.topk(g.deg.long(), 8).indices.tolist()
    rng = np.random.default_rng(seed)
    return hubs + rng.integers(0, n, k).tolist()


def _seq_sum(msg: np.ndarray) -> np.ndarray:
    """Sequential fp32 accumulation in edge order (np.add.accumulate adds one
    term at a time, unlike np.sum's pairwise tree) -- the order of the
    reference's scatter_add over the CSR row."""
    if msg.shape[0] == 0:
        return np.zeros(msg.shape[1], np.float32)
    return np.add.accumulate(msg.astype(np.float32), axis=0, dtype=np.float32)[-1]


def _reassoc_check(sp, ex, mag):
    """Split (re-associated) vs EXACT (sequential) row sums: both are fp32
    sums of the same terms, so they differ by at most the forward-error bound
    of a sum, which scales with the sum of |terms| (mag), not with the result:
    |sp - ex| <= 1e-5 max(1, mag)."""
    bad = (sp - ex).abs() > 1e-5 * mag.clamp_min(1.0)
    assert not bool(bad.any()), float(((sp - ex).abs() / mag.clamp_min(1.0)).max())


def _linearity_checksum(g, f, device):
    """Every CSR slot contributes exactly once: with integer-valued features
    in [-8, 8] every row sum (|sum| <= 8 x max degree < 2^24) is exact in fp32
    whatever the order, so the default (split-hub) sums' column totals equal
    the float64 sum over all edges bit for bit, and split == EXACT everywhere."""
    xi = torch.randint(-8, 9, (g.n_src, f), device=device, generator=torch.Generator(device=device).manual_seed(11),
                       dtype=torch.int32).float()
    assert 8 * g.max_degree < 1 << 24
    with torch.no_grad():
        sp = kops.aggregate(g, xi, "sum")
        ex = kops.aggregate(g, xi, "sum", exact=True)
    assert torch.equal(sp, ex)
    ref = torch.zeros(f, dtype=torch.float64, device=device)
    for i in range(0, g.kept, 10_000_000):
        ref += xi[g.col[i:i + 10_000_000].long()].double().sum(0)
    assert torch.equal(sp.double().sum(0), ref)


def _dense_bound_check(y, a, W, b, relu=False):
    """y (fp32, GPU) vs float64 relu?(a W + b) on the same rows, within the
    forward-error bound of an fp32 dot product over K terms."""
    a64, W64 = a.double(), W.double()
    ref = a64 @ W64 + (b.double() if b is not None else 0)
    bound = 4e-6 * (a64.abs() @ W64.abs() + (b.double().abs() if b is not None else 0)) + 1e-6
    if relu:
        ref = ref.clamp_min(0)
    assert bool(((y.double() - ref).abs() <= bound).all()), float(((y.double() - ref).abs() / bound).max())


# --------------------------------------------------------------------------- C2
C2 = (1_000_000, 10_000_000, 128)


def test_c2_gcn_layer_vs_oracle_fullgraph(dev):
    n, e, f = C2
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = _x(n, f, 1)
    rng = np.random.default_rng(2)
    W = (rng.standard_normal((f, f)) / np.sqrt(f)).astype(np.float32)
    b = rng.standard_normal(f).astype(np.float32)
    assert kops.fused_transform_supported(f, f)  # the default path under test is the fused kernel
    layer = kgx.GCNConv(f)
    xd = x.to(dev)
    with torch.no_grad():
        layer([xd, ei])
        layer.set_weights([W, b])
        kops.EVENT_SINK = []
        try:
            y = layer([xd, ei]).cpu()
        finally:
            ev, kops.EVENT_SINK = kops.EVENT_SINK, None
    assert len(ev) == 1  # one fused launch
    g = next(reversed(G._CACHE.values()))[1]
    assert g.n_split > 0  # hub rows were split: the default (re-associated) path is the one checked
    ref = R.gcn_forward(x, ei.cpu(), torch.from_numpy(W), torch.from_numpy(b))
    _tol(y, ref)


@pytest.mark.parametrize("aggr", ["sum", "mean", "max"])
def test_c2_exact_aggregation_bitwise_fullgraph(aggr, dev):
    n, e, f = C2
    ei = synthetic.rmat_edge_index(n, e, seed=3, device=dev)
    x = _x(n, f, 4)
    with torch.no_grad():
        got = kgx.MessagePassing(aggregator=aggr, exact=True)([x.to(dev), ei]).cpu()
    ref = R.propagate(x, ei.cpu(), aggr)
    assert torch.equal(got, ref)


# --------------------------------------------------------------------------- C3
def test_c3_gatv2_layer_vs_oracle_fullgraph(dev):
    n, e, H, C, fin = 1_000_000, 10_000_000, 8, 16, 128
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = _x(n, fin, 5)
    layer = kgx.GATv2Conv(C, heads=H)
    xd = x.to(dev)
    with torch.no_grad():
        layer([xd, ei])
        layer.bias.copy_(torch.randn(H * C, generator=torch.Generator().manual_seed(6)).to(dev))
        y = layer([xd, ei]).cpu()
    kern, att, bias = (t.detach().cpu() for t in (layer.linear_transform.kernel, layer.att, layer.bias))
    ref = R.gatv2_forward(x, ei.cpu(), kern, att, bias, heads=H, concat=True, negative_slope=0.2)
    _tol(y, ref)


# --------------------------------------------------------------------------- C4
C4 = (10_000_000, 100_000_000, 256)


@pytest.fixture(scope="module")
def c4(dev):
    n, e, f = C4
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = torch.randn(n, f, device=dev, generator=torch.Generator(device=dev).manual_seed(7))
    yield ei, x
    G.clear_cache()


def test_c4_gin_csr_and_exact_rows(c4):
    ei, x = c4
    n, e, f = C4
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, n_features=f)
    _csr_invariants(g, ei, n, e, self_loops=False)
    scale = float(np.float32(1 + 0.25))  # (1 + eps) with eps = 0.25, an fp32 scalar (gin_conv.py:217-222)
    with torch.no_grad():
        ex = kops.aggregate(g, x, "sum", epilogue=nat.EPI_GIN, xroot=x, gin_scale=scale, exact=True)
        sp = kops.aggregate(g, x, "sum", epilogue=nat.EPI_GIN, xroot=x, gin_scale=scale)
    rowptr = g.rowptr.cpu().numpy()
    for r in _sample_rows(g, n):
        b, en = int(rowptr[r]), int(rowptr[r + 1])
        acc = _seq_sum(x[g.col[b:en].long()].cpu().numpy())
        want = np.float32(scale) * x[r].cpu().numpy() + acc  # fp32 multiply, then fp32 add
        np.testing.assert_array_equal(ex[r].cpu().numpy(), want)
    with torch.no_grad():
        mag = kops.aggregate(g, x.abs(), "sum", epilogue=nat.EPI_GIN, xroot=x.abs(), gin_scale=scale)
    _reassoc_check(sp, ex, mag)
    unsplit = g.deg < g.split_len
    assert bool((sp[unsplit] == ex[unsplit]).all())


def test_c4_gin_linearity_and_mlp(c4):
    ei, x = c4
    n, e, f = C4
    layer = kgx.GINConv(f, aggregator="sum")
    with torch.no_grad():
        y = layer([x, ei])
    g = next(reversed(G._CACHE.values()))[1]
    _linearity_checksum(g, f, x.device)
    with torch.no_grad():  # the layer's own MLP input, from the same deterministic kernel
        h = kops.aggregate(g, x, "sum", epilogue=nat.EPI_GIN, xroot=x, gin_scale=layer._scale())
    dense = layer.mlp.layers[-1]
    rows = torch.tensor(_sample_rows(g, n, k=4000, seed=1), device=x.device)
    _dense_bound_check(y[rows], h[rows], dense.kernel.detach(), dense.bias.detach())


# --------------------------------------------------------------------------- C5
C5 = (2_449_029, 123_718_280, 100)


def test_c5_sage_mean_properties(dev):
    n, e, f = C5
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = torch.randn(n, f, device=dev, generator=torch.Generator(device=dev).manual_seed(8))
    layer = kgx.SAGEConv(f, aggregator="mean")
    with torch.no_grad():
        layer([x, ei])
        layer.bias.copy_(torch.randn(f, generator=torch.Generator().manual_seed(9)).to(dev))
        y = layer([x, ei])
    g = next(reversed(G._CACHE.values()))[1]
    _csr_invariants(g, ei, n, e, self_loops=False)
    with torch.no_grad():
        ex = kops.aggregate(g, x, "mean", exact=True)
        sp = kops.aggregate(g, x, "mean")
        s = kops.aggregate(g, x, "sum", exact=True)
    rowptr = g.rowptr.cpu().numpy()
    for r in _sample_rows(g, n):
        b, en = int(rowptr[r]), int(rowptr[r + 1])
        acc = _seq_sum(x[g.col[b:en].long()].cpu().numpy())
        np.testing.assert_array_equal(s[r].cpu().numpy(), acc)
        cnt = np.maximum(np.float32(min(en - b, 1 << 24)), np.float32(1e-8))  # fp32 count (aggregators.py:56-85)
        np.testing.assert_array_equal(ex[r].cpu().numpy(), acc / cnt)
    with torch.no_grad():
        mag = kops.aggregate(g, x.abs(), "mean")
    _reassoc_check(sp, ex, mag)
    _linearity_checksum(g, f, x.device)
    # the update: relu(x W_self + aggr W_neigh + b) (sage_conv.py:405-439) on the layer's own aggregation
    rows = torch.tensor(_sample_rows(g, n, k=4000, seed=2), device=x.device)
    a = torch.cat([x[rows], sp[rows]], 1)
    Wcat = torch.cat([layer.lin_self.kernel.detach(), layer.lin_neigh.kernel.detach()], 0)
    _dense_bound_check(y[rows], a, Wcat, layer.bias.detach(), relu=True)


# ------------------------------------------------ full-size layers vs the oracle on sampled rows
def _oracle_sampled(got, ref, scale, what):
    err = OS.scaled_err(got, ref, scale)
    print(f"{what}: layer vs oracle on {got.shape[0]} sampled rows, max scaled err {err:.3e}")
    assert err <= 1e-5, err


def test_c4_gin_layer_vs_oracle_sampled(c4):
    """The C4 GIN layer on the fused 256-wide kernels vs the oracle's op-for-op
    forward on ~1500 sampled rows incl. the largest hubs (tests/oracle_sample.py);
    bar: 1e-5 of the same forward on |x|, |W|, |b| (re-associated sums)."""
    ei, x = c4
    n, e, f = C4
    layer = kgx.GINConv(f, aggregator="sum", eps_init=0.25)
    with torch.no_grad():
        layer([x, ei])
        dense = layer.mlp.layers[-1]
        dense.bias.copy_(torch.randn(f, generator=torch.Generator().manual_seed(21)).to(x.device))
        y = layer([x, ei])
    W, b = dense.kernel.detach().cpu(), dense.bias.detach().cpu()
    rows = OS.sample_rows(ei, n)
    ref = OS.gin_rows(ei, x, rows, [(W, b, None)], 0.25)
    scale = OS.gin_rows(ei, x.abs(), rows, [(W.abs(), b.abs(), None)], 0.25)
    _oracle_sampled(y[rows], ref, scale, "C4 GINConv")


def test_c5_sage_layer_vs_oracle_sampled(dev):
    n, e, f = C5
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = torch.randn(n, f, device=dev, generator=torch.Generator(device=dev).manual_seed(8))
    layer = kgx.SAGEConv(f, aggregator="mean")
    with torch.no_grad():
        layer([x, ei])
        layer.bias.copy_(torch.randn(f, generator=torch.Generator().manual_seed(9)).to(dev))
        y = layer([x, ei])
    wn, ws, b = (t.detach().cpu() for t in (layer.lin_neigh.kernel, layer.lin_self.kernel, layer.bias))
    rows = OS.sample_rows(ei, n)
    ref = OS.sage_rows(ei, x, rows, wn, ws, b)
    scale = OS.sage_rows(ei, x.abs(), rows, wn.abs(), ws.abs(), b.abs())
    _oracle_sampled(y[rows], ref, scale, "C5 SAGEConv")
    G.clear_cache()
