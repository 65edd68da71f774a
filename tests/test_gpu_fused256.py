"""kgx_spmm_gemm_f256 (fused aggregate -> transform for 256-wide rows, GINConv
at BASELINE config C4) vs the oracle through the C-ABI (GPU).

The aggregation half keeps the reference's sequential per-row order
(aggregators.py:56-167), so the rows fed to the transform equal the unfused
kernel's; the transform is the f32-accurate bf16x3 MFMA product, checked
against a float64 matmul within the forward-error bound of an fp32 dot
product over K = 256 terms (gin_conv.py:216-225, gcn_conv.py:233-272).
"""

import numpy as np
import pytest
import torch

import keras_geometric_amd as kgx
from keras_geometric_amd import _native as nat
from keras_geometric_amd import graph as G
from keras_geometric_amd import ops as kops
from oracle import reference as R
from oracle.rmat import rmat_edges, scale_for

pytestmark = pytest.mark.gpu
T = torch.from_numpy
F = 256


def build(ei_np, N, dev, **kw):
    ei = T(np.ascontiguousarray(ei_np)).to(dev)
    return G.build_csr(ei[0].contiguous(), ei[1].contiguous(), N, N, n_features=F, **kw)


def assert_dot_bound(got, a64, W64, b64, k_eps=8e-6):
    """|got - a@W - b| <= k_eps * (|a|@|W| + |b|) + 1e-6 (fp32 dot, K = 256)."""
    ref = a64 @ W64 + b64
    bound = k_eps * (np.abs(a64) @ np.abs(W64) + np.abs(b64)) + 1e-6
    err = np.abs(got.astype(np.float64) - ref)
    assert (err <= bound).all(), f"max err/bound {(err / bound).max():.2f}"


def _graph(seed, N=3000, E=40000):
    s, d = rmat_edges(seed, scale_for(N), N, 0, E)
    return s, d


@pytest.mark.parametrize("F_out", [256, 128, 16])
@pytest.mark.parametrize("split_len", [0, 16])
def test_fused256_reductions(dev, F_out, split_len):
    N = 3000
    s, d = _graph(8, N)
    rng = np.random.default_rng(F_out + split_len)
    x = rng.standard_normal((N, F)).astype(np.float32)
    W = (rng.standard_normal((F, F_out)) * 0.06).astype(np.float32)
    b = rng.standard_normal(F_out).astype(np.float32)
    ei_l = R.add_self_loops(T(np.stack([s, d])), N)
    csr = build(np.stack([s, d]), N, dev, self_loops=True, gcn_norm=True, split_len=split_len)
    if split_len:
        assert csr.n_split > 0  # hub rows go through the fix-up kernel
    xd, Wd, bd = T(x).to(dev), T(W).to(dev), T(b).to(dev)
    W64, b64 = W.astype(np.float64), b.astype(np.float64)
    for red in ("sum", "mean", "max", "min"):
        aggr = R.aggregate(red, T(x)[ei_l[0].long()], ei_l[1], N).numpy().astype(np.float64)
        got = kops.aggregate_transform(csr, xd, Wd, red, bias=bd).cpu().numpy()
        assert_dot_bound(got, aggr, W64, b64, k_eps=8e-6 if red in ("max", "min") or not split_len else 3e-5)
    g = kops.aggregate_transform(csr, xd, Wd, "max", bias=None, pre_gin=True, gin_scale=1.5).cpu().numpy()
    h = (1.5 * T(x) + R.aggregate("max", T(x)[ei_l[0].long()], ei_l[1], N)).numpy().astype(np.float64)
    assert_dot_bound(g, h, W64, np.zeros_like(b64))


def test_fused256_gcn_layer_vs_oracle(dev, monkeypatch):
    """GCNConv 256 -> 256 on the fused path vs the reference order (per-edge
    x_j W, normalised segment sum, bias), north-star tolerance 1e-5."""
    N = 3000
    s, d = _graph(5, N)
    rng = np.random.default_rng(1)
    x = rng.standard_normal((N, F)).astype(np.float32)
    W = (rng.standard_normal((F, F)) / np.sqrt(F)).astype(np.float32)
    b = rng.standard_normal(F).astype(np.float32)
    monkeypatch.setenv("KGX_FUSED256", "1")
    assert kops.fused_transform_supported(F, F)
    layer = kgx.GCNConv(F)
    ei = T(np.stack([s, d]).astype(np.int64)).to(dev)
    layer([T(x).to(dev), ei])
    layer.set_weights([W, b])
    y = layer([T(x).to(dev), ei]).detach().cpu().numpy()
    ref = R.gcn_forward(T(x), T(np.stack([s, d])), T(W), T(b)).numpy()
    err = np.abs(y - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() <= 1e-5, err.max()


def test_fused256_gin_layer_matches_unfused(dev, monkeypatch):
    """GINConv(256) at C4's shape: the fused launch vs the unfused path
    (aggregation with the GIN epilogue, then kgx_dense) on the same weights."""
    N = 5000
    s, d = _graph(3, N, 60000)
    ei = T(np.stack([s, d]).astype(np.int64)).to(dev)
    x = torch.randn(N, F, device=dev, generator=torch.Generator(device=dev).manual_seed(2))
    layer = kgx.GINConv(F, aggregator="sum", eps_init=0.25)
    with torch.no_grad():
        monkeypatch.setenv("KGX_FUSED256", "1")
        y = layer([x, ei])
        monkeypatch.setenv("KGX_FUSED256", "0")
        y_ref = layer([x, ei])
        g = next(reversed(G._CACHE.values()))[1]
        h = kops.aggregate(g, x, "sum", epilogue=nat.EPI_GIN, xroot=x, gin_scale=layer._scale())
    dense = layer.mlp.layers[-1]
    a64, W64 = h.double().cpu().numpy(), dense.kernel.detach().double().cpu().numpy()
    b64 = dense.bias.detach().double().cpu().numpy()
    assert_dot_bound(y.cpu().numpy(), a64, W64, b64)
    assert_dot_bound(y_ref.cpu().numpy(), a64, W64, b64)


def test_fused256_accumulate_and_relu(dev):
    """out += (accumulate mode, the sharded layers' second pass) and the ReLU store."""
    N = 2000
    s, d = _graph(4, N, 30000)
    rng = np.random.default_rng(4)
    x = rng.standard_normal((N, F)).astype(np.float32)
    W = (rng.standard_normal((F, F)) * 0.06).astype(np.float32)
    b = rng.standard_normal(F).astype(np.float32)
    csr = build(np.stack([s, d]), N, dev, self_loops=True, gcn_norm=True, split_len=16)
    xd, Wd, bd = T(x).to(dev), T(W).to(dev), T(b).to(dev)
    n_own = N // 3
    g_own, g_oth = G.split_by_source(csr, n_own)
    out = kops.aggregate_transform(g_own, xd, Wd, "sum", weighted=True, bias=bd)
    kops.aggregate_transform(g_oth, xd[n_own:].contiguous(), Wd, "sum", weighted=True, out=out)
    rows = np.repeat(np.arange(N), csr.deg.cpu().numpy())
    aggr = np.zeros((N, F))
    np.add.at(aggr, rows, x[csr.col.cpu().numpy()].astype(np.float64) * csr.w.cpu().numpy()[:, None])
    assert_dot_bound(out.cpu().numpy(), aggr, W.astype(np.float64), b.astype(np.float64), k_eps=3e-5)
    r = kops.aggregate_transform(csr, xd, Wd, "sum", weighted=True, bias=bd, relu=True).cpu().numpy()
    one = kops.aggregate_transform(csr, xd, Wd, "sum", weighted=True, bias=bd).cpu().numpy()
    np.testing.assert_array_equal(r, np.maximum(one, 0.0))


def test_fused256_edge_cases(dev):
    """Empty rows (bias + gin_scale x_i W), a row count that is not a tile
    multiple, inf / NaN aggregates (IEEE products through the lo plane)."""
    N = 37
    s = np.array([0, 1, 2, 3, 3, 5, 36, 36, 36], np.int32)
    d = np.array([1, 1, 1, 2, 4, 4, 0, 0, 35], np.int32)
    rng = np.random.default_rng(6)
    x = rng.standard_normal((N, F)).astype(np.float32)
    x[5, 7] = np.inf
    x[3, 9] = np.nan
    W = (rng.standard_normal((F, F)) * 0.06).astype(np.float32)
    b = rng.standard_normal(F).astype(np.float32)
    csr = build(np.stack([s, d]), N, dev)
    xd, Wd, bd = T(x).to(dev), T(W).to(dev), T(b).to(dev)
    got = kops.aggregate_transform(csr, xd, Wd, "sum", bias=bd, pre_gin=True, gin_scale=1.25).cpu().numpy()
    h = (np.float32(1.25) * T(x) + R.aggregate("sum", T(x)[T(s).long()], T(d).long(), N)).numpy().astype(np.float64)
    fin = np.isfinite(h).all(axis=1)
    assert_dot_bound(got[fin], h[fin], W.astype(np.float64), b.astype(np.float64))
    ref = h @ W.astype(np.float64) + b
    bad = ~fin
    np.testing.assert_array_equal(np.isnan(got[bad]), np.isnan(ref[bad]))
    np.testing.assert_array_equal(np.isinf(got[bad]), np.isinf(ref[bad]))


def test_fused256_backward(dev):
    """d/dx, d/dW, d/db of the fused 256 layer (agg rows saved by the forward's
    agg_out store; dx on the transposed graph through the same fused kernel)
    vs float64 autograd of the oracle order."""
    N = 1500
    s, d = _graph(7, N, 20000)
    rng = np.random.default_rng(7)
    x = rng.standard_normal((N, F)).astype(np.float32)
    W = (rng.standard_normal((F, F)) * 0.06).astype(np.float32)
    b = rng.standard_normal(F).astype(np.float32)
    csr = build(np.stack([s, d]), N, dev, self_loops=True, gcn_norm=True, split_len=16)
    xd = T(x).to(dev).requires_grad_(True)
    Wd = T(W).to(dev).requires_grad_(True)
    bd = T(b).to(dev).requires_grad_(True)
    y = kops.aggregate_transform(csr, xd, Wd, "sum", weighted=True, bias=bd)
    go = torch.randn_like(y)
    y.backward(go)
    # float64 reference: A (weighted, CSR) x W + b
    rows = torch.repeat_interleave(torch.arange(N), csr.deg.cpu().long())
    A = torch.zeros(N, N, dtype=torch.float64)
    A.index_put_((rows, csr.col.cpu().long()), csr.w.cpu().double(), accumulate=True)
    x64 = T(x).double().requires_grad_(True)
    W64 = T(W).double().requires_grad_(True)
    b64 = T(b).double().requires_grad_(True)
    (A @ x64 @ W64 + b64).backward(go.cpu().double())
    for got, ref in ((xd.grad, x64.grad), (Wd.grad, W64.grad), (bd.grad, b64.grad)):
        got = got.cpu().double()
        scale = ref.abs().max().clamp_min(1.0)
        assert float((got - ref).abs().max() / scale) <= 2e-5


@pytest.mark.parametrize("red,weighted,gin", [("sum", False, True), ("sum", True, False), ("mean", False, False),
                                              ("max", False, True)])
def test_fused256_tiny_tail_bit_identical(dev, red, weighted, gin):
    """The degree <= 2 tail from the packed records (spmm_gemm256_tiny_kernel)
    gives the same bits as the same rows through the item path: each output
    row depends only on its own aggregated row and W."""
    N = 40000
    s, d = _graph(11, N, 90000)
    rng = np.random.default_rng(11)
    x = T(rng.standard_normal((N, F)).astype(np.float32)).to(dev)
    W = T((rng.standard_normal((F, F)) * 0.06).astype(np.float32)).to(dev)
    b = T(rng.standard_normal(F).astype(np.float32)).to(dev)
    g = build(np.stack([s, d]), N, dev, self_loops=True, gcn_norm=True)
    tpack, tw, n_se, n2 = kops._tiny_of(g, g.items)
    assert tpack is not None and g.n_items - n_se > 20000  # most rows take the record kernel
    w = g.w if weighted else None
    rid = kops._reduce_id(red)
    op = torch.ops.kgx.spmm_gemm
    with torch.no_grad():
        y = op(x, g.rowptr, g.rows, g.items, g.split, g.col, w, g.n_slots, rid, W, b, gin, 1.25, False, -1, tpack, tw,
               n_se, n2)
        y0 = op(x, g.rowptr, g.rows, g.items, g.split, g.col, w, g.n_slots, rid, W, b, gin, 1.25)
        # the saved-aggregate form (training forward: agg_out stores, non-FAST tail)
        ys, agg = torch.ops.kgx.spmm_gemm_save(x, g.rowptr, g.rows, g.items, g.split, g.col, w, g.n_slots, rid, W, b,
                                               gin, 1.25, -1, tpack, tw, n_se, n2)
        want = kops.aggregate(g, x, red, weighted=weighted, epilogue=nat.EPI_GIN if gin else nat.EPI_NONE,
                              xroot=x if gin else None, gin_scale=1.25)
    assert torch.equal(y, y0)
    assert torch.equal(ys, y)
    assert torch.equal(agg, want)
    ei_l = R.add_self_loops(T(np.stack([s, d])), N)
    xs = x.cpu()
    msg = xs[ei_l[0].long()]
    if weighted:
        rows = np.repeat(np.arange(N), g.deg.cpu().numpy())
        aggr = np.zeros((N, F))
        np.add.at(aggr, rows, xs.numpy()[g.col.cpu().numpy()].astype(np.float64) * g.w.cpu().numpy()[:, None])
    else:
        aggr = R.aggregate(red, msg, ei_l[1], N).numpy().astype(np.float64)
    if gin:
        aggr = np.float32(1.25) * xs.numpy().astype(np.float64) + aggr
    assert_dot_bound(y.cpu().numpy(), aggr, W.cpu().double().numpy(), b.cpu().double().numpy(), k_eps=3e-5)


@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("gin", [False, True])
def test_fused256_two_tables_bit_identical(dev, weighted, gin):
    """kgx_spmm_gemm_f256_ex with sources >= n_x1 read from a second table (the
    sharded GIN layer's merged halo pass) equals the one-table launch over the
    concatenated table bit for bit -- main kernel, degree 3..7 launch, tiny tail
    and hub fix-up alike -- in the new-output, overwrite (accumulate=False, rows
    outside a restricted schedule untouched) and accumulate forms."""
    N, H, E = 12000, 5000, 30000
    rng = np.random.default_rng(11 + 2 * weighted + gin)
    s, d = rmat_edges(3 + gin, scale_for(N + H), N + H, 0, E)
    d = d % N  # destinations are this shard's rows; sources own or halo
    ei = T(np.stack([s, d]).astype(np.int32)).to(dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), N + H, N, n_features=F, split_len=16)
    assert g.n_split > 0 and getattr(g, "_kgx_tiny", (None,))[0] is not None  # fix-up and tiny tail both run
    if weighted:
        g.w = T(rng.uniform(0.1, 1.0, g.kept).astype(np.float32)).to(dev)
    x_all = T(rng.standard_normal((N + H, F)).astype(np.float32)).to(dev)
    x_own, x_halo = x_all[:N].contiguous(), x_all[N:].contiguous()
    W = T((rng.standard_normal((F, F)) * 0.06).astype(np.float32)).to(dev)
    b = T(rng.standard_normal(F).astype(np.float32)).to(dev)
    kw = dict(weighted=weighted, bias=b, pre_gin=gin, gin_scale=1.25)
    with torch.no_grad():
        one = kops.aggregate_transform(g, x_all, W, "sum", **kw)
        two = kops.aggregate_transform(g, x_own, W, "sum", x2=x_halo, **kw)
        assert torch.equal(one, two)
        # overwrite the rows of a restricted schedule, leave the rest alone
        mask = torch.zeros(N, dtype=torch.bool, device=dev)
        mask[::3] = True
        gr = G.restrict_rows(g, mask)
        fill = torch.full((N, F), 7.0, device=dev)
        o1, o2 = fill.clone(), fill.clone()
        kops.aggregate_transform(gr, x_all, W, "sum", out=o1, accumulate=False, **kw)
        kops.aggregate_transform(gr, x_own, W, "sum", out=o2, x2=x_halo, accumulate=False, **kw)
        assert torch.equal(o1, o2)
        assert torch.equal(o1[mask], one[mask]) and bool((o1[~mask] == 7.0).all())
        # accumulate (plain sums; the later exchange groups of the sharded pass)
        a1, a2 = one.clone(), one.clone()
        kops.aggregate_transform(g, x_all, W, "sum", out=a1, weighted=weighted)
        kops.aggregate_transform(g, x_own, W, "sum", out=a2, x2=x_halo, weighted=weighted)
        assert torch.equal(a1, a2)


@pytest.mark.parametrize("per32,mid_tail", [("3", "0"), ("8", "0"), ("16", "0"), ("8", "250"), ("8", "1000")])
def test_fused256_cu_split_bit_identical(dev, monkeypatch, per32, mid_tail):
    """KGX_F256_CU_SPLIT: the degree <= 2 tail on a CU-masked stream beside the
    long-row and degree 3..7 launches on the other CUs (forked from and joined
    back into the caller's stream) gives the one-stream bits -- FAST tail (GIN,
    F_out 256), weighted non-FAST tail (F_out 128, accumulate), two tables, hub
    fix-up after the join -- and joins before the caller reads the output;
    KGX_F256_MID_TAIL moves the last of the degree 3..7 rows to the tail's CUs."""
    N, H, E = 30000, 8000, 90000
    rng = np.random.default_rng(23)
    s, d = rmat_edges(5, scale_for(N + H), N + H, 0, E)
    d = d % N
    ei = T(np.stack([s, d]).astype(np.int32)).to(dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), N + H, N, n_features=F, split_len=16)
    assert g.n_split > 0 and getattr(g, "_kgx_tiny", (None,))[0] is not None
    g.w = T(rng.uniform(0.1, 1.0, g.kept).astype(np.float32)).to(dev)
    x_all = T(rng.standard_normal((N + H, F)).astype(np.float32)).to(dev)
    x_own, x_halo = x_all[:N].contiguous(), x_all[N:].contiguous()
    W = T((rng.standard_normal((F, F)) * 0.06).astype(np.float32)).to(dev)
    W128 = W[:, :128].contiguous()
    b = T(rng.standard_normal(F).astype(np.float32)).to(dev)

    def run():
        with torch.no_grad():
            y1 = kops.aggregate_transform(g, x_all, W, "sum", bias=b, pre_gin=True, gin_scale=1.25)
            y2 = kops.aggregate_transform(g, x_own, W, "sum", bias=b, weighted=True, x2=x_halo)
            acc = torch.ones(N, 128, device=dev)
            kops.aggregate_transform(g, x_all, W128, "sum", out=acc, weighted=True)
            return y1, y2, acc

    monkeypatch.setenv("KGX_F256_CU_SPLIT", "0")
    ref = run()
    monkeypatch.setenv("KGX_F256_CU_SPLIT", per32)
    monkeypatch.setenv("KGX_F256_MID_TAIL", mid_tail)
    for _ in range(2):
        got = run()
        for a_, b_ in zip(got, ref):
            assert torch.equal(a_, b_)

