"""kgx_spmm_gemm below 128 columns and SAGEConv's fused update (GPU).

F_in < 128 (a multiple of 4): the lanes past F_in re-load column 0 and put
zeros in the bf16x3 planes, W's rows past F_in load as zero; F_out not a
multiple of 16: the stores stop at F_out.  SAGEConv at inference (root_weight,
mean / sum / max; opt-in, KGX_FUSED_SAGE=1) runs out = b + x W_self (kgx_dense) and then the fused
aggregation adds REDUCE(x) W_neigh into out in its store (relu there too) --
sage_conv.py:404-433 with the [N, F_in] aggregate never written.  Checked
against the oracle within the fp32 dot-product bound, on graphs whose rows
cover every fused kernel: hub chunks (fix-up), long rows, the degree <= 7
suffix and the degree <= 2 records.
"""

import numpy as np
import pytest
import torch

import keras_geometric_amd as kgx
from keras_geometric_amd import graph as G
from keras_geometric_amd import ops as kops
from oracle import reference as R
from oracle.rmat import rmat_edges, scale_for

pytestmark = pytest.mark.gpu
T = torch.from_numpy


def _graph(seed, N, E):
    return rmat_edges(seed, scale_for(N), N, 0, E)


def assert_dot_bound(got, ref, scale, k_eps=8e-6):
    """|got - ref| <= k_eps * scale + 1e-6, scale = the same sum over |terms|."""
    err = np.abs(got.astype(np.float64) - ref)
    bound = k_eps * scale + 1e-6
    assert (err <= bound).all(), f"max err/bound {(err / bound).max():.2f}"


@pytest.mark.parametrize("F_in,F_out", [(100, 100), (36, 52), (128, 100), (100, 128)])
@pytest.mark.parametrize("split_len", [0, 16])
def test_fused_narrow_accumulate(dev, F_in, F_out, split_len):
    """out = relu?(H + REDUCE(x) W) in place, H's spare columns untouched."""
    N = 3000
    s, d = _graph(11, N, 40000)
    rng = np.random.default_rng(F_in * 7 + F_out + split_len)
    x = rng.standard_normal((N, F_in)).astype(np.float32)
    W = (rng.standard_normal((F_in, F_out)) * 0.1).astype(np.float32)
    H = rng.standard_normal((N, F_out)).astype(np.float32)
    ei = T(np.stack([s, d]))
    csr = G.build_csr(ei[0].to(dev), ei[1].to(dev), N, N, n_features=F_in, split_len=split_len)
    if split_len:
        assert csr.n_split > 0  # hub rows go through the fix-up kernel
    xd, Wd = T(x).to(dev), T(W).to(dev)
    W64 = W.astype(np.float64)
    for red in ("mean", "sum", "max"):
        for relu in (False, True):
            buf = torch.full((N, F_out + 4), 7.0, device=dev)  # 4 spare columns past F_out
            out = buf[:, :F_out]
            out.copy_(T(H).to(dev))
            kops.aggregate_transform(csr, xd, Wd, red, out=out, relu=relu)
            aggr = R.aggregate(red, T(x)[ei[0].long()], ei[1].long(), N).numpy().astype(np.float64)
            ref = H.astype(np.float64) + aggr @ W64
            scale = np.abs(H) + np.abs(aggr) @ np.abs(W64)
            got = buf.cpu().numpy()
            assert (got[:, F_out:] == 7.0).all(), "store past F_out"
            assert_dot_bound(got[:, :F_out], np.maximum(ref, 0.0) if relu else ref, scale,
                             k_eps=3e-5 if split_len and red != "max" else 8e-6)


@pytest.mark.parametrize("F_in,F_out", [(100, 100), (64, 100)])
def test_fused_narrow_overwrite(dev, F_in, F_out):
    """The overwrite form (bias + REDUCE(x) W, GCN-style weights) at F_in < 128."""
    N = 2500
    s, d = _graph(12, N, 30000)
    rng = np.random.default_rng(F_in + F_out)
    x = rng.standard_normal((N, F_in)).astype(np.float32)
    W = (rng.standard_normal((F_in, F_out)) * 0.1).astype(np.float32)
    b = rng.standard_normal(F_out).astype(np.float32)
    ei = T(np.stack([s, d]))
    csr = G.build_csr(ei[0].to(dev), ei[1].to(dev), N, N, self_loops=True, gcn_norm=True, n_features=F_in,
                      split_len=16)
    got = kops.aggregate_transform(csr, T(x).to(dev), T(W).to(dev), "sum", weighted=True, bias=T(b).to(dev))
    rows = np.repeat(np.arange(N), csr.deg.cpu().numpy())
    wv = csr.w.cpu().numpy().astype(np.float64)
    aggr = np.zeros((N, F_in))
    np.add.at(aggr, rows, x[csr.col.cpu().numpy()].astype(np.float64) * wv[:, None])
    aabs = np.zeros((N, F_in))
    np.add.at(aabs, rows, np.abs(x[csr.col.cpu().numpy()]).astype(np.float64) * np.abs(wv)[:, None])
    W64 = W.astype(np.float64)
    assert_dot_bound(got.cpu().numpy(), aggr @ W64 + b, aabs @ np.abs(W64) + np.abs(b), k_eps=3e-5)


@pytest.mark.parametrize("aggr", ["mean", "sum", "max"])
@pytest.mark.parametrize("F_in,F_out", [(100, 100), (48, 24)])
def test_sage_layer_fused_vs_oracle(dev, monkeypatch, aggr, F_in, F_out):
    """SAGEConv inference takes the fused update (no kops.aggregate call) and
    matches the oracle's sage_forward (sage_conv.py:404-439) within 1e-5 of the
    same forward on |x|, |W|, |b| (KGX_FUSED_SAGE=1); KGX_FUSED_SAGE=0 gives the
    two-step path."""
    monkeypatch.setenv("KGX_FUSED_SAGE", "1")
    N = 4000
    s, d = _graph(13, N, 50000)
    rng = np.random.default_rng(3)
    x = rng.standard_normal((N, F_in)).astype(np.float32)
    ei = T(np.stack([s, d]).astype(np.int64))
    layer = kgx.SAGEConv(F_out, aggregator=aggr)
    xd, eid = T(x).to(dev), ei.to(dev)
    with torch.no_grad():
        layer([xd, eid])
        layer.bias.copy_(torch.randn(F_out, generator=torch.Generator().manual_seed(4)).to(dev))
        calls = []
        real = kops.aggregate
        monkeypatch.setattr(kops, "aggregate", lambda *a, **k: calls.append(1) or real(*a, **k))
        y = layer([xd, eid]).cpu().numpy()
        assert not calls, "the fused SAGE path should not materialise the aggregate"
        monkeypatch.setenv("KGX_FUSED_SAGE", "0")
        y2 = layer([xd, eid]).cpu().numpy()
        assert calls
    wn, ws, b = (t.detach().cpu() for t in (layer.lin_neigh.kernel, layer.lin_self.kernel, layer.bias))
    ref = R.sage_forward(T(x), ei, wn, ws, b, aggregator=aggr).numpy().astype(np.float64)
    scale = R.sage_forward(T(np.abs(x)), ei, wn.abs(), ws.abs(), b.abs(), aggregator=aggr,
                           activation=None).numpy().astype(np.float64)
    for got in (y, y2):
        err = np.abs(got.astype(np.float64) - ref) / np.maximum(scale, 1e-30)
        assert err.max() <= 1e-5, err.max()


def test_sage_layer_fused_degree_zero_rows(dev, monkeypatch):
    """Rows with no in-edges: the aggregate is 0, so out = relu(b + x W_self)."""
    monkeypatch.setenv("KGX_FUSED_SAGE", "1")
    N, F = 10, 100
    s = np.array([1, 2, 3], np.int64)
    d = np.array([0, 0, 9], np.int64)
    x = torch.randn(N, F, generator=torch.Generator().manual_seed(5))
    ei = torch.from_numpy(np.stack([s, d]))
    layer = kgx.SAGEConv(F, aggregator="mean")
    with torch.no_grad():
        layer([x.to(dev), ei.to(dev)])
        layer.bias.copy_(torch.randn(F, generator=torch.Generator().manual_seed(6)).to(dev))
        y = layer([x.to(dev), ei.to(dev)]).cpu()
    wn, ws, b = (t.detach().cpu() for t in (layer.lin_neigh.kernel, layer.lin_self.kernel, layer.bias))
    ref = R.sage_forward(x, ei, wn, ws, b, aggregator="mean")
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)
