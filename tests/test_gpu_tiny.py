"""The fused aggregate->transform's degree <= 2 tail on packed records
(spmm_gemm_tiny_kernel, kgx_spmm_gemm_ex2) against the same launch with the
tail on the short-row kernel: same edges, same order, same split product, so
the outputs must be bit-identical -- for every reduction, weighted and not,
with the GIN pre-scale, ReLU, the accumulate form and the saved aggregate.
And against the oracle's GCN forward."""

import numpy as np
import pytest
import torch

from keras_geometric_amd import graph as G
from keras_geometric_amd import ops as kops
from keras_geometric_amd import synthetic, tiny

pytestmark = pytest.mark.gpu


def _graph(dev, n=60_000, e=240_000, **kw):
    ei = synthetic.rmat_edge_index(n, e, seed=5, device=dev)
    return G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, **kw), ei


def _no_tiny(g):
    g._kgx_tiny = (None, None, -1, 0)


def _with_tiny(g):
    if hasattr(g, "_kgx_tiny"):
        del g._kgx_tiny
    pack, tw, start, n2 = tiny.tiny_pack(g)
    n = g.n_items - start
    assert pack is not None and n > 4096 and 0 < n2 < n
    deg = tiny.records(pack, tw, n, n2)[0][:, 1].cpu().numpy()
    assert (deg[:n2] == 2).all() and (deg[n2:] <= 1).all()


@pytest.mark.parametrize("red", ["sum", "mean", "max", "min"])
@pytest.mark.parametrize("weighted", [True, False])
def test_tiny_tail_bit_identical(dev, red, weighted):
    """Each launch is first held to the float64 restatement on every row
    (tests/fused_ref.py), so a wrong row is named with its kernel; then the two
    launches must agree bit for bit."""
    import fused_ref

    g, _ = _graph(dev, self_loops=True, gcn_norm=True)
    gen = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(g.rowptr.numel() - 1, 128, device=dev, generator=gen)
    W = torch.randn(128, 128, device=dev, generator=gen) * 0.1
    b = torch.randn(128, device=dev, generator=gen)
    ref = fused_ref.reference(g, x, W, red, weighted, b)
    outs = []
    for on in (False, True):
        _with_tiny(g) if on else _no_tiny(g)
        outs.append(kops.aggregate_transform(g, x, W, red, weighted=weighted, bias=b))
        fused_ref.check(outs[-1], g, ref, f"{red} weighted={weighted} tail on {'records' if on else 'short rows'}")
    torch.testing.assert_close(outs[1], outs[0], rtol=0, atol=0)


def test_tiny_tail_variants_bit_identical(dev):
    g, _ = _graph(dev, self_loops=False, gcn_norm=False)  # degree-0 rows in the tail too
    gen = torch.Generator(device=dev).manual_seed(2)
    n = g.rowptr.numel() - 1
    x = torch.randn(n, 128, device=dev, generator=gen)
    W = torch.randn(128, 64, device=dev, generator=gen) * 0.1
    b = torch.randn(64, device=dev, generator=gen)
    res = {}
    for on in (False, True):
        _with_tiny(g) if on else _no_tiny(g)
        r = {"gin": kops.aggregate_transform(g, x, W, "sum", bias=b, pre_gin=True, gin_scale=1.25),
             "relu": kops.aggregate_transform(g, x, W, "mean", bias=b, relu=True)}
        acc = torch.randn(n, 64, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
        with torch.no_grad():
            kops.aggregate_transform(g, x, W, "sum", bias=b, out=acc)
        r["acc"] = acc
        xg = x.clone().requires_grad_(True)
        Wg = W.clone().requires_grad_(True)
        y = kops.aggregate_transform(g, xg, Wg, "sum", bias=b)  # keeps the aggregate (spmm_gemm_save)
        y.square().sum().backward()
        r["save_y"], r["dW"] = y.detach(), Wg.grad
        res[on] = r
    for k in res[False]:
        torch.testing.assert_close(res[True][k], res[False][k], rtol=0, atol=0, msg=k)


def test_tiny_records_are_read(dev):
    """The fused launch really takes the tail from the records: scaling the
    packed weights (not the graph's) doubles exactly those rows."""
    g, _ = _graph(dev, self_loops=True, gcn_norm=True)
    _with_tiny(g)
    gen = torch.Generator(device=dev).manual_seed(6)
    x = torch.randn(g.rowptr.numel() - 1, 128, device=dev, generator=gen)
    W = torch.randn(128, 128, device=dev, generator=gen) * 0.1
    y0 = kops.aggregate_transform(g, x, W, "sum", weighted=True)
    pack, tw, start, n2 = g._kgx_tiny
    n = g.n_items - start
    rec, _ = tiny.records(pack, tw, n, n2)
    tw2 = tw * 2.0
    g._kgx_tiny = (pack, tw2, start, n2)
    y1 = kops.aggregate_transform(g, x, W, "sum", weighted=True)
    tail_rows = rec[:, 0][rec[:, 1] > 0].long()
    changed = (y1 != y0).any(1)
    assert bool(changed[tail_rows].float().mean() > 0.99)
    mask = torch.ones_like(changed)
    mask[rec[:, 0].long()] = False
    assert not bool(changed[mask].any())
    torch.testing.assert_close(y1[tail_rows], 2 * y0[tail_rows], rtol=1e-5, atol=1e-5)
    g._kgx_tiny = (pack, tw, start, n2)


def test_tiny_tail_gcn_vs_oracle(dev):
    from oracle import reference as R

    g, ei = _graph(dev, n=20_000, e=60_000, self_loops=True, gcn_norm=True)
    _with_tiny(g)
    gen = torch.Generator(device=dev).manual_seed(4)
    x = torch.randn(20_000, 128, device=dev, generator=gen)
    W = torch.randn(128, 128, device=dev, generator=gen) * (1 / 128) ** 0.5
    b = torch.randn(128, device=dev, generator=gen)
    y = kops.aggregate_transform(g, x, W, "sum", weighted=True, bias=b).cpu()
    ref = R.gcn_forward(x.cpu(), ei.cpu(), W.cpu(), b.cpu())
    err = ((y - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
    assert err <= 1e-5, err
    assert np.isfinite(y.numpy()).all()


@pytest.mark.parametrize("fork", ["3"])
def test_fused_fork_bit_identical(dev, fork, monkeypatch):
    """KGX_FUSED_FORK=3 (the CU split the KGX_FUSED_CU_SPLIT flag asks for): the
    short + tiny launches on a CU-masked stream beside the main kernel on
    another give the same bits as the one-stream launches (disjoint rows, same
    kernels), and both are joined: the next op on the stream sees every row."""
    import fused_ref

    g, _ = _graph(dev, self_loops=True, gcn_norm=True)
    _with_tiny(g)
    gen = torch.Generator(device=dev).manual_seed(9)
    x = torch.randn(g.rowptr.numel() - 1, 128, device=dev, generator=gen)
    W = torch.randn(128, 128, device=dev, generator=gen) * 0.1
    b = torch.randn(128, device=dev, generator=gen)
    monkeypatch.setenv("KGX_FUSED_FORK", "0")
    y0 = kops.aggregate_transform(g, x, W, "sum", weighted=True, bias=b)
    monkeypatch.setenv("KGX_FUSED_FORK", fork)
    y1 = kops.aggregate_transform(g, x, W, "sum", weighted=True, bias=b)
    s1 = y1.sum(1)  # consumed right away on the same stream
    torch.testing.assert_close(y1, y0, rtol=0, atol=0)
    torch.testing.assert_close(s1, y0.sum(1), rtol=0, atol=0)
    fused_ref.check(y1, g, fused_ref.reference(g, x, W, "sum", True, b), f"fork {fork}")


@pytest.mark.parametrize("weighted", [True, False])
def test_device_records_equal_host_restatement(weighted, dev):
    """kgx_tiny_pack / kgx_schedule_suffixes (the device build of the tail
    records and suffix starts) == tiny.py's torch restatement on the same
    schedule moved to the host, bit for bit."""
    from types import SimpleNamespace

    from keras_geometric_amd import graph as G
    from keras_geometric_amd import tiny as T

    g, _ = _graph(dev, n=20_000, e=60_000, self_loops=True, gcn_norm=weighted)
    pack, tw, start, n2 = T.tiny_pack(g, refresh=True)
    assert pack is not None and pack.is_cuda
    h = SimpleNamespace(items=g.items.cpu(), n_items=g.n_items, n_long=g.n_long, col=g.col.cpu(),
                        w=g.w.cpu() if g.w is not None else None)
    hp, htw, hstart, hn2 = T.tiny_pack(h)
    assert (start, n2) == (hstart, hn2)
    assert torch.equal(pack.cpu(), hp)
    assert (tw is None) == (htw is None) and (tw is None or torch.equal(tw.cpu(), htw))
    assert G.short_suffix_start(g.items) == G.short_suffix_start(g.items.cpu())
    assert T.tiny_suffix_start(g.items) == T.tiny_suffix_start(g.items.cpu())
