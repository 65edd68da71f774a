"""Pins the oracle's GCN normalisation and GATv2 softmax legs (and GIN) against
the algorithm the reference's own tests take as ground truth: PyTorch
Geometric's layers (restated in oracle/pyg_restated.py; torch_geometric is not
installed here), at the tolerances those tests use --
GCNConv vs PyG: tests/test_gcn_conv.py:556-631 (normalize=True; rtol 1e-4, atol 1e-5);
GATv2Conv vs PyG: tests/test_gatv2_conv.py:384-490 (rtol = atol = 1e-6);
GINConv vs PyG: tests/test_gin_conv.py:590-650 (rtol = atol = 1e-4).
Inputs: the reference fixtures' edge lists (test_gcn_conv.py:94-96,
test_gatv2_conv.py:94-100, test_gin_conv.py:94-100) with seeded features, and
a larger random graph without self loops (where the reference's
add_self_loops and PyG's add_remaining_self_loops coincide)."""

import numpy as np
import pytest
import torch

from oracle import pyg_restated as P
from oracle import reference as R

GCN_EDGES = np.array([[0, 1, 2, 3, 4, 1], [1, 2, 3, 4, 5, 0]], np.int64)
GAT_EDGES = np.array([[0, 1, 1, 2, 3, 4, 4, 5, 0, 3, 5, 1], [1, 0, 2, 1, 4, 3, 5, 4, 2, 5, 0, 0]], np.int64)


def _random_graph(seed, n=300, e=3000):
    rng = np.random.default_rng(seed)
    s, d = rng.integers(0, n, e), rng.integers(0, n, e)
    keep = s != d
    return np.stack([s[keep], d[keep]]), n


def _close(got, ref, rtol, atol):
    np.testing.assert_allclose(np.asarray(got, np.float64), ref, rtol=rtol, atol=atol)


@pytest.mark.parametrize("graph", ["fixture", "random"])
@pytest.mark.parametrize("use_bias,add_loops", [(True, True), (False, True), (True, False)])
def test_gcn_matches_pyg(graph, use_bias, add_loops):
    if graph == "fixture":
        ei, n = GCN_EDGES, 6
    else:
        ei, n = _random_graph(1)
        if not add_loops:  # every node needs an in-edge (the reference's deg = 0 gives dinv = 1e6, PyG's 0)
            ei = np.concatenate([ei, np.stack([np.roll(np.arange(n), 1), np.arange(n)])], axis=1)
    rng = np.random.RandomState(42)
    x = rng.randn(n, 10).astype(np.float32)
    W = (rng.randn(10, 12) * 0.3).astype(np.float32)
    b = rng.randn(12).astype(np.float32) if use_bias else None
    got = R.gcn_forward(torch.from_numpy(x), torch.from_numpy(ei), torch.from_numpy(W),
                        torch.from_numpy(b) if b is not None else None, add_self_loops_=add_loops).numpy()
    ref = P.gcn_forward(x, ei, W, b, add_self_loops=add_loops)
    _close(got, ref, 1e-4, 1e-5)


@pytest.mark.parametrize("graph", ["fixture", "random"])
@pytest.mark.parametrize("heads,concat", [(1, True), (3, True), (3, False), (4, True)])
def test_gatv2_matches_pyg(graph, heads, concat):
    ei, n = (GAT_EDGES, 6) if graph == "fixture" else _random_graph(2)
    rng = np.random.RandomState(44)
    x = rng.randn(n, 10).astype(np.float32)
    C = 16 if heads == 4 else 12
    W = (rng.randn(10, heads * C) * 0.3).astype(np.float32)
    att = (rng.randn(1, heads, C) * 0.3).astype(np.float32)
    b = rng.randn(heads * C if concat else C).astype(np.float32)
    got = R.gatv2_forward(torch.from_numpy(x), torch.from_numpy(ei), torch.from_numpy(W), torch.from_numpy(att),
                          torch.from_numpy(b), heads=heads, concat=concat, negative_slope=0.2).numpy()
    ref = P.gatv2_forward(x, ei, W, att, b, heads=heads, concat=concat, negative_slope=0.2)
    _close(got, ref, 1e-6, 1e-6)


@pytest.mark.parametrize("aggr", ["sum", "mean", "max"])
@pytest.mark.parametrize("eps", [0.0, 0.5])
def test_gin_matches_pyg(aggr, eps):
    for ei, n in ((GAT_EDGES, 6), _random_graph(3)):
        rng = np.random.RandomState(45)
        x = rng.randn(n, 10).astype(np.float32)
        W = (rng.randn(10, 12) * 0.3).astype(np.float32)
        b = rng.randn(12).astype(np.float32)
        got = R.gin_forward(torch.from_numpy(x), torch.from_numpy(ei), [(torch.from_numpy(W), torch.from_numpy(b), None)],
                            aggregator=aggr, eps=eps).numpy()
        ref = P.gin_forward(x, ei, W, b, eps=eps, aggr={"sum": "add"}.get(aggr, aggr))
        _close(got, ref, 1e-4, 1e-4)
