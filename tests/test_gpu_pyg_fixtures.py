"""The HIP layers on the reference tests' own numerical-comparison fixtures
against the ground truth those tests use -- PyTorch Geometric's layers,
restated in float64 (oracle/pyg_restated.py) -- at those tests' tolerances:
GCNConv vs PyG (tests/test_gcn_conv.py:556-631: rtol 1e-4, atol 1e-5),
GATv2Conv vs PyG (tests/test_gatv2_conv.py:384-490: rtol = atol = 1e-6),
GINConv vs PyG (tests/test_gin_conv.py:590-650: rtol = atol = 1e-4).
The fixtures' edge lists are the reference tests' (data); features and weights
are seeded here (the reference draws them from Keras initialisers)."""

import numpy as np
import pytest
import torch

from keras_geometric_amd import GATv2Conv, GCNConv, GINConv
from oracle import pyg_restated as P

pytestmark = pytest.mark.gpu

GCN_EDGES = np.array([[0, 1, 2, 3, 4, 1], [1, 2, 3, 4, 5, 0]], np.int64)  # test_gcn_conv.py:94-96
GAT_EDGES = np.array([[0, 1, 1, 2, 3, 4, 4, 5, 0, 3, 5, 1],
                      [1, 0, 2, 1, 4, 3, 5, 4, 2, 5, 0, 0]], np.int64)  # test_gatv2_conv.py:94-100


def _run(layer, x, ei, weights, dev):
    xd, eid = torch.from_numpy(x).to(dev), torch.from_numpy(ei).to(dev)
    layer([xd, eid])
    layer.set_weights(weights)
    with torch.no_grad():
        return layer([xd, eid]).detach().cpu().numpy()


@pytest.mark.parametrize("use_bias,add_loops", [(True, True), (False, True), (True, False)])
def test_gcn_fixture_vs_pyg(dev, use_bias, add_loops):
    rng = np.random.RandomState(42)
    x = rng.randn(6, 10).astype(np.float32)
    W = (rng.randn(10, 12) * 0.3).astype(np.float32)
    b = rng.randn(12).astype(np.float32)
    layer = GCNConv(12, use_bias=use_bias, add_self_loops=add_loops)
    got = _run(layer, x, GCN_EDGES, [W, b] if use_bias else [W], dev)
    ref = P.gcn_forward(x, GCN_EDGES, W, b if use_bias else None, add_self_loops=add_loops)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("heads,concat", [(1, True), (3, True), (3, False), (4, True)])
def test_gatv2_fixture_vs_pyg(dev, heads, concat):
    rng = np.random.RandomState(44)
    x = rng.randn(6, 10).astype(np.float32)
    C = 16 if heads == 4 else 12
    W = (rng.randn(10, heads * C) * 0.3).astype(np.float32)
    att = (rng.randn(1, heads, C) * 0.3).astype(np.float32)
    b = rng.randn(heads * C if concat else C).astype(np.float32)
    layer = GATv2Conv(output_dim=C, heads=heads, concat=concat, negative_slope=0.2)
    got = _run(layer, x, GAT_EDGES, [att, b, W], dev)
    ref = P.gatv2_forward(x, GAT_EDGES, W, att, b, heads=heads, concat=concat, negative_slope=0.2)
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("aggr", ["sum", "mean", "max"])
def test_gin_fixture_vs_pyg(dev, aggr):
    rng = np.random.RandomState(45)
    x = rng.randn(6, 10).astype(np.float32)
    W = (rng.randn(10, 12) * 0.3).astype(np.float32)
    b = rng.randn(12).astype(np.float32)
    layer = GINConv(12, aggregator=aggr)
    got = _run(layer, x, GAT_EDGES, [W, b], dev)
    ref = P.gin_forward(x, GAT_EDGES, W, b, eps=0.0, aggr={"sum": "add"}.get(aggr, aggr))
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)
