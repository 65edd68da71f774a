"""BatchGlobalPooling / GlobalPooling / batch_graphs on the GPU.

BatchGlobalPooling is one kgx_spmm over the batch vector's segment CSR; each
graph's nodes are reduced in node order by one lane -- the order the
reference's segment_sum scatter accumulates in -- so sum, mean and max are
bit-identical to the oracle (max without the aggregators' isinf guard:
empty graphs pool to -inf).  Gradients vs oracle autograd within 1e-5."""

import numpy as np
import pytest
import torch

import keras_geometric_amd as kgx
from keras_geometric_amd.layers import BatchGlobalPooling, GCNConv, GINConv, GlobalPooling
from oracle import reference as R

pytestmark = pytest.mark.gpu
T = torch.from_numpy


def exact(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    b = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else b
    np.testing.assert_array_equal(a, b)


def _batch(seed=0, sizes=(30, 45, 0, 25, 1, 700)):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((sum(sizes), 16)).astype(np.float32)
    batch = np.repeat(np.arange(len(sizes)), sizes).astype(np.int32)
    return x, batch


@pytest.mark.parametrize("pooling", ["mean", "max", "sum"])
def test_batch_global_pooling_bitwise(dev, pooling):
    x, batch = _batch()
    x[5, 3] = np.inf  # +inf survives max pooling (no isinf guard)
    x[100, 0] = -np.inf
    out = BatchGlobalPooling(pooling=pooling)([T(x).to(dev), T(batch).to(dev)])
    exact(out, R.batch_global_pooling(T(x), T(batch), pooling))


def test_batch_global_pooling_unsorted_and_large(dev):
    rng = np.random.default_rng(1)
    n, G = 200_000, 1000
    x = rng.standard_normal((n, 32)).astype(np.float32)
    batch = rng.integers(0, G, n).astype(np.int32)  # unsorted ids: segment order = node order
    for p in ("mean", "max", "sum"):
        exact(BatchGlobalPooling(pooling=p)([T(x).to(dev), T(batch).to(dev)]),
              R.batch_global_pooling(T(x), T(batch), p))


@pytest.mark.parametrize("pooling", ["mean", "max", "sum"])
def test_batch_global_pooling_backward(dev, pooling):
    x, batch = _batch(2)
    if pooling == "max":
        x = np.round(x)  # ties share the gradient
    gout = np.random.default_rng(3).standard_normal((int(batch.max()) + 1, 16)).astype(np.float32)
    xd = T(x).to(dev).requires_grad_(True)
    BatchGlobalPooling(pooling=pooling)([xd, T(batch).to(dev)]).backward(T(gout).to(dev))
    xr = T(x).requires_grad_(True)
    R.batch_global_pooling(xr, T(batch), pooling).backward(T(gout))
    g, r = xd.grad.cpu().numpy(), xr.grad.numpy()
    assert (np.abs(g - r) / np.maximum(1, np.abs(r))).max() <= 1e-5


def test_global_pooling(dev):
    x, _ = _batch(4)
    for p in ("mean", "max", "sum"):
        out = GlobalPooling(pooling=p)(T(x).to(dev)).cpu().numpy()
        ref = R.global_pooling(T(x), p).numpy()
        np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-5)
        assert out.shape == (1, 16)


def test_batch_graphs_and_graph_classification(dev):
    """batch_graphs layout vs the oracle restatement, then a GIN -> sum-pool
    graph readout over the batch equals the per-graph readouts."""
    rng = np.random.default_rng(5)
    graphs, dicts = [], []
    for n in (12, 7, 30, 1):
        x = rng.standard_normal((n, 8)).astype(np.float32)
        e = 3 * n
        ei = rng.integers(0, n, (2, e)).astype(np.int32)
        y = np.array([float(n)], np.float32)
        graphs.append(kgx.GraphData(x=x, edge_index=ei, y=y))
        dicts.append({"x": x, "edge_index": ei, "y": y})
    b = kgx.batch_graphs(graphs)
    ref = R.batch_graphs(dicts)
    exact(b.x, ref["x"])
    exact(b.edge_index, ref["edge_index"])
    exact(b.batch, ref["batch"])
    exact(b.y, ref["y"])
    assert b.num_nodes == 50 and b.num_edges == sum(3 * d["x"].shape[0] for d in dicts)
    gin = GINConv(output_dim=16, mlp_hidden=[16], aggregator="sum", exact=True)
    pool = BatchGlobalPooling(pooling="sum")
    batched = pool([gin([b.x, b.edge_index]), b.batch]).detach().cpu().numpy()
    for i, g in enumerate(graphs):
        single = GlobalPooling(pooling="sum")(gin([g.x, g.edge_index])).detach().cpu().numpy()
        np.testing.assert_allclose(batched[i], single[0], rtol=1e-5, atol=1e-5)
    with pytest.raises(ValueError, match="Cannot batch empty list"):
        kgx.batch_graphs([])
    # GCN on the batched graph equals GCN on each component (disjoint union)
    gcn = GCNConv(8, exact=True)
    yb = gcn([b.x, b.edge_index]).detach().cpu().numpy()
    off = 0
    for g in graphs:
        yi = gcn([g.x, g.edge_index]).detach().cpu().numpy()
        np.testing.assert_array_equal(yb[off:off + g.num_nodes], yi)
        off += g.num_nodes
