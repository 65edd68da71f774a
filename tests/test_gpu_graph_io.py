"""Persistent graph files: the reference's processed NPZ
layout (datasets/base.py:124-182) read and written, plus kgx CSRs that the
layers pick up from the cache instead of re-sorting the edges."""

import numpy as np
import pytest
import torch

import keras_geometric_amd as kgx
from keras_geometric_amd import graph as G
from keras_geometric_amd.layers import GCNConv
from keras_geometric_amd.utils import load_graphs, save_graphs
from oracle.rmat import rmat_edges, scale_for

pytestmark = pytest.mark.gpu


def _graphs():
    out = []
    for seed, (n, e) in enumerate(((3000, 30000), (500, 4000))):
        s, d = rmat_edges(seed + 30, scale_for(n), n, 0, e)
        x = np.random.default_rng(seed).standard_normal((n, 64)).astype(np.float32)
        out.append(kgx.GraphData(x=x, edge_index=np.stack([s, d]).astype(np.int32), y=np.array([seed], np.float32)))
    return out


def test_roundtrip_with_csr_and_cache_hit(dev, tmp_path, monkeypatch):
    graphs = _graphs()
    path = tmp_path / "processed.npz"
    save_graphs(path, graphs, num_classes=3, with_csr=True, self_loops=True, gcn_norm=True, n_features=64)
    G.clear_cache()
    loaded, ncls = load_graphs(path)
    assert ncls == 3 and len(loaded) == 2
    for a, b in zip(graphs, loaded):
        np.testing.assert_array_equal(a.x.cpu().numpy(), b.x.cpu().numpy())
        np.testing.assert_array_equal(a.edge_index.cpu().numpy(), b.edge_index.cpu().numpy())
        np.testing.assert_array_equal(a.y.cpu().numpy(), b.y.cpu().numpy())
        ref = G.build_csr(a.edge_index[0].contiguous(), a.edge_index[1].contiguous(), a.num_nodes, a.num_nodes,
                          self_loops=True, gcn_norm=True, n_features=64)
        for f in ("rowptr", "col", "eid", "deg", "dinv", "w", "rows", "items", "split"):
            np.testing.assert_array_equal(getattr(ref, f).cpu().numpy(), getattr(b.csr, f).cpu().numpy())
    # the layer finds the loaded CSR: no graph build happens
    layer = GCNConv(64)
    g0 = loaded[0]

    def no_build(*a, **k):
        raise AssertionError("CSR rebuilt instead of loaded")

    monkeypatch.setattr(G, "build_csr", no_build)
    y = layer([g0.x, g0.edge_index])
    monkeypatch.undo()
    y_ref = layer([graphs[0].x, graphs[0].edge_index])
    np.testing.assert_array_equal(y.detach().cpu().numpy(), y_ref.detach().cpu().numpy())


def test_reference_layout_without_csr(dev, tmp_path):
    """A file in the reference's own layout (no kgx arrays) loads as GraphData."""
    rng = np.random.default_rng(0)
    arrays = {"num_graphs": 2, "num_classes": 4}
    for i in range(2):
        arrays[f"x_{i}"] = rng.standard_normal((5 + i, 3)).astype(np.float32)
        arrays[f"edge_index_{i}"] = np.array([[0, 1], [1, 2]], np.int32)
    np.savez(tmp_path / "ref.npz", **arrays)
    loaded, ncls = load_graphs(tmp_path / "ref.npz")
    assert ncls == 4 and [g.num_nodes for g in loaded] == [5, 6]
    assert not hasattr(loaded[0], "csr") or loaded[0].__dict__.get("csr") is None
    np.testing.assert_array_equal(loaded[1].x.cpu().numpy(), arrays["x_1"])
