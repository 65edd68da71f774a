"""Host-side layer logic that needs no GPU (CPU)."""

import numpy as np
import pytest
import torch

from keras_geometric_amd import graph as G
from keras_geometric_amd.layers import (
    AggregatorFactory,
    GATv2Conv,
    GCNConv,
    GINConv,
    MessagePassing,
    SAGEConv,
)


def test_invalid_aggregators():
    """tests/unit/test_error_handling.py:26-40."""
    for bad in ["invalid", "median", "variance", ""]:
        with pytest.raises(ValueError, match="Invalid aggregator"):
            MessagePassing(aggregator=bad)
        with pytest.raises(ValueError, match="Invalid aggregator"):
            GINConv(output_dim=16, aggregator=bad)
        with pytest.raises(ValueError, match="Invalid aggregator"):
            SAGEConv(output_dim=16, aggregator=bad)
    with pytest.raises(ValueError, match="Invalid aggregator"):
        GINConv(output_dim=16, aggregator="min")
    assert AggregatorFactory.get_available_aggregators() == ["mean", "max", "sum", "min", "std"]


def test_message_passing_input_contract():
    mp = MessagePassing(aggregator="mean")
    with pytest.raises(ValueError):
        mp.call("invalid_input")
    with pytest.raises(ValueError):
        mp.call([])
    with pytest.raises(ValueError):
        mp([np.zeros((3, 2), np.float32)])


def test_configs_round_trip():
    for layer in (GCNConv(8, add_self_loops=False), GINConv(8, mlp_hidden=[4], eps_init=0.1),
                  SAGEConv(8, aggregator="pooling", pool_hidden_dim=6), GATv2Conv(4, heads=2, concat=False)):
        cfg = layer.get_config()
        again = type(layer).from_config(cfg)
        assert again.get_config() == cfg
    assert GCNConv(8).get_config()["aggregator"] == "sum"
    assert SAGEConv(8, aggregator="pooling").get_config()["aggregator"] == "pooling"


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure mode")
def test_no_cpu_fallback():
    layer = GCNConv(4)
    with pytest.raises(RuntimeError, match="no CPU execution path"):
        layer([np.zeros((3, 2), np.float32), np.array([[0, 1], [1, 2]])])


def test_split_len_policy():
    assert G.default_split_len(10_000, 128) == 256
    assert G.default_split_len(110_000_000, 128) == 1024
    assert G.default_split_len(11_000_000, 128) == 256
    for e in (0, 1, 10**9):
        v = G.default_split_len(e, 100)
        assert 256 <= v <= 8192 and v & (v - 1) == 0


def test_cache_key_tracks_version():
    t = torch.zeros((2, 4), dtype=torch.int32)
    k1 = G.cache_key(t, 1)
    t[0, 0] = 1
    assert G.cache_key(t, 1) != k1
    assert G.cache_key([[0, 1], [1, 2]], 1) is None  # a list becomes a new array on every call


def test_host_array_key():
    """A numpy edge_index is keyed like the reference's id()-keyed cast cache
    (message_passing.py:256-268), plus its address, shape, strides, dtype and a
    sampled fingerprint: the same array keys the same, an in-place change in
    the sampled positions or a different array does not."""
    a = np.arange(20_000, dtype=np.int64).reshape(2, -1)
    k = G.cache_key(a, 1)
    assert k is not None and k == G.cache_key(a, 1)
    assert G.cache_key(a, 2) != k
    a[:] = a[:, ::-1].copy()
    assert G.cache_key(a, 1) != k
    b = a.copy()
    assert G.cache_key(b, 1) != G.cache_key(a, 1)  # another array (id and address)
    assert G.host_array_key(torch.zeros(2, 3)) is None


def test_fused_shape_routing(monkeypatch):
    """Which shapes take a fused aggregate -> transform kernel: F_in 128 ->
    128 (kgx_spmm_gemm), 256 -> 256 (kgx_spmm_gemm_f256; the sharded passes'
    two-table gathers through kgx_spmm_gemm_f256_ex); KGX_FUSED256=0 /
    KGX_FUSED=0 turn them off."""
    from keras_geometric_amd import ops as kops

    monkeypatch.delenv("KGX_FUSED", raising=False)
    monkeypatch.delenv("KGX_FUSED256", raising=False)
    assert kops.fused_transform_supported(128, 128)
    assert not kops.fused_transform_supported(128, 64)  # F_out < F_in: transform first, gather the narrower rows
    assert not kops.fused_transform_supported(128, 256)  # F_in <= F_out but the 128 kernel stops at 128
    assert kops.fused_transform_supported(256, 256)
    assert not kops.fused_transform_supported(256, 128)  # transform first: narrower rows to gather
    assert kops.fused_transform_supported(256, 256, two_table=True)  # sharded GIN at C4: kgx_spmm_gemm_f256_ex
    assert kops.fused_transform_supported(128, 128, two_table=True)
    monkeypatch.setenv("KGX_FUSED256", "0")
    assert not kops.fused_transform_supported(256, 256) and kops.fused_transform_supported(128, 128)
    monkeypatch.setenv("KGX_FUSED", "0")
    assert not kops.fused_transform_supported(128, 128)


def test_fused_sage_routing(monkeypatch):
    """SAGEConv's fused update (kgx_spmm_gemm accumulating into b + x W_self):
    opt-in with KGX_FUSED_SAGE=1; any F_in, F_out <= 128 that are multiples of 4
    (C5: 100 -> 100); KGX_FUSED=0 turns it off too."""
    from keras_geometric_amd import ops as kops

    monkeypatch.delenv("KGX_FUSED", raising=False)
    monkeypatch.delenv("KGX_FUSED_SAGE", raising=False)
    assert not kops.fused_sage_supported(100, 100)  # opt-in: slower than the two-step path at C5
    monkeypatch.setenv("KGX_FUSED_SAGE", "1")
    assert kops.fused_sage_supported(100, 100) and kops.fused_sage_supported(128, 4)
    assert not kops.fused_sage_supported(102, 100)  # rows must be whole float4s
    assert not kops.fused_sage_supported(256, 256) and not kops.fused_sage_supported(100, 132)
    monkeypatch.setenv("KGX_FUSED_SAGE", "0")
    assert not kops.fused_sage_supported(100, 100)
    monkeypatch.setenv("KGX_FUSED_SAGE", "1")
    monkeypatch.setenv("KGX_FUSED", "0")
    assert not kops.fused_sage_supported(100, 100)


def _cpu_graph(deg):
    """A CSRGraph shell on the host: rows in descending degree, as build_csr orders them."""
    deg = torch.tensor(deg, dtype=torch.int32)
    rowptr = torch.zeros(len(deg) + 1, dtype=torch.int32)
    rowptr[1:] = torch.cumsum(deg, 0)
    kept = int(rowptr[-1])
    rows = torch.argsort(-deg.long(), stable=True).to(torch.int32)
    z = torch.zeros(max(kept, 1), dtype=torch.int32)
    return G.CSRGraph(n_src=len(deg), n_dst=len(deg), n_input_edges=kept, kept=kept, max_degree=int(deg.max()),
                      flags=0, rowptr=rowptr, col=z, eid=z, deg=deg, rows=rows)


def test_exact_short_start(monkeypatch):
    """EXACT mode's short-row suffix (kgx_spmm_ex n_long_items with items = NULL):
    the index in the degree-descending row list where degree <= 7 starts; -1 when
    every row is short or none is, or with KGX_SHORT_ROWS=0."""
    monkeypatch.delenv("KGX_SHORT_ROWS", raising=False)
    monkeypatch.delenv("KGX_SHORT_MAX", raising=False)
    g = _cpu_graph([3, 9, 0, 2048, 7, 8, 1])
    assert G.exact_short_start(g) == 3  # rows of degree 2048, 9, 8 come first
    assert g.extras["exact_short"] == 3
    assert G.exact_short_start(_cpu_graph([1, 2, 3])) == -1  # all short: the main kernel keeps them
    assert G.exact_short_start(_cpu_graph([8, 9, 100])) == -1  # none short
    monkeypatch.setenv("KGX_SHORT_ROWS", "0")
    assert G.exact_short_start(_cpu_graph([3, 9, 0])) == -1
