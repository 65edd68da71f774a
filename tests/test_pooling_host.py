"""Host-side (no GPU) checks of the readout/batching API and its oracle.

Pins: tests/test_pooling.py:41-124 (GlobalPooling init / forward = ops.mean,
max, sum over nodes / serialization) and :173-257 (BatchGlobalPooling init,
shapes, finite mean on the [30, 45, 25]-node fixture, invalid inputs,
serialization); utils/data_utils.py:139-272 batch layout."""

import numpy as np
import pytest
import torch

from keras_geometric_amd.layers import BatchGlobalPooling, GlobalPooling
from oracle import reference as R


def _fixture():  # tests/test_pooling.py:144-171
    np.random.seed(42)
    sizes = [30, 45, 25]
    x = np.random.randn(sum(sizes), 16).astype(np.float32)
    batch = np.repeat(np.arange(3), sizes).astype(np.int32)
    return x, batch, sizes


def test_pooling_init_and_config():
    for p in ("mean", "max", "sum"):
        assert GlobalPooling(pooling=p).pooling == p
        assert BatchGlobalPooling(pooling=p).pooling == p
    with pytest.raises(ValueError, match="pooling must be one of"):
        GlobalPooling(pooling="invalid")
    with pytest.raises(ValueError, match="pooling must be one of"):
        BatchGlobalPooling(pooling="invalid")
    layer = BatchGlobalPooling(pooling="sum")
    cfg = layer.get_config()
    assert cfg["pooling"] == "sum" and BatchGlobalPooling.from_config(cfg).pooling == "sum"
    assert GlobalPooling.from_config(GlobalPooling(pooling="max").get_config()).pooling == "max"


def test_pooling_shape_errors():
    assert GlobalPooling().compute_output_shape((10, 5)) == (1, 5)
    with pytest.raises(ValueError, match="Expected input shape to be 2D"):
        GlobalPooling().compute_output_shape((10, 5, 2))
    layer = BatchGlobalPooling(pooling="mean")
    with pytest.raises(ValueError, match="inputs must be a list/tuple"):
        layer.call(torch.zeros((10, 5)))
    with pytest.raises(ValueError, match="input_shape must be a list/tuple"):
        layer.compute_output_shape((10, 5))
    assert layer.compute_output_shape([(10, 5), (10,)]) == (None, 5)


def test_oracle_pooling_pins():
    x, batch, sizes = _fixture()
    for p in ("mean", "max", "sum"):
        out = R.batch_global_pooling(torch.from_numpy(x), torch.from_numpy(batch), p).numpy()
        assert out.shape == (3, 16) and np.isfinite(out).all()
        parts = np.split(x, np.cumsum(sizes)[:-1])
        ref = np.stack([{"mean": q.mean(0), "max": q.max(0), "sum": q.sum(0)}[p] for q in parts])
        np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-5)
        g = R.global_pooling(torch.from_numpy(x), p).numpy()
        np.testing.assert_allclose(g[0], {"mean": x.mean(0), "max": x.max(0), "sum": x.sum(0)}[p], rtol=1e-5,
                                   atol=1e-5)
    # empty graph id (no nodes with batch == 1): segment_max gives -inf, mean/sum give 0
    b = np.array([0, 0, 2, 2], np.int32)
    xx = np.ones((4, 3), np.float32)
    assert np.isneginf(R.batch_global_pooling(torch.from_numpy(xx), torch.from_numpy(b), "max")[1]).all()
    assert (R.batch_global_pooling(torch.from_numpy(xx), torch.from_numpy(b), "mean")[1] == 0).all()


def test_oracle_batch_graphs_layout():
    g1 = {"x": np.ones((3, 2), np.float32), "edge_index": np.array([[0, 1], [1, 2]], np.int32),
          "y": np.array([1.0], np.float32)}
    g2 = {"x": np.zeros((2, 2), np.float32), "edge_index": np.array([[1], [0]], np.int32),
          "y": np.array([0.0], np.float32)}
    b = R.batch_graphs([g1, g2])
    np.testing.assert_array_equal(b["edge_index"], [[0, 1, 4], [1, 2, 3]])
    np.testing.assert_array_equal(b["batch"], [0, 0, 0, 1, 1])
    assert b["y"].shape == (2, 1) and b["x"].shape == (5, 2)
