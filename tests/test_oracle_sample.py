"""The sampled-row oracle (tests/oracle_sample.py) against the whole-graph
oracle on a small R-MAT graph (CPU): the full-size GPU tests of C4 / C5 / NS
compare sampled rows with it, so it must reproduce the reference's rows --
aggregation order, degrees (GCN: the whole graph's) and the per-row dense maps."""

import numpy as np
import torch

import oracle_sample as OS
from oracle import reference as R
from oracle.rmat import rmat_edges, scale_for


def _graph(n=3000, e=30000, f=24, seed=5):
    s, d = rmat_edges(seed, scale_for(n), n, 0, e)
    rng = np.random.default_rng(seed)
    x = torch.from_numpy(rng.standard_normal((n, f)).astype(np.float32))
    return torch.from_numpy(np.stack([s, d]).astype(np.int32)), x, rng


def test_sampled_rows_equal_whole_graph_oracle():
    ei, x, rng = _graph()
    n, f = x.shape
    rows = OS.sample_rows(ei, n, k=300, hubs=4, seed=1)
    assert rows.numel() > 250
    W = torch.from_numpy((rng.standard_normal((f, 16)) * 0.3).astype(np.float32))
    W2 = torch.from_numpy((rng.standard_normal((f, 16)) * 0.3).astype(np.float32))
    b = torch.from_numpy(rng.standard_normal(16).astype(np.float32))
    full = R.gin_forward(x, ei, [(W, b, None)], "sum", eps=0.25)[rows]
    np.testing.assert_allclose(OS.gin_rows(ei, x, rows, [(W, b, None)], 0.25).numpy(), full.numpy(), rtol=1e-6,
                               atol=1e-6)
    full = R.sage_forward(x, ei, W, W2, b, "mean")[rows]
    np.testing.assert_allclose(OS.sage_rows(ei, x, rows, W, W2, b).numpy(), full.numpy(), rtol=1e-6, atol=1e-6)
    full = R.gcn_forward(x, ei, W, b)[rows]
    np.testing.assert_allclose(OS.gcn_rows(ei, x, rows, W, b).numpy(), full.numpy(), rtol=1e-6, atol=1e-6)
