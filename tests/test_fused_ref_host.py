"""tests/fused_ref.py (the float64 restatement the fused-op GPU tests hold
every row to) checked on the CPU against the oracle: the GCN forward
(oracle.reference.gcn_forward) and the reference aggregators
(oracle.reference.aggregate) followed by the product with W, on an R-MAT
graph with self loops and a CSR from oracle.reference.csr_by_destination."""

from types import SimpleNamespace

import numpy as np
import pytest
import torch

import fused_ref
from oracle import reference as R
from oracle.rmat import rmat_edges, scale_for

N, E, F, FO = 700, 5000, 16, 12


def _case():
    s, d = rmat_edges(4, scale_for(N), N, 0, E)
    rowptr, col, eid, deg = R.csr_by_destination(s, d, N, N, self_loops=True)
    ei = torch.from_numpy(np.stack([s, d]))
    norm = R.compute_gcn_normalization(R.add_self_loops(ei, N), N)  # per input edge (+ loops), input order
    g = SimpleNamespace(rowptr=torch.from_numpy(rowptr), col=torch.from_numpy(col), n_dst=N,
                        w=norm[torch.from_numpy(eid).long()].float().contiguous(), items=None)
    rng = np.random.default_rng(1)
    x = torch.from_numpy(rng.standard_normal((N, F)).astype(np.float32))
    W = torch.from_numpy((rng.standard_normal((F, FO)) * 0.3).astype(np.float32))
    b = torch.from_numpy(rng.standard_normal(FO).astype(np.float32))
    return ei, g, x, W, b


def test_reference_matches_gcn_forward():
    ei, g, x, W, b = _case()
    y, scale = fused_ref.reference(g, x, W, "sum", True, b, chunk_edges=997)  # several row chunks
    ref = R.gcn_forward(x, ei, W, b).double()
    assert float(((y - ref).abs() / scale.clamp_min(1.0)).max()) <= 1e-6
    fused_ref.check(ref.float(), g, (y, scale), "gcn_forward vs reference")


@pytest.mark.parametrize("red", ["sum", "mean", "max", "min"])
def test_reference_matches_aggregators(red):
    ei, g, x, W, b = _case()
    y, scale = fused_ref.reference(g, x, W, red, False, b, pre_gin=red == "sum", gin_scale=1.5, chunk_edges=1500)
    loops = R.add_self_loops(ei, N)
    agg = R.aggregate(red, x[loops[0].long()], loops[1], N)
    if red == "sum":
        agg = torch.tensor(1.5, dtype=torch.float32) * x + agg
    ref = agg.double() @ W.double() + b.double()
    assert float(((y - ref).abs() / scale.clamp_min(1.0)).max()) <= 1e-6


def test_check_names_the_row():
    ei, g, x, W, b = _case()
    ref = fused_ref.reference(g, x, W, "max", False, b)
    bad = ref[0].float().clone()
    bad[123, 4] += 0.5
    with pytest.raises(AssertionError, match=r"row 123 \(rows kernel\) feature 4"):
        fused_ref.check(bad, g, ref, "planted")
