"""The committed golden fixtures are reproducible from the oracle (CPU).

Integer CSR arrays are compared bit-exactly; floating outputs to 1e-6
(the fixtures were made on this container's AVX-512 ATen kernels; a host
with another vector ISA may differ in the last ulp of pow/exp)."""

import numpy as np
import torch

from oracle import reference as R

T = torch.from_numpy


def close(a, b):
    np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6)


def test_rmat_small_csr_bit_exact(golden):
    g = golden("rmat_small")
    s, d = g["edge_index"]
    N = g["x"].shape[0]
    rowptr, col, eid, deg = R.csr_by_destination(s, d, N, N, self_loops=True)
    for k, v in dict(csr_rowptr=rowptr, csr_col=col, csr_eid=eid, csr_deg=deg).items():
        np.testing.assert_array_equal(g[k], v)
    # fp32 degree of the reference == integer degree (utils/main.py:23-24)
    np.testing.assert_array_equal(g["deg_f32_loops"], deg.astype(np.float32))


def test_rmat_small_outputs(golden):
    g = golden("rmat_small")
    x, ei = T(g["x"]), T(g["edge_index"])
    for aggr in ("sum", "mean", "max", "min", "std"):
        close(R.propagate(x, ei, aggr).numpy(), g[f"aggr_{aggr}"])
    close(R.gcn_forward(x, ei, T(g["gcn_W"]), T(g["gcn_b"])).numpy(), g["gcn_y"])
    close(R.gatv2_forward(x, ei, T(g["gat_W"]), T(g["gat_att"]), T(g["gat_b"]), 4, True, 0.2).numpy(), g["gat_y"])


def test_toys(golden):
    g = golden("toy_gcn")
    close(R.gcn_forward(T(g["x"]), T(g["edge_index"]), T(g["kernel"]), T(g["bias"])).numpy(), g["y_default"])
    g = golden("toy_gin")
    mlp = [(T(g["W1"]), T(g["b1"]), "relu"), (T(g["W2"]), T(g["b2"]), None)]
    close(R.gin_forward(T(g["x"]), T(g["edge_index"]), mlp, "mean", 0.5).numpy(), g["y_mean_0.5"])
    g = golden("toy_gat")
    key = "h4_c8_1"
    close(R.gatv2_forward(T(g["x"]), T(g["edge_index"]), T(g[f"W_{key}"]), T(g[f"att_{key}"]), T(g[f"b_{key}"]),
                          4, True, 0.2).numpy(), g[f"y_{key}"])


def test_cora_like(golden):
    g = golden("cora_like")
    x = np.unpackbits(g["x_packed"], axis=1)[:, : int(g["n_features"])].astype(np.float32)
    h = torch.relu(R.gcn_forward(T(x), T(g["edge_index"]), T(g["W1"]), T(g["b1"])))
    close(h.numpy(), g["h1"])
    close(R.gcn_forward(h, T(g["edge_index"]), T(g["W2"]), T(g["b2"])).numpy(), g["y"])
