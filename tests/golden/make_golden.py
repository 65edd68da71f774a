"""Generate the golden fixtures in tests/golden/*.npz from the CPU oracle.

    python tests/golden/make_golden.py

Inputs are deterministic (numpy PCG64 / the counter-based R-MAT of
oracle/rmat.py); expected outputs come from oracle/reference.py, the op-for-op
restatement of the reference's Keras-torch CPU path.  The reference package
itself cannot be imported here (Keras is not installed), so the
fixtures pin the restatement, which tests/test_oracle_pins.py pins in turn
against the reference tests' own known answers.
Toy graphs are the reference tests' graphs:
  GCN  tests/test_gcn_conv.py:94-96        (6 nodes / 6 edges, in 10 -> out 12)
  GIN  tests/test_gin_conv.py:94-100       (6 / 12)
  GAT  tests/test_gatv2_conv.py:93-99      (6 / 12)
  SAGE tests/test_graphsage_conv.py:114-120 (7 / 14)
"""

from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from oracle import reference as R  # noqa: E402
from oracle.rmat import rmat_edges, scale_for  # noqa: E402

OUT = Path(__file__).resolve().parent
torch.set_num_threads(8)


def glorot(rng, shape):
    fan_in, fan_out = shape[0], shape[-1]
    lim = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=shape).astype(np.float32)


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def npy(x):
    return x.detach().cpu().numpy()


def toy_gcn():
    rng = np.random.default_rng(42)
    x = rng.standard_normal((6, 10)).astype(np.float32)
    ei = np.array([[0, 1, 2, 3, 4, 1], [1, 2, 3, 4, 5, 0]], dtype=np.int32)
    W = glorot(rng, (10, 12))
    b = rng.standard_normal(12).astype(np.float32) * 0.1
    out = {"x": x, "edge_index": ei, "kernel": W, "bias": b}
    for name, (use_b, norm, loops) in {
        "default": (True, True, True),
        "nobias": (False, True, True),
        "nonorm": (True, False, True),
        "noloops": (True, True, False),
    }.items():
        out[f"y_{name}"] = npy(R.gcn_forward(t(x), t(ei), t(W), t(b) if use_b else None, loops, norm))
    out["y_transposed_input"] = npy(R.gcn_forward(t(x), t(ei.T.copy()), t(W), t(b)))
    return out


def toy_gin():
    rng = np.random.default_rng(42)
    x = rng.standard_normal((6, 10)).astype(np.float32)
    ei = np.array([[0, 1, 1, 2, 3, 4, 4, 5, 0, 3, 5, 1], [1, 0, 2, 1, 4, 3, 5, 4, 2, 5, 0, 0]], dtype=np.int32)
    W1, b1 = glorot(rng, (10, 16)), rng.standard_normal(16).astype(np.float32) * 0.1
    W2, b2 = glorot(rng, (16, 12)), rng.standard_normal(12).astype(np.float32) * 0.1
    out = {"x": x, "edge_index": ei, "W1": W1, "b1": b1, "W2": W2, "b2": b2}
    mlp = [(t(W1), t(b1), "relu"), (t(W2), t(b2), None)]
    for aggr in ("sum", "mean", "max"):
        for eps in (0.0, 0.5):
            out[f"h_{aggr}_{eps}"] = npy(R.gin_aggregate_update_input(t(x), t(ei), aggr, eps))
            out[f"y_{aggr}_{eps}"] = npy(R.gin_forward(t(x), t(ei), mlp, aggr, eps))
    return out


def toy_sage():
    rng = np.random.default_rng(45)
    x = rng.standard_normal((7, 10)).astype(np.float32)
    ei = np.array(
        [[0, 1, 1, 2, 3, 4, 4, 5, 0, 3, 6, 5, 1, 6], [1, 0, 2, 1, 4, 3, 5, 4, 2, 5, 5, 6, 6, 0]], dtype=np.int32
    )
    Wn, Ws = glorot(rng, (10, 12)), glorot(rng, (10, 12))
    b = rng.standard_normal(12).astype(np.float32) * 0.1
    Wp, bp = glorot(rng, (10, 10)), rng.standard_normal(10).astype(np.float32) * 0.1
    Wnp = glorot(rng, (10, 12))
    out = {"x": x, "edge_index": ei, "Wn": Wn, "Ws": Ws, "b": b, "Wp": Wp, "bp": bp, "Wnp": Wnp}
    for aggr in ("mean", "max", "sum", "min", "std"):
        for root in (True, False):
            for norm in (False, True):
                out[f"y_{aggr}_{int(root)}_{int(norm)}"] = npy(
                    R.sage_forward(t(x), t(ei), t(Wn), t(Ws) if root else None, t(b), aggr, "relu", norm)
                )
        out[f"aggr_{aggr}"] = npy(R.propagate(t(x), t(ei), aggr))
    out["y_pooling"] = npy(
        R.sage_forward(t(x), t(ei), t(Wnp), t(Ws), t(b), "pooling", "relu", False, pool=(t(Wp), t(bp), "relu"))
    )
    return out


def toy_gat():
    rng = np.random.default_rng(44)
    x = rng.standard_normal((6, 10)).astype(np.float32)
    ei = np.array([[0, 1, 1, 2, 3, 4, 4, 5, 0, 3, 5, 1], [1, 0, 2, 1, 4, 3, 5, 4, 2, 5, 0, 0]], dtype=np.int32)
    out = {"x": x, "edge_index": ei}
    for heads, C in ((1, 8), (4, 8), (2, 16)):
        W = glorot(rng, (10, heads * C))
        att = glorot(rng, (1, heads, C))
        for concat in (True, False):
            b = rng.standard_normal(heads * C if concat else C).astype(np.float32) * 0.1
            key = f"h{heads}_c{C}_{int(concat)}"
            out[f"W_{key}"], out[f"att_{key}"], out[f"b_{key}"] = W, att, b
            out[f"y_{key}"] = npy(R.gatv2_forward(t(x), t(ei), t(W), t(att), t(b), heads, concat, 0.2))
    return out


def rmat_small():
    """Power-law graph in generation order + features; the aggregation outputs
    are bit-exact targets for EXACT mode."""
    N, E, F = 2048, 16384, 32
    s, d = rmat_edges(7, scale_for(N), N, 0, E)
    ei = np.stack([s, d]).astype(np.int32)
    rng = np.random.default_rng(1)
    x = rng.standard_normal((N, F)).astype(np.float32)
    out = {"x": x, "edge_index": ei}
    rowptr, col, eid, deg = R.csr_by_destination(s, d, N, N, self_loops=True)
    out.update(csr_rowptr=rowptr, csr_col=col, csr_eid=eid, csr_deg=deg)
    ei_l = R.add_self_loops(t(ei), N)
    out["deg_f32_loops"] = npy(R.degrees_f32(ei_l, N))
    out["gcn_norm_loops"] = npy(R.compute_gcn_normalization(ei_l, N))
    for aggr in ("sum", "mean", "max", "min", "std"):
        out[f"aggr_{aggr}"] = npy(R.propagate(t(x), t(ei), aggr))
    W = glorot(rng, (F, 32))
    b = rng.standard_normal(32).astype(np.float32) * 0.1
    out.update(gcn_W=W, gcn_b=b, gcn_y=npy(R.gcn_forward(t(x), t(ei), t(W), t(b))))
    # messages H = x W given: GCN aggregation alone (bit-exact target given H and the norms)
    H = (t(x) @ t(W)).numpy()
    out["gcn_H"] = H
    msg = torch.from_numpy(H)[ei_l[0].long()] * torch.from_numpy(out["gcn_norm_loops"]).unsqueeze(1)
    out["gcn_aggr_given_H"] = npy(R.aggregate("sum", msg, ei_l[1], N))
    Wg = glorot(rng, (F, 4 * 8))
    att = glorot(rng, (1, 4, 8))
    bg = rng.standard_normal(32).astype(np.float32) * 0.1
    out.update(gat_W=Wg, gat_att=att, gat_b=bg,
               gat_y=npy(R.gatv2_forward(t(x), t(ei), t(Wg), t(att), t(bg), 4, True, 0.2)))
    return out


def cora_like():
    """Cora-shaped (2,708 nodes / 10,556 directed edges = 5,278 undirected pairs
    both ways, 1,433 binary features at ~1.27% density), 2-layer GCN
    1433 -> 64 -> 7 with relu between (docs/tutorials/node_classification.md:55-73;
    dropout inactive at inference)."""
    rng = np.random.default_rng(2708)
    N, pairs, F = 2708, 5278, 1433
    seen = set()
    und = []
    while len(und) < pairs:
        a, b = (int(v) for v in rng.integers(0, N, 2))
        if a == b or (min(a, b), max(a, b)) in seen:
            continue
        seen.add((min(a, b), max(a, b)))
        und.append((a, b))
    und = np.array(und, dtype=np.int32)
    ei = np.concatenate([und.T, und[:, ::-1].T], axis=1).astype(np.int32)  # reverse edges appended (cora.py:100-110)
    x = (rng.random((N, F)) < 0.0127).astype(np.float32)
    W1, b1 = glorot(rng, (F, 64)), np.zeros(64, np.float32)
    W2, b2 = glorot(rng, (64, 7)), np.zeros(7, np.float32)
    h = torch.relu(R.gcn_forward(t(x), t(ei), t(W1), t(b1)))
    y = R.gcn_forward(h, t(ei), t(W2), t(b2))
    return {"x_packed": np.packbits(x.astype(np.uint8), axis=1), "n_features": np.int32(F), "edge_index": ei,
            "W1": W1, "b1": b1, "W2": W2, "b2": b2, "h1": npy(h), "y": npy(y)}


def edge_cases():
    rng = np.random.default_rng(3)
    N, F = 10, 8
    x = rng.standard_normal((N, F)).astype(np.float32)
    W = glorot(rng, (F, 16))
    b = np.zeros(16, np.float32)
    out = {"x": x, "W": W, "b": b}
    # duplicate edges + existing self loops + isolated nodes (test_error_handling.py:162-204)
    ei_dup = np.array([[0, 0, 0, 1, 2, 2, 5, 5], [1, 1, 1, 1, 2, 3, 5, 0]], dtype=np.int32)
    out["ei_dup"] = ei_dup
    out["y_dup"] = npy(R.gcn_forward(t(x), t(ei_dup), t(W), t(b)))
    for aggr in ("sum", "mean", "max", "min", "std"):
        out[f"aggr_dup_{aggr}"] = npy(R.propagate(t(x), t(ei_dup), aggr))
    # negative indices: src wraps, dst dropped from segments (test_error_handling.py:108-128)
    ei_neg = np.array([[0, -1, 2, 3], [1, 2, -3, 4]], dtype=np.int32)
    out["ei_neg"] = ei_neg
    out["y_neg"] = npy(R.gcn_forward(t(x), t(ei_neg), t(W), t(b)))
    out["aggr_neg_sum"] = npy(R.propagate(t(x), t(ei_neg), "sum"))
    # NaN / inf propagation (test_error_handling.py:233-258)
    ei_r = rng.integers(0, N, size=(2, 20)).astype(np.int32)
    out["ei_r"] = ei_r
    xn = x.copy()
    xn[0, 0] = np.nan
    xi = x.copy()
    xi[0, 0] = np.inf
    out["x_nan"], out["x_inf"] = xn, xi
    out["y_nan"] = npy(R.gcn_forward(t(xn), t(ei_r), t(W), t(b)))
    out["y_inf"] = npy(R.gcn_forward(t(xi), t(ei_r), t(W), t(b)))
    for aggr in ("sum", "max", "min", "mean"):
        out[f"aggr_nan_{aggr}"] = npy(R.propagate(t(xn), t(ei_r), aggr))
        out[f"aggr_inf_{aggr}"] = npy(R.propagate(t(xi), t(ei_r), aggr))
    # signed zeros in max/min ties
    xz = np.zeros((4, 2), np.float32)
    xz[1] = -0.0
    ei_z = np.array([[1, 0, 0, 1, 2, 3], [0, 0, 1, 1, 2, 2]], dtype=np.int32)
    out["x_zero"], out["ei_zero"] = xz, ei_z
    out["aggr_zero_max"] = npy(R.propagate(t(xz), t(ei_z), "max"))
    out["aggr_zero_min"] = npy(R.propagate(t(xz), t(ei_z), "min"))
    # bipartite (test_message_passing.py:196-216)
    xs = rng.standard_normal((4, 8)).astype(np.float32)
    xt = rng.standard_normal((3, 8)).astype(np.float32)
    ei_b = np.array([[0, 1, 2, 3, 0], [0, 1, 2, 0, 1]], dtype=np.int32)
    out["x_src"], out["x_dst"], out["ei_bip"] = xs, xt, ei_b
    out["aggr_bip_sum"] = npy(R.propagate(None, t(ei_b), "sum", x_pair=(t(xt), t(xs))))
    # degree >= 2^24 saturation of the fp32 degree count is exercised by the
    # GPU test directly (too large for a fixture)
    return out


def main():
    cases = {
        "toy_gcn": toy_gcn, "toy_gin": toy_gin, "toy_sage": toy_sage, "toy_gat": toy_gat,
        "rmat_small": rmat_small, "cora_like": cora_like, "edge_cases": edge_cases,
    }
    for name, fn in cases.items():
        data = fn()
        np.savez_compressed(OUT / f"{name}.npz", **data)
        print(f"{name}: {len(data)} arrays, {(OUT / f'{name}.npz').stat().st_size / 1024:.0f} KiB")


if __name__ == "__main__":
    main()
