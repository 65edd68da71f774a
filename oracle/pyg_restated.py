"""PyTorch Geometric's GCNConv / GATv2Conv / GINConv forwards, restated in
float64 numpy from their published algorithms (torch-geometric >= 2.6.1, the
version the reference pins for its numerical comparison tests,
pyproject.toml:51).  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference's own tests take PyG as ground truth for these layers
(tests/test_gcn_conv.py:556-631 at rtol 1e-4 / atol 1e-5, failing above 1e-3;
tests/test_gatv2_conv.py:384-490 at rtol = atol = 1e-6, with PyG's lin_l and
lin_r both set to the reference's one kernel and their biases zeroed;
tests/test_gin_conv.py:590-650 at 1e-4).  torch_geometric is not installed
here, so this module restates those algorithms; tests/test_oracle_pyg_pins.py
checks oracle/reference.py against it, which pins the GCN normalisation
(utils/main.py:20-33) and the GATv2 segment softmax (gatv2_conv.py:268-311)
legs that no reference-held vector covers.

Restated (PyG 2.6.1):
- gcn_norm(add_self_loops=True, improved=False): add_remaining_self_loops with
  fill value 1 (one loop per node; a node's existing loop keeps its weight),
  deg = scatter_add(w, col), dinv = deg^-1/2 with inf -> 0,
  w_e = dinv[row] w_e dinv[col]; GCNConv: x W (no bias in lin), sum of
  w_e (xW)[row] at col, + bias.
- GATv2Conv(share_weights=False, add_self_loops=True, edge_dim=None):
  x_l = lin_l(x), x_r = lin_r(x) as [N, H, C]; remove_self_loops then
  add_self_loops; per edge z = leaky_relu(x_r[dst] + x_l[src]),
  a = sum_c att[h, c] z[h, c]; softmax over dst: exp(a - max) / (sum + 1e-16);
  out[dst] += a x_l[src]; concat [N, H C] or mean over heads; + bias.
- GINConv(aggr='add' | 'mean' | 'max'): nn((1 + eps) x + aggr_j x_j).
"""

from __future__ import annotations

import numpy as np


def _add_remaining_self_loops(src, dst, w, n):
    keep = src != dst
    loop_w = np.ones(n)
    loop_w[dst[~keep]] = w[~keep]  # an existing loop keeps its weight
    loops = np.arange(n)
    return (np.concatenate([src[keep], loops]), np.concatenate([dst[keep], loops]),
            np.concatenate([w[keep], loop_w]))


def gcn_forward(x, edge_index, W, b=None, normalize=True, add_self_loops=True):
    x = np.asarray(x, np.float64)
    src, dst = (np.asarray(v, np.int64) for v in edge_index)
    n = x.shape[0]
    w = np.ones(src.shape[0])
    if normalize:
        if add_self_loops:
            src, dst, w = _add_remaining_self_loops(src, dst, w, n)
        deg = np.zeros(n)
        np.add.at(deg, dst, w)
        with np.errstate(divide="ignore"):
            dinv = deg ** -0.5
        dinv[np.isinf(dinv)] = 0.0
        w = dinv[src] * w * dinv[dst]
    h = x @ np.asarray(W, np.float64)
    out = np.zeros((n, h.shape[1]))
    np.add.at(out, dst, h[src] * w[:, None])
    return out + (np.asarray(b, np.float64) if b is not None else 0.0)


def gatv2_forward(x, edge_index, W, att, b=None, heads=1, concat=True, negative_slope=0.2,
                  add_self_loops=True):
    """W: [F_in, heads * C] (the reference's kernel; PyG's lin_l = lin_r = W^T)."""
    x = np.asarray(x, np.float64)
    src, dst = (np.asarray(v, np.int64) for v in edge_index)
    n = x.shape[0]
    W = np.asarray(W, np.float64)
    C = W.shape[1] // heads
    h = (x @ W).reshape(n, heads, C)  # x_l = x_r
    if add_self_loops:
        keep = src != dst
        src = np.concatenate([src[keep], np.arange(n)])
        dst = np.concatenate([dst[keep], np.arange(n)])
    z = h[dst] + h[src]
    z = np.where(z > 0, z, negative_slope * z)
    a = (z * np.asarray(att, np.float64).reshape(1, heads, C)).sum(-1)  # [E, H]
    amax = np.full((n, heads), -np.inf)
    np.maximum.at(amax, dst, a)
    ex = np.exp(a - amax[dst])
    ssum = np.zeros((n, heads))
    np.add.at(ssum, dst, ex)
    alpha = ex / (ssum[dst] + 1e-16)
    out = np.zeros((n, heads, C))
    np.add.at(out, dst, h[src] * alpha[:, :, None])
    out = out.reshape(n, heads * C) if concat else out.mean(axis=1)
    return out + (np.asarray(b, np.float64) if b is not None else 0.0)


def gin_forward(x, edge_index, W, b=None, eps=0.0, aggr="add"):
    """nn = one Linear (the reference's default MLP is one Dense)."""
    x = np.asarray(x, np.float64)
    src, dst = (np.asarray(v, np.int64) for v in edge_index)
    n, f = x.shape
    if aggr == "add":
        agg = np.zeros((n, f))
        np.add.at(agg, dst, x[src])
    elif aggr == "mean":
        agg = np.zeros((n, f))
        np.add.at(agg, dst, x[src])
        cnt = np.bincount(dst, minlength=n).astype(np.float64)
        agg = agg / np.maximum(cnt, 1.0)[:, None]
    else:  # max; PyG fills rows without messages with 0
        agg = np.full((n, f), -np.inf)
        np.maximum.at(agg, dst, x[src])
        agg[np.isinf(agg)] = 0.0
    hin = (1.0 + eps) * x + agg
    return hin @ np.asarray(W, np.float64) + (np.asarray(b, np.float64) if b is not None else 0.0)
