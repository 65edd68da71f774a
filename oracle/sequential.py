"""Plain sequential numpy restatements (small cases only).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Used to pin oracle/keras_torch.py's scatter-based lowering against the
definition the reference tests state in words: "for node i: aggr_i = Σ / max /
mean over j ∈ N(i) of m_{j→i}" (aggregators.py:48-232 docstrings), with the
accumulation order of the input edge list, and the manual SAGE-mean check of
tests/test_graphsage_conv.py:465-514.
"""

from __future__ import annotations

import numpy as np


def segment_sum_loop(messages: np.ndarray, target: np.ndarray, n: int) -> np.ndarray:
    out = np.zeros((n,) + messages.shape[1:], dtype=np.float32)
    for e in range(messages.shape[0]):
        t = int(target[e])
        if 0 <= t < n:
            out[t] = (out[t] + messages[e]).astype(np.float32)
    return out


def segment_max_loop(messages: np.ndarray, target: np.ndarray, n: int) -> np.ndarray:
    out = np.full((n,) + messages.shape[1:], -np.inf, dtype=np.float32)
    for e in range(messages.shape[0]):
        t = int(target[e])
        if 0 <= t < n:
            v = messages[e]
            cur = out[t]
            out[t] = np.where(np.isnan(v) | (v > cur), v, cur)
    return out


def mean_neighbors_loop(x: np.ndarray, edge_index: np.ndarray, n: int) -> np.ndarray:
    """tests/test_graphsage_conv.py:465-484 (defaultdict adjacency + np.mean)."""
    adj: dict[int, list[int]] = {}
    for s, t in zip(edge_index[0], edge_index[1]):
        adj.setdefault(int(t), []).append(int(s))
    out = np.zeros((n, x.shape[1]), dtype=np.float32)
    for i in range(n):
        nb = adj.get(i, [])
        if nb:
            out[i] = np.mean(x[nb], axis=0)
    return out
