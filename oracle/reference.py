"""Reference forward passes, restated op for op on the Keras-torch lowering.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Every function follows the cited reference lines (src/keras_geometric/...) and
calls the keras.ops lowering in oracle/keras_torch.py in the same order, on
the same dtypes, so its fp32 results are the reference's CPU results
(up to the unpinned Keras version, see oracle/__init__.py).
"""

from __future__ import annotations

import numpy as np
import torch

from . import keras_torch as K

# ---------------------------------------------------------------------------
# utils/main.py
# ---------------------------------------------------------------------------


def add_self_loops(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """utils/main.py:8-16 — loops appended AFTER the input edges."""
    if edge_index.shape[0] != 2:
        edge_index = torch.stack([edge_index[0], edge_index[1]], dim=0)
    loops = torch.arange(0, num_nodes, dtype=edge_index.dtype)
    return torch.cat([edge_index, torch.stack([loops, loops], dim=0)], dim=1)


def compute_gcn_normalization(edge_index: torch.Tensor, num_nodes: int, degrees=None) -> torch.Tensor:
    """utils/main.py:20-33.  degrees (test instrument, default None = the
    reference): the fp32 in-degree vector to use instead of the one this edge
    set gives -- the whole graph's, when edge_index holds only the in-edges of
    sampled rows (tests/oracle_sample.py)."""
    source, target = edge_index[0], edge_index[1]
    ones = torch.ones_like(source, dtype=K.FLOATX)
    if degrees is None:
        degrees = K.segment_sum(ones, target, num_nodes)
    dinv = K.power(K.add(degrees, 1e-12), -0.5)
    dinv = K.where(K.isinf(dinv), torch.zeros_like(dinv), dinv)
    return K.multiply(K.take(dinv, target, axis=0), K.take(dinv, source, axis=0))


def degrees_f32(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """The fp32 degree vector of utils/main.py:23-24 (exposed for the int/fp32 parity tests)."""
    ones = torch.ones_like(edge_index[1], dtype=K.FLOATX)
    return K.segment_sum(ones, edge_index[1], num_nodes)


# ---------------------------------------------------------------------------
# layers/aggregators.py
# ---------------------------------------------------------------------------


def aggregate(name: str, messages: torch.Tensor, target_idx: torch.Tensor, dim_size: int) -> torch.Tensor:
    """Aggregator.aggregate for mean/max/sum/min/std (aggregators.py:48-232)."""
    messages = K.convert(messages)
    if messages.shape[0] == 0:
        return torch.zeros((dim_size, messages.shape[1]), dtype=messages.dtype)
    target_idx = K.cast(target_idx, torch.int32)
    if name == "sum":  # :126-137
        return K.segment_sum(messages, target_idx, dim_size)
    if name == "mean":  # :56-85
        ones = torch.ones((messages.shape[0], 1), dtype=messages.dtype)
        degree = K.segment_sum(ones, target_idx, dim_size)
        s = K.segment_sum(messages, target_idx, dim_size)
        degree = K.maximum(degree, K.convert(1e-8, degree.dtype))
        return s / degree
    if name == "max":  # :99-112
        aggr = K.segment_max(messages, target_idx, dim_size)
        return K.where(K.isinf(aggr), torch.zeros_like(aggr), aggr)
    if name == "min":  # :151-167
        aggr = -K.segment_max(-messages, target_idx, dim_size)
        return K.where(K.isinf(aggr), torch.zeros_like(aggr), aggr)
    if name == "std":  # :182-228
        ones = torch.ones((messages.shape[0], 1), dtype=messages.dtype)
        count = K.segment_sum(ones, target_idx, dim_size)
        sums = K.segment_sum(messages, target_idx, dim_size)
        safe = K.maximum(count, K.convert(1e-8, count.dtype))
        mean = sums / safe
        mean_e = K.take(mean, target_idx, axis=0)
        sq = torch.square(messages - mean_e)
        ssd = K.segment_sum(sq, target_idx, dim_size)
        var = ssd / safe
        std = torch.sqrt(K.maximum(var, torch.zeros_like(var)))
        return K.where(count <= 1, torch.zeros_like(std), std)
    raise ValueError(f"Invalid aggregator: {name}")


def pooling_aggregate(messages, target_idx, dim_size, pool_kernel, pool_bias, pool_activation="relu"):
    """PoolingAggregator (aggregators.py:254-274): segment_max(pool_mlp(m)), isinf -> 0."""
    t = K.dense(messages, pool_kernel, pool_bias, pool_activation)
    aggr = K.segment_max(t, K.cast(target_idx, torch.int32), dim_size)
    return K.where(K.isinf(aggr), torch.zeros_like(aggr), aggr)


# ---------------------------------------------------------------------------
# layers/message_passing.py
# ---------------------------------------------------------------------------


def propagate(x, edge_index, aggregator: str = "mean", message=None, x_pair=None) -> torch.Tensor:
    """MessagePassing.propagate with the default message x_j (message_passing.py:147-220)."""
    if x_pair is not None:
        x_i, x_j = K.convert(x_pair[0]), K.convert(x_pair[1])
    else:
        x_i = x_j = K.convert(x)
    n = x_i.shape[0]
    if n == 0:
        return torch.zeros((0, x_i.shape[1] if x_i.dim() > 1 else 1), dtype=x_i.dtype)
    ei = K.cast(edge_index, torch.int32)
    if ei.shape[1] == 0:
        return torch.zeros((n, x_i.shape[1]), dtype=x_i.dtype)
    src, dst = ei[0], ei[1]
    xj = K.take(x_j, src, axis=0)
    xi = K.take(x_i, dst, axis=0)
    msg = xj if message is None else message(xi, xj)
    return aggregate(aggregator, msg, dst, n)


# ---------------------------------------------------------------------------
# layers/gcn_conv.py
# ---------------------------------------------------------------------------


def _as_2xE(ei: torch.Tensor) -> torch.Tensor:
    ei = K.cast(ei, torch.int32)
    if ei.shape[0] != 2:
        if ei.shape[1] == 2:
            return ei.t()
        raise ValueError(f"edge_index must have shape [2, E] or [E, 2], but got {tuple(ei.shape)}")
    return ei


def gcn_forward(x, edge_index, kernel, bias=None, add_self_loops_: bool = True, normalize: bool = True,
                degrees=None):
    """GCNConv.call (gcn_conv.py:275-364) incl. message (:233-248) and update (:266-272).
    degrees: see compute_gcn_normalization (sampled-row checks only)."""
    x = K.cast(x, torch.float32)
    ei = _as_2xE(edge_index)
    kernel = K.convert(kernel)
    n = x.shape[0]
    out_dim = kernel.shape[1]
    if n == 0:
        return torch.zeros((0, out_dim), dtype=x.dtype)
    if add_self_loops_:
        ei = add_self_loops(ei, n)
    e = ei.shape[1]
    if e == 0:
        y = torch.matmul(x, kernel)
        return y + bias if bias is not None else y
    w = compute_gcn_normalization(ei, n, degrees) if normalize else torch.ones((e,), dtype=torch.float32)
    src, dst = ei[0], ei[1]
    x_j = K.take(x, src, axis=0)
    _x_i = K.take(x, dst, axis=0)  # gathered by the reference (message_passing.py:196), unused by GCN
    msg = torch.matmul(x_j, kernel) * torch.unsqueeze(w, 1)
    aggr = aggregate("sum", msg, dst, n)
    return K.add(aggr, bias) if bias is not None else aggr


# ---------------------------------------------------------------------------
# layers/gin_conv.py
# ---------------------------------------------------------------------------


def gin_aggregate_update_input(x, edge_index, aggregator="sum", eps: float = 0.0, eps_tensor=None):
    """(1+eps)*x + AGG(x_j), the MLP input of GINConv.update (gin_conv.py:216-222)."""
    x = K.convert(x)
    ei = K.cast(edge_index, torch.int32)
    scale = (1 + eps_tensor) if eps_tensor is not None else (1 + eps)
    if ei.shape[1] == 0:  # :269-277
        return scale * x
    aggr = propagate(x, ei, aggregator)  # message x_j (:193) -> Sum/Mean/MaxAggregator
    return scale * x + aggr


def gin_forward(x, edge_index, mlp, aggregator="sum", eps: float = 0.0, eps_tensor=None):
    """GINConv.call (gin_conv.py:228-300); mlp = [(kernel, bias, activation), ...] (:129-162)."""
    x = K.convert(x)
    if x.shape[0] == 0:
        return torch.zeros((0, K.convert(mlp[-1][0]).shape[1]), dtype=x.dtype)
    h = gin_aggregate_update_input(x, edge_index, aggregator, eps, eps_tensor)
    for kernel, bias, act in mlp:
        h = K.dense(h, kernel, bias, act)
    return h


# ---------------------------------------------------------------------------
# layers/sage_conv.py
# ---------------------------------------------------------------------------


def sage_forward(x, edge_index, w_neigh, w_self=None, bias=None, aggregator="mean", activation="relu",
                 normalize=False, pool=None, msg_mask=None):
    """SAGEConv.call (sage_conv.py:351-439); pool = (kernel, bias, activation) for 'pooling';
    msg_mask [E, F]: training-mode Dropout(x_j) given its mask (sage_conv.py:280-298)."""
    x = K.cast(x, torch.float32)
    ei = _as_2xE(edge_index)
    n = x.shape[0]
    if ei.shape[1] == 0:  # :318-326
        feat = K.convert(pool[0]).shape[1] if aggregator == "pooling" else x.shape[1]
        aggr = torch.zeros((n, feat), dtype=x.dtype)
    else:
        src, dst = ei[0], ei[1]
        x_j = K.take(x, src, axis=0)
        _x_i = K.take(x, dst, axis=0)
        if msg_mask is not None:
            x_j = x_j * msg_mask
        if aggregator == "pooling":
            aggr = pooling_aggregate(x_j, dst, n, *pool)
        else:
            aggr = aggregate(aggregator, x_j, dst, n)
    h_neigh = K.dense(aggr, w_neigh)
    out = K.add(K.dense(x, w_self), h_neigh) if w_self is not None else h_neigh
    if bias is not None:
        out = K.add(out, bias)
    if activation == "relu":
        out = torch.relu(out)
    if normalize:
        out = K.normalize_l2(out)
    return out


# ---------------------------------------------------------------------------
# layers/gatv2_conv.py
# ---------------------------------------------------------------------------


def gatv2_forward(x, edge_index, kernel, att, bias=None, heads=1, concat=True, negative_slope=0.2,
                  add_self_loops_: bool = True, lrelu_positive=None):
    """GATv2Conv.call/_gatv2_propagate (gatv2_conv.py:129-352).

    lrelu_positive (test instrument, default None = the reference): a bool
    [E', heads, C] mask fixing which branch the leaky ReLU of :277-278 takes.
    Its derivative jumps from 1 to negative_slope at z = 0, so where an fp32
    and an fp64 evaluation put a z within ~1e-8 of 0 on opposite sides their
    gradients differ at O(1) for that edge (tests/test_gatv2_conditioning.py)."""
    x = K.convert(x)
    ei = K.cast(K.convert(edge_index), torch.int32)
    kernel = K.convert(kernel)
    C = kernel.shape[1] // heads
    n = x.shape[0]
    if add_self_loops_:
        ei = add_self_loops(ei, n)
    e = ei.shape[1]
    out_dim = heads * C if concat else C
    if n == 0:
        return torch.zeros((0, out_dim), dtype=x.dtype)
    if e == 0:
        return torch.zeros((n, out_dim), dtype=x.dtype)
    h = torch.matmul(x, kernel).reshape(n, heads, C)  # :224-228
    src, dst = ei[0], ei[1]
    h_j = K.take(h, src, axis=0)
    h_i = K.take(h, dst, axis=0)
    if lrelu_positive is None:
        z = K.leaky_relu(K.add(h_i, h_j), negative_slope)  # :277-278
    else:
        zin = K.add(h_i, h_j)
        z = torch.where(lrelu_positive, zin, zin * negative_slope)
    scores = torch.sum(K.multiply(z, K.convert(att)), dim=-1)  # :284
    mx = K.segment_max(scores, dst, n)  # :298
    ex = torch.exp(torch.subtract(scores, K.take(mx, dst, axis=0)))  # :299-302
    ssum = K.segment_sum(ex, dst, n)  # :305-308
    alpha = K.divide(ex, K.add(K.take(ssum, dst, axis=0), 1e-10))  # :311
    msg = torch.unsqueeze(alpha, -1) * h_j  # :257-258
    aggr = K.segment_sum(msg.reshape(e, heads * C), dst, n).reshape(n, heads, C)  # :321-333
    out = aggr.reshape(n, heads * C) if concat else torch.mean(aggr, dim=1)  # :341-346
    return out + K.convert(bias) if bias is not None else out


# ---------------------------------------------------------------------------
# layers/pooling/global_pooling.py, utils/data_utils.py
# ---------------------------------------------------------------------------


def global_pooling(x, pooling: str = "mean") -> torch.Tensor:
    """GlobalPooling.call (global_pooling.py:66-92): ops.mean/max/sum over axis 0, keepdims."""
    x = K.convert(x)
    if pooling == "mean":
        return torch.mean(x, dim=0, keepdim=True)
    if pooling == "max":
        return torch.amax(x, dim=0, keepdim=True)
    return torch.sum(x, dim=0, keepdim=True)


def batch_global_pooling(x, batch, pooling: str = "mean") -> torch.Tensor:
    """BatchGlobalPooling.call (global_pooling.py:214-251)."""
    x = K.convert(x)
    batch = K.cast(batch, torch.int32)
    num_graphs = int(torch.max(batch)) + 1  # :231
    if pooling == "mean":  # :235-247
        pooled_sum = K.segment_sum(x, batch, num_graphs)
        ones = torch.ones_like(batch, dtype=x.dtype)
        counts = K.segment_sum(ones, batch, num_graphs)
        counts = torch.maximum(counts, torch.tensor(1.0, dtype=x.dtype))
        return pooled_sum / torch.unsqueeze(counts, 1)
    if pooling == "max":  # :249-250, no isinf guard
        return K.segment_max(x, batch, num_graphs)
    return K.segment_sum(x, batch, num_graphs)  # :252-253


def batch_graphs(graphs):
    """batch_graphs (data_utils.py:139-272) on numpy dicts {x, edge_index, [edge_attr], [y]}:
    returns dict with x, edge_index (shifted by node offsets), batch, edge_attr, y."""
    xs = [np.asarray(g["x"]) for g in graphs]
    total = sum(x.shape[0] for x in xs)
    out = {"x": np.concatenate(xs, 0), "batch": np.zeros(total, np.int32)}
    eis, off = [], 0
    for i, g in enumerate(graphs):
        n = xs[i].shape[0]
        out["batch"][off:off + n] = i  # :219-223
        ei = np.asarray(g["edge_index"])
        if ei.shape[1]:
            eis.append(ei + off)  # :226-230
        off += n
    out["edge_index"] = np.concatenate(eis, 1) if eis else np.zeros((2, 0), np.int32)
    if all(g.get("edge_attr") is not None for g in graphs):
        out["edge_attr"] = np.concatenate([g["edge_attr"] for g in graphs], 0)
    if all(g.get("y") is not None for g in graphs):
        ys = [np.asarray(g["y"]) for g in graphs]
        out["y"] = np.stack(ys, 0) if ys[0].ndim == 1 else np.concatenate(ys, 0)  # :245-252
    return out


# ---------------------------------------------------------------------------
# stable CSR by destination (integer parity of kgx_csr_build)
# ---------------------------------------------------------------------------


def csr_by_destination(src: np.ndarray, dst: np.ndarray, n_src: int, n_dst: int, self_loops: bool):
    """rowptr/col/eid/deg the kgx CSR must reproduce bit for bit.

    Order = the reference's accumulation order: input edge order within each
    destination (scatter_add is sequential), self loop i (id E+i) last
    (utils/main.py:15).  Negative src wrap (take); negative dst are dropped
    (segment_sum's extra bucket).  Raises IndexError like take() on OOB.
    """
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    E = src.shape[0]
    if np.any((src < -n_src) | (src >= n_src) | (dst < -n_dst) | (dst >= n_dst)):
        raise IndexError("index out of range in edge_index")
    src = np.where(src < 0, src + n_src, src)
    eid = np.arange(E, dtype=np.int64)
    if self_loops:
        loops = np.arange(n_dst, dtype=np.int64)
        src = np.concatenate([src, loops])
        dst = np.concatenate([dst, loops])
        eid = np.concatenate([eid, E + loops])
    keep = dst >= 0
    src, dst, eid = src[keep], dst[keep], eid[keep]
    order = np.argsort(dst, kind="stable")
    deg = np.bincount(dst, minlength=n_dst).astype(np.int64)
    rowptr = np.zeros(n_dst + 1, dtype=np.int64)
    np.cumsum(deg, out=rowptr[1:])
    return (rowptr.astype(np.int32), src[order].astype(np.int32), eid[order].astype(np.int32),
            deg.astype(np.int32))
