"""Keras-3 `keras.ops` as lowered by the torch backend, restated on ATen CPU.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference calls keras.ops.* (message_passing.py:3, aggregators.py:11-12,
utils/main.py:3-4); with KERAS_BACKEND=torch every call becomes the ATen ops
below.  Restated from Keras 3.x keras/src/backend/torch (Keras is absent from
this container; version unpinned, reference pyproject.toml:33 `keras>=3.0`).
"""

from __future__ import annotations

import torch

FLOATX = torch.float32


def convert(x, dtype=None) -> torch.Tensor:
    """convert_to_tensor: python float -> floatx, python int -> int32."""
    if isinstance(x, torch.Tensor):
        return x if dtype is None else x.to(dtype)
    if isinstance(x, bool):
        return torch.as_tensor(x, dtype=torch.bool)
    if isinstance(x, int) and dtype is None:
        return torch.as_tensor(x, dtype=torch.int32)
    if isinstance(x, float) and dtype is None:
        return torch.as_tensor(x, dtype=FLOATX)
    return torch.as_tensor(x, dtype=dtype)


def cast(x, dtype) -> torch.Tensor:
    return convert(x).to(dtype)


def segment_sum(data, segment_ids, num_segments: int) -> torch.Tensor:
    """keras.ops.segment_sum (torch backend math.segment_sum).

    ids are repeated to data's shape as int64, ids < 0 or >= num_segments are
    redirected to an extra bucket that is dropped, then
    zeros[n+1,...].scatter_add(0, ids, data.float())[:-1] cast back.
    scatter_add on CPU accumulates each output element in index order
    (probed: bit-identical to a sequential np.add.at loop).
    """
    data = convert(data)
    ids = convert(segment_ids)
    reps = int(torch.prod(torch.tensor(data.shape[1:]))) if data.dim() > 1 else 1
    ids = ids.long().repeat_interleave(reps).view(*data.shape)
    ids = torch.where(ids >= 0, ids, num_segments)
    ids = torch.where(ids < num_segments, ids, num_segments)
    shape = (num_segments + 1,) + tuple(data.shape[1:])
    out = torch.zeros(*shape).scatter_add(0, ids, data.float())[:-1]
    return out.to(data.dtype)


def segment_max(data, segment_ids, num_segments: int) -> torch.Tensor:
    """keras.ops.segment_max: -inf[n+1,...].scatter_reduce(0, ids, data, "amax")[:-1]."""
    data = convert(data)
    ids = convert(segment_ids)
    reps = int(torch.prod(torch.tensor(data.shape[1:]))) if data.dim() > 1 else 1
    ids = ids.long().repeat_interleave(reps).view(*data.shape)
    ids = torch.where(ids >= 0, ids, num_segments)
    ids = torch.where(ids < num_segments, ids, num_segments)
    shape = (num_segments + 1,) + tuple(data.shape[1:])
    out = torch.full(shape, -float("inf")).scatter_reduce(0, ids, data.float(), "amax")[:-1]
    return out.to(data.dtype)


def take(x, indices, axis: int = 0) -> torch.Tensor:
    """keras.ops.take: negative ids wrap; 2-D x / axis 0 -> embedding (raises on OOB)."""
    x = convert(x)
    idx = convert(indices).long()
    dim = x.shape[axis]
    idx = torch.where(idx < 0, idx + dim, idx)
    if x.dim() == 2 and axis == 0:
        return torch.nn.functional.embedding(idx, x)
    return torch.index_select(x, axis, idx)


def power(x1, x2) -> torch.Tensor:
    """keras.ops.power: both operands converted to tensors -> torch.pow(Tensor, Tensor).

    NOTE: with a 0-dim tensor exponent ATen uses the general (Sleef) powf, which
    differs from correctly-rounded x**-0.5 by 1 ulp for ~23% of inputs
    (probed in this container) — the reason GCN norms are tolerance-checked.
    """
    return torch.pow(convert(x1), convert(x2))


def add(a, b) -> torch.Tensor:
    return torch.add(convert(a), convert(b))


def multiply(a, b) -> torch.Tensor:
    return torch.mul(convert(a), convert(b))


def divide(a, b) -> torch.Tensor:
    return torch.div(convert(a), convert(b))


def maximum(a, b) -> torch.Tensor:
    return torch.maximum(convert(a), convert(b))


def where(c, a, b) -> torch.Tensor:
    return torch.where(convert(c), convert(a), convert(b))


def isinf(x) -> torch.Tensor:
    return torch.isinf(convert(x))


def leaky_relu(x, negative_slope: float) -> torch.Tensor:
    return torch.nn.functional.leaky_relu(convert(x), negative_slope=negative_slope)


def normalize_l2(x, axis: int = -1, epsilon: float = 1e-7) -> torch.Tensor:
    """keras.ops.normalize(x, axis, order=2) (Keras 3.x nn._normalize special case):
    x * minimum(rsqrt(sum(square(x))), 1/epsilon).  Parity unpinned: Keras version
    is unpinned by the reference and older 3.x releases divided by max(norm, eps)."""
    x = convert(x)
    square_sum = torch.sum(torch.square(x), dim=axis, keepdim=True)
    inv_norm = torch.minimum(torch.rsqrt(square_sum), torch.tensor(1.0 / epsilon))
    return x * inv_norm


def dense(x, kernel, bias=None, activation=None) -> torch.Tensor:
    """keras.layers.Dense.call: matmul(x, kernel) (+ bias) then activation."""
    y = torch.matmul(convert(x), convert(kernel))
    if bias is not None:
        y = torch.add(y, convert(bias))
    if activation == "relu":
        y = torch.relu(y)
    elif activation not in (None, "linear"):
        raise ValueError(f"oracle: unsupported activation {activation}")
    return y
