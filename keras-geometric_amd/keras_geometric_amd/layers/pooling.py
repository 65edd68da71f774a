"""Graph-level readout (mirror of src/keras_geometric/layers/pooling/global_pooling.py).

GlobalPooling (global_pooling.py:9-143) reduces all rows of one graph
(`ops.mean/max/sum(axis=0, keepdims=True)`): a dense column reduction, done
by torch's reduction kernels.  BatchGlobalPooling (:146-316) is the segment
reduction of SURVEY.md §8f row 2: per graph of a batch, over a `batch` vector
of graph ids (:228-249) -- the propagate engine's own primitive.  Here the
batch vector becomes a segment CSR once (kgx_csr_build, cached on the batch
tensor) and the pooling is one kgx_spmm launch:
  sum  -> segment_sum;  mean -> segment_sum / max(count, 1) (the division is
  the MEAN reduce's: for an integer count the two guards agree);
  max  -> segment_max WITHOUT the aggregators' isinf guard (KGX_EPI_RAW):
  an empty graph pools to -inf, as keras.ops.segment_max does.
Differentiable through ops.aggregate's autograd.  AttentionPooling / Set2Set
(attention_pooling.py) are dense per-graph MLP/LSTM readouts outside the
propagate path and are not provided.
"""

from __future__ import annotations

from typing import Any

import torch

from .. import _native as nat
from .. import graph as G
from .. import ops as kops
from .base import Layer, to_device_tensor

_POOLINGS = ("mean", "max", "sum")


def _check_pooling(pooling: str) -> None:
    if pooling not in _POOLINGS:
        raise ValueError(f"pooling must be one of ['mean', 'max', 'sum'], got {pooling}")


class GlobalPooling(Layer):
    """Pool all nodes of one graph into a [1, F] row (global_pooling.py:9-143)."""

    def __init__(self, pooling: str = "mean", **kwargs: Any) -> None:
        super().__init__(**kwargs)
        _check_pooling(pooling)
        self.pooling = pooling

    def call(self, inputs, **kwargs):
        x = to_device_tensor(inputs, torch.float32)
        if self.pooling == "mean":
            return torch.mean(x, dim=0, keepdim=True)
        if self.pooling == "max":
            return torch.amax(x, dim=0, keepdim=True)
        return torch.sum(x, dim=0, keepdim=True)

    def compute_output_shape(self, input_shape):
        if len(input_shape) != 2:
            raise ValueError(
                f"Expected input shape to be 2D (num_nodes, num_features), got {len(input_shape)}D"
            )
        return (1, input_shape[1])

    def get_config(self) -> dict[str, Any]:
        config = super().get_config()
        config.update({"pooling": self.pooling})
        return config

    @classmethod
    def from_config(cls, config: dict[str, Any]) -> "GlobalPooling":
        return cls(**config)


def segment_graph(batch: torch.Tensor, num_graphs: int) -> G.CSRGraph:
    """Segment CSR of a batch vector (row g = the nodes of graph g, in node
    order -- the order segment_sum's scatter accumulates in), cached on the
    batch tensor like an edge_index."""
    n = int(batch.numel())
    b32 = batch if batch.dtype == torch.int32 else batch.to(torch.int32)
    key = G.cache_key(batch, "segments", num_graphs)

    def build():
        src = torch.arange(n, dtype=torch.int32, device=batch.device)
        return G.build_csr(src, b32.contiguous(), n, num_graphs, segment_only=True)

    return G.cached(key, batch, build)


class BatchGlobalPooling(Layer):
    """Per-graph pooling of a batch of graphs (global_pooling.py:146-316)."""

    def __init__(self, pooling: str = "mean", **kwargs: Any) -> None:
        super().__init__(**kwargs)
        _check_pooling(pooling)
        self.pooling = pooling

    def call(self, inputs, **kwargs):
        if not isinstance(inputs, (list, tuple)) or len(inputs) != 2:
            raise ValueError(
                "inputs must be a list/tuple of [node_features, batch], "
                f"got {type(inputs)} with length {len(inputs) if hasattr(inputs, '__len__') else 'unknown'}"
            )
        x = to_device_tensor(inputs[0], torch.float32)
        batch = to_device_tensor(inputs[1], torch.int32, x.device)
        num_graphs = int(batch.max()) + 1  # :231, ops.max(batch) + 1
        g = segment_graph(batch, num_graphs)
        if self.pooling == "max":
            return kops.aggregate(g, x.contiguous(), "max", epilogue=nat.EPI_RAW, exact=True)
        return kops.aggregate(g, x.contiguous(), self.pooling, exact=True)

    def compute_output_shape(self, input_shape):
        if not isinstance(input_shape, (list, tuple)) or len(input_shape) != 2:
            raise ValueError("input_shape must be a list/tuple of 2 shapes for [node_features, batch]")
        node_features_shape, batch_shape = input_shape
        if isinstance(node_features_shape, int):
            raise ValueError(
                "input_shape must be a list/tuple of 2 shapes for [node_features, batch], "
                f"got single shape {input_shape}"
            )
        if len(node_features_shape) != 2:
            raise ValueError(
                f"Expected node_features shape to be 2D (total_nodes, num_features), got {len(node_features_shape)}D"
            )
        if len(batch_shape) != 1:
            raise ValueError(f"Expected batch shape to be 1D (total_nodes,), got {len(batch_shape)}D")
        return (None, node_features_shape[1])

    def get_config(self) -> dict[str, Any]:
        config = super().get_config()
        config.update({"pooling": self.pooling})
        return config

    @classmethod
    def from_config(cls, config: dict[str, Any]) -> "BatchGlobalPooling":
        return cls(**config)
