"""MessagePassing base layer (mirror of src/keras_geometric/layers/message_passing.py).

Template method `propagate` with overridable `message / pre_aggregate /
aggregate / update / post_update` hooks, exactly as in the reference
(message_passing.py:47-220).  When a subclass keeps the default message
(x_j), pre_aggregate and aggregate, propagate runs as ONE fused kgx kernel
(gather of x_j rows straight into the segment reduction, never materialising
the [E,F] x_j / x_i gathers of message_passing.py:195-196).  Otherwise the
user hooks run on GPU tensors and the reduction still goes through the kgx
segment kernel.
"""

from __future__ import annotations

from typing import Any

import torch

from .. import ops as kops
from ..graph import CSRGraph, exact_mode_default
from ._edges import edge_index_tensor, graph_for
from .aggregators import Aggregator, AggregatorFactory
from .base import Layer, to_device_tensor


class MessagePassing(Layer):
    def __init__(self, aggregator: str = "mean", exact: bool | None = None, **kwargs) -> None:
        super().__init__(**kwargs)
        self.aggregator_name: str = aggregator
        self._aggregator: Aggregator = AggregatorFactory.create(aggregator)
        self.aggregator: str = aggregator
        self.supported_aggregators: list[str] = AggregatorFactory.get_available_aggregators()
        # cache of the int32 edge_index (message_passing.py:41-42, 256-268)
        self._cached_edge_idx: torch.Tensor | None = None
        self._cached_edge_idx_hash: int | None = None
        self.message_kwargs: dict[str, Any] = {}
        # EXACT: reduce every row sequentially in CSR order (no hub split);
        # bit-identical to the reference for identical messages.
        self.exact = exact_mode_default() if exact is None else bool(exact)

    # -- hooks (message_passing.py:47-145) -----------------------------------
    def message(self, x_i, x_j, edge_attr=None, edge_index=None, size=None, **kwargs):
        if edge_attr is not None:
            return torch.cat([x_j, edge_attr], dim=-1)
        return x_j

    def aggregate(self, messages, target_idx, num_nodes: int, dim_size: int | None = None, *,
                  graph: CSRGraph | None = None):
        if dim_size is None:
            dim_size = num_nodes
        return self._aggregator.aggregate(messages, target_idx, dim_size, graph=graph, exact=self.exact)

    def update(self, aggregated, x=None):
        return aggregated

    def pre_aggregate(self, messages):
        return messages

    def post_update(self, x, x_updated):
        return x_updated

    def _fusable(self) -> bool:
        cls = type(self)
        return (
            cls.message is MessagePassing.message
            and cls.pre_aggregate is MessagePassing.pre_aggregate
            and cls.aggregate is MessagePassing.aggregate
        )

    # -- propagate (message_passing.py:147-220) --------------------------------
    def propagate(self, x, edge_index, edge_attr=None, size=None, **kwargs):
        if isinstance(x, (list, tuple)):
            x_i = to_device_tensor(x[0], torch.float32)
            x_j = to_device_tensor(x[1], torch.float32, x_i.device)
        else:
            x_i = x_j = to_device_tensor(x, torch.float32)
        n_dst, n_src = x_i.shape[0], x_j.shape[0]
        if n_dst == 0:  # :180-182
            feature_dim = x_i.shape[1] if x_i.dim() > 1 else 1
            return torch.zeros((0, feature_dim), dtype=x_i.dtype, device=x_i.device)
        ei = edge_index_tensor(edge_index, x_i.device, allow_transpose=False)
        if ei.shape[1] == 0:  # :185-188
            return torch.zeros((n_dst, x_i.shape[1]), dtype=x_i.dtype, device=x_i.device)
        g = graph_for(edge_index, ei, n_src, n_dst, n_features=x_j.shape[1])

        if edge_attr is None and self._fusable():
            aggregated = kops.aggregate(g, x_j.contiguous(), self._aggregator.reduce, exact=self.exact)
        else:
            # generic path: user hooks on per-edge tensors (indices validated by the CSR build)
            src = ei[0].long()
            dst = ei[1].long()
            src = torch.where(src < 0, src + n_src, src)
            dst_g = torch.where(dst < 0, dst + n_dst, dst)
            x_j_g = x_j.index_select(0, src)
            x_i_g = x_i.index_select(0, dst_g)
            if edge_attr is not None:
                edge_attr = to_device_tensor(edge_attr, torch.float32, x_i.device)
            messages = self.message(x_i_g, x_j_g, edge_attr=edge_attr, edge_index=ei, size=(n_dst, n_src), **kwargs)
            messages = self.pre_aggregate(messages)
            if type(self).aggregate is MessagePassing.aggregate:
                aggregated = self.aggregate(messages, ei[1], n_dst, dim_size=n_dst, graph=g)
            else:
                aggregated = self.aggregate(messages, ei[1], n_dst, dim_size=n_dst)
        updated = self.update(aggregated, x=x_i)
        return self.post_update(x_i, updated)

    # -- call (message_passing.py:223-275) ---------------------------------------
    def call(self, inputs, edge_attr=None, training=None):
        if not isinstance(inputs, (list, tuple)):
            raise ValueError("Inputs must be a list or tuple containing [x, edge_index]")
        if len(inputs) < 2:
            raise ValueError("Inputs must contain at least [x, edge_index]")
        x, edge_index = inputs[0], inputs[1]
        if len(inputs) >= 3 and inputs[2] is not None:
            edge_attr = inputs[2]
        h = id(edge_index)
        if self._cached_edge_idx is None or self._cached_edge_idx_hash != h:
            dev = x.device if isinstance(x, torch.Tensor) and x.device.type == "cuda" else None
            self._cached_edge_idx = edge_index_tensor(edge_index, dev, allow_transpose=False)
            self._cached_edge_idx_hash = h
        self.message_kwargs = {}
        # the CSR cache keys on the caller's tensor; numpy input uses the cast copy
        ei = edge_index if isinstance(edge_index, torch.Tensor) else self._cached_edge_idx
        return self.propagate(x=x, edge_index=ei, edge_attr=edge_attr, training=training)

    def forward(self, inputs, *args, **kwargs):
        if not isinstance(inputs, (list, tuple)):
            return self.call(inputs, *args, **kwargs)  # raises the reference ValueError
        return super().forward(inputs, *args, **kwargs)

    def compute_output_shape(self, input_shape):
        return input_shape[0] if isinstance(input_shape, (list, tuple)) else input_shape

    def get_config(self) -> dict[str, Any]:
        config = super().get_config()
        config.update({"aggregator": self.aggregator})
        return config
