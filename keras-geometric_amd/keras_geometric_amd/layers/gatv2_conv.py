"""GATv2Conv (mirror of src/keras_geometric/layers/gatv2_conv.py).

h = x @ W (one shared Dense, no bias; gatv2_conv.py:95-101, 224-239), then ONE
fused kgx kernel per layer: per-edge score a . leaky_relu(h_i + h_j), segment
softmax by target, alpha-weighted sum of h_j, + bias (concat) — instead of the
reference's 4 gathers, 3 segment ops and E x H x C intermediates
(gatv2_conv.py:241-352).
"""

from __future__ import annotations

from typing import Any

import torch

from .. import ops as kops
from ._edges import edge_index_tensor, graph_for
from .base import Dense, to_device_tensor
from .message_passing import MessagePassing


class GATv2Conv(MessagePassing):
    def __init__(
        self,
        output_dim: int,
        heads: int = 1,
        concat: bool = True,
        negative_slope: float = 0.2,
        dropout: float = 0.0,
        use_bias: bool = True,
        kernel_initializer: str = "glorot_uniform",
        bias_initializer: str = "zeros",
        att_initializer: str = "glorot_uniform",
        add_self_loops: bool = True,
        **kwargs,
    ) -> None:
        super().__init__(aggregator="sum", **kwargs)
        self.output_dim = output_dim
        self.heads = heads
        self.concat = concat
        self.negative_slope = negative_slope
        self.dropout_rate = dropout
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        self.bias_initializer = bias_initializer
        self.att_initializer = att_initializer
        self.add_self_loops_flag = add_self_loops
        self.features_per_head = output_dim
        self.linear_transform: Dense | None = None
        self.att = None
        self.bias = None

    def build(self, input_shape) -> None:
        shape = input_shape[0] if isinstance(input_shape, list) and len(input_shape) >= 1 else input_shape
        shape = tuple(shape) if shape is not None else None
        if shape is None or len(shape) != 2:
            raise ValueError(f"Expected features input shape like (N, F), but got {shape}")
        if shape[1] is None:
            raise ValueError("Input feature dimension cannot be None.")
        self.linear_transform = Dense(self.heads * self.features_per_head, use_bias=False,
                                      kernel_initializer=self.kernel_initializer, name="linear_transform")
        self.linear_transform._build_device = getattr(self, "_build_device", None)
        self.linear_transform.build((None, shape[1]))
        self.att = self.add_weight((1, self.heads, self.features_per_head), self.att_initializer, name="att")
        if self.use_bias:
            n = self.heads * self.features_per_head if self.concat else self.features_per_head
            self.bias = self.add_weight((n,), self.bias_initializer, name="final_bias")
        self.built = True

    def _out_dim(self) -> int:
        return self.heads * self.features_per_head if self.concat else self.features_per_head

    def call(self, inputs, edge_attr=None, training=None):
        if isinstance(inputs, (list, tuple)) and len(inputs) >= 2:
            x, edge_index = inputs[0], inputs[1]
        else:
            raise ValueError(f"Expected inputs to be [x, edge_index], got {inputs}")
        if isinstance(x, (list, tuple)):
            x_i = to_device_tensor(x[0], torch.float32)
            x_j = to_device_tensor(x[1], torch.float32, x_i.device)
        else:
            x_i = x_j = to_device_tensor(x, torch.float32)
        ei = edge_index_tensor(edge_index, x_i.device, allow_transpose=False)
        return self._gatv2_propagate(x_i, x_j, ei, edge_index, training=training)

    def propagate(self, x, edge_index, edge_attr=None, size=None, **kwargs):
        if isinstance(x, (list, tuple)):
            x_i = to_device_tensor(x[0], torch.float32)
            x_j = to_device_tensor(x[1], torch.float32, x_i.device)
        else:
            x_i = x_j = to_device_tensor(x, torch.float32)
        ei = edge_index_tensor(edge_index, x_i.device, allow_transpose=False)
        return self._gatv2_propagate(x_i, x_j, ei, edge_index, self_loops=False)

    def _gatv2_propagate(self, x_i, x_j, ei, edge_index_obj, self_loops: bool | None = None, training=None):
        n, n_src = x_i.shape[0], x_j.shape[0]
        loops = self.add_self_loops_flag if self_loops is None else self_loops
        if loops and x_i is not x_j:
            raise ValueError("GATv2Conv: add_self_loops requires a non-bipartite graph")
        if n == 0:
            return torch.zeros((0, self._out_dim()), dtype=x_i.dtype, device=x_i.device)
        e = ei.shape[1] + (n if loops else 0)
        if e == 0:  # gatv2_conv.py:204-210 (no bias)
            return torch.zeros((n, self._out_dim()), dtype=x_i.dtype, device=x_i.device)
        H, C = self.heads, self.features_per_head
        h_dst = self.linear_transform(x_i).contiguous()
        h_src = h_dst if x_j is x_i else self.linear_transform(x_j).contiguous()
        g = graph_for(edge_index_obj, ei, n_src, n, self_loops=loops, n_features=H * C)
        use_b = self.use_bias and self.bias is not None
        drop = bool(training) and self.dropout_rate > 0  # attention dropout, gatv2_conv.py:252-253
        out = kops.gatv2_aggregate(g, h_src, h_dst, self.att, H, C, self.negative_slope,
                                   bias=self.bias if (use_b and self.concat) else None, exact=self.exact,
                                   dropout=self.dropout_rate if drop else 0.0,
                                   seed=int(torch.randint(0, 2**62, (1,)).item()) if drop else 0)
        if not self.concat:
            out = out.view(n, H, C).mean(dim=1)
            if use_b:
                out = out + self.bias
        return out

    def message(self, x_i, x_j, edge_attr=None, edge_index=None, size=None, **kwargs):
        return x_j

    def get_config(self) -> dict[str, Any]:
        config = super().get_config()
        config.update(
            {
                "output_dim": self.output_dim,
                "heads": self.heads,
                "concat": self.concat,
                "negative_slope": self.negative_slope,
                "dropout": self.dropout_rate,
                "use_bias": self.use_bias,
                "kernel_initializer": self.kernel_initializer,
                "bias_initializer": self.bias_initializer,
                "att_initializer": self.att_initializer,
                "add_self_loops": self.add_self_loops_flag,
            }
        )
        return config

    @classmethod
    def from_config(cls, config: dict[str, Any]) -> "GATv2Conv":
        config = dict(config)
        config.pop("aggregator", None)
        return cls(**config)
