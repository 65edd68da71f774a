"""GCNConv (mirror of src/keras_geometric/layers/gcn_conv.py).

Reference forward (gcn_conv.py:275-364): add self loops, norm_e =
dinv[dst]*dinv[src], per-EDGE matmul x_j @ W (:233-235), * norm (:246),
segment_sum (:79 forces "sum"), + bias (:266-272).

kgx forward (default): ONE fused kernel out = bias + (sum_e w_e x[col_e]) W
(aggregate-then-transform, kgx_spmm_gemm).  EXACT mode / other shapes:
H = x @ W once per NODE, then out_i = bias + sum_{e in CSR row i} H[col_e] * w_e
in the reference's edge order.  Training with dropout_rate > 0: the same
unfused order with every message element of H[col_e] dropped/scaled by a
counter-based mask of (seed, edge, column) before the * norm (gcn_conv.py:237-242).
"""

from __future__ import annotations

from typing import Any

import torch

from .. import _native as nat
from .. import ops as kops
from ._edges import edge_index_tensor, graph_for
from .base import get_initializer, serialize_initializer, to_device_tensor
from .message_passing import MessagePassing


class GCNConv(MessagePassing):
    def __init__(
        self,
        output_dim: int,
        use_bias: bool = True,
        kernel_initializer="glorot_uniform",
        bias_initializer="zeros",
        kernel_regularizer=None,
        bias_regularizer=None,
        kernel_constraint=None,
        bias_constraint=None,
        add_self_loops: bool = True,
        normalize: bool = True,
        dropout_rate: float = 0.0,
        **kwargs: Any,
    ) -> None:
        kwargs["aggregator"] = "sum"  # gcn_conv.py:79
        super().__init__(**kwargs)
        self.output_dim = output_dim
        self.use_bias = use_bias
        self.add_self_loops = add_self_loops
        self.normalize = normalize
        self.dropout_rate = dropout_rate
        self.kernel_initializer = get_initializer(kernel_initializer)
        self.bias_initializer = get_initializer(bias_initializer)
        self.kernel_regularizer = kernel_regularizer
        self.bias_regularizer = bias_regularizer
        self.kernel_constraint = kernel_constraint
        self.bias_constraint = bias_constraint
        self.kernel = None
        self.bias = None

    def build(self, input_shape) -> None:
        if input_shape is None:
            return
        if not isinstance(input_shape, (list, tuple)) or len(input_shape) < 2:
            raise ValueError(
                "Expected input_shape to be a list/tuple with at least 2 elements "
                f"[(node_features_shape), (edge_index_shape)], but got {input_shape}"
            )
        node_shape = input_shape[0]
        if node_shape is None or len(node_shape) < 2:
            raise ValueError(f"Expected node features shape to be (N, F), but got {node_shape}")
        input_dim = node_shape[-1]
        if input_dim is None or input_dim <= 0:
            raise ValueError(f"Input dimension must be a positive integer, but got {input_dim}")
        self.kernel = self.add_weight((input_dim, self.output_dim), self.kernel_initializer, name="kernel")
        self.bias = self.add_weight((self.output_dim,), self.bias_initializer, name="bias") if self.use_bias else None
        self.built = True

    def compute_output_shape(self, input_shape) -> tuple:
        node_shape = input_shape[0] if isinstance(input_shape, (list, tuple)) and input_shape else None
        return (node_shape[0] if node_shape else None, self.output_dim)

    def message(self, x_i, x_j, edge_attr=None, edge_index=None, size=None, **kwargs):
        """Per-edge message (gcn_conv.py:208-250); only used by an explicit propagate()."""
        x_j_transformed = torch.matmul(x_j, self.kernel)
        if edge_attr is not None:
            return x_j_transformed * edge_attr.unsqueeze(1)
        return x_j_transformed

    def update(self, aggregated, x=None):
        if self.use_bias and self.bias is not None:
            return aggregated + self.bias
        return aggregated

    def call(self, inputs, training=None, mask=None):
        if not isinstance(inputs, (list, tuple)) or len(inputs) < 2:
            raise ValueError("GCNConv expects inputs to be a list/tuple of [node_features, edge_index]")
        x = to_device_tensor(inputs[0], torch.float32)
        edge_index = inputs[1]
        ei = edge_index_tensor(edge_index, x.device, allow_transpose=True)
        N = x.shape[0]
        if N == 0:
            return torch.zeros((0, self.output_dim), dtype=x.dtype, device=x.device)
        drop = bool(training) and self.dropout_rate > 0  # gcn_conv.py:237-242
        n_edges = ei.shape[1] + (N if self.add_self_loops else 0)
        if n_edges == 0:  # gcn_conv.py:332-347
            out = torch.matmul(x, self.kernel)
            return out + self.bias if (self.use_bias and self.bias is not None) else out
        g = graph_for(edge_index, ei, N, N, self_loops=self.add_self_loops, gcn_norm=self.normalize,
                      n_features=self.output_dim)
        use_b = self.use_bias and self.bias is not None
        if drop:  # per-message dropout of x_j W: the unfused order (H = x W, then masked messages)
            h = torch.matmul(x, self.kernel)
            return kops.aggregate(
                g, h, "sum", weighted=self.normalize,
                epilogue=nat.EPI_BIAS if use_b else nat.EPI_NONE, bias=self.bias if use_b else None,
                exact=self.exact, dropout=self.dropout_rate, seed=int(torch.randint(0, 2**62, (1,)).item()),
            )
        if not self.exact and kops.fused_transform_supported(x.shape[1], self.output_dim):
            # aggregate-then-transform in one launch (W on f32 MFMA in the epilogue)
            return kops.aggregate_transform(g, x.contiguous(), self.kernel, "sum", weighted=self.normalize,
                                            bias=self.bias if use_b else None)
        h = kops.dense(x, self.kernel)  # node-level X W (kgx_dense on MFMA; library GEMM past 256)
        return kops.aggregate(
            g, h, "sum", weighted=self.normalize,
            epilogue=nat.EPI_BIAS if use_b else nat.EPI_NONE, bias=self.bias if use_b else None,
            exact=self.exact,
        )

    def get_config(self) -> dict[str, Any]:
        config = super().get_config()
        config.update(
            {
                "output_dim": self.output_dim,
                "use_bias": self.use_bias,
                "kernel_initializer": serialize_initializer(self.kernel_initializer),
                "bias_initializer": serialize_initializer(self.bias_initializer),
                "kernel_regularizer": self.kernel_regularizer,
                "bias_regularizer": self.bias_regularizer,
                "kernel_constraint": self.kernel_constraint,
                "bias_constraint": self.bias_constraint,
                "add_self_loops": self.add_self_loops,
                "normalize": self.normalize,
                "dropout_rate": self.dropout_rate,
            }
        )
        return config

    @classmethod
    def from_config(cls, config: dict[str, Any]) -> "GCNConv":
        config = dict(config)
        config.pop("aggregator", None)  # gcn_conv.py:424
        return cls(**config)
