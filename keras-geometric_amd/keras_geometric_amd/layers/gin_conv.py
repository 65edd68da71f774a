"""GINConv (mirror of src/keras_geometric/layers/gin_conv.py).

h'_i = MLP((1+eps) * x_i + AGG_{j->i} x_j)   (gin_conv.py:216-225)

kgx forward: ONE fused kernel gathers x_j rows, reduces (sum/mean/max) in the
reference's edge order and applies the (1+eps)*x_i + aggr epilogue; the MLP's
Dense layers run on kgx_dense (bf16x3-split MFMA, f32-accurate; the library
fp32 GEMM only past its K/N <= 256 shapes).  When the MLP's first Dense fits a
fused kernel (F_in 128 -> <= 128 units: kgx_spmm_gemm; F_in 256 -> 256 units,
BASELINE config C4: kgx_spmm_gemm_f256; bias, none/ReLU), that Dense runs in the
aggregation's epilogue on MFMA too (KGX_FUSED_PRE_GIN), so the [N, F_in]
aggregate is never written; EXACT mode keeps the separate, bit-exact aggregation.
"""

from __future__ import annotations

from typing import Any

import numpy as np
import torch

from .. import _native as nat
from .. import ops as kops
from ._edges import edge_index_tensor, graph_for
from .base import Constant, Dense, Dropout, Sequential, to_device_tensor
from .message_passing import MessagePassing


class GINConv(MessagePassing):
    def __init__(
        self,
        output_dim: int,
        mlp_hidden: list[int] | None = None,
        aggregator: str = "sum",
        eps_init: float = 0.0,
        train_eps: bool = False,
        use_bias: bool = True,
        dropout: float = 0.0,
        kernel_initializer: str = "glorot_uniform",
        bias_initializer: str = "zeros",
        activation: str = "relu",
        **kwargs: Any,
    ) -> None:
        super().__init__(aggregator=aggregator, **kwargs)
        self.output_dim = output_dim
        self.mlp_hidden = list(mlp_hidden) if mlp_hidden is not None else []
        self.eps_init = eps_init
        self.train_eps = train_eps
        self.use_bias = use_bias
        self.dropout_rate = dropout
        self.kernel_initializer = kernel_initializer
        self.bias_initializer = bias_initializer
        self.activation = activation
        self.mlp = None
        self.eps = None
        if self.aggregator not in ["mean", "max", "sum"]:  # gin_conv.py:80-84
            raise ValueError(f"Invalid aggregator: {self.aggregator}. Must be one of ['mean', 'max', 'sum']")

    def build(self, input_shape: Any) -> None:
        node_shape = input_shape[0] if isinstance(input_shape, (list, tuple)) and len(input_shape) >= 1 \
            and isinstance(input_shape[0], (list, tuple)) else input_shape
        if node_shape is None or len(node_shape) < 2:
            raise ValueError(f"Expected node features shape (N, F), got {node_shape}")
        input_dim = node_shape[1]
        if input_dim is None:
            raise ValueError("Input feature dimension cannot be None")
        if self.train_eps:
            self.eps = self.add_weight((1,), Constant(self.eps_init), name="eps")
        else:
            self.eps = self.eps_init
        layers = []
        for i, hidden in enumerate(self.mlp_hidden):
            layers.append(Dense(hidden, activation=self.activation, use_bias=self.use_bias,
                                kernel_initializer=self.kernel_initializer,
                                bias_initializer=self.bias_initializer, name=f"mlp_hidden_{i}"))
            if self.dropout_rate > 0:
                layers.append(Dropout(self.dropout_rate))
        layers.append(Dense(self.output_dim, activation=None, use_bias=self.use_bias,
                            kernel_initializer=self.kernel_initializer,
                            bias_initializer=self.bias_initializer, name="mlp_output"))
        self.mlp = Sequential(layers, name="gin_mlp")
        self.mlp._build_device = getattr(self, "_build_device", None)
        self.mlp.build((None, input_dim))
        self.built = True

    def _scale(self) -> float:
        # (1 + eps) as the reference computes it: python float -> fp32 scalar, or
        # fp32 1 + eps_variable (gin_conv.py:217-222)
        if self.train_eps:
            return float((1 + self.eps.detach()).float().item())
        return float(np.float32(1 + self.eps_init))

    def update(self, aggregated, x=None):
        if x is None:
            raise ValueError("Original node features x are required for GIN update")
        if self.mlp is None:
            raise RuntimeError("MLP not initialized. Call build() first.")
        h = (1 + self.eps) * x + aggregated if self.train_eps else (1 + self.eps_init) * x + aggregated
        return self.mlp(h)

    def call(self, inputs, edge_attr=None, training=None):
        if not isinstance(inputs, (list, tuple)):
            raise ValueError("Inputs must be a list or tuple containing [x, edge_index]")
        if len(inputs) < 2:
            raise ValueError("Inputs must contain at least [x, edge_index]")
        x = to_device_tensor(inputs[0], torch.float32)
        edge_index = inputs[1]
        N = x.shape[0]
        if N == 0:
            return torch.zeros((0, self.output_dim), dtype=x.dtype, device=x.device)
        ei = edge_index_tensor(edge_index, x.device, allow_transpose=False)
        if ei.shape[1] == 0:  # gin_conv.py:269-280
            h = (1 + self.eps) * x if self.train_eps else (1 + self.eps_init) * x
            return self.mlp(h, training=training)
        g = graph_for(edge_index, ei, N, N, n_features=x.shape[1])
        if self.train_eps and torch.is_grad_enabled() and self.eps.requires_grad:
            # trainable eps: keep (1 + eps) in the autograd graph (gin_conv.py:216-225)
            h = (1 + self.eps) * x + kops.aggregate(g, x.contiguous(), self.aggregator, exact=self.exact)
            return self.mlp(h, training=training)
        first = self.mlp.layers[0]
        if (not self.exact and first.activation in (None, torch.relu)
                and kops.fused_transform_supported(x.shape[1], first.units)):
            # (1+eps) x + aggr -> the MLP's first Dense (bias, ReLU) in one fused launch
            h = kops.aggregate_transform(g, x.contiguous(), first.kernel, self.aggregator,
                                         bias=first.bias if first.use_bias else None, pre_gin=True,
                                         gin_scale=self._scale(), relu=first.activation is torch.relu)
            for layer in self.mlp.layers[1:]:
                h = layer(h, training=training) if isinstance(layer, Dropout) else layer(h)
            return h
        h = kops.aggregate(g, x.contiguous(), self.aggregator, epilogue=nat.EPI_GIN, xroot=x.contiguous(),
                           gin_scale=self._scale(), exact=self.exact)
        return self.mlp(h, training=training)

    def compute_output_shape(self, input_shape):
        x_shape = input_shape[0] if isinstance(input_shape, (list, tuple)) else input_shape
        return (x_shape[0], self.output_dim)

    def get_config(self) -> dict[str, Any]:
        config = super().get_config()
        config.update(
            {
                "output_dim": self.output_dim,
                "mlp_hidden": self.mlp_hidden,
                "eps_init": float(self.eps_init),
                "train_eps": self.train_eps,
                "use_bias": self.use_bias,
                "dropout": self.dropout_rate,
                "kernel_initializer": self.kernel_initializer,
                "bias_initializer": self.bias_initializer,
                "activation": self.activation,
            }
        )
        return config
