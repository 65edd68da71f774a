"""SAGEConv (mirror of src/keras_geometric/layers/sage_conv.py).

out = act(lin_self(x) + lin_neigh(AGG_{j->i} m_j) + b), optional L2 normalize
(sage_conv.py:351-439).  m_j = x_j, or pool_mlp(x_j) for aggregator="pooling"
(PoolingAggregator, aggregators.py:254-274).  pool_mlp is row-wise, so it is
applied once per NODE and the kgx kernel gathers its rows (same values as the
reference's per-edge application).
"""

from __future__ import annotations

from typing import Any

import torch

from .. import ops as kops
from ._edges import edge_index_tensor, graph_for
from .base import Dense, get_activation, get_initializer, serialize_activation, serialize_initializer, \
    to_device_tensor
from .message_passing import MessagePassing

_VALID = ["mean", "max", "sum", "min", "std", "pooling"]


def l2_normalize(x: torch.Tensor, epsilon: float = 1e-7) -> torch.Tensor:
    """keras.ops.normalize(x, axis=-1, order=2): x * min(rsqrt(sum(x^2)), 1/eps)."""
    square_sum = torch.sum(torch.square(x), dim=-1, keepdim=True)
    inv_norm = torch.minimum(torch.rsqrt(square_sum), torch.tensor(1.0 / epsilon, device=x.device))
    return x * inv_norm


class SAGEConv(MessagePassing):
    def __init__(
        self,
        output_dim: int,
        aggregator: str = "mean",
        normalize: bool = False,
        root_weight: bool = True,
        use_bias: bool = True,
        activation: str | None = "relu",
        pool_activation: str | None = "relu",
        pool_hidden_dim: int | None = None,
        kernel_initializer="glorot_uniform",
        bias_initializer="zeros",
        kernel_regularizer=None,
        bias_regularizer=None,
        kernel_constraint=None,
        bias_constraint=None,
        dropout_rate: float = 0.0,
        **kwargs: Any,
    ) -> None:
        if aggregator not in _VALID:  # sage_conv.py:99-103
            raise ValueError(f"Invalid aggregator '{aggregator}'. Must be one of {_VALID}")
        super().__init__(aggregator="mean" if aggregator == "pooling" else aggregator, **kwargs)
        self.actual_aggregator = aggregator
        self.output_dim = output_dim
        self.normalize = normalize
        self.root_weight = root_weight
        self.use_bias = use_bias
        self.pool_hidden_dim = pool_hidden_dim
        self.dropout_rate = dropout_rate
        self.activation = get_activation(activation)
        self.pool_activation = get_activation(pool_activation)
        self.kernel_initializer = get_initializer(kernel_initializer)
        self.bias_initializer = get_initializer(bias_initializer)
        self.kernel_regularizer = kernel_regularizer
        self.bias_regularizer = bias_regularizer
        self.kernel_constraint = kernel_constraint
        self.bias_constraint = bias_constraint
        self.lin_neigh = None
        self.lin_self = None
        self.pool_mlp = None
        self.bias = None

    def build(self, input_shape) -> None:
        if input_shape is None:
            return
        if not isinstance(input_shape, (list, tuple)) or len(input_shape) < 2:
            raise ValueError(f"Expected input_shape to be [(N, F), (2, E)], got {input_shape}")
        node_shape = input_shape[0]
        if node_shape is None or len(node_shape) < 2:
            raise ValueError(f"Expected node shape (N, F), got {node_shape}")
        input_dim = node_shape[-1]
        if input_dim is None or input_dim <= 0:
            raise ValueError(f"Input dimension must be positive, got {input_dim}")
        dev = getattr(self, "_build_device", None)
        if self.actual_aggregator == "pooling":
            self.pool_mlp = Dense(self.pool_hidden_dim or input_dim, activation=self.pool_activation,
                                  use_bias=self.use_bias, kernel_initializer=self.kernel_initializer,
                                  bias_initializer=self.bias_initializer, name="pool_mlp")
            self.pool_mlp._build_device = dev
            self.pool_mlp.build((None, input_dim))
        self.lin_neigh = Dense(self.output_dim, use_bias=False, kernel_initializer=self.kernel_initializer,
                               name="linear_neigh")
        self.lin_neigh._build_device = dev
        neigh_dim = (self.pool_hidden_dim or input_dim) if self.actual_aggregator == "pooling" else input_dim
        self.lin_neigh.build((None, neigh_dim))
        if self.root_weight:
            self.lin_self = Dense(self.output_dim, use_bias=False, kernel_initializer=self.kernel_initializer,
                                  name="linear_self")
            self.lin_self._build_device = dev
            self.lin_self.build((None, input_dim))
        if self.use_bias:
            self.bias = self.add_weight((self.output_dim,), self.bias_initializer, name="bias")
        self.built = True

    def compute_output_shape(self, input_shape) -> tuple:
        node_shape = input_shape[0] if isinstance(input_shape, (list, tuple)) and input_shape else None
        return (node_shape[0] if node_shape else None, self.output_dim)

    def aggregate_neighbors(self, x, edge_index, num_nodes, training=None, *, edge_index_obj=None):
        """sage_conv.py:300-348 as one fused kgx reduction over gathered rows."""
        if edge_index.shape[1] == 0:
            feat = self.pool_mlp.units if (self.actual_aggregator == "pooling" and self.pool_mlp) else x.shape[1]
            return torch.zeros((num_nodes, feat), dtype=x.dtype, device=x.device)
        g = graph_for(edge_index_obj if edge_index_obj is not None else edge_index, edge_index,
                      x.shape[0], num_nodes, n_features=x.shape[1])
        if training and self.dropout_rate > 0:
            return self._aggregate_dropped(x, edge_index, g)
        if self.actual_aggregator == "pooling":
            return kops.aggregate(g, self.pool_mlp(x).contiguous(), "max", exact=self.exact)
        return kops.aggregate(g, x.contiguous(), self.actual_aggregator, exact=self.exact)

    def _aggregate_dropped(self, x, edge_index, g):
        """Training-mode message dropout (sage_conv.py:280-298): every message
        x_j (and, for 'pooling', the pool MLP's input) is its own masked copy,
        so the messages are materialised per input edge -- x[src_e] times the
        counter-based kgx mask of (seed, input edge id, column), 0 or 1/(1-p)
        like keras Dropout -- and reduced by edge (idx = eid), with autograd
        through the mask multiply and the reduction.  Keras' own RNG cannot be
        matched bit for bit; the arithmetic given the mask is (tests/test_gpu_dropout.py)."""
        n_src, E = x.shape[0], edge_index.shape[1]
        src = edge_index[0].long()
        src = torch.where(src < 0, src + n_src, src)  # take() wrap; out-of-range ids were rejected by graph_for
        seed = int(torch.randint(0, 2**62, (1,)).item())
        keys = torch.arange(E, dtype=torch.int32, device=x.device)
        msg = x.index_select(0, src) * kops.dropout_mask(seed, self.dropout_rate, keys, x.shape[1])
        reduce = self.actual_aggregator
        if reduce == "pooling":
            msg, reduce = self.pool_mlp(msg), "max"
        return kops.aggregate(g, msg.contiguous(), reduce, by_edge=True, exact=self.exact)

    def call(self, inputs, training=None, mask=None):
        if not isinstance(inputs, (list, tuple)) or len(inputs) < 2:
            raise ValueError("SAGEConv expects inputs to be a list/tuple of [node_features, edge_index]")
        x = to_device_tensor(inputs[0], torch.float32)
        edge_index = inputs[1]
        ei = edge_index_tensor(edge_index, x.device, allow_transpose=True)
        num_nodes = x.shape[0]
        out = self._call_fused(x, ei, edge_index, training)
        if out is not None:
            return out
        aggregated = self.aggregate_neighbors(x, ei, num_nodes, training=training, edge_index_obj=edge_index)
        return self.update_nodes(x, aggregated)

    def _call_fused(self, x, ei, edge_index_obj, training):
        """Inference with root_weight and a mean / sum / max aggregator: the
        neighbour map fused into the aggregation (sage_conv.py:404-433 in two
        launches): out = b + x W_self (kgx_dense), then kgx_spmm_gemm gathers,
        reduces, multiplies by W_neigh and adds into out in its store (relu
        there too), so the [N, F_in] aggregate is never written or re-read.
        Same terms as the reference, summed as (b + x W_self) + aggr W_neigh
        instead of (x W_self + aggr W_neigh) + b (tolerance-checked).  None
        when the shapes or the mode need the two-step path."""
        use_b = self.use_bias and self.bias is not None
        if (not self.root_weight or self.lin_self is None or self.exact or not x.is_cuda
                or self.actual_aggregator not in ("mean", "sum", "max") or ei.shape[1] == 0
                or (training and self.dropout_rate > 0)
                or not kops.fused_sage_supported(x.shape[1], self.output_dim)):
            return None
        W_self, W_neigh = self.lin_self.kernel, self.lin_neigh.kernel
        b = self.bias if use_b else None
        if kops._needs_grad(x, W_self, W_neigh, b):
            return None
        g = graph_for(edge_index_obj, ei, x.shape[0], x.shape[0], n_features=x.shape[1])
        relu = self.activation is torch.relu
        out = kops.dense(x, W_self, b)
        kops.aggregate_transform(g, x.contiguous(), W_neigh, self.actual_aggregator, out=out, relu=relu)
        if self.activation is not None and not relu:
            out = self.activation(out)
        if self.normalize:
            out = l2_normalize(out)
        return out

    def update_nodes(self, x, aggregated):
        """lin_neigh(aggr) + lin_self(x) + bias, activation, L2 norm (sage_conv.py:409-439);
        also the update step of distributed.ShardedSAGEConv on a shard's rows."""
        use_b = self.use_bias and self.bias is not None
        relu = self.activation is torch.relu
        if self.root_weight and self.lin_self is not None:
            # ONE kgx_dense pass: relu?(b + x W_self + aggr W_neigh), reading x and aggr once
            out = kops.dense(x, self.lin_self.kernel, self.bias if use_b else None,
                             x1=aggregated, W1=self.lin_neigh.kernel, relu=relu)
        else:
            out = kops.dense(aggregated, self.lin_neigh.kernel, self.bias if use_b else None, relu=relu)
        if self.activation is not None and not relu:
            out = self.activation(out)
        if self.normalize:
            out = l2_normalize(out)
        return out

    def get_config(self) -> dict[str, Any]:
        config = super().get_config()
        config.update(
            {
                "output_dim": self.output_dim,
                "normalize": self.normalize,
                "root_weight": self.root_weight,
                "use_bias": self.use_bias,
                "activation": serialize_activation(self.activation),
                "pool_activation": serialize_activation(self.pool_activation),
                "pool_hidden_dim": self.pool_hidden_dim,
                "kernel_initializer": serialize_initializer(self.kernel_initializer),
                "bias_initializer": serialize_initializer(self.bias_initializer),
                "kernel_regularizer": self.kernel_regularizer,
                "bias_regularizer": self.bias_regularizer,
                "kernel_constraint": self.kernel_constraint,
                "bias_constraint": self.bias_constraint,
                "dropout_rate": self.dropout_rate,
            }
        )
        config.pop("aggregator", None)
        config["aggregator"] = self.actual_aggregator  # sage_conv.py:467-469
        return config
