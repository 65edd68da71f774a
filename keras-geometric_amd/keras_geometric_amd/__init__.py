"""keras_geometric_amd — MI355X-native message-passing aggregation engine.

Drop-in for keras-geometric's MessagePassing.propagate() hot path
(GCNConv, GINConv, SAGEConv, GATv2Conv) on hand-written gfx950 HIP kernels
behind the C-ABI in include/kgx.h, registered as torch.ops.kgx.*.
"""

from . import _native, graph, ops
from .graph import CSRGraph, build_csr, clear_cache
from .layers import (
    AggregatorFactory,
    BatchGlobalPooling,
    GATv2Conv,
    GCNConv,
    GINConv,
    GlobalPooling,
    MessagePassing,
    SAGEConv,
    set_random_seed,
)
from .utils import GraphData, add_self_loops, batch_graphs, compute_gcn_normalization

__version__ = "0.1.0"

__all__ = [
    "AggregatorFactory",
    "BatchGlobalPooling",
    "CSRGraph",
    "GATv2Conv",
    "GCNConv",
    "GINConv",
    "GlobalPooling",
    "GraphData",
    "MessagePassing",
    "SAGEConv",
    "add_self_loops",
    "batch_graphs",
    "build_csr",
    "clear_cache",
    "compute_gcn_normalization",
    "graph",
    "ops",
    "set_random_seed",
]
