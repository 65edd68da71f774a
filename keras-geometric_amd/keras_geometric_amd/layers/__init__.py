"""Drop-in layer API (mirror of src/keras_geometric/layers/__init__.py)."""

from .aggregators import (
    Aggregator,
    AggregatorFactory,
    MaxAggregator,
    MeanAggregator,
    MinAggregator,
    PoolingAggregator,
    StdAggregator,
    SumAggregator,
)
from .base import Dense, Layer, Sequential, set_random_seed
from .gatv2_conv import GATv2Conv
from .gcn_conv import GCNConv
from .gin_conv import GINConv
from .message_passing import MessagePassing
from .pooling import BatchGlobalPooling, GlobalPooling
from .sage_conv import SAGEConv

__all__ = [
    "Aggregator",
    "AggregatorFactory",
    "BatchGlobalPooling",
    "Dense",
    "GATv2Conv",
    "GCNConv",
    "GINConv",
    "GlobalPooling",
    "Layer",
    "MaxAggregator",
    "MeanAggregator",
    "MessagePassing",
    "MinAggregator",
    "PoolingAggregator",
    "SAGEConv",
    "Sequential",
    "StdAggregator",
    "SumAggregator",
    "set_random_seed",
]
