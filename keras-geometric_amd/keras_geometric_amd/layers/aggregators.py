"""Aggregation strategies (mirror of src/keras_geometric/layers/aggregators.py).

Same names, registry, validation and error messages as the reference
(`AggregatorFactory._AGGREGATORS`, aggregators.py:289-295; ValueError
"Invalid aggregator: ...", :312-317).  `aggregate(messages, target_idx,
dim_size)` runs the kgx segment-reduction kernel over a per-edge message
tensor (CSR by target built on the GPU, cached per target_idx tensor), with
the reference's segment semantics: target ids outside [0, dim_size) are
dropped (Keras-torch segment_sum extra bucket).
"""

from __future__ import annotations

from abc import ABC, abstractmethod

import torch

from .. import _native as nat
from .. import ops as kops
from ..graph import CSRGraph
from ._edges import graph_for
from .base import to_device_tensor


class Aggregator(ABC):
    """Abstract strategy (aggregators.py:16-45)."""

    reduce: str = "sum"

    def aggregate(self, messages, target_idx, dim_size: int, *, graph: CSRGraph | None = None,
                  exact: bool = False) -> torch.Tensor:
        messages = to_device_tensor(messages, torch.float32)
        if messages.dim() == 1:
            messages = messages.unsqueeze(-1)
        if messages.shape[0] == 0:  # aggregators.py:59-61 (and each subclass)
            return torch.zeros((dim_size, messages.shape[1]), dtype=messages.dtype, device=messages.device)
        if graph is None:
            tgt = to_device_tensor(target_idx, torch.int32, messages.device).reshape(-1)
            ei = torch.stack([torch.zeros_like(tgt), tgt])
            graph = graph_for(target_idx, ei, 0, int(dim_size), segment_only=True, n_features=messages.shape[1])
            if self.reduce == "std":
                # StdAggregator gathers mean[target] with take() (aggregators.py:208), which
                # wraps ids in [-dim_size, 0) and raises outside [-dim_size, dim_size); the
                # segment sums alone would drop them.  Checked once per cached graph (one host
                # sync beside the CSR build's own), not on every call.
                oob = getattr(graph, "_take_oob", None)
                if oob is None:
                    oob = bool(((tgt >= dim_size) | (tgt < -dim_size)).any())
                    graph._take_oob = oob
                if oob:
                    raise IndexError("index out of range in self")
        return self._reduce(graph, messages, exact)

    def _reduce(self, graph: CSRGraph, messages: torch.Tensor, exact: bool) -> torch.Tensor:
        return kops.aggregate(graph, messages, self.reduce, by_edge=True, exact=exact)

    @property
    @abstractmethod
    def name(self) -> str: ...


class MeanAggregator(Aggregator):
    """sum / max(count, 1e-8) (aggregators.py:48-89)."""

    reduce = "mean"

    @property
    def name(self) -> str:
        return "mean"


class MaxAggregator(Aggregator):
    """segment_max, isinf -> 0 (aggregators.py:92-116)."""

    reduce = "max"

    @property
    def name(self) -> str:
        return "max"


class SumAggregator(Aggregator):
    """segment_sum (aggregators.py:119-141)."""

    reduce = "sum"

    @property
    def name(self) -> str:
        return "sum"


class MinAggregator(Aggregator):
    """-segment_max(-m), isinf -> 0 (aggregators.py:144-171)."""

    reduce = "min"

    @property
    def name(self) -> str:
        return "min"


class StdAggregator(Aggregator):
    """Two-pass std with N divisor, count <= 1 -> 0 (aggregators.py:174-232)."""

    reduce = "std"

    @property
    def name(self) -> str:
        return "std"


class PoolingAggregator(Aggregator):
    """max over pool_mlp(messages), isinf -> 0 (aggregators.py:235-278)."""

    reduce = "max"

    def __init__(self, pool_mlp) -> None:
        self.pool_mlp = pool_mlp

    def aggregate(self, messages, target_idx, dim_size: int, *, graph: CSRGraph | None = None,
                  exact: bool = False) -> torch.Tensor:
        messages = to_device_tensor(messages, torch.float32)
        if messages.shape[0] == 0:
            probe = self.pool_mlp(torch.zeros((1, messages.shape[1]), device=messages.device))
            return torch.zeros((dim_size, probe.shape[1]), dtype=messages.dtype, device=messages.device)
        return super().aggregate(self.pool_mlp(messages), target_idx, dim_size, graph=graph, exact=exact)

    @property
    def name(self) -> str:
        return "pooling"


class AggregatorFactory:
    """Registry (aggregators.py:281-343)."""

    _AGGREGATORS: dict[str, type[Aggregator]] = {
        "mean": MeanAggregator,
        "max": MaxAggregator,
        "sum": SumAggregator,
        "min": MinAggregator,
        "std": StdAggregator,
    }

    @classmethod
    def create(cls, aggregator_name: str, **kwargs) -> Aggregator:
        if aggregator_name not in cls._AGGREGATORS:
            available = list(cls._AGGREGATORS.keys())
            raise ValueError(f"Invalid aggregator: {aggregator_name}. Available aggregators: {available}")
        return cls._AGGREGATORS[aggregator_name](**kwargs)

    @classmethod
    def create_pooling(cls, pool_mlp) -> PoolingAggregator:
        return PoolingAggregator(pool_mlp)

    @classmethod
    def get_available_aggregators(cls) -> list[str]:
        return list(cls._AGGREGATORS.keys())


REDUCE_IDS = nat.REDUCE_IDS
