"""GraphData and batch_graphs (mirror of src/keras_geometric/utils/data_utils.py).

GraphData (data_utils.py:8-136) holds a graph's tensors; here they live on the
GPU (int32 edge_index, fp32 features) so a batch feeds the kgx layers without
a host round trip.  batch_graphs (data_utils.py:139-272) concatenates graphs
into one graph of disjoint components: node features and edge attributes
concatenated, every graph's edge_index shifted by its node offset, a `batch`
vector of graph ids (node i -> its graph), graph-level targets (1-D y)
stacked to [num_graphs, y_dim] and node-level targets concatenated -- the
same layout the reference builds with slice_update loops, built here with one
concatenation per field.  The batch vector is what BatchGlobalPooling
segments by.
"""

from __future__ import annotations

from typing import Any

import numpy as np
import torch

from ..layers.base import default_device


def _tensor(data, dtype: torch.dtype | None = None, device=None):
    if data is None:
        return None
    if isinstance(data, torch.Tensor):
        t = data
        if t.device.type != "cuda":
            t = t.to(device or default_device())
    else:
        t = torch.as_tensor(np.asarray(data)).to(device or default_device())
    return t.to(dtype) if dtype is not None and t.dtype != dtype else t


class GraphData:
    """A graph's tensors: x [N, F], edge_index [2, E], optional edge_attr, y,
    explicit num_nodes and extra named tensors (data_utils.py:8-136)."""

    def __init__(self, x, edge_index, edge_attr=None, y=None, num_nodes: int | None = None, **kwargs: Any) -> None:
        self.x = _tensor(x)
        self.edge_index = _tensor(edge_index, torch.int32, self.x.device if self.x is not None else None)
        dev = self.edge_index.device
        self.edge_attr = _tensor(edge_attr, device=dev) if edge_attr is not None else None
        self.y = _tensor(y, device=dev) if y is not None else None
        self._num_nodes = int(self.x.shape[0]) if num_nodes is None else int(num_nodes)
        self._additional_data = {k: _tensor(v, device=dev) for k, v in kwargs.items()}

    @property
    def num_nodes(self) -> int:
        return self._num_nodes

    @property
    def num_edges(self) -> int:
        return 0 if self.edge_index is None else int(self.edge_index.shape[1])

    @property
    def num_node_features(self) -> int:
        return 0 if self.x is None else int(self.x.shape[1])

    @property
    def num_edge_features(self) -> int:
        return 0 if self.edge_attr is None else int(self.edge_attr.shape[1])

    def to_dict(self) -> dict[str, Any]:
        d = {"x": self.x, "edge_index": self.edge_index}
        if self.edge_attr is not None:
            d["edge_attr"] = self.edge_attr
        if self.y is not None:
            d["y"] = self.y
        d.update(self._additional_data)
        return d

    def to_inputs(self) -> list:
        inputs = [self.x, self.edge_index]
        if self.edge_attr is not None:
            inputs.append(self.edge_attr)
        return inputs

    def __getattr__(self, name: str) -> Any:
        extra = self.__dict__.get("_additional_data", {})
        if name in extra:
            return extra[name]
        raise AttributeError(f"'{type(self).__name__}' object has no attribute '{name}'")


def batch_graphs(graphs: list[GraphData]) -> GraphData:
    """One GraphData of disjoint components with a `batch` vector (data_utils.py:139-272)."""
    if not graphs:
        raise ValueError("Cannot batch empty list of graphs")
    dev = graphs[0].x.device
    sizes = [g.num_nodes for g in graphs]
    offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    total = int(sum(sizes))
    x = torch.cat([g.x.to(dev) for g in graphs], dim=0)
    ei = [g.edge_index.to(dev) for g in graphs]
    edge_dtype = ei[0].dtype
    edge_index = torch.cat(
        [e + int(o) if e.shape[1] else e for e, o in zip(ei, offsets)], dim=1
    ).to(edge_dtype) if sum(e.shape[1] for e in ei) else torch.zeros((2, 0), dtype=edge_dtype, device=dev)
    batch = torch.repeat_interleave(
        torch.arange(len(graphs), dtype=torch.int32, device=dev),
        torch.as_tensor(sizes, dtype=torch.int64, device=dev), output_size=total,
    )
    edge_attr = None
    if all(g.edge_attr is not None for g in graphs):
        edge_attr = torch.cat([g.edge_attr.to(dev) for g in graphs], dim=0)
    y = None
    if all(g.y is not None for g in graphs):
        if graphs[0].y.dim() == 1:  # graph-level targets -> [num_graphs, y_dim]
            y = torch.stack([g.y.to(dev) for g in graphs], dim=0)
        else:  # node-level targets
            y = torch.cat([g.y.to(dev) for g in graphs], dim=0)
    return GraphData(x=x, edge_index=edge_index, edge_attr=edge_attr, y=y, num_nodes=total, batch=batch)
