"""Persistent graph files: the reference's processed-dataset NPZ plus kgx CSRs.

The reference saves a processed dataset as one `.npz` with, per graph i,
`x_{i}`, `edge_index_{i}`, optional `edge_attr_{i}` / `y_{i}`, and the
scalars `num_graphs`, `num_classes` (datasets/base.py:124-154), and reloads
it into GraphData objects (:156-182).  Every layer call then rebuilds what
the kernels need from edge_index (message_passing.py:256-268 re-casts per
call).  This module reads and writes that same layout and can add, per
graph, the destination CSR and its row schedule (`kgx_csr_{i}_<field>`
arrays + an int64 `kgx_csr_{i}_meta` row; format tag `kgx_format`), so a
100M-edge graph is loaded instead of re-sorted.
Loaded CSRs are registered in the layer cache under the loaded edge_index
tensor, exactly where the layers look them up.

Files are read with numpy.load(allow_pickle=False): numeric arrays only,
nothing in a file is executed.  A reference-written file (no kgx arrays)
loads as plain GraphData.
"""

from __future__ import annotations

import os

import numpy as np
import torch

from .. import graph as G
from .data import GraphData

FORMAT = "kgx-csr-1"
_FIELDS = ("rowptr", "col", "eid", "deg", "dinv", "w", "rows", "items", "split")
_META = ("n_src", "n_dst", "n_input_edges", "kept", "max_degree", "flags", "n_items", "n_split", "n_slots",
         "split_len")


def csr_arrays(g: G.CSRGraph) -> dict[str, np.ndarray]:
    """Host copies of a CSRGraph's arrays (+ a meta row)."""
    out = {}
    for f in _FIELDS:
        t = getattr(g, f)
        if t is not None:
            out[f] = t.detach().cpu().numpy()
    out["meta"] = np.array([getattr(g, m) for m in _META], dtype=np.int64)
    return out


def csr_from_arrays(d: dict[str, np.ndarray], device: torch.device) -> G.CSRGraph:
    meta = dict(zip(_META, (int(v) for v in d["meta"])))
    t = {f: torch.from_numpy(np.ascontiguousarray(d[f])).to(device) for f in _FIELDS if f in d}
    g = G.CSRGraph(
        n_src=meta["n_src"], n_dst=meta["n_dst"], n_input_edges=meta["n_input_edges"], kept=meta["kept"],
        max_degree=meta["max_degree"], flags=meta["flags"], rowptr=t["rowptr"], col=t["col"], eid=t["eid"],
        deg=t["deg"], dinv=t.get("dinv"), w=t.get("w"), rows=t.get("rows"), items=t.get("items"),
        split=t.get("split"), n_items=meta["n_items"], n_split=meta["n_split"], n_slots=meta["n_slots"],
        split_len=meta["split_len"],
    )
    if g.rowptr.numel() != g.n_dst + 1 or g.col.numel() != g.kept or g.eid.numel() != g.kept:
        raise ValueError("kgx graph file: CSR array sizes do not match its meta row")
    if g.items is not None:
        g.n_long = G.short_suffix_start(g.items[: g.n_items])
    return g


def register(edge_index: torch.Tensor, g: G.CSRGraph) -> None:
    """Make `g` the cached CSR the layers find for `edge_index` (same key as layers/_edges.graph_for)."""
    self_loops = bool(g.flags & 1)
    segment_only = bool(g.flags & 2)
    gcn_norm = bool(g.flags & 4)
    key = G.cache_key(edge_index, int(edge_index.shape[1]), g.n_src, g.n_dst, self_loops, gcn_norm, segment_only,
                      g.split_len)
    G.cached(key, edge_index, lambda: g)


def save_graphs(path: str | os.PathLike, graphs: list[GraphData], num_classes: int | None = None, *,
                with_csr: bool = False, self_loops: bool = False, gcn_norm: bool = False,
                n_features: int | None = None) -> None:
    """Write the reference's processed layout; with_csr=True adds each graph's
    kgx CSR (built with the given flags, as the layer that will read it does)."""
    arrays: dict[str, np.ndarray] = {}
    for i, g in enumerate(graphs):
        arrays[f"x_{i}"] = g.x.detach().cpu().numpy()
        arrays[f"edge_index_{i}"] = g.edge_index.detach().cpu().numpy()
        if g.edge_attr is not None:
            arrays[f"edge_attr_{i}"] = g.edge_attr.detach().cpu().numpy()
        if g.y is not None:
            arrays[f"y_{i}"] = g.y.detach().cpu().numpy()
        if with_csr:
            ei = g.edge_index
            n = g.num_nodes
            feats = n_features if n_features is not None else g.num_node_features
            csr = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=self_loops,
                              gcn_norm=gcn_norm, n_features=feats)
            for k, v in csr_arrays(csr).items():
                arrays[f"kgx_csr_{i}_{k}"] = v
    arrays["num_graphs"] = np.array(len(graphs), dtype=np.int64)
    if num_classes is not None:
        arrays["num_classes"] = np.array(int(num_classes), dtype=np.int64)
    if with_csr:
        arrays["kgx_format"] = np.frombuffer(FORMAT.encode(), dtype=np.uint8)
    np.savez(path, **arrays)


def load_graphs(path: str | os.PathLike, device: torch.device | None = None) -> tuple[list[GraphData], int | None]:
    """Read a processed NPZ (reference layout, optionally with kgx CSRs) into
    GraphData on `device`; kgx CSRs are registered for the layers' lookups."""
    with np.load(path, allow_pickle=False) as data:
        files = set(data.files)
        has_csr = "kgx_format" in files
        if has_csr and bytes(data["kgx_format"]).decode() != FORMAT:
            raise ValueError(f"unsupported kgx graph file format {bytes(data['kgx_format'])!r}")
        num_graphs = int(data["num_graphs"])
        num_classes = int(data["num_classes"]) if "num_classes" in files else None
        out = []
        for i in range(num_graphs):
            g = GraphData(
                x=data[f"x_{i}"], edge_index=data[f"edge_index_{i}"],
                edge_attr=data[f"edge_attr_{i}"] if f"edge_attr_{i}" in files else None,
                y=data[f"y_{i}"] if f"y_{i}" in files else None,
            )
            if device is not None:
                g.x, g.edge_index = g.x.to(device), g.edge_index.to(device)
            prefix = f"kgx_csr_{i}_"
            if has_csr and prefix + "meta" in files:
                arrs = {k[len(prefix):]: data[k] for k in files if k.startswith(prefix)}
                csr = csr_from_arrays(arrs, g.edge_index.device)
                g.csr = csr  # also reachable directly
                register(g.edge_index, csr)
            out.append(g)
    return out, num_classes
