"""edge_index normalisation + cached CSR lookup shared by the layers."""

from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

from .. import graph as G
from .base import default_device


_HOST_CAST: "OrderedDict[tuple, tuple]" = OrderedDict()  # host edge_index -> (the array, its device copy)
_HOST_CAST_SIZE = 4


def edge_index_tensor(edge_index, device: torch.device | None, *, allow_transpose: bool) -> torch.Tensor:
    """Cast to int32 [2,E] on `device` (reference: ops.cast(edge_index,"int32"),
    message_passing.py:265 / gcn_conv.py:307; [E,2] transposed for the layers
    that accept it, gcn_conv.py:309-318, sage_conv.py:384-393).  A numpy
    edge_index's device copy is cached like the reference's cast
    (message_passing.py:256-268; graph.host_array_key), so a reference-style
    caller passing the same array every step pays the host-to-device copy once."""
    hk = G.host_array_key(edge_index)
    if hk is not None:
        key = (*hk, str(device), allow_transpose)
        hit = _HOST_CAST.get(key)
        if hit is not None:
            _HOST_CAST.move_to_end(key)
            return hit[1]
        ei = _edge_index_tensor(edge_index, device, allow_transpose=allow_transpose)
        _HOST_CAST[key] = (edge_index, ei)
        while len(_HOST_CAST) > _HOST_CAST_SIZE:
            _HOST_CAST.popitem(last=False)
        return ei
    return _edge_index_tensor(edge_index, device, allow_transpose=allow_transpose)


def _edge_index_tensor(edge_index, device: torch.device | None, *, allow_transpose: bool) -> torch.Tensor:
    if isinstance(edge_index, torch.Tensor):
        ei = edge_index
        if ei.device.type != "cuda":
            ei = ei.to(device or default_device())
    else:
        ei = torch.as_tensor(np.asarray(edge_index)).to(device or default_device())
    if ei.dim() == 1 and ei.numel() == 0:
        ei = ei.reshape(2, 0)
    if ei.dim() != 2:
        raise ValueError(f"edge_index must have shape [2, E] or [E, 2], but got {tuple(ei.shape)}")
    if ei.shape[0] != 2:
        if allow_transpose and ei.shape[1] == 2:
            ei = ei.t()
        else:
            raise ValueError(f"edge_index must have shape [2, E] or [E, 2], but got {tuple(ei.shape)}")
    if ei.dtype != torch.int32:
        ei = ei.to(torch.int32)
    return ei


def graph_for(
    edge_index_obj,
    ei: torch.Tensor,
    n_src: int,
    n_dst: int,
    *,
    self_loops: bool = False,
    gcn_norm: bool = False,
    segment_only: bool = False,
    n_features: int = 128,
) -> G.CSRGraph:
    """CSRGraph for ei, cached on the caller's original edge_index tensor."""
    key = G.cache_key(edge_index_obj, ei.shape[1], n_src, n_dst, self_loops, gcn_norm, segment_only,
                      G.default_split_len(ei.shape[1] + (n_dst if self_loops else 0), n_features))
    src = ei[0].contiguous()
    dst = ei[1].contiguous()

    def build():
        g = G.build_csr(src, dst, n_src, n_dst, self_loops=self_loops, gcn_norm=gcn_norm,
                        segment_only=segment_only, n_features=n_features)
        if segment_only:
            # StdAggregator's take(mean, target) raises for ids outside [-n, n)
            # (aggregators.py:208); decided here, where the build syncs anyway
            g._take_oob = bool(((dst >= n_dst) | (dst < -n_dst)).any()) if dst.numel() else False
        return g

    return G.cached(key, edge_index_obj, build)
