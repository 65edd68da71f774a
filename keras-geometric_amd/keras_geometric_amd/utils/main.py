"""Graph preprocessing helpers (mirror of src/keras_geometric/utils/main.py).

Both return tensors in the caller's INPUT edge order, like the reference.
The layers themselves never call these: they use the cached CSRGraph, whose
self loops / degrees / norms come out of the same kgx_csr_build kernels.
"""

from __future__ import annotations

import torch

from .. import graph as G
from .. import ops as kops
from ..layers._edges import edge_index_tensor


def add_self_loops(edge_index, num_nodes: int) -> torch.Tensor:
    """Append (i, i) for i < num_nodes AFTER the existing edges (utils/main.py:8-16)."""
    ei = edge_index_tensor(edge_index, None, allow_transpose=False)
    loops = torch.arange(num_nodes, dtype=ei.dtype, device=ei.device)
    return torch.cat([ei, torch.stack([loops, loops])], dim=1)


def compute_gcn_normalization(edge_index, num_nodes: int) -> torch.Tensor:
    """norm_e = dinv[dst] * dinv[src], dinv = (deg + 1e-12)^-0.5, deg = in-degree
    counted over targets (utils/main.py:20-33), in input edge order.

    Computed by kgx_csr_build (KGX_CSR_GCN_NORM) and scattered back from CSR
    order through the CSR's edge-id permutation; edges whose target is
    negative (dropped by the reference's segment_sum) keep norm 0.
    """
    ei = edge_index_tensor(edge_index, None, allow_transpose=False)
    E = ei.shape[1]
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), num_nodes, num_nodes, gcn_norm=True, split_len=0)
    if E == 0:
        return torch.zeros(0, dtype=torch.float32, device=ei.device)
    return kops.scatter_f32(g.w, g.eid, E)
