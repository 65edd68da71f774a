"""The oracle on sampled rows of a full-size graph (test infrastructure).

The BASELINE configs C4 / C5 / NS are too large for the oracle's op-for-op CPU
forward (its [E', F] intermediates alone need 200-400 GB).  A destination row's
output depends only on its in-edges, its own features and the layer's weights
(plus, for GCN, its sources' degrees), so the oracle runs on the subgraph of
the sampled rows' in-edges, in input order, over the nodes they touch: the
sampled rows' outputs are the reference's outputs on the whole graph, computed
by the same ops (oracle/reference.py).  The rows sampled: the largest hubs, and
a seeded uniform sample of the rest (zero in-degree rows included).
"""

from __future__ import annotations

import torch

from oracle import reference as R


def sample_rows(ei: torch.Tensor, n: int, k: int = 1500, hubs: int = 6, seed: int = 0) -> torch.Tensor:
    """Sorted node ids: the `hubs` largest in-degree rows + k uniform ones (device of ei)."""
    deg = torch.bincount(ei[1].long(), minlength=n)
    top = torch.topk(deg, hubs).indices
    g = torch.Generator(device=ei.device).manual_seed(seed)
    rnd = torch.randint(0, n, (k,), device=ei.device, generator=g)
    return torch.unique(torch.cat([top, rnd]))


def subgraph(ei: torch.Tensor, x: torch.Tensor, rows: torch.Tensor):
    """(x_sub, ei_sub, pos, nodes) on the CPU: the in-edges of `rows` in input
    order, relabelled onto the nodes they touch; pos[i] = row i's index."""
    n = x.shape[0]
    want = torch.zeros(n, dtype=torch.bool, device=ei.device)
    want[rows] = True
    keep = want[ei[1].long()]
    src, dst = ei[0][keep].long(), ei[1][keep].long()
    nodes = torch.unique(torch.cat([rows, src]))
    remap = torch.full((n,), -1, dtype=torch.long, device=ei.device)
    remap[nodes] = torch.arange(nodes.numel(), device=ei.device)
    ei_sub = torch.stack([remap[src], remap[dst]]).to(torch.int32).cpu()
    return x[nodes].cpu(), ei_sub, remap[rows].cpu(), nodes


def gin_rows(ei, x, rows, mlp, eps):
    x_sub, ei_sub, pos, _ = subgraph(ei, x, rows)
    return R.gin_forward(x_sub, ei_sub, mlp, "sum", eps=eps)[pos]


def sage_rows(ei, x, rows, w_neigh, w_self, bias):
    x_sub, ei_sub, pos, _ = subgraph(ei, x, rows)
    return R.sage_forward(x_sub, ei_sub, w_neigh, w_self, bias, "mean")[pos]


def gcn_rows(ei, x, rows, W, b):
    """GCN with the whole graph's degrees (self loops included: + 1)."""
    n = x.shape[0]
    x_sub, ei_sub, pos, nodes = subgraph(ei, x, rows)
    deg = (torch.bincount(ei[1].long(), minlength=n) + 1).to(torch.float32)
    return R.gcn_forward(x_sub, ei_sub, W, b, degrees=deg[nodes].cpu())[pos]


def scaled_err(got_rows: torch.Tensor, ref: torch.Tensor, scale: torch.Tensor) -> float:
    """max |got - ref| / max(1, scale): scale = the same layer on |x|, |weights|
    (the forward-error bound of re-associated fp32 sums)."""
    return float(((got_rows.cpu() - ref).abs() / scale.cpu().clamp_min(1.0)).max())
