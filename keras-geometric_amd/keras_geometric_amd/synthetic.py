"""Synthetic power-law graphs generated on the GPU (kgx_rmat_edges).

R-MAT (a, b, c) = (0.57, 0.19, 0.19), scale = ceil(log2 N), ids mod N then
relabelled by a keyed Feistel permutation; COO int32 [2, E] in generation
order (unsorted, not deduplicated), as the reference would receive it.  The
generator is counter based: oracle/rmat.py restates it bit for bit.
"""

from __future__ import annotations

import ctypes
import math

import torch

from . import _native as nat


def scale_for(n: int) -> int:
    return max(1, math.ceil(math.log2(max(n, 2))))


def _p24(p: float) -> int:
    return int(round(p * (1 << 24)))


def rmat_edges_into(src: torch.Tensor, dst: torch.Tensor, n_nodes: int, e_begin: int, seed: int = 0,
                    a: float = 0.57, b: float = 0.19, c: float = 0.19) -> None:
    dev = nat.require_device(src, dst)
    n = src.numel()
    nat.check(
        nat.lib().kgx_rmat_edges(
            seed, scale_for(n_nodes), n_nodes, _p24(a), _p24(b), _p24(c), e_begin, n, nat.ptr(src), nat.ptr(dst),
            nat.stream(dev),
        ),
        "kgx_rmat_edges",
    )


def rmat_edge_index(n_nodes: int, n_edges: int, seed: int = 0, device: torch.device | None = None,
                    a: float = 0.57, b: float = 0.19, c: float = 0.19) -> torch.Tensor:
    """[2, n_edges] int32 edge_index on `device`."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    ei = torch.empty((2, n_edges), dtype=torch.int32, device=device)
    if n_edges:
        rmat_edges_into(ei[0], ei[1], n_nodes, 0, seed, a, b, c)
    return ei


def rmat_dst_shard(n_nodes: int, n_edges: int, lo: int, hi: int, seed: int = 0,
                   device: torch.device | None = None, batch: int = 1 << 26) -> torch.Tensor:
    """Edges of the global R-MAT graph whose destination lies in [lo, hi).

    Every rank generates the same global edge stream in batches and keeps its
    destination range (stream compaction on the GPU), so shards of one graph
    agree across ranks without any communication.
    """
    device = device or torch.device("cuda", torch.cuda.current_device())
    L = nat.lib()
    bsz = min(batch, max(n_edges, 1))
    s = torch.empty(bsz, dtype=torch.int32, device=device)
    d = torch.empty(bsz, dtype=torch.int32, device=device)
    so = torch.empty(bsz, dtype=torch.int32, device=device)
    do = torch.empty(bsz, dtype=torch.int32, device=device)
    nbytes = ctypes.c_size_t(0)
    nat.check(L.kgx_select_workspace_bytes(bsz, ctypes.byref(nbytes)), "kgx_select_workspace_bytes")
    ws = torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=device)
    parts_s, parts_d = [], []
    for e0 in range(0, n_edges, bsz):
        n = min(bsz, n_edges - e0)
        rmat_edges_into(s[:n], d[:n], n_nodes, e0, seed)
        cnt = ctypes.c_int64(0)
        nat.check(
            L.kgx_select_dst_range(nat.ptr(s), nat.ptr(d), n, lo, hi, nat.ptr(so), nat.ptr(do), nat.ptr(ws),
                                   nbytes.value, ctypes.byref(cnt), nat.stream(device)),
            "kgx_select_dst_range",
        )
        parts_s.append(so[: cnt.value].clone())
        parts_d.append(do[: cnt.value].clone())
    if not parts_s:
        return torch.empty((2, 0), dtype=torch.int32, device=device)
    return torch.stack([torch.cat(parts_s), torch.cat(parts_d)])
