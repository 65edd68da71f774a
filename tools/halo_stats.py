"""Halo sizes of destination-range shards of the R-MAT graphs (one GPU, no comm).

  python tools/halo_stats.py

For weak scaling (P x 10M nodes / P x 100M edges) and strong scaling (10M /
100M fixed) at P = 2, 4, 8: per rank, edges kept, unique sources, and unique
REMOTE sources (the halo rows a layer must receive).  A measurement helper
for DESIGN.md §Multi-GPU; not part of the product.
"""

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import distributed as kd  # noqa: E402
from keras_geometric_amd import synthetic  # noqa: E402


def shard_stats(n, e, P, ranks):
    dev = torch.device("cuda", 0)
    bounds = kd.equal_bounds(n, P)
    out = []
    for r in ranks:
        lo, hi = bounds[r], bounds[r + 1]
        ei = synthetic.rmat_dst_shard(n, e, lo, hi, seed=0, device=dev)
        src = ei[0].long()
        u = torch.unique(src)
        remote = int(((u < lo) | (u >= hi)).sum())
        out.append({"rank": r, "edges": int(src.numel()), "unique_src": int(u.numel()), "halo_rows": remote})
        del ei, src, u
        torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    for P in (2, 4, 8):
        print(json.dumps({"mode": "weak", "P": P, "ranks": shard_stats(P * 10_000_000, P * 100_000_000, P, [0, P - 1])}),
              flush=True)
    for P in (2, 4, 8):
        print(json.dumps({"mode": "strong", "P": P, "ranks": shard_stats(10_000_000, 100_000_000, P, [0, P - 1])}),
              flush=True)
