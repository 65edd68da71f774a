"""Probe (CPU, measurement only): rows the push-pull halo moves into one rank
under ShardedGraph.push_pull_plan's degree rule, under that rule followed by
dropping pulled sources whose every halo edge is also served by a pushed
partial, and the exact minimum (König: minimum vertex cover of the bipartite
(source, destination) halo graph per owner = its maximum matching).

    python tools/exp_cover.py N E [world] [rank]
"""

from __future__ import annotations

import os
import sys
import time

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import maximum_bipartite_matching

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from oracle import rmat  # noqa: E402


def main():
    n, e = int(sys.argv[1]), int(sys.argv[2])
    world = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    rank = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    b = [0]
    base, rem = divmod(n, world)
    for r in range(world):
        b.append(b[-1] + base + (1 if r < rem else 0))
    lo, hi = b[rank], b[rank + 1]
    t0 = time.time()
    ss, dd = [], []
    for e0 in range(0, e, 1 << 24):
        s, d = rmat.rmat_edges(0, rmat.scale_for(n), n, e0, min(1 << 24, e - e0))
        m = (d >= lo) & (d < hi) & ((s < lo) | (s >= hi))
        ss.append(s[m].astype(np.int64))
        dd.append(d[m].astype(np.int64) - lo)
    hs, hd = np.concatenate(ss), np.concatenate(dd)
    print(f"gen {time.time() - t0:.1f}s, halo edges {hs.size}")
    owner = np.searchsorted(np.array(b[1:-1]), hs, side="right")
    tot = {"pull": 0, "rule": 0, "pruned": 0, "min": 0}
    for o in range(world):
        if o == rank:
            continue
        m = owner == o
        s, d = hs[m], hd[m]
        us, inv_s, cs = np.unique(s, return_inverse=True, return_counts=True)
        ud, inv_d, cd = np.unique(d, return_inverse=True, return_counts=True)
        # the plan's rule (counts with multiplicity, as torch.unique over the edge list)
        push = cd[inv_d] > cs[inv_s]
        pulled = np.zeros(us.size, bool)
        pulled[inv_s[~push]] = True
        used = np.zeros(ud.size, bool)
        used[inv_d[~pulled[inv_s]]] = True
        rule = int(pulled.sum() + used.sum())
        # prune: a pulled source all of whose destinations are pushed anyway
        all_pushed = np.ones(us.size, bool)
        np.logical_and.at(all_pushed, inv_s, used[inv_d])
        pruned = rule - int((pulled & all_pushed).sum())
        adj = sp.csr_matrix((np.ones(s.size, np.int8), (inv_s, inv_d)), shape=(us.size, ud.size))
        adj.sum_duplicates()
        t1 = time.time()
        match = maximum_bipartite_matching(adj, perm_type="column")
        mm = int((match >= 0).sum())
        print(f"owner {o}: sources {us.size} dests {ud.size} pull {us.size} rule {rule} pruned {pruned} "
              f"min {mm} ({time.time() - t1:.1f}s)")
        tot["pull"] += us.size
        tot["rule"] += rule
        tot["pruned"] += pruned
        tot["min"] += mm
    print(tot, {k: round(v / tot["rule"], 3) for k, v in tot.items()})


if __name__ == "__main__":
    main()
