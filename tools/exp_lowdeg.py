"""Where the NS fused kernel's time goes by row degree (a measurement helper).

  python tools/exp_lowdeg.py

The schedule lists items in descending-degree order (log2 buckets), so rows
of degree <= d form a suffix of it.  Times the fused GCN aggregate->transform
launch over the whole schedule and over the prefix / suffix split at degree
1, 3, 7 and 15, with bytes per part, to show whether the many short rows
(53 % of R-MAT rows are the self loop alone) cost more than their bytes.
"""

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import graph as G  # noqa: E402
from keras_geometric_amd import synthetic  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main(n=10_000_000, e=100_000_000, f=128):
    dev = torch.device("cuda", 0)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=True, gcn_norm=True)
    x = torch.randn(n, f, device=dev)
    W = torch.randn(f, f, device=dev) * (1.0 / f) ** 0.5
    items = g.items
    lens = (items[:, 2] - items[:, 1]).long()
    split_items = int((items[:, 3] >= 0).sum())

    def run(its):
        n_split = g.n_split if split_items and its.shape[0] and int(its[0, 3]) >= 0 else 0
        return torch.ops.kgx.spmm_gemm(x, g.rowptr, g.rows, its.contiguous(), g.split if n_split else None,
                                      g.col, g.w, g.n_slots, 0, W, None, False, 1.0, False)

    def run_spmm(its):  # the plain weighted aggregation (kgx_spmm) over the same items
        n_split = g.n_split if split_items and its.shape[0] and int(its[0, 3]) >= 0 else 0
        return torch.ops.kgx.spmm(x, g.rowptr, g.rows, its.contiguous(), g.split if n_split else None, g.col, g.w,
                                  g.n_slots, 0, 0, None, None, 1.0)

    if len(sys.argv) > 1 and sys.argv[1] == "spmm":
        run = run_spmm  # noqa: F811
    full = timeit(lambda: run(items))
    out = {"full_ms": full, "items": items.shape[0]}
    for d in (1, 3, 7, 15):  # log2-bucket boundaries: rows of degree <= d are a suffix of the schedule
        k = int(torch.nonzero(lens <= d)[0]) if bool((lens <= d).any()) else items.shape[0]
        hi, lo = items[:k], items[k:]
        e_hi, e_lo = int(lens[:k].sum()), int(lens[k:].sum())
        t_hi, t_lo = timeit(lambda: run(hi)), timeit(lambda: run(lo))
        b_lo = e_lo * (4 + 4 + 512) + lo.shape[0] * 512
        out[f"deg<={d}"] = {"items": lo.shape[0], "edges": e_lo, "ms": round(t_lo, 3), "TBps": round(b_lo / t_lo / 1e9, 2),
                            "rest_items": hi.shape[0], "rest_edges": e_hi, "rest_ms": round(t_hi, 3)}
        print(json.dumps({d: out[f"deg<={d}"]}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
