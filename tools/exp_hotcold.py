"""Hot/cold source split of the NS GCN aggregation (one MI355X).

  python tools/exp_hotcold.py [--fracs 0.005,0.01,0.02,0.05]

R-MAT sources are heavily skewed (at 1M/10M the top 1 % of sources feed
51 % of the edges).  In one destination-major pass every hot row's uses are
spread over the whole launch and the stream of cold rows evicts it from
L2/MALL between uses.  Split: a cold pass (edges from sources below the
out-degree threshold, with bias, all rows) and a hot pass (edges from the top
sources only, accumulate-only) whose whole source set fits the 256 MB MALL.
Times the fused kernel both ways and checks the split result against the
one-pass result (tolerance).  Measurement helper, not part of the product.
"""

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import graph as G  # noqa: E402
from keras_geometric_amd import ops as kops  # noqa: E402
from keras_geometric_amd import synthetic  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=10_000_000)
    ap.add_argument("--edges", type=int, default=100_000_000)
    ap.add_argument("--fracs", default="0.005,0.01,0.02,0.05")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    N = args.nodes
    ei = synthetic.rmat_edge_index(N, args.edges, seed=0, device=dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), N, N, self_loops=True, gcn_norm=True)
    x = torch.randn(N, 128, device=dev)
    W = torch.randn(128, 128, device=dev) * 0.1
    b = torch.randn(128, device=dev)
    with torch.no_grad():
        ref = kops.aggregate_transform(g, x, W, "sum", weighted=True, bias=b)
        t1 = timeit(lambda: kops.aggregate_transform(g, x, W, "sum", weighted=True, bias=b))
        print(json.dumps({"mode": "one pass", "ms": round(t1, 3)}), flush=True)
        outdeg = torch.bincount(g.col.long(), minlength=N)
        srt = torch.sort(outdeg, descending=True).values
        for frac in [float(v) for v in args.fracs.split(",")]:
            k = max(1, int(N * frac))
            thr = int(srt[k - 1])
            hot = (outdeg[g.col.long()] >= thr).to(torch.int64)  # part 1 = hot
            cold_g, hot_g = G.split_by_part(g, hot, [(0, N), (0, N)])

            def two():
                out = kops.aggregate_transform(cold_g, x, W, "sum", weighted=True, bias=b)
                kops.aggregate_transform(hot_g, x, W, "sum", weighted=True, out=out)
                return out

            y = two()
            err = ((y - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
            tc = timeit(lambda: kops.aggregate_transform(cold_g, x, W, "sum", weighted=True, bias=b))
            out = ref.clone()
            th = timeit(lambda: kops.aggregate_transform(hot_g, x, W, "sum", weighted=True, out=out))
            t2 = timeit(two)
            print(json.dumps({"mode": "hot/cold", "top_frac": frac, "hot_rows": int((outdeg >= thr).sum()),
                              "hot_MB": int((outdeg >= thr).sum()) * 512 / 1e6, "hot_edges": hot_g.kept,
                              "cold_edges": cold_g.kept, "hot_rows_touched": hot_g.n_items,
                              "ms_cold": round(tc, 3), "ms_hot": round(th, 3), "ms_total": round(t2, 3),
                              "max_err_vs_one_pass": err}), flush=True)
            del cold_g, hot_g, hot
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
