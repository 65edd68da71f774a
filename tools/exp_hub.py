"""EXACT-mode long rows at NS (a measurement helper).

  python tools/exp_hub.py

Prints how many rows reach spmm_hub_kernel (degree >= 2048), the edges they
hold and the largest degrees, and times the EXACT weighted aggregation.
"""

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import graph as G  # noqa: E402
from keras_geometric_amd import ops as kops  # noqa: E402
from keras_geometric_amd import synthetic  # noqa: E402


def main(n=10_000_000, e=100_000_000, f=128):
    dev = torch.device("cuda", 0)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=True, gcn_norm=True)
    deg = g.deg.long()
    long = deg >= 2048
    top = torch.topk(deg, 8).values.tolist()
    h = torch.randn(n, f, device=dev)
    fn = lambda: kops.aggregate(g, h, "sum", weighted=True, exact=True)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        fn()
    t.record()
    torch.cuda.synchronize()
    print(json.dumps({"long_rows": int(long.sum()), "long_edges": int(deg[long].sum()),
                      "edges_ge_8192": int(deg[deg >= 8192].sum()), "rows_ge_8192": int((deg >= 8192).sum()),
                      "top_degrees": top, "exact_weighted_ms": round(s.elapsed_time(t) / 10, 3)}), flush=True)


if __name__ == "__main__":
    main()
