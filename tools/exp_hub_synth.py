"""EXACT hub rows in isolation (a measurement helper).

  python tools/exp_hub_synth.py

Times EXACT weighted F=128 aggregation on synthetic graphs whose only rows
are hubs: one row of 138.5k edges (the NS graph's largest: the chain bound),
and 256 rows of 54k edges (13.8M edges, the NS long-row volume: the
throughput bound).  Sources are uniform over 1M nodes.
"""

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import graph as G  # noqa: E402
from keras_geometric_amd import ops as kops  # noqa: E402


def run(n_rows, deg, n=1_000_000, f=128):
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(0)
    src = torch.randint(0, n, (n_rows * deg,), device=dev, generator=gen, dtype=torch.int32)
    dst = torch.arange(n_rows, device=dev, dtype=torch.int32).repeat_interleave(deg)
    g = G.build_csr(src, dst.contiguous(), n, n, gcn_norm=True)
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
    ms = s.elapsed_time(t) / 10
    return {"rows": n_rows, "deg": deg, "ms": round(ms, 3), "edges_per_us": round(n_rows * deg / ms / 1e3, 1),
            "GBps": round(n_rows * deg * 520 / ms / 1e6, 1)}


if __name__ == "__main__":
    if len(sys.argv) > 1:  # rows deg [n_src] [F]
        a = [int(v) for v in sys.argv[1:]]
        print(json.dumps(run(a[0], a[1], *(a[2:4]))), flush=True)
    else:
        for nr, d in ((1, 138_539), (256, 54_000), (2048, 6_700)):
            print(json.dumps(run(nr, d)), flush=True)
