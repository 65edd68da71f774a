"""The fused GCN kernel's short-row part alone (a measurement helper).

  python tools/exp_short.py

Times torch.ops.kgx.spmm_gemm over the NS schedule's short-row suffix
(degree <= 7, spmm_gemm_short_kernel: n_long = 0) and over the long prefix
(spmm_gemm_kernel), with the library named by KGX_LIB (an experiments build
honours KGX_FUSED_DEBUG: 1 skip MFMA, 2 skip stores).
"""

import json
import os
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
    short = g.items[g.n_long:].contiguous()
    long_ = g.items[:g.n_long].contiguous()
    op = torch.ops.kgx.spmm_gemm
    t_short = timeit(lambda: op(x, g.rowptr, g.rows, short, None, g.col, g.w, g.n_slots, 0, W, None, False, 1.0,
                                False, 0))
    t_long = timeit(lambda: op(x, g.rowptr, g.rows, long_, g.split, g.col, g.w, g.n_slots, 0, W, None, False, 1.0,
                               False, -1))
    lens = (short[:, 2] - short[:, 1]).long()
    print(json.dumps({"lib": os.path.basename(os.environ.get("KGX_LIB", "libkgx.so")),
                      "debug": os.environ.get("KGX_FUSED_DEBUG", "0"), "short_rows": short.shape[0],
                      "short_edges": int(lens.sum()), "short_ms": round(t_short, 3), "long_ms": round(t_long, 3)}),
          flush=True)


if __name__ == "__main__":
    main()
