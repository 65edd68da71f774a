"""The 256-wide fused kernel (kgx_spmm_gemm_f256) on the C4 graph, by part
(a measurement helper).

  python tools/exp_f256.py

Times torch.ops.kgx.spmm_gemm (GIN epilogue, F 256 -> 256) over the whole C4
schedule, its long prefix (rows of degree > 7 and hub chunks, + fix-up) and
its short suffix, beside the unfused pair (kgx_spmm with the GIN epilogue,
then kgx_dense).  KGX_LIB names the library (variant builds).
"""

import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import _native as nat  # noqa: E402
from keras_geometric_amd import graph as G  # noqa: E402
from keras_geometric_amd import ops as kops  # noqa: E402
from keras_geometric_amd import synthetic  # noqa: E402


def timeit(fn, reps=6):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main(n=10_000_000, e=100_000_000, f=256):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)  # same x / W / b in every process: variants' out_bits compare
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, n_features=f)
    x = torch.randn(n, f, device=dev)
    W = torch.randn(f, f, device=dev) * (1.0 / f) ** 0.5
    b = torch.randn(f, device=dev)
    tpack, tw, n_se, n2 = kops._tiny_of(g, g.items)
    long_ = g.items[:g.n_long].contiguous()
    mid = g.items[g.n_long:n_se].contiguous()  # unsplit rows of degree 3..7
    tail = g.items[n_se:].contiguous()          # degree <= 2: the tiny-record kernel
    op = torch.ops.kgx.spmm_gemm
    res = {"lib": os.path.basename(os.environ.get("KGX_LIB", "libkgx.so")), "n_long": g.n_long, "n_short_end": n_se,
           "n_items": g.n_items, "n_split": g.n_split}
    with torch.no_grad():
        res["fused_ms"] = timeit(lambda: op(x, g.rowptr, g.rows, g.items, g.split, g.col, None, g.n_slots, 0, W, b,
                                            True, 1.25, False, g.n_long, tpack, tw, n_se, n2))
        res["fused_notiny_ms"] = timeit(lambda: op(x, g.rowptr, g.rows, g.items, g.split, g.col, None, g.n_slots, 0,
                                                   W, b, True, 1.25))
        res["fused_long_ms"] = timeit(lambda: op(x, g.rowptr, g.rows, long_, g.split, g.col, None, g.n_slots, 0, W, b,
                                                 True, 1.25))
        res["fused_mid_ms"] = timeit(lambda: op(x, g.rowptr, g.rows, mid, None, g.col, None, 0, 0, W, b, True, 1.25,
                                                False, 0))  # n_long = 0: the degree 3-7 launch
        res["fused_tiny_ms"] = timeit(lambda: op(x, g.rowptr, g.rows, tail, None, g.col, None, 0, 0, W, b, True, 1.25,
                                                 False, -1, tpack, tw, 0, n2))
        y = op(x, g.rowptr, g.rows, g.items, g.split, g.col, None, g.n_slots, 0, W, b, True, 1.25, False, g.n_long,
               tpack, tw, n_se, n2)
        bits = y.view(torch.int32).to(torch.int64)
        res["out_bits"] = int(bits.sum()) + 3 * int(bits[::7].sum())  # variants must match bit for bit
        del y, bits
        if os.environ.get("KGX_EXP_UNFUSED", "1") == "1":
            h = kops.aggregate(g, x, "sum", epilogue=nat.EPI_GIN, xroot=x, gin_scale=1.25)
            res["unfused_agg_ms"] = timeit(lambda: kops.aggregate(g, x, "sum", epilogue=nat.EPI_GIN, xroot=x,
                                                                  gin_scale=1.25))
            res["unfused_dense_ms"] = timeit(lambda: kops.dense(h, W, b))
    print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
