"""kgx_dense vs the fp32 library GEMM (torch.addmm -> hipBLASLt) at the
BASELINE configs' dense shapes; prints one JSON line per shape.

  python tools/bench_dense.py [--reps 20]
"""

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import ops as kops  # noqa: E402

SHAPES = {  # name: (M, K0, K1, N, relu)
    "C4 GIN MLP Dense 10M x 256->256": (10_000_000, 256, 0, 256, False),
    "C5 SAGE lin_self+lin_neigh 2.45M x (100+100)->100 relu": (2_449_029, 100, 100, 100, True),
    "C3 GATv2 xW 1M x 128->128": (1_000_000, 128, 0, 128, False),
    "NS GCN xW 10M x 128->128": (10_000_000, 128, 0, 128, False),
}


def timeit(fn, reps):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated substrings of shape names to run")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    only = [o for o in args.only.split(",") if o]
    for name, (M, K0, K1, N, relu) in SHAPES.items():
        if only and not any(o in name for o in only):
            continue
        x0 = torch.randn(M, K0, device=dev)
        W0 = torch.randn(K0, N, device=dev) * 0.05
        x1 = torch.randn(M, K1, device=dev) if K1 else None
        W1 = torch.randn(K1, N, device=dev) * 0.05 if K1 else None
        b = torch.randn(N, device=dev)
        with torch.no_grad():
            def lib():
                y = torch.addmm(b, x0, W0)
                if x1 is not None:
                    y = torch.addmm(y, x1, W1)
                return torch.relu_(y) if relu else y

            def kgx():
                return torch.ops.kgx.dense(x0, W0, x1, W1, b, relu)

            t_lib = timeit(lib, args.reps)
            t_kgx = timeit(kgx, args.reps)
            err = ((kgx().double() - lib().double()).abs() / lib().double().abs().clamp_min(1)).max().item()
        flops = 2 * M * (K0 + K1) * N
        hbm = 4 * M * (K0 + K1 + N)
        print(json.dumps({
            "shape": name, "kgx_ms": round(t_kgx, 4), "lib_fp32_ms": round(t_lib, 4),
            "speedup": round(t_lib / t_kgx, 2), "kgx_alg_TBps": round(hbm / t_kgx / 1e9, 3),
            "kgx_fp32_TFLOPs": round(flops / t_kgx / 1e9, 1),
            "kgx_bf16x6_mfma_frac": round(6 * flops / t_kgx / 1e9 / 2500.0, 3),
            "max_scaled_diff_vs_lib": err,
        }), flush=True)
        del x0, W0, x1, W1
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
