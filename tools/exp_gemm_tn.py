"""Time kgx_gemm_tn (dW = P^T dOut, db = colsum dOut) at the NS training shape
(measurement helper; the form is picked by KGX_TN_LDS / KGX_TN_STAGGER in the environment).

  python tools/exp_gemm_tn.py [--n 10000000 --k 128 --m 128]"""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--m", type=int, default=128)
ap.add_argument("--reps", type=int, default=20)
args = ap.parse_args()
dev = torch.device("cuda", 0)
P = torch.randn(args.n, args.k, device=dev)
D = torch.randn(args.n, args.m, device=dev)
for _ in range(3):
    ops.gemm_tn(P, D, with_db=True)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(args.reps):
    dW, db = ops.gemm_tn(P, D, with_db=True)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / args.reps
ref = (P[:200_000].double().t() @ D[:200_000].double())
part = ops.gemm_tn(P[:200_000], D[:200_000])[0].double()
err = float(((part - ref).abs() / (P[:200_000].double().abs().t() @ D[:200_000].double().abs())).max())
print(json.dumps({"n": args.n, "k": args.k, "m": args.m, "ms": round(ms, 4),
                  "TBps": round(4 * args.n * (args.k + args.m) / ms / 1e9, 3), "rel_err_vs_abs": err,
                  "env": {k: v for k, v in os.environ.items() if k.startswith("KGX_TN")}}), flush=True)
