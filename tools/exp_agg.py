"""Aggregation-kernel experiments on the GPU (timing sweeps + PMC calibration).

  python tools/exp_agg.py sweep        # NS graph: exact vs split lengths, event timing
  python tools/exp_agg.py calib        # permutation graph with a known byte count (run under rocprofv3 --pmc)

Not part of the product; a measurement helper whose results feed DESIGN.md.
"""

import json
import sys
import time
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
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def b_alg(n, e, f, weighted=True):
    return 4 * (n + 1) + e * (4 + (4 if weighted else 0) + 4 * f) + 4 * n * f


def sweep(n=10_000_000, e=100_000_000, f=128):
    dev = torch.device("cuda", 0)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    h = torch.randn(n, f, device=dev)
    out = {}
    for T in [0, 256, 512, 1024, 2048, 4096, 8192]:
        g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=True, gcn_norm=True,
                        split_len=T if T else 0)
        ms = timeit(lambda: kops.aggregate(g, h, "sum", weighted=True, exact=(T == 0)))
        out[f"split{T}"] = {"ms": ms, "TBps_alg": b_alg(n, g.kept, f) / ms / 1e9, "n_items": g.n_items,
                            "n_split": g.n_split}
        print(T, out[f"split{T}"], flush=True)
        del g
        torch.cuda.empty_cache()
    for red in ["sum", "mean", "max"]:
        g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=False)
        ms = timeit(lambda: kops.aggregate(g, h, red))
        out[f"unweighted_{red}_noloops"] = {"ms": ms, "TBps_alg": b_alg(n, g.kept, f, False) / ms / 1e9}
        print(red, out[f"unweighted_{red}_noloops"], flush=True)
        del g
    # GEMM for reference
    W = torch.randn(f, f, device=dev)
    out["gemm_ms"] = timeit(lambda: h @ W)
    print(json.dumps(out))


def calib(n=10_000_000, f=128):
    """Each row has exactly one in-edge from a distinct random source: the table is
    read exactly once -> known bytes.  Run under rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE."""
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(0)
    src = torch.randperm(n, device=dev, generator=gen).to(torch.int32)
    dst = torch.arange(n, device=dev, dtype=torch.int32)
    h = torch.randn(n, f, device=dev)
    for name, s in (("perm", src), ("ident", dst.clone())):
        g = G.build_csr(s, dst, n, n, split_len=0)
        torch.cuda.synchronize()
        for _ in range(3):
            kops.aggregate(g, h, "sum", exact=True)
        torch.cuda.synchronize()
        known = n * f * 4 + n * 4 + n * 4 + (n + 1) * 4  # table + col + rows + rowptr
        print(json.dumps({"case": name, "known_read_bytes": known, "write_bytes": n * f * 4}), flush=True)
        time.sleep(0.1)


def ns_once(n=10_000_000, e=100_000_000, f=128, split=512):
    """One NS weighted aggregation timing (env knobs such as KGX_SPMM_HINTS apply)."""
    import os

    dev = torch.device("cuda", 0)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    h = torch.randn(n, f, device=dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=True, gcn_norm=True, split_len=split)
    ms = timeit(lambda: kops.aggregate(g, h, "sum", weighted=True), reps=20)
    print(json.dumps({"hints": os.environ.get("KGX_SPMM_HINTS", "0"), "split": split, "ms": ms,
                      "TBps_alg": b_alg(n, g.kept, f) / ms / 1e9}), flush=True)


def exact_once(n=10_000_000, e=100_000_000, f=128):
    """NS EXACT-mode weighted aggregation (hub rows + dynamic row pickup; env
    knobs KGX_EXACT_FORK, KGX_HUB apply)."""
    import os

    dev = torch.device("cuda", 0)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    h = torch.randn(n, f, device=dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=True, gcn_norm=True)
    ms = timeit(lambda: kops.aggregate(g, h, "sum", weighted=True, exact=True), reps=10)
    print(json.dumps({"lib": os.path.basename(os.environ.get("KGX_LIB", "libkgx.so")),
                      "fork": os.environ.get("KGX_EXACT_FORK", "1"), "exact_ms": round(ms, 4),
                      "TBps_alg": round(b_alg(n, g.kept, f) / ms / 1e9, 3)}), flush=True)


def ns_both(n=10_000_000, e=100_000_000, f=128):
    """NS timing of the unfused weighted aggregation and the fused GCN kernel
    with the library named by KGX_LIB (used by `ab`)."""
    import os

    dev = torch.device("cuda", 0)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    h = torch.randn(n, f, device=dev)
    W = torch.randn(f, f, device=dev) * (1.0 / f) ** 0.5
    split = int(os.environ.get("KGX_EXP_SPLIT", "0")) or None
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=True, gcn_norm=True, split_len=split)
    if os.environ.get("KGX_EXP_SORT"):  # experiment: exact descending-degree item order (stable)
        it = g.items
        pre = int((it[:, 3] >= 0).sum())
        rest = it[pre:]
        order = torch.sort(rest[:, 2] - rest[:, 1], descending=True, stable=True).indices
        g.items = torch.cat([it[:pre], rest[order]]).contiguous()
    ms = timeit(lambda: kops.aggregate(g, h, "sum", weighted=True), reps=20)
    msf = timeit(lambda: kops.aggregate_transform(g, h, W, "sum", weighted=True), reps=20)
    print(json.dumps({"lib": os.path.basename(os.environ.get("KGX_LIB", "libkgx.so")),
                      "env": {k: v for k, v in os.environ.items() if k.startswith("KGX_") and k != "KGX_LIB"},
                      "spmm_ms": round(ms, 3), "fused_ms": round(msf, 3),
                      "TBps_alg": round(b_alg(n, g.kept, f) / ms / 1e9, 3)}), flush=True)


def gat_once(n=1_000_000, e=10_000_000, H=8, C=16):
    """C3-shaped GATv2 aggregation timing with the library named by KGX_LIB."""
    import os

    dev = torch.device("cuda", 0)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=True)
    h = torch.randn(n, H * C, device=dev)
    att = torch.randn(H * C, device=dev)
    ms = timeit(lambda: kops.gatv2_aggregate(g, h, h, att, H, C, 0.2), reps=20)
    b = 4 * (n + 1) + g.kept * (4 + 4 * H * C) + 8 * n * H * C
    print(json.dumps({"lib": os.path.basename(os.environ.get("KGX_LIB", "libkgx.so")), "gat_ms": round(ms, 4),
                      "TBps_alg": round(b / ms / 1e9, 3)}), flush=True)


def ab(specs, rounds=2):
    """A/B over library variants / env knobs, each in its own process, interleaved.
    spec = "libname[:KEY=VAL,...]" with libname "main" or a lib/variants/libkgx_<name>.so.
    This parent never touches the GPU (children are started before any HIP call)."""
    import os
    import subprocess

    for r in range(rounds):
        for spec in specs:
            name, _, kv = spec.partition(":")
            env = dict(os.environ)
            if name != "main":
                env["KGX_LIB"] = str(ROOT / "keras-geometric_amd" / "lib" / "variants" / f"libkgx_{name}.so")
            for item in filter(None, kv.split(",")):
                k, _, v = item.partition("=")
                env[k] = v
            res = subprocess.run([sys.executable, __file__, os.environ.get("KGX_AB_WORK", "both")], env=env, timeout=300,
                                 capture_output=True, text=True)
            line = " | ".join(res.stdout.strip().splitlines()[-2:]) if res.stdout.strip() else res.stderr[-2000:]
            print(f"round{r} {spec}: {line}", flush=True)
            if res.returncode != 0:
                raise SystemExit(res.returncode)


if __name__ == "__main__":
    if sys.argv[1] == "ab":
        ab(sys.argv[2:])
    else:
        {"sweep": sweep, "calib": calib, "ns": ns_once, "both": ns_both, "gat": gat_once,
         "exact": exact_once}[sys.argv[1]]()
