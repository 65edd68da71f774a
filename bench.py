"""bench.py — GCNConv forward on MI355X: aggregated edges/s + achieved HBM GB/s.

Metric (BASELINE.json): "aggregated edges/sec + achieved HBM GB/s, GCNConv fwd,
1/2/4/8 MI355X".  A step is one full GCNConv forward (node-level X·W GEMM +
the fused kgx aggregation with bias epilogue) over a device-resident synthetic
R-MAT graph.  The graph's CSR/schedule is built once (graph preparation,
reported separately as graph_build_ms) and reused across steps, as a GNN
training loop over a fixed graph does.

N = 1 : north-star workload — R-MAT 10M nodes / 100M edges (+10M self loops),
        F 128 -> 128, fp32.
N > 1 : one process per GPU (torchrun), weak scaling — every rank owns a
        contiguous destination range of 10M nodes and ~100M edges of one global
        R-MAT graph of N x 10M nodes / N x 100M edges; source rows owned by other
        ranks arrive by a halo all-to-all over RCCL (xGMI) every layer.

Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for _p in (ROOT, ROOT / "keras-geometric_amd"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "aggregated edges/sec + achieved HBM GB/s, GCNConv fwd, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (nodes per GPU, edges per GPU, F_in, F_out)
    "ns": (10_000_000, 100_000_000, 128, 128),
    "c2": (1_000_000, 10_000_000, 128, 128),
    "tiny": (100_000, 1_000_000, 128, 128),
}


def b_alg_spmm(n: int, e_agg: int, f: int, weighted: bool, f_out: int | None = None) -> int:
    """4(N+1) + E_agg (4 col + 4 w + 4F src row) + 4 N F out.
    (fused aggregate->transform: gathered rows are F_in wide, outputs F_out.)"""
    f_out = f if f_out is None else f_out
    return 4 * (n + 1) + e_agg * (4 + (4 if weighted else 0) + 4 * f) + 4 * n * f_out


def pmc_traffic(config: str, kernel: str) -> tuple[float | None, str | None]:
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC
    summary (profiles/r*/pmc_<config>.json, written by tools/pmc_summary.py),
    used only if it was profiled from the kernel sources being run."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("pmc_summary", ROOT / "tools" / "pmc_summary.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for path in sorted(ROOT.glob(f"profiles/r*/pmc_{config}.json"), reverse=True):
        d = json.loads(path.read_text())
        if d.get("source_hash") != mod.source_hash() or kernel not in d.get("kernels", {}):
            continue
        return d["kernels"][kernel]["traffic_bytes_per_launch"], str(path.relative_to(ROOT))
    return None, None


def log(msg: str) -> None:
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(device: torch.device, seconds_hint: str) -> dict:
    """Time the oracle's op-for-op Keras-torch CPU GCNConv forward (the reference's
    CPU path) on a bounded sample: the C2-shaped 1M-node / 10M-edge R-MAT graph."""
    from keras_geometric_amd import synthetic
    from oracle import reference as R

    n, e, f = 1_000_000, 10_000_000, 128
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=device).cpu()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(n, f, generator=g)
    w = (torch.rand(f, f, generator=g) * 2 - 1) * (6.0 / (2 * f)) ** 0.5
    b = torch.zeros(f)
    t0 = time.perf_counter()
    y = R.gcn_forward(x, ei, w, b)
    dt = time.perf_counter() - t0
    del y
    return {
        "value": (e + n) / dt,
        "unit": "edges/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle GCNConv fwd (Keras-torch CPU lowering, op for op) on R-MAT N={n} E={e} "
                  f"(+{n} self loops) F {f}->{f}, 1 timed forward = {dt:.2f} s, torch threads={threads}"
                  f"{seconds_hint}",
    }


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="ns", choices=sorted(CONFIGS))
    ap.add_argument("--exact", action="store_true", help="EXACT mode (no hub split)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 with torch.distributed.run")
    # KGX_BENCH_REHEARSAL=1 (test only, one-GPU box): all ranks share cuda:0 and
    # the exchange is staged through host memory over gloo -- exercises the N>1
    # control flow and halo plumbing where RCCL cannot run (one GPU); never a
    # measurement.
    rehearsal = os.environ.get("KGX_BENCH_REHEARSAL", "0") == "1"
    gpu = 0 if rehearsal else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    comm = None
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo")
            from keras_geometric_amd.distributed import HostStagedComm

            comm = HostStagedComm()
        else:
            dist.init_process_group("nccl", device_id=dev)

    import keras_geometric_amd as kgx
    from keras_geometric_amd import ops as kops
    from keras_geometric_amd import synthetic

    n_local, e_local, f_in, f_out = CONFIGS[args.config]
    torch.manual_seed(args.seed + 17 * rank)

    if world == 1:
        log(f"generating R-MAT N={n_local} E={e_local}")
        ei = synthetic.rmat_edge_index(n_local, e_local, seed=args.seed, device=dev)
        x = torch.randn(n_local, f_in, device=dev)
        layer = kgx.GCNConv(f_out, exact=args.exact)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        layer([x, ei])  # build: weights + CSR + schedule (cached)
        torch.cuda.synchronize()
        first_call_ms = (time.perf_counter() - t0) * 1e3
        # steady-state graph preparation (CSR + schedule), timed warm: once per graph, not per step
        t0 = time.perf_counter()
        kgx.graph.build_csr(ei[0].contiguous(), ei[1].contiguous(), n_local, n_local, self_loops=True,
                            gcn_norm=True, n_features=f_out)
        torch.cuda.synchronize()
        graph_build_ms = (time.perf_counter() - t0) * 1e3
        g = next(iter(kgx.graph._CACHE.values()))[1]
        e_agg, n_rows, max_deg = g.kept, g.n_dst, g.max_degree
        def step():  # the forward (inference) pass: no autograd state kept
            with torch.no_grad():
                return layer([x, ei])

        shard_info = {}
    else:
        from keras_geometric_amd import distributed as kd

        log(f"world={world}: generating shards of R-MAT N={n_local * world} E={e_local * world}")
        t0 = time.perf_counter()
        sg = kd.ShardedGraph.rmat(n_local * world, e_local * world, seed=args.seed, device=dev, comm=comm,
                                  self_loops=True, gcn_norm=True, exact=args.exact)
        x = torch.randn(sg.n_local, f_in, device=dev)
        layer = kd.ShardedGCNConv(f_out, sg)
        layer(x)
        torch.cuda.synchronize()
        graph_build_ms = first_call_ms = (time.perf_counter() - t0) * 1e3  # incl. shard generation + halo plan
        e_agg, n_rows, max_deg = sg.graph.kept, sg.n_local, sg.graph.max_degree
        def step():
            with torch.no_grad():
                return layer(x)

        pp = sg._pp  # push-pull halo plan of the default path (None: pull-only or EXACT)
        n_moved = pp.n_rows if pp is not None else sg.n_halo
        shard_info = {"halo_rows_pull_only_per_rank": sg.n_halo, "halo_rows_per_rank": n_moved,
                      "halo_rows_pushed_partials": pp.n_push if pp is not None else 0,
                      "halo_MB_per_layer": n_moved * f_in * 4 / 1e6,
                      "halo_chunks": sg.halo_k if sg.halo_k is not None else len(sg.chunks),
                      "halo_chunk_tuning_s": sg.tuning}

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    kops.EVENT_SINK = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    events = kops.EVENT_SINK
    kops.EVENT_SINK = None
    # kernel time per step (N>1 default path: own-source + halo-source launches)
    kern_ms = sum(s.elapsed_time(e) for s, e in events) / args.steps
    launches = len(events) // args.steps

    if world > 1:
        rdev = torch.device("cpu") if rehearsal else dev
        t = torch.tensor([elapsed, kern_ms], device=rdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        tot = torch.tensor([e_agg], device=rdev, dtype=torch.float64)
        dist.all_reduce(tot)
        e_total = float(tot[0])
    else:
        e_total = float(e_agg)

    ms_per_step = elapsed / args.steps * 1e3
    value = e_total * args.steps / elapsed
    from keras_geometric_amd import ops as _ops

    fused = not args.exact and _ops.fused_transform_supported(f_in, f_out)
    # SURVEY.md §8d per rank; at N>1 the accumulating halo-chunk passes' re-reads
    # of the rows they add to are implementation overhead, not algorithmic bytes
    balg = b_alg_spmm(n_rows, e_agg, f_in if fused else f_out, weighted=True, f_out=f_out)
    achieved = balg / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = (None, None)
    if world == 1:
        traffic, traffic_src = pmc_traffic(args.config, "spmm_gemm_kernel" if fused else "spmm_kernel")
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": f"synthetic R-MAT (a,b,c=.57,.19,.19, seed {args.seed}), x~N(0,1), glorot weights",
        "config": {
            "workload": f"GCNConv fwd (normalized, self loops, bias), R-MAT "
                        f"{n_local * world} nodes / {e_local * world} edges (+self loops), "
                        f"F {f_in}->{f_out}" + (", dst-range shards, RCCL halo all-to-all overlapped with the own-source part"
                                                 if world > 1 else ""),
            "nodes_per_gpu": n_local,
            "edges_per_gpu": e_local,
            "e_agg_per_gpu": e_agg,
            "max_in_degree": max_deg,
            "features": [f_in, f_out],
            "mode": ("exact" if args.exact else "split-hub") + (", fused aggregate->transform (W on bf16x3-split MFMA, f32-accurate)"
                                                                 if fused else ", X.W GEMM then aggregate"),
            "parallelism": f"dst-shard{world}" if world > 1 else "single",
        },
        "edges_per_s_aggregation_kernel": e_agg * world / (kern_ms * 1e-3),
        "aggregation_ms": kern_ms,
        "aggregation_launches_per_step": launches,
        "graph_build_ms": graph_build_ms,
        "first_call_ms": first_call_ms,
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": balg,
        },
        **shard_info,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "ns":
        log("timing the CPU baseline (oracle, C2-sized sample)")
        del x, layer, ei
        kgx.clear_cache()
        torch.cuda.empty_cache()
        result["cpu_baseline"] = cpu_baseline(dev, "")
    elif rank == 0:
        result["cpu_baseline"] = None
    if rehearsal:
        result["data"] += " [REHEARSAL: ranks share one GPU, host-staged gloo exchange -- not a measurement]"
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
