"""bench.py — GCNConv forward on MI355X: aggregated edges/s + achieved HBM GB/s.

Metric (BASELINE.json): "aggregated edges/sec + achieved HBM GB/s, GCNConv fwd,
1/2/4/8 MI355X".  A step is one full layer forward over a device-resident
synthetic R-MAT graph.  The graph's CSR/schedule is built once (graph
preparation, reported separately as graph_build_ms; `cold_layer_ms` is one
forward from a fresh edge_index, CSR + norm + forward, as the reference pays on
every call) and reused across steps, as a GNN training loop over a fixed graph does.

--config ns (default), c2: GCNConv F 128 -> 128, WEAK scaling
    N = 1 : R-MAT 10M nodes / 100M edges (+10M self loops)   [ns]
    N > 1 : every rank owns a contiguous destination range of 10M nodes and
            ~100M edges of one global R-MAT graph of N x 10M nodes / N x 100M
            edges; source rows owned by other ranks arrive by a halo all-to-all
            over RCCL (xGMI), pipelined under the own-source pass.
--config ns_strong: the north-star GCNConv, STRONG scaling: the one 10M / 100M
            graph split by destination range over the N GPUs (N = 1: ns).
--config c4: GINConv sum, F 256, STRONG scaling: one 10M / 100M graph split by
            destination range over the N GPUs (BASELINE.json configs[3]).
--config c5: SAGEConv mean, F 100, STRONG scaling: the ogbn-products-shaped
            2,449,029 / 123,718,280 graph split over the N GPUs (configs[4]).

N > 1 runs one process per GPU.  The driver launches it under
`torch.distributed.run`; a plain `python bench.py --gpus N` (no WORLD_SIZE in
the environment) starts that launcher as a child process before touching the
GPU and relays rank 0's line.  Prints ONE JSON line on stdout (rank 0); every
other byte any rank or library writes goes to stderr.
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for _p in (ROOT, ROOT / "keras-geometric_amd"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

import torch  # noqa: E402  (importing torch does not initialise the GPU)
import torch.distributed as dist  # noqa: E402

METRIC = "aggregated edges/sec + achieved HBM GB/s, GCNConv fwd, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

# name: (layer, nodes, edges, F_in, F_out, scaling); weak: nodes/edges per GPU, strong: the whole graph
CONFIGS = {  # name: (layer, nodes, edges, F_in, F_out, scaling); "tiny" is a control-flow size, not a BASELINE config
    "ns": ("gcn", 10_000_000, 100_000_000, 128, 128, "weak"),
    # the same 10M / 100M north-star graph split by destination range over the N GPUs
    "ns_strong": ("gcn", 10_000_000, 100_000_000, 128, 128, "strong"),
    "c2": ("gcn", 1_000_000, 10_000_000, 128, 128, "weak"),
    "tiny": ("gcn", 100_000, 1_000_000, 128, 128, "weak"),
    "c3": ("gat", 1_000_000, 10_000_000, 128, 128, "weak"),
    "c4": ("gin", 10_000_000, 100_000_000, 256, 256, "strong"),
    "c5": ("sage", 2_449_029, 123_718_280, 100, 100, "strong"),
}
LAYER_NAME = {"gcn": "GCNConv", "gin": "GINConv(sum)", "sage": "SAGEConv(mean)", "gat": "GATv2Conv(8 heads x 16)"}
GAT_HEADS = 8


def b_alg_spmm(n: int, e_agg: int, f: int, weighted: bool, f_out: int | None = None) -> int:
    """4(N+1) + E_agg (4 col + 4 w + 4F src row) + 4 N F out.
    (fused aggregate->transform: gathered rows are F_in wide, outputs F_out.)"""
    f_out = f if f_out is None else f_out
    return 4 * (n + 1) + e_agg * (4 + (4 if weighted else 0) + 4 * f) + 4 * n * f_out


def pmc_traffic(config: str, kernels) -> tuple[float | None, str | None]:
    """HBM bytes per step of the launches in `kernels` (summed: one op may be
    several kernels) from the newest committed rocprofv3 PMC summary
    (profiles/r*/pmc_<config>.json, written by tools/pmc_summary.py), used only
    if every kernel it sums was profiled from the source files being run: each
    kernel entry carries the hash of the .hip file defining it plus its headers
    (older summaries: one hash over all of csrc/)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("pmc_summary", ROOT / "tools" / "pmc_summary.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    kernels = [kernels] if isinstance(kernels, str) else list(kernels)
    for path in sorted(ROOT.glob(f"profiles/r*/pmc_{config}.json"), reverse=True):
        d = json.loads(path.read_text())
        have = d.get("kernels", {})
        if kernels[0] not in have:
            continue
        used = [k for k in kernels if k in have]
        if all("source_hash" in have[k] for k in used):
            if any(have[k]["source_hash"] != mod.kernel_source_hash(k) for k in used):
                continue
        elif d.get("source_hash") != mod.source_hash():
            continue
        return sum(have[k]["traffic_bytes_per_launch"] for k in used), str(path.relative_to(ROOT))
    return None, None


def pmc_step_traffic(name: str) -> tuple[float | None, str | None]:
    """HBM bytes per training step (profiles/r*/pmc_<name>.json, tools/pmc_step.py),
    used only when every kernel of the step was profiled from the sources being run."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("pmc_summary", ROOT / "tools" / "pmc_summary.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for path in sorted(ROOT.glob(f"profiles/r*/pmc_{name}.json"), reverse=True):
        d = json.loads(path.read_text())
        ks = d.get("kernels", {})
        if ks and all(v.get("source_hash") == mod.kernel_source_hash(k) for k, v in ks.items()):
            return d["traffic_bytes_per_step"], str(path.relative_to(ROOT))
    return None, None


def log(msg: str) -> None:
    r = int(os.environ.get("RANK", "0"))
    if r == 0 or int(os.environ.get("WORLD_SIZE", "1")) > 1:  # N > 1: every rank reports its own progress
        print(f"[bench r{r}] {msg}", file=sys.stderr, flush=True)


def host_cpus() -> dict:
    """The host's CPU model and counts (lscpu's fields, read from /proc and sysfs)."""
    model, cores = None, set()
    try:
        phys = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model is None:
                model = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                core = v
            elif not k and phys is not None:
                cores.add((phys, core))
                phys = core = None
    except OSError:
        pass
    quota = None
    try:  # cgroup v2 CPU quota ("max" = none)
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"model": model, "os_cpu_count": os.cpu_count(), "physical_cores": len(cores) or None,
            "affinity_cpus": affinity, "cgroup_cpu_quota": quota}


def cpu_baseline(device: torch.device, repeats: int = 3) -> dict:
    """Time the oracle's op-for-op Keras-torch CPU GCNConv forward (the reference's
    CPU path) on a bounded sample: the C2-shaped 1M-node / 10M-edge R-MAT graph,
    with every CPU this process may run on (os.cpu_count(), limited by its
    affinity mask and cgroup quota when those are smaller)."""
    from keras_geometric_amd import synthetic
    from oracle import reference as R

    n, e, f = 1_000_000, 10_000_000, 128
    info = host_cpus()
    threads = max(1, min(v for v in (info["os_cpu_count"], info["affinity_cpus"],
                                     int(info["cgroup_cpu_quota"] or 1 << 30)) if v))
    torch.set_num_threads(threads)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=device).cpu()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(n, f, generator=g)
    w = (torch.rand(f, f, generator=g) * 2 - 1) * (6.0 / (2 * f)) ** 0.5
    b = torch.zeros(f)
    # SURVEY.md §8(d) / BASELINE.md §3: median of 3 timed forwards after 1 warm-up
    times = []
    for i in range(1 + repeats):
        t0 = time.perf_counter()
        y = R.gcn_forward(x, ei, w, b)
        dt = time.perf_counter() - t0
        del y
        if i:
            times.append(dt)
    med = sorted(times)[len(times) // 2]
    return {
        "value": (e + n) / med,
        "unit": "edges/s",
        "cores": threads,
        "kind": "port",
        "host": info,
        "sample": f"oracle GCNConv fwd (Keras-torch CPU lowering, op for op) on R-MAT N={n} E={e} "
                  f"(+{n} self loops) F {f}->{f}, median of {repeats} timed forwards after 1 warm-up = "
                  f"{med:.2f} s (all: {', '.join(f'{t:.2f}' for t in times)} s), torch threads={threads}",
    }


def _rccl_version():
    try:
        v = torch.cuda.nccl.version()
        return ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 -- diagnostics only
        return None


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(n_gpus: int) -> int:
    """`python bench.py --gpus N` without a launcher: start torch.distributed.run
    as a CHILD process (no GPU has been touched here), one rank per GPU, and
    relay rank 0's JSON line to stdout."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n_gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve()),
           *sys.argv[1:]]
    print(f"[bench] launching {n_gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, env=env)
    out = proc.stdout.decode(errors="replace").splitlines()
    lines = [ln for ln in out if ln.startswith('{"metric"')]
    for ln in out:
        if ln not in lines:
            print(ln, file=sys.stderr)
    if lines:
        print(lines[-1], flush=True)
    elif proc.returncode == 0:
        print("[bench] no result line from rank 0", file=sys.stderr)
        return 1
    return proc.returncode


def _build_single(kind: str, n: int, e: int, f_in: int, f_out: int, seed: int, exact: bool, dev):
    import keras_geometric_amd as kgx
    from keras_geometric_amd import synthetic

    log(f"generating R-MAT N={n} E={e}")
    ei = synthetic.rmat_edge_index(n, e, seed=seed, device=dev)
    x = torch.randn(n, f_in, device=dev)
    if kind == "gcn":
        layer = kgx.GCNConv(f_out, exact=exact)
    elif kind == "gin":
        layer = kgx.GINConv(f_out, aggregator="sum", exact=exact)
    elif kind == "gat":
        layer = kgx.GATv2Conv(f_out // GAT_HEADS, heads=GAT_HEADS, exact=exact)
    else:
        layer = kgx.SAGEConv(f_out, aggregator="mean", exact=exact)
    return ei, x, layer


def _build_sharded(kind: str, n_global: int, e_global: int, f_in: int, f_out: int, seed: int, exact: bool,
                   dev, comm):
    from keras_geometric_amd import distributed as kd

    gcn = kind == "gcn"
    # GATv2 (BASELINE configs[2] is one GPU; N > 1 runs it weak-scaled like NS): self loops, no norm
    sg = kd.ShardedGraph.rmat(n_global, e_global, seed=seed, device=dev, comm=comm, self_loops=kind in ("gcn", "gat"),
                              gcn_norm=gcn, exact=exact, n_features=f_in)
    x = torch.randn(sg.n_local, f_in, device=dev)
    if kind == "gcn":
        layer = kd.ShardedGCNConv(f_out, sg)
    elif kind == "gat":
        layer = kd.ShardedGATv2Conv(f_out // GAT_HEADS, sg, heads=GAT_HEADS)
    elif kind == "gin":
        layer = kd.ShardedGINConv(f_out, sg, aggregator="sum")
    else:
        layer = kd.ShardedSAGEConv(f_out, sg, aggregator="mean")
    return sg, x, layer


def shard_summary(sg, kind: str, f_in: int, f_out: int, exact: bool) -> dict:
    """This rank's exchange, as the N > 1 line reports it per rank: the process
    group as torch.distributed reports it (backend, world size), the exchange
    the tuner chose (kind, K, merge unit) with every candidate's agreed time and
    the tuner's own wall time, and the halo sizes."""
    from keras_geometric_amd import distributed as kd
    from keras_geometric_amd import ops as kops

    world = sg.world
    pp = sg._pp  # exchange plan of the default path (None: pull-only table path or EXACT)
    if pp is not None and pp.kind == "allgather":  # every rank's rows; this rank's own slice is not moved
        n_moved = pp.n_rows * (world - 1) // world
    else:
        n_moved = pp.n_rows if pp is not None else sg.n_halo
    # exchanged row width: X rows (F_in) on the aggregate-first paths, X W rows
    # (F_out) when the GCN layer transforms first (shapes the fused kernel does not take)
    transform_first = kind == "gcn" and (exact or not kops.fused_transform_supported(f_in, f_out) and f_out < f_in)
    f_x = f_out if transform_first else f_in
    init = dist.is_available() and dist.is_initialized()
    return {"backend": dist.get_backend() if init else None,
            "world_size_reported": dist.get_world_size() if init else None,
            "exchange": pp.kind if pp is not None else "pull-table",
            "halo_rows_pull_only": sg.n_halo, "halo_rows": n_moved,
            "halo_rows_pushed_partials": pp.n_push if pp is not None else 0,
            "halo_MB_per_layer": n_moved * f_x * 4 / 1e6,
            "halo_GB_per_layer": n_moved * f_x * 4 / 1e9,
            "halo_chunks": sg.halo_k if sg.halo_k is not None else (len(pp.chunks) if pp else len(sg.chunks)),
            # the tuner's unit, or (tuning skipped: K fixed) the one the merged passes use
            "merge_unit": sg.merge_unit or (os.environ.get("KGX_HALO_MERGE", "step")
                                            if pp is not None and kd.use_merged_halo() else None),
            "exchange_tuning_s": sg.tuning,
            "exchange_tuning_total_s": sg.tuning_s,
            "exchange_tuning_skipped": sg.tuning_skipped}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="ns", choices=sorted(CONFIGS))
    ap.add_argument("--exact", action="store_true", help="EXACT mode (no hub split)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cold", action="store_true", help="skip the cold-graph layer timing")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--train", action="store_true",
                    help="a step is one training step: forward keeping the aggregate P, then backward "
                         "(dx over the transposed graph, dW = P^T dOut, db); GCN, one GPU")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.train and (world > 1 or CONFIGS[args.config][0] != "gcn" or args.exact):
        raise SystemExit("--train: the GCN configs on one GPU (the fused forward + backward)")
    # stdout discipline: the one JSON line goes to the original stdout; anything
    # a library prints (gloo/RCCL banners, warnings) lands on stderr
    result_fd = os.dup(1) if rank == 0 else None
    sys.stdout.flush()
    os.dup2(2, 1)

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
        os.environ.setdefault("KGX_LOG", "1")  # the sharded layers' progress (exchange tuner) on stderr
        if rehearsal:
            dist.init_process_group("gloo")
            from keras_geometric_amd.distributed import HostStagedComm

            comm = HostStagedComm()
        else:
            # RCCL on high-priority streams: its all-to-all kernels get block slots
            # while the own-source pass (a resident grid) holds the rest
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            dist.init_process_group("nccl", device_id=dev, pg_options=opts)
        log(f"process group: backend={dist.get_backend()} world_size={dist.get_world_size()}")

    import keras_geometric_amd as kgx
    from keras_geometric_amd import ops as kops

    kind, n_cfg, e_cfg, f_in, f_out, scaling = CONFIGS[args.config]
    n_global, e_global = (n_cfg * world, e_cfg * world) if scaling == "weak" else (n_cfg, e_cfg)
    torch.manual_seed(args.seed + 17 * rank)
    cold_ms = None
    shard_info = {}

    if world == 1:
        ei, x, layer = _build_single(kind, n_global, e_global, f_in, f_out, args.seed, args.exact, dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.no_grad():
            layer([x, ei])  # build: weights + CSR + schedule (cached)
        torch.cuda.synchronize()
        first_call_ms = (time.perf_counter() - t0) * 1e3
        g = next(reversed(kgx.graph._CACHE.values()))[1]
        # steady-state graph preparation (CSR + schedule), timed warm: once per graph, not per step
        t0 = time.perf_counter()
        kgx.graph.build_csr(ei[0].contiguous(), ei[1].contiguous(), n_global, n_global,
                            self_loops=kind in ("gcn", "gat"), gcn_norm=kind == "gcn", n_features=f_in)
        torch.cuda.synchronize()
        graph_build_ms = (time.perf_counter() - t0) * 1e3
        e_agg, n_rows, max_deg = g.kept, g.n_dst, g.max_degree

        def step():  # the forward (inference) pass: no autograd state kept
            with torch.no_grad():
                return layer([x, ei])

        if args.train:
            x.requires_grad_(True)
            kgx.graph.transpose(g)  # the backward's graph, built once per graph like the forward CSR
            gout = torch.randn(n_rows, f_out, device=dev)

            def step():  # one training step: forward (P kept), backward (dx, dW, db)
                x.grad = None
                layer.zero_grad(set_to_none=True)
                layer([x, ei]).backward(gout)
    else:
        from keras_geometric_amd.distributed import heartbeat

        log(f"world={world}: generating shards of R-MAT N={n_global} E={e_global}")
        t0 = time.perf_counter()
        # a line per rank at least every KGX_HEARTBEAT_S (30 s) while the shard
        # build and the first forward (plans, the KGX_TUNE_BUDGET_S-bounded
        # exchange tuner) run, so a stall names its rank and phase
        with heartbeat(rank, "shard build"):
            sg, x, layer = _build_sharded(kind, n_global, e_global, f_in, f_out, args.seed, args.exact, dev, comm)
            torch.cuda.synchronize()
        log(f"shard graph built in {time.perf_counter() - t0:.1f} s; first forward (plans, exchange tuner)")
        with heartbeat(rank, "first forward (plans, exchange tuner)"), torch.no_grad():
            layer(x)  # build, plans, and (GCN) the halo chunk count measured at the first forward
            torch.cuda.synchronize()
        graph_build_ms = first_call_ms = (time.perf_counter() - t0) * 1e3  # incl. shard generation + halo plan
        e_agg, n_rows, max_deg = sg.graph.kept, sg.n_local, sg.graph.max_degree

        def step():
            with torch.no_grad():
                return layer(x)

        shard_info = shard_summary(sg, kind, f_in, f_out, args.exact)

    if world > 1:
        log(f"first forward done ({first_call_ms / 1e3:.1f} s since the shard build began); warmup")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    kops.EVENT_SINK = []
    split0 = kops.CU_SPLIT_LAUNCHES
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
    cu_split = kops.CU_SPLIT_LAUNCHES > split0
    # aggregation-kernel time per step (N>1: own-source + halo launches, which overlap)
    kern_ms = sum(s.elapsed_time(e) for s, e in events) / args.steps
    launches = len(events) // args.steps

    fused = kind == "gcn" and not args.exact and kops.fused_transform_supported(f_in, f_out)
    # GINConv's (1+eps) x_i + aggr -> Dense in one launch (1 GPU), or in each of the sharded layer's
    # merged halo passes (N > 1: two-table gathers, kgx_spmm_gemm_f256_ex)
    fused_gin = kind == "gin" and not args.exact and kops.fused_transform_supported(f_in, f_out,
                                                                                     two_table=world > 1)
    # SAGEConv's neighbour map in the aggregation's store (1 GPU; the sharded layer keeps kgx_dense)
    fused_sage = kind == "sage" and world == 1 and not args.exact and kops.fused_sage_supported(f_in, f_out)
    train_parts = None
    if kind == "gcn" and args.train:
        # a training step's algorithmic bytes: the forward + writing P
        # [N, F_in]; dx = (A^T dOut) W^T, the same fused op over the transposed graph (E' edges, rows
        # of dOut gathered, N rows of dx written); dW = P^T dOut and db = colsum(dOut): P and dOut
        # read once
        b_fwd = b_alg_spmm(n_rows, e_agg, f_in, weighted=True, f_out=f_out) + 4 * n_rows * f_in
        b_dx = b_alg_spmm(n_rows, e_agg, f_out, weighted=True, f_out=f_in)
        b_dw = 4 * n_rows * (f_in + f_out) + 4 * f_out * (f_in + 1)
        balg = b_fwd + b_dx + b_dw
        kernel = ("spmm_gemm_kernel", "spmm_gemm_short_kernel", "spmm_gemm_tiny_kernel", "spmm_gemm_fixup_kernel",
                  "gemm_tn_ws_kernel", "gemm_tn_finish_kernel")
        ev_ms = [s.elapsed_time(e) for s, e in events]
        per = len(ev_ms) // args.steps if args.steps else 0
        fwd_ms = sum(ev_ms[i] for i in range(0, len(ev_ms), per)) / args.steps if per else None
        dx_ms = sum(ev_ms[i] for i in range(1, len(ev_ms), per)) / args.steps if per >= 2 else None
        train_parts = {"forward_keep_P": {"bytes": b_fwd, "ms": fwd_ms},
                       "dx_transposed": {"bytes": b_dx, "ms": dx_ms},
                       "dW_db": {"bytes": b_dw, "ms": (elapsed / args.steps * 1e3 - fwd_ms - dx_ms)
                                 if fwd_ms is not None and dx_ms is not None else None}}
        for v in train_parts.values():
            v["GBps"] = v["bytes"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] else None
    elif kind == "gcn":
        # SURVEY.md §8d per rank; at N>1 the accumulating halo-chunk passes' re-reads
        # of the rows they add to are implementation overhead, not algorithmic bytes
        balg = b_alg_spmm(n_rows, e_agg, f_in if fused else f_out, weighted=True, f_out=f_out)
        # the fused op: long rows, the short-row suffix (degree <= 7) and the hub fix-up
        kernel = ("spmm_gemm_kernel", "spmm_gemm_short_kernel", "spmm_gemm_tiny_kernel", "spmm_gemm_fixup_kernel") if fused \
            else ("spmm_kernel", "spmm_short_kernel", "spmm_hub_kernel", "spmm_fixup_kernel")
    elif kind == "gat":  # one pass: h_src row per edge, h_dst row + output row per node
        balg = 4 * (n_rows + 1) + e_agg * (4 + 4 * f_out) + 8 * n_rows * f_out
        kernel = ("gatv2_kernel", "gatv2_fixup_kernel")
    elif fused_gin:
        # fused (1+eps) x_i + aggr -> Dense (kgx_spmm_gemm_f256): gathered rows F_in wide, the x_i root row,
        # output rows F_out wide; no [N, F_in] intermediate
        balg = b_alg_spmm(n_rows, e_agg, f_in, weighted=False, f_out=f_out) + 4 * n_rows * f_in
        kernel = ("spmm_gemm256_kernel", "spmm_gemm256_tiny2_kernel", "spmm_gemm256_tiny_kernel",
                  "spmm_gemm256_fixup_kernel")
    elif fused_sage:
        # SAGE mean with W_neigh fused into the aggregation's store (kgx_spmm_gemm, F_in 100):
        # gathered rows F_in wide, output rows F_out wide (the accumulate's re-read of the
        # kgx_dense x W_self + b rows is implementation overhead, not counted)
        balg = b_alg_spmm(n_rows, e_agg, f_in, weighted=False, f_out=f_out)
        kernel = ("spmm_gemm_kernel", "spmm_gemm_short_kernel", "spmm_gemm_tiny_kernel", "spmm_gemm_fixup_kernel")
    else:  # GIN: + the x_i root row of the (1+eps) x_i + aggr epilogue; SAGE mean: plain gather-sum
        balg = b_alg_spmm(n_rows, e_agg, f_in, weighted=False) + (4 * n_rows * f_in if kind == "gin" else 0)
        kernel = ("spmm_kernel", "spmm_short_kernel", "spmm_fixup_kernel")
    step_ms = elapsed / args.steps * 1e3
    if train_parts is not None:  # a training step: its kernels run back to back on one stream
        achieved = balg / (step_ms * 1e-3) / 1e9
    elif world == 1:  # the op's own event time (one launch, or one fork-to-join of a CU-split op)
        achieved = balg / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    else:
        # N > 1: a step is a pipeline of passes, packing and transfers that overlap in time, so
        # the sum of their event times means nothing; a rank's rate is its algorithmic bytes over
        # its own step time
        achieved = balg / (step_ms * 1e-3) / 1e9
    mine = {"rank": rank, "e_agg": e_agg, "rows": n_rows, "ms_per_step": step_ms,
            "aggregation_ms": kern_ms, "launches_per_step": launches, "algorithmic_bytes": balg,
            "roofline_achieved_GBps": achieved, "roofline_frac": achieved / HBM_PEAK_GBS, **shard_info}
    if world > 1:
        # every exchange step's pack-to-landing time (ShardedGraph.link_report), in a few extra
        # steps after the timed ones: the probe's timing events and stream waits cost ~3 % of a
        # step (tools/shard_sim.py --link-probe, profiles/r06/probe/), so they stay out of `value`
        n_probe = min(args.steps, 5)
        sg.link_probe = []
        try:  # a diagnostic: it must never cost the measured line
            for _ in range(n_probe):
                step()
            torch.cuda.synchronize()
            links = sg.link_report(n_probe)
        except Exception as exc:  # noqa: BLE001 -- every rank runs the same code, so all fail alike
            links = []
            mine["link_probe_error"] = f"{type(exc).__name__}: {exc}"[:300]
        mine["link_probe_steps"] = n_probe
        mine["links"] = links
        mine["link_measured_ms_sum"] = sum(r["measured_ms"] for r in links)
        mine["link_modelled_ms_sum_at_400GBps"] = sum(r["modelled_ms_at_400GBps"] for r in links)
        sg.link_probe = None

    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        elapsed = max(r["ms_per_step"] for r in ranks) * args.steps / 1e3
        e_total = float(sum(r["e_agg"] for r in ranks))
        slow = max(ranks, key=lambda r: r["ms_per_step"])  # the rank that sets the step
        achieved, balg = slow["roofline_achieved_GBps"], slow["algorithmic_bytes"]
    else:
        ranks = None
        e_total = float(e_agg)

    ms_per_step = elapsed / args.steps * 1e3
    value = e_total * args.steps / elapsed
    traffic, traffic_src = (None, None)
    if world == 1 and train_parts is None:
        traffic, traffic_src = pmc_traffic(args.config, kernel)
    elif world == 1 and kind == "gcn":
        traffic, traffic_src = pmc_step_traffic(f"{args.config}_train")
    if world == 1 and not args.train:
        if not args.no_cold:
            # cold layer: CSR + (GCN) norm + schedule + forward from a fresh edge_index,
            # what the reference pays on every call (utils/main.py:8-33 per call)
            colds = []
            for _ in range(3):
                kgx.clear_cache()
                ei_c = ei.clone()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                with torch.no_grad():
                    layer([x, ei_c])
                torch.cuda.synchronize()
                colds.append((time.perf_counter() - t0) * 1e3)
                del ei_c
            cold_ms = sorted(colds)[1]
    wl = f"{LAYER_NAME[kind]} fwd, R-MAT {n_global} nodes / {e_global} edges"
    wl += " (+self loops), normalized, bias" if kind == "gcn" else ""
    wl += f", F {f_in}->{f_out}"
    if world > 1:
        wl += (", dst-range shards, RCCL all-gather of node rows" if shard_info.get("exchange") == "allgather"
               else ", dst-range shards, RCCL halo all-to-all") + " pipelined under the own-source pass"
    result = {
        "metric": METRIC if kind == "gcn" else f"aggregated edges/sec + achieved HBM GB/s, {LAYER_NAME[kind]} fwd",
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "fp32",
        "data": f"synthetic R-MAT (a,b,c=.57,.19,.19, seed {args.seed}), x~N(0,1), glorot weights",
        "config": {
            "workload": wl,
            "name": args.config,
            "nodes": n_global,
            "edges": e_global,
            "nodes_per_gpu": n_rows,
            "e_agg_per_gpu": e_agg,
            "max_in_degree": max_deg,
            "features": [f_in, f_out],
            "mode": ("exact" if args.exact else "split-hub")
                    + (", fused aggregate->transform (W on bf16x3-split MFMA, f32-accurate)" if fused or fused_gin
                       else ", W_neigh fused into the aggregation's store (bf16x3-split MFMA), x W_self + b by kgx_dense"
                       if fused_sage else ""),
            "parallelism": f"dst-shard{world}" if world > 1 else "single",
        },
        "edges_per_s_aggregation_kernel": e_total / (kern_ms * 1e-3) if kern_ms > 0 else None,
        "aggregation_ms": kern_ms,
        "aggregation_launches_per_step": launches,
        "graph_build_ms": graph_build_ms,
        "first_call_ms": first_call_ms,
        "cold_layer_ms": cold_ms,
        "roofline": {
            "bound": "hbm",
            "kernel": "+".join(kernel),
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            # FETCH_SIZE x 2 + WRITE_SIZE: L2 <-> fabric bytes, Infinity-Cache (MALL) hits included
            "traffic_kind": "L2-fabric bytes (TCC FETCH_SIZE/WRITE_SIZE, MALL hits included)" if traffic else None,
            "algorithmic_bytes_per_launch": balg,
            # N > 1: the slowest rank's B_alg / its ms_per_step (per-rank values in per_rank)
            "achieved_basis": ("training step: forward (P kept) + dx + dW + db bytes / ms_per_step"
                               if train_parts is not None else "op event time" if world == 1 else
                               "slowest rank: its SURVEY 8(d) bytes / its ms_per_step (pipelined step)"),
            # KGX_FUSED_CU_SPLIT: the op's launches ran side by side on two CU-masked streams (main
            # kernel on 192 CUs, tail launches on 64); `achieved` divides by the op's fork-to-join event
            # time, and rocprof's per-kernel averages of those launches overlap in time
            "concurrent_launches": "cu-split 192/64" if cu_split else None,
        },
        **({"per_rank": ranks} if ranks is not None else shard_info),
    }
    if train_parts is not None:
        result["metric"] = "aggregated edges/sec + achieved HBM GB/s, GCNConv fwd+bwd (training step)"
        result["training_step"] = train_parts
    if world > 1:  # self-diagnosing multi-GPU line: the process group as the library reports it
        result["distributed"] = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                                 "rccl_version": _rccl_version() if dist.get_backend() == "nccl" else None,
                                 "exchange": shard_info.get("exchange"), "halo_chunks": shard_info.get("halo_chunks"),
                                 "merge_unit": shard_info.get("merge_unit"),
                                 "tuning_s": max((r.get("exchange_tuning_total_s") or 0.0) for r in ranks)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and kind == "gcn" and args.config != "tiny" \
            and not args.train:
        log("timing the CPU baseline (oracle, C2-sized sample)")
        del x, layer, ei
        kgx.clear_cache()
        torch.cuda.empty_cache()
        result["cpu_baseline"] = cpu_baseline(dev)
    elif rank == 0:
        result["cpu_baseline"] = None
    if rehearsal:
        result["data"] += " [REHEARSAL: ranks share one GPU, host-staged gloo exchange -- not a measurement]"
    if rank == 0:
        os.write(result_fd, (json.dumps(result) + "\n").encode())
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
