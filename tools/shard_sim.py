"""One rank's device work of a sharded layer, on one GPU.

  python tools/shard_sim.py [--config ns|c4|c5] [--world 8] [--chunks 1,2,4,8]
                            [--exchange halo,allgather] [--link-gbps 400] [--steps 10]

ns: GCN weak scaling (every rank 10M nodes / 100M edges of one N x 10M graph);
c4: GIN-sum 10M / 100M F256 and c5: SAGE-mean 2.45M / 123.7M F100, strong
scaling (rank 0's shard of the one graph), as bench.py --config c4 / c5.

Builds rank 0's shard of the P x 10M-node / P x 100M-edge R-MAT graph as
bench.py --gpus P does, but with a loopback comm: the peers' requests are
synthetic (this rank's own requests mirrored, folded into its range, so as
many rows as it requests from them) and the all-to-all is an asynchronous
device copy on the side stream.  So the timed step is the
rank's compute side of ShardedGCNConv -- send-row packing, the own-source
pass and one accumulating pass per halo chunk -- with the exchange itself
free.  It prices the chunked pipeline's extra passes against one halo pass
(DESIGN.md §6); the link time has to be added from the halo bytes.
A measurement helper, not part of the product.
"""

import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import distributed as kd  # noqa: E402
from keras_geometric_amd import ops as kops  # noqa: E402


TIMELINE: list | None = None  # (what, start event, end event, bytes) when --timeline


def _mark():
    if TIMELINE is None:
        return None
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    return ev


def _note(what, t0, t1, nbytes=0):
    if TIMELINE is not None and t0 is not None:
        TIMELINE.append((what, t0, t1, nbytes))


class _EventWork:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class LoopbackComm(kd.TorchComm):
    """Rank 0 of a `world`-rank job whose peers mirror it (measurement stand-in).

    link_gbps > 0 models the links: each started all-to-all runs on one "link"
    stream (chunks in order, as RCCL's own stream does) after the send rows are
    ready, and occupies it for bytes / link_gbps (a spin of one wave, so the
    modelled transfer takes time but no HBM bandwidth) before its copy lands."""

    def __init__(self, world: int, n_local: int, link_gbps: float = 0.0, cycles_per_ms: float = 0.0,
                 free_exchange: bool = False):
        self.w, self.n_local = world, n_local
        self.link_gbps, self.cycles_per_ms = link_gbps, cycles_per_ms
        self.link = None
        # free_exchange: after a buffer's first landing (real values), later exchanges into it
        # move nothing -- the step is the rank's compute alone; otherwise the loopback copy
        # (a local read + write of every received byte) stands in for RCCL's receive writes
        self.free_exchange, self._landed = free_exchange, set()

    def _land(self, out) -> bool:
        """True when this exchange should copy (always, unless free_exchange and out has landed once)."""
        if not self.free_exchange:
            return True
        key = (out.data_ptr(), out.numel())
        if key in self._landed:
            return False
        self._landed.add(key)
        return True

    def rank(self):
        return 0

    def world(self):
        return self.w

    def all_to_all_single(self, out, inp, out_splits=None, in_splits=None):
        if out.dtype == torch.int64 and out_splits is None:  # the count exchange: symmetric peers
            out.copy_(inp)
        elif out.dtype == torch.int64:  # peers' requests mirror ours, folded into this rank's range
            out.copy_(inp.view_as(out) % self.n_local)
        elif out.numel():
            out.copy_(inp.view_as(out))

    def all_to_all_start(self, out, inp, out_splits=None, in_splits=None):
        """Asynchronous like RCCL's: the copy is queued on the current (side)
        stream and wait() makes the then-current stream wait for it."""
        if self.link_gbps <= 0:
            if self._land(out):
                self.all_to_all_single(out, inp, out_splits, in_splits)
            ev = torch.cuda.Event()
            ev.record()
            return _EventWork(ev)
        if self.link is None:
            self.link = torch.cuda.Stream(priority=-1)
        ready = torch.cuda.Event()
        ready.record()
        self.link.wait_event(ready)
        with torch.cuda.stream(self.link):
            ms = out.numel() * out.element_size() / (self.link_gbps * 1e6)
            t0 = _mark()
            if ms > 0:
                torch.cuda._sleep(int(ms * self.cycles_per_ms))
            if self._land(out):
                self.all_to_all_single(out, inp, out_splits, in_splits)
            _note("link", t0, _mark(), out.numel() * out.element_size())
            inp.record_stream(self.link)
            out.record_stream(self.link)
            ev = torch.cuda.Event()
            ev.record()
        return _EventWork(ev)

    def broadcast(self, t, src=0):
        pass

    def all_gather(self, out, inp):
        """Peers mirror this rank: every rank's slice is a copy of ours."""
        out.view(self.w, *inp.shape).copy_(inp.unsqueeze(0).expand(self.w, *inp.shape))

    def all_gather_start(self, out, inp):
        """As all_to_all_start: the modelled link time covers the (world-1)/world received share."""
        if self.link_gbps <= 0:
            if self._land(out):
                self.all_gather(out, inp)
            ev = torch.cuda.Event()
            ev.record()
            return _EventWork(ev)
        if self.link is None:
            self.link = torch.cuda.Stream(priority=-1)
        ready = torch.cuda.Event()
        ready.record()
        self.link.wait_event(ready)
        with torch.cuda.stream(self.link):
            ms = out.numel() * out.element_size() * (self.w - 1) / self.w / (self.link_gbps * 1e6)
            if ms > 0:
                torch.cuda._sleep(int(ms * self.cycles_per_ms))
            if self._land(out):
                self.all_gather(out, inp)
            inp.record_stream(self.link)
            out.record_stream(self.link)
            ev = torch.cuda.Event()
            ev.record()
        return _EventWork(ev)


CONFIGS = {  # name: (layer, nodes, edges, features, scaling) -- bench.py's configs
    "ns": ("gcn", 10_000_000, 100_000_000, 128, "weak"),
    # the north-star 10M / 100M graph split over the world (bench.py --config ns_strong)
    "ns_strong": ("gcn", 10_000_000, 100_000_000, 128, "strong"),
    "c4": ("gin", 10_000_000, 100_000_000, 256, "strong"),
    "c5": ("sage", 2_449_029, 123_718_280, 100, "strong"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ns", choices=sorted(CONFIGS),
                    help="ns: GCN weak (N x 10M / N x 100M); c4: GIN-sum 10M/100M F256 strong; "
                         "c5: SAGE-mean 2.45M/123.7M F100 strong")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--chunks", default="1,2,4,8")
    ap.add_argument("--exchange", default="halo", help="halo,pull,allgather: exchanges to run")
    ap.add_argument("--push", default="1", help="KGX_HALO_PUSH values to run (0: pull-only halo)")
    ap.add_argument("--merged", default="1", help="KGX_HALO_MERGED values to run (0: round-2 own pass + chunk passes)")
    ap.add_argument("--merge-unit", default="step", help="KGX_HALO_MERGE values: step, chunk")
    ap.add_argument("--a-late", default="auto",
                    help="KGX_HALO_A_LATE values (1: own-only rows after the merged pass; auto: the layer's rule)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--share-den", default="8",
                    help="KGX_SHARE_DEN values timed on each built shard (the overlapped passes leave 1/den of "
                         "the block slots to the side stream)")
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--edges", type=int, default=None)
    ap.add_argument("--link-gbps", type=float, default=0.0,
                    help="model the exchange: per-GPU receive rate in GB/s (0: no link time)")
    ap.add_argument("--timeline", action="store_true",
                    help="print one more line per run: every kgx op, packing copy and modelled transfer of the "
                         "last timed step as [start, end] ms from the step's start (which stream: 'link' = the "
                         "modelled transfer; ops in issue order)")
    ap.add_argument("--free-exchange", action="store_true",
                    help="received buffers land once (a loopback device copy), later exchanges copy nothing: "
                         "with --link-gbps 0 the step is the rank's compute alone; with a link rate the "
                         "modelled transfer time stands for RCCL's receive (default: a loopback device copy "
                         "per exchange, after the modelled link time)")
    ap.add_argument("--link-probe", action="store_true",
                    help="time every exchange step's pack-to-landing in the timed steps as bench.py does at "
                         "N > 1 (ShardedGraph.link_probe / link_report) and add it to the JSON line")
    args = ap.parse_args()
    layer_kind, n_cfg, e_cfg, F, scaling = CONFIGS[args.config]
    n_cfg = args.nodes or n_cfg
    e_cfg = args.edges or e_cfg
    dev = torch.device("cuda", 0)
    P = args.world
    n_glob, e_glob = (n_cfg * P, e_cfg * P) if scaling == "weak" else (n_cfg, e_cfg)
    cycles_per_ms = 0.0
    if args.link_gbps > 0:  # calibrate torch.cuda._sleep's cycles against events
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(10_000_000)
        t0.record()
        torch.cuda._sleep(100_000_000)
        t1.record()
        torch.cuda.synchronize()
        cycles_per_ms = 100_000_000 / t0.elapsed_time(t1)
    runs = [(x, m, p, int(v), mu, al) for x in args.exchange.split(",") for m in args.merged.split(",")
            for p in args.push.split(",") for v in args.chunks.split(",") for mu in args.merge_unit.split(",")
            for al in args.a_late.split(",")]
    for exchange, merged, push, K, unit, a_late in runs:
        if exchange == "allgather" and (push == "0" or merged == "0"):
            continue  # the all-gather has neither pulls nor pushes, and always runs merged
        if merged == "0" and (unit != "step" or a_late == "1"):
            continue
        os.environ["KGX_HALO_PUSH"] = push
        os.environ["KGX_HALO_MERGED"] = merged
        os.environ["KGX_HALO_MERGE"] = unit
        if a_late in ("0", "1", "2"):
            os.environ["KGX_HALO_A_LATE"] = a_late
        else:
            os.environ.pop("KGX_HALO_A_LATE", None)
        n_local = kd.equal_bounds(n_glob, P)[1]
        comm = LoopbackComm(P, n_local, args.link_gbps, cycles_per_ms, free_exchange=args.free_exchange)
        gcn = layer_kind == "gcn"
        sg = kd.ShardedGraph.rmat(n_glob, e_glob, seed=0, device=dev, comm=comm, self_loops=gcn, gcn_norm=gcn,
                                  halo_chunks=K, n_features=F)
        sg.exchange = exchange
        x = torch.randn(sg.n_local, F, device=dev)
        if layer_kind == "gcn":
            layer = kd.ShardedGCNConv(F, sg)
        elif layer_kind == "gin":
            layer = kd.ShardedGINConv(F, sg, aggregator="sum")
        else:
            layer = kd.ShardedSAGEConv(F, sg, aggregator="mean")
        for den in args.share_den.split(","):
            os.environ["KGX_SHARE_DEN"] = den
            with torch.no_grad():
                layer(x)
                g_own, g_chunks = sg.own_halo_parts()
                for _ in range(2):
                    layer(x)
                torch.cuda.synchronize()
                if args.timeline:  # one extra, separately recorded step
                    global TIMELINE
                    TIMELINE = []
                    kops.EVENT_SINK = []
                    ref = torch.cuda.Event(enable_timing=True)
                    ref.record()
                    gr = kops.gather_rows

                    def timed_gather(table, rows):
                        t0 = _mark()
                        out = gr(table, rows)
                        _note("pack rows", t0, _mark(), 2 * out.numel() * 4)
                        return out

                    kops.gather_rows = timed_gather
                    be = sg.backend
                    saved = {}
                    for name in ("aggregate_transform", "aggregate", "aggregate_accumulate"):
                        fn = getattr(be, name)
                        saved[name] = fn

                        def wrapped(g, *a, _fn=fn, _name=name, **kw):
                            t0 = _mark()
                            out = _fn(g, *a, **kw)
                            what = f"{_name}{'(2 tables)' if kw.get('x2') is not None else ''}" \
                                   f"{'' if kw.get('accumulate', True) or _name != 'aggregate_transform' else ' overwrite'}"
                            _note(f"{what} items={g.n_items} edges={g.kept}", t0, _mark())
                            return out

                        setattr(be, name, wrapped)
                    kops.EVENT_SINK = None
                    try:
                        layer(x)
                        end = torch.cuda.Event(enable_timing=True)
                        end.record()
                        torch.cuda.synchronize()
                    finally:
                        kops.gather_rows = gr
                        for name, fn in saved.items():
                            setattr(be, name, fn)
                    items = TIMELINE
                    TIMELINE = None
                    tl = sorted(([w, round(ref.elapsed_time(a), 3), round(ref.elapsed_time(b), 3), nb]
                                 for w, a, b, nb in items), key=lambda r: r[1])
                    print(json.dumps({"timeline": tl, "step_ms": round(ref.elapsed_time(end), 3),
                                      "share_den": int(den), "chunks": K, "link_gbps": args.link_gbps,
                                      "a_late": a_late, "config": args.config, "world": P,
                                      "env": {k: v for k, v in os.environ.items() if k.startswith("KGX_")}}),
                          flush=True)
                kops.EVENT_SINK = []
                if args.link_probe:
                    sg.link_probe = []
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record()
                for _ in range(args.steps):
                    layer(x)
                t1.record()
                torch.cuda.synchronize()
                links = sg.link_report(args.steps) if args.link_probe else None
                sg.link_probe = None
            ev = kops.EVENT_SINK
            kops.EVENT_SINK = None
            per = len(ev) // args.steps
            launch_ms = [sum(ev[i * per + j][0].elapsed_time(ev[i * per + j][1]) for i in range(args.steps))
                         / args.steps for j in range(per)]
            pp = sg._pp
            if pp is not None:
                g_chunks = pp.parts
            recv_rows = (pp.n_rows * (P - 1) // P if pp.kind == "allgather" else pp.n_rows) if pp else sg.n_halo
            print(json.dumps({
                "config": args.config, "layer": layer_kind, "scaling": scaling, "nodes": n_glob, "edges": e_glob,
                "features": F, "world": P, "exchange": pp.kind if pp else "pull", "chunks": K,
                "push_pull": pp is not None and pp.kind == "halo", "merged": merged == "1", "merge_unit": unit,
                "a_late": a_late, "share_den": int(den),
                "link_gbps": args.link_gbps,
                "exchange_model": ("modelled-link" if args.link_gbps > 0 else "free" if comm.free_exchange
                                   else "loopback-copy") + ("" if args.link_gbps <= 0 or not comm.free_exchange
                                                            else ", no local copy"), "step_ms": round(t0.elapsed_time(t1) / args.steps, 3),
                "launch_ms": [round(v, 3) for v in launch_ms],
                **({"links": links} if links is not None else {}),
                "own_edges": g_own.kept, "chunk_edges": [g.kept for g in g_chunks],
                "halo_rows_pull_only": sg.n_halo, "halo_rows": pp.n_rows if pp else sg.n_halo,
                "received_MB": recv_rows * F * 4 / 1e6,
                "pulled": pp.n_pull if pp else sg.n_halo, "pushed": pp.n_push if pp else 0,
                "chunk_items": [g.n_items for g in g_chunks], "n_local": sg.n_local,
            }), flush=True)
        os.environ.pop("KGX_SHARE_DEN", None)
        del sg, layer, x, g_own, g_chunks
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
