"""Sharded propagation on the GPU with the HIP backend.

The GPU box has one MI355X and GPU tests must not start processes, so the
ranks run as THREADS of the test process sharing cuda:0, with a thread-hub
comm shim standing in for RCCL's all-to-all (test infrastructure).  Every
device operation — R-MAT shard generation, shard CSR build with halo sources,
GCN norms from exchanged degrees, halo row packing, fused aggregation — runs
through the kgx HIP kernels as it does with RCCL.  Each rank keeps its rows'
edges in global input order, so EXACT-mode sharded propagation must equal the
single-GPU result bit for bit."""

import threading

import numpy as np
import pytest
import torch

from keras_geometric_amd import distributed as kd

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]

N, E, F = 50_000, 600_000, 64


class ThreadHub:
    def __init__(self, world):
        self.world = world
        self.barrier = threading.Barrier(world, timeout=120)
        self.slots = [None] * world


class ThreadComm(kd.TorchComm):
    def __init__(self, hub, rank):
        self.hub, self.r = hub, rank

    def rank(self):
        return self.r

    def world(self):
        return self.hub.world

    def all_to_all_single(self, out, inp, out_splits=None, in_splits=None):
        w = self.hub.world
        in_splits = in_splits or [inp.shape[0] // w] * w
        self.hub.slots[self.r] = [c.clone() for c in torch.split(inp, list(in_splits))]
        # the clones are queued on this rank's stream: they must have run before
        # a peer (another thread, another stream) reads them
        torch.cuda.synchronize()
        self.hub.barrier.wait()
        parts = [self.hub.slots[src][self.r] for src in range(w)]
        if out.numel():
            out.copy_(torch.cat(parts))
        torch.cuda.synchronize()
        self.hub.barrier.wait()

    def all_to_all_start(self, out, inp, out_splits=None, in_splits=None):
        self.all_to_all_single(out, inp, out_splits, in_splits)  # synchronous: rows ordered on return
        return None

    def all_gather(self, out, inp):
        w = self.hub.world
        self.all_to_all_single(out, inp.repeat(w, *([1] * (inp.dim() - 1))).contiguous())

    def all_gather_start(self, out, inp):
        self.all_gather(out, inp)
        return None

    def all_reduce(self, t):
        self.hub.slots[self.r] = t.detach().clone()
        torch.cuda.synchronize()
        self.hub.barrier.wait()
        total = self.hub.slots[0].clone()
        for i in range(1, self.hub.world):  # rank order: the same bits on every rank
            total += self.hub.slots[i]
        torch.cuda.synchronize()
        self.hub.barrier.wait()
        t.copy_(total)
        torch.cuda.synchronize()

    def broadcast(self, t, src=0):
        if self.r == src:
            self.hub.slots[src] = t.detach().clone()
            torch.cuda.synchronize()
        self.hub.barrier.wait()
        t.copy_(self.hub.slots[src])
        torch.cuda.synchronize()
        self.hub.barrier.wait()


class AsyncThreadComm(ThreadComm):
    """all_to_all_start with RCCL's stream semantics: the copy runs on this
    rank's own copy stream after the send rows are ready (an event on every
    rank's calling stream), the peers' send buffers are recorded on that stream
    (as ProcessGroupNCCL does) and wait() makes the then-current stream wait for
    the copy.  delay_cycles > 0 spins the copy stream first, so a missing
    wait(), a missing wait_stream or a reused send / halo buffer reads rows
    that have not landed and the result comes out wrong."""

    def __init__(self, hub, rank, delay_cycles=0):
        super().__init__(hub, rank)
        self.delay = delay_cycles
        self.copy_stream = None
        self.started = 0

    def all_to_all_start(self, out, inp, out_splits=None, in_splits=None):
        w = self.hub.world
        if self.copy_stream is None:
            self.copy_stream = torch.cuda.Stream(device=inp.device)
        in_splits = list(in_splits or [inp.shape[0] // w] * w)
        out_splits = list(out_splits or [out.shape[0] // w] * w)
        ready = torch.cuda.Event()
        ready.record()  # on the caller's current stream: the packed send rows
        self.hub.slots[self.r] = (torch.split(inp, in_splits), ready)
        self.hub.barrier.wait()
        peers = list(self.hub.slots)
        self.hub.barrier.wait()
        cs = self.copy_stream
        for _, ev in peers:
            cs.wait_event(ev)
        with torch.cuda.stream(cs):
            if self.delay:
                torch.cuda._sleep(self.delay)
            off = 0
            for p, (parts, _) in enumerate(peers):
                src = parts[self.r]
                src.record_stream(cs)
                if src.numel():
                    out[off: off + out_splits[p]].copy_(src)
                off += out_splits[p]
        out.record_stream(cs)
        done = torch.cuda.Event()
        done.record(cs)
        self.started += 1

        class Work:
            def wait(self_inner):
                torch.cuda.current_stream().wait_event(done)

        return Work()

    def all_gather_start(self, out, inp):
        w = self.hub.world
        n = inp.shape[0]
        return self.all_to_all_start(out, inp.repeat(w, *([1] * (inp.dim() - 1))), [n] * w, [n] * w)


COMMS = {"sync": lambda hub, r: ThreadComm(hub, r),
         "async": lambda hub, r: AsyncThreadComm(hub, r),
         "async_delayed": lambda hub, r: AsyncThreadComm(hub, r, delay_cycles=20_000_000)}


def _run_rank(rank, hub, dev, x, out):
    try:
        comm = ThreadComm(hub, rank)
        sg = kd.ShardedGraph.rmat(N, E, seed=5, device=dev, comm=comm, exact=True, n_features=F)
        xl = x[sg.lo: sg.lo + sg.n_local]
        s = sg.propagate(xl, "sum")
        m = sg.propagate(xl, "max")
        layer = kd.ShardedGCNConv(32, sg)
        with torch.no_grad():
            y = layer(xl)
            sg.exact = False  # default path (F = 64, unfused): X W, then the push-pull halo pipelined under the own pass
            y2 = layer(xl)
        torch.cuda.synchronize()
        out[rank] = (s.cpu().numpy(), m.cpu().numpy(), y.detach().cpu().numpy(), layer.kernel.detach().cpu().numpy(),
                     sg.n_halo, y2.detach().cpu().numpy())
    except BaseException as e:  # surface worker failures in the test thread
        out[rank] = e
        hub.barrier.abort()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_hip_equals_single_gpu(world, dev):
    import keras_geometric_amd as kgx
    from keras_geometric_amd import synthetic

    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, F, generator=g).to(dev)
    hub = ThreadHub(world)
    res = {}
    threads = [threading.Thread(target=_run_rank, args=(r, hub, dev, x, res)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    for r in range(world):
        if isinstance(res.get(r), BaseException):
            raise res[r]
    assert all(res[r][4] > 0 for r in range(world))  # real halo traffic
    ei = synthetic.rmat_edge_index(N, E, seed=5, device=dev)
    ei_loops = kgx.add_self_loops(ei, N)  # the shard graph carries GCN's self loops (appended last)
    for k, aggr in ((0, "sum"), (1, "max")):
        ref = kgx.MessagePassing(aggregator=aggr, exact=True)([x, ei_loops]).cpu().numpy()
        got = np.concatenate([res[r][k] for r in range(world)])
        np.testing.assert_array_equal(got, ref)
    layer = kgx.GCNConv(32, exact=True)
    layer([x, ei])
    layer.set_weights([res[0][3], np.zeros(32, np.float32)])
    ref = layer([x, ei]).detach().cpu().numpy()
    got = np.concatenate([res[r][2] for r in range(world)])
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() <= 1e-5
    got = np.concatenate([res[r][5] for r in range(world)])  # overlapped, split-sum path
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() <= 1e-5


F_FUSED = 128  # the fused aggregate->transform kernel's F_in: the default (chunk-pipelined) GCN path


def _run_fused_rank(rank, hub, dev, x, chunks, out, comm_kind="sync"):
    try:
        comm = COMMS[comm_kind](hub, rank)
        sg = kd.ShardedGraph.rmat(N, E, seed=8, device=dev, comm=comm, n_features=F_FUSED, halo_chunks=chunks)
        xl = x[sg.lo: sg.lo + sg.n_local]
        layer = kd.ShardedGCNConv(128, sg)  # F_out >= F_in = 128: the fused, chunk-pipelined path
        with torch.no_grad():
            y = layer(xl)
            if comm_kind != "sync":  # forwards back to back reuse the persistent halo buffer
                y_next = layer(xl)
                x_other = torch.randn_like(xl)
                layer(x_other)  # different rows in flight through the same buffers
                y_last = layer(xl)
                torch.cuda.synchronize()
                assert torch.equal(y_next, y) and torch.equal(y_last, y), "halo buffer reuse across forwards"
                assert comm.started > 0
        torch.cuda.synchronize()
        assert (sg._pp is not None) == kd.use_push_pull()
        g_own, g_chunks = sg.own_halo_parts()
        covered = all(bool((g.items[:, 2] > g.items[:, 1]).all()) for g in g_chunks if g.n_items)
        whole = g_own.kept + sum(g.kept for g in g_chunks) == sg.graph.kept
        if sg._pp is not None:  # push-pull: every halo row is a source row or a pushed partial
            pp = sg._pp
            covered = covered and all(bool((g.items[:, 2] > g.items[:, 1]).all()) for g in pp.parts if g.n_items)
            whole = whole and pp.n_rows == pp.n_pull + pp.n_push == pp.chunks[-1].hi and len(pp.chunks) == chunks
        out[rank] = (y.detach().cpu().numpy(), layer.kernel.detach().cpu().numpy(), len(g_chunks), whole, covered)
    except BaseException as e:
        out[rank] = e
        hub.barrier.abort()


@pytest.mark.parametrize("world,chunks,push,comm", [(2, 1, "1", "sync"), (2, 4, "1", "sync"), (3, 3, "1", "sync"),
                                                    (2, 4, "0", "sync"), (2, 1, "1", "async_delayed"),
                                                    (2, 4, "1", "async_delayed"), (3, 3, "1", "async"),
                                                    (2, 4, "0", "async_delayed")])
def test_sharded_gcn_chunked_halo_pipeline(world, chunks, push, comm, dev, monkeypatch):
    """The default multi-GPU GCN path on the HIP kernels: owners pack pulled
    rows and pushed partial sums in one weighted-sum pass (push="1"; "0":
    pull-only halo), the own-source fused pass runs, then one accumulating
    fused pass per halo chunk (only over the rows the chunk touches); equals
    the single-GPU layer within the north-star tolerance (re-associated row
    sums)."""
    import keras_geometric_amd as kgx
    from keras_geometric_amd import synthetic

    monkeypatch.setenv("KGX_HALO_PUSH", push)
    x = torch.randn(N, F_FUSED, generator=torch.Generator().manual_seed(2)).to(dev)
    hub = ThreadHub(world)
    res = {}
    threads = [threading.Thread(target=_run_fused_rank, args=(r, hub, dev, x, chunks, res, comm))
               for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    for r in range(world):
        if isinstance(res.get(r), BaseException):
            raise res[r]
    for r in range(world):
        assert res[r][2] == chunks and res[r][3] and res[r][4]
    ei = synthetic.rmat_edge_index(N, E, seed=8, device=dev)
    layer = kgx.GCNConv(128)
    layer([x, ei])
    layer.set_weights([res[0][1], np.zeros(128, np.float32)])
    ref = layer([x, ei]).detach().cpu().numpy()
    got = np.concatenate([res[r][0] for r in range(world)])
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() <= 1e-5


def _run_conv_rank(rank, hub, dev, x, out):
    try:
        comm = ThreadComm(hub, rank)
        sg = kd.ShardedGraph.rmat(N, E, seed=6, device=dev, comm=comm, exact=True, n_features=F,
                                  self_loops=False, gcn_norm=False)
        xl = x[sg.lo: sg.lo + sg.n_local]
        res = []
        for layer in (kd.ShardedGINConv(32, sg, mlp_hidden=[48], aggregator="sum", eps_init=0.5),
                      kd.ShardedSAGEConv(32, sg, aggregator="mean"),
                      kd.ShardedSAGEConv(32, sg, aggregator="max", normalize=True)):
            with torch.no_grad():
                y = layer(xl)
            torch.cuda.synchronize()
            res.append((y.cpu().numpy(), layer.conv.get_weights()))
        out[rank] = res
    except BaseException as e:
        out[rank] = e
        hub.barrier.abort()


def test_sharded_gin_sage_hip(dev):
    """C4/C5 shapes in miniature: sharded GIN (sum) and SAGE (mean, max) on the
    HIP backend equal the single-GPU layers with rank 0's weights."""
    import keras_geometric_amd as kgx
    from keras_geometric_amd import synthetic

    world = 2
    x = torch.randn(N, F, generator=torch.Generator().manual_seed(1)).to(dev)
    hub = ThreadHub(world)
    res = {}
    threads = [threading.Thread(target=_run_conv_rank, args=(r, hub, dev, x, res)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    for r in range(world):
        if isinstance(res.get(r), BaseException):
            raise res[r]
    ei = synthetic.rmat_edge_index(N, E, seed=6, device=dev)
    singles = [kgx.GINConv(32, mlp_hidden=[48], aggregator="sum", eps_init=0.5, exact=True),
               kgx.SAGEConv(32, aggregator="mean", exact=True),
               kgx.SAGEConv(32, aggregator="max", normalize=True, exact=True)]
    for i, layer in enumerate(singles):
        layer([x, ei])
        layer.set_weights(res[0][i][1])
        ref = layer([x, ei]).detach().cpu().numpy()
        got = np.concatenate([res[r][i][0] for r in range(world)])
        err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= 1e-5, (i, err.max())


def _run_pipelined_rank(rank, hub, dev, x, out, comm_kind="sync", exchange="halo"):
    try:
        comm = COMMS[comm_kind](hub, rank)
        sg = kd.ShardedGraph.rmat(N, E, seed=9, device=dev, comm=comm, n_features=F, self_loops=False,
                                  gcn_norm=False, halo_chunks=2)
        sg.exchange = exchange
        xl = x[sg.lo: sg.lo + sg.n_local]
        res = []
        for layer in (kd.ShardedGINConv(32, sg, mlp_hidden=[48], aggregator="sum", eps_init=0.5),
                      kd.ShardedGINConv(32, sg, aggregator="mean", eps_init=0.25),
                      kd.ShardedSAGEConv(32, sg, aggregator="mean")):
            with torch.no_grad():
                y = layer(xl)
                if comm_kind != "sync":
                    layer(torch.randn_like(xl))  # other rows through the same halo buffer
                    assert torch.equal(layer(xl), y), "halo buffer reuse across forwards"
            torch.cuda.synchronize()
            res.append((y.cpu().numpy(), layer.conv.get_weights()))
        out[rank] = (res, sg._pp.n_push, len(sg._pp.chunks), sg._pp.kind)
    except BaseException as e:
        out[rank] = e
        hub.barrier.abort()


@pytest.mark.parametrize("comm,exchange", [("sync", "halo"), ("async_delayed", "halo"), ("sync", "allgather"),
                                           ("async_delayed", "allgather")])
def test_sharded_gin_sage_pipelined_hip(comm, exchange, dev):
    """Sharded GIN (sum, mean) and SAGE (mean) on the default path: push-pull
    halo in chunks, own-source kgx_spmm pass, then KGX_EPI_ACCUM passes per
    landed chunk.  Equal to the single-GPU layers within the forward-error
    bound of the re-associated row sums (the same layer on |x| with |weights|)."""
    import keras_geometric_amd as kgx
    from keras_geometric_amd import synthetic

    world = 2
    x = torch.randn(N, F, generator=torch.Generator().manual_seed(3)).to(dev)
    hub = ThreadHub(world)
    res = {}
    threads = [threading.Thread(target=_run_pipelined_rank, args=(r, hub, dev, x, res, comm, exchange))
               for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    for r in range(world):
        if isinstance(res.get(r), BaseException):
            raise res[r]
    assert all(res[r][2] == 2 and res[r][3] == exchange for r in range(world))
    if exchange == "halo":
        assert sum(res[r][1] for r in range(world)) > 0  # partial sums were pushed
    ei = synthetic.rmat_edge_index(N, E, seed=9, device=dev)
    singles = [lambda: kgx.GINConv(32, mlp_hidden=[48], aggregator="sum", eps_init=0.5, exact=True),
               lambda: kgx.GINConv(32, aggregator="mean", eps_init=0.25, exact=True),
               lambda: kgx.SAGEConv(32, aggregator="mean", exact=True)]
    for i, make in enumerate(singles):
        layer, layer_abs = make(), make()
        w = res[0][0][i][1]
        layer([x, ei])
        layer.set_weights(w)
        ref = layer([x, ei]).detach().cpu().numpy()
        layer_abs([x, ei])
        layer_abs.set_weights([np.abs(a) for a in w])
        scale = layer_abs([x.abs(), ei]).detach().cpu().numpy()
        got = np.concatenate([res[r][0][i][0] for r in range(world)])
        err = np.abs(got - ref) / np.maximum(1.0, scale)
        assert err.max() <= 1e-5, (i, err.max())


def _run_no_halo_rank(rank, hub, dev, s, d, x, out):
    try:
        comm = ThreadComm(hub, rank)
        bounds = kd.equal_bounds(N, hub.world)
        lo, hi = bounds[rank], bounds[rank + 1]
        keep = (d >= lo) & (d < hi)
        sg = kd.ShardedGraph.build(torch.from_numpy(s[keep]).to(dev), torch.from_numpy(d[keep]).to(dev), bounds,
                                   comm=comm, n_features=F_FUSED)
        layer = kd.ShardedGCNConv(128, sg)
        with torch.no_grad():
            y = layer(x[lo:hi])
        torch.cuda.synchronize()
        out[rank] = (y.detach().cpu().numpy(), layer.kernel.detach().cpu().numpy(), sg.n_halo, sg._pp.n_rows,
                     sg.halo_k)
    except BaseException as e:
        out[rank] = e
        hub.barrier.abort()


def test_sharded_gcn_no_halo_hip(dev):
    """Shards with no remote source on the HIP kernels: empty pull and push
    plans, empty chunk parts and the K tuning still run; the result equals the
    single-GPU layer."""
    import keras_geometric_amd as kgx
    from oracle.rmat import rmat_edges, scale_for

    s, d = rmat_edges(12, scale_for(N), N, 0, E)
    half = N // 2
    s = np.where((s < half) == (d < half), s, (s + half) % N).astype(np.int32)
    d = d.astype(np.int32)
    x = torch.randn(N, F_FUSED, generator=torch.Generator().manual_seed(4)).to(dev)
    world = 2
    hub = ThreadHub(world)
    res = {}
    threads = [threading.Thread(target=_run_no_halo_rank, args=(r, hub, dev, s, d, x, res)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    for r in range(world):
        if isinstance(res.get(r), BaseException):
            raise res[r]
    assert all(res[r][2] == 0 and res[r][3] == 0 and res[r][4] in (1, 2, 4, 8) for r in range(world))
    ei = torch.from_numpy(np.stack([s, d])).to(dev)
    layer = kgx.GCNConv(128)
    layer([x, ei])
    layer.set_weights([res[0][1], np.zeros(128, np.float32)])
    ref = layer([x, ei]).detach().cpu().numpy()
    got = np.concatenate([res[r][0] for r in range(world)])
    assert (np.abs(got - ref) / np.maximum(1.0, np.abs(ref))).max() <= 1e-5


def _run_wide_rank(rank, hub, dev, x128, x256, out):
    try:
        comm = ThreadComm(hub, rank)
        res = {}
        # GIN sum, 128 -> first Dense 128: the fused two-table pass with GIN's
        # pre-scale (kgx_spmm_gemm_ex3, x2 + KGX_FUSED_PRE_GIN)
        sg = kd.ShardedGraph.rmat(N, E, seed=10, device=dev, comm=comm, n_features=128, self_loops=False,
                                  gcn_norm=False, halo_chunks=2)
        gin = kd.ShardedGINConv(32, sg, mlp_hidden=[128], aggregator="sum", eps_init=0.5)
        xl = x128[sg.lo: sg.lo + sg.n_local]
        with torch.no_grad():
            res["gin"] = (gin(xl).cpu().numpy(), gin.conv.get_weights())
        assert gin._fused(xl.contiguous())  # the MLP exists once built: the route the forward took
        # GCN 256 -> 256: the weighted two-table 256-wide kernels (kgx_spmm_gemm_f256_ex)
        sg2 = kd.ShardedGraph.rmat(N, E, seed=11, device=dev, comm=comm, n_features=256, halo_chunks=2)
        gcn = kd.ShardedGCNConv(256, sg2)
        xl2 = x256[sg2.lo: sg2.lo + sg2.n_local]
        with torch.no_grad():
            res["gcn"] = (gcn(xl2).cpu().numpy(), [gcn.kernel.detach().cpu().numpy()])
        torch.cuda.synchronize()
        out[rank] = res
    except BaseException as e:
        out[rank] = e
        hub.barrier.abort()


def test_sharded_fused_two_table_gin128_gcn256(dev):
    """The fused two-table passes the sharded layers route to: GIN
    sum at F_in 128 with a 128-unit first Dense (pre-scale with two tables in
    the 128-wide kernels) and GCN 256 -> 256 (the 256-wide weighted kernels),
    against the single-GPU layers with rank 0's weights, within the forward-
    error bound of the re-associated row sums."""
    import keras_geometric_amd as kgx
    from keras_geometric_amd import synthetic

    world = 2
    x128 = torch.randn(N, 128, generator=torch.Generator().manual_seed(5)).to(dev)
    x256 = torch.randn(N, 256, generator=torch.Generator().manual_seed(6)).to(dev)
    hub = ThreadHub(world)
    res = {}
    threads = [threading.Thread(target=_run_wide_rank, args=(r, hub, dev, x128, x256, res)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    for r in range(world):
        if isinstance(res.get(r), BaseException):
            raise res[r]
    for key, seed, x, make in (
            ("gin", 10, x128, lambda: kgx.GINConv(32, mlp_hidden=[128], aggregator="sum", eps_init=0.5, exact=True)),
            ("gcn", 11, x256, lambda: kgx.GCNConv(256, exact=True))):
        ei = synthetic.rmat_edge_index(N, E, seed=seed, device=dev)
        w = res[0][key][1]
        if key == "gcn":
            w = w + [np.zeros(256, np.float32)]
        layer, layer_abs = make(), make()
        layer([x, ei])
        layer.set_weights(w)
        ref = layer([x, ei]).detach().cpu().numpy()
        layer_abs([x, ei])
        layer_abs.set_weights([np.abs(a) for a in w])
        scale = np.abs(layer_abs([x.abs(), ei]).detach().cpu().numpy())
        got = np.concatenate([res[r][key][0] for r in range(world)])
        err = np.abs(got - ref) / np.maximum(1.0, scale)
        assert err.max() <= 1e-5, (key, err.max())


N3, E3 = 1_000_000, 10_000_000  # BASELINE config C3 (GATv2, 8 heads x 16)


def _run_gat_rank(rank, hub, dev, x, out):
    try:
        comm = ThreadComm(hub, rank)
        res = {}
        for exact in (True, False):
            sg = kd.ShardedGraph.rmat(N3, E3, seed=3, device=dev, comm=comm, n_features=128, gcn_norm=False,
                                      exact=exact)
            layer = kd.ShardedGATv2Conv(16, sg, heads=8, bias_initializer="glorot_uniform")
            xl = x[sg.lo: sg.lo + sg.n_local]
            with torch.no_grad():
                res[exact] = (layer(xl).cpu().numpy(), layer.conv.get_weights(), sg.n_halo)
        torch.cuda.synchronize()
        out[rank] = res
    except BaseException as e:
        out[rank] = e
        hub.barrier.abort()


def test_sharded_gatv2_c3_hip(dev):
    """ShardedGATv2Conv on the HIP kernels at BASELINE config C3's size (1M
    nodes / 10M edges, 8 heads x 16), two threaded ranks: EXACT mode equals the
    single-GPU EXACT layer bit for bit (each destination's softmax over its
    in-edges in global input order, on its owner); the default (split hub
    rows) within 1e-5 of the single-GPU layer."""
    import keras_geometric_amd as kgx
    from keras_geometric_amd import synthetic

    world = 2
    x = torch.randn(N3, 128, generator=torch.Generator().manual_seed(7)).to(dev)
    hub = ThreadHub(world)
    res = {}
    threads = [threading.Thread(target=_run_gat_rank, args=(r, hub, dev, x, res)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=280)
    for r in range(world):
        if isinstance(res.get(r), BaseException):
            raise res[r]
    assert all(res[r][True][2] > 0 for r in range(world))  # real halo traffic
    ei = synthetic.rmat_edge_index(N3, E3, seed=3, device=dev)
    for exact in (True, False):
        layer = kgx.GATv2Conv(16, heads=8, exact=exact)
        layer([x, ei])
        layer.set_weights(res[0][exact][1])
        ref = layer([x, ei]).detach().cpu().numpy()
        got = np.concatenate([res[r][exact][0] for r in range(world)])
        if exact:
            np.testing.assert_array_equal(got, ref)
        else:
            assert (np.abs(got - ref) / np.maximum(1.0, np.abs(ref))).max() <= 1e-5



class _FnCtx:
    """The autograd context _ShardedGCNFn uses, for calling it directly."""
    needs_input_grad = (True, True, True, False)

    def save_for_backward(self, *t):
        self.saved_tensors = t


def _run_train_rank(rank, hub, dev, x, r_grad, out):
    try:
        comm = ThreadComm(hub, rank)
        sg = kd.ShardedGraph.rmat(N, E, seed=12, device=dev, comm=comm, n_features=F_FUSED, halo_chunks=2)
        layer = kd.ShardedGCNConv(64, sg, bias_initializer="glorot_uniform")
        xl = x[sg.lo: sg.lo + sg.n_local].contiguous()
        with torch.no_grad():
            layer(xl)  # builds the weights (rank 0's, broadcast)
        # the training step's Function driven directly: torch autograd runs CUDA
        # backward functions on ONE engine thread per device, so two threaded
        # ranks' .backward() calls on the same GPU would run one after the other
        # and the first would wait forever in a collective for the second (the
        # autograd wiring itself is covered by the gloo test, one process per rank)
        ctx = _FnCtx()
        y = kd._ShardedGCNFn.forward(ctx, xl, layer.kernel.detach(), layer.bias.detach(), layer)
        dx, dW, db, _ = kd._ShardedGCNFn.backward(ctx, r_grad[sg.lo: sg.lo + sg.n_local])
        torch.cuda.synchronize()
        out[rank] = (y.cpu().numpy(), dx.cpu().numpy(), dW.cpu().numpy(), db.cpu().numpy(), layer.get_weights())
    except BaseException as e:
        out[rank] = e
        hub.barrier.abort()


def test_sharded_gcn_backward_hip(dev):
    """A sharded GCNConv training step on the HIP kernels (two threaded ranks):
    the forward over the pulled halo table, dX through the transposed shard CSR
    with the halo gradients pushed back to their owners, dW / db all-reduced --
    against the single-GPU layer's autograd with rank 0's weights (1e-5 of
    max(1, |ref|); dW / db sum over all rows: sqrt(N) * 1e-5)."""
    import keras_geometric_amd as kgx
    from keras_geometric_amd import synthetic

    world = 2
    x = torch.randn(N, F_FUSED, generator=torch.Generator().manual_seed(8)).to(dev)
    r_grad = torch.randn(N, 64, generator=torch.Generator().manual_seed(9)).to(dev)
    hub = ThreadHub(world)
    res = {}
    threads = [threading.Thread(target=_run_train_rank, args=(r, hub, dev, x, r_grad, res)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    for r in range(world):
        if isinstance(res.get(r), BaseException):
            raise res[r]
    ei = synthetic.rmat_edge_index(N, E, seed=12, device=dev)
    layer = kgx.GCNConv(64)
    layer([x, ei])
    layer.set_weights(res[0][4])
    xg = x.clone().requires_grad_(True)
    y = layer([xg, ei])
    (y * r_grad).sum().backward()

    def close(got, ref, tol):
        err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() <= tol, err.max()

    close(np.concatenate([res[r][0] for r in range(world)]), y.detach().cpu().numpy(), 1e-5)
    close(np.concatenate([res[r][1] for r in range(world)]), xg.grad.cpu().numpy(), 1e-5)
    np.testing.assert_array_equal(res[0][2], res[1][2])
    close(res[0][2], layer.kernel.grad.cpu().numpy(), 1e-5 * np.sqrt(N))
    close(res[0][3], layer.bias.grad.cpu().numpy(), 1e-5 * np.sqrt(N))


class _AggCtx:
    """The autograd context _ShardedAggFn uses, for calling it directly."""
    needs_input_grad = (True, False, False)


def _run_agg_train_rank(rank, hub, dev, x, r_grad, reduce, out):
    try:
        comm = ThreadComm(hub, rank)
        sg = kd.ShardedGraph.rmat(N, E, seed=13, device=dev, comm=comm, n_features=F, self_loops=False,
                                  gcn_norm=False, halo_chunks=2, exact=True)
        xl = x[sg.lo: sg.lo + sg.n_local].contiguous()
        ctx = _AggCtx()  # driven directly: see _run_train_rank
        agg = kd._ShardedAggFn.forward(ctx, xl, sg, reduce)
        dx, _, _ = kd._ShardedAggFn.backward(ctx, r_grad[sg.lo: sg.lo + sg.n_local])
        torch.cuda.synchronize()
        out[rank] = (agg.cpu().numpy(), dx.cpu().numpy())
    except BaseException as e:
        out[rank] = e
        hub.barrier.abort()


@pytest.mark.parametrize("reduce", ["sum", "mean"])
def test_sharded_aggregation_backward_hip(reduce, dev):
    """The neighbour reduction of the sharded GINConv / SAGEConv training step
    (_ShardedAggFn) on the HIP kernels, two threaded ranks: AGG over the pulled
    halo table in EXACT mode (each row one chain in global input order:
    bit-identical to one GPU), and dX through the transposed shard CSR with
    the halo gradients pushed back to their owners and added in chunk order --
    against the single-GPU aggregation's autograd within 1e-5 of the sum of
    |terms| (A^T |dOut|: a re-associated sum's forward-error bound)."""
    import keras_geometric_amd as kgx
    from keras_geometric_amd import synthetic

    world = 2
    x = torch.randn(N, F, generator=torch.Generator().manual_seed(14)).to(dev)
    r_grad = torch.randn(N, F, generator=torch.Generator().manual_seed(15)).to(dev)
    hub = ThreadHub(world)
    res = {}
    threads = [threading.Thread(target=_run_agg_train_rank, args=(r, hub, dev, x, r_grad, reduce, res))
               for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    for r in range(world):
        if isinstance(res.get(r), BaseException):
            raise res[r]
    ei = synthetic.rmat_edge_index(N, E, seed=13, device=dev)
    xg = x.clone().requires_grad_(True)
    y = kgx.MessagePassing(aggregator=reduce, exact=True)([xg, ei])
    (y * r_grad).sum().backward()
    np.testing.assert_array_equal(np.concatenate([res[r][0] for r in range(world)]), y.detach().cpu().numpy())
    ref = xg.grad.cpu().numpy()
    xa = x.clone().requires_grad_(True)
    (kgx.MessagePassing(aggregator=reduce, exact=True)([xa, ei]) * r_grad.abs()).sum().backward()
    mag = xa.grad.cpu().numpy()  # A^T |dOut| (mean: over the counts): the sum of |terms|
    got = np.concatenate([res[r][1] for r in range(world)])
    assert (np.abs(got - ref) / np.maximum(1.0, mag)).max() <= 1e-5
