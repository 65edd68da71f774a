"""Sharded C4 and C5 at their own size, on the HIP kernels.

BASELINE.json configs[3] (C4: GINConv sum, 10M nodes / 100M edges, F 256,
dst-sharded over 8 GPUs) and configs[4] (C5: SAGEConv mean, 2,449,029 /
123,718,280, F 100, over 4 GPUs) are the layers the driver's 8-GPU node runs
(bench.py --config c4 / c5).  The one-GPU box cannot run RCCL between ranks,
so the ranks are THREADS sharing cuda:0 with the asynchronous thread comm of
test_gpu_distributed.py standing in for RCCL's all-to-all (copies on a comm
stream behind a spin, so a missing wait reads rows that have not landed).
Every device operation -- shard generation, shard CSR, push-pull halo plan,
halo packing, the own-source pass under the exchange, one accumulating pass
per halo chunk, the node update (GIN's MLP Dense; SAGE's two linear maps +
bias + ReLU) -- runs through the kgx kernels exactly as with RCCL.  C5 runs
with both exchanges the layer can pick (push-pull halo all-to-all, and the
all-gather of every rank's rows).

Each rank's rows are compared with the single-GPU layer (rank 0's weights) on
the whole graph (gin_conv.py:228-300, sage_conv.py:351-439).  The sharded
path re-associates every row sum (own sources, then halo chunks; pushed
partials), so the bar is the forward-error bound of a re-associated fp32 sum,
scaled by the same layer run on |x| with |weights|:
|sharded - single| <= 1e-5 max(1, layer_abs(|x|)).
"""

from __future__ import annotations

import threading

import pytest
import torch

import keras_geometric_amd as kgx
from keras_geometric_amd import distributed as kd
from keras_geometric_amd import graph as G
from keras_geometric_amd import synthetic
import oracle_sample as OS
from test_gpu_distributed import AsyncThreadComm, ThreadHub

pytestmark = [pytest.mark.gpu, pytest.mark.slow, pytest.mark.timeout(900)]


def _run(world, make_layer, n, e, f, x, seed, chunks, exchange="halo"):
    hub = ThreadHub(world)
    hub.barrier = threading.Barrier(world, timeout=600)
    res = {}

    def rank_main(r):
        try:
            comm = AsyncThreadComm(hub, r, delay_cycles=5_000_000)
            sg = kd.ShardedGraph.rmat(n, e, seed=seed, device=x.device, comm=comm, self_loops=False,
                                      gcn_norm=False, n_features=f, halo_chunks=chunks)
            sg.exchange = exchange
            xl = x[sg.lo: sg.lo + sg.n_local]
            layer = make_layer(sg)
            with torch.no_grad():
                y = layer(xl)
                y2 = layer(xl)  # the persistent halo buffers reused by a second forward
            torch.cuda.synchronize()
            assert torch.equal(y, y2), "halo buffer reuse across forwards"
            assert sg._pp is not None and sg._pp.n_rows > 0 and len(sg._pp.chunks) == chunks
            assert sg._pp.kind == exchange
            res[r] = (sg.lo, y, [w.detach().clone() for w in layer.conv.weights], sg._pp.n_push)
        except BaseException as exc:  # surface worker failures in the test thread
            res[r] = exc
            hub.barrier.abort()

    threads = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=800)
    for r in range(world):
        if isinstance(res.get(r), BaseException):
            raise res[r]
        assert r in res, f"rank {r} did not finish"
    assert [res[r][0] for r in range(world)] == kd.equal_bounds(n, world)[:-1]
    if exchange == "halo":
        assert sum(res[r][3] for r in range(world)) > 0  # pushed partials were exercised
    return torch.cat([res[r][1] for r in range(world)]), res[0][2]


def _check(got, single, abs_single, x, ei, weights, oracle_rows=None):
    """The sharded rows vs the single-GPU layer on every row, and (oracle_rows:
    weights, x -> the oracle on sampled rows, tests/oracle_sample.py) vs the
    CPU oracle on ~1500 sampled rows incl. the largest hubs."""
    with torch.no_grad():
        single([x, ei])
        single.set_weights([w.cpu().numpy() for w in weights])
        ref = single([x, ei])
        abs_single([x, ei])
        abs_single.set_weights([w.abs().cpu().numpy() for w in weights])
        scale = abs_single([x.abs(), ei])
        err = ((got - ref).abs() / scale.clamp_min(1.0)).max().item()
    print(f"sharded vs single-GPU: max scaled err {err:.3e}")
    assert err <= 1e-5, err
    assert got.abs().max().item() > 0
    if oracle_rows is not None:
        rows = OS.sample_rows(ei, x.shape[0])
        ref_o = oracle_rows([w.detach().cpu() for w in weights], x, rows)
        err_o = OS.scaled_err(got[rows], ref_o, scale[rows])
        print(f"sharded vs oracle on {rows.numel()} sampled rows: max scaled err {err_o:.3e}")
        assert err_o <= 1e-5, err_o
    return err


@pytest.fixture(autouse=True)
def _release():
    yield
    G.clear_cache()
    torch.cuda.empty_cache()


def test_c4_sharded_gin_sum_world8_fullsize(dev):
    n, e, f, world = 10_000_000, 100_000_000, 256, 8
    x = torch.randn(n, f, device=dev, generator=torch.Generator(device=dev).manual_seed(41))
    got, weights = _run(world, lambda sg: kd.ShardedGINConv(f, sg, aggregator="sum", eps_init=0.25),
                        n, e, f, x, seed=0, chunks=2)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    _check(got, kgx.GINConv(f, aggregator="sum", eps_init=0.25), kgx.GINConv(f, aggregator="sum", eps_init=0.25),
           x, ei, weights, lambda w, x_, rows: OS.gin_rows(ei, x_, rows, [(w[0], w[1], None)], 0.25))


@pytest.mark.parametrize("exchange", ["halo", "allgather"])
def test_c5_sharded_sage_mean_world4_fullsize(dev, exchange):
    n, e, f, world = 2_449_029, 123_718_280, 100, 4
    x = torch.randn(n, f, device=dev, generator=torch.Generator(device=dev).manual_seed(42))
    got, weights = _run(world, lambda sg: kd.ShardedSAGEConv(f, sg, aggregator="mean"), n, e, f, x, seed=0,
                        chunks=2, exchange=exchange)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    # SAGEConv.weights: bias, lin_neigh, lin_self (sage_conv.py:405-439)
    _check(got, kgx.SAGEConv(f, aggregator="mean"), kgx.SAGEConv(f, aggregator="mean"), x, ei, weights,
           lambda w, x_, rows: OS.sage_rows(ei, x_, rows, w[1], w[2], w[0]))
