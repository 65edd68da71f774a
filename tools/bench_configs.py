"""Per-config GPU measurements for BASELINE.json's configs (one MI355X).

  python tools/bench_configs.py [c1 c2 c3 c4 c5 ...]

C1 Cora-shaped 2-layer GCN; C2 GCN 1M/10M F128; C3 GATv2 1M/10M H8xC16;
C4 GIN-sum 10M/100M F256 (one GPU; the 8-GPU sharded run is bench.py --gpus 8
with GCN); C5 SAGE-mean ogbn-products-shaped 2,449,029 / 123,718,280 F100.
Reports layer ms, aggregation-kernel ms (events on the launch stream),
algorithmic GB/s (SURVEY.md §8d byte model) and edges/s.  A measurement
helper, not part of the product.
"""

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

import keras_geometric_amd as kgx  # noqa: E402
from keras_geometric_amd import ops as kops  # noqa: E402
from keras_geometric_amd import synthetic  # noqa: E402


def run(step, steps=10, warmup=2, grad=False):
    if not grad:  # forward configs: inference, no autograd state
        inner = step

        def step():
            with torch.no_grad():
                return inner()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    kops.EVENT_SINK = []
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps * 1e3
    ev = kops.EVENT_SINK
    kops.EVENT_SINK = None
    per_step = len(ev) // steps
    agg = sum(s.elapsed_time(e) for s, e in ev) / steps
    return dt, agg, per_step


def graph(layer_obj):
    return next(reversed(kgx.graph._CACHE.values()))[1]


def spmm_bytes(n, e, f_gather, f_out, weighted):
    return 4 * (n + 1) + e * (4 + (4 if weighted else 0) + 4 * f_gather) + 4 * n * f_out


def c2(dev):
    n, e, f = 1_000_000, 10_000_000, 128
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = torch.randn(n, f, device=dev)
    layer = kgx.GCNConv(f)
    layer([x, ei])
    g = graph(layer)
    ms, agg, _ = run(lambda: layer([x, ei]))
    b = spmm_bytes(n, g.kept, f, f, True)
    return dict(config="C2 GCN 1M/10M F128", layer_ms=ms, agg_ms=agg, e_agg=g.kept,
                edges_per_s=g.kept / ms * 1e3, alg_GBps=b / agg / 1e6)


def c3(dev):
    n, e, H, C, fin = 1_000_000, 10_000_000, 8, 16, 128
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = torch.randn(n, fin, device=dev)
    layer = kgx.GATv2Conv(C, heads=H)
    layer([x, ei])
    g = graph(layer)
    ms, agg, _ = run(lambda: layer([x, ei]))
    hc = H * C
    b = 4 * (n + 1) + g.kept * (4 + 4 * hc) + 8 * n * hc
    return dict(config="C3 GATv2 1M/10M H8xC16", layer_ms=ms, agg_ms=agg, e_agg=g.kept,
                edges_per_s=g.kept / ms * 1e3, alg_GBps=b / agg / 1e6)


def c4(dev):
    n, e, f = 10_000_000, 100_000_000, 256
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = torch.randn(n, f, device=dev)
    layer = kgx.GINConv(f, aggregator="sum")
    layer([x, ei])
    g = graph(layer)
    ms, agg, _ = run(lambda: layer([x, ei]), steps=5)
    b = spmm_bytes(n, g.kept, f, f, False) + 4 * n * f  # + x root row for the GIN epilogue
    return dict(config="C4 GIN-sum 10M/100M F256 (1 GPU)", layer_ms=ms, agg_ms=agg, e_agg=g.kept,
                edges_per_s=g.kept / ms * 1e3, alg_GBps=b / agg / 1e6)


def gin128(dev):
    """GIN-sum 10M/100M F128 -> MLP [128] + 128: fused (aggregation + first
    Dense + ReLU in one launch) vs EXACT (aggregation, then the MLP GEMMs)."""
    n, e, f = 10_000_000, 100_000_000, 128
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = torch.randn(n, f, device=dev)
    out = {}
    for exact in (False, True):
        layer = kgx.GINConv(f, mlp_hidden=[f], aggregator="sum", exact=exact)
        layer([x, ei])
        ms, agg, _ = run(lambda: layer([x, ei]), steps=5)
        out["exact_layer_ms" if exact else "layer_ms"] = ms
        out["exact_agg_ms" if exact else "agg_ms"] = agg
    g = graph(layer)
    return dict(config="GIN-sum 10M/100M F128 MLP[128]+128 (1 GPU)", e_agg=g.kept,
                edges_per_s=g.kept / out["layer_ms"] * 1e3, **out)


def c5(dev):
    n, e, f = 2_449_029, 123_718_280, 100
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = torch.randn(n, f, device=dev)
    layer = kgx.SAGEConv(f, aggregator="mean")
    layer([x, ei])
    g = graph(layer)
    ms, agg, _ = run(lambda: layer([x, ei]), steps=5)
    b = spmm_bytes(n, g.kept, f, f, False)
    return dict(config="C5 SAGE-mean 2.45M/123.7M F100 (1 GPU)", layer_ms=ms, agg_ms=agg, e_agg=g.kept,
                edges_per_s=g.kept / ms * 1e3, alg_GBps=b / agg / 1e6)


def ns_train(dev):
    """NS GCNConv forward + backward (d/dx, d/dW, d/db): one training step's
    propagate work (fused forward, recompute of A x for dW, dOut W^T GEMM,
    transposed aggregation for dx)."""
    n, e, f = 10_000_000, 100_000_000, 128
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = torch.randn(n, f, device=dev, requires_grad=True)
    layer = kgx.GCNConv(f)
    layer([x, ei])
    g = graph(layer)
    gout = torch.randn(n, f, device=dev)
    kgx.graph.transpose(g)  # built once per graph, like the forward CSR

    def step():
        x.grad = None
        layer.zero_grad(set_to_none=True)
        layer([x, ei]).backward(gout)

    ms, agg, per = run(step, steps=5, grad=True)
    return dict(config="NS GCNConv fwd+bwd 10M/100M F128", step_ms=ms, aggregation_kernels_ms=agg,
                launches_per_step=per, e_agg=g.kept, edges_per_s=g.kept / ms * 1e3)


def c3_train(dev):
    """C3 GATv2 forward + backward (d/dx, d/dW, d/d att, d/d bias)."""
    n, e, H, C, fin = 1_000_000, 10_000_000, 8, 16, 128
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = torch.randn(n, fin, device=dev, requires_grad=True)
    layer = kgx.GATv2Conv(C, heads=H)
    layer([x, ei])
    g = graph(layer)
    gout = torch.randn(n, H * C, device=dev)
    kgx.graph.transpose(g)

    def step():
        x.grad = None
        layer.zero_grad(set_to_none=True)
        layer([x, ei]).backward(gout)

    ms, agg, per = run(step, steps=5, grad=True)
    return dict(config="C3 GATv2 fwd+bwd 1M/10M H8xC16", step_ms=ms, forward_kernel_ms=agg, e_agg=g.kept,
                edges_per_s=g.kept / ms * 1e3)


def pool(dev):
    """BatchGlobalPooling (sum / mean / max) over 10M nodes, F 128, 100k graphs:
    a segment reduction whose rows are contiguous -- a streaming read of x."""
    from keras_geometric_amd.layers import BatchGlobalPooling

    n, f, G = 10_000_000, 128, 100_000
    x = torch.randn(n, f, device=dev)
    batch = torch.sort(torch.randint(0, G, (n,), device=dev, dtype=torch.int32)).values
    out = {}
    for p in ("sum", "mean", "max"):
        layer = BatchGlobalPooling(pooling=p)
        layer([x, batch])
        ms, agg, _ = run(lambda: layer([x, batch]), steps=10)
        out[p] = dict(layer_ms=ms, kernel_ms=agg, GBps=(4 * n * f + 4 * n + 4 * G * f) / agg / 1e6)
    return dict(config="BatchGlobalPooling 10M nodes F128 100k graphs", **out)


def io(dev):
    """Persistent graph file: NS graph (10M/100M, GCN CSR + schedule) loaded
    from an NPZ vs rebuilt from edge_index (x is 1 feature wide to keep the
    file to the graph)."""
    import os
    import tempfile

    from keras_geometric_amd.utils import load_graphs, save_graphs

    n, e = 10_000_000, 100_000_000
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    gd = kgx.GraphData(x=torch.zeros(n, 1, device=dev), edge_index=ei)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    G = kgx.graph.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=True, gcn_norm=True)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    del G
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        path = os.path.join(d, "ns.npz")
        save_graphs(path, [gd], with_csr=True, self_loops=True, gcn_norm=True, n_features=128)
        size = os.path.getsize(path)
        kgx.clear_cache()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loaded, _ = load_graphs(path)
        torch.cuda.synchronize()
        load_s = time.perf_counter() - t0
    return dict(config="NS graph CSR: build vs load", build_s=build_s, load_s=load_s, file_GB=size / 1e9,
                kept=loaded[0].csr.kept)


def c1(dev):
    n, e, fin = 2708, 10556, 1433
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    x = (torch.rand(n, fin, device=dev) < 0.0127).float()
    l1, l2 = kgx.GCNConv(64), kgx.GCNConv(7)

    def fwd():
        return l2([torch.relu(l1([x, ei])), ei])

    fwd()
    ms, agg, _ = run(fwd, steps=50, warmup=5)
    # the same forward captured once into a HIP graph and replayed (launch-bound at this size)
    with torch.no_grad():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fwd()
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            fwd()
        for _ in range(5):
            graph.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            graph.replay()
        torch.cuda.synchronize()
        g_ms = (time.perf_counter() - t0) / 200 * 1e3
    return dict(config="C1 Cora-shaped 2-layer GCN 1433-64-7", layer_ms=ms, agg_ms=agg, hip_graph_ms=g_ms)


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    names = sys.argv[1:] or ["c1", "c2", "c3", "c4", "c5", "ns_train", "c3_train", "pool", "io"]
    for name in names:
        r = globals()[name](dev)
        print(json.dumps(r), flush=True)
        kgx.clear_cache()
        torch.cuda.empty_cache()
