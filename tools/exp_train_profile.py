"""Which torch ops a GCNConv training step runs besides the kgx kernels
(torch.profiler, CPU-side op names and shapes with their device time).

  python tools/exp_train_profile.py [--n 1000000 --e 10000000]

A measurement helper, not part of the product."""

import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

import keras_geometric_amd as kgx  # noqa: E402
from keras_geometric_amd import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--e", type=int, default=10_000_000)
    ap.add_argument("--host", action="store_true", help="only: host enqueue time of 10 steps against their total")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ei = synthetic.rmat_edge_index(args.n, args.e, seed=0, device=dev)
    x = torch.randn(args.n, 128, device=dev, requires_grad=True)
    layer = kgx.GCNConv(128)
    layer([x, ei])
    g = next(reversed(kgx.graph._CACHE.values()))[1]
    kgx.graph.transpose(g)
    gout = torch.randn(args.n, 128, device=dev)

    def step():
        x.grad = None
        layer.zero_grad(set_to_none=True)
        layer([x, ei]).backward(gout)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    if args.host:  # a host that is not ahead of the GPU shows as enqueue time ~ total time
        import time

        for rep in range(3):
            t0 = time.perf_counter()
            for _ in range(10):
                step()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(f"10 steps: enqueue {1e3 * (t1 - t0):.2f} ms, total {1e3 * (t2 - t0):.2f} ms", flush=True)
        return
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=25), flush=True)
    print(prof.key_averages(group_by_stack_n=8).table(sort_by="cuda_time_total", row_limit=8), flush=True)


if __name__ == "__main__":
    main()
