"""C5's 400-byte rows: does the row stride decide the bytes fetched?

  python tools/exp_c5_stride.py --ld 100 [--reps 10] [--features F]

The C5 aggregation (SAGE mean, F = 100, 2,449,029 rows / 123,718,280 edges)
reads 400-byte source rows.  At a 400-byte stride a row starts at any 16-byte
offset of a 64-byte sector and spans 7 sectors (448 bytes), whichever lanes
issue which 16-byte pieces; at a 448-byte stride (--ld 112) every row starts
on a sector and spans exactly 7; at 512 (--ld 128) rows are whole 128-byte
lines.  Same graph, same values in the first 100 columns, same kernel
(kgx_spmm_ex2, MEAN), only the table's leading dimension changes: run each --ld
under rocprofv3 --pmc FETCH_SIZE to read the bytes fetched per launch, and
without it for the time.  A measurement helper, not part of the product.

--features F (round 6) changes the ROW WIDTH instead (ld = F unless given):
F = 96 (384-byte rows, exactly six 64-byte sectors), 112 (448 bytes, seven),
100 (400 bytes: 6.25 sectors, so a row touches seven and wastes 48 bytes of
the last one, wherever it starts) and 128.  If the memory side moves whole
64-byte sectors, fetched / algorithmic read bytes is ~1.0 at 96, 112 and 128
(less the cache hits of hub rows) and ~448 / 400 = 1.12 less hits at 100.
"""

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import _native as nat  # noqa: E402
from keras_geometric_amd import graph as G  # noqa: E402
from keras_geometric_amd import synthetic  # noqa: E402

N, E, F = 2_449_029, 123_718_280, 100


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ld", type=int, default=None)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--features", type=int, default=F)
    args = ap.parse_args()
    f = args.features
    if args.ld is None or args.ld < f:
        args.ld = f
    dev = torch.device("cuda", 0)
    ei = synthetic.rmat_edge_index(N, E, seed=0, device=dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), N, N, n_features=f)
    del ei
    gen = torch.Generator(device=dev).manual_seed(1)
    base = torch.randn(N, args.ld, device=dev, generator=gen)
    table = base[:, :f]  # the first f columns of an [N, ld] buffer
    out = torch.empty(N, f, device=dev)
    items, _, split, _, n_slots = g.work(False)
    partials = torch.empty(max(n_slots, 1), f, device=dev)
    n_items = items.shape[0]
    n_split = 0 if split is None else split.shape[0]

    def run():
        nat.check(nat.lib().kgx_spmm_ex2(
            nat.MEAN, nat.EPI_NONE, nat.ptr(g.rowptr), nat.ptr(g.rows), N, nat.ptr(items), n_items, g.n_long,
            nat.ptr(split), n_split, nat.ptr(g.col), None, nat.ptr(table), table.stride(0), None, 0, f,
            nat.ptr(out), out.stride(0), None, None, 0, 1.0, None, 0.0, 0, nat.ptr(partials), None,
            nat.stream(dev)), "kgx_spmm_ex2")

    for _ in range(2):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(args.reps):
        run()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / args.reps
    alg = 4 * (N + 1) + g.kept * (4 + 4 * f) + 4 * N * f
    alg_read = 4 * (N + 1) + g.kept * (4 + 4 * f)
    print(json.dumps({"features": f, "ld": args.ld, "row_stride_bytes": 4 * args.ld, "ms": ms, "alg_bytes": alg,
                      "alg_read_bytes": alg_read,
                      "alg_TBps": alg / ms / 1e9, "checksum": float(out.double().sum())}))


if __name__ == "__main__":
    main()
