"""Tiny-row (degree <= 2) warp-specialised fused kernel vs the short-row path
(a measurement and correctness helper).

  python tools/exp_tiny.py

Calls kgx_spmm_gemm_ex2 with and without the packed tail on the NS graph and
checks the two outputs agree (tolerance: both are f32-accurate transforms of
the same in-order sums), then times both.
"""

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import _native as nat  # noqa: E402
from keras_geometric_amd import graph as G  # noqa: E402
from keras_geometric_amd import synthetic  # noqa: E402
from keras_geometric_amd import tiny  # noqa: E402


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


def main(n=10_000_000, e=100_000_000, f=128, weighted=True, red=0):
    dev = torch.device("cuda", 0)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, self_loops=True, gcn_norm=True)
    x = torch.randn(n, f, device=dev)
    W = torch.randn(f, f, device=dev) * (1.0 / f) ** 0.5
    b = torch.randn(f, device=dev)
    pack, tw, start, n2 = tiny.tiny_pack(g)
    assert pack is not None
    out_a = torch.empty(n, f, device=dev)
    out_b = torch.empty(n, f, device=dev)
    partials = torch.empty(max(g.n_slots, 1), f, device=dev)
    w = g.w if weighted else None

    def call(out, use_tiny):
        nat.check(nat.lib().kgx_spmm_gemm_ex2(
            red, nat.ptr(g.rowptr), nat.ptr(g.rows), n, nat.ptr(g.items), g.n_items, g.n_long,
            start if use_tiny else g.n_items, nat.ptr(pack) if use_tiny else None,
            nat.ptr(tw) if (use_tiny and weighted) else None, n2 if use_tiny else 0, nat.ptr(g.split), g.n_split,
            nat.ptr(g.col), nat.ptr(w), nat.ptr(x), x.stride(0), f, nat.ptr(W), f, nat.ptr(b), 0, 1.0,
            nat.ptr(out), out.stride(0), nat.ptr(partials), None, 0, nat.stream(dev)), "ex2")

    call(out_a, False)
    call(out_b, True)
    torch.cuda.synchronize()
    err = ((out_a - out_b).abs() / out_a.abs().clamp_min(1.0)).max().item()
    t_a = timeit(lambda: call(out_a, False))
    t_b = timeit(lambda: call(out_b, True))
    deg = (pack[:, 1]).long()
    print(json.dumps({"weighted": weighted, "red": red, "tiny_rows": int(pack.shape[0]), "tiny_start": start,
                      "n_long": g.n_long, "n_items": g.n_items, "deg0": int((deg == 0).sum()),
                      "deg1": int((deg == 1).sum()), "deg2": int((deg == 2).sum()), "max_rel_err": err,
                      "ms_short_path": round(t_a, 3), "ms_tiny_path": round(t_b, 3)}), flush=True)
    assert err <= 1e-5, err


if __name__ == "__main__":
    main()
    main(weighted=False, red=2)
