"""C4 (GIN-sum 10M/100M, F 256 -> 256) fused kernels on CU-partitioned streams
(a measurement helper).  The long-row launch is memory-bound (MFMA ~9 % busy),
the degree <= 2 tail MFMA-bound (56 % busy, its memory phase serialised with the
MFMA phase inside each block): run side by side on disjoint CU sets
(hipExtStreamCreateWithCUMask) they could overlap.  Measures each launch alone
on N CUs and the pair concurrently, with the outputs compared bit for bit
against the one-stream launch.  Needs a build with -DKGX_EXP_GRID_CUS
(KGX_LIB=...libkgx_cupart.so): the grid follows KGX_EXP_CUS.

  python tools/exp_cupart.py
"""

import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import graph as G  # noqa: E402
from keras_geometric_amd import ops as kops  # noqa: E402
from keras_geometric_amd import synthetic  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch loaded (same soname as libkgx binds)


def masked_stream(bits):
    words = (ctypes.c_uint32 * 8)()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    h = ctypes.c_void_p()
    err = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(8), words)
    assert err == 0, err
    return torch.cuda.ExternalStream(h.value)


def elapsed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main(n=10_000_000, e=100_000_000, f=256):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ei = synthetic.rmat_edge_index(n, e, seed=0, device=dev)
    g = G.build_csr(ei[0].contiguous(), ei[1].contiguous(), n, n, n_features=f)
    x = torch.randn(n, f, device=dev)
    W = torch.randn(f, f, device=dev) * (1.0 / f) ** 0.5
    b = torch.randn(f, device=dev)
    tpack, tw, n_se, n2 = kops._tiny_of(g, g.items)
    head = g.items[:n_se].contiguous()  # hub chunks, long rows, degree 3..7
    tail = g.items[n_se:].contiguous()
    op = torch.ops.kgx.spmm_gemm

    def run_head(cus):
        os.environ["KGX_EXP_CUS"] = str(cus)
        return op(x, g.rowptr, g.rows, head, g.split, g.col, None, g.n_slots, 0, W, b, True, 1.25, False, g.n_long)

    def run_tail(cus):
        os.environ["KGX_EXP_CUS"] = str(cus)
        return op(x, g.rowptr, g.rows, tail, None, g.col, None, 0, 0, W, b, True, 1.25, False, -1, tpack, tw, 0, n2)

    res = {}
    with torch.no_grad():
        ref = op(x, g.rowptr, g.rows, g.items, g.split, g.col, None, g.n_slots, 0, W, b, True, 1.25, False, g.n_long,
                 tpack, tw, n_se, n2)
        rows_tail = tail[:, 0].long()
        res["full_ms"] = elapsed(lambda: op(x, g.rowptr, g.rows, g.items, g.split, g.col, None, g.n_slots, 0, W, b,
                                            True, 1.25, False, g.n_long, tpack, tw, n_se, n2))
        res["head_256"] = elapsed(lambda: run_head(256))
        res["tail_256"] = elapsed(lambda: run_tail(256))
        layouts = {"inter": lambda k: [c for c in range(256) if (c % 8) < k],  # k of every 8 CUs
                   "contig": lambda k: list(range(32 * k))}                     # the first 32 k CUs
        for lay, pick in layouts.items():
            for kt in (2, 3, 4):  # tail on kt / 8 of the CUs
                tb = set(pick(kt))
                hb = [c for c in range(256) if c not in tb]
                sh, st = masked_stream(hb), masked_stream(sorted(tb))
                nh, nt = len(hb), len(tb)
                with torch.cuda.stream(sh):
                    th = elapsed(lambda: run_head(nh))
                with torch.cuda.stream(st):
                    tt = elapsed(lambda: run_tail(nt))
                main_s = torch.cuda.current_stream()

                def both():
                    ev = torch.cuda.Event()
                    ev.record(main_s)
                    sh.wait_event(ev)
                    st.wait_event(ev)
                    with torch.cuda.stream(sh):
                        yh = run_head(nh)
                    with torch.cuda.stream(st):
                        yt = run_tail(nt)
                    eh, et = torch.cuda.Event(), torch.cuda.Event()
                    eh.record(sh)
                    et.record(st)
                    main_s.wait_event(eh)
                    main_s.wait_event(et)
                    return yh, yt

                tb_ms = elapsed(both)
                yh, yt = both()
                torch.cuda.synchronize()
                same = bool(torch.equal(yt[rows_tail], ref[rows_tail]))
                head_rows = head[:, 0].long()
                same = same and bool(torch.equal(yh[head_rows], ref[head_rows]))
                res[f"{lay}_tail{nt}"] = {"head_ms": round(th, 3), "tail_ms": round(tt, 3), "both_ms": round(tb_ms, 3),
                                          "bits_equal": same}
    print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
