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
        mid = g.items[g.n_long:n_se].contiguous()
        lng = g.items[:g.n_long].contiguous()

        def run_long(cus):
            os.environ["KGX_EXP_CUS"] = str(cus)
            return op(x, g.rowptr, g.rows, lng, g.split, g.col, None, g.n_slots, 0, W, b, True, 1.25)

        def run_midtail(cus):
            os.environ["KGX_EXP_CUS"] = str(cus)
            y = op(x, g.rowptr, g.rows, mid, None, g.col, None, 0, 0, W, b, True, 1.25, False, 0)
            y2 = op(x, g.rowptr, g.rows, tail, None, g.col, None, 0, 0, W, b, True, 1.25, False, -1, tpack, tw, 0, n2)
            return y, y2

        main_s = torch.cuda.current_stream()
        head_rows, long_rows, mid_rows = head[:, 0].long(), lng[:, 0].long(), mid[:, 0].long()
        for split in ("head|tail", "long|mid+tail"):
            for nt in (40, 48, 56, 64, 72, 80):
                tb = {c for c in range(256) if (c % 32) < nt // 8}  # nt // 8 of every 32 CUs
                hb = [c for c in range(256) if c not in tb]
                sh, st = masked_stream(hb), masked_stream(sorted(tb))
                nh = len(hb)
                fa, fb = (run_head, run_tail) if split == "head|tail" else (run_long, run_midtail)

                def both():
                    ev = torch.cuda.Event()
                    ev.record(main_s)
                    sh.wait_event(ev)
                    st.wait_event(ev)
                    with torch.cuda.stream(sh):
                        ya = fa(nh)
                    with torch.cuda.stream(st):
                        yb = fb(nt)
                    eh, et = torch.cuda.Event(), torch.cuda.Event()
                    eh.record(sh)
                    et.record(st)
                    main_s.wait_event(eh)
                    main_s.wait_event(et)
                    return ya, yb

                t = elapsed(both)
                ya, yb = both()
                torch.cuda.synchronize()
                if split == "head|tail":
                    same = torch.equal(ya[head_rows], ref[head_rows]) and torch.equal(yb[rows_tail], ref[rows_tail])
                else:
                    same = (torch.equal(ya[long_rows], ref[long_rows]) and torch.equal(yb[0][mid_rows], ref[mid_rows])
                            and torch.equal(yb[1][rows_tail], ref[rows_tail]))
                res[f"{split}:{nt}"] = {"both_ms": round(t, 3), "bits_equal": bool(same)}
    print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
