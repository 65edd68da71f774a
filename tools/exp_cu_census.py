"""Where a CU-masked stream's blocks run, per split size (kgx_cu_split_census):
for t of every 32 CUs on the tail, the distinct CUs each stream's blocks reached,
per XCD and per shader engine.  A measurement helper, not part of the product.

  python tools/exp_cu_census.py [t ...]   (default 4..12 and 16)"""
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "keras-geometric_amd")]

import torch  # noqa: E402

from keras_geometric_amd import _native as nat  # noqa: E402

dev = torch.device("cuda", 0)
n = 8192
for per32 in [int(a) for a in sys.argv[1:]] or [4, 5, 6, 7, 8, 9, 10, 12, 16]:
    head = torch.full((n,), -1, dtype=torch.int32, device=dev)
    tail = torch.full((n,), -1, dtype=torch.int32, device=dev)
    cus = (ctypes.c_int * 2)()
    rc = nat.lib().kgx_cu_split_census(per32, n, nat.ptr(head), nat.ptr(tail), cus, nat.stream(dev))
    if rc != 0:
        print(json.dumps({"per32": per32, "error": nat.lib().kgx_last_error().decode()}), flush=True)
        continue
    h, t = set(head.cpu().tolist()), set(tail.cpu().tolist())

    def spread(ids, shift, mask):
        out = {}
        for c in ids:
            k = (c >> shift) & mask
            out[k] = out.get(k, 0) + 1
        return dict(sorted(out.items()))

    print(json.dumps({"per32": per32, "claimed": [cus[0], cus[1]], "head_cus": len(h), "tail_cus": len(t),
                      "shared": len(h & t), "tail_per_xcd": spread(t, 8, 0xf),
                      "tail_per_xcd_se": spread(t, 5, 0x7f), "head_per_xcd": spread(h, 8, 0xf)}), flush=True)
