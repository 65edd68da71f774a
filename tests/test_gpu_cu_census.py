"""The CU split's masks, checked on the hardware (kgx_cu_split_census, include/kgx.h):
blocks launched on the head and tail CU-masked streams record the CU they ran on
(XCC, SE, SH and CU ids from the hardware registers).  The two sets must be
disjoint and hold exactly the CU counts the split assumes (192 / 64 at 8 of every
32 CUs on the validated 256-CU gfx950 layout), so a launch that runs split really
runs its tail on CUs the main kernel cannot take -- the mapping DESIGN.md §4
relies on, verified on the box instead of assumed."""

import ctypes

import pytest
import torch

from keras_geometric_amd import _native as nat
from keras_geometric_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("per32", [8, 16])
def test_cu_split_masks_disjoint_and_complete(per32):
    dev = torch.device("cuda", 0)
    if nat.lib().kgx_cu_split_supported(0) != 1:
        pytest.skip("no validated CU-split layout on this device")
    n = 8192
    head = torch.full((n,), -1, dtype=torch.int32, device=dev)
    tail = torch.full((n,), -1, dtype=torch.int32, device=dev)
    cus = (ctypes.c_int * 2)()
    nat.check(nat.lib().kgx_cu_split_census(per32, n, nat.ptr(head), nat.ptr(tail), cus, nat.stream(dev)),
              "kgx_cu_split_census")
    h, t = set(head.cpu().tolist()), set(tail.cpu().tolist())
    assert -1 not in h and -1 not in t  # every block recorded
    assert len(h & t) == 0, f"head and tail masks share CUs: {sorted(h & t)[:8]}"
    assert len(h) == cus[0] and len(t) == cus[1], (len(h), cus[0], len(t), cus[1])
    assert cus[0] + cus[1] == 256 and cus[1] == 8 * per32
    # where the masks land (printed for the record: -s shows it)
    per_xcc_t = {x: sum(1 for c in t if c >> 8 == x) for x in sorted({c >> 8 for c in t})}
    per_xcc_h = {x: sum(1 for c in h if c >> 8 == x) for x in sorted({c >> 8 for c in h})}
    print(f"per32 {per32}: tail CUs per XCC {per_xcc_t}, head CUs per XCC {per_xcc_h}")
