"""GATv2 backward at the leaky-ReLU kink: which side is noisy.

The reference's attention score is s = sum_c att_c lrelu(h_i + h_j)_c
(gatv2_conv.py:277-284); lrelu's derivative jumps from 1 to negative_slope at
z = 0, so the gradient is discontinuous there.  On some weight draws exactly
one z of the N=900 / E=8000 fixture lies within ~1e-8 of zero and an fp32 and
an fp64 evaluation put it on opposite sides: the fp32 oracle's gradients then
miss the fp64 oracle's by up to 1.2e-3 (d/dx) and 1.1e-2 (d/dkernel) although
the forward agrees to 1e-6.  Round 2 saw one such draw (7.7e-4) and switched
its test to an fp64 reference without showing this; these tests pin it:

CPU (oracle only): on the kink draws (tests/golden/gatv2_bwd_draws.npz) the
fp32 and fp64 oracles straddle a z within 1e-7 of 0 and miss each other past
1e-4; given the same branch (the fp64 one) they agree within the north-star
1e-5 (d/dx) and 1e-5 sqrt(N) (weight gradients, sums over N rows).

GPU (kgx_gatv2_backward): against the fp32 AND the fp64 oracle evaluated with
the kernel's own branch (z = h_i + h_j from the layer's device h, the same fp32
add as gatv2.hip), within those tolerances; against each oracle on its own
branches within tolerance wherever their branches agree with the kernel's, and
where it sits on the fp64 side its error is no larger than the fp32 oracle's.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import reference as R
from oracle.rmat import rmat_edges, scale_for

T = torch.from_numpy
N, E, FI, HEADS, C = 900, 8000, 24, 8, 16
SLOPE = 0.2


def _inputs():
    s, d = rmat_edges(24, scale_for(N), N, 0, E)
    ei = np.stack([s, d]).astype(np.int32)
    x = np.random.default_rng(25).standard_normal((N, FI)).astype(np.float32)
    gout = np.random.default_rng(26).standard_normal((N, HEADS * C)).astype(np.float32)
    bias = np.random.default_rng(27).standard_normal((1, HEADS * C)).astype(np.float32)[0]
    return ei, x, gout, bias


def _draws(golden, kind):
    z = golden("gatv2_bwd_draws")
    keys = sorted({k.rsplit("_", 1)[0] for k in z if k.startswith(kind + "_")})
    return [(k, z[k + "_kernel"], z[k + "_att"]) for k in keys]


def _z(h, ei):
    """Leaky-ReLU inputs [E', H, C] (self loops appended last, utils/main.py:8-16)."""
    loops = torch.arange(N, dtype=torch.int64)
    src = torch.cat([T(ei[0]).long(), loops])
    dst = torch.cat([T(ei[1]).long(), loops])
    h = h.reshape(N, HEADS, C)
    return h[dst] + h[src]


def _oracle_grads(dtype, x, ei, kern, att, bias, gout, branch=None):
    xr = T(x).to(dtype).requires_grad_(True)
    kr, ar, br = (T(np.asarray(a)).to(dtype).requires_grad_(True) for a in (kern, att, bias))
    yr = R.gatv2_forward(xr, T(ei), kr, ar, br, heads=HEADS, concat=True, negative_slope=SLOPE,
                         lrelu_positive=branch)
    yr.backward(T(gout).to(dtype))
    return {"y": yr.detach(), "dx": xr.grad, "dkernel": kr.grad, "datt": ar.grad, "dbias": br.grad}


TOL = {"y": 1e-5, "dx": 1e-5, "dkernel": 1e-5 * np.sqrt(N), "datt": 1e-5 * np.sqrt(N), "dbias": 1e-5 * np.sqrt(N)}


def _err(a, b) -> float:
    a = a.detach().cpu().double()
    b = b.detach().cpu().double()
    return float(((a - b).abs() / b.abs().clamp_min(1.0)).max())


def test_fixture_draws_match_generator(golden):
    """The committed weights are the glorot draws the generator script names."""
    import importlib.util
    from pathlib import Path

    p = Path(__file__).resolve().parent / "golden" / "make_gatv2_draws.py"
    spec = importlib.util.spec_from_file_location("make_gatv2_draws", p)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for kind in ("well", "kink"):
        for key, kern, att in _draws(golden, kind):
            k2, a2 = mod.draw(int(key.rsplit("_", 1)[1]))
            np.testing.assert_array_equal(kern, k2)
            np.testing.assert_array_equal(att, a2)


@pytest.mark.parametrize("kind", ["well", "kink"])
def test_oracle_fp32_fp64_gap_is_the_kink(golden, kind):
    ei, x, gout, bias = _inputs()
    for key, kern, att in _draws(golden, kind):
        z32 = _z(T(x) @ T(kern), ei)
        z64 = _z(T(x).double() @ T(kern).double(), ei)
        flips = (z32 > 0) != (z64 > 0)
        g32 = _oracle_grads(torch.float32, x, ei, kern, att, bias, gout)
        g64 = _oracle_grads(torch.float64, x, ei, kern, att, bias, gout)
        if kind == "well":
            assert not bool(flips.any()), key
            for k in TOL:
                assert _err(g32[k], g64[k]) <= TOL[k], (key, k)
            continue
        # exactly the ill-conditioned case: a z within 1e-7 of 0 on opposite sides ...
        assert int(flips.sum()) >= 1 and float(z64[flips].abs().max()) < 1e-7, key
        assert _err(g32["y"], g64["y"]) <= 1e-5  # the forward agrees
        assert _err(g32["dx"], g64["dx"]) > 1e-4, key  # ... and the fp32 gradient misses past 1e-4
        # given fp64's branch the fp32 oracle is within the north-star tolerance
        g32b = _oracle_grads(torch.float32, x, ei, kern, att, bias, gout, branch=z64 > 0)
        for k in TOL:
            assert _err(g32b[k], g64[k]) <= TOL[k], (key, k, _err(g32b[k], g64[k]))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["well", "kink"])
def test_gatv2_backward_at_the_kink(golden, kind, dev):
    from keras_geometric_amd.layers import GATv2Conv

    ei, x, gout, bias = _inputs()
    for key, kern, att in _draws(golden, kind):
        layer = GATv2Conv(C, heads=HEADS, concat=True, negative_slope=SLOPE, exact=True)
        xd = T(x).to(dev).requires_grad_(True)
        layer([xd, T(ei).to(dev)])
        layer.set_weights([att, bias, kern])  # own weights, then the linear_transform sublayer's
        y = layer([xd, T(ei).to(dev)])
        y.backward(T(gout).to(dev))
        kg = {"y": y.detach(), "dx": xd.grad, "dkernel": layer.linear_transform.kernel.grad,
              "datt": layer.att.grad, "dbias": layer.bias.grad}
        with torch.no_grad():  # the kernel's own branch: its z is h_i + h_j of the device h, in fp32
            z_dev = _z(layer.linear_transform(T(x).to(dev)).cpu(), ei)
        mine = z_dev > 0
        g32b = _oracle_grads(torch.float32, x, ei, kern, att, bias, gout, branch=mine)
        g64b = _oracle_grads(torch.float64, x, ei, kern, att, bias, gout, branch=mine)
        for k in TOL:  # same branch: the fp32 parity contract, and fp64
            assert _err(kg[k], g32b[k]) <= TOL[k], (key, k, "fp32, same branch", _err(kg[k], g32b[k]))
            assert _err(kg[k], g64b[k]) <= TOL[k], (key, k, "fp64, same branch", _err(kg[k], g64b[k]))
        g32 = _oracle_grads(torch.float32, x, ei, kern, att, bias, gout)
        g64 = _oracle_grads(torch.float64, x, ei, kern, att, bias, gout)
        z32 = _z(T(x) @ T(kern), ei)
        z64 = _z(T(x).double() @ T(kern).double(), ei)
        for k in TOL:  # each oracle on its own branches: within tolerance wherever the branches agree
            if bool((mine == (z32 > 0)).all()):
                assert _err(kg[k], g32[k]) <= TOL[k], (key, k, "fp32")
            if bool((mine == (z64 > 0)).all()):
                assert _err(kg[k], g64[k]) <= TOL[k], (key, k, "fp64")
        if bool((mine == (z64 > 0)).all()):  # the kernel is on the fp64 side of every kink
            for k in TOL:
                assert _err(kg[k], g64[k]) <= max(_err(g32[k], g64[k]), TOL[k]), (key, k)
