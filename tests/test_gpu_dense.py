"""kgx_dense (bf16x3-split MFMA node transform) vs an fp64 torch reference (GPU).

The layers' keras Dense / ops.matmul (gin_conv.py:129-162, sage_conv.py:407-428,
gatv2_conv.py:224-239) compute in fp32; kgx_dense must match an fp32 GEMM to
fp32 accuracy.  Tolerance (written here, as the north star asks):
|a - b| <= 1e-5 * max(1, |b|) against the fp64 product, and no worse than 4x
torch's own fp32 GEMM error on the same inputs.
"""

import numpy as np
import pytest
import torch

from keras_geometric_amd import _native as nat
from keras_geometric_amd import ops as kops

pytestmark = pytest.mark.gpu
TOL = 1e-5


def ref64(x0, W0, x1=None, W1=None, bias=None, relu=False):
    y = x0.double() @ W0.double()
    if x1 is not None:
        y = y + x1.double() @ W1.double()
    if bias is not None:
        y = y + bias.double()
    return torch.relu(y) if relu else y


def scaled_err(a, b):
    a, b = a.double(), b.double()
    m = torch.isfinite(b)
    if not m.any():
        return 0.0
    return ((a[m] - b[m]).abs() / b[m].abs().clamp_min(1.0)).max().item()


def glorot(k, n, g):
    lim = (6.0 / (k + n)) ** 0.5
    return (torch.rand(k, n, generator=g) * 2 - 1) * lim


SHAPES = [  # (M, K0, K1, N)
    (1000, 128, 0, 128),    # GATv2 / GCN x W (C3 shape)
    (777, 256, 0, 256),     # GIN MLP Dense (C4 shape, two column groups)
    (1234, 100, 100, 100),  # SAGE lin_self + lin_neigh (C5 shape)
    (50, 4, 0, 7),          # tiny, N not a multiple of 16
    (33, 64, 0, 64),
    (4099, 160, 0, 192),    # K 160 (5 k-steps), N 192
    (300, 252, 4, 200),
    (17, 32, 32, 48),
    (20000, 96, 0, 130),    # N just over 128 (second group nearly empty)
]


@pytest.mark.parametrize("M,K0,K1,N", SHAPES)
@pytest.mark.parametrize("bias,relu", [(True, False), (False, False), (True, True)])
def test_dense_matches_fp64(dev, M, K0, K1, N, bias, relu):
    g = torch.Generator().manual_seed(M * 7 + K0 + N)
    x0 = torch.randn(M, K0, generator=g)
    W0 = glorot(K0, N, g)
    x1 = torch.randn(M, K1, generator=g) if K1 else None
    W1 = glorot(K1, N, g) if K1 else None
    b = torch.randn(N, generator=g) if bias else None
    cu = lambda t: None if t is None else t.to(dev)
    assert kops.dense_supported(cu(x0), cu(W0), cu(W1))
    y = torch.ops.kgx.dense(cu(x0), cu(W0), cu(x1), cu(W1), cu(b), relu).cpu()
    ref = ref64(x0, W0, x1, W1, b, relu)
    err = scaled_err(y, ref)
    assert err <= TOL, f"max scaled err {err:.3e}"
    # no worse than the fp32 library GEMM (hipBLASLt) on the same inputs
    y32 = cu(x0) @ cu(W0)
    if K1:
        y32 = y32 + cu(x1) @ cu(W1)
    if bias:
        y32 = y32 + cu(b)
    if relu:
        y32 = torch.relu(y32)
    err32 = scaled_err(y32.cpu(), ref)
    assert err <= max(4 * err32, 2e-6), f"kgx {err:.3e} vs fp32 GEMM {err32:.3e}"


def test_dense_strided_and_unaligned_inputs(dev):
    g = torch.Generator().manual_seed(3)
    base = torch.randn(500, 140, generator=g).to(dev)
    x0 = base[:, 4:132]  # ld 140, 16-byte aligned start
    W0 = glorot(128, 64, g).to(dev)
    y = kops.dense(x0, W0)
    assert scaled_err(y.cpu(), ref64(x0.cpu(), W0.cpu())) <= TOL
    x_odd = base.reshape(-1)[1:1 + 500 * 128].view(500, 128)  # 4-byte offset: copied to an aligned buffer
    y = kops.dense(x_odd, W0)
    assert scaled_err(y.cpu(), ref64(x_odd.cpu(), W0.cpu())) <= TOL


def test_dense_nonfinite_propagates(dev):
    x = torch.randn(64, 32)
    W = glorot(32, 32, torch.Generator().manual_seed(0))
    x[3, 5] = float("nan")
    x[10, 0] = float("inf")
    y = torch.ops.kgx.dense(x.to(dev), W.to(dev), None, None, None, False).cpu()
    ref = x @ W
    assert torch.equal(torch.isnan(y), torch.isnan(ref))
    assert torch.equal(torch.isinf(y), torch.isinf(ref))
    m = torch.isfinite(ref)
    assert scaled_err(y[m], ref[m].double()) <= TOL


@pytest.mark.parametrize("K", [128, 256])
def test_dense_huge_finite_pairs(dev, K):
    """Finite activations whose RNE bf16 rounds to inf (|x| >= 0x1.ffp127),
    paired with a cancelling partner in the same float4 (a signed
    running sum hid them from the fast split's guard, which then produced NaN):
    every output stays finite and f32-accurate."""
    g = torch.Generator().manual_seed(K)
    x = torch.randn(96, K, generator=g)
    W = glorot(K, 64, g) * 0.5
    x[5, 0], x[5, 2] = -1.70e38, 3.397e38   # the advisor's pair: 2x overflows, the fma chain did not
    x[9, 4], x[9, 5] = 3.40e38, -3.40e38    # exact cancellation
    x[40, K - 1] = -3.4028e38               # a lone near-FLT_MAX value
    y = torch.ops.kgx.dense(x.to(dev), W.to(dev), None, None, None, False).cpu()
    ref = ref64(x, W)
    assert bool(torch.isfinite(y).all())
    assert scaled_err(y, ref) <= TOL


def test_dense_empty_and_limits(dev):
    W = torch.randn(128, 64, device=dev)
    assert torch.ops.kgx.dense(torch.empty(0, 128, device=dev), W, None, None, None, False).shape == (0, 64)
    assert not kops.dense_supported(torch.empty(4, 260, device=dev), torch.empty(260, 8, device=dev))
    assert not kops.dense_supported(torch.empty(4, 6, device=dev), torch.empty(6, 8, device=dev))
    with pytest.raises(ValueError, match="K0 \\+ K1"):
        torch.ops.kgx.dense(torch.empty(4, 260, device=dev), torch.empty(260, 8, device=dev), None, None, None,
                            False)
    # unsupported shapes run as the library GEMM through kops.dense
    x = torch.randn(10, 6, device=dev)
    W6 = torch.randn(6, 8, device=dev)
    assert torch.allclose(kops.dense(x, W6), x @ W6)


def test_dense_autograd(dev):
    g = torch.Generator().manual_seed(5)
    x0 = torch.randn(300, 100, generator=g, dtype=torch.float64)
    x1 = torch.randn(300, 100, generator=g, dtype=torch.float64)
    W0 = glorot(100, 100, g).double()
    W1 = glorot(100, 100, g).double()
    b = torch.randn(100, generator=g, dtype=torch.float64)
    leaves64 = [t.clone().requires_grad_() for t in (x0, W0, x1, W1, b)]
    y64 = torch.relu(leaves64[0] @ leaves64[1] + leaves64[2] @ leaves64[3] + leaves64[4])
    gy = torch.randn_like(y64)
    (y64 * gy).sum().backward()
    leaves = [t.float().to(dev).requires_grad_() for t in (x0, W0, x1, W1, b)]
    y = kops.dense(leaves[0], leaves[1], leaves[4], x1=leaves[2], W1=leaves[3], relu=True)
    (y * gy.float().to(dev)).sum().backward()
    assert scaled_err(y.detach().cpu(), y64.detach()) <= TOL
    for got, want in zip(leaves, leaves64):
        e = scaled_err(got.grad.cpu(), want.grad)
        assert e <= 1e-4, f"grad err {e:.3e}"
