"""kgx_gemm_tn: dW = P^T D and db = colsum(D) in one pass (the weight and bias
gradients of the fused layers' and kgx_dense's backward), against float64.

Bound: the bf16x3 products are f32-accurate and the sum over N nodes is
re-associated (32-node MFMA steps, per-block chains, block partials summed in
order), so |dW - ref| <= 1e-5 * sum_n |P[n,k]| |D[n,m]| (+ tiny); db likewise
against sum_n |D[n,m]|.  Non-finite inputs take the f32 slow path: IEEE
propagation, compared position by position with float64's inf / NaN pattern."""

import numpy as np
import pytest
import torch

from keras_geometric_amd import ops as kops

pytestmark = [pytest.mark.gpu]


def _check(P, D, with_db=True):
    dW, db = kops.gemm_tn(P, D, with_db=with_db)
    P64, D64 = P.double(), D.double()
    ref = P64.t() @ D64
    mag = P64.abs().t() @ D64.abs()
    err = (dW.double() - ref).abs()
    assert bool((err <= 1e-5 * mag + 1e-30).all()), float((err / mag.clamp_min(1e-30)).max())
    if with_db:
        rb = D64.sum(0)
        eb = (db.double() - rb).abs()
        assert bool((eb <= 1e-5 * D64.abs().sum(0) + 1e-30).all())
    else:
        assert db is None
    return dW, db


@pytest.mark.parametrize("N", [1, 31, 33, 1000, 100_003])
@pytest.mark.parametrize("K,M", [(128, 128), (100, 100), (64, 200), (256, 256), (8, 4), (129, 17)])
def test_gemm_tn_shapes(N, K, M, dev):
    gen = torch.Generator(device=dev).manual_seed(N * 7 + K)
    P = torch.randn(N, K, device=dev, generator=gen)
    D = torch.randn(N, M, device=dev, generator=gen)
    _check(P, D, with_db=(K + M) % 2 == 0)


def test_gemm_tn_strided_and_fullsize(dev):
    """Row strides != width (column slices of wider tensors) and the north-star
    row count (10M nodes, 128 x 128)."""
    gen = torch.Generator(device=dev).manual_seed(3)
    big = torch.randn(20_000, 300, device=dev, generator=gen)
    _check(big[:, 10:138], big[:, 150:278])
    N = 10_000_000
    P = torch.randn(N, 128, device=dev, generator=gen)
    D = torch.randn(N, 128, device=dev, generator=gen)
    dW, db = kops.gemm_tn(P, D, with_db=True)
    ref = torch.zeros(128, 128, dtype=torch.float64, device=dev)
    mag = torch.zeros_like(ref)
    for i in range(0, N, 1_000_000):
        p, d = P[i:i + 1_000_000].double(), D[i:i + 1_000_000].double()
        ref += p.t() @ d
        mag += p.abs().t() @ d.abs()
    assert bool(((dW.double() - ref).abs() <= 1e-5 * mag).all())
    assert bool(((db.double() - D.double().sum(0)).abs() <= 1e-5 * D.double().abs().sum(0)).all())


def test_gemm_tn_nonfinite(dev):
    gen = torch.Generator(device=dev).manual_seed(4)
    N, K, M = 5000, 128, 64
    P = torch.randn(N, K, device=dev, generator=gen)
    D = torch.randn(N, M, device=dev, generator=gen)
    P[17, 3] = float("inf")
    P[4000, 9] = float("nan")
    D[123, 5] = -float("inf")
    dW, db = kops.gemm_tn(P, D, with_db=True)
    ref = (P.double().t() @ D.double())
    fin = torch.isfinite(ref)
    assert torch.equal(torch.isnan(dW), torch.isnan(ref)) and torch.equal(torch.isinf(dW), torch.isinf(ref))
    assert torch.equal(torch.sign(dW[torch.isinf(ref)]), torch.sign(ref[torch.isinf(ref)]).float())
    mag = P.double().abs().t() @ D.double().abs()
    assert bool(((dW.double() - ref).abs()[fin] <= 1e-5 * mag[fin] + 1e-30).all())
    rb = D.double().sum(0)
    assert torch.equal(torch.isinf(db), torch.isinf(rb))


def test_gemm_tn_huge_finite(dev):
    """A finite value whose bf16 rounding overflows (|x| >= 0x1.ffp127) is not split exactly: its
    block takes the plain f32 path and the result stays finite and f32-accurate."""
    gen = torch.Generator(device=dev).manual_seed(5)
    N, K, M = 5000, 128, 128
    P = torch.randn(N, K, device=dev, generator=gen)
    D = torch.randn(N, M, device=dev, generator=gen)
    P[250, 7] = 3.4e38  # bf16 RNE: inf
    D[250] *= 1e-3
    D[2600, 100] = -3.39e38  # bf16 RNE: the largest finite bf16
    P[2600] *= 1e-3
    dW, db = kops.gemm_tn(P, D, with_db=True)
    ref = P.double().t() @ D.double()
    mag = P.double().abs().t() @ D.double().abs()
    assert bool(torch.isfinite(dW).all()) and bool(torch.isfinite(db).all())
    assert bool(((dW.double() - ref).abs() <= 1e-5 * mag).all())
    assert bool(((db.double() - D.double().sum(0)).abs() <= 1e-5 * D.double().abs().sum(0)).all())


def test_gemm_tn_zero_rows(dev):
    P = torch.empty(0, 128, device=dev)
    D = torch.empty(0, 64, device=dev)
    dW, db = kops.gemm_tn(P, D, with_db=True)
    assert torch.equal(dW, torch.zeros(128, 64, device=dev)) and torch.equal(db, torch.zeros(64, device=dev))
