"""The f16x2 operand split (csrc/kgx_f16x2.h) restated in numpy: per-row /
per-column power-of-two scales, RNE fp16 hi plane, RNE fp16 lo residual, three
products (hi*hi, hi*lo, lo*hi) summed in float64 (the MFMA's f32 accumulation
error is the dot product's own and is covered by the GPU tests' bound).

Checks the header's claim: |x w - (xh wh + xh wl + xl wh)| <= 3 * 2^-22 |x w|
per product for values within 2^20 of their row / column maximum, and the
documented absolute floor (2^-39 of the row maximum) below that; and that the
K = 256 dot products stay inside the 4e-6 (|a| |W|) bound the GPU tests use.
"""

import numpy as np
import pytest


def split_f16x2(v: np.ndarray, axis: int):
    """(hi, lo, shift) with v * 2^shift = hi + lo + e, scales per slice along axis."""
    v = v.astype(np.float32)
    a = np.abs(v)
    m = np.where(np.isfinite(a), a, 0).max(axis=axis, keepdims=True).astype(np.float32)
    bits = m.view(np.uint32)
    sh = 14 - ((bits >> 23).astype(np.int32) - 127)
    s = np.ldexp(v, sh).astype(np.float32)
    hi = s.astype(np.float16)
    r = (s - hi.astype(np.float32)).astype(np.float32)  # exact
    lo = r.astype(np.float16)
    return hi, lo, sh


def test_split_represents_values():
    rng = np.random.default_rng(0)
    x = (rng.standard_normal((64, 256)) * np.exp2(rng.integers(-30, 30, (64, 1)))).astype(np.float32)
    hi, lo, sh = split_f16x2(x, axis=1)
    rec = np.ldexp(hi.astype(np.float64) + lo.astype(np.float64), -sh)
    rowmax = np.abs(x).max(axis=1, keepdims=True).astype(np.float64)
    err = np.abs(rec - x.astype(np.float64))
    # relative 2^-22 within 2^10 of the row maximum, absolute 2^-39 of the maximum below
    big = np.abs(x) >= rowmax * 2.0**-10
    assert (err[big] <= 2.0**-22 * np.abs(x[big])).all()
    assert (err <= np.maximum(2.0**-22 * np.abs(x), 2.0**-38 * rowmax)).all()
    assert np.isfinite(hi.astype(np.float32)).all() and np.abs(hi.astype(np.float32)).max() < 65504


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_three_products_within_dot_bound(seed):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((512, 256)).astype(np.float32)
    a[::7] *= np.float32(1e30)  # rows far from 1: the scales keep fp16 in range
    a[1::7] *= np.float32(1e-30)
    W = (rng.standard_normal((256, 64)) * 0.06).astype(np.float32)
    W[:, 3] *= np.float32(1e-20)  # a column far below the others: its own scale
    ah, al, sa = split_f16x2(a, axis=1)
    wh, wl, sw = split_f16x2(W, axis=0)
    A = lambda h: h.astype(np.float64)  # noqa: E731
    d = A(ah) @ A(wh) + A(ah) @ A(wl) + A(al) @ A(wh)
    y = np.ldexp(d, -(sa + sw))
    ref = a.astype(np.float64) @ W.astype(np.float64)
    scale = np.abs(a.astype(np.float64)) @ np.abs(W.astype(np.float64))
    err = np.abs(y - ref)
    assert (err <= 3 * 2.0**-22 * scale).all(), float((err / scale).max())
    assert (err <= 4e-6 * scale).all()


def test_non_finite_to_lo_plane():
    """inf / NaN activations go to the lo plane (hi = 0): lo meets only W's hi
    plane, so x*w is +-inf (NaN for w = 0) as in f32."""
    x = np.array([[1.0, np.inf, -2.0, np.nan]], np.float32)
    fin = np.where(np.isfinite(x), x, 0)
    hi, lo, sh = split_f16x2(fin, axis=1)
    lo = np.where(np.isfinite(x), lo, x.astype(np.float16))
    hi = np.where(np.isfinite(x), hi, np.float16(0))
    w = np.array([0.5, 0.25, 1.0, 3.0], np.float32)
    wh, wl, sw = split_f16x2(w[:, None], axis=0)
    with np.errstate(invalid="ignore"):
        terms = hi[0].astype(np.float32) * wh[:, 0] + hi[0].astype(np.float32) * wl[:, 0] + \
            lo[0].astype(np.float32) * wh[:, 0]
    assert np.isposinf(terms[1]) and np.isnan(terms[3])
