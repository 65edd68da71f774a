// Two-way fp16 split of f32 operands with power-of-two scaling ("f16x2"), the
// 256-wide fused kernels' transform (spmm_gemm256.hip, KGX_F256_SPLIT = 2).
//
// bf16x3 (kgx_bf16x3.h) needs six bf16 MFMAs per f32 product; fp16 carries 11
// significant bits against bf16's 8, so two planes hold 22 bits and THREE
// products (hi*hi, hi*lo, lo*hi) give
//   |x w - (xh wh + xh wl + xl wh)| <= (2^-22 + 2^-22 + 2^-22) |x w|
// (representation of x, of w, the dropped lo*lo term), 2^-20.4 |x w|: about
// 12x f32's unit roundoff per product, far inside the forward-error bound of
// the K = 256 f32 dot product the MFMA accumulates (K u = 2^-16 |x| |w|).
// fp16's range (max 65504, normal min 2^-14) is the catch: every tile row is
// scaled by its own power of two so its largest finite magnitude lies in
// [2^14, 2^15), every W column likewise; the MFMA sums the scaled products in
// f32 (at most 2^38, no overflow) and the epilogue undoes both scales with one
// exact v_ldexp_f32.  Values more than ~2^28 below their row's maximum lose
// bits to fp16 subnormals: absolute error <= 2^-39 of the row maximum.
//
// Infinities / NaN: as in bf16x3, a non-finite activation goes to the lo plane
// (hi = 0), which meets only W's hi plane, so x*w is +-inf (NaN for w = 0) as
// in f32; the row's scale comes from its finite values.  Infinite weights are
// not covered (their lo residual is NaN).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace kgx {

typedef _Float16 kgx_h8_t __attribute__((ext_vector_type(8)));
typedef _Float16 kgx_h2_t __attribute__((ext_vector_type(2)));
typedef float kgx_f2v_t __attribute__((ext_vector_type(2)));

// maximum of v over the wave's 64 lanes (every lane active), wave-uniform:
// DPP within each 16-lane row, then the four rows' values through readlane
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0xB1, 0xF, 0xF, false)));   // quad_perm 1,0,3,2
  v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x4E, 0xF, 0xF, false)));   // quad_perm 2,3,0,1
  v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x141, 0xF, 0xF, false)));  // row_half_mirror
  v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x140, 0xF, 0xF, false)));  // row_mirror
  const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
  const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  return max(max(a, b), max(c, d));
}

// maximum of v over each 32-lane half of the wave (lanes 0-31, 32-63: the
// 128-wide kernels' row groups), every lane active; each lane gets its half's
__device__ __forceinline__ uint32_t half_max_u32(uint32_t v) {
  v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0xB1, 0xF, 0xF, false)));
  v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x4E, 0xF, 0xF, false)));
  v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x141, 0xF, 0xF, false)));
  v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x140, 0xF, 0xF, false)));
  const uint32_t lo = max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16));
  const uint32_t hi = max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48));
  return (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 32) ? hi : lo;
}

// |x| as bits (monotone in |x| for finite x; inf / NaN above 0x7f7fffff)
__device__ __forceinline__ uint32_t abs_bits(float x) { return __builtin_bit_cast(uint32_t, x) & 0x7fffffffu; }

// scale exponent for a largest finite magnitude with bits m: x * 2^sh has its
// maximum in [2^14, 2^15) (m a normal) or below it (denormal m, zero row)
__device__ __forceinline__ int h2_shift(uint32_t m) { return 14 - (int(m >> 23) - 127); }

// finite x: x 2^sh = f32(hi) + f32(lo) + e, |e| <= 2^-22 |x 2^sh| (+ fp16 subnormal steps);
// a pair packed, element 0 in the low half
__device__ __forceinline__ void split2h_pair(float a, float b, int sh, uint32_t& hi, uint32_t& lo) {
  const kgx_f2v_t v = {__builtin_ldexpf(a, sh), __builtin_ldexpf(b, sh)};
  const kgx_h2_t h = __builtin_convertvector(v, kgx_h2_t);  // v_cvt_pk_f16_f32, RNE
  const kgx_f2v_t hf = __builtin_convertvector(h, kgx_f2v_t);
  const kgx_f2v_t r = {__fsub_rn(v[0], hf[0]), __fsub_rn(v[1], hf[1])};  // exact
  hi = __builtin_bit_cast(uint32_t, h);
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, kgx_h2_t));
}

// the rare path: non-finite values to the lo plane (hi = 0, lo = +-inf / NaN)
__device__ __forceinline__ void split2h_pair_nf(float a, float b, int sh, uint32_t& hi, uint32_t& lo) {
  split2h_pair(__builtin_isfinite(a) ? a : 0.0f, __builtin_isfinite(b) ? b : 0.0f, sh, hi, lo);
  if (!__builtin_isfinite(a)) {
    hi &= 0xffff0000u;
    lo = (lo & 0xffff0000u) | uint32_t(__builtin_bit_cast(uint16_t, static_cast<_Float16>(a)));
  }
  if (!__builtin_isfinite(b)) {
    hi &= 0x0000ffffu;
    lo = (lo & 0x0000ffffu) | (uint32_t(__builtin_bit_cast(uint16_t, static_cast<_Float16>(b))) << 16);
  }
}

// A 128-wide row held by a 32-lane group (four values per lane; both groups of
// the wave call this together) -> this lane's packed hi / lo planes; returns
// the row's unscale exponent.  A row with an inf / NaN gives non-finite
// outputs in every column (inf * w, or inf * 0 = NaN, as in f32), so its scale
// is taken with those magnitudes clamped to FLT_MAX (one reduction) and only
// the non-finite values' own placement (the lo plane) matters.
__device__ __forceinline__ int split_row_h2_half(const float (&v)[4], uint2& ph, uint2& pl) {
  const uint32_t raw = max(max(abs_bits(v[0]), abs_bits(v[1])), max(abs_bits(v[2]), abs_bits(v[3])));
  const int sh = h2_shift(half_max_u32(min(raw, 0x7f7fffffu)));
  uint32_t h0, l0, h1, l1;
  if (raw < 0x7f800000u) {
    split2h_pair(v[0], v[1], sh, h0, l0);
    split2h_pair(v[2], v[3], sh, h1, l1);
  } else {
    split2h_pair_nf(v[0], v[1], sh, h0, l0);
    split2h_pair_nf(v[2], v[3], sh, h1, l1);
  }
  ph = make_uint2(h0, h1);
  pl = make_uint2(l0, l1);
  return -sh;
}

}  // namespace kgx
