// Three-way bf16 split of f32 operands ("bf16x3") shared by the MFMA kernels
// (spmm_gemm.hip's fused transform, dense.hip).
//
// x = hi + mid + lo exactly for finite x (each a bf16, round-to-nearest-even
// residuals).  x*w is then taken as the six bf16 x bf16 products whose orders
// sum to <= 2 (dropped terms <= 2^-24 |x w|, the f32 rounding level), each
// exact in the MFMA's f32 accumulator.
//
// Infinities: weights are split with split3_a; activations with split3_a_lo,
// which stores a non-finite x as (hi, mid, lo) = (0, 0, x).  The lo plane of
// one operand meets only the hi plane of the other, so x*w becomes exactly
// x * hi(w) -- IEEE f32's +-inf (or NaN for w = 0) and NaN propagation.  Kept
// in hi, inf would also meet w's residual planes, whose zeros (inf * 0) and
// opposite signs (inf - inf) turn +-inf into NaN.  Not covered: infinite
// weights (their zero residuals meet the activations' planes).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace kgx {

__device__ __forceinline__ short bf16_bits(float x) {
  const __bf16 h = static_cast<__bf16>(x);  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return __builtin_bit_cast(short, h);
}
__device__ __forceinline__ float bf16_value(short b) {
  return __builtin_bit_cast(float, static_cast<uint32_t>(static_cast<uint16_t>(b)) << 16);
}

// RNE split; a non-finite x stays in hi with zero residuals (weights)
__device__ __forceinline__ void split3_a(float x, short& hi, short& mid, short& lo) {
  hi = bf16_bits(x);
  const float h = bf16_value(hi);
  float r = __builtin_isfinite(h) ? __fsub_rn(x, h) : 0.0f;  // exact
  mid = bf16_bits(r);
  r = __fsub_rn(r, bf16_value(mid));  // exact
  lo = bf16_bits(r);
}

// activation split for the rare path: non-finite values moved to the lo plane,
// (0, 0, x); a finite x whose RNE bf16 overflows (|x| >= 0x1.ffp127) keeps
// bf16's largest finite value (rounded toward zero) in hi, so x = hi + mid +
// lo still holds exactly (Sterbenz: x - hi is exact) and x*w stays finite.
__device__ __forceinline__ void split3_a_lo(float x, short& hi, short& mid, short& lo) {
  if (__builtin_isfinite(x)) {
    short h = bf16_bits(x);
    if (!__builtin_isfinite(bf16_value(h))) h = x < 0.0f ? short(0xff7f) : short(0x7f7f);
    float r = __fsub_rn(x, bf16_value(h));  // exact
    const short m = bf16_bits(r);
    r = __fsub_rn(r, bf16_value(m));  // exact
    hi = h;
    mid = m;
    lo = bf16_bits(r);
  } else {
    hi = 0;
    mid = 0;
    lo = bf16_bits(x);  // +-inf or NaN
  }
}

// The fast split (split3_a) is exact for four values iff none is inf / NaN
// (their sum is then finite) and their largest magnitude is below 0x1.ffp127
// (RNE to bf16 then stays finite: no cancellation in the sum can hide a huge
// pair).  Otherwise the caller takes split3_a_lo.
__device__ __forceinline__ bool split_fast_ok(float a, float b, float c, float d) {
  const float m = fmaxf(fmaxf(fabsf(a), fabsf(b)), fmaxf(fabsf(c), fabsf(d)));
  return __builtin_isfinite(__fadd_rn(__fadd_rn(a, b), __fadd_rn(c, d))) && m < 0x1.ffp127f;
}

// split3_a of a pair, packed (element 0 in the low half): fragments assembled
// from 32-bit words keep the compiler from holding unpacked 16-bit copies
// across the main loops.
__device__ __forceinline__ void split3_pair(float w0, float w1, uint32_t& hi, uint32_t& mid, uint32_t& lo) {
  short h0, m0, l0, h1, m1, l1;
  split3_a(w0, h0, m0, l0);
  split3_a(w1, h1, m1, l1);
  hi = uint32_t(uint16_t(h0)) | (uint32_t(uint16_t(h1)) << 16);
  mid = uint32_t(uint16_t(m0)) | (uint32_t(uint16_t(m1)) << 16);
  lo = uint32_t(uint16_t(l0)) | (uint32_t(uint16_t(l1)) << 16);
}

typedef float kgx_f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 kgx_bf16x2_t __attribute__((ext_vector_type(2)));

// two RNE bf16 conversions in one v_cvt_pk_bf16_f32 (a in the low half)
__device__ __forceinline__ uint32_t bf16_pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((kgx_f32x2_t{a, b}), kgx_bf16x2_t));
}

// split3_a of a pair, packed, in 9 VALU ops (three packed conversions; the
// planes' f32 values are the packed words shifted / masked).  Equal to
// split3_a element by element whenever bf16(a) and bf16(b) are finite; the
// caller checks that (dense.hip: a non-finite running sum of 2x sends the
// thread's slots to split3_a_lo).
__device__ __forceinline__ void split3_pair_rn(float a, float b, uint32_t& hi, uint32_t& mid, uint32_t& lo) {
  hi = bf16_pack2(a, b);
  const float ra = __fsub_rn(a, __builtin_bit_cast(float, hi << 16));
  const float rb = __fsub_rn(b, __builtin_bit_cast(float, hi & 0xffff0000u));
  mid = bf16_pack2(ra, rb);
  lo = bf16_pack2(__fsub_rn(ra, __builtin_bit_cast(float, mid << 16)),
                  __fsub_rn(rb, __builtin_bit_cast(float, mid & 0xffff0000u)));
}

}  // namespace kgx
