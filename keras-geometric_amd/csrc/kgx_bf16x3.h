// Three-way bf16 split of f32 operands ("bf16x3") shared by the MFMA kernels
// (spmm_gemm.hip's fused transform, dense.hip).
//
// x = hi + mid + lo exactly for finite x (each a bf16, round-to-nearest-even
// residuals).  x*w is then taken as the six bf16 x bf16 products whose orders
// sum to <= 2 (dropped terms <= 2^-24 |x w|, the f32 rounding level), each
// exact in the MFMA's f32 accumulator.
//
// Non-finite x (+-inf, NaN) is stored as (hi, mid, lo) = (0, 0, x): the
// only product that meets the lo plane of one operand is the one with the hi
// plane of the other, so x*w becomes exactly x * hi(w) -- IEEE f32's inf*w
// (+-inf, or NaN for w == 0) and NaN propagation.  Keeping x in hi instead
// would multiply inf by w's residual planes, whose zeros and opposite signs
// turn +-inf into NaN.  (Both operands non-finite at once -- an infinite
// weight times an infinite feature -- gives NaN where f32 gives +-inf.)
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
// Branch-free (selects only): the staging loops call this per element.
__device__ __forceinline__ void split3(float x, short& hi, short& mid, short& lo) {
  const bool fin = __builtin_isfinite(x);
  short h0 = bf16_bits(x);
  // |x| near FLT_MAX rounds up to inf: truncate instead
  h0 = __builtin_isfinite(bf16_value(h0)) ? h0 : short(__builtin_bit_cast(uint32_t, x) >> 16);
  const float r1 = __fsub_rn(x, bf16_value(h0));  // exact for finite x
  const short m = bf16_bits(r1);
  const short l = bf16_bits(__fsub_rn(r1, bf16_value(m)));  // exact
  hi = fin ? h0 : short(0);
  mid = fin ? m : short(0);
  lo = fin ? l : bf16_bits(x);  // +-inf / NaN: lo plane only (see above)
}

// Packed split of four values for staging loops (about 5 VALU ops per value
// instead of ~19): pairs go through v_cvt_pk_bf16_f32 and v_pk_add_f32, and
// each plane comes out as a bf16x4 (two packed dwords) ready for one 8-byte
// LDS store.  Valid only when every hi value is finite and their sum does not
// overflow; `bad` is set otherwise (inf / NaN, or |x| near FLT_MAX), and the
// caller redoes those values with split3.
typedef float kgx_f32x2 __attribute__((ext_vector_type(2)));
typedef float kgx_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 kgx_bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t bf16_pack2(kgx_f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, kgx_bf16x2));  // RNE
}
__device__ __forceinline__ kgx_f32x2 bf16_unpack2(uint32_t p) {
  return kgx_f32x2{__builtin_bit_cast(float, p << 16), __builtin_bit_cast(float, p & 0xffff0000u)};
}
__device__ __forceinline__ void split3x4_fast(kgx_f32x4 x, uint32_t (&h)[2], uint32_t (&m)[2], uint32_t (&l)[2],
                                              bool& bad) {
  const kgx_f32x2 a = {x[0], x[1]}, b = {x[2], x[3]};
  h[0] = bf16_pack2(a);
  h[1] = bf16_pack2(b);
  const kgx_f32x2 ha = bf16_unpack2(h[0]), hb = bf16_unpack2(h[1]);
  const kgx_f32x2 hs = ha + hb;
  bad = !__builtin_isfinite(hs[0] + hs[1]);
  kgx_f32x2 ra = a - ha, rb = b - hb;  // exact
  m[0] = bf16_pack2(ra);
  m[1] = bf16_pack2(rb);
  ra = ra - bf16_unpack2(m[0]);  // exact
  rb = rb - bf16_unpack2(m[1]);
  l[0] = bf16_pack2(ra);
  l[1] = bf16_pack2(rb);
}

}  // namespace kgx
