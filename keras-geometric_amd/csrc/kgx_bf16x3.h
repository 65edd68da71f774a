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

}  // namespace kgx
