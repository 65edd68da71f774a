// Vector load/store helpers and reference-exact scalar semantics shared by the
// aggregation kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace kgx {

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// 1 KB of zeros in every code object, never written.  A row gather whose edge
// is absent (past a row's degree, or a past-the-end item) reads this row
// instead of being skipped under an exec mask: every lane of the wave issues
// the same loads on every path, so no gather destination is a partially
// written register and the compiler's vmcnt accounting is path-independent.
// The fold masks the value.  Offsets up to 256 floats (a 64-lane x float4 row).
namespace {
[[maybe_unused]] __device__ __attribute__((aligned(16))) float kgx_zero_row[256];
}

// Load/store VEC consecutive floats (VEC in {1,2,4,8,16}; >=4 uses float4 pieces).
template <int VEC>
__device__ __forceinline__ void vload(float (&d)[VEC], const float* __restrict__ p) {
  if constexpr (VEC >= 4) {
#pragma unroll
    for (int i = 0; i < VEC / 4; ++i) {
      const float4 v = reinterpret_cast<const float4*>(p)[i];
      d[4 * i + 0] = v.x;
      d[4 * i + 1] = v.y;
      d[4 * i + 2] = v.z;
      d[4 * i + 3] = v.w;
    }
  } else if constexpr (VEC == 2) {
    const float2 v = *reinterpret_cast<const float2*>(p);
    d[0] = v.x;
    d[1] = v.y;
  } else {
    d[0] = *p;
  }
}

template <int VEC>
__device__ __forceinline__ void vstore(float* __restrict__ p, const float (&d)[VEC]) {
  if constexpr (VEC >= 4) {
#pragma unroll
    for (int i = 0; i < VEC / 4; ++i)
      reinterpret_cast<float4*>(p)[i] = make_float4(d[4 * i], d[4 * i + 1], d[4 * i + 2], d[4 * i + 3]);
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(d[0], d[1]);
  } else {
    *p = d[0];
  }
}

// Non-temporal variants (global_load/store ... nt): for data streamed once
// (CSR indices / weights, output rows) so it does not displace reused rows.

template <int VEC>
__device__ __forceinline__ void vstore_nt(float* __restrict__ p, const float (&d)[VEC]) {
  if constexpr (VEC >= 4) {
#pragma unroll
    for (int i = 0; i < VEC / 4; ++i) {
      f32x4_t v = {d[4 * i], d[4 * i + 1], d[4 * i + 2], d[4 * i + 3]};
      __builtin_nontemporal_store(v, reinterpret_cast<f32x4_t*>(p) + i);
    }
  } else if constexpr (VEC == 2) {
    f32x2_t v = {d[0], d[1]};
    __builtin_nontemporal_store(v, reinterpret_cast<f32x2_t*>(p));
  } else {
    __builtin_nontemporal_store(d[0], p);
  }
}

template <typename T>
__device__ __forceinline__ T ld_nt(const T* p) {
  return __builtin_nontemporal_load(p);
}

// fp32 degree as the reference computes it: segment_sum of fp32 ones, which a
// sequential fp32 accumulation saturates at 2^24 (aggregators.py:66-69,194-196).
__device__ __forceinline__ float ref_count_f32(int32_t n) {
  return float(n < (1 << 24) ? n : (1 << 24));
}

// torch scatter_reduce "amax" update: self = isnan(src) ? src : max(self, src),
// std::max keeps `self` on ties (so -0 vs +0 keeps the first seen).
__device__ __forceinline__ float amax_update(float acc, float v) {
  return (v > acc || v != v) ? v : acc;
}

__device__ __forceinline__ bool is_inf(float v) { return __builtin_isinf(v); }

// Row offset idx * ld for a gathered row: both operands are non-negative and
// below 2^32 (checked at the C-ABI), so one 32x32->64 v_mad_u64_u32 replaces
// the sign-extended 64-bit multiply (six VALU ops, three of them quarter rate)
// the int64 expression compiles to -- per gathered row, in the hot loops.
__device__ __forceinline__ uint64_t row_off(int32_t idx, int64_t ld) {
  return uint64_t(uint32_t(idx)) * uint32_t(ld);
}

// Counter-based dropout mask: element (key, f) is kept iff the high 32 bits of
// splitmix64(seed ^ (key << 32 | f) * golden) are >= thresh = p * 2^32.  A
// function of (seed, edge id, feature) only, so the forward, its backward over
// the transposed graph and the test oracle (kgx_dropout_mask) agree.
__host__ __device__ __forceinline__ uint32_t drop_hash(uint64_t seed, uint32_t key, uint32_t f) {
  uint64_t z = seed ^ ((uint64_t(key) << 32 | f) * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return uint32_t(z >> 32);
}
__device__ __forceinline__ float drop_scale(uint64_t seed, uint32_t key, uint32_t f, uint32_t thresh, float keep_scale) {
  return drop_hash(seed, key, f) >= thresh ? keep_scale : 0.0f;
}

// IEEE round-to-nearest sqrt.  NOTE: on gfx950 `__fsqrt_rn` lowers to a bare
// v_sqrt_f32 (~1 ulp); plain sqrtf under hipcc's default
// -fhip-fp32-correctly-rounded-divide-sqrt expands to v_sqrt + an fma-based
// correction and is correctly rounded, like the CPU's vsqrtps.
__device__ __forceinline__ float sqrt_rn(float x) { return sqrtf(x); }

}  // namespace kgx
