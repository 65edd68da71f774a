// Per-row reduction semantics (sum / mean / max / min) shared by the fused
// aggregate -> transform kernels, in the reference's order and special cases
// (aggregators.py:56-167): sequential RN adds, fp32 count for the mean, amax
// updates with the empty-row / isinf guard.
#pragma once

#include "kgx.h"
#include "kgx_vec.h"

namespace kgx {

template <int RED>
struct RowRed {
  static __device__ __forceinline__ float init() {
    if constexpr (RED == KGX_MAX || RED == KGX_MIN) return -__builtin_inff();
    return 0.0f;
  }
  static __device__ __forceinline__ float msg(float v) {
    if constexpr (RED == KGX_MIN) return -v;
    return v;
  }
  static __device__ __forceinline__ float combine(float a, float v) {
    if constexpr (RED == KGX_MAX || RED == KGX_MIN) return amax_update(a, v);
    return __fadd_rn(a, v);
  }
  static __device__ __forceinline__ float finish(float a, int32_t deg) {
    if constexpr (RED == KGX_MEAN) return __fdiv_rn(a, fmaxf(ref_count_f32(deg), 1e-8f));
    if constexpr (RED == KGX_MAX) return is_inf(a) ? 0.0f : a;
    if constexpr (RED == KGX_MIN) {
      const float r = -a;
      return is_inf(r) ? 0.0f : r;
    }
    return a;
  }
};

}  // namespace kgx
