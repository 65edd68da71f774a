// Backward of the segment max / min reduction (kgx_spmm_max_backward).
//
// Forward (Keras-torch lowering, aggregators.py:99-112 / 151-167):
//   m[i,f] = segment_max over the row's messages  (torch scatter_reduce "amax",
//            include_self on a -inf init), then where(isinf(m), 0, m);
//   min    = -segment_max(-msg), then the same isinf guard.
// torch's scatter_reduce amax/amin backward spreads grad[i,f] evenly over the
// edges whose message equals the result (ties share); the isinf guard passes
// no gradient where the result was +-inf (empty rows included).  Per
// (row, feature): pass 1 recomputes the raw extreme in CSR order, pass 2
// counts the ties, pass 3 adds grad/count to every tied edge's source row
// (float atomics: several rows may share a source, so the summation order
// across rows is not fixed -- tolerance-equal, like the reference on GPU).
//
// Sum / mean / weighted-sum backward needs no kernel of its own: it is the
// same kgx_spmm over the transposed graph (graph.transpose, ops.py).
#include "kgx_internal.h"
#include "kgx_vec.h"

namespace kgx {
namespace {

template <int RED>
__global__ __launch_bounds__(kBlock) void max_backward_kernel(int raw, const int32_t* __restrict__ rowptr, int64_t n_rows,
                                                              const int32_t* __restrict__ idx,
                                                              const float* __restrict__ table, int64_t ld_t,
                                                              int64_t F, const float* __restrict__ grad_out,
                                                              int64_t ld_g, float* __restrict__ grad_table,
                                                              int64_t ld_gt) {
  const int64_t total = n_rows * F;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t row = t / F;
    const int64_t f = t - row * F;
    const int32_t beg = rowptr[row], end = rowptr[row + 1];
    // pass 1: the raw extreme, exactly as the forward (NaN sticky, first of ties)
    float m = -__builtin_inff();
    for (int32_t e = beg; e < end; ++e) {
      const float v = table[int64_t(idx[e]) * ld_t + f];
      m = amax_update(m, RED == KGX_MIN ? -v : v);
    }
    if (RED == KGX_MIN) m = -m;
    if (m != m) continue;                         // NaN: no edge equals the result
    if (!raw && __builtin_isinf(m)) continue;     // the aggregators' isinf guard passes nothing
    // pass 2: ties (raw: the -inf init of the scatter counts as one more tie)
    int32_t cnt = (raw && m == (RED == KGX_MIN ? __builtin_inff() : -__builtin_inff())) ? 1 : 0;
    for (int32_t e = beg; e < end; ++e) cnt += table[int64_t(idx[e]) * ld_t + f] == m;
    if (cnt == 0) continue;
    // pass 3: share the gradient
    const float g = __fdiv_rn(grad_out[row * ld_g + f], float(cnt));
    for (int32_t e = beg; e < end; ++e) {
      const int64_t src = idx[e];
      if (table[src * ld_t + f] == m) atomicAdd(grad_table + src * ld_gt + f, g);
    }
  }
}

}  // namespace
}  // namespace kgx

using namespace kgx;

extern "C" int kgx_spmm_max_backward(int reduce, int raw, const int32_t* rowptr, int64_t n_rows, const int32_t* idx,
                                     const float* table, int64_t ld_table, int64_t F, const float* grad_out,
                                     int64_t ld_grad_out, float* grad_table, int64_t ld_grad_table,
                                     kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(reduce == KGX_MAX || reduce == KGX_MIN, KGX_ERR_ARG,
              "kgx_spmm_max_backward: reduce must be MAX or MIN (got %d)", reduce);
  KGX_REQUIRE(n_rows >= 0 && F >= 0, KGX_ERR_ARG, "kgx_spmm_max_backward: negative size");
  if (n_rows == 0 || F == 0) return KGX_OK;
  KGX_REQUIRE(rowptr && idx && table && grad_out && grad_table, KGX_ERR_ARG, "kgx_spmm_max_backward: null pointer");
  KGX_REQUIRE(ld_table >= F && ld_grad_out >= F && ld_grad_table >= F, KGX_ERR_ARG,
              "kgx_spmm_max_backward: leading dimension < F");
  const unsigned grid = grid_for(n_rows * F, 16384);
  if (reduce == KGX_MAX)
    hipLaunchKernelGGL(max_backward_kernel<KGX_MAX>, dim3(grid), dim3(kBlock), 0, stream, raw, rowptr, n_rows, idx, table,
                       ld_table, F, grad_out, ld_grad_out, grad_table, ld_grad_table);
  else
    hipLaunchKernelGGL(max_backward_kernel<KGX_MIN>, dim3(grid), dim3(kBlock), 0, stream, raw, rowptr, n_rows, idx, table,
                       ld_table, F, grad_out, ld_grad_out, grad_table, ld_grad_table);
  KGX_CHECK_LAUNCH();
  return KGX_OK;
}

namespace kgx {
namespace {

__global__ __launch_bounds__(kBlock) void dropout_mask_kernel(uint64_t seed, uint32_t thresh, float keep_scale,
                                                              const int32_t* __restrict__ keys, int64_t n,
                                                              int64_t F, float* __restrict__ out) {
  const int64_t total = n * F;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t i = t / F;
    out[t] = drop_scale(seed, uint32_t(keys[i]), uint32_t(t - i * F), thresh, keep_scale);
  }
}

}  // namespace
}  // namespace kgx

extern "C" int kgx_dropout_mask(uint64_t seed, float p, const int32_t* keys, int64_t n, int64_t F, float* out,
                                kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(n >= 0 && F >= 0 && p >= 0.0f && p < 1.0f, KGX_ERR_ARG, "kgx_dropout_mask: bad arguments");
  if (n == 0 || F == 0) return KGX_OK;
  KGX_REQUIRE(keys && out, KGX_ERR_ARG, "kgx_dropout_mask: null pointer");
  const uint32_t thresh = p > 0.0f ? uint32_t(double(p) * 4294967296.0) : 0u;
  const float scale = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  hipLaunchKernelGGL(dropout_mask_kernel, dim3(grid_for(n * F, 16384)), dim3(kBlock), 0, stream, seed, thresh, scale,
                     keys, n, F, out);
  KGX_CHECK_LAUNCH();
  return KGX_OK;
}

