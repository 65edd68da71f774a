// Fused aggregate -> dense transform for the kgx engine (gfx950, wave64).
//
//   out[i, :] = bias + PRE( REDUCE_{e in CSR row i} x[col_e, :] * (w_e) ) @ W
//
// GCNConv's reference order is transform-then-aggregate (per-edge x_j @ W,
// gcn_conv.py:233-248); for F_in <= F_out the same linear map applied after
// the (linear) aggregation reads the narrower rows and needs no [N, F_out]
// intermediate: the separate X.W GEMM pass (read X, write H: 10.24 GB at the
// north-star size) disappears.  The result differs from the reference's by
// re-association only (tolerance-checked, not bit-checked).
//
// Block = 512 threads = 16 row-groups of 32 lanes (F_in = 128: float4 per
// lane; F_in < 128, a multiple of 4: the lanes past it re-load column 0 and
// put zeros in the planes, W's rows past F_in load as zero).  Per iteration the block takes 16 consecutive schedule items; each
// group reduces its item's edges exactly like spmm_kernel (4 gathers in
// flight, sequential RN adds) and writes the row, split three ways into bf16
// hi/mid/lo planes, to an LDS tile; then wave w (of 8) computes output columns
// [16w, 16w+16) of the 16-row tile with 24 v_mfma_f32_16x16x32_bf16 (the six
// significant cross products of the split operands over K = 128), W's split
// fragments held in 48 VGPRs per lane for the whole kernel.  The split product
// is f32-accurate (dropped terms <= 2^-24 |x w|) and runs at 16x the per-clock
// rate of the f32-input MFMA, which on this kernel could not be hidden behind
// the gathers (NS: 11.37 ms with f32 MFMA, 10.43 with the split; 10.3 with no
// MFMA at all).  The next tile's first U rows are prefetched before the MFMA
// phase; barriers are LDS-only so those gathers stay in flight.  Hub-row
// chunks write raw partials; the fix-up kernel combines them and applies W in
// f32 on the VALU.
#include <cstdlib>
#include <type_traits>

#include "kgx_bf16x3.h"
#include "kgx_internal.h"
#include "kgx_vec.h"

namespace kgx {
namespace {

constexpr int kFin = 128;
constexpr int kGroups = 16;       // rows per block iteration
constexpr int kThreads = kGroups * 32;
constexpr int kTileLd = kFin + 4;  // padded LDS row of the short-row kernel's f32 out tile

typedef float f32x4 __attribute__((ext_vector_type(4)));

// The transform's operand split, the same in the main, short-row and tiny-row
// kernels so their outputs stay bit-identical to each other: three bf16 planes
// (hi / mid / lo), six MFMAs per k-step, W's fragments in 48 VGPRs
// (kgx_bf16x3.h).  Measured alternatives (the f32-input MFMA, the f16x2 split,
// f32 LDS out tiles in the main and tiny kernels) are kept out of this file:
// tools/experiments/round4_variants.patch.
constexpr int kFPlanes = 3;

struct FusedArgs {
  const int32_t* rowptr;
  const int32_t* rows;
  int64_t n_rows;
  const int4* items;
  int64_t n_items;
  int64_t n_long;  // items [0, n_long): spmm_gemm_kernel; [n_long, n_items): rows of degree <= kShortMax
  const int4* split;
  int64_t n_split;
  const int32_t* idx;
  const float* w;
  const float* x;  // [*, 128] gathered rows
  int64_t ld_x;
  const float* W;  // [F_in, F_out] row-major
  int F_in;   // <= 128: lanes past it gather nothing new and carry zeros
  int F_out;
  const float* bias;  // [F_out] or null
  float* out;
  int64_t ld_o;
  float* partials;  // [n_slots, 128]
  float* agg_out;   // optional [n, 128]: the aggregated rows before the transform (kept for backward)
  int64_t ld_agg;
  int pre_gin;      // apply gin_scale * x[row] + aggr before the transform
  int accumulate;   // out += result
  int share_gpu;    // launch (den - 1) / den of the resident grid (shared_cap)
  int relu;         // out = max(result, 0), after the accumulate
  float gin_scale;
  int64_t n_short_end;  // items [n_long, n_short_end): spmm_gemm_short_kernel
  const int4* tpack;    // rows of degree <= 2 as {row, degree, col0, col1} (spmm_gemm_tiny_kernel)
  const float2* tw;     // their weights {w0, w1} (weighted reductions)
  int64_t n_tiny;       // rows in tpack
  int64_t n_tiny2;      // the first n_tiny2 of them have degree 2 (the rest <= 1)
  // two-table gathers (kgx_spmm_gemm_ex3): sources col >= n_x1 are rows of a
  // second table x2 (same ld_x); x2b = x2 - n_x1 * ld_x (host address math), so
  // the gather address is one select of the base.  n_x1 = INT32_MAX: one table.
  const float* x2b;
  int32_t n_x1;
  bool cu_split;  // KGX_FUSED_CU_SPLIT (host side only)
};

// Source row of column c: x[c], or with TWO x2[c - n_x1] (one 64-bit select per
// gathered row; a separate instantiation, so the one-table kernels keep their
// register budget).
template <bool TWO>
__device__ __forceinline__ const float* gsrc(const FusedArgs& a, int32_t c) {
  if constexpr (TWO) return (c >= a.n_x1 ? a.x2b : a.x) + row_off(c, a.ld_x);
  return a.x + row_off(c, a.ld_x);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops
// (lgkmcnt) but NOT for its outstanding global loads (vmcnt), unlike
// __syncthreads(), so gathers prefetched for the next tile stay in flight.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---- three-way bf16 split of f32 operands (the "bf16x3" product) ---------
// split3_a / split3_a_lo (kgx_bf16x3.h): x = hi + mid + lo; x*w is taken as the
// six significant bf16 x bf16 products (dropped terms <= 2^-24 |x w|), each
// exact in the MFMA's f32 accumulator, on v_mfma_f32_16x16x32_bf16 -- 16x the
// per-clock rate of the f32-input MFMA.  Infinite / NaN aggregates follow
// IEEE f32 products (non-finite aggregates go to the lo plane, kgx_bf16x3.h).
typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short bf16x4_t __attribute__((ext_vector_type(4)));

// W's split B-fragments for this lane's output column n_col: k-step s (0..3)
// of lane group q covers k = 32 q + 8 s + j (j = 0..7), so each A fragment is
// 8 contiguous elements of a tile row (one ds_read_b128); hi / mid / lo planes.
template <bool NARROW, typename Args>
__device__ __forceinline__ void load_w128(const Args& a, bool w_ok, int n_col, int q, bf16x8_t (&wfh)[4],
                                          bf16x8_t (&wfm)[4], bf16x8_t (&wfl)[4]) {
  auto wv = [&](int k) { return w_ok && (!NARROW || k < a.F_in) ? a.W[int64_t(k) * a.F_out + n_col] : 0.0f; };
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
    u32x4_t ph, pm, pl;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const float v0 = wv(32 * q + 8 * s + j), v1 = wv(32 * q + 8 * s + j + 1);
      uint32_t h, m_, l;
      split3_pair(v0, v1, h, m_, l);
      ph[j / 2] = h;
      pm[j / 2] = m_;
      pl[j / 2] = l;
    }
    wfh[s] = __builtin_bit_cast(bf16x8_t, ph);
    wfm[s] = __builtin_bit_cast(bf16x8_t, pm);
    wfl[s] = __builtin_bit_cast(bf16x8_t, pl);
  }
}

// One k-step of a 16-row block on one accumulator, D^T += W^T x^T: the six
// significant products of the split operands, small terms first (the tile's
// planes ah / am / al)
__device__ __forceinline__ f32x4 kstep_t(const bf16x8_t& wh, const bf16x8_t& wm, const bf16x8_t& wl,
                                         const bf16x8_t& ah, const bf16x8_t& am, const bf16x8_t& al, f32x4 d) {
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, al, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, ah, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm, am, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, am, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm, ah, d, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, ah, d, 0, 0, 0);
}

// The same products with the operands swapped, D += x W (the short-row
// kernel's f32 out tile): same order, the same bits transposed
__device__ __forceinline__ f32x4 kstep_n(const bf16x8_t& wh, const bf16x8_t& wm, const bf16x8_t& wl,
                                         const bf16x8_t& ah, const bf16x8_t& am, const bf16x8_t& al, f32x4 d) {
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, wh, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wl, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, wm, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, wh, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wm, d, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wh, d, 0, 0, 0);
}

// A tile row's split planes from this lane's four values: the fast split, or
// split3_a_lo (non-finite values to the lo plane) when the lane holds one.
__device__ __forceinline__ void split_row128(const float (&v)[4], bf16x4_t& ph, bf16x4_t& pm, bf16x4_t& pl) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    short h, m_, l;
    split3_a(v[k], h, m_, l);
    ph[k] = h;
    pm[k] = m_;
    pl[k] = l;
  }
  // inf / NaN in this lane's values (their sum is then non-finite): move them
  // to the lo plane (split3_a_lo) -- a rare branch instead of two selects per
  // value on every row
  if (!split_fast_ok(v[0], v[1], v[2], v[3])) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      short h, m_, l;
      split3_a_lo(v[k], h, m_, l);
      ph[k] = h;
      pm[k] = m_;
      pl[k] = l;
    }
  }
}

// A row gather that is never exec-masked: lanes whose edge is absent (u >= the
// row's degree, past-the-end items) read the zero row instead and the fold
// masks them; see kgx_zero_row (kgx_vec.h).
template <bool TWO>
__device__ __forceinline__ const float* gsrc_or_zero(const FusedArgs& a, bool present, int32_t c, int fg) {
  return present ? gsrc<TWO>(a, c) + fg : kgx_zero_row + fg;
}

template <int RED>
struct Red {
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

// NARROW: F_in < 128 or F_out not a multiple of 16 (masks compiled in only there)
template <int RED, bool WEIGHTED, bool TWO, bool NARROW>
__global__ __launch_bounds__(kThreads, TWO ? 4 : 1) void spmm_gemm_kernel(FusedArgs a) {  // TWO: hold 4 waves per SIMD
  using R = Red<RED>;
  // gathers in flight per group: at F_in 128 (GCN, NS) 4 beat 6 and 8 with PF = U
  // (each cost occupancy) and U = 8 with PF = 2 (NS 8.90 -> 9.05-9.15 ms); the
  // narrow unweighted form (SAGE at C5: 50 edges per row on average) takes 6 in
  // 124 VGPRs, occupancy kept (C5 main kernel 7.70 ms at U = 4, 7.37-7.48 at
  // U = 6, 7.77 at U = 8 with PF = 2)
  constexpr int U = (NARROW && !WEIGHTED) ? 6 : 4;
  constexpr int PF = 4;  // rows prefetched per group for the next tile (live across the MFMA phase)
  __shared__ __attribute__((aligned(16))) short tile3[kFPlanes][kGroups][kFin + 8];  // split planes of the aggregated rows
  __shared__ __attribute__((aligned(16))) float sbias[kFin];  // read at the stores (4 VGPRs fewer than a register copy)
  __shared__ int32_t tile_row[kGroups];

  const int tid = threadIdx.x;
  const int g = tid >> 5;     // row-group 0..15
  const int lane = tid & 31;  // lane in the group
  const int f = lane * 4;
  const bool f_ok = !NARROW || f < a.F_in;  // lanes past F_in (F_in < 128) load column 0 again and carry zeros
  const int fg = f_ok ? f : 0;
  const int wave = tid >> 6;  // 0..7 -> output columns [16 wave, 16 wave + 16)
  const int wl = tid & 63;    // lane in the wave
  const int n_col = wave * 16 + (wl & 15);
  const int q = wl >> 4;
  const bool mfma_wave = wave * 16 < a.F_out;
  const bool w_ok = mfma_wave && (!NARROW || n_col < a.F_out);  // W rows k >= F_in and columns >= F_out load as 0

  // W fragment for this wave's 16 columns, K permuted: k = 32 q + s.
  bf16x8_t wfh[4], wfm[4], wfl[4];
  load_w128<NARROW>(a, w_ok, n_col, q, wfh, wfm, wfl);
  const int c4 = wave * 16 + 4 * q;
  if (tid < kFin) sbias[tid] = (a.bias && tid < a.F_out) ? a.bias[tid] : 0.0f;  // first read after the tile barrier

  const int64_t n_work = a.items ? a.n_long : a.n_rows;
  const int64_t stride = int64_t(gridDim.x) * kGroups;

  // software pipeline: the next item's descriptor and its first PF neighbour rows
  // are loaded before the MFMA phase of the current tile, so the gathers are in
  // flight while the matrix pipe works.
  int32_t row = -1, beg = 0, end = 0, slot = -1;
  int pn = 0;
  float pv[PF][4], pw[PF];
  auto fetch = [&](int64_t it) {
    // the descriptor from a clamped slot (n_work >= 1 in a launched kernel),
    // never under an exec mask; past-the-end groups get an empty item
    const bool live = it < n_work;
    const int64_t itc = live ? it : n_work - 1;
    if (a.items) {
      const int4 v = a.items[itc];
      row = live ? v.x : -1;
      beg = live ? v.y : 0;
      end = live ? v.z : 0;
      slot = live ? v.w : -1;
    } else {
      const int32_t rw = a.rows[itc];
      const int32_t b0 = a.rowptr[rw], b1 = a.rowptr[rw + 1];
      row = live ? rw : -1;
      beg = live ? b0 : 0;
      end = live ? b1 : 0;
      slot = -1;
    }
    pn = (end - beg) < PF ? (end - beg) : PF;
    // unconditional loads: index / weight from clamped slots (idx / w hold >= 1
    // element), rows past the item's edges from the zero row; masking happens
    // when the values are folded in, never around a load
    int32_t c[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int32_t ee = pn > 0 ? beg + (u < pn ? u : pn - 1) : 0;
      c[u] = a.idx[ee];
      if constexpr (WEIGHTED) pw[u] = a.w[ee];
    }
#pragma unroll
    for (int u = 0; u < PF; ++u) vload<4>(pv[u], gsrc_or_zero<TWO>(a, u < pn, c[u], fg));
  };

  fetch(int64_t(blockIdx.x) * kGroups + g);
  for (int64_t base = int64_t(blockIdx.x) * kGroups; base < n_work; base += stride) {
    float acc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = R::init();
#pragma unroll
    for (int u = 0; u < PF; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float m = WEIGHTED ? __fmul_rn(pv[u][k], pw[u]) : pv[u][k];
        acc[k] = R::combine(acc[k], u < pn ? R::msg(m) : R::init());
      }
    auto block = [&](auto UB, int32_t e) {
      constexpr int B = decltype(UB)::value;
      const int n = end - e;
      int32_t c[B];
      float wt[B];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int32_t ee = u < n ? e + u : end - 1;
        c[u] = a.idx[ee];
        if constexpr (WEIGHTED) wt[u] = a.w[ee];
      }
      float v[B][4];
#pragma unroll
      for (int u = 0; u < B; ++u) vload<4>(v[u], gsrc<TWO>(a, c[u]) + fg);
#pragma unroll
      for (int u = 0; u < B; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float m = WEIGHTED ? __fmul_rn(v[u][k], wt[u]) : v[u][k];
          acc[k] = R::combine(acc[k], u < n ? R::msg(m) : R::init());
        }
    };
    int32_t e = beg + PF;
    // full blocks, then half-width tail blocks (at most U/2 - 1 clamped redundant loads)
    for (; e + U <= end; e += U) block(std::integral_constant<int, U>{}, e);
    for (; e < end; e += U / 2) block(std::integral_constant<int, U / 2>{}, e);
    const bool full_row = row >= 0 && slot < 0;
    if (row >= 0 && slot >= 0) vstore<4>(a.partials + int64_t(slot) * kFin + f, acc);
    float r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = full_row ? R::finish(acc[k], end - beg) : 0.0f;
    if (full_row && a.pre_gin) {
      float xv[4];
      vload<4>(xv, a.x + int64_t(row) * a.ld_x + fg);
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = __fadd_rn(__fmul_rn(a.gin_scale, xv[k]), r[k]);
    }
    if (full_row && a.agg_out && f_ok) vstore<4>(a.agg_out + int64_t(row) * a.ld_agg + f, r);
    if (NARROW && a.F_in < kFin) {  // wave-uniform: lanes past F_in put zeros in the planes
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = f_ok ? r[k] : 0.0f;
    }
    {
      bf16x4_t ph, pm, pl;
      split_row128(r, ph, pm, pl);
      *reinterpret_cast<bf16x4_t*>(&tile3[0][g][f]) = ph;
      *reinterpret_cast<bf16x4_t*>(&tile3[1][g][f]) = pm;
      *reinterpret_cast<bf16x4_t*>(&tile3[2][g][f]) = pl;
    }
    if (lane == 0) tile_row[g] = full_row ? row : -1;
    lds_barrier();

    fetch(base + stride + g);  // next tile's first gathers fly during the MFMAs

    if (mfma_wave) {
      const int m = wl & 15;
      f32x4 d0 = {0.0f, 0.0f, 0.0f, 0.0f};
      f32x4 d1 = {0.0f, 0.0f, 0.0f, 0.0f};  // two accumulation chains
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const bf16x8_t ah = *reinterpret_cast<const bf16x8_t*>(&tile3[0][m][32 * q + 8 * s4]);
        const bf16x8_t am = *reinterpret_cast<const bf16x8_t*>(&tile3[1][m][32 * q + 8 * s4]);
        const bf16x8_t al = *reinterpret_cast<const bf16x8_t*>(&tile3[2][m][32 * q + 8 * s4]);
        // D^T = W^T x^T, small terms first
        d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfh[s4], al, d1, 0, 0, 0);
        d0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfl[s4], ah, d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfm[s4], am, d1, 0, 0, 0);
        d0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfh[s4], am, d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfm[s4], ah, d1, 0, 0, 0);
        d0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfh[s4], ah, d0, 0, 0, 0);
      }
      // straight from the accumulators: lane (m, q) writes columns 16 wave + 4 q .. + 3 of tile row m
      const int rr = tile_row[m];
      if (rr >= 0 && (!NARROW || c4 < a.F_out)) {
        float4* dst = reinterpret_cast<float4*>(a.out + int64_t(rr) * a.ld_o + c4);
        const float4 b4 = *reinterpret_cast<const float4*>(&sbias[c4]);
        float4 v = make_float4((d0[0] + d1[0]) + b4.x, (d0[1] + d1[1]) + b4.y, (d0[2] + d1[2]) + b4.z,
                               (d0[3] + d1[3]) + b4.w);
        if (a.accumulate) {
          const float4 p = *dst;
          v = make_float4(__fadd_rn(p.x, v.x), __fadd_rn(p.y, v.y), __fadd_rn(p.z, v.z), __fadd_rn(p.w, v.w));
        }
        if (a.relu) v = make_float4(fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f), fmaxf(v.z, 0.0f), fmaxf(v.w, 0.0f));
        *dst = v;
      }
    }
    lds_barrier();  // every wave is done with the planes and tile_row before the next tile's are written
  }
}

// Rows of degree <= KGX_SHORT_ROW_MAX (the schedule's suffix; 78 % of an R-MAT graph's
// rows, 11 % of its edges).  spmm_gemm_kernel gives each row-group ONE row per
// 16-row tile, so on these rows a group has one or two gathers in flight and
// the tile's fixed chain (item, index, row, split, MFMA, store) dominates:
// NS rows of degree <= 7 ran at 3.4 TB/s against 7.7 TB/s for the rest
// (tools/exp_lowdeg.py).  Here a block iteration takes 32 rows, 2 per group,
// whose first three edges are all gathered together, and the MFMA phase runs
// two 16-row blocks per wave; the results go through an f32 LDS out tile and
// are stored as whole rows (measured 0.98 against 0.99 ms for stores straight
// from the accumulators).
static_assert(KGX_SHORT_ROW_MAX == 7, "the short kernel gathers three edges per row up front, then pairs");
constexpr int kRPG = 2;        // rows per group per tile
constexpr int kSPF = 3;         // edges per row gathered up front (all rows together)
constexpr int kShortRows = kGroups * kRPG;

template <int RED, bool WEIGHTED, bool TWO, bool NARROW>
__global__ __launch_bounds__(kThreads, 4) void spmm_gemm_short_kernel(FusedArgs a) {  // 4 waves per SIMD: two blocks per CU
  using R = Red<RED>;
  // split planes of the 32 aggregated rows; after the MFMAs the same bytes hold the f32 results
  __shared__ __attribute__((aligned(16))) short tile3[kFPlanes][kShortRows][kFin + 8];
  __shared__ int32_t tile_row[kShortRows];
  static_assert(sizeof(tile3) >= sizeof(float) * kShortRows * kTileLd, "output tile must fit the plane buffer");
  float(*otile)[kTileLd] = reinterpret_cast<float(*)[kTileLd]>(&tile3[0][0][0]);

  const int tid = threadIdx.x;
  const int g = tid >> 5;
  const int lane = tid & 31;
  const int f = lane * 4;
  const bool f_ok = !NARROW || f < a.F_in;  // lanes past F_in (F_in < 128) load column 0 again and carry zeros
  const int fg = f_ok ? f : 0;
  const int wave = tid >> 6;
  const int wl = tid & 63;
  const int n_col = wave * 16 + (wl & 15);
  const int q = wl >> 4;
  const bool mfma_wave = wave * 16 < a.F_out;
  const bool w_ok = mfma_wave && (!NARROW || n_col < a.F_out);  // W rows k >= F_in and columns >= F_out load as 0

  bf16x8_t wfh[4], wfm[4], wfl[4];
  load_w128<NARROW>(a, w_ok, n_col, q, wfh, wfm, wfl);
  const float bcol = (mfma_wave && a.bias) ? a.bias[n_col] : 0.0f;

  for (int64_t base = a.n_long + int64_t(blockIdx.x) * kShortRows; base < a.n_short_end;
       base += int64_t(gridDim.x) * kShortRows) {
    int32_t row[kRPG], beg[kRPG], deg[kRPG];
#pragma unroll
    for (int r = 0; r < kRPG; ++r) {
      const int64_t it = base + g + kGroups * r;
      row[r] = -1;
      beg[r] = 0;
      deg[r] = 0;
      if (it < a.n_short_end) {
        const int4 v = a.items[it];
        row[r] = v.x;
        beg[r] = v.y;
        deg[r] = v.z - v.y;
      }
    }
    // the first kSPF edges of all the group's rows in flight together
    // (unconditional loads: indices from clamped slots, absent edges' rows
    // from the zero row; masked at the fold)
    float acc[kRPG][4];
    {
      int32_t c[kRPG][kSPF];
      float wt[kRPG][kSPF];
#pragma unroll
      for (int r = 0; r < kRPG; ++r)
#pragma unroll
        for (int u = 0; u < kSPF; ++u) {
          const int32_t ee = deg[r] > 0 ? beg[r] + (u < deg[r] ? u : deg[r] - 1) : 0;
          c[r][u] = a.idx[ee];
          if constexpr (WEIGHTED) wt[r][u] = a.w[ee];
        }
      float v[kRPG][kSPF][4];
#pragma unroll
      for (int r = 0; r < kRPG; ++r)
#pragma unroll
        for (int u = 0; u < kSPF; ++u) vload<4>(v[r][u], gsrc_or_zero<TWO>(a, u < deg[r], c[r][u], fg));
#pragma unroll
      for (int r = 0; r < kRPG; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float t = R::init();
#pragma unroll
          for (int u = 0; u < kSPF; ++u) {
            const float m = WEIGHTED ? __fmul_rn(v[r][u][k], wt[r][u]) : v[r][u][k];
            t = R::combine(t, u < deg[r] ? R::msg(m) : R::init());
          }
          acc[r][k] = t;
        }
    }
    // edges kSPF .. deg-1, two at a time, in order
#pragma unroll
    for (int r = 0; r < kRPG; ++r) {
      for (int32_t e = kSPF; e < deg[r]; e += 2) {
        const int n = deg[r] - e;
        int32_t c[2];
        float wt[2], v[2][4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int32_t ee = beg[r] + e + (u < n ? u : n - 1);
          c[u] = a.idx[ee];
          if constexpr (WEIGHTED) wt[u] = a.w[ee];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) vload<4>(v[u], gsrc<TWO>(a, c[u]) + fg);
        // both loads stay unconditional: unweighted, hipcc otherwise sinks the
        // second (masked at the fold when n == 1) into an exec-masked branch
        asm volatile("" ::"v"(v[1][0]), "v"(v[1][1]), "v"(v[1][2]), "v"(v[1][3]));
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float m = WEIGHTED ? __fmul_rn(v[u][k], wt[u]) : v[u][k];
            acc[r][k] = R::combine(acc[r][k], u < n ? R::msg(m) : R::init());
          }
      }
    }
    lds_barrier();  // the previous tile's output rows (same LDS bytes) have been stored
#pragma unroll
    for (int r = 0; r < kRPG; ++r) {
      const bool ok = row[r] >= 0;
      float v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = ok ? R::finish(acc[r][k], deg[r]) : 0.0f;
      if (ok && a.pre_gin) {
        float xv[4];
        vload<4>(xv, a.x + int64_t(row[r]) * a.ld_x + fg);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __fadd_rn(__fmul_rn(a.gin_scale, xv[k]), v[k]);
      }
      if (ok && a.agg_out && f_ok) vstore<4>(a.agg_out + int64_t(row[r]) * a.ld_agg + f, v);
      if (NARROW && a.F_in < kFin) {  // wave-uniform: lanes past F_in put zeros in the planes
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = f_ok ? v[k] : 0.0f;
      }
      bf16x4_t ph, pm, pl;
      split_row128(v, ph, pm, pl);
      const int tr = g + kGroups * r;
      *reinterpret_cast<bf16x4_t*>(&tile3[0][tr][f]) = ph;
      *reinterpret_cast<bf16x4_t*>(&tile3[1][tr][f]) = pm;
      *reinterpret_cast<bf16x4_t*>(&tile3[2][tr][f]) = pl;
      if (lane == 0) tile_row[tr] = row[r];
    }
    lds_barrier();
    f32x4 d[kRPG];
    if (mfma_wave) {
      const int m = wl & 15;
#pragma unroll
      for (int rb = 0; rb < kRPG; ++rb) d[rb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
#pragma unroll
        for (int rb = 0; rb < kRPG; ++rb) {
          const int tr = 16 * rb + m;
          const bf16x8_t ah = *reinterpret_cast<const bf16x8_t*>(&tile3[0][tr][32 * q + 8 * s4]);
          const bf16x8_t am = *reinterpret_cast<const bf16x8_t*>(&tile3[1][tr][32 * q + 8 * s4]);
          const bf16x8_t al = *reinterpret_cast<const bf16x8_t*>(&tile3[2][tr][32 * q + 8 * s4]);
          d[rb] = kstep_n(wfh[s4], wfm[s4], wfl[s4], ah, am, al, d[rb]);
        }
      }
    }
    lds_barrier();  // every wave has read the planes: their bytes now take the f32 results
    if (mfma_wave) {
#pragma unroll
      for (int rb = 0; rb < kRPG; ++rb)
#pragma unroll
        for (int j = 0; j < 4; ++j) otile[16 * rb + 4 * q + j][n_col] = d[rb][j] + bcol;
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < kRPG; ++r) {
      const int tr = g + kGroups * r;
      const int rr = tile_row[tr];
      if (rr >= 0 && f < a.F_out) {
        float4* dst = reinterpret_cast<float4*>(a.out + int64_t(rr) * a.ld_o + f);
        float4 v = *reinterpret_cast<const float4*>(&otile[tr][f]);
        if (a.accumulate) {
          const float4 p = *dst;
          v = make_float4(__fadd_rn(p.x, v.x), __fadd_rn(p.y, v.y), __fadd_rn(p.z, v.z), __fadd_rn(p.w, v.w));
        }
        if (a.relu) v = make_float4(fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f), fmaxf(v.z, 0.0f), fmaxf(v.w, 0.0f));
        *dst = v;
      }
    }
  }
}

// Rows of degree <= 2 (an R-MAT graph's self-loop-only rows are half of all
// rows), warp-specialised.  spmm_gemm_short_kernel's waves each gather, split,
// run the MFMAs and store in turn, and its waves sit in s_waitcnt / barriers
// 71 % of their cycles: the MFMA phase and the stores add to the gathers
// instead of hiding behind them, and W's 48 fragment registers per lane leave
// no room to prefetch.  Here, in a 1024-thread block:
//  - producer waves 8..15 (16 groups of 32 lanes, 2 rows each per 32-row tile)
//    read a packed record per row {row, degree, col0, col1} (+ {w0, w1}),
//    gather both source rows unconditionally (col1 = col0 for degree 1;
//    absent edges fold in the reduction's identity), split the aggregated
//    rows into the bf16 planes of one of two LDS tiles.  Their loads run two
//    tiles ahead: while tile t is folded, tile t+1's rows and tile t+2's
//    records are in flight (all loads unconditional, so hipcc's vmcnt counts
//    stay exact and it never drains the queue);
//  - MFMA waves 0..7 hold W's split fragments (16 output columns each), take
//    the other tile and store their results straight from the accumulators.
// One barrier per tile hands a tile from producers to MFMA waves.
constexpr int kTinyThreads = 1024;
constexpr int kTinyGroups = 16;  // producer row groups
// rows per group per tile (= 16-row MFMA blocks per tile): two-edge rows / one-edge rows
constexpr int kTinyRPG2 = 2;  // two-edge rows
constexpr int kTinyRPG1 = 4;  // one-edge rows
template <int NG>
constexpr int tiny_rows() { return kTinyGroups * (NG == 1 ? kTinyRPG1 : kTinyRPG2); }

// NG: edges gathered per row (2 for the degree-2 head of the tail, 1 for the
// degree <= 1 rest: the schedule is degree-descending, so each is a range).
template <int RED, bool WEIGHTED, bool EXTRA, int NG, bool TWO, bool NARROW>  // EXTRA: pre_gin or agg_out (loads / stores under a row mask)
__global__ __launch_bounds__(kTinyThreads, 1) void spmm_gemm_tiny_kernel(FusedArgs a) {
  using R = Red<RED>;
  constexpr int kTinyRPG = NG == 1 ? kTinyRPG1 : kTinyRPG2;  // rows per group per tile
  constexpr int kTinyRows = kTinyGroups * kTinyRPG;
  __shared__ __attribute__((aligned(16))) short planes[2][kFPlanes][kTinyRows][kFin + 8];
  __shared__ int32_t trow[2][kTinyRows];
  __shared__ __attribute__((aligned(16))) float sbias[kFin];  // read at the stores
  if (threadIdx.x < kFin)  // first read after a hand-off barrier
    sbias[threadIdx.x] = (a.bias && int(threadIdx.x) < a.F_out) ? a.bias[threadIdx.x] : 0.0f;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t n_tiles = (a.n_tiny + kTinyRows - 1) / kTinyRows;
  const int64_t my_tiles = int64_t(blockIdx.x) < n_tiles ? (n_tiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;

  if (wave < 8) {  // ---- MFMA waves: tile i-1 at iteration i
    const int wl = tid & 63;
    const int q = wl >> 4, m = wl & 15;
    const int n_col = wave * 16 + m;
    const bool mfma_wave = wave * 16 < a.F_out;
    const bool w_ok = mfma_wave && (!NARROW || n_col < a.F_out);
    bf16x8_t wfh[4], wfm[4], wfl[4];
    load_w128<NARROW>(a, w_ok, n_col, q, wfh, wfm, wfl);
    const int c4 = wave * 16 + 4 * q;
    for (int64_t i = 0; i <= my_tiles; ++i) {
      if (i >= 1 && mfma_wave) {
        const int b = int((i - 1) & 1);
        f32x4 d[kTinyRPG];
#pragma unroll
        for (int rb = 0; rb < kTinyRPG; ++rb) d[rb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
#pragma unroll
          for (int rb = 0; rb < kTinyRPG; ++rb) {
            const int tr = 16 * rb + m;
            const bf16x8_t ah = *reinterpret_cast<const bf16x8_t*>(&planes[b][0][tr][32 * q + 8 * s4]);
            const bf16x8_t am = *reinterpret_cast<const bf16x8_t*>(&planes[b][1][tr][32 * q + 8 * s4]);
            const bf16x8_t al = *reinterpret_cast<const bf16x8_t*>(&planes[b][2][tr][32 * q + 8 * s4]);
            // D^T = W^T x^T: same products, same k order as the short-row kernel
            d[rb] = kstep_t(wfh[s4], wfm[s4], wfl[s4], ah, am, al, d[rb]);
          }
        }
        // lane (m, q) holds columns 16 wave + 4 q .. + 3 of tile row 16 rb + m: one
        // dwordx4 per lane, four store instructions per tile
#pragma unroll
        for (int rb = 0; rb < kTinyRPG; ++rb) {
          const int rr = trow[b][16 * rb + m];
          if (rr >= 0 && (!NARROW || c4 < a.F_out)) {
            float4* dst = reinterpret_cast<float4*>(a.out + int64_t(rr) * a.ld_o + c4);
            const float4 b4 = *reinterpret_cast<const float4*>(&sbias[c4]);
            float4 v = make_float4(d[rb][0] + b4.x, d[rb][1] + b4.y, d[rb][2] + b4.z, d[rb][3] + b4.w);
            if (a.accumulate) {
              const float4 p = *dst;
              v = make_float4(__fadd_rn(p.x, v.x), __fadd_rn(p.y, v.y), __fadd_rn(p.z, v.z), __fadd_rn(p.w, v.w));
            }
            if (a.relu) v = make_float4(fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f), fmaxf(v.z, 0.0f), fmaxf(v.w, 0.0f));
            *dst = v;
          }
        }
      }
      lds_barrier();
    }
    return;
  }

  // ---- producers: tile i at iteration i
  const int pt = tid - 512;
  const int g = pt >> 5, lane = pt & 31, f = lane * 4;
  const bool f_ok = !NARROW || f < a.F_in;  // lanes past F_in (F_in < 128) load column 0 again and carry zeros
  const int fg = f_ok ? f : 0;
  struct Rec {
    int4 p[kTinyRPG];
    float2 w[kTinyRPG];
  };
  auto rec = [&](int64_t k, Rec& r) {  // tile k's records (clamped; rows past the end get row -1)
#pragma unroll
    for (int j = 0; j < kTinyRPG; ++j) {
      const int64_t t = int64_t(blockIdx.x) + k * gridDim.x;
      const int64_t e = t * kTinyRows + g + kTinyGroups * j;
      const int64_t ec = e < a.n_tiny ? e : a.n_tiny - 1;
      r.p[j] = a.tpack[ec];
      if (e >= a.n_tiny) r.p[j].x = -1;
      if constexpr (WEIGHTED) r.w[j] = a.tw[ec];
    }
  };
  typedef float f4 __attribute__((ext_vector_type(4)));
  auto gather = [&](const Rec& r, f4 (&v)[kTinyRPG][NG]) {
#pragma unroll
    for (int j = 0; j < kTinyRPG; ++j) {
      v[j][0] = *reinterpret_cast<const f4*>(gsrc<TWO>(a, r.p[j].z) + fg);
      if constexpr (NG == 2) v[j][1] = *reinterpret_cast<const f4*>(gsrc<TWO>(a, r.p[j].w) + fg);
    }
  };
  auto produce = [&](int64_t i, const auto& c, const f4 (&v)[kTinyRPG][NG]) {
    const int b = int(i & 1);
#pragma unroll
    for (int j = 0; j < kTinyRPG; ++j) {
      const int32_t row = c.row[j], deg = c.deg[j];
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float t = R::init();
        const float m0 = WEIGHTED ? __fmul_rn(v[j][0][k], c.w[j].x) : v[j][0][k];
        t = R::combine(t, deg > 0 ? R::msg(m0) : R::init());
        if constexpr (NG == 2) {
          const float m1 = WEIGHTED ? __fmul_rn(v[j][1][k], c.w[j].y) : v[j][1][k];
          t = R::combine(t, deg > 1 ? R::msg(m1) : R::init());
        }
        o[k] = row >= 0 ? R::finish(t, deg) : 0.0f;
      }
      if constexpr (EXTRA) {
        if (row >= 0 && a.pre_gin) {
          float xv[4];
          vload<4>(xv, a.x + int64_t(row) * a.ld_x + fg);
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] = __fadd_rn(__fmul_rn(a.gin_scale, xv[k]), o[k]);
        }
        if (row >= 0 && a.agg_out && f_ok) vstore<4>(a.agg_out + int64_t(row) * a.ld_agg + f, o);
      }
      if (NARROW && a.F_in < kFin) {  // wave-uniform: lanes past F_in put zeros in the planes
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = f_ok ? o[k] : 0.0f;
      }
      bf16x4_t ph, pm, pl;
      split_row128(o, ph, pm, pl);
      const int tr = g + kTinyGroups * j;
      *reinterpret_cast<bf16x4_t*>(&planes[b][0][tr][f]) = ph;
      *reinterpret_cast<bf16x4_t*>(&planes[b][1][tr][f]) = pm;
      *reinterpret_cast<bf16x4_t*>(&planes[b][2][tr][f]) = pl;
      if (lane == 0) trow[b][tr] = row;
    }
  };
  // Pipeline, at iteration i: issue tile i+2's records, issue tile i+1's row
  // gathers (its records arrived a step ago), fold tile i (rows in flight
  // since i-1).  Every load is unconditional, so when a value is used the
  // loads issued after it are a known count and hipcc's vmcnt wait leaves
  // them in flight.  Unrolled by two so register sets rotate by name.
  struct Cur {
    int32_t row[kTinyRPG], deg[kTinyRPG];
    float2 w[kTinyRPG];
  };
  auto take = [&](const Rec& r, Cur& c) {
#pragma unroll
    for (int j = 0; j < kTinyRPG; ++j) {
      c.row[j] = r.p[j].x;
      c.deg[j] = r.p[j].y;
      c.w[j] = WEIGHTED ? r.w[j] : float2{1.0f, 1.0f};
    }
  };
  Rec ra, rb;
  Cur cur;
  f4 v0[kTinyRPG][NG], v1[kTinyRPG][NG];
  rec(0, rb);
  take(rb, cur);
  rec(1, ra);
  gather(rb, v0);
  auto step = [&](int64_t i, Rec& rn, Rec& rfree, f4 (&vc)[kTinyRPG][NG], f4 (&vn)[kTinyRPG][NG]) {
    rec(i + 2, rfree);  // tile i+2's records
    gather(rn, vn);     // tile i+1's rows
    produce(i, cur, vc);
    take(rn, cur);
    lds_barrier();
  };
  for (int64_t i = 0; i <= my_tiles; i += 2) {
    step(i, ra, rb, v0, v1);
    if (i + 1 > my_tiles) break;
    step(i + 1, rb, ra, v1, v0);
  }
}

// Split rows: combine chunk partials in order, finish, then out = v @ W + b (VALU).
template <int RED, bool NARROW>
__global__ __launch_bounds__(256) void spmm_gemm_fixup_kernel(FusedArgs a) {
  using R = Red<RED>;
  __shared__ float vrow[8][kFin];
  const int g = threadIdx.x >> 5, lane = threadIdx.x & 31;
  for (int64_t base = int64_t(blockIdx.x) * 8; base < a.n_split; base += int64_t(gridDim.x) * 8) {
    const int64_t it = base + g;
    int32_t row = -1;
    if (it < a.n_split) {
      const int4 s = a.split[it];
      row = s.x;
      float acc[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = R::init();
      constexpr int B = 8;  // chunk loads in flight, then the in-order combine
      for (int32_t c0 = 0; c0 < s.z; c0 += B) {
        float p[B][4];
#pragma unroll
        for (int u = 0; u < B; ++u) vload<4>(p[u], a.partials + int64_t(s.y + (c0 + u < s.z ? c0 + u : s.z - 1)) * kFin + lane * 4);
#pragma unroll
        for (int u = 0; u < B; ++u)
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[k] = c0 + u < s.z ? R::combine(acc[k], p[u][k]) : acc[k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = R::finish(acc[k], s.w);
      if (a.pre_gin) {
        float xv[4];
        vload<4>(xv, a.x + int64_t(row) * a.ld_x + (!NARROW || lane * 4 < a.F_in ? lane * 4 : 0));
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] = __fadd_rn(__fmul_rn(a.gin_scale, xv[k]), acc[k]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) vrow[g][lane * 4 + k] = acc[k];
      if (a.agg_out && (!NARROW || lane * 4 < a.F_in)) vstore<4>(a.agg_out + int64_t(row) * a.ld_agg + lane * 4, acc);
    }
    __syncthreads();
    if (row >= 0) {
      for (int c = lane; c < a.F_out; c += 32) {
        float s = 0.0f;
        for (int k = 0; k < (NARROW ? a.F_in : kFin); ++k) s = fmaf(vrow[g][k], a.W[int64_t(k) * a.F_out + c], s);
        float v = s + (a.bias ? a.bias[c] : 0.0f);
        if (a.accumulate) v = __fadd_rn(a.out[int64_t(row) * a.ld_o + c], v);
        if (a.relu) v = fmaxf(v, 0.0f);
        a.out[int64_t(row) * a.ld_o + c] = v;
      }
    }
    __syncthreads();
  }
}

// The CU split (KGX_FUSED_CU_SPLIT flag, or KGX_FUSED_FORK=3 read per launch for
// measurement): the main kernel and the short + tiny launches on disjoint CU
// sets (24 / 8 of every 32 CUs, CU-masked streams, kgx_internal.h cu_split).
// Disjoint output rows; the tail launches' MFMA phases overlap the main
// kernel's gathers instead of starting after it; joined before the hub
// fix-up.  Measured and removed (tools/experiments/round5_fork_modes.patch):
// the tails forked onto an unmasked side stream (tiny only: NS 9.51-9.66 ms;
// short + tiny: 8.89-8.94), and the main kernel capped to (den - 1) / den of
// its grid with the tails in the slots left on every CU (8.82-8.86 at den 8;
// 10.1-10.2 at den 2), against 8.63-8.67 split and 8.87-8.94 one-stream.
inline int fused_fork_mode() {  // read per launch (tests switch it in-process)
  const char* h = getenv("KGX_FUSED_FORK");
  return h ? atoi(h) : 0;
}

template <int RED, bool W, bool TWO, bool NARROW>
int launch_short(const FusedArgs& a, hipStream_t s, int cus = 0) {
  int per_cu = 0;
  auto k = spmm_gemm_short_kernel<RED, W, TWO, NARROW>;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kThreads, 0) != hipSuccess || per_cu <= 0) per_cu = 2;
  const int64_t need = (a.n_short_end - a.n_long + kShortRows - 1) / kShortRows;
  const int64_t full = int64_t(per_cu) * (cus > 0 ? cus : cu_count());
  const int64_t cap = a.share_gpu ? shared_cap(full) : full;
  hipLaunchKernelGGL(k, dim3(unsigned(need < cap ? need : cap)), dim3(kThreads), 0, s, a);
  KGX_CHECK_LAUNCH();
  return KGX_OK;
}

template <int RED, bool W, bool TWO, bool NARROW>
int launch_tiny(const FusedArgs& a, hipStream_t s, int cus = 0) {
  const bool extra = a.pre_gin || a.agg_out;
  for (int part = 0; part < 2; ++part) {  // one 1024-thread block per CU; degree-2 head, then the degree <= 1 rest
    FusedArgs b = a;
    b.tpack = a.tpack + (part ? a.n_tiny2 : 0);
    b.tw = a.tw ? a.tw + (part ? a.n_tiny2 : 0) : nullptr;
    b.n_tiny = part ? a.n_tiny - a.n_tiny2 : a.n_tiny2;
    if (b.n_tiny <= 0) continue;
    auto k = part ? (extra ? spmm_gemm_tiny_kernel<RED, W, true, 1, TWO, NARROW>
                           : spmm_gemm_tiny_kernel<RED, W, false, 1, TWO, NARROW>)
                  : (extra ? spmm_gemm_tiny_kernel<RED, W, true, 2, TWO, NARROW>
                           : spmm_gemm_tiny_kernel<RED, W, false, 2, TWO, NARROW>);
    const int rows = part ? tiny_rows<1>() : tiny_rows<2>();
    const int64_t need = (b.n_tiny + rows - 1) / rows;
    const int64_t full = cus > 0 ? cus : cu_count();
    const int64_t cap = a.share_gpu ? shared_cap(full) : full;
    hipLaunchKernelGGL(k, dim3(unsigned(need < cap ? need : cap)), dim3(kTinyThreads), 0, s, b);
    KGX_CHECK_LAUNCH();
  }
  return KGX_OK;
}

template <int RED, bool W, bool TWO = false, bool NARROW = false>
int launch(const FusedArgs& a, hipStream_t s) {
  const int64_t work = a.items ? a.n_long : a.n_rows;
  const bool has_short = a.items && a.n_long < a.n_short_end;
  const bool split = a.cu_split || fused_fork_mode() == 3;
  if (split && work > 0 && ((a.tpack && a.n_tiny > 0) || has_short)) {
    // the main kernel on a CU-masked stream over 24 of every 32 CUs, the
    // short-row and tiny-row launches on another over the other 8 (cu_split)
    const char* e = getenv("KGX_FUSED_CU_SPLIT");  // tail CUs per 32 (default 8)
    CuSplit* cs = cu_split(e ? atoi(e) : 8, s);
    if (cs) {
      SplitJoin join;
      KGX_CHECK_HIP(hipEventRecord(cs->fork, s));
      KGX_CHECK_HIP(hipStreamWaitEvent(cs->head, cs->fork, 0));
      KGX_CHECK_HIP(hipStreamWaitEvent(cs->tail, cs->fork, 0));
      join.cs = cs;
      join.s = s;
      int per_cu = 0;
      auto k = spmm_gemm_kernel<RED, W, TWO, NARROW>;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kThreads, 0) != hipSuccess || per_cu <= 0)
        per_cu = 2;
      const int64_t need = (work + kGroups - 1) / kGroups;
      const int64_t full = int64_t(per_cu) * cs->n_head;
      const int64_t cap = a.share_gpu ? shared_cap(full) : full;
      hipLaunchKernelGGL(k, dim3(unsigned(need < cap ? need : cap)), dim3(kThreads), 0, cs->head, a);
      KGX_CHECK_LAUNCH();
      if (a.items && a.n_split > 0) {
        // the hub fix-up reads only the main kernel's partials and writes only split rows:
        // on the head's CUs right after it, hidden behind the longer tail leg
        const int64_t blocks = (a.n_split + 7) / 8;
        auto fk = spmm_gemm_fixup_kernel<RED, NARROW>;
        hipLaunchKernelGGL(fk, dim3(unsigned(blocks < 4096 ? blocks : 4096)), dim3(256), 0, cs->head, a);
        KGX_CHECK_LAUNCH();
      }
      if (has_short && launch_short<RED, W, TWO, NARROW>(a, cs->tail, cs->n_tail) != KGX_OK) return KGX_ERR_HIP;
      if (a.tpack && a.n_tiny > 0 && launch_tiny<RED, W, TWO, NARROW>(a, cs->tail, cs->n_tail) != KGX_OK)
        return KGX_ERR_HIP;
      join.cs = nullptr;
      KGX_CHECK_HIP(hipEventRecord(cs->jh, cs->head));
      KGX_CHECK_HIP(hipEventRecord(cs->jt, cs->tail));
      KGX_CHECK_HIP(hipStreamWaitEvent(s, cs->jh, 0));
      KGX_CHECK_HIP(hipStreamWaitEvent(s, cs->jt, 0));
      return KGX_OK;
    }
  }
  if (work > 0) {
    static int cus = 0;
    if (cus == 0) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    }
    int per_cu = 0;
    auto k = spmm_gemm_kernel<RED, W, TWO, NARROW>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kThreads, 0) != hipSuccess || per_cu <= 0)
      per_cu = 2;
    const int64_t need = (work + kGroups - 1) / kGroups;
    // KGX_FUSED_SHARE_GPU: leave 1/den of the block slots free (share_den(),
    // default a sixteenth) so a concurrent collective's kernels (RCCL halo
    // all-to-all) and the side stream's packing are not starved
    const int64_t cap = a.share_gpu ? shared_cap(int64_t(per_cu) * cus) : int64_t(per_cu) * cus;
    hipLaunchKernelGGL(k, dim3(unsigned(need < cap ? need : cap)), dim3(kThreads), 0, s, a);
    KGX_CHECK_LAUNCH();
  }
  if (has_short && launch_short<RED, W, TWO, NARROW>(a, s) != KGX_OK) return KGX_ERR_HIP;
  if (a.tpack && a.n_tiny > 0 && launch_tiny<RED, W, TWO, NARROW>(a, s) != KGX_OK) return KGX_ERR_HIP;
  if (a.items && a.n_split > 0) {
    const int64_t blocks = (a.n_split + 7) / 8;
    auto fk = spmm_gemm_fixup_kernel<RED, NARROW>;
    hipLaunchKernelGGL(fk, dim3(unsigned(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, a);
    KGX_CHECK_LAUNCH();
  }
  return KGX_OK;
}

}  // namespace
}  // namespace kgx

using namespace kgx;

extern "C" int kgx_spmm_gemm(int reduce, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                             const int32_t* items, int64_t n_items, const int32_t* split, int64_t n_split,
                             const int32_t* idx, const float* w, const float* x, int64_t ld_x, int64_t F_in,
                             const float* W, int64_t F_out, const float* bias, int flags, float gin_scale,
                             float* out, int64_t ld_out, float* partials, float* agg_out, int64_t ld_agg,
                             kgx_stream_t stream_) {
  return kgx_spmm_gemm_ex(reduce, rowptr, rows, n_rows, items, n_items, n_items, split, n_split, idx, w, x, ld_x,
                          F_in, W, F_out, bias, flags, gin_scale, out, ld_out, partials, agg_out, ld_agg, stream_);
}

extern "C" int kgx_spmm_gemm_ex(int reduce, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                                const int32_t* items, int64_t n_items, int64_t n_long_items, const int32_t* split,
                                int64_t n_split, const int32_t* idx, const float* w, const float* x, int64_t ld_x,
                                int64_t F_in, const float* W, int64_t F_out, const float* bias, int flags,
                                float gin_scale, float* out, int64_t ld_out, float* partials, float* agg_out,
                                int64_t ld_agg, kgx_stream_t stream_) {
  return kgx_spmm_gemm_ex2(reduce, rowptr, rows, n_rows, items, n_items, n_long_items, n_items, nullptr, nullptr, 0,
                           split, n_split, idx, w, x, ld_x, F_in, W, F_out, bias, flags, gin_scale, out, ld_out,
                           partials, agg_out, ld_agg, stream_);
}

extern "C" int kgx_spmm_gemm_ex2(int reduce, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                                 const int32_t* items, int64_t n_items, int64_t n_long_items, int64_t n_short_end,
                                 const int32_t* tiny_pack, const float* tiny_w, int64_t n_tiny_deg2,
                                 const int32_t* split,
                                 int64_t n_split, const int32_t* idx, const float* w, const float* x, int64_t ld_x,
                                 int64_t F_in, const float* W, int64_t F_out, const float* bias, int flags,
                                 float gin_scale, float* out, int64_t ld_out, float* partials, float* agg_out,
                                 int64_t ld_agg, kgx_stream_t stream_) {
  return kgx_spmm_gemm_ex3(reduce, rowptr, rows, n_rows, items, n_items, n_long_items, n_short_end, tiny_pack, tiny_w,
                           n_tiny_deg2, split, n_split, idx, w, x, ld_x, nullptr, 0, F_in, W, F_out, bias, flags,
                           gin_scale, out, ld_out, partials, agg_out, ld_agg, stream_);
}

extern "C" int kgx_spmm_gemm_ex3(int reduce, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                                 const int32_t* items, int64_t n_items, int64_t n_long_items, int64_t n_short_end,
                                 const int32_t* tiny_pack, const float* tiny_w, int64_t n_tiny_deg2,
                                 const int32_t* split, int64_t n_split, const int32_t* idx, const float* w,
                                 const float* x, int64_t ld_x, const float* x2, int64_t n_x1, int64_t F_in,
                                 const float* W, int64_t F_out, const float* bias, int flags, float gin_scale,
                                 float* out, int64_t ld_out, float* partials, float* agg_out, int64_t ld_agg,
                                 kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(!x2 || (n_x1 >= 0 && n_x1 < (int64_t(1) << 31) && reinterpret_cast<uintptr_t>(x2) % 16 == 0),
              KGX_ERR_ARG, "kgx_spmm_gemm: x2 must be 16-byte aligned and 0 <= n_x1 < 2^31");
  // (GIN's pre-scale reads the rows' own x: rows of the first table, local rows)
  KGX_REQUIRE(!x2 || (reduce == KGX_SUM && F_in == kFin && F_out % 16 == 0), KGX_ERR_UNSUPPORTED,
              "kgx_spmm_gemm: two-table gathers are implemented for sums at F_in 128, F_out %% 16 == 0 "
              "(the sharded GCN / GIN passes)");
  KGX_REQUIRE(!items || tiny_pack || n_short_end == n_items, KGX_ERR_ARG,
              "kgx_spmm_gemm: without tiny_pack, n_short_end must equal n_items");
  KGX_REQUIRE(!items || (n_long_items >= 0 && n_long_items <= n_short_end && n_short_end <= n_items), KGX_ERR_ARG,
              "kgx_spmm_gemm: need 0 <= n_long_items <= n_short_end <= n_items");
  KGX_REQUIRE(!tiny_pack || (items && (w == nullptr || tiny_w)), KGX_ERR_ARG,
              "kgx_spmm_gemm: the tiny-row records need the schedule (and weights when weighted)");
  KGX_REQUIRE(!tiny_pack || (n_tiny_deg2 >= 0 && n_tiny_deg2 <= n_items - n_short_end), KGX_ERR_ARG,
              "kgx_spmm_gemm: n_tiny_deg2 must lie in [0, n_items - n_short_end]");
  KGX_REQUIRE(reduce >= KGX_SUM && reduce <= KGX_MIN, KGX_ERR_ARG, "kgx_spmm_gemm: reduce %d unsupported", reduce);
  KGX_REQUIRE(F_in > 0 && F_in <= kFin && F_in % 4 == 0, KGX_ERR_UNSUPPORTED,
              "kgx_spmm_gemm: F_in must be a multiple of 4 <= %d (got %lld)", kFin, (long long)F_in);
  KGX_REQUIRE(F_out > 0 && F_out <= 128 && F_out % 4 == 0, KGX_ERR_UNSUPPORTED,
              "kgx_spmm_gemm: F_out must be a multiple of 4 <= 128 (got %lld)", (long long)F_out);
  KGX_REQUIRE(n_rows >= 0 && n_items >= 0 && n_split >= 0, KGX_ERR_ARG, "kgx_spmm_gemm: negative size");
  KGX_REQUIRE((flags & ~(KGX_FUSED_PRE_GIN | KGX_FUSED_ACCUMULATE | KGX_FUSED_SHARE_GPU | KGX_FUSED_RELU |
                         KGX_FUSED_CU_SPLIT)) == 0,
              KGX_ERR_ARG, "kgx_spmm_gemm: unknown flags 0x%x", flags);
  KGX_REQUIRE(!agg_out || (ld_agg >= F_in && reinterpret_cast<uintptr_t>(agg_out) % 16 == 0 && ld_agg % 4 == 0),
              KGX_ERR_ARG, "kgx_spmm_gemm: agg_out must be 16-byte aligned with ld >= F_in, ld %% 4 == 0");
  if (n_rows == 0) return KGX_OK;
  KGX_REQUIRE(rowptr && rows && idx && x && W && out, KGX_ERR_ARG, "kgx_spmm_gemm: null pointer");
  KGX_REQUIRE(ld_x >= F_in && ld_x < (int64_t(1) << 31), KGX_ERR_ARG,
              "kgx_spmm_gemm: x leading dimension must lie in [F_in, 2^31)");
  KGX_REQUIRE(ld_x % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 && ld_out >= F_out, KGX_ERR_ARG,
              "kgx_spmm_gemm: x must be 16-byte aligned with ld %% 4 == 0");
  KGX_REQUIRE(ld_out % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0, KGX_ERR_ARG,
              "kgx_spmm_gemm: out must be 16-byte aligned with ld %% 4 == 0 (row stores are dwordx4)");
  KGX_REQUIRE(!items || n_split == 0 || (split && partials), KGX_ERR_ARG,
              "kgx_spmm_gemm: split rows need split list and partials");
  FusedArgs a{};
  a.rowptr = rowptr;
  a.rows = rows;
  a.n_rows = n_rows;
  a.items = reinterpret_cast<const int4*>(items);
  a.n_items = items ? n_items : 0;
  a.n_long = items ? n_long_items : 0;
  a.n_short_end = items ? n_short_end : 0;
  a.tpack = items ? reinterpret_cast<const int4*>(tiny_pack) : nullptr;
  a.tw = reinterpret_cast<const float2*>(tiny_w);
  a.n_tiny = (items && tiny_pack) ? n_items - n_short_end : 0;
  a.n_tiny2 = a.n_tiny ? n_tiny_deg2 : 0;
  a.split = reinterpret_cast<const int4*>(split);
  a.n_split = items ? n_split : 0;
  a.idx = idx;
  a.w = w;
  a.x = x;
  a.ld_x = ld_x;
  a.n_x1 = x2 ? int32_t(n_x1) : INT32_MAX;
  // x2 - n_x1 * ld_x as an address (modular): gsrc adds row_off(c) for c >= n_x1
  a.x2b = x2 ? reinterpret_cast<const float*>(reinterpret_cast<uintptr_t>(x2) -
                                               uintptr_t(n_x1) * uintptr_t(ld_x) * sizeof(float))
             : x;
  a.W = W;
  a.F_in = int(F_in);
  a.F_out = int(F_out);
  a.bias = bias;
  a.out = out;
  a.ld_o = ld_out;
  a.partials = partials;
  a.agg_out = agg_out;
  a.ld_agg = ld_agg;
  a.pre_gin = (flags & KGX_FUSED_PRE_GIN) != 0;
  a.accumulate = (flags & KGX_FUSED_ACCUMULATE) != 0;
  a.share_gpu = (flags & KGX_FUSED_SHARE_GPU) != 0;
  a.relu = (flags & KGX_FUSED_RELU) != 0;
  a.cu_split = (flags & KGX_FUSED_CU_SPLIT) != 0;
  a.gin_scale = gin_scale;
  const bool wt = w != nullptr;
  if (x2) return wt ? launch<KGX_SUM, true, true>(a, stream) : launch<KGX_SUM, false, true>(a, stream);
  if (F_in < kFin || F_out % 16 != 0) {  // the masked instantiations (SAGEConv at C5: 100 -> 100)
    switch (reduce) {
      case KGX_SUM: return wt ? launch<KGX_SUM, true, false, true>(a, stream) : launch<KGX_SUM, false, false, true>(a, stream);
      case KGX_MEAN: return wt ? launch<KGX_MEAN, true, false, true>(a, stream) : launch<KGX_MEAN, false, false, true>(a, stream);
      case KGX_MAX: return wt ? launch<KGX_MAX, true, false, true>(a, stream) : launch<KGX_MAX, false, false, true>(a, stream);
      default: return wt ? launch<KGX_MIN, true, false, true>(a, stream) : launch<KGX_MIN, false, false, true>(a, stream);
    }
  }
  switch (reduce) {
    case KGX_SUM: return wt ? launch<KGX_SUM, true>(a, stream) : launch<KGX_SUM, false>(a, stream);
    case KGX_MEAN: return wt ? launch<KGX_MEAN, true>(a, stream) : launch<KGX_MEAN, false>(a, stream);
    case KGX_MAX: return wt ? launch<KGX_MAX, true>(a, stream) : launch<KGX_MAX, false>(a, stream);
    default: return wt ? launch<KGX_MIN, true>(a, stream) : launch<KGX_MIN, false>(a, stream);
  }
}
