// Fused aggregate -> dense transform for 256-wide rows (gfx950, wave64):
//
//   out[i, :] = bias + PRE( REDUCE_{e in CSR row i} x[col_e, :] * (w_e) ) @ W,   W [256, F_out <= 256]
//
// GINConv at BASELINE config C4 (F 256 -> 256, sum): (1+eps) x_i + aggr feeds
// the MLP's Dense (gin_conv.py:216-225, 129-162).  Unfused, the aggregation
// writes a [N, 256] intermediate that the dense kernel reads back (20.5 GB of
// HBM traffic at 10M rows); here each aggregated row goes from registers to
// LDS to the matrix cores and only the transformed row is written.
//
// Block = 512 threads = 8 waves (2 per SIMD, 256 VGPRs each), one block per CU.
// Per tile the block takes 16 consecutive schedule items; wave w reduces items
// 2w, 2w+1 with 64 lanes x float4 (one 1-KB row per gather, both rows' edges in
// flight together, sequential RN adds as in spmm_kernel) and writes the rows,
// split three ways into bf16 hi/mid/lo planes, to an LDS tile.  Then wave w
// computes output columns [32w, 32w + 32) of the 16-row tile as D^T = W^T x^T
// with 96 v_mfma_f32_16x16x32_bf16 (the six significant cross products of the
// split operands over K = 256; f32-accurate, kgx_bf16x3.h).  W's split planes
// take 384 KB: the hi and mid B-fragments of a wave's 32 columns live in 128
// VGPRs for the whole kernel, the lo plane (used by one product of the six) in
// 128 KB of LDS, read once per k-step.  The next tile's first gathers are
// issued before the MFMA phase (LDS-only barriers keep them in flight).  Hub-row
// chunks write raw partials; the fix-up kernel combines them in order and
// applies W in f32 on the VALU.  The degree <= 2 tail has its own kernel below.
#include <cstdlib>

#include "kgx_bf16x3.h"
#include "kgx_internal.h"
#include "kgx_red.h"
#include "kgx_vec.h"

namespace kgx {
namespace {

constexpr int kF = 256;            // F_in
constexpr int kWaves = 8;          // waves per block (one block per CU, 2 waves per SIMD)
constexpr int kRows = 2 * kWaves;  // rows per tile: two per wave
constexpr int kColBlocks = 16;     // 16-column blocks of F_out: two per wave
constexpr int kThreads = kWaves * 64;
constexpr int kLd = kF + 8;        // LDS plane row (bf16): +16 B keeps the B-fragment reads conflict-free
constexpr int kSteps = kF / 32;    // k-steps of 32 per MFMA chain
// The transform's operand split: three bf16 planes (kgx_bf16x3.h), six MFMAs
// per k-step, W's lo plane in LDS.  The measured f16x2 split (three products,
// 2^-20.4-accurate: outside the f32 contract) and the cost-decomposition
// builds are kept out of this file: tools/experiments/round4_variants.patch.
constexpr int kPlanes = 3;  // activation planes per tile row

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

struct F256Args {
  const int32_t* rowptr;
  const int32_t* rows;
  int64_t n_rows;
  const int4* items;  // {row, beg, end, slot}
  int64_t n_items;
  int64_t n_work;     // items [0, n_work) to spmm_gemm256_kernel; [n_work, n_items) are the tiny records' rows
  int64_t n_long;     // items [0, n_long): hub chunks and rows of degree > 7 (-1: not given)
  const int4* tpack;  // [n_tiny] {row, degree <= 2, col0, col1}
  const float2* tw;   // [n_tiny] {w0, w1} (weighted)
  int64_t n_tiny;
  const int4* split;  // {row, first slot, chunks, degree}
  int64_t n_split;
  const int32_t* idx;
  const float* w;
  const float* x;
  int64_t ld_x;
  const float* W;  // [256, F_out] row-major
  int F_out;
  const float* bias;
  float* out;
  int64_t ld_o;
  float* partials;  // [n_slots, 256]
  float* agg_out;   // optional [n, ld_agg]: PRE(REDUCE(...)) rows (backward's dW)
  int64_t ld_agg;
  int pre_gin;
  int accumulate;
  int relu;
  float gin_scale;
  // two-table gathers (kgx_spmm_gemm_f256_ex): source columns c >= n_x1 are rows
  // c - n_x1 of a second table x2 (same ld_x); x2b = x2 - n_x1 * ld_x (host
  // address math), so a gather's address is one select of the base
  const float* x2b;
  int32_t n_x1;
  bool cu_split;  // KGX_FUSED_CU_SPLIT (host side only)
};

// Source row of column c: x[c], or with TWO x2[c - n_x1].  Root rows (pre_gin's
// x_i) are always rows of x.
template <bool TWO>
__device__ __forceinline__ const float* gsrc256(const F256Args& a, int32_t c) {
  if constexpr (TWO) return (c >= a.n_x1 ? a.x2b : a.x) + row_off(c, a.ld_x);
  return a.x + row_off(c, a.ld_x);
}

// workgroup barrier for LDS hand-offs only (lgkmcnt, not vmcnt): gathers
// prefetched for the next tile stay in flight across it
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// W fragments of this wave's two 16-column blocks, k permuted: k-step s of lane
// group q covers k = 64 q + 8 s + j (j = 0..7), so each x fragment is 8
// contiguous bf16 of a tile row.  hi / mid planes to registers, lo to LDS.
__device__ __forceinline__ void load_w(const F256Args& a, int wave, int wl, bf16x8_t (&wfh)[2][kSteps],
                                       bf16x8_t (&wfm)[2][kSteps], u32x4_t* wlo) {
  const int cl = wl & 15, q = wl >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int n_col = 32 * wave + 16 * i + cl;
    const bool on = n_col < a.F_out;  // F_out % 16 == 0: whole column blocks
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      u32x4_t ph, pm, pl;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const int k = 64 * q + 8 * s + j;
        const float v0 = on ? a.W[int64_t(k) * a.F_out + n_col] : 0.0f;
        const float v1 = on ? a.W[int64_t(k + 1) * a.F_out + n_col] : 0.0f;
        uint32_t h, m_, l;
        split3_pair(v0, v1, h, m_, l);
        ph[j / 2] = h;
        pm[j / 2] = m_;
        pl[j / 2] = l;
      }
      wfh[i][s] = __builtin_bit_cast(bf16x8_t, ph);
      wfm[i][s] = __builtin_bit_cast(bf16x8_t, pm);
      wlo[((2 * wave + i) * kSteps + s) * 64 + wl] = pl;
    }
  }
}

// One aggregated row (this lane's 4 features) into the split planes of LDS tile row t.
// Fast path: split3_pair_rn (three packed conversions per pair, equal to
// split3_a whenever both bf16 values are finite, which split_fast_ok checks);
// otherwise the per-value split3_a_lo (non-finite values to the lo plane).
__device__ __forceinline__ void put_row(short (*tile3)[kRows][kLd], int t, int f, const float (&v)[4]) {
  uint32_t h0, m0, l0, h1, m1, l1;
  split3_pair_rn(v[0], v[1], h0, m0, l0);
  split3_pair_rn(v[2], v[3], h1, m1, l1);
  uint2 ph = make_uint2(h0, h1), pm = make_uint2(m0, m1), pl = make_uint2(l0, l1);
  if (!split_fast_ok(v[0], v[1], v[2], v[3])) {  // inf / NaN / huge
    short h[4], m_[4], l[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) split3_a_lo(v[k], h[k], m_[k], l[k]);
    auto pk = [](short a, short b) { return uint32_t(uint16_t(a)) | (uint32_t(uint16_t(b)) << 16); };
    ph = make_uint2(pk(h[0], h[1]), pk(h[2], h[3]));
    pm = make_uint2(pk(m_[0], m_[1]), pk(m_[2], m_[3]));
    pl = make_uint2(pk(l[0], l[1]), pk(l[2], l[3]));
  }
  *reinterpret_cast<uint2*>(&tile3[0][t][f]) = ph;
  *reinterpret_cast<uint2*>(&tile3[1][t][f]) = pm;
  *reinterpret_cast<uint2*>(&tile3[2][t][f]) = pl;
}

// The 16-row tile in LDS times W: this wave's 32 output columns as D^T = W^T x^T
// (six significant products per k-step, small terms first), stored from the
// accumulators -- lane (cl, q) writes columns 32 wave + 16 i + 4 q .. + 3 of
// tile row cl (rows with tile_row < 0 are not stored).
__device__ __forceinline__ void transform_tile(const F256Args& a, const short (*tile3)[kRows][kLd],
                                               const bf16x8_t (&wfh)[2][kSteps], const bf16x8_t (&wfm)[2][kSteps],
                                               const u32x4_t* wlo, const float* sbias, const int32_t* tile_row,
                                               int wave, int wl) {
  const int cl = wl & 15, q = wl >> 4;
  const bool mf0 = 32 * wave < a.F_out, mf1 = 32 * wave + 16 < a.F_out;
  if (!mf0) return;
  f32x4 d[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
#pragma unroll
  for (int s = 0; s < kSteps; ++s) {
    const int kk = 64 * q + 8 * s;
    const bf16x8_t xh = *reinterpret_cast<const bf16x8_t*>(&tile3[0][cl][kk]);
    const bf16x8_t xm = *reinterpret_cast<const bf16x8_t*>(&tile3[1][cl][kk]);
    const bf16x8_t xl = *reinterpret_cast<const bf16x8_t*>(&tile3[2][cl][kk]);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i == 1 && !mf1) break;
      const bf16x8_t wf_lo = __builtin_bit_cast(bf16x8_t, wlo[((2 * wave + i) * kSteps + s) * 64 + wl]);
      d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfh[i][s], xl, d[i], 0, 0, 0);
      d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf_lo, xh, d[i], 0, 0, 0);
      d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfm[i][s], xm, d[i], 0, 0, 0);
      d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfh[i][s], xm, d[i], 0, 0, 0);
      d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfm[i][s], xh, d[i], 0, 0, 0);
      d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfh[i][s], xh, d[i], 0, 0, 0);
    }
  }
  const int rr = tile_row[cl];
  if (rr < 0) return;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (i == 1 && !mf1) break;
    const int c4 = 32 * wave + 16 * i + 4 * q;
    float4* dst = reinterpret_cast<float4*>(a.out + int64_t(rr) * a.ld_o + c4);
    const float4 b4 = *reinterpret_cast<const float4*>(&sbias[c4]);
    float4 v = make_float4(d[i][0] + b4.x, d[i][1] + b4.y, d[i][2] + b4.z, d[i][3] + b4.w);
    if (a.accumulate) {
      const float4 p = *dst;
      v = make_float4(__fadd_rn(p.x, v.x), __fadd_rn(p.y, v.y), __fadd_rn(p.z, v.z), __fadd_rn(p.w, v.w));
    }
    if (a.relu) v = make_float4(fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f), fmaxf(v.z, 0.0f), fmaxf(v.w, 0.0f));
    *dst = v;
  }
}

// Items [0, n_work): hub-row chunks, long rows and rows of degree 3..7 (the
// degree <= 2 tail goes to spmm_gemm256_tiny2_kernel when its records exist).
// PF = edges per row gathered ahead, during the previous tile's MFMAs: 4 for the
// long rows; kMidPF = 6 for the schedule's rows of degree 3..7 (a second
// launch over items [n_long, n_work)), most of which are then gathered whole a
// tile ahead.
constexpr int kMidPF = 6;
// pre_gin: the rows' own x rows are loaded with the next tile's prefetch
// instead of after the fold, where their latency was exposed once per tile
// (C4 layer 21.51-21.53 -> 21.20-21.21 ms interleaved; 8 more VGPRs spilled
// in a kernel already at 256, which costs less than the wait)
template <int RED, bool WEIGHTED, int PF, bool TWO>
__global__ __launch_bounds__(kThreads, 1) void spmm_gemm256_kernel(F256Args a) {
  using R = RowRed<RED>;
  constexpr int U = 4;  // gathers in flight per row in the two-row loop (8 per wave)
  __shared__ u32x4_t wlo[kColBlocks * kSteps * 64];  // W lo-plane B-fragments, 128 KB
  __shared__ __attribute__((aligned(16))) short tile3[kPlanes][kRows][kLd];  // the split planes of the tile's rows
  __shared__ __attribute__((aligned(16))) float sbias[kF];
  __shared__ int32_t tile_row[kRows];

  const int wave = threadIdx.x >> 6;  // reduces tile rows 2 wave, 2 wave + 1; owns output columns [32 wave, +32)
  const int wl = threadIdx.x & 63;
  const int f = wl * 4;
  bf16x8_t wfh[2][kSteps], wfm[2][kSteps];
  load_w(a, wave, wl, wfh, wfm, wlo);
  if (threadIdx.x < kF) sbias[threadIdx.x] = (a.bias && int(threadIdx.x) < a.F_out) ? a.bias[threadIdx.x] : 0.0f;
  // (both are first read after the first tile's barrier)

  const int64_t n_work = a.items ? a.n_work : a.n_rows;
  const int64_t stride = int64_t(gridDim.x) * kRows;

  int32_t row[2], beg[2], end[2], slot[2];
  int pn[2];
  float pv[2][PF][4], pw[2][PF];
  float px[2][4];  // pre_gin: the rows' own x rows, loaded with the prefetch
  // descriptors of items it, it + 1 and their first PF gathers
  auto fetch = [&](int64_t it) {
    int32_t c[2][PF];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      row[r] = -1;
      beg[r] = end[r] = 0;
      slot[r] = -1;
      if (it + r < n_work) {
        if (a.items) {
          const int4 v = a.items[it + r];
          row[r] = v.x;
          beg[r] = v.y;
          end[r] = v.z;
          slot[r] = v.w;
        } else {
          row[r] = a.rows[it + r];
          beg[r] = a.rowptr[row[r]];
          end[r] = a.rowptr[row[r] + 1];
        }
      }
      pn[r] = (end[r] - beg[r]) < PF ? (end[r] - beg[r]) : PF;
#pragma unroll
      for (int u = 0; u < PF; ++u) {  // clamped addresses (idx / w hold >= 1 element); masked at the fold
        const int32_t ee = pn[r] > 0 ? beg[r] + (u < pn[r] ? u : pn[r] - 1) : 0;
        const int32_t ci = a.idx[ee];
        c[r][u] = pn[r] > 0 ? ci : 0;
        if constexpr (WEIGHTED) pw[r][u] = a.w[ee];
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int u = 0; u < PF; ++u)
        if (u < pn[r]) vload<4>(pv[r][u], gsrc256<TWO>(a, c[r][u]) + f);
    if (a.pre_gin) {  // wave-uniform; clamped rows, unconditional per lane
#pragma unroll
      for (int r = 0; r < 2; ++r) vload<4>(px[r], a.x + int64_t(row[r] >= 0 ? row[r] : 0) * a.ld_x + f);
    }
  };

  fetch(int64_t(blockIdx.x) * kRows + 2 * wave);
  for (int64_t base = int64_t(blockIdx.x) * kRows; base < n_work; base += stride) {
    float acc[2][4];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[r][k] = R::init();
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int u = 0; u < PF; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float m = WEIGHTED ? __fmul_rn(pv[r][u][k], pw[r][u]) : pv[r][u][k];
          acc[r][k] = R::combine(acc[r][k], u < pn[r] ? R::msg(m) : R::init());
        }
    // B edges of row r from edge e (the last ones clamped / masked when fewer remain)
    auto block = [&](auto RR, auto UB, int32_t e) {
      constexpr int r = decltype(RR)::value;
      constexpr int B = decltype(UB)::value;
      const int n = end[r] - e;
      int32_t c[B];
      float wt[B];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int32_t ee = u < n ? e + u : end[r] - 1;
        c[u] = a.idx[ee];
        if constexpr (WEIGHTED) wt[u] = a.w[ee];
      }
      float v[B][4];
#pragma unroll
      for (int u = 0; u < B; ++u) vload<4>(v[u], gsrc256<TWO>(a, c[u]) + f);
#pragma unroll
      for (int u = 0; u < B; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float m = WEIGHTED ? __fmul_rn(v[u][k], wt[u]) : v[u][k];
          acc[r][k] = R::combine(acc[r][k], u < n ? R::msg(m) : R::init());
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    int32_t e0 = beg[0] + PF, e1 = beg[1] + PF;
    // both rows together (a tile's rows have similar degrees: degree-ordered schedule), then each alone
    for (; e0 + U <= end[0] && e1 + U <= end[1]; e0 += U, e1 += U) {
      int32_t c[2][U];
      float wt[2][U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        c[0][u] = a.idx[e0 + u];
        c[1][u] = a.idx[e1 + u];
        if constexpr (WEIGHTED) {
          wt[0][u] = a.w[e0 + u];
          wt[1][u] = a.w[e1 + u];
        }
      }
      float v[2][U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        vload<4>(v[0][u], gsrc256<TWO>(a, c[0][u]) + f);
        vload<4>(v[1][u], gsrc256<TWO>(a, c[1][u]) + f);
      }
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int k = 0; k < 4; ++k)
            acc[r][k] = R::combine(acc[r][k], R::msg(WEIGHTED ? __fmul_rn(v[r][u][k], wt[r][u]) : v[r][u][k]));
    }
    for (; e0 + 8 <= end[0]; e0 += 8) block(I0{}, std::integral_constant<int, 8>{}, e0);
    for (; e0 < end[0]; e0 += 4) block(I0{}, std::integral_constant<int, 4>{}, e0);
    for (; e1 + 8 <= end[1]; e1 += 8) block(I1{}, std::integral_constant<int, 8>{}, e1);
    for (; e1 < end[1]; e1 += 4) block(I1{}, std::integral_constant<int, 4>{}, e1);

#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const bool full_row = row[r] >= 0 && slot[r] < 0;
      if (row[r] >= 0 && slot[r] >= 0) vstore<4>(a.partials + int64_t(slot[r]) * kF + f, acc[r]);
      float v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = full_row ? R::finish(acc[r][k], end[r] - beg[r]) : 0.0f;
      if (full_row && a.pre_gin) {
        float xv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) xv[k] = px[r][k];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __fadd_rn(__fmul_rn(a.gin_scale, xv[k]), v[k]);
      }
      if (full_row && a.agg_out) vstore<4>(a.agg_out + int64_t(row[r]) * a.ld_agg + f, v);
      put_row(tile3, 2 * wave + r, f, v);
      if (wl == 0) tile_row[2 * wave + r] = full_row ? row[r] : -1;
    }
    lds_barrier();
    fetch(base + stride + 2 * wave);  // the next tile's first gathers fly during the MFMAs
    transform_tile(a, tile3, wfh, wfm, wlo, sbias, tile_row, wave, wl);
    lds_barrier();  // the planes and tile_row are free for the next tile
  }
}

// The schedule's tail of rows of degree <= 2, from the packed records {row,
// degree, col0, col1} (+ {w0, w1}; tiny.py), double-buffered.  W's lo
// plane is split: k-steps 0..3 in 32 VGPRs, 4..7 in 64 KB of LDS, which leaves
// room for two 16-row plane tiles.  One barrier per tile period: in period t
// every wave runs tile t's MFMAs (buffer t & 1) and prepares tile t+1 (fold,
// split, planes into buffer (t+1) & 1, then issues tile t+2's gathers and
// loads tile t+3's records), preparation first.  One gather stage: tile t+2's
// rows are issued right after tile t+1's are folded and have a whole period to
// land.  Loads are
// unconditional (col1 = col0 for degree 1, 0 for degree 0 and past the end;
// masked at the fold), records are marked past the end only where used (a
// select right after the load would make hipcc wait for it), and with FAST
// (F_out = 256, no accumulate, no saved aggregate) every full tile's stores are
// unconditional too: the count of memory operations in flight is then the same
// on every path, so the compiler's waits before a fold stay partial.
template <int RED, bool WEIGHTED, bool GIN, bool FAST, bool TWO>
__global__ __launch_bounds__(kThreads, 1) void spmm_gemm256_tiny2_kernel(F256Args a) {
  using R = RowRed<RED>;
  constexpr int RPW = 2;  // rows per wave per tile
  constexpr int kHalf = kSteps / 2;
  __shared__ u32x4_t wlo[kColBlocks * kHalf * 64];  // lo plane, k-steps 4..7: 64 KB
  __shared__ __attribute__((aligned(16))) short tile3[2][kPlanes][kRows][kLd];  // two tiles of split planes
  __shared__ __attribute__((aligned(16))) float sbias[kF];
  __shared__ int32_t tile_row[2][kRows];

  const int wave = threadIdx.x >> 6;
  const int wl = threadIdx.x & 63;
  const int f = wl * 4;
  const int cl = wl & 15, q = wl >> 4;
  bf16x8_t wfh[2][kSteps], wfm[2][kSteps], wfl[2][kHalf];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int n_col = 32 * wave + 16 * i + cl;
    const bool on = n_col < a.F_out;
#pragma unroll
    for (int st = 0; st < kSteps; ++st) {
      u32x4_t ph, pm, pl;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const int k = 64 * q + 8 * st + j;
        const float v0 = on ? a.W[int64_t(k) * a.F_out + n_col] : 0.0f;
        const float v1 = on ? a.W[int64_t(k + 1) * a.F_out + n_col] : 0.0f;
        uint32_t h, m_, l;
        split3_pair(v0, v1, h, m_, l);
        ph[j / 2] = h;
        pm[j / 2] = m_;
        pl[j / 2] = l;
      }
      wfh[i][st] = __builtin_bit_cast(bf16x8_t, ph);
      wfm[i][st] = __builtin_bit_cast(bf16x8_t, pm);
      if (st < kHalf)
        wfl[i][st] = __builtin_bit_cast(bf16x8_t, pl);
      else
        wlo[((2 * wave + i) * kHalf + st - kHalf) * 64 + wl] = pl;
    }
  }
  if (threadIdx.x < kF) sbias[threadIdx.x] = (a.bias && int(threadIdx.x) < a.F_out) ? a.bias[threadIdx.x] : 0.0f;

  const int64_t n = a.n_tiny;
  const int64_t stride = int64_t(gridDim.x) * kRows;
  int32_t rid[RPW], rdeg[RPW];
  float pv[RPW][2][4], px[RPW][4], pw[RPW][2];
  int4 rec[2][RPW];
  float2 rw[2][RPW];
  bool rval[2][RPW];
  auto load_rec = [&](int b, int64_t it) {  // records of rows it, it + 1 into buffer b (clamped, marked when used)
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const bool v = it + r < n;
      const int64_t i = v ? it + r : n - 1;
      if (b == 0) {
        rval[0][r] = v;
        rec[0][r] = a.tpack[i];
        if constexpr (WEIGHTED) rw[0][r] = a.tw[i];
      } else {
        rval[1][r] = v;
        rec[1][r] = a.tpack[i];
        if constexpr (WEIGHTED) rw[1][r] = a.tw[i];
      }
    }
  };
  auto issue = [&](auto BT) {  // the gathers of the rows in record buffer B (one dependent load each)
    constexpr int B = decltype(BT)::value;
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      rid[r] = rval[B][r] ? rec[B][r].x : -1;
      rdeg[r] = rval[B][r] ? rec[B][r].y : 0;
      if constexpr (WEIGHTED) {
        pw[r][0] = rw[B][r].x;
        pw[r][1] = rw[B][r].y;
      }
      vload<4>(pv[r][0], gsrc256<TWO>(a, rec[B][r].z) + f);
      vload<4>(pv[r][1], gsrc256<TWO>(a, rec[B][r].w) + f);
      if constexpr (GIN) vload<4>(px[r], a.x + row_off(rec[B][r].x, a.ld_x) + f);
    }
  };
  // fold the gathered rows, split them into plane buffer pb; tile_row too
  auto put = [&](int pb) {
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      float val[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float acc = R::init();
        const float m0 = WEIGHTED ? __fmul_rn(pv[r][0][k], pw[r][0]) : pv[r][0][k];
        const float m1 = WEIGHTED ? __fmul_rn(pv[r][1][k], pw[r][1]) : pv[r][1][k];
        acc = R::combine(acc, rdeg[r] > 0 ? R::msg(m0) : R::init());
        acc = R::combine(acc, rdeg[r] > 1 ? R::msg(m1) : R::init());
        float v = R::finish(acc, rdeg[r]);
        if constexpr (GIN) v = __fadd_rn(__fmul_rn(a.gin_scale, px[r][k]), v);
        val[k] = rid[r] >= 0 ? v : 0.0f;
      }
      if (!FAST && rid[r] >= 0 && a.agg_out) vstore<4>(a.agg_out + int64_t(rid[r]) * a.ld_agg + f, val);
      put_row(tile3[pb], RPW * wave + r, f, val);
      if (wl == 0) tile_row[pb][RPW * wave + r] = rid[r];
    }
  };
  // tile in plane buffer pb times W; FASTS = unconditional stores (every row valid)
  auto mfma = [&](auto FT, int pb) {
    constexpr bool FASTS = decltype(FT)::value;
    const short(*t3)[kRows][kLd] = tile3[pb];
    const bool mf0 = FASTS || 32 * wave < a.F_out, mf1 = FASTS || 32 * wave + 16 < a.F_out;
    if (!mf0) return;
    f32x4 d[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
#pragma unroll
    for (int st = 0; st < kSteps; ++st) {
      const int kk = 64 * q + 8 * st;
      const bf16x8_t xh = *reinterpret_cast<const bf16x8_t*>(&t3[0][cl][kk]);
      const bf16x8_t xm = *reinterpret_cast<const bf16x8_t*>(&t3[1][cl][kk]);
      const bf16x8_t xl = *reinterpret_cast<const bf16x8_t*>(&t3[2][cl][kk]);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (i == 1 && !mf1) break;
        const bf16x8_t wf_lo = st < kHalf ? wfl[i][st < kHalf ? st : 0]
                                          : __builtin_bit_cast(bf16x8_t, wlo[((2 * wave + i) * kHalf + (st >= kHalf ? st - kHalf : 0)) * 64 + wl]);
        d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfh[i][st], xl, d[i], 0, 0, 0);
        d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf_lo, xh, d[i], 0, 0, 0);
        d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfm[i][st], xm, d[i], 0, 0, 0);
        d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfh[i][st], xm, d[i], 0, 0, 0);
        d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfm[i][st], xh, d[i], 0, 0, 0);
        d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfh[i][st], xh, d[i], 0, 0, 0);
      }
    }
    const int rr = tile_row[pb][cl];
    if (!FASTS && rr < 0) return;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i == 1 && !mf1) break;
      const int c4 = 32 * wave + 16 * i + 4 * q;
      float4* dst = reinterpret_cast<float4*>(a.out + int64_t(rr) * a.ld_o + c4);
      const float4 b4 = *reinterpret_cast<const float4*>(&sbias[c4]);
      float4 v = make_float4(d[i][0] + b4.x, d[i][1] + b4.y, d[i][2] + b4.z, d[i][3] + b4.w);
      if (!FASTS && a.accumulate) {
        const float4 p = *dst;
        v = make_float4(__fadd_rn(p.x, v.x), __fadd_rn(p.y, v.y), __fadd_rn(p.z, v.z), __fadd_rn(p.w, v.w));
      }
      if (a.relu) v = make_float4(fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f), fmaxf(v.z, 0.0f), fmaxf(v.w, 0.0f));
      *dst = v;
    }
  };
  // period t (parity p): tile t's MFMAs; tile t+1 folded into buffer p^1; tile
  // t+2's gathers issued from record buffer p; tile t+3's records into buffer p^1
  auto period = [&](auto FT, auto PT, int64_t base) {
    constexpr int P = decltype(PT)::value;
    auto prep = [&]() {
      put(P ^ 1);
      issue(std::integral_constant<int, P>{});
      load_rec(P ^ 1, base + 3 * stride + RPW * wave);
    };
    // prepare first: tile t+2's gathers are issued as early as possible and have
    // the whole period; measured against MFMA-first and a half / half split of
    // the waves (tools/gpu_jobs/gpu_r3_order.sh), this order was fastest
    prep();
    mfma(FT, P);
    lds_barrier();
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;

  const int64_t first = int64_t(blockIdx.x) * kRows + RPW * wave;
  // prologue: tile 0 into plane buffer 0, tile 1's gathers in flight, tile 2's records loaded
  load_rec(0, first);
  issue(P0{});
  load_rec(1, first + stride);
  put(0);
  issue(P1{});
  load_rec(0, first + 2 * stride);
  lds_barrier();
  int64_t base = int64_t(blockIdx.x) * kRows;
  int par = 0;
  for (;;) {
    if (base + kRows > n) break;
    period(std::integral_constant<bool, FAST>{}, P0{}, base);
    base += stride;
    par = 1;
    if (base + kRows > n) break;
    period(std::integral_constant<bool, FAST>{}, P1{}, base);
    base += stride;
    par = 0;
  }
  if (base < n) {  // the one partial tile (last block only)
    if (par == 0)
      period(std::false_type{}, P0{}, base);
    else
      period(std::false_type{}, P1{}, base);
  }
}

// Split hub rows: combine the chunk partials in order, finish, PRE, then
// out = v @ W + b in f32 on the VALU (a few thousand rows per graph).
template <int RED>
__global__ __launch_bounds__(256) void spmm_gemm256_fixup_kernel(F256Args a) {
  using R = RowRed<RED>;
  __shared__ float vrow[4][kF];
  const int g = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int64_t base = int64_t(blockIdx.x) * 4; base < a.n_split; base += int64_t(gridDim.x) * 4) {
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
        for (int u = 0; u < B; ++u)
          vload<4>(p[u], a.partials + int64_t(s.y + (c0 + u < s.z ? c0 + u : s.z - 1)) * kF + lane * 4);
#pragma unroll
        for (int u = 0; u < B; ++u)
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[k] = c0 + u < s.z ? R::combine(acc[k], p[u][k]) : acc[k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = R::finish(acc[k], s.w);
      if (a.pre_gin) {
        float xv[4];
        vload<4>(xv, a.x + int64_t(row) * a.ld_x + lane * 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] = __fadd_rn(__fmul_rn(a.gin_scale, xv[k]), acc[k]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) vrow[g][lane * 4 + k] = acc[k];
      if (a.agg_out) vstore<4>(a.agg_out + int64_t(row) * a.ld_agg + lane * 4, acc);
    }
    __syncthreads();
    if (row >= 0) {
      for (int c = lane; c < a.F_out; c += 64) {
        float s = 0.0f;
        for (int k = 0; k < kF; ++k) s = fmaf(vrow[g][k], a.W[int64_t(k) * a.F_out + c], s);
        float v = s + (a.bias ? a.bias[c] : 0.0f);
        if (a.accumulate) v = __fadd_rn(a.out[int64_t(row) * a.ld_o + c], v);
        if (a.relu) v = fmaxf(v, 0.0f);
        a.out[int64_t(row) * a.ld_o + c] = v;
      }
    }
    __syncthreads();
  }
}

template <typename K>
unsigned grid256(K k, int64_t tiles, int cus = 0) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kThreads, 0) != hipSuccess || per_cu <= 0) per_cu = 1;
  const int64_t cap = int64_t(per_cu) * (cus > 0 ? cus : cu_count());
  return unsigned(tiles < cap ? tiles : cap);
}

// Spatial split of the GPU for one launch (KGX_FUSED_CU_SPLIT; KGX_F256_CU_SPLIT
// = t, read per launch, default 8; 0 = off): the degree <= 2 tail -- MFMA-bound, its memory phase
// serialised with its MFMA phase inside every block -- runs on t of every 32
// CUs, beside the long-row and degree 3..7 launches -- memory-bound, MFMA pipes
// ~9 % busy -- on the other CUs, each on a CU-masked stream
// (hipExtStreamCreateWithCUMask) forked from and joined back into the caller's
// stream, each grid sized to its CU set.  Every row is still reduced by one
// kernel in the same order: the outputs are bit-identical to the one-stream
// order (tools/exp_cupart.py, tests/test_gpu_fused256.py).  Measured on C4
// (profiles/r05/c4_cupart*.json): see DESIGN.md §4.
inline int cu_split_per32() {
  const char* e = getenv("KGX_F256_CU_SPLIT");
  const int v = e ? atoi(e) : 8;
  return v > 0 && v < 32 ? v : 0;
}

// KGX_F256_MID_TAIL (per mille, read per launch; default 200): the share of the degree 3..7
// rows a split launch runs on the tail's CUs after the degree <= 2 tail instead of on the
// head's.  C4 (interleaved, three rounds, profiles/r06/c4_balance/): 0 20.01-20.07 ms, 150
// 19.69-19.70, 200 19.52-19.61, 250 19.49-19.65, 300 19.99-20.17 (the tail leg then longer)
inline int mid_tail_permille() {
  const char* e = getenv("KGX_F256_MID_TAIL");
  const int v = e ? atoi(e) : 200;
  return v < 0 ? 0 : (v > 1000 ? 1000 : v);
}

template <int RED, bool WT, bool TWO>
int launch256(const F256Args& a, hipStream_t s) {
  const int64_t work = a.items ? a.n_work : a.n_rows;
  hipStream_t sh = s, st = s;  // head (long + degree 3..7) and tail streams
  int cus_h = 0, cus_t = 0;
  SplitJoin join;
  const int per32 = (a.cu_split && a.tpack && a.n_tiny > 0 && work > 0) ? cu_split_per32() : 0;
  if (per32) {
    if (CuSplit* cs = cu_split(per32, s)) {
      KGX_CHECK_HIP(hipEventRecord(cs->fork, s));
      KGX_CHECK_HIP(hipStreamWaitEvent(cs->head, cs->fork, 0));
      KGX_CHECK_HIP(hipStreamWaitEvent(cs->tail, cs->fork, 0));
      join.cs = cs;
      join.s = s;
      sh = cs->head;
      st = cs->tail;
      cus_h = cs->n_head;
      cus_t = cs->n_tail;
    }
  }
  // long rows and hub chunks [0, n_long), then the rows of degree 3..7 [n_long, n_work)
  const int64_t n_long = (a.items && a.n_long >= 0 && a.n_long < work) ? a.n_long : work;
  if (n_long > 0) {
    F256Args b = a;
    b.n_work = n_long;
    if (!a.items) b.n_rows = n_long;
    auto k = spmm_gemm256_kernel<RED, WT, 4, TWO>;
    hipLaunchKernelGGL(k, dim3(grid256(k, (n_long + kRows - 1) / kRows, cus_h)), dim3(kThreads), 0, sh, b);
    KGX_CHECK_LAUNCH();
  }
  // split: the last mid_tail / 1000 of the degree 3..7 rows (the lowest degrees) go to the
  // tail's CUs after the degree <= 2 tail, balancing the two legs
  const int64_t n_cut = (sh != st && work > n_long) ? work - (work - n_long) * mid_tail_permille() / 1000 : work;
  if (n_cut > n_long) {
    F256Args b = a;
    b.items = a.items + n_long;
    b.n_work = n_cut - n_long;
    auto k = spmm_gemm256_kernel<RED, WT, kMidPF, TWO>;
    hipLaunchKernelGGL(k, dim3(grid256(k, (b.n_work + kRows - 1) / kRows, cus_h)), dim3(kThreads), 0, sh, b);
    KGX_CHECK_LAUNCH();
  }
  if (a.tpack && a.n_tiny > 0) {
    const bool fast = a.F_out == kF && !a.accumulate && !a.agg_out;
    auto k = a.pre_gin
                 ? (fast ? spmm_gemm256_tiny2_kernel<RED, WT, true, true, TWO> : spmm_gemm256_tiny2_kernel<RED, WT, true, false, TWO>)
                 : (fast ? spmm_gemm256_tiny2_kernel<RED, WT, false, true, TWO>
                         : spmm_gemm256_tiny2_kernel<RED, WT, false, false, TWO>);
    hipLaunchKernelGGL(k, dim3(grid256(k, (a.n_tiny + kRows - 1) / kRows, cus_t)), dim3(kThreads), 0, st, a);
    KGX_CHECK_LAUNCH();
  }
  if (work > n_cut) {
    F256Args b = a;
    b.items = a.items + n_cut;
    b.n_work = work - n_cut;
    auto k = spmm_gemm256_kernel<RED, WT, kMidPF, TWO>;
    hipLaunchKernelGGL(k, dim3(grid256(k, (b.n_work + kRows - 1) / kRows, cus_t)), dim3(kThreads), 0, st, b);
    KGX_CHECK_LAUNCH();
  }
  if (join.cs) {  // the fix-up reads the long launch's partials: join first
    CuSplit* cs = join.cs;
    join.cs = nullptr;
    KGX_CHECK_HIP(hipEventRecord(cs->jh, cs->head));
    KGX_CHECK_HIP(hipEventRecord(cs->jt, cs->tail));
    KGX_CHECK_HIP(hipStreamWaitEvent(s, cs->jh, 0));
    KGX_CHECK_HIP(hipStreamWaitEvent(s, cs->jt, 0));
  }
  if (a.items && a.n_split > 0) {
    const int64_t blocks = (a.n_split + 3) / 4;
    hipLaunchKernelGGL(spmm_gemm256_fixup_kernel<RED>, dim3(unsigned(blocks < 4096 ? blocks : 4096)), dim3(256), 0,
                       s, a);
    KGX_CHECK_LAUNCH();
  }
  return KGX_OK;
}

}  // namespace
}  // namespace kgx

using namespace kgx;

extern "C" int kgx_spmm_gemm_f256_ex(int reduce, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                                     const int32_t* items, int64_t n_items, int64_t n_long_items, int64_t n_short_end,
                                     const int32_t* tiny_pack, const float* tiny_w, const int32_t* split,
                                     int64_t n_split, const int32_t* idx, const float* w, const float* x,
                                     int64_t ld_x, const float* x2, int64_t n_x1, int64_t F_in, const float* W,
                                     int64_t F_out, const float* bias, int flags, float gin_scale, float* out,
                                     int64_t ld_out, float* partials, float* agg_out, int64_t ld_agg,
                                     kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(reduce >= KGX_SUM && reduce <= KGX_MIN, KGX_ERR_ARG, "kgx_spmm_gemm_f256: reduce %d unsupported",
              reduce);
  KGX_REQUIRE(F_in == kF, KGX_ERR_UNSUPPORTED, "kgx_spmm_gemm_f256: F_in must be %d (got %lld)", kF,
              (long long)F_in);
  KGX_REQUIRE(F_out > 0 && F_out <= kF && F_out % 16 == 0, KGX_ERR_UNSUPPORTED,
              "kgx_spmm_gemm_f256: F_out must be a multiple of 16 <= 256 (got %lld)", (long long)F_out);
  KGX_REQUIRE(n_rows >= 0 && n_items >= 0 && n_split >= 0, KGX_ERR_ARG, "kgx_spmm_gemm_f256: negative size");
  KGX_REQUIRE(!items || tiny_pack || n_short_end == n_items, KGX_ERR_ARG,
              "kgx_spmm_gemm_f256: without tiny_pack, n_short_end must equal n_items");
  KGX_REQUIRE(!tiny_pack || (items && n_short_end >= 0 && n_short_end <= n_items && (w == nullptr || tiny_w)),
              KGX_ERR_ARG, "kgx_spmm_gemm_f256: the tiny-row records need the schedule, 0 <= n_short_end <= n_items "
              "(and weights when weighted)");
  KGX_REQUIRE((flags & ~(KGX_FUSED_PRE_GIN | KGX_FUSED_ACCUMULATE | KGX_FUSED_SHARE_GPU | KGX_FUSED_RELU |
                         KGX_FUSED_CU_SPLIT)) == 0,
              KGX_ERR_ARG, "kgx_spmm_gemm_f256: unknown flags 0x%x", flags);
  KGX_REQUIRE(!((flags & KGX_FUSED_RELU) && (flags & KGX_FUSED_ACCUMULATE)), KGX_ERR_ARG,
              "kgx_spmm_gemm_f256: KGX_FUSED_RELU cannot be combined with KGX_FUSED_ACCUMULATE");
  KGX_REQUIRE(!agg_out || (ld_agg >= F_in && reinterpret_cast<uintptr_t>(agg_out) % 16 == 0 && ld_agg % 4 == 0),
              KGX_ERR_ARG, "kgx_spmm_gemm_f256: agg_out must be 16-byte aligned with ld >= F_in, ld %% 4 == 0");
  KGX_REQUIRE(!x2 || (n_x1 >= 0 && n_x1 < (int64_t(1) << 31) && reinterpret_cast<uintptr_t>(x2) % 16 == 0),
              KGX_ERR_ARG, "kgx_spmm_gemm_f256: x2 must be 16-byte aligned and 0 <= n_x1 < 2^31");
  KGX_REQUIRE(!x2 || reduce == KGX_SUM, KGX_ERR_UNSUPPORTED,
              "kgx_spmm_gemm_f256: two-table gathers are implemented for the sum");
  if (n_rows == 0) return KGX_OK;
  KGX_REQUIRE(rowptr && rows && idx && x && W && out, KGX_ERR_ARG, "kgx_spmm_gemm_f256: null pointer");
  KGX_REQUIRE(ld_x < (int64_t(1) << 31), KGX_ERR_ARG, "kgx_spmm_gemm_f256: x leading dimension >= 2^31");
  KGX_REQUIRE(ld_x % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0, KGX_ERR_ARG,
              "kgx_spmm_gemm_f256: x must be 16-byte aligned with ld %% 4 == 0");
  KGX_REQUIRE(ld_out >= F_out && ld_out % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0, KGX_ERR_ARG,
              "kgx_spmm_gemm_f256: out must be 16-byte aligned with ld >= F_out, ld %% 4 == 0");
  KGX_REQUIRE(!items || n_split == 0 || (split && partials), KGX_ERR_ARG,
              "kgx_spmm_gemm_f256: split rows need split list and partials");
  F256Args a{};
  a.rowptr = rowptr;
  a.rows = rows;
  a.n_rows = n_rows;
  a.items = reinterpret_cast<const int4*>(items);
  a.n_items = items ? n_items : 0;
  a.n_work = items ? (tiny_pack ? n_short_end : n_items) : 0;
  a.n_long = items ? n_long_items : -1;
  a.tpack = items ? reinterpret_cast<const int4*>(tiny_pack) : nullptr;
  a.tw = reinterpret_cast<const float2*>(tiny_w);
  a.n_tiny = (items && tiny_pack) ? n_items - n_short_end : 0;
  a.split = reinterpret_cast<const int4*>(split);
  a.n_split = items ? n_split : 0;
  a.idx = idx;
  a.w = w;
  a.x = x;
  a.ld_x = ld_x;
  a.W = W;
  a.F_out = int(F_out);
  a.bias = bias;
  a.out = out;
  a.ld_o = ld_out;
  a.partials = partials;
  a.agg_out = agg_out;
  a.ld_agg = ld_agg;
  a.pre_gin = (flags & KGX_FUSED_PRE_GIN) != 0;
  a.accumulate = (flags & KGX_FUSED_ACCUMULATE) != 0;
  a.relu = (flags & KGX_FUSED_RELU) != 0;
  a.gin_scale = gin_scale;
  a.cu_split = (flags & KGX_FUSED_CU_SPLIT) != 0;
  a.n_x1 = x2 ? int32_t(n_x1) : INT32_MAX;
  // x2 - n_x1 * ld_x as an address (modular): gsrc256 adds row_off(c) for c >= n_x1
  a.x2b = x2 ? reinterpret_cast<const float*>(reinterpret_cast<uintptr_t>(x2) -
                                               uintptr_t(n_x1) * uintptr_t(ld_x) * sizeof(float))
             : nullptr;
  const bool wt = w != nullptr;
  if (x2) return wt ? launch256<KGX_SUM, true, true>(a, stream) : launch256<KGX_SUM, false, true>(a, stream);
  switch (reduce) {
    case KGX_SUM: return wt ? launch256<KGX_SUM, true, false>(a, stream) : launch256<KGX_SUM, false, false>(a, stream);
    case KGX_MEAN: return wt ? launch256<KGX_MEAN, true, false>(a, stream) : launch256<KGX_MEAN, false, false>(a, stream);
    case KGX_MAX: return wt ? launch256<KGX_MAX, true, false>(a, stream) : launch256<KGX_MAX, false, false>(a, stream);
    default: return wt ? launch256<KGX_MIN, true, false>(a, stream) : launch256<KGX_MIN, false, false>(a, stream);
  }
}

extern "C" int kgx_spmm_gemm_f256(int reduce, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                                  const int32_t* items, int64_t n_items, int64_t n_long_items, int64_t n_short_end,
                                  const int32_t* tiny_pack, const float* tiny_w, const int32_t* split, int64_t n_split,
                                  const int32_t* idx, const float* w, const float* x, int64_t ld_x, int64_t F_in,
                                  const float* W, int64_t F_out, const float* bias, int flags, float gin_scale,
                                  float* out, int64_t ld_out, float* partials, float* agg_out, int64_t ld_agg,
                                  kgx_stream_t stream) {
  return kgx_spmm_gemm_f256_ex(reduce, rowptr, rows, n_rows, items, n_items, n_long_items, n_short_end, tiny_pack,
                               tiny_w, split, n_split, idx, w, x, ld_x, nullptr, 0, F_in, W, F_out, bias, flags,
                               gin_scale, out, ld_out, partials, agg_out, ld_agg, stream);
}
