// Fused GATv2 attention aggregation for the kgx engine (gfx950, wave64).
//
// Reference (src/keras_geometric/layers/gatv2_conv.py) materialises, per layer,
// h_j and h_i ([E,H,C] gathers, :245-246), the per-edge scores (:277-284), a
// segment_max / take / exp / segment_sum / take / divide softmax (:291-311),
// alpha*h_j (:257-258) and a segment_sum over [E,H*C] (:313-335).  Here one
// group of G lanes owns a destination row; lane l holds K consecutive channels
// of head l/LH.  Each edge's source row is gathered ONCE; the score is a
// per-lane partial dot product reduced across the LH lanes of the head with
// xor-shuffles; the softmax is computed online (running max m, running sum l,
// rescaled accumulator), U edges per rescale.  HBM traffic is one h_src row per
// edge plus h_dst and out per row — the reference's E x (3 x H*C) intermediates
// never exist.
//
// Numerics: algebraically identical to the reference; the score reduction order
// over C, exp, and the division placement differ at the ulp level, so GATv2 is
// tolerance-checked (|a-b| <= 1e-5*max(1,|b|)), not bit-checked.  The softmax
// numerator and denominator are accumulated in fp64 (exact to ~1e-7 even on
// 10^5-edge hub rows; the fp64 FMAs are free in this HBM-bound kernel).
#include <cstdlib>

#include "kgx_internal.h"
#include "kgx_vec.h"

namespace kgx {
namespace {

struct GatArgs {
  const int32_t* rowptr;
  const int32_t* rows;
  int64_t n_rows;
  const int4* items;
  int64_t n_items;
  const int4* split;
  int64_t n_split;
  const int32_t* col;
  const float* h_src;
  const float* h_dst;
  int64_t ld_h;
  const float* att;
  int H, C;
  float slope;
  float* out;
  int64_t ld_o;
  const float* bias;
  float* partials;  // per slot: [H*C acc | H m | H l]
  float* stats;     // optional [n, 2H]: per row and head, the softmax max m and denominator l + 1e-10
  // attention dropout (training): alpha_e *= keep(seed, drop_key[e], head) / (1 - p)
  const int32_t* drop_key;
  uint64_t drop_seed;
  uint32_t drop_thresh;
  float drop_scale;
  int G, lgG, LH, lgLH;
};

// Sum over the LH (power of two) lanes of a head, result in every lane.
// Within 16 lanes the exchanges are DPP moves (VALU, no LDS round trip):
// quad_perm xor 1 and xor 2, then row_half_mirror (lane i <-> 7-i) and
// row_mirror (i <-> 15-i) pair each lane with one holding the other half's sum.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int K>
__device__ __forceinline__ float head_reduce(float p, int LH) {
  if (LH > 1) p += dpp<0xB1>(p);   // quad_perm [1,0,3,2]
  if (LH > 2) p += dpp<0x4E>(p);   // quad_perm [2,3,0,1]
  if (LH > 4) p += dpp<0x141>(p);  // row_half_mirror
  if (LH > 8) p += dpp<0x140>(p);  // row_mirror
  if (LH > 16) p += __shfl_xor(p, 16, 64);
  if (LH > 32) p += __shfl_xor(p, 32, 64);
  return p;
}

template <int K>
__global__ __launch_bounds__(kBlock) void gatv2_kernel(GatArgs a) {
  // edges per online-softmax block: 3 measured best at C3 (K = 4): 1.27 ms vs 1.41 at 8, 1.30 at 4
  constexpr int U = K <= 4 ? 3 : (K == 8 ? 3 : 2);
  const int G = a.G;
  const int lane = threadIdx.x & (G - 1);
  const int head = lane >> a.lgLH;
  const int sub = lane & (a.LH - 1);
  const bool valid = head < a.H && sub * K < a.C;
  const int f = head * a.C + sub * K;
  const int HC = a.H * a.C;
  const int64_t ngroups = (int64_t(gridDim.x) * kBlock) >> a.lgG;
  const int64_t n_work = a.items ? a.n_items : a.n_rows;

  float att[K];
#pragma unroll
  for (int k = 0; k < K; ++k) att[k] = 0.0f;
  if (valid) vload<K>(att, a.att + f);

  for (int64_t it = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> a.lgG; it < n_work; it += ngroups) {
    int32_t row, beg, end, slot;
    if (a.items) {
      const int4 v = a.items[it];
      row = v.x;
      beg = v.y;
      end = v.z;
      slot = v.w;
    } else {
      row = a.rows[it];
      beg = a.rowptr[row];
      end = a.rowptr[row + 1];
      slot = -1;
    }
    // softmax numerator / denominator accumulated in fp64: a hub row sums
    // 10^5 terms, whose fp32 rounding (~sqrt(n) ulp) would exceed 1e-5.
    float hd[K];
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      hd[k] = 0.0f;
      acc[k] = 0.0;
    }
    if (valid) vload<K>(hd, a.h_dst + int64_t(row) * a.ld_h + f);
    float m = -__builtin_inff();
    double l = 0.0;

    for (int32_t e = beg; e < end; e += U) {
      const int n = (end - e) < U ? (end - e) : U;
      int32_t c[U];
#pragma unroll
      for (int u = 0; u < U; ++u) c[u] = a.col[u < n ? e + u : end - 1];
      float dm[U];  // attention dropout multiplier per edge (this lane's head)
#pragma unroll
      for (int u = 0; u < U; ++u)
        dm[u] = a.drop_key ? drop_scale(a.drop_seed, uint32_t(a.drop_key[u < n ? e + u : end - 1]), uint32_t(head),
                                        a.drop_thresh, a.drop_scale)
                           : 1.0f;
      // unconditional loads from clamped addresses (padding lanes read column 0
      // of the row; edges past the end re-read the last one), masked on use
      float hs[U][K];
#pragma unroll
      for (int u = 0; u < U; ++u) vload<K>(hs[u], a.h_src + row_off(c[u], a.ld_h) + (valid ? f : 0));
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < K; ++k) hs[u][k] = valid ? hs[u][k] : 0.0f;
      float s[U];
      float mc = -__builtin_inff();
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float p = 0.0f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float g = hd[k] + hs[u][k];
          const float z = g > 0.0f ? g : g * a.slope;  // leaky_relu
          p += z * att[k];
        }
        p = head_reduce<K>(p, a.LH);
        s[u] = p;
        if (u < n) mc = fmaxf(mc, p);
      }
      const float m_new = fmaxf(m, mc);
      const double scale = double(expf(m - m_new));
      l *= scale;
#pragma unroll
      for (int k = 0; k < K; ++k) acc[k] *= scale;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u < n) {
          const double pu = double(expf(s[u] - m_new));
          l += pu;  // the denominator sees every edge; dropout masks the normalised alpha
          const double pd = pu * double(dm[u]);
#pragma unroll
          for (int k = 0; k < K; ++k) acc[k] = fma(pd, double(hs[u][k]), acc[k]);
        }
      }
      m = m_new;
    }

    if (!valid) continue;
    if (slot >= 0) {
      float* p = a.partials + int64_t(slot) * (HC + 2 * a.H);
      float accf[K];
#pragma unroll
      for (int k = 0; k < K; ++k) accf[k] = float(acc[k]);
      vstore<K>(p + f, accf);
      if (sub == 0) {
        p[HC + head] = m;
        p[HC + a.H + head] = float(l);
      }
    } else {
      const double den = l + 1e-10;
      if (a.stats && sub == 0) {
        a.stats[int64_t(row) * 2 * a.H + head] = m;
        a.stats[int64_t(row) * 2 * a.H + a.H + head] = float(den);
      }
      float r[K];
#pragma unroll
      for (int k = 0; k < K; ++k) r[k] = float(acc[k] / den);
      if (a.bias) {
        float b[K];
        vload<K>(b, a.bias + f);
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] += b[k];
      }
      vstore<K>(a.out + int64_t(row) * a.ld_o + f, r);
    }
  }
}

template <int K>
__global__ __launch_bounds__(kBlock) void gatv2_fixup_kernel(GatArgs a) {
  const int G = a.G;
  const int lane = threadIdx.x & (G - 1);
  const int head = lane >> a.lgLH;
  const int sub = lane & (a.LH - 1);
  const bool valid = head < a.H && sub * K < a.C;
  const int f = head * a.C + sub * K;
  const int HC = a.H * a.C;
  const int64_t ngroups = (int64_t(gridDim.x) * kBlock) >> a.lgG;
  for (int64_t it = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> a.lgG; it < a.n_split; it += ngroups) {
    if (!valid) continue;
    const int4 sp = a.split[it];
    const int32_t row = sp.x, slot0 = sp.y, nc = sp.z;
    // One pass over the chunk partials, B chunks' loads in flight per step
    // (clamped, unconditional), the running max rescaled online as in the main
    // kernel: a hub row's ~160 partials cost ~10 load latencies, not ~320.
    constexpr int B = 16;
    const int64_t ld_p = HC + 2 * a.H;
    float M = -__builtin_inff();
    double L = 0.0, acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    for (int32_t c0 = 0; c0 < nc; c0 += B) {
      float mv[B], lv[B], v[B][K];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const float* p = a.partials + int64_t(slot0 + (c0 + u < nc ? c0 + u : nc - 1)) * ld_p;
        mv[u] = p[HC + head];
        lv[u] = p[HC + a.H + head];
        vload<K>(v[u], p + f);
      }
      float mb = M;
#pragma unroll
      for (int u = 0; u < B; ++u) mb = fmaxf(mb, mv[u]);  // clamped repeats leave the max unchanged
      if (mb > M) {
        const double r = double(expf(M - mb));
        L *= r;
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] *= r;
        M = mb;
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const bool in = c0 + u < nc;  // clamped repeats add nothing (selected, not multiplied by 0: inf rows stay inf)
        const double sc = double(expf(mv[u] - M));
        L = in ? L + double(lv[u]) * sc : L;
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = in ? acc[k] + double(v[u][k]) * sc : acc[k];
      }
    }
    const double den = L + 1e-10;
    if (a.stats && sub == 0) {
      a.stats[int64_t(row) * 2 * a.H + head] = M;
      a.stats[int64_t(row) * 2 * a.H + a.H + head] = float(den);
    }
    float r[K];
#pragma unroll
    for (int k = 0; k < K; ++k) r[k] = float(acc[k] / den);
    if (a.bias) {
      float b[K];
      vload<K>(b, a.bias + f);
#pragma unroll
      for (int k = 0; k < K; ++k) r[k] += b[k];
    }
    vstore<K>(a.out + int64_t(row) * a.ld_o + f, r);
  }
}



template <int K>
int launch(const GatArgs& a, hipStream_t s) {
  const int64_t work = a.items ? a.n_items : a.n_rows;
  if (work > 0) {
    auto k = gatv2_kernel<K>;
    hipLaunchKernelGGL(k, dim3(resident_grid(k, work, a.G)), dim3(kBlock), 0, s, a);
    KGX_CHECK_LAUNCH();
  }
  if (a.items && a.n_split > 0) {
    auto k = gatv2_fixup_kernel<K>;
    hipLaunchKernelGGL(k, dim3(resident_grid(k, a.n_split, a.G)), dim3(kBlock), 0, s, a);
    KGX_CHECK_LAUNCH();
  }
  return KGX_OK;
}

}  // namespace
}  // namespace kgx

using namespace kgx;

extern "C" int kgx_gatv2(const int32_t* rowptr, const int32_t* rows, int64_t n_rows, const int32_t* items,
                         int64_t n_items, const int32_t* split, int64_t n_split, const int32_t* col,
                         const float* h_src, const float* h_dst, int64_t ld_h, const float* att, int heads,
                         int channels, float negative_slope, float* out, int64_t ld_out, const float* bias,
                         float* partials, float* stats, const int32_t* drop_key, float drop_p,
                         uint64_t drop_seed, kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(heads > 0 && channels > 0 && n_rows >= 0 && n_items >= 0 && n_split >= 0, KGX_ERR_ARG,
              "kgx_gatv2: bad sizes");
  if (n_rows == 0) return KGX_OK;
  const int64_t HC = int64_t(heads) * channels;
  KGX_REQUIRE(rowptr && rows && col && h_src && h_dst && att && out, KGX_ERR_ARG, "kgx_gatv2: null pointer");
  KGX_REQUIRE(ld_h >= HC && ld_out >= HC, KGX_ERR_ARG, "kgx_gatv2: leading dimension < heads*channels");
  KGX_REQUIRE(ld_h < (int64_t(1) << 31), KGX_ERR_ARG, "kgx_gatv2: leading dimension >= 2^31");
  const bool use_items = items != nullptr;
  KGX_REQUIRE(!use_items || n_split == 0 || (split && partials), KGX_ERR_ARG,
              "kgx_gatv2: split rows need split list and partials");
  auto al = [](const void* p, int b) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % b == 0; };
  // channels per lane: 8 first (C3, 8 heads x 16: two lanes per head, four rows
  // per wave -- 0.94 ms against 1.13 at K = 4 and 0.98 at K = 16, measured
  // interleaved; more rows per wave in flight, one DPP step per score), then 4, 16
  int K = 1;
  const int cands[3] = {8, 4, 16};
  bool found = false;
  const bool vec4 = !(ld_h % 4 || ld_out % 4 || !al(h_src, 16) || !al(h_dst, 16) || !al(out, 16) || !al(att, 16) ||
                      !al(bias, 16) || !al(partials, 16));
  for (int ci = 0; ci < 3 && !found && vec4; ++ci) {
    const int k = cands[ci];
    if (channels % k) continue;
    if (heads * next_pow2(channels / k) <= 64) {
      K = k;
      found = true;
    }
  }
  if (!found) {
    K = (channels % 2 == 0 && ld_h % 2 == 0 && ld_out % 2 == 0 && al(h_src, 8) && al(h_dst, 8) && al(out, 8) &&
         al(att, 8) && al(bias, 8) && al(partials, 8))
            ? 2
            : 1;
    if (heads * next_pow2((channels + K - 1) / K) > 64) K = 0;
  }
  KGX_REQUIRE(K > 0, KGX_ERR_UNSUPPORTED,
              "kgx_gatv2: heads=%d x channels=%d needs more than 64 lanes per row (unsupported shape)", heads,
              channels);
  {  // experiment knob (A/B only): KGX_GAT_K = channels per lane, if the shape allows it
    static const int kf = [] {
      const char* h = getenv("KGX_GAT_K");
      return h ? atoi(h) : 0;
    }();
    if (found && (kf == 4 || kf == 8 || kf == 16) && channels % kf == 0 && heads * next_pow2(channels / kf) <= 64)
      K = kf;  // same lane budget as the automatic choice
  }
  GatArgs a{};
  a.rowptr = rowptr;
  a.rows = rows;
  a.n_rows = n_rows;
  a.items = use_items ? reinterpret_cast<const int4*>(items) : nullptr;
  a.n_items = use_items ? n_items : 0;
  a.split = reinterpret_cast<const int4*>(split);
  a.n_split = use_items ? n_split : 0;
  a.col = col;
  a.h_src = h_src;
  a.h_dst = h_dst;
  a.ld_h = ld_h;
  a.att = att;
  a.H = heads;
  a.C = channels;
  a.slope = negative_slope;
  a.out = out;
  a.ld_o = ld_out;
  a.bias = bias;
  a.partials = partials;
  a.stats = stats;
  KGX_REQUIRE(drop_p >= 0.0f && drop_p < 1.0f, KGX_ERR_ARG, "kgx_gatv2: dropout p must be in [0, 1)");
  if (drop_key && drop_p > 0.0f) {
    a.drop_key = drop_key;
    a.drop_seed = drop_seed;
    a.drop_thresh = uint32_t(double(drop_p) * 4294967296.0);
    a.drop_scale = 1.0f / (1.0f - drop_p);
  }
  a.LH = next_pow2((channels + K - 1) / K);
  a.lgLH = log2i(a.LH);
  a.G = next_pow2(heads * a.LH);
  a.lgG = log2i(a.G);
  switch (K) {
    case 1: return launch<1>(a, stream);
    case 2: return launch<2>(a, stream);
    case 4: return launch<4>(a, stream);
    case 8: return launch<8>(a, stream);
    default: return launch<16>(a, stream);
  }
}

// ===========================================================================
// Backward (kgx_gatv2_backward).  Forward per destination row i, head h:
//   z_e = h_dst[i] + h_src[j_e];  s_e = sum_c att[c] lrelu(z_e[c]);
//   alpha_e = exp(s_e - m) / (sum_e' exp(s_e' - m) + 1e-10);
//   out_i = sum_e alpha_e h_src[j_e]  (+ bias)
// With G = d loss / d out (the max shift m carries a ~1e-10-relative term
// through the 1e-10 guard, ignored):
//   dalpha_e = <G_i, h_src[j_e]>_h;  ds_e = alpha_e (dalpha_e - D_i)
//   D_i      = sum_e alpha_e dalpha_e = <G_i, out_i - bias>_h   (no pass over edges)
//   dz_e[c]  = ds_e att[c] lrelu'(z_e[c])          (lrelu'(0) = slope, as torch)
//   d att[c] = sum_e ds_e lrelu(z_e[c]);  d h_dst[i] = sum_e dz_e
//   d h_src[j] = sum_{e: j_e = j} (alpha_e G_i + dz_e)
// The forward keeps (m, denominator) per row and head (kgx_gatv2 `stats`), so
// kernel A is ONE pass over a row's edges, and needs only row constants: hub
// rows are split into the forward's chunks (partial d h_dst rows + fix-up).
// Kernel A stores alpha and ds per (edge, head); kernel B walks the
// TRANSPOSED CSR (its own split schedule) and pulls d h_src -- no atomics
// except the H*C-float d att.
// ===========================================================================

namespace kgx {
namespace {

struct GatBwdArgs {
  // destination CSR + its schedule
  const int32_t* rowptr;
  const int32_t* rows;
  int64_t n_rows;
  const int4* items;
  int64_t n_items;
  const int4* split;
  int64_t n_split;
  const int32_t* col;
  const float* h_src;
  const float* h_dst;
  int64_t ld_h;
  const float* att;
  int H, C;
  float slope;
  const float* out;  // forward output (bias included if bias != null)
  int64_t ld_out;
  const float* bias;
  const float* stats;  // [n, 2H] from the forward
  const int32_t* drop_key;  // attention dropout keys per CSR slot (or null)
  uint64_t drop_seed;
  uint32_t drop_thresh;
  float drop_scale;
  const float* grad;
  int64_t ld_g;
  float* alpha;  // [E', H] CSR slot order
  float* ds;     // [E', H]
  float* grad_h_dst;
  int64_t ld_gd;
  float* grad_att;  // [H*C], atomically accumulated
  float* partials;  // [max(n_slots, t_n_slots), H*C]
  // transposed graph + its schedule (kernel B)
  const int32_t* t_rowptr;
  const int32_t* t_rows;
  int64_t t_n_rows;
  const int4* t_items;
  int64_t t_n_items;
  const int4* t_split;
  int64_t t_n_split;
  const int32_t* t_col;   // destination row of each transposed slot
  const int32_t* t_slot;  // forward CSR slot of each transposed slot
  float* grad_h_src;
  int64_t ld_gs;
  int G, lgG, LH, lgLH;
};

template <int K>
constexpr int bwd_unroll() {
  return K <= 4 ? 8 : 4;
}

__device__ __forceinline__ void work_item(const int4* items, const int32_t* rows, const int32_t* rowptr, int64_t it,
                                          int32_t& row, int32_t& beg, int32_t& end, int32_t& slot) {
  if (items) {
    const int4 v = items[it];
    row = v.x;
    beg = v.y;
    end = v.z;
    slot = v.w;
  } else {
    row = rows[it];
    beg = rowptr[row];
    end = rowptr[row + 1];
    slot = -1;
  }
}

template <int K>
__global__ __launch_bounds__(kBlock) void gatv2_bwd_rows_kernel(GatBwdArgs a) {
  constexpr int U = bwd_unroll<K>();
  const int G = a.G;
  const int lane = threadIdx.x & (G - 1);
  const int head = lane >> a.lgLH;
  const int sub = lane & (a.LH - 1);
  const bool valid = head < a.H && sub * K < a.C;
  const int f = valid ? head * a.C + sub * K : 0;  // padding lanes read a valid address and use nothing
  const int HC = a.H * a.C;
  const int64_t ngroups = (int64_t(gridDim.x) * kBlock) >> a.lgG;
  const int64_t n_work = a.items ? a.n_items : a.n_rows;
  float att[K], gatt[K];
  vload<K>(att, a.att + f);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    gatt[k] = 0.0f;
    if (!valid) att[k] = 0.0f;
  }
  auto lrelu = [&](float g) { return g > 0.0f ? g : g * a.slope; };
  for (int64_t it = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> a.lgG; it < n_work; it += ngroups) {
    int32_t row, beg, end, slot;
    work_item(a.items, a.rows, a.rowptr, it, row, beg, end, slot);
    float hd[K], gr[K], o[K];
    vload<K>(hd, a.h_dst + int64_t(row) * a.ld_h + f);
    vload<K>(gr, a.grad + int64_t(row) * a.ld_g + f);
    vload<K>(o, a.out + int64_t(row) * a.ld_out + f);
    if (a.bias) {
      float b[K];
      vload<K>(b, a.bias + f);
#pragma unroll
      for (int k = 0; k < K; ++k) o[k] -= b[k];
    }
    if (!valid) {
#pragma unroll
      for (int k = 0; k < K; ++k) gr[k] = 0.0f;
    }
    float dp = 0.0f;
#pragma unroll
    for (int k = 0; k < K; ++k) dp += gr[k] * o[k];
    const float D = head_reduce<K>(dp, a.LH);
    const float m = a.stats[int64_t(row) * 2 * a.H + (valid ? head : 0)];
    const float den = a.stats[int64_t(row) * 2 * a.H + a.H + (valid ? head : 0)];
    float gd[K];
#pragma unroll
    for (int k = 0; k < K; ++k) gd[k] = 0.0f;
    for (int32_t e = beg; e < end; e += U) {
      float hs[U][K];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int32_t ee = e + u < end ? e + u : end - 1;
        vload<K>(hs[u], a.h_src + row_off(a.col[ee], a.ld_h) + f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float ps = 0.0f, pa = 0.0f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          ps += lrelu(hd[k] + hs[u][k]) * att[k];
          pa += gr[k] * hs[u][k];
        }
        const float sc = head_reduce<K>(ps, a.LH);
        const float da = head_reduce<K>(pa, a.LH);
        if (e + u < end) {
          const float al = __fdiv_rn(expf(sc - m), den);
          // dropout: out = sum alpha*d*h, so d alpha = d * <G, h>; D = <G, out - b> already includes d
          const float dmu = a.drop_key ? drop_scale(a.drop_seed, uint32_t(a.drop_key[e + u]), uint32_t(head),
                                                    a.drop_thresh, a.drop_scale)
                                       : 1.0f;
          const float dsv = al * (dmu * da - D);
#pragma unroll
          for (int k = 0; k < K; ++k) {
            const float g = hd[k] + hs[u][k];
            gd[k] += dsv * att[k] * (g > 0.0f ? 1.0f : a.slope);
            gatt[k] += dsv * lrelu(g);
          }
          if (valid && sub == 0) {
            a.alpha[int64_t(e + u) * a.H + head] = al * dmu;  // the message weight kernel B pulls with
            a.ds[int64_t(e + u) * a.H + head] = dsv;
          }
        }
      }
    }
    if (!valid) continue;
    if (slot >= 0) vstore<K>(a.partials + int64_t(slot) * HC + f, gd);
    else vstore<K>(a.grad_h_dst + int64_t(row) * a.ld_gd + f, gd);
  }
  if (valid) {
#pragma unroll
    for (int k = 0; k < K; ++k) atomicAdd(a.grad_att + f + k, gatt[k]);
  }
}

template <int K>
__global__ __launch_bounds__(kBlock) void gatv2_bwd_src_kernel(GatBwdArgs a) {
  constexpr int U = bwd_unroll<K>();
  const int G = a.G;
  const int lane = threadIdx.x & (G - 1);
  const int head = lane >> a.lgLH;
  const int sub = lane & (a.LH - 1);
  const bool valid = head < a.H && sub * K < a.C;
  const int HC = a.H * a.C;
  const int64_t ngroups = (int64_t(gridDim.x) * kBlock) >> a.lgG;
  const int64_t n_work = a.t_items ? a.t_n_items : a.t_n_rows;
  if (!valid) return;  // no cross-lane work in this kernel
  const int f = head * a.C + sub * K;
  float att[K];
  vload<K>(att, a.att + f);
  for (int64_t it = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> a.lgG; it < n_work; it += ngroups) {
    int32_t j, beg, end, slot;
    work_item(a.t_items, a.t_rows, a.t_rowptr, it, j, beg, end, slot);
    float hs[K], acc[K];
    vload<K>(hs, a.h_src + int64_t(j) * a.ld_h + f);
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0f;
    for (int32_t e = beg; e < end; e += U) {
      float gr[U][K], hd[U][K], al[U], dsv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int32_t ee = e + u < end ? e + u : end - 1;
        const int32_t i = a.t_col[ee];
        const int32_t s = a.t_slot[ee];
        al[u] = a.alpha[row_off(s, a.H) + head];
        dsv[u] = a.ds[row_off(s, a.H) + head];
        vload<K>(gr[u], a.grad + row_off(i, a.ld_g) + f);
        vload<K>(hd[u], a.h_dst + row_off(i, a.ld_h) + f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (e + u < end) {
#pragma unroll
          for (int k = 0; k < K; ++k) {
            const float g = hd[u][k] + hs[k];
            acc[k] += al[u] * gr[u][k] + dsv[u] * att[k] * (g > 0.0f ? 1.0f : a.slope);
          }
        }
      }
    }
    if (slot >= 0) vstore<K>(a.partials + int64_t(slot) * HC + f, acc);
    else vstore<K>(a.grad_h_src + int64_t(j) * a.ld_gs + f, acc);
  }
}

// Sum the chunk partials of split rows in chunk order into out rows.
template <int K>
__global__ __launch_bounds__(kBlock) void gatv2_bwd_fixup_kernel(const int4* __restrict__ split, int64_t n_split,
                                                                 const float* __restrict__ partials, int HC,
                                                                 float* __restrict__ out, int64_t ld_out, int G,
                                                                 int lgG) {
  const int lane = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t(gridDim.x) * kBlock) >> lgG;
  for (int64_t it = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> lgG; it < n_split; it += ngroups) {
    const int4 sp = split[it];
    for (int f = lane; f < HC; f += G) {
      float acc = 0.0f;
      constexpr int B = 8;  // chunk loads in flight, then the in-order sum
      for (int32_t c0 = 0; c0 < sp.z; c0 += B) {
        float v[B];
#pragma unroll
        for (int u = 0; u < B; ++u) v[u] = partials[int64_t(sp.y + (c0 + u < sp.z ? c0 + u : sp.z - 1)) * HC + f];
#pragma unroll
        for (int u = 0; u < B; ++u) acc = c0 + u < sp.z ? acc + v[u] : acc;
      }
      out[int64_t(sp.x) * ld_out + f] = acc;
    }
  }
}

template <int K>
int launch_bwd(const GatBwdArgs& a, hipStream_t s) {
  const int HC = a.H * a.C;
  const int64_t work = a.items ? a.n_items : a.n_rows;
  if (work > 0) {
    auto k = gatv2_bwd_rows_kernel<K>;
    hipLaunchKernelGGL(k, dim3(resident_grid(k, work, a.G)), dim3(kBlock), 0, s, a);
    KGX_CHECK_LAUNCH();
  }
  if (a.items && a.n_split > 0) {
    hipLaunchKernelGGL(gatv2_bwd_fixup_kernel<K>, dim3(grid_for(a.n_split * 64, 4096)), dim3(kBlock), 0, s, a.split,
                       a.n_split, a.partials, HC, a.grad_h_dst, a.ld_gd, 64, 6);
    KGX_CHECK_LAUNCH();
  }
  const int64_t t_work = a.t_items ? a.t_n_items : a.t_n_rows;
  if (t_work > 0) {
    auto k = gatv2_bwd_src_kernel<K>;
    hipLaunchKernelGGL(k, dim3(resident_grid(k, t_work, a.G)), dim3(kBlock), 0, s, a);
    KGX_CHECK_LAUNCH();
  }
  if (a.t_items && a.t_n_split > 0) {
    hipLaunchKernelGGL(gatv2_bwd_fixup_kernel<K>, dim3(grid_for(a.t_n_split * 64, 4096)), dim3(kBlock), 0, s,
                       a.t_split, a.t_n_split, a.partials, HC, a.grad_h_src, a.ld_gs, 64, 6);
    KGX_CHECK_LAUNCH();
  }
  return KGX_OK;
}

}  // namespace
}  // namespace kgx

extern "C" int kgx_gatv2_backward(const int32_t* rowptr, const int32_t* rows, int64_t n_rows, const int32_t* items,
                                  int64_t n_items, const int32_t* split, int64_t n_split, const int32_t* col,
                                  const float* h_src, const float* h_dst, int64_t ld_h, const float* att, int heads,
                                  int channels, float negative_slope, const float* out, int64_t ld_out,
                                  const float* bias, const float* stats, const float* grad_out, int64_t ld_grad,
                                  const int32_t* t_rowptr, const int32_t* t_rows, int64_t n_src,
                                  const int32_t* t_items, int64_t t_n_items, const int32_t* t_split,
                                  int64_t t_n_split, const int32_t* t_col, const int32_t* t_slot,
                                  float* grad_h_src, float* grad_h_dst, int64_t ld_grad_h, float* grad_att,
                                  float* alpha_ws, float* ds_ws, float* partials, const int32_t* drop_key,
                                  float drop_p, uint64_t drop_seed, kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(heads > 0 && channels > 0 && n_rows >= 0 && n_src >= 0 && n_items >= 0 && n_split >= 0 &&
                  t_n_items >= 0 && t_n_split >= 0,
              KGX_ERR_ARG, "kgx_gatv2_backward: bad sizes");
  const int64_t HC = int64_t(heads) * channels;
  KGX_REQUIRE(rowptr && rows && col && h_src && h_dst && att && out && stats && grad_out && t_rowptr && t_rows &&
                  t_col && t_slot && grad_h_src && grad_h_dst && grad_att && alpha_ws && ds_ws,
              KGX_ERR_ARG, "kgx_gatv2_backward: null pointer");
  KGX_REQUIRE(ld_h >= HC && ld_grad >= HC && ld_grad_h >= HC && ld_out >= HC, KGX_ERR_ARG,
              "kgx_gatv2_backward: leading dimension < heads*channels");
  KGX_REQUIRE(ld_h < (int64_t(1) << 31) && ld_grad < (int64_t(1) << 31), KGX_ERR_ARG,
              "kgx_gatv2_backward: leading dimension >= 2^31");
  KGX_REQUIRE(((!items || n_split == 0) && (!t_items || t_n_split == 0)) || partials, KGX_ERR_ARG,
              "kgx_gatv2_backward: split rows need partials");
  // K channels per lane: the smallest K (dividing C, with aligned vector
  // accesses) that fits one row's heads into a 64-lane group
  auto al = [](const void* p, int b) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % b == 0; };
  int K = 0;
  for (int k = 1; k <= 16 && !K; k <<= 1) {
    const int va = 4 * (k < 4 ? k : 4);  // byte alignment vload<k> needs
    if (channels % k || ld_h % (va / 4) || ld_grad % (va / 4) || ld_grad_h % (va / 4) || ld_out % (va / 4)) continue;
    if (!al(h_src, va) || !al(h_dst, va) || !al(att, va) || !al(grad_out, va) || !al(grad_h_src, va) ||
        !al(grad_h_dst, va) || !al(out, va) || !al(bias, va) || !al(partials, va))
      continue;
    if (heads * next_pow2(channels / k) <= 64) K = k;
  }
  KGX_REQUIRE(K > 0, KGX_ERR_UNSUPPORTED,
              "kgx_gatv2_backward: heads=%d x channels=%d does not fit 64 lanes per row", heads, channels);
  GatBwdArgs a{};
  a.rowptr = rowptr;
  a.rows = rows;
  a.n_rows = n_rows;
  a.items = items ? reinterpret_cast<const int4*>(items) : nullptr;
  a.n_items = items ? n_items : 0;
  a.split = reinterpret_cast<const int4*>(split);
  a.n_split = items ? n_split : 0;
  a.col = col;
  a.h_src = h_src;
  a.h_dst = h_dst;
  a.ld_h = ld_h;
  a.att = att;
  a.H = heads;
  a.C = channels;
  a.slope = negative_slope;
  a.out = out;
  a.ld_out = ld_out;
  a.bias = bias;
  a.stats = stats;
  KGX_REQUIRE(drop_p >= 0.0f && drop_p < 1.0f, KGX_ERR_ARG, "kgx_gatv2_backward: dropout p must be in [0, 1)");
  if (drop_key && drop_p > 0.0f) {
    a.drop_key = drop_key;
    a.drop_seed = drop_seed;
    a.drop_thresh = uint32_t(double(drop_p) * 4294967296.0);
    a.drop_scale = 1.0f / (1.0f - drop_p);
  }
  a.grad = grad_out;
  a.ld_g = ld_grad;
  a.alpha = alpha_ws;
  a.ds = ds_ws;
  a.grad_h_dst = grad_h_dst;
  a.ld_gd = ld_grad_h;
  a.grad_att = grad_att;
  a.partials = partials;
  a.t_rowptr = t_rowptr;
  a.t_rows = t_rows;
  a.t_n_rows = n_src;
  a.t_items = t_items ? reinterpret_cast<const int4*>(t_items) : nullptr;
  a.t_n_items = t_items ? t_n_items : 0;
  a.t_split = reinterpret_cast<const int4*>(t_split);
  a.t_n_split = t_items ? t_n_split : 0;
  a.t_col = t_col;
  a.t_slot = t_slot;
  a.grad_h_src = grad_h_src;
  a.ld_gs = ld_grad_h;
  a.LH = next_pow2(channels / K);
  a.lgLH = log2i(a.LH);
  a.G = next_pow2(heads * a.LH);
  a.lgG = log2i(a.G);
  switch (K) {
    case 1: return launch_bwd<1>(a, stream);
    case 2: return launch_bwd<2>(a, stream);
    case 4: return launch_bwd<4>(a, stream);
    case 8: return launch_bwd<8>(a, stream);
    default: return launch_bwd<16>(a, stream);
  }
}
