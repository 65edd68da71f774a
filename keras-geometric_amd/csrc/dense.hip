// Dense node transform on MFMA for the kgx engine (gfx950, wave64).
//
//   out[i, :] (+)= ACT( bias + x0[i, :K0] @ W0 + x1[i, :K1] @ W1 )
//
// The dense half of the layers on the propagate path: GINConv's MLP Dense
// (gin_conv.py:129-162, applied at :225), SAGEConv's lin_self / lin_neigh pair
// (sage_conv.py:407-428; two terms = ONE pass over x and the aggregate),
// GATv2Conv's shared linear map (gatv2_conv.py:224-239) and GCNConv's X W when
// the fused aggregate->transform kernel does not apply.  The reference runs
// these as fp32 keras Dense / ops.matmul; here the product is taken on the
// bf16 matrix cores as the six significant cross products of a three-way bf16
// split of both operands (kgx_bf16x3.h: f32-accurate, IEEE inf/NaN), 16x the
// per-clock rate of f32-input MFMA.
//
// Tiling: a block of WAVES waves owns 32-row tiles of the output and 16 WAVES
// of its columns; for N > 128 two blocks on the same XCD take the two column
// halves of the same tiles (blocks b and b + 8 under the round-robin
// block->XCD dispatch), so x comes from HBM once and from that XCD's L2 the
// second time.  Wave w owns 16 output columns and keeps W's split fragments for
// them in registers for the whole kernel (K <= 256: 96 VGPRs), which leaves
// room for two waves per SIMD.  Per tile the block loads the 32 x K f32 rows
// (dwordx4, coalesced, two tiles ahead in registers), splits them into three
// bf16 planes in LDS (double-buffered; row stride = 32 mod 256 bytes, so the
// ds_read_b128 A-fragment reads are conflict-free), then every wave runs
// v_mfma_f32_16x16x32_bf16 over K for its columns and stores its 16x16 blocks
// with the bias / ReLU / accumulate epilogue.  One LDS barrier per tile.
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "kgx_bf16x3.h"
#include "kgx_internal.h"

namespace kgx {
namespace {

constexpr int kBM = 32;  // rows per tile

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops
// (lgkmcnt), not its outstanding global loads / stores (vmcnt).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct DenseArgs {
  int64_t M;
  const float* x0;
  int64_t ld0;
  int K0;
  const float* x1;
  int64_t ld1;
  int K1;
  const float* W0;  // [K0, N] row-major
  const float* W1;  // [K1, N] row-major
  int N;
  const float* bias;
  float* out;
  int64_t ld_out;
  int relu;
  int accumulate;
  int cg_count;  // column groups of 16 WAVES columns (1 or 2)
  int vec_out;   // N, ld_out multiples of 4 and out 16-byte aligned: dwordx4 output stores
  // Always 0 in this build.  They are kept as kernel arguments because the
  // producer pipeline's register allocation, hand-checked on the ISA
  // (tools/isa_hazard_check.py), is sensitive to the branches they guard:
  // removing them gave an allocation the checker rejects (a register set
  // reused while its loads were still in flight).
  int pstore;
  int debug;
};

template <int KS>
struct Geom {
  static constexpr int KP = 32 * KS;                                         // padded K
  static constexpr int ROWB = 2 * KP;                                        // bytes of one bf16 plane row
  static constexpr int STRIDE_B = ROWB + (((32 - ROWB) % 256) + 256) % 256;  // == 32 (mod 256)
  static constexpr int STRIDE = STRIDE_B / 2;                                // in bf16
  static constexpr int F4_PER_ROW = KP / 4;
  static constexpr int F4_PER_TILE = kBM * F4_PER_ROW;
};

// W element (k, n) of the stacked [W0; W1] (zero outside)
__device__ __forceinline__ float w_at(const DenseArgs& a, int k, int n) {
  if (n >= a.N) return 0.0f;
  if (k < a.K0) return a.W0[int64_t(k) * a.N + n];
  k -= a.K0;
  if (k < a.K1) return a.W1[int64_t(k) * a.N + n];
  return 0.0f;
}

constexpr int kProducerWaves = 4;

// WAVES consumer waves (MFMA + stores) and kProducerWaves producer waves
// (global loads -> bf16x3 split -> LDS planes).  The roles only meet at one
// workgroup barrier per tile: producers stage tile i+1 into one LDS buffer
// while consumers run tile i from the other.  Keeping the loads (and their
// vmcnt waits) in waves that issue no MFMA means a wait on a prefetch never
// stalls the matrix pipe, and the consumers' output stores never delay a
// prefetch wait.
//
// LS (non-accumulating form, vec_out): full-line output stores.  The 16x16
// MFMA result leaves each lane one column of four rows, so a wave's dword
// stores cover 64 B of a row per 128-B line (its neighbour wave writes the
// other half).  With LS the consumers park each finished tile in an LDS out
// tile (Os, double-buffered by tile parity) and, during the next tile's last
// k-step, every wave reads two whole-row float4 runs back and stores them with
// dwordx4: one wave instruction = two 512-B rows.
// PS: the opt-in producer-store experiment (KGX_DENSE_PSTORE); only LS and PS
// instantiations carry the LDS out tile.
template <int KS, int WAVES, bool ACC, bool TWO, bool LS = false, bool PS = false>
__global__ __launch_bounds__(64 * (WAVES + kProducerWaves)) void dense_kernel(DenseArgs a) {
  using G = Geom<KS>;
  constexpr int TP = 64 * kProducerWaves;
  static_assert(TP % G::F4_PER_ROW == 0, "producer load slots must tile whole rows");
  constexpr int NL = G::F4_PER_TILE / TP;  // float4 loads per producer thread per tile
  constexpr int RSTEP = TP / G::F4_PER_ROW;
  __shared__ short As[2][3][kBM][G::STRIDE];
  // output tile staged for the producers' stores (a.pstore), double-buffered by step parity
  constexpr int OCOLS = 16 * WAVES;
  constexpr int OSTRIDE = OCOLS + 4;  // floats; 4 mod 32 dwords between rows
  __shared__ float Os[2][(LS || PS) ? kBM : 1][(LS || PS) ? OSTRIDE : 1];
  __shared__ float Ob[LS ? OCOLS : 1];  // LS: this block's bias columns (read beside the out rows)

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: roles branch on SCC, not exec

  int cg = 0;
  int64_t pid = blockIdx.x, n_pairs = gridDim.x;
  if (a.cg_count == 2) {
    if (gridDim.x >= 16) {
      cg = (blockIdx.x >> 3) & 1;
      pid = (blockIdx.x & 7) | ((blockIdx.x >> 4) << 3);
    } else {
      cg = blockIdx.x & 1;
      pid = blockIdx.x >> 1;
    }
    n_pairs = gridDim.x / 2;
  }
  const int64_t n_tiles = (a.M + kBM - 1) / kBM;
  if (pid >= n_tiles) return;  // uniform per block
  // tiles of this block: pid, pid + n_pairs, ... (both roles run the same count)
  const int64_t my_tiles = (n_tiles - 1 - pid) / n_pairs + 1;

  if (wave >= WAVES) {
    // ---------------- producer ----------------
    // slot j of a thread covers columns [kk, kk + 4) of the stacked [x0 | x1]
    // row srow0 + j RSTEP.  Loads are raw buffer loads through a per-tile
    // descriptor whose record count ends at the tile's last valid row: rows
    // past M and K padding (offset 0x80000000) read as zero with no branch.
    // They are issued as inline asm with explicit partial waits: the two
    // register sets are always in flight in a fixed order, so staging one set
    // waits with vmcnt(LPS) (the other set's loads stay in flight), where the
    // compiler's own accounting would drain both (vmcnt(0)).
    constexpr int LPS = TWO ? 2 * NL : NL;  // loads per register set
    // register sets in flight: about 128 KB of x per CU (4 x 32 KB tiles at
    // K 256, 8 x 16 KB at K 128; half with two operands, whose sets take
    // twice the registers).  The loads are latency-bound, not bandwidth-bound,
    // below that: 64 KB per CU measured 3 TB/s.
    // K 256: three sets (four spilled address registers once the split took fewer VALU but more live values)
    constexpr int NSETS_ = KS == 8 ? 3 : (32 / KS < 2 ? 2 : (32 / KS > 8 ? 8 : 32 / KS));
    constexpr int NSETS = TWO ? (NSETS_ / 2 < 2 ? 2 : NSETS_ / 2) : NSETS_;
    const int ptid = tid - 64 * WAVES;
    const int kk = 4 * (ptid % G::F4_PER_ROW);
    const int srow0 = ptid / G::F4_PER_ROW;
    uint32_t vo0[NL], vo1[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int64_t row = srow0 + j * RSTEP;
      vo0[j] = kk < a.K0 ? uint32_t((row * a.ld0 + kk) * 4) : 0x80000000u;
      vo1[j] = (kk >= a.K0 && kk - a.K0 < a.K1) ? uint32_t((row * a.ld1 + (kk - a.K0)) * 4) : 0x80000000u;
    }
    // buffer descriptor {base lo, base hi (stride 0), bytes, config} in SGPRs
    auto rsrc = [&](const float* base, int64_t ld, int64_t tile) {
      const int64_t r0 = tile * kBM;
      int64_t rows = a.M - r0;
      rows = rows < 0 ? 0 : (rows > kBM ? kBM : rows);
      const uint64_t addr = reinterpret_cast<uint64_t>(base) + uint64_t(r0 * ld * 4);
      u32x4 d;
      d[0] = __builtin_amdgcn_readfirstlane(uint32_t(addr));
      d[1] = __builtin_amdgcn_readfirstlane(uint32_t(addr >> 32) & 0xffffu);
      d[2] = __builtin_amdgcn_readfirstlane(uint32_t(rows * ld * 4));
      d[3] = 0x00020000u;
      return d;
    };
    auto ld16 = [](f32x4& v, uint32_t off, const u32x4& d) {
      asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(d) : "memory");
    };
    f32x4 P[NSETS][NL], Q[NSETS][NL];  // register sets (Q: x1 columns)
    auto load_tile = [&](f32x4(&p)[NL], f32x4(&q)[NL], int64_t tile) {
      const u32x4 d0 = rsrc(a.x0 ? a.x0 : a.x1, a.ld0, tile);
#pragma unroll
      for (int j = 0; j < NL; ++j) ld16(p[j], vo0[j], d0);
      if constexpr (TWO) {
        const u32x4 d1 = rsrc(a.x1, a.ld1, tile);
#pragma unroll
        for (int j = 0; j < NL; ++j) ld16(q[j], vo1[j], d1);
      }
    };
    // wait until at most `newer` loads are outstanding, then pin the set's
    // registers behind the wait (the empty asm "redefines" them)
    auto wait_set = [&](f32x4(&p)[NL], f32x4(&q)[NL], auto newer) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(newer)::value) : "memory");
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        asm volatile("" : "+v"(p[j]));
        if constexpr (TWO) asm volatile("" : "+v"(q[j]));
      }
    };
    auto stage = [&](const f32x4(&p)[NL], const f32x4(&q)[NL], int buf) {
      // fast path: paired conversions (split3_pair_rn, ~4.5 VALU per element:
      // the producer's split must fit in the issue slots the consumers' MFMAs
      // leave free on its SIMD).  chk = sum of 2|x| over the thread's slots
      // (|x| is a free source modifier of v_fma_f32): a sum of non-negative
      // terms, so it is non-finite whenever one element is inf / NaN or
      // >= 2^127 (where bf16(x) could round to inf) -- no cancellation can hide
      // one -- and the slots are then redone with split3_a_lo below.
      float chk0 = 0.0f, chk1 = 0.0f;
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        const int row = srow0 + j * RSTEP;
        f32x4 x = p[j];
        if constexpr (TWO)
          x = __builtin_bit_cast(f32x4, __builtin_bit_cast(u32x4, p[j]) | __builtin_bit_cast(u32x4, q[j]));
        chk0 = fmaf(fabsf(x[0]), 2.0f, chk0);
        chk1 = fmaf(fabsf(x[1]), 2.0f, chk1);
        chk0 = fmaf(fabsf(x[2]), 2.0f, chk0);
        chk1 = fmaf(fabsf(x[3]), 2.0f, chk1);
        uint32_t h0, m0, l0, h1, m1, l1;
        split3_pair_rn(x[0], x[1], h0, m0, l0);
        split3_pair_rn(x[2], x[3], h1, m1, l1);
        *reinterpret_cast<uint2*>(&As[buf][0][row][kk]) = make_uint2(h0, h1);
        *reinterpret_cast<uint2*>(&As[buf][1][row][kk]) = make_uint2(m0, m1);
        *reinterpret_cast<uint2*>(&As[buf][2][row][kk]) = make_uint2(l0, l1);
      }
      if (__builtin_expect(__builtin_isfinite(chk0 + chk1), 1)) return;
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        const int row = srow0 + j * RSTEP;
        f32x4 x = p[j];
        if constexpr (TWO)  // each slot read zero bits from one of the two descriptors
          x = __builtin_bit_cast(f32x4, __builtin_bit_cast(u32x4, p[j]) | __builtin_bit_cast(u32x4, q[j]));
        bf16x4_t ph, pm, pl;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          short h, m, lo;
          split3_a(x[e], h, m, lo);
          ph[e] = h;
          pm[e] = m;
          pl[e] = lo;
        }
        // inf / NaN or a magnitude bf16 rounds to inf among the four: split3_a_lo (rare)
        if (!split_fast_ok(x[0], x[1], x[2], x[3])) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            short h, m, lo;
            split3_a_lo(x[e], h, m, lo);
            ph[e] = h;
            pm[e] = m;
            pl[e] = lo;
          }
        }
        *reinterpret_cast<bf16x4_t*>(&As[buf][0][row][kk]) = ph;
        *reinterpret_cast<bf16x4_t*>(&As[buf][1][row][kk]) = pm;
        *reinterpret_cast<bf16x4_t*>(&As[buf][2][row][kk]) = pl;
      }
    };
    // Producer-side output stores (a.pstore): the consumers leave each finished
    // 32-row tile in LDS (Os) and the producers store it during the next step
    // as whole-row dwordx4 runs with the bias / ReLU epilogue, so the MFMA waves
    // issue no global stores (their stores at the tile end did not overlap the
    // MFMAs: 1.3 ms of the C4 shape's 7.1).  Every step issues NST stores
    // (out-of-range, so dropped, where there is no tile to store yet), which
    // keeps the vmcnt count of the prefetch waits a constant.
    constexpr int OC4 = OCOLS / 4;         // float4 per out-tile row
    constexpr int NST = kBM * OC4 / TP;    // out-tile float4 per producer thread
    constexpr int PRSTEP = TP / OC4;       // out-tile rows between a thread's float4s
    static_assert(NST * TP == kBM * OC4, "producer store slots must tile the out tile");
    const int pc4 = ptid % OC4;
    const int prow0 = ptid / OC4;
    const int ocol = cg * OCOLS + 4 * pc4;
    float ob4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) ob4[j] = (PS && a.bias && ocol + j < a.N) ? a.bias[ocol + j] : 0.0f;
    auto store_out = [&](int64_t step) {  // step < 0: dummy stores (dropped)
      const int64_t tile = pid + (step < 0 ? 0 : step) * n_pairs;
      const int64_t r0 = tile * kBM;
      int64_t rows = a.M - r0;
      rows = step < 0 ? 0 : (rows < 0 ? 0 : (rows > kBM ? kBM : rows));
      const uint64_t addr = reinterpret_cast<uint64_t>(a.out) + uint64_t(r0 * a.ld_out * 4);
      const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(addr));
      const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(addr >> 32));
      const int bytes = __builtin_amdgcn_readfirstlane(int(rows * a.ld_out * 4));
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t(hi) << 32) | lo), 0,
                                                        bytes, 0x00020000);
      const int ob = int((step < 0 ? 0 : step) & 1);
#pragma unroll
      for (int m = 0; m < NST; ++m) {
        const int row = prow0 + m * PRSTEP;
        f32x4 v = *reinterpret_cast<const f32x4*>(&Os[ob][row][4 * pc4]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = v[j] + ob4[j];
          if (a.relu) v[j] = fmaxf(v[j], 0.0f);
        }
        const uint32_t off = ocol < a.N ? uint32_t((row * a.ld_out + ocol) * 4) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, off, 0, 0);
      }
    };
    using Zero = std::integral_constant<int, 0>;
    using Others = std::integral_constant<int, (NSETS - 1) * LPS>;
    using OthersP = std::integral_constant<int, (NSETS - 1) * (LPS + NST)>;
    static_assert((NSETS - 1) * (LPS + NST) <= 63, "vmcnt immediate");
    if (a.debug & 4) {  // experiment: no loads, no split -- the consumers' time alone
      for (int64_t i = 0; i <= my_tiles; ++i) lds_barrier();
      return;
    }
    // two operands hold two register sets per slot: no registers left for the store path
    constexpr bool pstore = PS && !TWO && !ACC;
    int64_t t = pid;
    load_tile(P[0], Q[0], t);
    wait_set(P[0], Q[0], Zero{});
    stage(P[0], Q[0], 0);
#pragma unroll
    for (int k = 0; k < NSETS; ++k) {
      if (pstore) store_out(-1);
      load_tile(P[k], Q[k], t + (k + 1) * n_pairs);
    }
    lds_barrier();
    // step i (tile i of this block): consumers run tile i from buffer i & 1;
    // producers stage tile i + 1 (register set i % NSETS) into the other
    // buffer and refill that set with tile i + 1 + NSETS.  Outstanding loads,
    // oldest first, are the sets in cyclic order, so a set's wait leaves the
    // other NSETS - 1 sets in flight.
    // The last step leaves both loops straight to the epilogue (goto), so the
    // loop's back edge is taken only after all NSETS steps issued their loads:
    // every path into a step's wait has the same loads outstanding (what the
    // counted waits assume; tools/isa_hazard_check.py proves it on the ISA).
    for (int64_t i = 0; i < my_tiles; i += NSETS, t += NSETS * n_pairs) {
#pragma unroll
      for (int k = 0; k < NSETS; ++k) {
        if (pstore) wait_set(P[k], Q[k], OthersP{});
        else wait_set(P[k], Q[k], Others{});
        stage(P[k], Q[k], int((i + k + 1) & 1));
        if (pstore) store_out(i + k - 1);  // the tile the consumers finished at the last barrier
        load_tile(P[k], Q[k], t + (k + 1 + NSETS) * n_pairs);
        lds_barrier();
        if (i + k + 1 >= my_tiles) goto producer_done;
      }
    }
  producer_done:
    // The last steps' prefetches (tiles past the end, read as zeros) are still
    // landing in the now-dead sets, and hipcc, which cannot see inline asm's
    // loads as pending, hands dead registers to store_out's values: so wait for
    // them first, and fence the scheduler so none of store_out's arithmetic is
    // hoisted above the wait (tools/isa_hazard_check.py found both: store_out
    // after the loop, and its row address computed above a bare wait).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (pstore) store_out(my_tiles - 1);
    return;
  }

  // ---------------- consumer ----------------
  const int l = tid & 63;
  const int lr = l & 15;  // fragment row / column
  const int lq = l >> 4;  // fragment k-chunk / row quad
  const int n_col = cg * 16 * WAVES + wave * 16 + lr;  // this lane's output column

  // W's split fragments for this wave's columns: lane holds B[k = 32 s + 8 lq + j][n_col]
  bf16x8_t wh[KS], wm[KS], wl[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      short h, m, lo;
      split3_a(w_at(a, 32 * s + 8 * lq + j, n_col), h, m, lo);
      wh[s][j] = h;
      wm[s][j] = m;
      wl[s][j] = lo;
    }
  const float bcol = (a.bias && n_col < a.N) ? a.bias[n_col] : 0.0f;
  // byte offset of this lane's first output element within a tile (row 4 lq, column n_col);
  // out-of-range for columns past N, so their stores are dropped
  const uint32_t out_lane = n_col < a.N ? uint32_t((4 * lq * a.ld_out + n_col) * 4) : 0x80000000u;
  if constexpr (LS) {
    if (wave == 0)
      for (int c = l; c < OCOLS; c += 64) Ob[c] = (a.bias && cg * OCOLS + c < a.N) ? a.bias[cg * OCOLS + c] : 0.0f;
  }
  lds_barrier();

  // LS: out-tile float4 q = 128 wave + 64 m + l (m = 0, 1) -> row q / OC4, float4 column l % OC4
  constexpr int OC4L = OCOLS / 4;
  const int lc4 = l % OC4L;
  const int lrow0 = (wave * 128 + l) / OC4L;
  constexpr int LROWS = 64 / OC4L;  // rows between a lane's two float4
  const int locol = cg * OCOLS + 4 * lc4;
  const uint32_t lo_off = locol < a.N ? uint32_t((lrow0 * a.ld_out + locol) * 4) : 0x80000000u;
  auto tile_rsrc_ls = [&](int64_t tile) {  // rows past M fall outside the record count
    const int64_t r0 = tile * kBM;
    int64_t rows = a.M - r0;
    rows = rows > kBM ? kBM : rows;
    const uint64_t addr = reinterpret_cast<uint64_t>(a.out) + uint64_t(r0 * a.ld_out * 4);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(addr));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(addr >> 32));
    const int bytes = __builtin_amdgcn_readfirstlane(int(rows * a.ld_out * 4));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t(hi) << 32) | lo), 0, bytes,
                                             0x00020000);
  };
  auto lprev_rs = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, 0, 0x00020000);  // zero records: first tile's stores dropped
  f32x4 lov[2], lb4;
  auto lstore_prev = [&]() {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      f32x4 v = lov[m];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = v[j] + lb4[j];
        if (a.relu) v[j] = fmaxf(v[j], 0.0f);
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), lprev_rs, lo_off,
                                             int(m * LROWS * a.ld_out * 4), 0);
    }
  };

  int64_t t = pid;
  for (int64_t i = 0; i < my_tiles; ++i, t += n_pairs) {
    const int buf = int(i & 1);
    f32x4 acc[2];
    acc[0] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    acc[1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    // A fragments are software-pipelined one k-step ahead: the six LDS reads
    // of step s + 1 are issued (inline asm, so the scheduler cannot sink them
    // next to their use) before step s's 12 MFMAs, and step s waits with
    // lgkmcnt(6), leaving step s + 1's reads in flight.  The empty asm after
    // each wait pins the fragments (and the accumulators, which orders the
    // MFMAs of step s before the wait of step s + 1).
    struct Frags {
      bf16x8_t h[2], m[2], l[2];
    };
    const uint32_t lds_lane = uint32_t(reinterpret_cast<uintptr_t>(&As[buf][0][lr][8 * lq]));
    auto read_frags = [](Frags& f, auto S, uint32_t lane) {
      constexpr int s = decltype(S)::value;
      constexpr uint32_t P = uint32_t(kBM) * G::STRIDE * 2;  // bytes per plane
      constexpr uint32_t R = 16u * G::STRIDE * 2;            // bytes per 16 rows
      constexpr uint32_t K = 64u * s;                        // 32 bf16 per k-step
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.h[r]) : "v"(lane), "i"(0 * P + R * r + K));
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.m[r]) : "v"(lane), "i"(1 * P + R * r + K));
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.l[r]) : "v"(lane), "i"(2 * P + R * r + K));
      }
    };
    auto wait_frags = [](Frags& f, f32x4(&acc)[2], auto N) {
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(decltype(N)::value) : "memory");
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        asm volatile("" : "+v"(f.h[r]), "+v"(f.m[r]), "+v"(f.l[r]), "+v"(acc[r]));
      }
    };
    Frags fa, fb;
    if (!(a.debug & 1)) {
      read_frags(fa, std::integral_constant<int, 0>{}, lds_lane);
      auto step = [&](auto S) {
        constexpr int s = decltype(S)::value;
        Frags& cur = (s & 1) ? fb : fa;
        Frags& nxt = (s & 1) ? fa : fb;
        if constexpr (LS && s == KS - 1) {  // the previous tile's out rows (last k-step: no next-step fragments live; its lgkmcnt(0) covers them)
          const uint32_t ob = uint32_t(reinterpret_cast<uintptr_t>(&Os[buf ^ 1][lrow0][4 * lc4]));
          asm volatile("ds_read_b128 %0, %1" : "=v"(lov[0]) : "v"(ob));
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(lov[1]) : "v"(ob), "i"(LROWS * OSTRIDE * 4));
          asm volatile("ds_read_b128 %0, %1" : "=v"(lb4) : "v"(uint32_t(reinterpret_cast<uintptr_t>(&Ob[4 * lc4]))));
        }
        if constexpr (s + 1 < KS) {
          read_frags(nxt, std::integral_constant<int, s + 1>{}, lds_lane);
          wait_frags(cur, acc, std::integral_constant<int, 6>{});
        } else {
          wait_frags(cur, acc, std::integral_constant<int, 0>{});
        }
        if constexpr (LS && s == KS - 1) asm volatile("" : "+v"(lov[0]), "+v"(lov[1]), "+v"(lb4));
        // small terms first; two independent accumulator chains (row tiles).
        // (Measured and not kept: D = W^T x^T, a lane holding 4 consecutive
        // columns of one row for one dwordx4 store per block, 1-6 % slower:
        // C4 7.12 vs 7.02 ms, NS 2.24 vs 2.12.)
#define KGX_MF(X, W, ACC_) __builtin_amdgcn_mfma_f32_16x16x32_bf16(X, W, ACC_, 0, 0, 0)
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r] = KGX_MF(cur.l[r], wh[s], acc[r]);
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r] = KGX_MF(cur.h[r], wl[s], acc[r]);
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r] = KGX_MF(cur.m[r], wm[s], acc[r]);
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r] = KGX_MF(cur.m[r], wh[s], acc[r]);
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r] = KGX_MF(cur.h[r], wm[s], acc[r]);
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r] = KGX_MF(cur.h[r], wh[s], acc[r]);
#undef KGX_MF
        if constexpr (LS && s == KS - 1) lstore_prev();
      };
      [&]<int... S>(std::integer_sequence<int, S...>) {
        (step(std::integral_constant<int, S>{}), ...);
      }(std::make_integer_sequence<int, KS>{});
    }
    // Raw buffer stores through a per-tile descriptor: rows past M fall
    // outside its record count and columns past N carry an out-of-range
    // offset, so both are dropped by the range check (no branches).
    if constexpr (LS) {
      // this tile into the LDS out tile (stored during the next tile); lane holds rows 4 lq + j of column lr
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) Os[buf][16 * r + 4 * lq + j][wave * 16 + lr] = acc[r][j];
      lprev_rs = tile_rsrc_ls(t);
    } else if constexpr (PS && !TWO && !ACC) {
      // lane holds rows 4 lq + j of column lr of each 16x16 block: into the LDS
      // out tile for the producers' stores (bias / ReLU applied there)
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) Os[buf][16 * r + 4 * lq + j][wave * 16 + lr] = acc[r][j];
    } else if (!(a.debug & 2)) {
      const int64_t r0 = t * kBM;
      int64_t rows = a.M - r0;
      rows = rows > kBM ? kBM : rows;
      const uint64_t addr = reinterpret_cast<uint64_t>(a.out) + uint64_t(r0 * a.ld_out * 4);
      const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(addr));
      const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(addr >> 32));
      const int bytes = __builtin_amdgcn_readfirstlane(int(rows * a.ld_out * 4));
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t(hi) << 32) | lo), 0,
                                                        bytes, 0x00020000);
      // lane holds rows 4 lq + j of column lr of each 16x16 block (soffset = the row)
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int soff = int((16 * r + j) * a.ld_out * 4);
          float v = acc[r][j] + bcol;
          if constexpr (ACC)
            v = __fadd_rn(__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, out_lane, soff, 0)), v);
          if (a.relu) v = fmaxf(v, 0.0f);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rs, out_lane, soff, 0);
        }
    }
    lds_barrier();  // buffer `buf` free for the producers; the stores stay in flight
  }
  if constexpr (LS) {  // the last tile's rows (written before the last barrier)
    const int lb = int((my_tiles - 1) & 1);
#pragma unroll
    for (int m = 0; m < 2; ++m) lov[m] = *reinterpret_cast<const f32x4*>(&Os[lb][lrow0 + m * LROWS][4 * lc4]);
    lb4 = *reinterpret_cast<const f32x4*>(&Ob[4 * lc4]);
    lstore_prev();
  }
}

template <int KS, int WAVES>
int launch(const DenseArgs& a, hipStream_t s) {
  auto k = a.accumulate ? (a.K1 > 0 ? dense_kernel<KS, WAVES, true, true> : dense_kernel<KS, WAVES, true, false>)
                        : (a.K1 > 0 ? dense_kernel<KS, WAVES, false, true> : dense_kernel<KS, WAVES, false, false>);
  // K > 128 only: measured C4 (K 256) 6.91 -> 6.66 ms, C5 (K 200) 0.90 -> 0.86 ms, but the
  // 10M x 128 -> 128 shape 2.13 -> 2.18 ms (half the MFMA time per tile to hide the extra LDS traffic)
  if constexpr (KS == 8) {
    if (!a.accumulate && a.vec_out && !a.pstore && a.debug == 0)
      k = a.K1 > 0 ? dense_kernel<KS, WAVES, false, true, true> : dense_kernel<KS, WAVES, false, false, true>;
  }
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 64 * (WAVES + kProducerWaves), 0) != hipSuccess ||
      per_cu <= 0)
    per_cu = 1;
  const int64_t n_tiles = (a.M + kBM - 1) / kBM;
  const int64_t cap = int64_t(per_cu) * cus;
  const int64_t want = n_tiles * a.cg_count;
  int64_t grid = want < cap ? want : cap;
  if (a.cg_count == 2) grid = grid >= 16 ? grid / 16 * 16 : grid / 2 * 2;  // whole XCD pairs
  hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(64 * (WAVES + kProducerWaves)), 0, s, a);
  KGX_CHECK_LAUNCH();
  return KGX_OK;
}

// K padded to 32, 64, 128 or 256 (whole rows per load slot; see load_tile)
template <int WAVES>
int launch_ks(int K, const DenseArgs& a, hipStream_t s) {
  if (K <= 32) return launch<1, WAVES>(a, s);
  if (K <= 64) return launch<2, WAVES>(a, s);
  if (K <= 128) return launch<4, WAVES>(a, s);
  return launch<8, WAVES>(a, s);
}

}  // namespace
}  // namespace kgx

using namespace kgx;

extern "C" int kgx_dense(int64_t M, const float* x0, int64_t ld_x0, int64_t K0, const float* W0,
                         const float* x1, int64_t ld_x1, int64_t K1, const float* W1, int64_t N,
                         const float* bias, int flags, float* out, int64_t ld_out, kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(M >= 0 && K0 >= 0 && K1 >= 0 && N >= 0, KGX_ERR_ARG, "kgx_dense: negative size");
  KGX_REQUIRE((flags & ~(KGX_DENSE_RELU | KGX_DENSE_ACCUMULATE)) == 0, KGX_ERR_ARG, "kgx_dense: unknown flags 0x%x",
              flags);
  KGX_REQUIRE(K0 + K1 <= KGX_DENSE_MAX_K && N <= KGX_DENSE_MAX_N, KGX_ERR_UNSUPPORTED,
              "kgx_dense: K0 + K1 must be <= %d and N <= %d (got K %lld, N %lld)", KGX_DENSE_MAX_K,
              KGX_DENSE_MAX_N, (long long)(K0 + K1), (long long)N);
  KGX_REQUIRE(K0 % 4 == 0 && K1 % 4 == 0, KGX_ERR_UNSUPPORTED, "kgx_dense: K0 and K1 must be multiples of 4");
  if (M == 0 || N == 0) return KGX_OK;
  KGX_REQUIRE(out && ld_out >= N, KGX_ERR_ARG, "kgx_dense: null out or ld_out < N");
  KGX_REQUIRE(K0 == 0 || (x0 && W0 && ld_x0 >= K0 && ld_x0 % 4 == 0 && reinterpret_cast<uintptr_t>(x0) % 16 == 0),
              KGX_ERR_ARG, "kgx_dense: x0 must be 16-byte aligned with ld %% 4 == 0 and ld >= K0");
  KGX_REQUIRE(K1 == 0 || (x1 && W1 && ld_x1 >= K1 && ld_x1 % 4 == 0 && reinterpret_cast<uintptr_t>(x1) % 16 == 0),
              KGX_ERR_ARG, "kgx_dense: x1 must be 16-byte aligned with ld %% 4 == 0 and ld >= K1");
  KGX_REQUIRE(ld_x0 < (int64_t(1) << 24) && ld_x1 < (int64_t(1) << 24) && ld_out < (int64_t(1) << 24), KGX_ERR_ARG,
              "kgx_dense: leading dimension >= 2^24 (32-bit tile offsets)");
  DenseArgs a{};
  a.M = M;
  a.x0 = x0;
  a.ld0 = ld_x0;
  a.K0 = int(K0);
  a.x1 = x1;
  a.ld1 = ld_x1;
  a.K1 = int(K1);
  a.W0 = W0;
  a.W1 = W1;
  a.N = int(N);
  a.bias = bias;
  a.out = out;
  a.ld_out = ld_out;
  a.relu = (flags & KGX_DENSE_RELU) != 0;
  a.accumulate = (flags & KGX_DENSE_ACCUMULATE) != 0;
  const int K = int(K0 + K1);
  a.cg_count = N <= 128 ? 1 : 2;
  a.vec_out = N % 4 == 0 && ld_out % 4 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0;
  // a.pstore / a.debug stay 0: the producer-store form (measured slower, C4 7.7
  // vs 7.1 ms) and the cost-decomposition builds are no longer instantiated
  // (tools/experiments/round4_variants.patch restores their switches)
  if (N <= 64) return launch_ks<4>(K, a, stream);
  return launch_ks<8>(K, a, stream);
}
