// Weight and bias gradients of the fused layers' training step (the backward
// of kgx_spmm_gemm's `out = bias + P W`, DESIGN.md §4 "Backward"):
//
//   dW[k, m] = sum_n P[n, k] D[n, m]      (P^T D, the sum over all N nodes)
//   db[m]    = sum_n D[n, m]              (column sums of D = dOut)
//
// in ONE pass over P and D.  The torch path it replaces (ops._gemm_tn_tall: a
// split-K batched fp32 GEMM, then D.sum(0) as a second pass) read D twice and
// ran the fp32 GEMM at ~2 TB/s (NS: 5.2 ms of a 24.5 ms training step).
//
// Three forms (kgx_gemm_tn picks by KGX_TN_LDS): gemm_tn_ws_kernel (default,
// below: producer waves split into LDS, consumer waves run the MFMAs),
// gemm_tn_lds_kernel (the same two phases on every wave in turn) and
// gemm_tn_kernel (every wave splits its own operands, described first).
//
// Layout: the reduction runs over the node dimension n, which is the stored
// row index of both operands, so the MFMA's K dimension is n.  For
// v_mfma_f32_16x16x32_bf16, lane l supplies A[l % 16][8 (l / 16) + t] and
// B[8 (l / 16) + t][l % 16], t = 0..7: eight consecutive NODES of one column.
// A lane loads float4 pieces of eight rows (four columns each); element e of
// every lane's pieces is the operand of MFMA e, whose 16 output rows are then
// every fourth column -- so the operands come straight from HBM in 1-KB
// coalesced loads, with no LDS transpose, and the stores unscramble the
// columns.  Products are the bf16x3 split
// (kgx_bf16x3.h: six bf16 products per f32 product, f32-accurate).
//
// Block: 256 threads, a 128 x 128 tile of dW; wave w owns rows k in
// [64 (w >> 1), +64) and columns m in [64 (w & 1), +64): 16 MFMA tiles, 64
// accumulator registers, plus three steps' operand values (this step's, and
// the next two steps' loads in flight): one wave per SIMD.  Grid: x = contiguous
// row ranges (split-K, one block per CU), y = dW tiles.  Each block writes its partial tile (and partial db)
// to the workspace; gemm_tn_finish sums the partials in block order, so the
// result is deterministic.
//
// Non-finite inputs: a block that loads an inf or NaN recomputes its partial
// with plain f32 multiply-adds (IEEE propagation), the slow path.

#include "kgx_bf16x3.h"
#include "kgx_internal.h"

namespace kgx {
namespace {

typedef short kgx_bf16x8_t __attribute__((ext_vector_type(8)));
typedef float kgx_f32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t kgx_u32x4_t __attribute__((ext_vector_type(4)));

constexpr int kTile = 128;          // dW tile edge per block
constexpr int kTn = 256;            // threads per block (4 waves)
constexpr int kStep = 32;           // nodes per MFMA K step (8 per lane group)
constexpr int kPart = kTile * kTile + kTile;  // floats per partial: tile + db

struct TnArgs {
  const float* P;
  const float* D;
  float* part;
  int64_t N, ldp, ldd, K, M;
  int64_t steps;   // ceil(N / kStep)
  int tiles_m;     // dW tiles along m
  int with_db;
};

struct Planes {
  kgx_bf16x8_t hi, mid, lo;
};

// eight f32 values -> three bf16x8 planes (pairs through split3_pair_rn)
__device__ __forceinline__ Planes split8(const float (&v)[8]) {
  kgx_u32x4_t h, m, l;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    uint32_t a, b, c;
    split3_pair_rn(v[2 * p], v[2 * p + 1], a, b, c);
    h[p] = a;
    m[p] = b;
    l[p] = c;
  }
  Planes r;
  r.hi = __builtin_bit_cast(kgx_bf16x8_t, h);
  r.mid = __builtin_bit_cast(kgx_bf16x8_t, m);
  r.lo = __builtin_bit_cast(kgx_bf16x8_t, l);
  return r;
}

__device__ __forceinline__ kgx_f32x4_t mfma6(const Planes& a, const Planes& b, kgx_f32x4_t acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.mid, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.mid, b.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.mid, b.mid, acc, 0, 0, 0);
  return acc;
}

// One step's operand values per lane: for nodes n = 32 s + 8 g + t (t = 0..7),
// P[n][k0 + 4 c .. +3] and D[n][m0 + 4 c .. +3] as float4 -- 16 dwordx4 loads
// per lane, each instruction reading four rows x 256 contiguous bytes.  Buffer
// loads through a per-step descriptor: rows past N fall outside its record
// count and column groups past K / M get an out-of-range offset, so both read
// as 0 with no branch -- every load is unconditional and the next step's
// loads stay in flight across this step's MFMAs.
//
// Element e of lane c's float4 is column 4 c + e: MFMA e of a k (or m) block
// takes element e of every lane, so its 16 output rows are the columns
// k0 + 4 c + e, c = 0..15 (a strided set; the store unscrambles it).
typedef float kgx_f32x4v_t __attribute__((ext_vector_type(4)));

struct StepVals {
  kgx_f32x4v_t p[8], d[8];
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t step_rsrc(const float* base, int64_t ld, int64_t s, int64_t N) {
  const int64_t r0 = s * kStep;
  int64_t rows = N - r0;
  rows = rows > kStep ? kStep : (rows < 0 ? 0 : rows);
  const uint64_t addr = reinterpret_cast<uint64_t>(base) + uint64_t(r0 * ld * 4);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(addr));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(addr >> 32));
  const int bytes = __builtin_amdgcn_readfirstlane(int(rows * ld * 4));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uint64_t(hi) << 32) | lo), 0, bytes, 0x00020000);
}

__device__ __forceinline__ void load_step(StepVals& v, const TnArgs& a, int64_t s, uint32_t po, uint32_t dof) {
  const auto rp = step_rsrc(a.P, a.ldp, s, a.N);
  const auto rd = step_rsrc(a.D, a.ldd, s, a.N);
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    v.p[t] = __builtin_bit_cast(kgx_f32x4v_t, __builtin_amdgcn_raw_buffer_load_b128(rp, po, int(t * a.ldp * 4), 0));
    v.d[t] = __builtin_bit_cast(kgx_f32x4v_t, __builtin_amdgcn_raw_buffer_load_b128(rd, dof, int(t * a.ldd * 4), 0));
  }
}

__global__ __launch_bounds__(kTn, 1) void gemm_tn_kernel(TnArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  const int tile = blockIdx.y;
  const int64_t k0 = int64_t(tile / a.tiles_m) * kTile + (wave >> 1) * 64;
  const int64_t m0 = int64_t(tile % a.tiles_m) * kTile + (wave & 1) * 64;
  const int64_t s_lo = a.steps * blockIdx.x / gridDim.x, s_hi = a.steps * (blockIdx.x + 1) / gridDim.x;
  const bool do_db = a.with_db && k0 == 0;  // the waves of the first k half of the first tile row

  // this lane's byte offsets within a step (row 8 g, columns 4 c .. 4 c + 3 of the wave's
  // 64); column groups past K / M get an offset past every record count (K, M % 4 == 0)
  const int64_t kq = k0 + 4 * c, mq = m0 + 4 * c;
  const uint32_t po = kq < a.K ? uint32_t((8 * g * a.ldp + kq) * 4) : 0x80000000u;
  const uint32_t dof = mq < a.M ? uint32_t((8 * g * a.ldd + mq) * 4) : 0x80000000u;
  const bool wave_live = k0 < a.K && m0 < a.M;

  kgx_f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = kgx_f32x4_t{0.f, 0.f, 0.f, 0.f};
  float dbs[4] = {0.f, 0.f, 0.f, 0.f};
  int bad = 0;

  auto compute = [&](const StepVals& v) {
    if (!wave_live) return;
    // finite and split-safe (|x| < 0x1.ffp127, kgx_bf16x3.h) for every value iff the sum of |x| is
    // below that (an inf / NaN propagates; a sum of huge finite values sends the block to the slow
    // path too, which is only slower)
    float sa = 0.0f;
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) sa += fabsf(v.p[t][e]) + fabsf(v.d[t][e]);
    bad |= sa < 0x1.ffp127f ? 0 : 1;
    Planes B[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float col[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) col[t] = v.d[t][j];
      B[j] = split8(col);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float col[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) col[t] = v.p[t][i];
      const Planes A = split8(col);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma6(A, B[j], acc[i][j]);
    }
    if (do_db) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < 8; ++t) dbs[j] = __fadd_rn(dbs[j], v.d[t][j]);
    }
  };

  // Three register sets in turn: step s's values are consumed while the loads of steps s + 1
  // and s + 2 are in flight (32 KB per wave, 128 KB per CU).  Every load is unconditional (a step
  // past the block's range is valid memory or reads 0), so the count of loads issued after a
  // set's loads is the same on every path and the compiler's waits before its use stay partial
  // (vmcnt(32)).
  StepVals v0, v1, v2;
  load_step(v0, a, s_lo, po, dof);
  load_step(v1, a, s_lo + 1, po, dof);
  for (int64_t s = s_lo; s < s_hi; s += 3) {
    load_step(v2, a, s + 2, po, dof);
    compute(v0);
    if (s + 1 >= s_hi) break;
    load_step(v0, a, s + 3, po, dof);
    compute(v1);
    if (s + 2 >= s_hi) break;
    load_step(v1, a, s + 4, po, dof);
    compute(v2);
  }

  float* part = a.part + (int64_t(blockIdx.x) * gridDim.y + tile) * kPart;
  const int kl0 = (wave >> 1) * 64, ml0 = (wave & 1) * 64;
  if (__syncthreads_or(bad)) {
    // slow path: this block's rows in plain f32, one thread per (k, m) pair in turn
    for (int o = threadIdx.x; o < kTile * kTile; o += kTn) {
      const int64_t k = int64_t(tile / a.tiles_m) * kTile + o / kTile;
      const int64_t m = int64_t(tile % a.tiles_m) * kTile + o % kTile;
      float s = 0.0f;
      if (k < a.K && m < a.M)
        for (int64_t n = s_lo * kStep; n < s_hi * kStep && n < a.N; ++n)
          s = __fadd_rn(s, __fmul_rn(a.P[n * a.ldp + k], a.D[n * a.ldd + m]));
      part[o] = s;
    }
    if (a.with_db && tile / a.tiles_m == 0)
      for (int o = threadIdx.x; o < kTile; o += kTn) {
        const int64_t m = int64_t(tile % a.tiles_m) * kTile + o;
        float s = 0.0f;
        if (m < a.M)
          for (int64_t n = s_lo * kStep; n < s_hi * kStep && n < a.N; ++n) s = __fadd_rn(s, a.D[n * a.ldd + m]);
        part[kTile * kTile + o] = s;
      }
    return;
  }
  // accumulator (i, j), element r: MFMA row 4 g + r = column k0 + 4 (4 g + r) + i of P, MFMA
  // column c = column m0 + 4 c + j of D
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[(kl0 + 4 * (4 * g + r) + i) * kTile + ml0 + 4 * c + j] = acc[i][j][r];
  if (do_db) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = dbs[j];
      v = __fadd_rn(v, __shfl_xor(v, 16, 64));
      v = __fadd_rn(v, __shfl_xor(v, 32, 64));
      if (g == 0) part[kTile * kTile + ml0 + 4 * c + j] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// The LDS form (default): each operand value is split ONCE per block.  512
// threads = 8 waves.  Per 32-node step every thread loads two float4 of P and
// two of D (coalesced rows), splits them into bf16 hi / mid / lo and writes the
// planes to LDS ([node][column] images, 256 B rows, the 16-byte chunks of a
// row XOR-swizzled by the row); the waves then read their MFMA operands with
// ds_read_b64_tr_b16 (four nodes of one column per lane: the transpose the
// node-dimension reduction needs).  Wave w owns dW rows [32 (w >> 1), +32) and
// columns [64 (w & 1), +64): 2 x 4 MFMA tiles.  Planes are double-buffered
// (one barrier per step); the global loads run three steps ahead.
// ---------------------------------------------------------------------------
constexpr int kTnL = 512;                       // threads per block (8 waves)
constexpr int kPlaneBytes = kStep * kTile * 2;  // one [32][128] bf16 plane: 8 KB
constexpr int kBufBytes = 6 * kPlaneBytes;      // P hi/mid/lo, D hi/mid/lo
constexpr int kSets = 4;                        // register sets: one consumed, three in flight

typedef short kgx_bf16x4_t __attribute__((ext_vector_type(4)));
typedef kgx_bf16x4_t __attribute__((address_space(3))) lds_bf16x4_t;

// byte offset of 16-byte chunk ch (0..15) of plane row r: conflict-free for the
// transposed reads of two 4-row blocks 8 rows apart (cdna_hip_programming.md T10, image (b))
__device__ __forceinline__ int swz(int r, int ch) { return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))); }

struct LoadSet {
  kgx_f32x4v_t p[2], d[2];
};

// step s's loads; steps at or past s_end (the block's range) read 0 (a zero record count)
__device__ __forceinline__ void load_set(LoadSet& v, const TnArgs& a, int64_t s, int64_t s_end,
                                         const uint32_t (&po)[2], const uint32_t (&dof)[2]) {
  const int64_t n_end = s_end * kStep < a.N ? s_end * kStep : a.N;
  const auto rp = step_rsrc(a.P, a.ldp, s, n_end);
  const auto rd = step_rsrc(a.D, a.ldd, s, n_end);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    v.p[j] = __builtin_bit_cast(kgx_f32x4v_t, __builtin_amdgcn_raw_buffer_load_b128(rp, po[j], 0, 0));
    v.d[j] = __builtin_bit_cast(kgx_f32x4v_t, __builtin_amdgcn_raw_buffer_load_b128(rd, dof[j], 0, 0));
  }
}

__global__ __launch_bounds__(kTnL, 1) void gemm_tn_lds_kernel(TnArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[2 * kBufBytes];  // two buffers of six planes: 96 KB
  __shared__ float sdb[8][kTile];

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int tile = blockIdx.y;
  const int64_t tk0 = int64_t(tile / a.tiles_m) * kTile, tm0 = int64_t(tile % a.tiles_m) * kTile;
  const int64_t s_lo = a.steps * blockIdx.x / gridDim.x, s_hi = a.steps * (blockIdx.x + 1) / gridDim.x;
  const bool with_db = a.with_db && tk0 == 0;

  // loads: float4 q = t + 512 j of the step's [32][32] float4 grid -> node n = q >> 5, columns 4 (q & 31) ..
  const int c4 = t & 31;
  int nrow[2];
  uint32_t po[2], dof[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    nrow[j] = (t + 512 * j) >> 5;
    const int64_t k = tk0 + 4 * c4, m = tm0 + 4 * c4;
    po[j] = k < a.K ? uint32_t((nrow[j] * a.ldp + k) * 4) : 0x80000000u;
    dof[j] = m < a.M ? uint32_t((nrow[j] * a.ldd + m) * 4) : 0x80000000u;
  }
  // MFMA operand reads (ds_read_b64_tr_b16): lane 16 gq + 4 q + p supplies row 8 gq + 4 h + q, columns
  // cb + 4 p .. + 3 of the plane; it receives column cb + (lane & 15) of rows 8 gq + 4 h .. + 3
  const int gq = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int kw0 = 32 * (wave >> 1), mw0 = 64 * (wave & 1);  // this wave's dW block within the tile
  auto rd_off = [&](int cb, int h) { return swz(8 * gq + 4 * h + qq, (cb >> 3) + (pp >> 1)) + 8 * (pp & 1); };
  int offA[2][2], offB[4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 2; ++i) offA[i][h] = rd_off(kw0 + 16 * i, h);
#pragma unroll
    for (int j = 0; j < 4; ++j) offB[j][h] = rd_off(mw0 + 16 * j, h);
  }

  kgx_f32x4_t acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = kgx_f32x4_t{0.f, 0.f, 0.f, 0.f};
  float dbs[4] = {0.f, 0.f, 0.f, 0.f};

  // one step's values -> the split planes of LDS buffer b.  No per-value check: a value the split
  // does not represent exactly (inf, NaN, or |x| >= 0x1.ffp127, whose bf16 hi is inf) leaves an
  // inf - inf or inf * 0 NaN, or an inf, in the planes, so every accumulator its row or column
  // meets ends non-finite, and the block takes the slow path (checked once, after the loop)
  auto put = [&](const LoadSet& v, int b) {
    char* base = lds + b * kBufBytes;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int off = swz(nrow[j], c4 >> 1) + 8 * (c4 & 1);
#pragma unroll
      for (int o = 0; o < 2; ++o) {  // P, then D
        const kgx_f32x4v_t x = o ? v.d[j] : v.p[j];
        uint32_t h0, m0, l0, h1, m1, l1;
        split3_pair_rn(x[0], x[1], h0, m0, l0);
        split3_pair_rn(x[2], x[3], h1, m1, l1);
        char* pl = base + 3 * o * kPlaneBytes + off;
        *reinterpret_cast<uint2*>(pl) = make_uint2(h0, h1);
        *reinterpret_cast<uint2*>(pl + kPlaneBytes) = make_uint2(m0, m1);
        *reinterpret_cast<uint2*>(pl + 2 * kPlaneBytes) = make_uint2(l0, l1);
      }
      if (with_db) {
#pragma unroll
        for (int e = 0; e < 4; ++e) dbs[e] = __fadd_rn(dbs[e], v.d[j][e]);
      }
    }
  };

  // this wave's MFMAs over LDS buffer b
  auto mma = [&](int b) {
    const char* base = lds + b * kBufBytes;
    auto rd = [&](int plane, int off) {
      return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_bf16x4_t*)(const_cast<char*>(base) + plane * kPlaneBytes + off));
    };
    auto operand = [&](int plane, const int (&off)[2]) {
      const kgx_bf16x4_t lo = rd(plane, off[0]), hi = rd(plane, off[1]);
      return kgx_bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    };
    Planes B[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      B[j].hi = operand(3, offB[j]);
      B[j].mid = operand(4, offB[j]);
      B[j].lo = operand(5, offB[j]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      Planes A;
      A.hi = operand(0, offA[i]);
      A.mid = operand(1, offA[i]);
      A.lo = operand(2, offA[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma6(A, B[j], acc[i][j]);
    }
  };

  auto barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // steps s_lo .. s_hi - 1, padded to a multiple of four with steps that read 0 (and add
  // nothing); set (s - s_lo) % 4 holds step s; the loads run three steps ahead of the step
  // being split.  Every load is unconditional and the unrolled body has no exit, so the count
  // of loads in flight is the same on every path and the compiler's waits stay partial.
  LoadSet v[kSets];
  load_set(v[0], a, s_lo, s_hi, po, dof);
  load_set(v[1], a, s_lo + 1, s_hi, po, dof);
  load_set(v[2], a, s_lo + 2, s_hi, po, dof);
  put(v[0], 0);
  barrier();
  const int64_t n_pad = (s_hi - s_lo + kSets - 1) / kSets * kSets;
  for (int64_t u0 = 0; u0 < n_pad; u0 += kSets) {
#pragma unroll
    for (int u = 0; u < kSets; ++u) {
      load_set(v[(u + 3) % kSets], a, s_lo + u0 + u + 3, s_hi, po, dof);
      put(v[(u + 1) % kSets], (u + 1) & 1);  // the next step's planes
      mma(u & 1);
      barrier();
    }
  }

  float* part = a.part + (int64_t(blockIdx.x) * gridDim.y + tile) * kPart;
  float chk = 0.0f;  // non-finite iff some accumulator or column sum is (0 * inf and inf - inf: NaN)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) chk += 0.0f * acc[i][j][r];
#pragma unroll
  for (int e = 0; e < 4; ++e) chk += 0.0f * dbs[e];
  if (__syncthreads_or(chk != 0.0f)) {
    for (int o = t; o < kTile * kTile; o += kTnL) {
      const int64_t k = tk0 + o / kTile, m = tm0 + o % kTile;
      float sum = 0.0f;
      if (k < a.K && m < a.M)
        for (int64_t n = s_lo * kStep; n < s_hi * kStep && n < a.N; ++n)
          sum = __fadd_rn(sum, __fmul_rn(a.P[n * a.ldp + k], a.D[n * a.ldd + m]));
      part[o] = sum;
    }
    if (with_db)
      for (int o = t; o < kTile; o += kTnL) {
        const int64_t m = tm0 + o;
        float sum = 0.0f;
        if (m < a.M)
          for (int64_t n = s_lo * kStep; n < s_hi * kStep && n < a.N; ++n) sum = __fadd_rn(sum, a.D[n * a.ldd + m]);
        part[kTile * kTile + o] = sum;
      }
    return;
  }
  // accumulator (i, j), element r: dW row kw0 + 16 i + 4 gq + r, column mw0 + 16 j + (lane & 15)
  const int cl = lane & 15;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[(kw0 + 16 * i + 4 * gq + r) * kTile + mw0 + 16 * j + cl] = acc[i][j][r];
  if (with_db) {  // columns 4 c4 .. + 3: lanes l and l + 32 of a wave, then the 8 waves in order
#pragma unroll
    for (int e = 0; e < 4; ++e) dbs[e] = __fadd_rn(dbs[e], __shfl_xor(dbs[e], 32, 64));
    if (lane < 32)
#pragma unroll
      for (int e = 0; e < 4; ++e) sdb[wave][4 * c4 + e] = dbs[e];
    __syncthreads();
    if (t < kTile) {
      float sum = 0.0f;
#pragma unroll
      for (int w = 0; w < 8; ++w) sum = __fadd_rn(sum, sdb[w][t]);
      part[kTile * kTile + t] = sum;
    }
  }
}

// ---------------------------------------------------------------------------
// The warp-specialised form (default): the LDS form's two phases on separate
// waves.  Waves 4-7 (producers, one per SIMD) load P and D three steps ahead,
// split and write the planes of step s + 1; waves 0-3 (consumers, one per
// SIMD) run step s's MFMAs -- 16 tiles of 16 x 16, a 64 x 64 block of dW per
// wave -- so a SIMD issues the producer's VALU and LDS writes in its
// consumer's MFMA gaps instead of after them, and each operand plane is read
// from LDS by two consumers instead of two / four waves (96 KB of
// transposed reads per step instead of 147).  One barrier per step hands a
// buffer over, as in the LDS form; each role runs its own loop with the same
// barrier count, so the producer's load waits stay partial.
// ---------------------------------------------------------------------------
constexpr int kPj = 4;  // float4 loads of P (and of D) per producer thread per step

struct ProdSet {
  kgx_f32x4v_t p[kPj], d[kPj];
};

__device__ __forceinline__ void prod_load(ProdSet& v, const TnArgs& a, int64_t s, int64_t s_end,
                                          const uint32_t (&po)[kPj], const uint32_t (&dof)[kPj]) {
  const int64_t n_end = s_end * kStep < a.N ? s_end * kStep : a.N;
  const auto rp = step_rsrc(a.P, a.ldp, s, n_end);
  const auto rd = step_rsrc(a.D, a.ldd, s, n_end);
#pragma unroll
  for (int j = 0; j < kPj; ++j) {
    v.p[j] = __builtin_bit_cast(kgx_f32x4v_t, __builtin_amdgcn_raw_buffer_load_b128(rp, po[j], 0, 0));
    v.d[j] = __builtin_bit_cast(kgx_f32x4v_t, __builtin_amdgcn_raw_buffer_load_b128(rd, dof[j], 0, 0));
  }
}

__global__ __launch_bounds__(kTnL, 1) void gemm_tn_ws_kernel(TnArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[2 * kBufBytes];  // two buffers of six planes: 96 KB
  __shared__ float sdb[4][kTile];

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool producer = wave >= 4;
  const int tile = blockIdx.y;
  const int64_t tk0 = int64_t(tile / a.tiles_m) * kTile, tm0 = int64_t(tile % a.tiles_m) * kTile;
  const int64_t s_lo = a.steps * blockIdx.x / gridDim.x, s_hi = a.steps * (blockIdx.x + 1) / gridDim.x;
  const bool with_db = a.with_db && tk0 == 0;
  const int64_t n_pad = (s_hi - s_lo + kSets - 1) / kSets * kSets;

  auto barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  kgx_f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = kgx_f32x4_t{0.f, 0.f, 0.f, 0.f};
  float dbs[4] = {0.f, 0.f, 0.f, 0.f};
  // producer thread p: float4 q = p + 256 j of the step's [32][32] float4 grid -> node q >> 5, columns 4 (q & 31) ..
  const int p = t & 255;
  const int c4 = p & 31;

  if (producer) {
    int nrow[kPj];
    uint32_t po[kPj], dof[kPj];
#pragma unroll
    for (int j = 0; j < kPj; ++j) {
      nrow[j] = (p + 256 * j) >> 5;
      const int64_t k = tk0 + 4 * c4, m = tm0 + 4 * c4;
      po[j] = k < a.K ? uint32_t((nrow[j] * a.ldp + k) * 4) : 0x80000000u;
      dof[j] = m < a.M ? uint32_t((nrow[j] * a.ldd + m) * 4) : 0x80000000u;
    }
    // one step's values -> the split planes of LDS buffer b (no per-value check: see the LDS form)
    auto put = [&](const ProdSet& v, int b) {
      char* base = lds + b * kBufBytes;
#pragma unroll
      for (int j = 0; j < kPj; ++j) {
        const int off = swz(nrow[j], c4 >> 1) + 8 * (c4 & 1);
#pragma unroll
        for (int o = 0; o < 2; ++o) {  // P, then D
          const kgx_f32x4v_t x = o ? v.d[j] : v.p[j];
          uint32_t h0, m0, l0, h1, m1, l1;
          split3_pair_rn(x[0], x[1], h0, m0, l0);
          split3_pair_rn(x[2], x[3], h1, m1, l1);
          char* pl = base + 3 * o * kPlaneBytes + off;
          *reinterpret_cast<uint2*>(pl) = make_uint2(h0, h1);
          *reinterpret_cast<uint2*>(pl + kPlaneBytes) = make_uint2(m0, m1);
          *reinterpret_cast<uint2*>(pl + 2 * kPlaneBytes) = make_uint2(l0, l1);
        }
        if (with_db) {
#pragma unroll
          for (int e = 0; e < 4; ++e) dbs[e] = __fadd_rn(dbs[e], v.d[j][e]);
        }
      }
    };
    // steps padded to a multiple of four with steps that read 0; set (s - s_lo) % 4 holds step s
    ProdSet v[kSets];
    prod_load(v[0], a, s_lo, s_hi, po, dof);
    prod_load(v[1], a, s_lo + 1, s_hi, po, dof);
    prod_load(v[2], a, s_lo + 2, s_hi, po, dof);
    put(v[0], 0);
    barrier();
    for (int64_t u0 = 0; u0 < n_pad; u0 += kSets) {
#pragma unroll
      for (int u = 0; u < kSets; ++u) {
        prod_load(v[(u + 3) % kSets], a, s_lo + u0 + u + 3, s_hi, po, dof);
        put(v[(u + 1) % kSets], (u + 1) & 1);  // the next step's planes
        barrier();
      }
    }
  } else {
    // operand reads (ds_read_b64_tr_b16), as in the LDS form; wave w owns dW rows
    // [64 (w >> 1), +64) and columns [64 (w & 1), +64)
    const int gq = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    const int kw0 = 64 * (wave >> 1), mw0 = 64 * (wave & 1);
    auto rd_off = [&](int cb, int h) { return swz(8 * gq + 4 * h + qq, (cb >> 3) + (pp >> 1)) + 8 * (pp & 1); };
    int offA[4][2], offB[4][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        offA[i][h] = rd_off(kw0 + 16 * i, h);
        offB[i][h] = rd_off(mw0 + 16 * i, h);
      }
    auto mma = [&](int b) {
      const char* base = lds + b * kBufBytes;
      auto rd = [&](int plane, int off) {
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_bf16x4_t*)(const_cast<char*>(base) + plane * kPlaneBytes + off));
      };
      auto operand = [&](int plane, const int (&off)[2]) {
        const kgx_bf16x4_t lo = rd(plane, off[0]), hi = rd(plane, off[1]);
        return kgx_bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      };
      Planes B[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        B[j].hi = operand(3, offB[j]);
        B[j].mid = operand(4, offB[j]);
        B[j].lo = operand(5, offB[j]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        Planes A;
        A.hi = operand(0, offA[i]);
        A.mid = operand(1, offA[i]);
        A.lo = operand(2, offA[i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma6(A, B[j], acc[i][j]);
      }
    };
    barrier();  // the producers' first planes
    for (int64_t u0 = 0; u0 < n_pad; u0 += kSets) {
#pragma unroll
      for (int u = 0; u < kSets; ++u) {
        mma(u & 1);
        barrier();
      }
    }
  }

  float* part = a.part + (int64_t(blockIdx.x) * gridDim.y + tile) * kPart;
  float chk = 0.0f;  // non-finite iff some accumulator or column sum is (0 * inf and inf - inf: NaN)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) chk += 0.0f * acc[i][j][r];
#pragma unroll
  for (int e = 0; e < 4; ++e) chk += 0.0f * dbs[e];
  if (__syncthreads_or(chk != 0.0f)) {
    for (int o = t; o < kTile * kTile; o += kTnL) {
      const int64_t k = tk0 + o / kTile, m = tm0 + o % kTile;
      float sum = 0.0f;
      if (k < a.K && m < a.M)
        for (int64_t n = s_lo * kStep; n < s_hi * kStep && n < a.N; ++n)
          sum = __fadd_rn(sum, __fmul_rn(a.P[n * a.ldp + k], a.D[n * a.ldd + m]));
      part[o] = sum;
    }
    if (with_db)
      for (int o = t; o < kTile; o += kTnL) {
        const int64_t m = tm0 + o;
        float sum = 0.0f;
        if (m < a.M)
          for (int64_t n = s_lo * kStep; n < s_hi * kStep && n < a.N; ++n) sum = __fadd_rn(sum, a.D[n * a.ldd + m]);
        part[kTile * kTile + o] = sum;
      }
    return;
  }
  if (!producer) {
    // accumulator (i, j), element r: dW row kw0 + 16 i + 4 (lane >> 4) + r, column mw0 + 16 j + (lane & 15)
    const int kw0 = 64 * (wave >> 1), mw0 = 64 * (wave & 1), gq = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) part[(kw0 + 16 * i + 4 * gq + r) * kTile + mw0 + 16 * j + cl] = acc[i][j][r];
  }
  if (with_db) {  // columns 4 c4 .. + 3: lanes l and l + 32 of a producer wave, then the 4 producer waves in order
    if (producer) {
#pragma unroll
      for (int e = 0; e < 4; ++e) dbs[e] = __fadd_rn(dbs[e], __shfl_xor(dbs[e], 32, 64));
      if (lane < 32)
#pragma unroll
        for (int e = 0; e < 4; ++e) sdb[wave - 4][4 * c4 + e] = dbs[e];
    }
    __syncthreads();
    if (t < kTile) {
      float sum = 0.0f;
#pragma unroll
      for (int w = 0; w < 4; ++w) sum = __fadd_rn(sum, sdb[w][t]);
      part[kTile * kTile + t] = sum;
    }
  }
}

// dW[k, m] = sum over blocks b (in order) of part[b][tile(k, m)][k % 128][m % 128]; db likewise
__global__ void gemm_tn_finish_kernel(const float* __restrict__ part, int nb, int tiles, int tiles_m, int64_t K,
                                      int64_t M, float* __restrict__ dW, int64_t ld_dw, float* __restrict__ db) {
  const int64_t o = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t n_w = K * M;
  if (o < n_w) {
    const int64_t k = o / M, m = o % M;
    const int tile = int(k / kTile) * tiles_m + int(m / kTile);
    const int64_t off = (k % kTile) * kTile + (m % kTile);
    float s = 0.0f;
    for (int b = 0; b < nb; ++b) s = __fadd_rn(s, part[(int64_t(b) * tiles + tile) * kPart + off]);
    dW[k * ld_dw + m] = s;
  } else if (db && o < n_w + M) {
    const int64_t m = o - n_w;
    const int tile = int(m / kTile);  // tile row 0
    float s = 0.0f;
    for (int b = 0; b < nb; ++b) s = __fadd_rn(s, part[(int64_t(b) * tiles + tile) * kPart + kTile * kTile + m % kTile]);
    db[m] = s;
  }
}

int gemm_tn_blocks(int64_t N) {
  const int64_t steps = (N + kStep - 1) / kStep;
  const int64_t want = cu_count();
  return int(steps < want ? (steps > 0 ? steps : 1) : want);
}

}  // namespace
}  // namespace kgx

using namespace kgx;

extern "C" int kgx_gemm_tn_workspace_bytes(int64_t N, int64_t K, int64_t M, size_t* bytes) {
  KGX_REQUIRE(bytes && N >= 0 && K > 0 && M > 0, KGX_ERR_ARG, "kgx_gemm_tn_workspace_bytes: bad arguments");
  const int64_t tiles = ((K + kTile - 1) / kTile) * ((M + kTile - 1) / kTile);
  *bytes = size_t(gemm_tn_blocks(N)) * size_t(tiles) * kPart * sizeof(float);
  return KGX_OK;
}

extern "C" int kgx_gemm_tn(int64_t N, const float* P, int64_t ldp, int64_t K, const float* D, int64_t ldd, int64_t M,
                           float* dW, int64_t ld_dw, float* db, void* workspace, size_t workspace_bytes,
                           kgx_stream_t stream_) {
  KGX_REQUIRE(N >= 0 && K > 0 && M > 0 && ldp >= K && ldd >= M && ld_dw >= M, KGX_ERR_ARG,
              "kgx_gemm_tn: bad shapes (N=%lld K=%lld M=%lld ldp=%lld ldd=%lld ld_dw=%lld)", (long long)N,
              (long long)K, (long long)M, (long long)ldp, (long long)ldd, (long long)ld_dw);
  KGX_REQUIRE(dW && (N == 0 || (P && D)), KGX_ERR_ARG, "kgx_gemm_tn: null pointer");
  size_t need = 0;
  (void)kgx_gemm_tn_workspace_bytes(N, K, M, &need);
  KGX_REQUIRE(workspace && workspace_bytes >= need, KGX_ERR_ARG, "kgx_gemm_tn: workspace %zu < %zu bytes",
              workspace_bytes, need);
  hipStream_t s = as_stream(stream_);
  const int tiles_m = int((M + kTile - 1) / kTile);
  const int tiles = int((K + kTile - 1) / kTile) * tiles_m;
  const int nb = gemm_tn_blocks(N);
  if (N > 0) {
    TnArgs a{P, D, static_cast<float*>(workspace), N, ldp, ldd, K, M, (N + kStep - 1) / kStep, tiles_m, db ? 1 : 0};
    // measurement A/B: KGX_TN_LDS 0 = the per-wave split form, 1 = the LDS form, 2 (default) = warp-specialised
    const char* e = getenv("KGX_TN_LDS");
    const int form = e ? atoi(e) : 2;
    if (form == 2 && K % 4 == 0 && M % 4 == 0) {
      hipLaunchKernelGGL(gemm_tn_ws_kernel, dim3(nb, tiles), dim3(kTnL), 0, s, a);
    } else if (form != 0 && K % 4 == 0 && M % 4 == 0) {
      hipLaunchKernelGGL(gemm_tn_lds_kernel, dim3(nb, tiles), dim3(kTnL), 0, s, a);
    } else {
      hipLaunchKernelGGL(gemm_tn_kernel, dim3(nb, tiles), dim3(kTn), 0, s, a);
    }
    KGX_CHECK_LAUNCH();
  } else {
    KGX_CHECK_HIP(hipMemsetAsync(workspace, 0, need, s));
  }
  const int64_t outs = K * M + (db ? M : 0);
  hipLaunchKernelGGL(gemm_tn_finish_kernel, dim3(unsigned((outs + 255) / 256)), dim3(256), 0, s,
                     static_cast<const float*>(workspace), nb, tiles, tiles_m, K, M, dW, ld_dw, db);
  KGX_CHECK_LAUNCH();
  return KGX_OK;
}
