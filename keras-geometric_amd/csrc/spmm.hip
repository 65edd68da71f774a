// Fused gather -> message -> segment reduction -> epilogue for the kgx engine
// (gfx950, wave64).
//
// One "group" of G lanes (G = pow2 >= F/VEC, <= 64) owns one destination row
// (or one chunk of a split hub row); lane l holds features
// (t*G + l)*VEC .. +VEC for t < NT.  The group walks its CSR edges IN ORDER,
// U edges at a time: the U neighbour indices are loaded, the U neighbour rows
// are gathered with VEC-wide loads (all U in flight), then folded into the
// accumulator strictly sequentially with round-to-nearest adds and no FMA
// contraction — the same per-(row, feature) operation sequence as the
// reference's sequential scatter_add, hence bit-identical results for
// identical messages.  Rows come in descending-degree order (schedule) and
// every group walks the work list grid-stride, so hub rows start first.
//
// Reference semantics restated here (src/keras_geometric/...):
//   sum  : layers/aggregators.py:126-137 (segment_sum, zeros init)
//   mean : layers/aggregators.py:56-85   (sum / max(count_f32, 1e-8))
//   max  : layers/aggregators.py:99-112  (segment_max, -inf init; isinf -> 0)
//   min  : layers/aggregators.py:151-167 (-segment_max(-m); isinf -> 0)
//   std  : layers/aggregators.py:182-228 (two-pass, N divisor, count<=1 -> 0)
//   GCN message x_j W * norm (gcn_conv.py:233-248) with W pre-applied per node,
//   GCN update + bias (gcn_conv.py:266-272), GIN (1+eps)*x + aggr (gin_conv.py:216-222).
#include <cstdlib>

#include "kgx_internal.h"
#include "kgx_vec.h"

namespace kgx {
namespace {

struct SpmmArgs {
  const int32_t* rowptr;
  const int32_t* rows;
  int64_t n_rows;
  const int4* items;
  int64_t n_items;
  const int4* split;
  int64_t n_split;
  const int32_t* idx;
  const float* w;
  const float* table;
  int64_t ld_t;
  int F;  // columns handled by this launch
  float* out;
  int64_t ld_o;
  const float* bias;
  const float* xroot;
  int64_t ld_x;
  float gin_scale;
  float* partials;
  int64_t ld_p;
  int epi;
  int G;
  int lgG;
  int hints;  // bit0: nt loads of idx/w, bit1: nt stores of out (experiment knob, KGX_SPMM_HINTS)
  // message dropout (training): message *= keep(seed, drop_key[e], column) / (1 - p)
  const int32_t* drop_key;
  uint64_t drop_seed;
  uint32_t drop_thresh;
  float drop_scale;
  int f_base;  // first column of this launch (column slicing of wide F)
  int long_rows;  // EXACT mode: rows of degree >= kLongRow are reduced by spmm_long_kernel
  int64_t n_long;  // items [n_long, n_items): short rows (degree <= KGX_SHORT_ROW_MAX) for spmm_short_kernel
  // EXACT mode (no items): rows[n_rows_long, n_rows) of the degree-ordered list have degree <=
  // KGX_SHORT_ROW_MAX and go to spmm_short_kernel (each row still one chain in CSR order)
  int64_t n_rows_long;
  // two-table gathers (kgx_spmm_ex2): sources c >= n_t1 are rows c - n_t1 of a second
  // table (same ld_t); t2b = table2 - n_t1 * ld_t as an address.  n_t1 = INT32_MAX: one table.
  const float* t2b;
  int32_t n_t1;
  // EXACT mode, dynamic pickup (kgx_spmm_ex2 counters): dyn[0] hands out the hub
  // kernel's (row, column group) items; with dyn_rows = 1, dyn[1] hands out
  // spmm_kernel's interleaved row batches.  NULL: the static grid-stride schedule.
  int32_t* dyn;
  int dyn_rows;
};

// Source row of column c: table[c], or with TWO table2[c - n_t1] (a separate
// instantiation, so the one-table kernels keep their registers and issue).
template <bool TWO>
__device__ __forceinline__ const float* tsrc(const SpmmArgs& a, int32_t c) {
  if constexpr (TWO) return (c >= a.n_t1 ? a.t2b : a.table) + row_off(c, a.ld_t);
  return a.table + row_off(c, a.ld_t);
}

// EXACT mode has no hub split (each row is one sequential reduction), so a hub
// row of 10^5 edges is a latency chain; rows this long get their own kernel
// with 32 gathers in flight per group instead of 6.
constexpr int kLongRow = 2048;
// split-row partials loaded together by the fix-up kernels
constexpr int kFixB = 8;

template <int RED>
struct Reducer {
  // init() is also the identity of combine(): +0 for sums (the accumulator
  // starts at +0 and an RN sum never produces -0 from it, so acc + 0 == acc
  // bit for bit, NaN and inf included) and -inf for the amax form.
  static __device__ __forceinline__ float init() {
    if constexpr (RED == KGX_MAX || RED == KGX_MIN) return -__builtin_inff();
    return 0.0f;
  }
  // message value as it enters the reduction
  static __device__ __forceinline__ float msg(float v) {
    if constexpr (RED == KGX_MIN) return -v;  // min = -segment_max(-m)
    return v;
  }
  static __device__ __forceinline__ float combine(float acc, float v) {
    if constexpr (RED == KGX_MAX || RED == KGX_MIN) return amax_update(acc, v);
    return __fadd_rn(acc, v);
  }
  // KGX_EPI_RAW: max / min as plain segment_max (no isinf guard)
  static __device__ __forceinline__ float finish_raw(float acc, int32_t deg) {
    if constexpr (RED == KGX_MAX) return acc;
    if constexpr (RED == KGX_MIN) return -acc;
    return finish(acc, deg);
  }
  static __device__ __forceinline__ float finish(float acc, int32_t deg) {
    if constexpr (RED == KGX_MEAN) return __fdiv_rn(acc, fmaxf(ref_count_f32(deg), 1e-8f));
    if constexpr (RED == KGX_MAX) return is_inf(acc) ? 0.0f : acc;
    if constexpr (RED == KGX_MIN) {
      const float r = -acc;
      return is_inf(r) ? 0.0f : r;
    }
    return acc;
  }
};

template <int VEC>
__device__ __forceinline__ void epilogue(const SpmmArgs& a, int32_t row, int f, float (&v)[VEC]) {
  if (a.epi == KGX_EPI_BIAS) {
    float b[VEC];
    vload<VEC>(b, a.bias + f);
#pragma unroll
    for (int k = 0; k < VEC; ++k) v[k] = __fadd_rn(v[k], b[k]);
  } else if (a.epi == KGX_EPI_GIN) {
    float x[VEC];
    vload<VEC>(x, a.xroot + int64_t(row) * a.ld_x + f);
#pragma unroll
    for (int k = 0; k < VEC; ++k) v[k] = __fadd_rn(__fmul_rn(a.gin_scale, x[k]), v[k]);
  } else if (a.epi == KGX_EPI_ACCUM) {  // out += this part's sum (sharded halo chunks)
    float o[VEC];
    vload<VEC>(o, a.out + int64_t(row) * a.ld_o + f);
#pragma unroll
    for (int k = 0; k < VEC; ++k) v[k] = __fadd_rn(o[k], v[k]);
  }
}

// U consecutive edges [e, e+U) of a row ending at `end`: U index (and weight)
// loads, then U row gathers, all unconditional (indices past `end` are clamped
// to end-1, whose row is already being fetched), then an in-order fold where
// clamped edges contribute the reduction's identity.  No load sits under a
// lane-dependent branch, so hipcc keeps all U gathers in flight.
template <int U, int VEC, int NT, int RED, bool WEIGHTED, bool DROP = false, bool TWO = false>
__device__ __forceinline__ void edge_block(const SpmmArgs& a, int32_t e, int32_t end, const int (&fl)[NT],
                                           float (&acc)[NT][VEC]) {
  using R = Reducer<RED>;
  const int n = end - e;
  int32_t c[U];
  float wt[U];
  uint32_t dk[U];
  if constexpr (DROP) {
#pragma unroll
    for (int u = 0; u < U; ++u) dk[u] = uint32_t(a.drop_key[u < n ? e + u : end - 1]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int32_t ee = u < n ? e + u : end - 1;
    if (a.hints & 1) {
      c[u] = ld_nt(a.idx + ee);
      if constexpr (WEIGHTED) wt[u] = ld_nt(a.w + ee);
    } else {
      c[u] = a.idx[ee];
      if constexpr (WEIGHTED) wt[u] = a.w[ee];
    }
  }
  float v[U][NT][VEC];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int t = 0; t < NT; ++t) vload<VEC>(v[u][t], tsrc<TWO>(a, c[u]) + fl[t]);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        float m = v[u][t][k];
        if constexpr (DROP)  // reference order: dropout(x_j W), then * norm (gcn_conv.py:237-248)
          m = __fmul_rn(m, drop_scale(a.drop_seed, dk[u], uint32_t(a.f_base + fl[t] + k), a.drop_thresh,
                                      a.drop_scale));
        if constexpr (WEIGHTED) m = __fmul_rn(m, wt[u]);
        acc[t][k] = R::combine(acc[t][k], u < n ? R::msg(m) : R::init());
      }
}

template <int VEC, int NT, int RED, bool WEIGHTED, bool DROP = false, bool TWO = false>
__global__ __launch_bounds__(kBlock) void spmm_kernel(SpmmArgs a) {
  using R = Reducer<RED>;
  // gathers in flight per group (NT = 1: 6 measured best at NS, 9.2-9.4 ms vs 9.5 at 8, 9.9 at 12)
  constexpr int U = NT >= 4 ? 2 : (NT == 2 ? 4 : 6);
  const int G = a.G;
  const int lane = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t(gridDim.x) * kBlock) >> a.lgG;
  const int64_t n_work = a.items ? a.n_long : a.n_rows_long;

  // Every global load below is unconditional (clamped to a valid address) and
  // masked work is folded in as the reduction's identity: a load under a
  // lane-dependent branch makes hipcc wait for it at the branch join, which
  // would serialise the U gathers that are meant to be in flight together.
  int fo[NT], fl[NT];
  bool fv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    fo[t] = (t * G + lane) * VEC;
    fv[t] = fo[t] < a.F;
    fl[t] = fv[t] ? fo[t] : a.F - VEC;  // load offset, always in range
  }

  // EXACT mode beside the forked hub kernel (a.dyn, dyn_rows = 1): each group
  // takes batches of kDynRows rows from a counter (lane 0's atomic, broadcast to
  // the group), so groups whose blocks started late -- behind the hub kernel --
  // take less, and the launch ends together.  Batch b is rows b, b + NB,
  // b + 2 NB, ... -- one row from each kDynRows-th of the degree-descending
  // list, so every batch carries about the same work, heaviest batches first.
  // Otherwise: static grid-stride.
  const bool dyn = a.dyn != nullptr && a.dyn_rows && !a.items;
  constexpr int kDynRows = 8;
  const int64_t gid = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> a.lgG;
  const int64_t NB = (n_work + kDynRows - 1) / kDynRows;
  int64_t it = gid;
  int jj = kDynRows;
  for (;;) {
    int64_t cur;
    if (dyn) {
      if (jj >= kDynRows) {
        int64_t b = 0;
        if (lane == 0) b = int64_t(atomicAdd(a.dyn + 1, 1));
        it = __shfl(b, 0, G);
        jj = 0;
      }
      if (it >= NB) break;
      cur = it + int64_t(jj) * NB;
      ++jj;
      if (cur >= n_work) {  // the later rows of this batch are past the end too
        jj = kDynRows;
        continue;
      }
    } else {
      if (it >= n_work) break;
      cur = it;
      it += ngroups;
    }
    int32_t row, beg, end, slot;
    if (a.items) {
      const int4 v = a.items[cur];
      row = v.x;
      beg = v.y;
      end = v.z;
      slot = v.w;
    } else {
      row = a.rows[cur];
      beg = a.rowptr[row];
      end = a.rowptr[row + 1];
      slot = -1;
      if (a.long_rows && end - beg >= kLongRow) continue;  // spmm_long_kernel's row
    }

    float acc[NT][VEC];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[t][k] = R::init();

    int32_t e = beg;
    for (; e + U <= end; e += U) edge_block<U, VEC, NT, RED, WEIGHTED, DROP, TWO>(a, e, end, fl, acc);
    // tail in half-width blocks: at most TU-1 clamped (redundant, cache-hit) loads
    constexpr int TU = U > 1 ? U / 2 : 1;
    for (; e < end; e += TU) edge_block<TU, VEC, NT, RED, WEIGHTED, DROP, TWO>(a, e, end, fl, acc);

#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (!fv[t]) continue;
      if (slot >= 0) {  // chunk of a split hub row: raw partial, finished by the fix-up
        vstore<VEC>(a.partials + int64_t(slot) * a.ld_p + fo[t], acc[t]);
      } else {
        float r[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k)
          r[k] = a.epi == KGX_EPI_RAW ? R::finish_raw(acc[t][k], end - beg) : R::finish(acc[t][k], end - beg);
        epilogue<VEC>(a, row, fo[t], r);
        if (a.hints & 2) vstore_nt<VEC>(a.out + int64_t(row) * a.ld_o + fo[t], r);
        else vstore<VEC>(a.out + int64_t(row) * a.ld_o + fo[t], r);
      }
    }
  }
}

// EXACT-mode rows of degree >= kLongRow (a prefix of the degree-ordered row
// list): the same in-order reduction as spmm_kernel, 32 gathers per block.
template <int VEC, int RED, bool WEIGHTED, bool DROP = false>
__global__ __launch_bounds__(kBlock) void spmm_long_kernel(SpmmArgs a) {
  using R = Reducer<RED>;
  constexpr int U = 32;
  const int G = a.G;
  const int lane = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t(gridDim.x) * kBlock) >> a.lgG;
  int fo[1], fl[1];
  fo[0] = lane * VEC;
  const bool fv = fo[0] < a.F;
  fl[0] = fv ? fo[0] : a.F - VEC;
  for (int64_t it = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> a.lgG; it < a.n_rows; it += ngroups) {
    const int32_t row = a.rows[it];
    const int32_t beg = a.rowptr[row], end = a.rowptr[row + 1];
    if (end - beg < kLongRow) break;  // rows are in descending degree order
    float acc[1][VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[0][k] = R::init();
    int32_t e = beg;
    for (; e + U <= end; e += U) edge_block<U, VEC, 1, RED, WEIGHTED, DROP>(a, e, end, fl, acc);
    for (; e < end; e += 4) edge_block<4, VEC, 1, RED, WEIGHTED, DROP>(a, e, end, fl, acc);
    if (!fv) continue;
    float r[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k)
      r[k] = a.epi == KGX_EPI_RAW ? R::finish_raw(acc[0][k], end - beg) : R::finish(acc[0][k], end - beg);
    epilogue<VEC>(a, row, fo[0], r);
    vstore<VEC>(a.out + int64_t(row) * a.ld_o + fo[0], r);
  }
}

// EXACT-mode rows of degree >= kLongRow, one 16-wave block per row.  Such a
// row is one chain of adds in CSR order that no split may re-associate, and
// spmm_long_kernel walks it with one 32-lane group (32 gathers in flight): the
// NS graph's largest row (138k edges) alone took 9.3 ms.  Here producer waves
// stream the row's messages (neighbour row x weight, rounded as the reference
// rounds them) into a two-stage LDS ring, kHubD stages of gathers in flight
// per lane, and CW consumer waves fold each stage in edge order, one feature
// per lane -- the same per-(row, feature) operation sequence, bit for bit.
// The gathers and their index / weight loads are inline-asm loads with
// counted vmcnt waits: the compiler's accounting would wait for the whole
// queue whenever an index it loaded is used.
constexpr int kHubThreads = 1024;
constexpr int kHubD = 8;      // rows in flight per producer lane
constexpr int kHubRPL = 2;  // rows per producer lane per stage
constexpr int kHubSMax = 56;
constexpr int kHubG = 16;  // hub column group: 4 x kHubG features

__device__ __forceinline__ void hub_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// The consumers' side: their LDS reads of stage s-1 need not land before the
// barrier (producers overwrite that buffer two barriers later, and the reads
// are waited for by the fold one iteration later), so no lgkmcnt(0) here.
__device__ __forceinline__ void hub_barrier_reader() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int G, int RED, bool WEIGHTED>
__global__ __launch_bounds__(kHubThreads, 1) void spmm_hub_kernel(SpmmArgs a) {
  using R = Reducer<RED>;
  constexpr int CW = G >= 16 ? G / 16 : 1;  // consumer waves (64 features each)
  constexpr int NPW = kHubThreads / 64 - CW;  // producer waves
  constexpr int RPW = 64 / G;                 // rows per producer wave per pass
  // a consumer lane holds two stages in registers: at most kHubSMax rows per
  // stage (a multiple of RPW, so narrow rows leave whole producer waves idle)
  constexpr int SP = NPW * RPW < kHubSMax ? NPW * RPW : kHubSMax;  // producer slots
  constexpr int RPL = SP * kHubRPL <= kHubSMax ? kHubRPL : 1;       // rows per slot per stage
  constexpr int S = SP * RPL;                 // rows (edges) per stage
  constexpr int RL = 4 * G;                   // floats per ring row
  constexpr int D = kHubD / RPL;              // stages of loads in flight (D x RPL rows per lane)
  static_assert(kHubSMax % 8 == 0 && D >= 2 && D % 2 == 0, "hub pipeline shape");
  __shared__ __attribute__((aligned(16))) float ring[3][S * RL];
  __shared__ int32_t hub_next[2];  // dynamic pickup: the block's next item, by row parity

  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  // Items (row, column group) in descending row degree.  Static: p += gridDim.x.
  // Dynamic (a.dyn): thread 0 (a consumer) takes the block's next item from a
  // counter while the row runs and parks it in LDS; one extra barrier per row
  // (rows here have >= 2048 edges) hands it to every wave, so blocks that drew
  // short hubs take more of them instead of idling behind the largest row.
  const int64_t n_hub_items = a.n_rows * ((a.F + 4 * G - 1) / (4 * G));
  int par = 0;
  auto next_item = [&](int64_t p) -> int64_t {
    if (!a.dyn) return p + gridDim.x;
    hub_barrier();  // thread 0's LDS write (waited for with lgkmcnt(0) here) is visible
    const int64_t q = hub_next[par];
    par ^= 1;
    return q;
  };
  auto claim_next = [&]() {  // thread 0, at a row's start: the item after this one
    if (a.dyn && threadIdx.x == 0) hub_next[par] = int32_t(gridDim.x) + atomicAdd(a.dyn, 1);
  };

  // Row h of the degree-ordered list; false past the long rows.  Iteration s
  // of a row: producers write stage s into ring[s % 3]; consumers read stage
  // s-1 into registers and fold stage s-2 (read one iteration earlier).
  // Consumers and producers run separate copies of the row loop (same rows,
  // same iteration counts, one barrier per iteration) so that neither's
  // loop-invariant values occupy the other's registers.
  static_assert(D % 2 == 0, "consumer iterations come in pairs");
  // A row's features are independent chains: the row is split into column
  // groups of FW features, one block each, so a hub row's bytes spread over
  // ncg CUs (one CU moves ~50-60 GB/s through this pipeline).
  constexpr int FW = 4 * G;
  const int ncg = (a.F + FW - 1) / FW;
#define KGX_HUB_ROW(p)                                                  \
  const int64_t h = (p) / ncg;                                          \
  const int c0 = int((p) % ncg) * FW; /* first column of the group */   \
  const int fw = a.F - c0 < FW ? a.F - c0 : FW;                         \
  const int32_t row = a.rows[h];                                        \
  const int32_t beg = a.rowptr[row], end = a.rowptr[row + 1];           \
  if (end - beg < kLongRow) break; /* rows come in descending degree */ \
  const int32_t n_st = (end - beg + S - 1) / S;                         \
  const int32_t n_iter = (n_st + 2 + 2 * D - 1) / (2 * D) * (2 * D);

  if (wave < CW) {  // ---- consumers
    for (int64_t p = blockIdx.x; p < n_hub_items; p = next_item(p)) {
      KGX_HUB_ROW(p)
      claim_next();
      const int f = wave * 64 + lane;
      const int fc = f < RL ? f : RL - 1;
      float acc = R::init();
      // Iteration s reads stage s-1 into registers (one LDS read per two
      // edges) and folds stage s-2, read one iteration earlier, so the LDS
      // latency stays behind the add chain.  (Streaming the fold through a
      // short register ring -- one read per edge -- measured 1.7x slower:
      // the consumer wave is bound by its LDS instruction issue.)
      float va[S], vb[S];
      auto rd = [&](float(&v)[S], int32_t t) {
        const float* rb = &ring[t % 3][fc];
#pragma unroll
        for (int i = 0; i < S; ++i) v[i] = rb[i * RL];
      };
      auto fold = [&](const float(&v)[S], int32_t t) {
        if (t == n_st - 1) {  // the row's last stage: slots past `end` hold clamped duplicates
          const int32_t n = end - beg - t * S;
#pragma unroll
          for (int i = 0; i < S; ++i) acc = R::combine(acc, i < n ? v[i] : R::init());  // init(): exact identity
        } else {
#pragma unroll
          for (int i = 0; i < S; ++i) acc = R::combine(acc, v[i]);
        }
      };
      for (int32_t s = 0; s < n_iter; s += 2) {
        if (s >= 1 && s - 1 < n_st) rd(va, s - 1);
        __builtin_amdgcn_sched_barrier(0);  // the reads fly while the previous stage folds
        if (s >= 2 && s - 2 < n_st) fold(vb, s - 2);
        hub_barrier_reader();
        if (s < n_st) rd(vb, s);
        __builtin_amdgcn_sched_barrier(0);
        if (s >= 1 && s - 1 < n_st) fold(va, s - 1);
        hub_barrier_reader();
      }
      if (f < fw) {
        float r[1] = {a.epi == KGX_EPI_RAW ? R::finish_raw(acc, end - beg) : R::finish(acc, end - beg)};
        epilogue<1>(a, row, c0 + f, r);
        vstore<1>(a.out + int64_t(row) * a.ld_o + c0 + f, r);
      }
    }
    return;
  }

  // ---- producers: lane (slot r, features f..f+3) of every stage
  for (int64_t p = blockIdx.x; p < n_hub_items; p = next_item(p)) {
    KGX_HUB_ROW(p)
    const int slot = (wave - CW) * RPW + lane / G;
    if (__builtin_amdgcn_readfirstlane(slot) >= SP) {  // idle producer wave: barriers only
      for (int32_t s = 0; s < n_iter; ++s) hub_barrier();
      continue;
    }
    const int f = (lane % G) * 4;
    const int fl = f < fw ? f : fw - 4;  // lanes past the group load (and write) a valid duplicate
    const float* tab = a.table + c0 + fl;
    float* lds_row = &ring[0][slot * RL + f];
    auto edge = [&](int32_t t, int r) {  // stage t's edge of row r of this slot, clamped into the row
      const int32_t e = beg + t * S + r * SP + slot;
      return e < end ? e : end - 1;
    };
    int32_t ci[2][D][RPL];  // index batches: stages of chunk c in set c & 1
    f32x4_t gv[D][RPL];     // gathers in flight: stage t in gv[t % D]
    float wr[D][RPL];       // ... and their weights, loaded with them
    auto batch = [&](int set, int32_t chunk) {
#pragma unroll
      for (int j = 0; j < D; ++j)
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
          const int32_t* pi = a.idx + edge(chunk * D + j, r);
          asm volatile("global_load_dword %0, %1, off" : "=v"(ci[set][j][r]) : "v"(pi) : "memory");
        }
    };
    auto gather = [&](int j, int32_t t, const int32_t(&c)[RPL]) {  // weights, then rows, of stage t
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        if constexpr (WEIGHTED) {
          const float* pw = a.w + edge(t, r);
          asm volatile("global_load_dword %0, %1, off" : "=v"(wr[j][r]) : "v"(pw) : "memory");
        }
        const float* p = tab + row_off(c[r], a.ld_t);
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(gv[j][r]) : "v"(p) : "memory");
      }
    };
    auto pin_batch = [&](int set) {
#pragma unroll
      for (int j = 0; j < D; ++j)
#pragma unroll
        for (int r = 0; r < RPL; ++r) asm volatile("" : "+v"(ci[set][j][r]));
    };
    // vector-memory ops per iteration (weights + rows) and the vmcnt waits:
    // stage s's loads are the oldest we need; newer are the D-1 later
    // iterations' loads, plus (after the chunk's first iteration) its batch
    constexpr int OPI = RPL * (WEIGHTED ? 2 : 1);
    constexpr int NB = D * RPL;
    static_assert(OPI * (D - 1) + NB <= 63, "vmcnt immediate");
    // prologue: index batches of chunks 0 and 1, then the loads of stages 0..D-1
    batch(0, 0);
    batch(1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pin_batch(0);
    pin_batch(1);
#pragma unroll
    for (int j = 0; j < D; ++j) gather(j, j, ci[0][j]);
    // one chunk = D iterations; during chunk k the set holding chunk k+1's
    // indices issues the loads of stages (k+1)D.., and the other set is
    // refilled with chunk k+2 at the chunk's first iteration
    auto chunk = [&](int32_t k, auto use_c) {
      constexpr int use = decltype(use_c)::value, fill = 1 - use;
#pragma unroll
      for (int j = 0; j < D; ++j) {
        const int32_t s = k * D + j;
        if (j == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPI * (D - 1)) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPI * (D - 1) + NB) : "memory");
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
          asm volatile("" : "+v"(gv[j][r]));
          if constexpr (WEIGHTED) asm volatile("" : "+v"(wr[j][r]));
          f32x4_t m;
#pragma unroll
          for (int q = 0; q < 4; ++q) m[q] = R::msg(WEIGHTED ? __fmul_rn(gv[j][r][q], wr[j][r]) : gv[j][r][q]);
          *reinterpret_cast<f32x4_t*>(lds_row + (s % 3) * (S * RL) + r * (SP * RL)) = m;
        }
        if (j == 0) batch(fill, k + 2);
        gather(j, s + D, ci[use][j]);
        hub_barrier();
      }
      // the batch issued at j = 0 has landed (only this chunk's loads are
      // newer): the compiler may copy its registers at the loop's back edge
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPI * D) : "memory");
      pin_batch(fill);
    };
    // one exit, at the bottom, where the in-flight registers are exactly
    // those of the back edge (an exit between the two chunks made hipcc
    // shuffle still-loading registers)
    for (int32_t k = 0; k * D < n_iter; k += 2) {
      chunk(k, std::integral_constant<int, 1>{});
      chunk(k + 1, std::integral_constant<int, 0>{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no loads in flight past the row
    // Keep every asm-load destination live up to that wait: the last chunk's
    // loads are never consumed, and a dead destination register could be
    // handed to other code while its load is still in flight.
#pragma unroll
    for (int j = 0; j < D; ++j)
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        asm volatile("" ::"v"(gv[j][r]), "v"(ci[0][j][r]), "v"(ci[1][j][r]));
        if constexpr (WEIGHTED) asm volatile("" ::"v"(wr[j][r]));
      }
  }
#undef KGX_HUB_ROW
}

// The schedule's suffix of unsplit rows of degree <= KGX_SHORT_ROW_MAX (78 %
// of an R-MAT graph's rows, 11 % of its edges).  spmm_kernel's groups take one
// row per item, so on these rows a group has one or two gathers in flight and
// each row pays a chain of dependent loads (item, index, row) for 0.5-4 KB:
// NS rows of degree <= 7 ran at 5.1 TB/s against 7.7 TB/s for the rest
// (tools/exp_lowdeg.py spmm).  Here a group takes kSR consecutive items and
// gathers the first kSPF edges of all of them together (never exec-masked:
// absent edges read kgx_zero_row and are masked at the fold), the rest in
// pairs, each row still reduced in its CSR order.
constexpr int kSR = 4;
constexpr int kSPF = 2;

template <int VEC, int RED, bool WEIGHTED, bool TWO = false>
__global__ __launch_bounds__(kBlock) void spmm_short_kernel(SpmmArgs a) {
  using R = Reducer<RED>;
  const int G = a.G;
  const int lane = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t(gridDim.x) * kBlock) >> a.lgG;
  const int fo = lane * VEC;
  const bool fv = fo < a.F;
  const int fl = fv ? fo : a.F - VEC;
  // the schedule's items [n_long, n_items), or in EXACT mode rows [n_rows_long, n_rows)
  const int64_t s0 = a.items ? a.n_long : a.n_rows_long;
  const int64_t s1 = a.items ? a.n_items : a.n_rows;
  const int64_t n_short = s1 - s0;
  for (int64_t q = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> a.lgG; q * kSR < n_short; q += ngroups) {
    int32_t row[kSR], beg[kSR], deg[kSR];
#pragma unroll
    for (int r = 0; r < kSR; ++r) {
      const int64_t it = s0 + q * kSR + r;
      row[r] = -1;
      beg[r] = 0;
      deg[r] = 0;
      if (it < s1) {
        if (a.items) {
          const int4 v = a.items[it];
          row[r] = v.x;
          beg[r] = v.y;
          deg[r] = v.z - v.y;
        } else {
          row[r] = a.rows[it];
          beg[r] = a.rowptr[row[r]];
          deg[r] = a.rowptr[row[r] + 1] - beg[r];
        }
      }
    }
    float acc[kSR][VEC];
    {
      int32_t c[kSR][kSPF];
      float wt[kSR][kSPF];
#pragma unroll
      for (int r = 0; r < kSR; ++r)
#pragma unroll
        for (int u = 0; u < kSPF; ++u) {
          const int32_t ee = deg[r] > 0 ? beg[r] + (u < deg[r] ? u : deg[r] - 1) : 0;
          c[r][u] = a.idx[ee];
          if constexpr (WEIGHTED) wt[r][u] = a.w[ee];
        }
      float v[kSR][kSPF][VEC];
#pragma unroll
      for (int r = 0; r < kSR; ++r)
#pragma unroll
        for (int u = 0; u < kSPF; ++u)
          vload<VEC>(v[r][u], u < deg[r] ? tsrc<TWO>(a, c[r][u]) + fl : kgx_zero_row + fl);
#pragma unroll
      for (int r = 0; r < kSR; ++r)
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          float t = R::init();
#pragma unroll
          for (int u = 0; u < kSPF; ++u) {
            float m = v[r][u][k];
            if constexpr (WEIGHTED) m = __fmul_rn(m, wt[r][u]);
            t = R::combine(t, u < deg[r] ? R::msg(m) : R::init());
          }
          acc[r][k] = t;
        }
    }
#pragma unroll
    for (int r = 0; r < kSR; ++r) {
      for (int32_t e = kSPF; e < deg[r]; e += 2) {
        const int n = deg[r] - e;
        int32_t c[2];
        float wt[2], v[2][VEC];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int32_t ee = beg[r] + e + (u < n ? u : n - 1);
          c[u] = a.idx[ee];
          if constexpr (WEIGHTED) wt[u] = a.w[ee];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) vload<VEC>(v[u], tsrc<TWO>(a, c[u]) + fl);
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int k = 0; k < VEC; ++k) {
            float m = v[u][k];
            if constexpr (WEIGHTED) m = __fmul_rn(m, wt[u]);
            acc[r][k] = R::combine(acc[r][k], u < n ? R::msg(m) : R::init());
          }
      }
    }
    if (!fv) continue;
#pragma unroll
    for (int r = 0; r < kSR; ++r) {
      if (row[r] < 0) continue;
      float o[VEC];
#pragma unroll
      for (int k = 0; k < VEC; ++k)
        o[k] = a.epi == KGX_EPI_RAW ? R::finish_raw(acc[r][k], deg[r]) : R::finish(acc[r][k], deg[r]);
      epilogue<VEC>(a, row[r], fo, o);
      vstore<VEC>(a.out + int64_t(row[r]) * a.ld_o + fo, o);
    }
  }
}

// Combine the chunk partials of split rows in chunk order, then finish.
template <int VEC, int NT, int RED>
__global__ __launch_bounds__(kBlock) void spmm_fixup_kernel(SpmmArgs a) {
  using R = Reducer<RED>;
  const int G = a.G;
  const int lane = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t(gridDim.x) * kBlock) >> a.lgG;
  for (int64_t it = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> a.lgG; it < a.n_split; it += ngroups) {
    const int4 s = a.split[it];
    const int32_t row = s.x, slot0 = s.y, nc = s.z, deg = s.w;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int f = (t * G + lane) * VEC;
      if (f >= a.F) continue;
      float acc[VEC];
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] = R::init();
      // kFixB chunk loads in flight (clamped, unconditional), then the in-order
      // combine: a hub row's chain of ~100 partials is not ~100 serial latencies
      for (int32_t c0 = 0; c0 < nc; c0 += kFixB) {
        float p[kFixB][VEC];
#pragma unroll
        for (int u = 0; u < kFixB; ++u)
          vload<VEC>(p[u], a.partials + int64_t(slot0 + (c0 + u < nc ? c0 + u : nc - 1)) * a.ld_p + f);
#pragma unroll
        for (int u = 0; u < kFixB; ++u)
#pragma unroll
          for (int k = 0; k < VEC; ++k) acc[k] = c0 + u < nc ? R::combine(acc[k], p[u][k]) : acc[k];
      }
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] = a.epi == KGX_EPI_RAW ? R::finish_raw(acc[k], deg) : R::finish(acc[k], deg);
      epilogue<VEC>(a, row, f, acc);
      vstore<VEC>(a.out + int64_t(row) * a.ld_o + f, acc);
    }
  }
}

// StdAggregator (aggregators.py:182-228), two sequential passes per row, EXACT.
template <int VEC, int NT>
__global__ __launch_bounds__(kBlock) void spmm_std_kernel(SpmmArgs a) {
  const int G = a.G;
  const int lane = threadIdx.x & (G - 1);
  const int64_t ngroups = (int64_t(gridDim.x) * kBlock) >> a.lgG;
  for (int64_t it = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> a.lgG; it < a.n_rows; it += ngroups) {
    const int32_t row = a.rows[it];
    const int32_t beg = a.rowptr[row], end = a.rowptr[row + 1];
    const float cnt = ref_count_f32(end - beg);
    const float safe = fmaxf(cnt, 1e-8f);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int f = (t * G + lane) * VEC;
      if (f >= a.F) continue;
      float sum[VEC], ssd[VEC], mean[VEC];
#pragma unroll
      for (int k = 0; k < VEC; ++k) sum[k] = ssd[k] = 0.0f;
      for (int32_t e = beg; e < end; ++e) {
        float v[VEC];
        vload<VEC>(v, a.table + int64_t(a.idx[e]) * a.ld_t + f);
#pragma unroll
        for (int k = 0; k < VEC; ++k) sum[k] = __fadd_rn(sum[k], v[k]);
      }
#pragma unroll
      for (int k = 0; k < VEC; ++k) mean[k] = __fdiv_rn(sum[k], safe);
      for (int32_t e = beg; e < end; ++e) {
        float v[VEC];
        vload<VEC>(v, a.table + int64_t(a.idx[e]) * a.ld_t + f);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          const float d = __fsub_rn(v[k], mean[k]);
          ssd[k] = __fadd_rn(ssd[k], __fmul_rn(d, d));
        }
      }
      float r[VEC];
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        const float var = __fdiv_rn(ssd[k], safe);
        const float sd = sqrt_rn(fmaxf(var, 0.0f) /* maximum(variance, 0) */);
        r[k] = cnt <= 1.0f ? 0.0f : (var != var ? var : sd);
      }
      epilogue<VEC>(a, row, f, r);
      vstore<VEC>(a.out + int64_t(row) * a.ld_o + f, r);
    }
  }
}



template <int VEC, int NT, int RED, bool W, bool TWO = false>
int launch_main(const SpmmArgs& a_in, hipStream_t s) {
  SpmmArgs a = a_in;
  ForkJoin* joined = nullptr;
  JoinGuard guard;
  if constexpr (NT == 1) {
    static const bool hub_off = [] {
      const char* h = getenv("KGX_HUB");
      return h && atoi(h) == 0;
    }();
    if (VEC == 4 && !a.items && a.n_rows > 0 && !a.drop_key && a.G >= 8 && !hub_off) {
      a.long_rows = 1;  // EXACT: long rows first, one block per row
      const int gh = a.G < kHubG ? a.G : kHubG;  // column group = 4 x gh features
      auto kh = spmm_hub_kernel<64, RED, W>;
      if (gh == 32) kh = spmm_hub_kernel<32, RED, W>;
      else if (gh == 16) kh = spmm_hub_kernel<16, RED, W>;
      else if (gh == 8) kh = spmm_hub_kernel<8, RED, W>;
      const int64_t work = a.n_rows * ((a.F + 4 * gh - 1) / (4 * gh));
      const int64_t nb = work < cu_count() ? work : cu_count();  // one resident block per CU
      // KGX_EXACT_FORK=3 (default): the hub kernel forked beside spmm_kernel,
      // which runs on its full grid taking interleaved row batches from a
      // counter (one atomic per kDynRows rows), and the short-row kernel after
      // it, once the hub kernel's tail is over.  The hub kernel's mass of rows
      // ends in ~0.3 ms; its largest row then holds two CUs for ~1 ms, which
      // spmm_kernel's batches fill: NS EXACT aggregation 9.69-9.73 -> 8.96-8.98
      // ms (profiles/r04/exact_fork3_ab.jsonl).  0: sequential.  Measured and
      // removed (tools/experiments/round5_exact_fork_modes.patch): contiguous
      // row batches (12.7-65 ms against 10.9 static) and a grid cut to the
      // block slots the hub blocks leave (10.29-10.32 against 9.92-10.01 ms).
      static const int fork_mode = [] {
        const char* h = getenv("KGX_EXACT_FORK");
        return h ? atoi(h) : 3;
      }();
      const bool fork_on = fork_mode == 3;
      a.dyn_rows = fork_on ? 1 : 0;
      if (a.dyn && fork_on) {
        // dynamic pickup: the hub kernel runs on a forked stream BESIDE spmm_kernel
        // (which skips the hub rows and takes its rows from a counter), so the CUs
        // the hub kernel's tail leaves idle -- its largest row alone is ~1 ms at
        // NS -- run ordinary rows instead of waiting; joined back below.
        ForkJoin& fj = fork_join();
        if (hipEventRecord(fj.fork, s) != hipSuccess || hipStreamWaitEvent(fj.side, fj.fork, 0) != hipSuccess) {
          set_error("kgx_spmm: stream fork failed");
          return KGX_ERR_HIP;
        }
        hipLaunchKernelGGL(kh, dim3(unsigned(nb)), dim3(kHubThreads), 0, fj.side, a);
        KGX_CHECK_LAUNCH();
        if (hipEventRecord(fj.join, fj.side) != hipSuccess) {
          set_error("kgx_spmm: stream join failed");
          return KGX_ERR_HIP;
        }
        joined = &fj;
        guard.fj = &fj;
        guard.s = s;
      } else {
        hipLaunchKernelGGL(kh, dim3(unsigned(nb)), dim3(kHubThreads), 0, s, a);
        KGX_CHECK_LAUNCH();
      }
    } else if (!a.items && a.n_rows > 0) {  // EXACT: long rows first, on their own kernel
      a.long_rows = 1;
      auto kl = spmm_long_kernel<VEC, RED, W>;
      if constexpr (RED == KGX_SUM) {
        if (a.drop_key) kl = spmm_long_kernel<VEC, RED, W, true>;
      }
      const int64_t cand = a.n_rows < 16384 ? a.n_rows : 16384;
      hipLaunchKernelGGL(kl, dim3(resident_grid(kl, cand, a.G)), dim3(kBlock), 0, s, a);
      KGX_CHECK_LAUNCH();
    }
  }
  bool short_on = false;
  int64_t n_short = 0;
  if constexpr (NT == 1) {
    n_short = a.items ? a.n_items - a.n_long : a.n_rows - a.n_rows_long;
    short_on = n_short > 0 && !a.drop_key;
  }
  if (!short_on) {
    a.n_long = a.n_items;
    a.n_rows_long = a.n_rows;
  }
  auto launch_short = [&]() -> int {
    if constexpr (NT == 1) {
      if (short_on) {
        auto ks = spmm_short_kernel<VEC, RED, W, TWO>;
        hipLaunchKernelGGL(ks, dim3(resident_grid(ks, (n_short + kSR - 1) / kSR, a.G)), dim3(kBlock), 0, s, a);
        KGX_CHECK_LAUNCH();
      }
    }
    return KGX_OK;
  };
  // the short-row kernel first, except beside a forked hub kernel whose rows
  // spmm_kernel's dynamic batches work around (KGX_EXACT_FORK=3)
  const bool short_last = a.dyn_rows && joined;
  if (!short_last && launch_short() != KGX_OK) return KGX_ERR_HIP;
  const int64_t work_long = a.items ? a.n_long : a.n_rows_long;
  if (work_long > 0) {
    auto k = spmm_kernel<VEC, NT, RED, W, false, TWO>;
    if constexpr (RED == KGX_SUM && !TWO) {
      if (a.drop_key) k = spmm_kernel<VEC, NT, RED, W, true>;
    }
    hipLaunchKernelGGL(k, dim3(resident_grid(k, work_long, a.G)), dim3(kBlock), 0, s, a);
    KGX_CHECK_LAUNCH();
  }
  if (short_last && launch_short() != KGX_OK) return KGX_ERR_HIP;
  if (joined) {
    guard.fj = nullptr;  // joined here, with the status checked
    if (hipStreamWaitEvent(s, joined->join, 0) != hipSuccess) {
      set_error("kgx_spmm: stream join failed");
      return KGX_ERR_HIP;
    }
  }
  if (a.items && a.n_split > 0) {
    auto k = spmm_fixup_kernel<VEC, NT, RED>;
    hipLaunchKernelGGL(k, dim3(resident_grid(k, a.n_split, a.G)), dim3(kBlock), 0, s, a);
    KGX_CHECK_LAUNCH();
  }
  return KGX_OK;
}

template <int VEC, int NT, int RED>
int dispatch_w(const SpmmArgs& a, hipStream_t s) {
  if (RED == KGX_STD) {
    if (a.n_rows > 0) {
      auto k = spmm_std_kernel<VEC, NT>;
      hipLaunchKernelGGL(k, dim3(resident_grid(k, a.n_rows, a.G)), dim3(kBlock), 0, s, a);
      KGX_CHECK_LAUNCH();
    }
    return KGX_OK;
  }
  constexpr int RR = RED == KGX_STD ? KGX_SUM : RED;
  if constexpr (RR == KGX_SUM) {
    if (a.n_t1 != INT32_MAX)  // two tables: plain / weighted sums (the sharded layers' merged pass)
      return a.w ? launch_main<VEC, NT, RR, true, true>(a, s) : launch_main<VEC, NT, RR, false, true>(a, s);
  }
  return a.w ? launch_main<VEC, NT, RR, true>(a, s) : launch_main<VEC, NT, RR, false>(a, s);
}

template <int VEC, int NT>
int dispatch_red(int red, const SpmmArgs& a, hipStream_t s) {
  switch (red) {
    case KGX_SUM: return dispatch_w<VEC, NT, KGX_SUM>(a, s);
    case KGX_MEAN: return dispatch_w<VEC, NT, KGX_MEAN>(a, s);
    case KGX_MAX: return dispatch_w<VEC, NT, KGX_MAX>(a, s);
    case KGX_MIN: return dispatch_w<VEC, NT, KGX_MIN>(a, s);
    case KGX_STD: return dispatch_w<VEC, NT, KGX_STD>(a, s);
  }
  set_error("kgx_spmm: unknown reduce %d", red);
  return KGX_ERR_ARG;
}

template <int VEC>
int dispatch_nt(int nt, int red, const SpmmArgs& a, hipStream_t s) {
  if (nt == 1) return dispatch_red<VEC, 1>(red, a, s);
  if (nt == 2) return dispatch_red<VEC, 2>(red, a, s);
  return dispatch_red<VEC, 4>(red, a, s);
}

bool aligned(const void* p, int bytes) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % bytes == 0; }

}  // namespace
}  // namespace kgx

using namespace kgx;

extern "C" int kgx_spmm(int reduce, int epilogue, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                        const int32_t* items, int64_t n_items, const int32_t* split, int64_t n_split,
                        const int32_t* idx, const float* w, const float* table, int64_t ld_table, int64_t F,
                        float* out, int64_t ld_out, const float* bias, const float* xroot, int64_t ld_x,
                        float gin_scale, const int32_t* drop_key, float drop_p, uint64_t drop_seed,
                        float* partials, kgx_stream_t stream_) {
  return kgx_spmm_ex(reduce, epilogue, rowptr, rows, n_rows, items, n_items, n_items, split, n_split, idx, w, table,
                     ld_table, F, out, ld_out, bias, xroot, ld_x, gin_scale, drop_key, drop_p, drop_seed, partials,
                     stream_);
}

extern "C" int kgx_spmm_ex(int reduce, int epilogue, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                           const int32_t* items, int64_t n_items, int64_t n_long_items, const int32_t* split,
                           int64_t n_split, const int32_t* idx, const float* w, const float* table, int64_t ld_table,
                           int64_t F, float* out, int64_t ld_out, const float* bias, const float* xroot,
                           int64_t ld_x, float gin_scale, const int32_t* drop_key, float drop_p, uint64_t drop_seed,
                           float* partials, kgx_stream_t stream_) {
  return kgx_spmm_ex2(reduce, epilogue, rowptr, rows, n_rows, items, n_items, n_long_items, split, n_split, idx, w,
                      table, ld_table, nullptr, 0, F, out, ld_out, bias, xroot, ld_x, gin_scale, drop_key, drop_p,
                      drop_seed, partials, nullptr, stream_);
}

extern "C" int kgx_spmm_ex2(int reduce, int epilogue, const int32_t* rowptr, const int32_t* rows, int64_t n_rows,
                            const int32_t* items, int64_t n_items, int64_t n_long_items, const int32_t* split,
                            int64_t n_split, const int32_t* idx, const float* w, const float* table, int64_t ld_table,
                            const float* table2, int64_t n_table1, int64_t F, float* out, int64_t ld_out,
                            const float* bias, const float* xroot, int64_t ld_x, float gin_scale,
                            const int32_t* drop_key, float drop_p, uint64_t drop_seed, float* partials,
                            int32_t* counters, kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(!table2 || (n_table1 >= 0 && n_table1 < (int64_t(1) << 31) && items), KGX_ERR_ARG,
              "kgx_spmm: a second table needs 0 <= n_table1 < 2^31 and the schedule (not EXACT mode)");
  KGX_REQUIRE(!table2 || (reduce == KGX_SUM && !drop_key), KGX_ERR_UNSUPPORTED,
              "kgx_spmm: two-table gathers are implemented for plain / weighted sums");
  KGX_REQUIRE(!items || (n_long_items >= 0 && n_long_items <= n_items), KGX_ERR_ARG,
              "kgx_spmm: n_long_items must lie in [0, n_items]");
  KGX_REQUIRE(reduce >= KGX_SUM && reduce <= KGX_STD, KGX_ERR_ARG, "kgx_spmm: unknown reduce %d", reduce);
  KGX_REQUIRE(epilogue >= KGX_EPI_NONE && epilogue <= KGX_EPI_ACCUM, KGX_ERR_ARG, "kgx_spmm: unknown epilogue %d",
              epilogue);
  KGX_REQUIRE(epilogue != KGX_EPI_ACCUM || reduce == KGX_SUM, KGX_ERR_ARG,
              "kgx_spmm: KGX_EPI_ACCUM accumulates plain sums only (got reduce %d)", reduce);
  KGX_REQUIRE(F >= 0 && n_rows >= 0 && n_items >= 0 && n_split >= 0, KGX_ERR_ARG, "kgx_spmm: negative size");
  if (F == 0 || n_rows == 0) return KGX_OK;
  KGX_REQUIRE(out && ld_out >= F && ld_table >= F, KGX_ERR_ARG, "kgx_spmm: bad output / leading dimensions");
  KGX_REQUIRE(ld_table < (int64_t(1) << 31), KGX_ERR_ARG, "kgx_spmm: table leading dimension >= 2^31");
  KGX_REQUIRE(rowptr && rows && idx && table, KGX_ERR_ARG, "kgx_spmm: null CSR / table pointer");
  KGX_REQUIRE(epilogue != KGX_EPI_BIAS || bias, KGX_ERR_ARG, "kgx_spmm: EPI_BIAS needs bias");
  KGX_REQUIRE(epilogue != KGX_EPI_GIN || (xroot && ld_x >= F), KGX_ERR_ARG, "kgx_spmm: EPI_GIN needs xroot");
  KGX_REQUIRE(!drop_key || (reduce == KGX_SUM && drop_p >= 0.0f && drop_p < 1.0f), KGX_ERR_ARG,
              "kgx_spmm: message dropout needs reduce SUM and 0 <= p < 1 (got reduce %d, p %g)", reduce,
              double(drop_p));
  const bool use_items = items != nullptr && reduce != KGX_STD;
  KGX_REQUIRE(!use_items || n_split == 0 || (split && partials), KGX_ERR_ARG,
              "kgx_spmm: split rows need split list and partials");

  SpmmArgs a{};
  a.rowptr = rowptr;
  a.rows = rows;
  a.n_rows = n_rows;
  a.items = use_items ? reinterpret_cast<const int4*>(items) : nullptr;
  a.n_items = use_items ? n_items : 0;
  a.split = reinterpret_cast<const int4*>(split);
  a.n_split = use_items ? n_split : 0;
  a.n_long = use_items ? n_long_items : 0;
  // EXACT mode: 0 < n_long_items < n_rows names the short-row suffix of the degree-ordered rows
  a.n_rows_long = (!use_items && reduce != KGX_STD && n_long_items > 0 && n_long_items < n_rows) ? n_long_items : n_rows;
  a.idx = idx;
  a.w = w;
  a.epi = epilogue;
  a.gin_scale = gin_scale;
  a.ld_t = ld_table;
  a.ld_o = ld_out;
  a.ld_x = ld_x;
  a.ld_p = F;
  static const int hints = [] {
    const char* h = getenv("KGX_SPMM_HINTS");
    return h ? atoi(h) : 0;
  }();
  a.hints = hints;
  if (drop_key && drop_p > 0.0f) {
    a.drop_key = drop_key;
    a.drop_seed = drop_seed;
    a.drop_thresh = uint32_t(double(drop_p) * 4294967296.0);
    a.drop_scale = 1.0f / (1.0f - drop_p);
  }

  // widest vector the shapes and pointers allow
  a.n_t1 = table2 ? int32_t(n_table1) : INT32_MAX;
  a.dyn = (!use_items && reduce != KGX_STD) ? counters : nullptr;
  auto ok = [&](int v) {
    const int b = 4 * v;
    return F % v == 0 && ld_table % v == 0 && ld_out % v == 0 && aligned(table, b) && aligned(out, b) &&
           (!table2 || aligned(table2, b)) &&
           (epilogue != KGX_EPI_BIAS || aligned(bias, b)) &&
           (epilogue != KGX_EPI_GIN || (ld_x % v == 0 && aligned(xroot, b))) && aligned(partials, b);
  };
  const int VEC = ok(4) ? 4 : (ok(2) ? 2 : 1);
  const int64_t fvec = F / VEC;
  const int G = int(fvec >= 64 ? 64 : next_pow2(int(fvec)));
  int lg = 0;
  while ((1 << lg) < G) ++lg;
  // column slices of at most 4*64*VEC features per launch
  const int64_t slice = int64_t(4) * 64 * VEC;
  for (int64_t c0 = 0; c0 < F; c0 += slice) {
    const int64_t cw = (F - c0) < slice ? (F - c0) : slice;
    const int64_t cv = cw / VEC;
    const int nt = cv <= 64 ? 1 : (cv <= 128 ? 2 : 4);
    SpmmArgs s = a;
    s.F = int(cw);
    s.G = G;
    s.lgG = lg;
    s.table = table + c0;
    // table2 - n_t1 * ld_t (+ the slice's first column), as an address; tsrc adds row_off(c)
    s.t2b = table2 ? reinterpret_cast<const float*>(reinterpret_cast<uintptr_t>(table2 + c0) -
                                                    uintptr_t(n_table1) * uintptr_t(ld_table) * sizeof(float))
                   : s.table;
    s.out = out + c0;
    s.bias = bias ? bias + c0 : nullptr;
    s.xroot = xroot ? xroot + c0 : nullptr;
    s.partials = partials ? partials + c0 : nullptr;
    s.f_base = int(c0);
    if (s.dyn && c0 > 0 && hipMemsetAsync(s.dyn, 0, 2 * sizeof(int32_t), stream) != hipSuccess) {
      set_error("kgx_spmm: counter reset failed");  // each column slice hands its rows out again
      return KGX_ERR_HIP;
    }
    int rc;
    if (VEC == 4) rc = dispatch_nt<4>(nt, reduce, s, stream);
    else if (VEC == 2) rc = dispatch_nt<2>(nt, reduce, s, stream);
    else rc = dispatch_nt<1>(nt, reduce, s, stream);
    if (rc != KGX_OK) return rc;
  }
  return KGX_OK;
}
