// Graph preparation for the kgx aggregation engine (gfx950).
//
//   COO [2,E] -> stable CSR by destination  (kgx_csr_build)
//   degree-ordered row schedule + hub split (kgx_schedule_build)
//   R-MAT synthetic edges                    (kgx_rmat_edges)
//   dst-range shard selection, row gather, scatter utilities
//
// The CSR order is the order the reference accumulates in: Keras-3's torch
// segment_sum is `scatter_add` over edges in input order (probed: bit-identical
// to sequential accumulation), so a STABLE sort by destination reproduces the
// per-destination message sequence, and add_self_loops (utils/main.py:8-16)
// appends loop i after all input edges, i.e. last in row i.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "kgx_internal.h"
#include "kgx_vec.h"

namespace kgx {
namespace {

// --------------------------------------------------------------------------
// CSR build kernels
// --------------------------------------------------------------------------
struct CsrStatus {
  unsigned long long bad;      // out-of-range indices
  unsigned long long max_deg;  // max in-degree
  unsigned long long kept;     // rowptr[n_dst]
  unsigned long long table_miss;  // rows whose fp32 degree the dinv table does not cover
};

__global__ void csr_prep_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                int64_t E, int64_t n_src, int64_t n_dst, int flags,
                                uint32_t* __restrict__ keys, uint64_t* __restrict__ vals,
                                CsrStatus* __restrict__ st) {
  const bool segment_only = flags & KGX_CSR_SEGMENT_ONLY;
  const bool loops = flags & KGX_CSR_SELF_LOOPS;
  const int64_t total = E + (loops ? n_dst : 0);
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  unsigned long long bad = 0;
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < total; e += stride) {
    if (e < E) {
      int64_t s = src[e];
      int64_t d = dst[e];
      bool keep;
      if (segment_only) {
        // segment_sum semantics: ids < 0 or >= num_segments go to a dropped bucket
        keep = (d >= 0) && (d < n_dst);
      } else {
        // take(x, idx): negative ids wrap, ids outside [-n, n) raise
        const bool bad_e = (s < -n_src) || (s >= n_src) || (d < -n_dst) || (d >= n_dst);
        bad += bad_e;
        keep = !bad_e && d >= 0;
        if (s < 0) s += n_src;
      }
      keys[e] = keep ? uint32_t(d) : uint32_t(n_dst);
      vals[e] = (uint64_t(uint32_t(s)) << 32) | uint32_t(e);  // {input edge id, wrapped source}
    } else {
      const int64_t i = e - E;
      keys[e] = uint32_t(i);
      vals[e] = (uint64_t(uint32_t(i)) << 32) | uint32_t(e);
    }
  }
  if (bad) atomicAdd(&st->bad, bad);
}

// rowptr[r] = lower_bound(keys_sorted, r) for r in [0, n_dst]
__global__ void csr_rowptr_kernel(const uint32_t* __restrict__ keys, int64_t total, int64_t n_dst,
                                  int32_t* __restrict__ rowptr, CsrStatus* __restrict__ st) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t r = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; r <= n_dst; r += stride) {
    int64_t lo = 0, hi = total;
    const uint32_t key = uint32_t(r);
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < key) lo = mid + 1; else hi = mid;
    }
    rowptr[r] = int32_t(lo);
    if (r == n_dst) st->kept = (unsigned long long)lo;
  }
}

// The sorted {input edge id, source} pairs -> eid[e] and col[e] (the source of
// every CSR slot), and with NORM the GCN edge norm w[e] = dinv[dst(e)] *
// dinv[col[e]] (utils/main.py:29-32, take(dinv, target) * take(dinv, source))
// in the same pass.  The source travels through the sort with the edge id, so
// only dinv[col] is a random read (a 4-byte read from the n-entry dinv table);
// each thread takes kColIlp slots per iteration (coalesced across the block)
// and issues their loads before the first use.
constexpr int kColIlp = 4;

template <bool NORM>
__global__ void csr_col_kernel(const uint64_t* __restrict__ vals_sorted, const uint32_t* __restrict__ keys_sorted,
                               const int32_t* __restrict__ rowptr, int64_t n_dst, const float* __restrict__ dinv,
                               int32_t* __restrict__ eid, int32_t* __restrict__ col, float* __restrict__ w) {
  const int64_t kept = rowptr[n_dst];
  if (kept <= 0) return;
  const int64_t chunk = int64_t(blockDim.x) * kColIlp;
  for (int64_t base = int64_t(blockIdx.x) * chunk; base < kept; base += int64_t(gridDim.x) * chunk) {
    uint64_t v[kColIlp];
#pragma unroll
    for (int j = 0; j < kColIlp; ++j) {
      const int64_t e = base + int64_t(j) * blockDim.x + threadIdx.x;
      v[j] = vals_sorted[e < kept ? e : kept - 1];
    }
    if constexpr (NORM) {
      float dd[kColIlp], ds[kColIlp];
#pragma unroll
      for (int j = 0; j < kColIlp; ++j) {
        const int64_t e = base + int64_t(j) * blockDim.x + threadIdx.x;
        dd[j] = dinv[keys_sorted[e < kept ? e : kept - 1]];
        ds[j] = dinv[int32_t(v[j] >> 32)];
      }
#pragma unroll
      for (int j = 0; j < kColIlp; ++j) {
        const int64_t e = base + int64_t(j) * blockDim.x + threadIdx.x;
        if (e < kept) w[e] = __fmul_rn(dd[j], ds[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < kColIlp; ++j) {
      const int64_t e = base + int64_t(j) * blockDim.x + threadIdx.x;
      if (e < kept) {
        eid[e] = int32_t(uint32_t(v[j]));
        col[e] = int32_t(v[j] >> 32);
      }
    }
  }
}

// Integer in-degree; fp32 degree as the reference computes it: a sequential
// fp32 sum of ones (utils/main.py:23-24, aggregators.py:66-69) saturates at 2^24.

__device__ __forceinline__ float gcn_dinv(int32_t d) {
  // pow(deg + 1e-12, -0.5), correctly rounded (= 1/sqrt in IEEE RN); deg 0 -> 1e6.
  return __fdiv_rn(1.0f, sqrt_rn(__fadd_rn(ref_count_f32(d), 1e-12f)));
}

// dinv from the caller's table of the reference's own values: table[k] =
// (float(k) + 1e-12f)^-0.5 as ATen's tensor-exponent pow evaluates it
// (utils/main.py:25 -> keras.ops.power -> torch.pow(Tensor, Tensor); built on
// the host by graph.gcn_dinv_table).  The index is the fp32 count, which
// saturates at 2^24 (ref_count_f32).  A degree past the table counts as a miss
// and takes the correctly-rounded value; the caller then redoes dinv with a
// longer table (kgx_gcn_dinv_table).
__device__ __forceinline__ float gcn_dinv_lookup(int32_t d, const float* __restrict__ table, int64_t len,
                                                 unsigned* miss) {
  const int64_t k = d < (1 << 24) ? d : (1 << 24);
  if (k < len) return table[k];
  *miss += 1;
  return gcn_dinv(d);
}

__global__ void csr_deg_kernel(const int32_t* __restrict__ rowptr, int64_t n_dst, int flags,
                               int32_t* __restrict__ deg, float* __restrict__ dinv,
                               const float* __restrict__ table, int64_t table_len,
                               CsrStatus* __restrict__ st) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  unsigned long long mx = 0;
  unsigned miss = 0;
  for (int64_t r = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < n_dst; r += stride) {
    const int32_t d = rowptr[r + 1] - rowptr[r];
    deg[r] = d;
    mx = d > (int64_t)mx ? (unsigned long long)d : mx;
    if (flags & KGX_CSR_GCN_NORM) dinv[r] = table ? gcn_dinv_lookup(d, table, table_len, &miss) : gcn_dinv(d);
  }
  // wave max, then block max, then one atomic per block (per-wave atomics on one address
  // serialised at the L2: 0.39 ms at NS for a 0.1 GB pass)
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long other = __shfl_xor(mx, o, 64);
    mx = other > mx ? other : mx;
    miss += __shfl_xor(miss, o, 64);
  }
  __shared__ unsigned long long red_mx[kBlock / 64];
  __shared__ unsigned red_miss[kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    red_mx[threadIdx.x >> 6] = mx;
    red_miss[threadIdx.x >> 6] = miss;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < kBlock / 64; ++k) {
      mx = red_mx[k] > mx ? red_mx[k] : mx;
      miss += red_miss[k];
    }
    if (mx) atomicMax(&st->max_deg, mx);
    if (miss) atomicAdd(&st->table_miss, (unsigned long long)miss);
  }
}

size_t sort_temp_bytes(int64_t n, int end_bit) {
  size_t bytes = 0;
  uint32_t* k = nullptr;
  int32_t* v = nullptr;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, k, k, v, v, (unsigned)n, 0, end_bit, 0, false);
  return bytes;
}

size_t sort_temp_bytes64(int64_t n, int end_bit) {
  size_t bytes = 0;
  uint32_t* k = nullptr;
  uint64_t* v = nullptr;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, k, k, v, v, (unsigned)n, 0, end_bit, 0, false);
  return bytes;
}

struct CsrLayout {
  uint32_t* keys;
  uint32_t* keys_sorted;
  uint64_t* vals;         // {input edge id, source} per edge
  uint64_t* vals_sorted;
  CsrStatus* st;
  void* sort_tmp;
  size_t sort_bytes;
  size_t total;
};

CsrLayout csr_layout(void* ws, int64_t total, int64_t n_dst) {
  Carve c(ws, ~size_t(0));
  CsrLayout L;
  L.keys = c.take<uint32_t>(total);
  L.keys_sorted = c.take<uint32_t>(total);
  L.vals = c.take<uint64_t>(total);
  L.vals_sorted = c.take<uint64_t>(total);
  L.st = c.take<CsrStatus>(1);
  const int end_bit = ceil_log2_u64(uint64_t(n_dst) + 1);
  L.sort_bytes = sort_temp_bytes64(total, end_bit > 0 ? end_bit : 1);
  L.sort_tmp = c.take<char>(L.sort_bytes);
  L.total = c.used();
  return L;
}

__global__ void gcn_dinv_kernel(const int32_t* __restrict__ deg, int64_t n, float* __restrict__ dinv) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) dinv[i] = gcn_dinv(deg[i]);
}

__global__ void gcn_dinv_table_kernel(const int32_t* __restrict__ deg, int64_t n, const float* __restrict__ table,
                                      int64_t len, float* __restrict__ dinv) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int32_t d = deg[i];
    const int64_t k = d < (1 << 24) ? d : (1 << 24);
    dinv[i] = table[k < len ? k : len - 1];  // the caller covers max(deg) (kgx.h)
  }
}

// w_e = dinv_dst[row(e)] * dinv_src[col[e]].  A group of 8 lanes per row
// (8 rows per wave: most rows of a power-law graph have a few edges); rows of
// degree > 64 are left to the wave pass below, which strides a whole wave
// over them, so a hub row does not serialise on 8 lanes.
__global__ void gcn_edge_norm_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                     int64_t n_dst, const float* __restrict__ dinv_dst,
                                     const float* __restrict__ dinv_src, float* __restrict__ w) {
  const int sub = threadIdx.x & 7;
  const int64_t ng = (int64_t(gridDim.x) * blockDim.x) >> 3;
  for (int64_t r = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 3; r < n_dst; r += ng) {
    const int32_t b = rowptr[r], e1 = rowptr[r + 1];
    if (e1 - b > 64) continue;
    const float dr = dinv_dst[r];
    for (int32_t e = b + sub; e < e1; e += 8) w[e] = __fmul_rn(dr, dinv_src[col[e]]);
  }
}

__global__ void gcn_edge_norm_long_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                          int64_t n_dst, const float* __restrict__ dinv_dst,
                                          const float* __restrict__ dinv_src, float* __restrict__ w) {
  // each wave scans 64 rows at a time (one per lane) and takes the rows of degree > 64 one
  // after another with all its lanes
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t r0 = ((int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6) * 64; r0 < n_dst; r0 += nw * 64) {
    const int64_t r = r0 + lane;
    const int32_t b = r < n_dst ? rowptr[r] : 0, e1 = r < n_dst ? rowptr[r + 1] : 0;
    unsigned long long long_rows = __ballot(e1 - b > 64);
    while (long_rows) {
      const int k = __ffsll(long_rows) - 1;
      long_rows &= long_rows - 1;
      const int32_t bk = __shfl(b, k, 64), ek = __shfl(e1, k, 64);
      const float dr = dinv_dst[r0 + k];
      for (int32_t e = bk + lane; e < ek; e += 64) w[e] = __fmul_rn(dr, dinv_src[col[e]]);
    }
  }
}

// --------------------------------------------------------------------------
// Schedule kernels
// --------------------------------------------------------------------------
// Rows are scheduled in descending exact degree (stable: ascending row id
// among equal degrees).  The fused kernel reduces 16 consecutive items in
// lock-step, so equal-length neighbours matter: exact order measured 2.8 %
// faster than log2 degree buckets at NS.  Degrees >= 2^24 tie (such rows are
// split into chunks anyway).
constexpr int kDegKeyBits = 24;
__device__ __forceinline__ uint32_t degree_key(int32_t d) {
  const uint32_t c = uint32_t(d) < (1u << kDegKeyBits) ? uint32_t(d) : (1u << kDegKeyBits) - 1u;
  return ((1u << kDegKeyBits) - 1u) - c;
}

__global__ void sched_keys_kernel(const int32_t* __restrict__ rowptr, int64_t n_dst,
                                  uint32_t* __restrict__ keys, int32_t* __restrict__ iota) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t r = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < n_dst; r += stride) {
    keys[r] = degree_key(rowptr[r + 1] - rowptr[r]);
    iota[r] = int32_t(r);
  }
}

__global__ void sched_count_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ rows,
                                   int64_t n_dst, int32_t split_len, int32_t* __restrict__ nchunks,
                                   int32_t* __restrict__ nslots) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n_dst; i += stride) {
    const int32_t r = rows[i];
    const int32_t d = rowptr[r + 1] - rowptr[r];
    const bool split = split_len > 0 && d >= split_len;
    const int32_t nc = split ? (d + split_len - 1) / split_len : 1;
    nchunks[i] = nc;
    nslots[i] = split ? nc : 0;
  }
}

struct SchedStatus {
  unsigned long long n_items;
  unsigned long long n_split;
  unsigned long long n_slots;
  unsigned long long overflow;
};

__global__ void sched_emit_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ rows,
                                  int64_t n_dst, int32_t split_len,
                                  const int32_t* __restrict__ nchunks, const int32_t* __restrict__ item_off,
                                  const int32_t* __restrict__ nslots, const int32_t* __restrict__ slot_off,
                                  int4* __restrict__ items, int64_t cap_items, int4* __restrict__ split,
                                  SchedStatus* __restrict__ st) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  unsigned long long nsplit = 0;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n_dst; i += stride) {
    const int32_t r = rows[i];
    const int32_t beg = rowptr[r];
    const int32_t end = rowptr[r + 1];
    const int32_t nc = nchunks[i];
    const int32_t off = item_off[i];
    if (int64_t(off) + nc > cap_items) {
      atomicAdd(&st->overflow, 1ull);
      continue;
    }
    if (nslots[i] > 0) {
      const int32_t s0 = slot_off[i];
      for (int32_t c = 0; c < nc; ++c) {
        const int32_t b = beg + c * split_len;
        const int32_t e = min(end, b + split_len);
        items[off + c] = make_int4(r, b, e, s0 + c);
      }
      split[i] = make_int4(r, s0, nc, end - beg);  // split rows are a schedule prefix
      ++nsplit;
    } else {
      items[off] = make_int4(r, beg, end, -1);
    }
    if (i == n_dst - 1) {
      st->n_items = (unsigned long long)(off + nc);
      st->n_slots = (unsigned long long)(slot_off[i] + nslots[i]);
    }
  }
  if (nsplit) atomicAdd(&st->n_split, nsplit);
}

struct SchedLayout {
  uint32_t* keys;
  uint32_t* keys_sorted;
  int32_t* iota;
  int32_t* nchunks;
  int32_t* item_off;
  int32_t* nslots;
  int32_t* slot_off;
  SchedStatus* st;
  void* tmp;
  size_t tmp_bytes;
  size_t total;
};

SchedLayout sched_layout(void* ws, int64_t n) {
  Carve c(ws, ~size_t(0));
  SchedLayout L;
  L.keys = c.take<uint32_t>(n);
  L.keys_sorted = c.take<uint32_t>(n);
  L.iota = c.take<int32_t>(n);
  L.nchunks = c.take<int32_t>(n);
  L.item_off = c.take<int32_t>(n);
  L.nslots = c.take<int32_t>(n);
  L.slot_off = c.take<int32_t>(n);
  L.st = c.take<SchedStatus>(1);
  size_t sb = sort_temp_bytes(n, kDegKeyBits);
  size_t scb = 0;
  const int32_t* si = nullptr;
  int32_t* so = nullptr;
  (void)rocprim::exclusive_scan(nullptr, scb, si, so, 0, (size_t)n, rocprim::plus<int32_t>(), 0, false);
  L.tmp_bytes = sb > scb ? sb : scb;
  L.tmp = c.take<char>(L.tmp_bytes);
  L.total = c.used();
  return L;
}

// --------------------------------------------------------------------------
// R-MAT generator (counter-based; restated bit-for-bit in oracle/rmat.py)
// --------------------------------------------------------------------------
__device__ __host__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Feistel {
  uint64_t keys[4];
  int hb;          // half width in bits
  uint64_t mask;   // (1 << hb) - 1
};

__device__ __forceinline__ uint64_t feistel_once(const Feistel& f, uint64_t x) {
  uint64_t L = x >> f.hb, R = x & f.mask;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint64_t nl = R;
    R = L ^ (splitmix64(f.keys[i] ^ R) & f.mask);
    L = nl;
  }
  return (L << f.hb) | R;
}

__device__ __forceinline__ uint64_t relabel(const Feistel& f, uint64_t x, uint64_t n) {
  uint64_t y = feistel_once(f, x);
  while (y >= n) y = feistel_once(f, y);  // cycle walking: terminates (bijection on a superset)
  return y;
}

__global__ void rmat_kernel(uint64_t base, Feistel fs, int scale, uint64_t n,
                            uint32_t ta, uint32_t tab, uint32_t tabc,
                            int64_t e_begin, int64_t e_count,
                            int32_t* __restrict__ src, int32_t* __restrict__ dst) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < e_count; i += stride) {
    const uint64_t k = uint64_t(e_begin + i);
    uint64_t s = 0, d = 0;
    for (int l = 0; l < scale; ++l) {
      const uint32_t r = uint32_t(splitmix64(base + k * 64ull + uint64_t(l)) >> 40);
      const uint32_t sb = r >= tab;                       // quadrants c, d
      const uint32_t db = (r >= ta && r < tab) || r >= tabc;  // quadrants b, d
      s = (s << 1) | sb;
      d = (d << 1) | db;
    }
    src[i] = int32_t(relabel(fs, s % n, n));
    dst[i] = int32_t(relabel(fs, d % n, n));
  }
}

// --------------------------------------------------------------------------
// small utilities
// --------------------------------------------------------------------------
__global__ void range_flags_kernel(const int32_t* __restrict__ dst, int64_t n, int64_t lo, int64_t hi,
                                   int32_t* __restrict__ flags) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t d = dst[i];
    flags[i] = (d >= lo && d < hi) ? 1 : 0;
  }
}

__global__ void range_scatter_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                     const int32_t* __restrict__ flags, const int32_t* __restrict__ pos,
                                     int64_t n, int32_t* __restrict__ so, int32_t* __restrict__ dout,
                                     unsigned long long* __restrict__ count) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (flags[i]) {
      so[pos[i]] = src[i];
      dout[pos[i]] = dst[i];
    }
    if (i == n - 1) *count = (unsigned long long)(pos[i] + flags[i]);
  }
}

template <int VEC>
__global__ void gather_rows_kernel(const float* __restrict__ table, int64_t ld_t,
                                   const int32_t* __restrict__ rows, int64_t n, int64_t F,
                                   float* __restrict__ out, int64_t ld_o) {
  using V = typename std::conditional<VEC == 4, float4, float>::type;
  const int64_t nv = F / VEC;
  const int64_t total = n * nv;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t i = t / nv, j = t - i * nv;
    const V v = *reinterpret_cast<const V*>(table + int64_t(rows[i]) * ld_t + j * VEC);
    *reinterpret_cast<V*>(out + i * ld_o + j * VEC) = v;
  }
}

__global__ void scatter_f32_kernel(const float* __restrict__ in, const int32_t* __restrict__ perm, int64_t n,
                                   float* __restrict__ out) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    out[perm[i]] = in[i];
}

}  // namespace
}  // namespace kgx

using namespace kgx;

extern "C" int kgx_csr_workspace_bytes(int64_t E, int64_t n_dst, int flags, size_t* bytes) {
  KGX_REQUIRE(bytes && E >= 0 && n_dst >= 0, KGX_ERR_ARG, "kgx_csr_workspace_bytes: bad arguments");
  const int64_t total = E + ((flags & KGX_CSR_SELF_LOOPS) ? n_dst : 0);
  *bytes = csr_layout(nullptr, total, n_dst).total;
  return KGX_OK;
}

extern "C" int kgx_csr_build2(const int32_t* src, const int32_t* dst, int64_t E, int64_t n_src,
                              int64_t n_dst, int flags, int32_t* rowptr, int32_t* col, int32_t* eid,
                              int32_t* deg, float* dinv, float* w, const float* dinv_table,
                              int64_t table_len, void* workspace, size_t workspace_bytes, int64_t* info,
                              kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  const bool loops = flags & KGX_CSR_SELF_LOOPS;
  const bool norm = flags & KGX_CSR_GCN_NORM;
  KGX_REQUIRE(E >= 0 && n_dst >= 0 && n_src >= 0, KGX_ERR_ARG, "kgx_csr_build: negative sizes");
  KGX_REQUIRE(!loops || n_src == n_dst, KGX_ERR_ARG,
              "kgx_csr_build: self loops need n_src == n_dst (got %lld, %lld)", (long long)n_src,
              (long long)n_dst);
  const int64_t total = E + (loops ? n_dst : 0);
  KGX_REQUIRE(total < (int64_t(1) << 31) - 1 && n_dst < (int64_t(1) << 31) - 1, KGX_ERR_ARG,
              "kgx_csr_build: graph too large for int32 CSR (E'=%lld)", (long long)total);
  KGX_REQUIRE(rowptr && deg && (total == 0 || (col && eid)), KGX_ERR_ARG, "kgx_csr_build: null output");
  KGX_REQUIRE(E == 0 || (src && dst), KGX_ERR_ARG, "kgx_csr_build: null input");
  KGX_REQUIRE(!norm || (dinv && (total == 0 || w)), KGX_ERR_ARG, "kgx_csr_build: GCN_NORM needs dinv and w");
  KGX_REQUIRE(!dinv_table || table_len > 0, KGX_ERR_ARG, "kgx_csr_build2: empty dinv table");
  CsrLayout L = csr_layout(workspace, total, n_dst);
  KGX_REQUIRE(workspace && workspace_bytes >= L.total, KGX_ERR_ARG,
              "kgx_csr_build: workspace %zu < %zu bytes", workspace_bytes, L.total);

  KGX_CHECK_HIP(hipMemsetAsync(L.st, 0, sizeof(CsrStatus), stream));
  if (total > 0) {
    hipLaunchKernelGGL(csr_prep_kernel, dim3(grid_for(total, 8192)), dim3(kBlock), 0, stream, src, dst, E,
                       n_src, n_dst, flags, L.keys, L.vals, L.st);
    KGX_CHECK_LAUNCH();
    const int end_bit = ceil_log2_u64(uint64_t(n_dst) + 1);
    size_t sb = L.sort_bytes;
    KGX_CHECK_HIP(rocprim::radix_sort_pairs(L.sort_tmp, sb, L.keys, L.keys_sorted, L.vals, L.vals_sorted,
                                            (unsigned)total, 0, end_bit > 0 ? end_bit : 1, stream,
                                            false));
  }
  hipLaunchKernelGGL(csr_rowptr_kernel, dim3(grid_for(n_dst + 1, 8192)), dim3(kBlock), 0, stream,
                     L.keys_sorted, total, n_dst, rowptr, L.st);
  KGX_CHECK_LAUNCH();
  if (n_dst > 0) {  // degrees (and dinv) first: the col pass below computes the norms with it
    hipLaunchKernelGGL(csr_deg_kernel, dim3(grid_for(n_dst, 1024)), dim3(kBlock), 0, stream, rowptr, n_dst,
                       flags, deg, dinv, dinv_table, table_len, L.st);
    KGX_CHECK_LAUNCH();
  }
  if (total > 0) {
    const dim3 grid(grid_for(total / kColIlp + 1, 8192));
    if (norm)
      hipLaunchKernelGGL(csr_col_kernel<true>, grid, dim3(kBlock), 0, stream, L.vals_sorted, L.keys_sorted, rowptr,
                         n_dst, dinv, eid, col, w);
    else
      hipLaunchKernelGGL(csr_col_kernel<false>, grid, dim3(kBlock), 0, stream, L.vals_sorted, L.keys_sorted, rowptr,
                         n_dst, dinv, eid, col, w);
    KGX_CHECK_LAUNCH();
  }
  CsrStatus hs;
  KGX_CHECK_HIP(hipMemcpyAsync(&hs, L.st, sizeof(CsrStatus), hipMemcpyDeviceToHost, stream));
  KGX_CHECK_HIP(hipStreamSynchronize(stream));
  if (info) {
    info[0] = int64_t(hs.kept);
    info[1] = int64_t(hs.max_deg);
    info[2] = int64_t(hs.bad);
    info[3] = int64_t(hs.table_miss);
  }
  KGX_REQUIRE(hs.bad == 0, KGX_ERR_INDEX,
              "index out of range in edge_index: %llu edge(s) reference a node outside "
              "[-n, n) (n_src=%lld, n_dst=%lld)",
              hs.bad, (long long)n_src, (long long)n_dst);
  return KGX_OK;
}

extern "C" int kgx_csr_build(const int32_t* src, const int32_t* dst, int64_t E, int64_t n_src,
                             int64_t n_dst, int flags, int32_t* rowptr, int32_t* col, int32_t* eid,
                             int32_t* deg, float* dinv, float* w, void* workspace,
                             size_t workspace_bytes, int64_t* info, kgx_stream_t stream_) {
  return kgx_csr_build2(src, dst, E, n_src, n_dst, flags, rowptr, col, eid, deg, dinv, w, nullptr, 0, workspace,
                        workspace_bytes, info, stream_);
}

extern "C" int kgx_schedule_workspace_bytes(int64_t n_dst, size_t* bytes) {
  KGX_REQUIRE(bytes && n_dst >= 0, KGX_ERR_ARG, "kgx_schedule_workspace_bytes: bad arguments");
  *bytes = sched_layout(nullptr, n_dst).total;
  return KGX_OK;
}

extern "C" int kgx_schedule_build(const int32_t* rowptr, int64_t n_dst, int32_t split_len, int32_t* rows,
                                  int32_t* items, int64_t cap_items, int32_t* split, void* workspace,
                                  size_t workspace_bytes, int64_t* info, kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(rowptr && n_dst >= 0, KGX_ERR_ARG, "kgx_schedule_build: bad arguments");
  KGX_REQUIRE(split_len <= 0 || (split_len & (split_len - 1)) == 0, KGX_ERR_ARG,
              "kgx_schedule_build: split_len must be a power of two (got %d)", split_len);
  if (n_dst == 0) {
    if (info) info[0] = info[1] = info[2] = info[3] = 0;
    return KGX_OK;
  }
  KGX_REQUIRE(rows && items && split, KGX_ERR_ARG, "kgx_schedule_build: null output");
  SchedLayout L = sched_layout(workspace, n_dst);
  KGX_REQUIRE(workspace && workspace_bytes >= L.total, KGX_ERR_ARG,
              "kgx_schedule_build: workspace %zu < %zu bytes", workspace_bytes, L.total);
  KGX_CHECK_HIP(hipMemsetAsync(L.st, 0, sizeof(SchedStatus), stream));
  const unsigned g = grid_for(n_dst, 8192);
  hipLaunchKernelGGL(sched_keys_kernel, dim3(g), dim3(kBlock), 0, stream, rowptr, n_dst, L.keys, L.iota);
  KGX_CHECK_LAUNCH();
  size_t tb = L.tmp_bytes;
  KGX_CHECK_HIP(rocprim::radix_sort_pairs(L.tmp, tb, L.keys, L.keys_sorted, L.iota, rows, (unsigned)n_dst, 0,
                                          kDegKeyBits, stream, false));
  hipLaunchKernelGGL(sched_count_kernel, dim3(g), dim3(kBlock), 0, stream, rowptr, rows, n_dst, split_len,
                     L.nchunks, L.nslots);
  KGX_CHECK_LAUNCH();
  tb = L.tmp_bytes;
  KGX_CHECK_HIP(rocprim::exclusive_scan(L.tmp, tb, (const int32_t*)L.nchunks, L.item_off, 0, (size_t)n_dst,
                                        rocprim::plus<int32_t>(), stream, false));
  tb = L.tmp_bytes;
  KGX_CHECK_HIP(rocprim::exclusive_scan(L.tmp, tb, (const int32_t*)L.nslots, L.slot_off, 0, (size_t)n_dst,
                                        rocprim::plus<int32_t>(), stream, false));
  hipLaunchKernelGGL(sched_emit_kernel, dim3(g), dim3(kBlock), 0, stream, rowptr, rows, n_dst, split_len,
                     L.nchunks, L.item_off, L.nslots, L.slot_off, reinterpret_cast<int4*>(items), cap_items,
                     reinterpret_cast<int4*>(split), L.st);
  KGX_CHECK_LAUNCH();
  SchedStatus hs;
  KGX_CHECK_HIP(hipMemcpyAsync(&hs, L.st, sizeof(SchedStatus), hipMemcpyDeviceToHost, stream));
  KGX_CHECK_HIP(hipStreamSynchronize(stream));
  KGX_REQUIRE(hs.overflow == 0, KGX_ERR_ARG, "kgx_schedule_build: cap_items %lld too small",
              (long long)cap_items);
  if (info) {
    info[0] = int64_t(hs.n_items);
    info[1] = int64_t(hs.n_split);
    info[2] = int64_t(hs.n_slots);
    info[3] = 0;
  }
  return KGX_OK;
}

extern "C" int kgx_rmat_edges(uint64_t seed, int scale, int64_t n_nodes, uint32_t a24, uint32_t b24,
                              uint32_t c24, int64_t e_begin, int64_t e_count, int32_t* src, int32_t* dst,
                              kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(scale > 0 && scale <= 62 && n_nodes > 0 && n_nodes <= (int64_t(1) << scale) &&
                  n_nodes < (int64_t(1) << 31),
              KGX_ERR_ARG, "kgx_rmat_edges: need 0 < n_nodes <= 2^scale < 2^31 (scale=%d, n=%lld)", scale,
              (long long)n_nodes);
  KGX_REQUIRE(uint64_t(a24) + b24 + c24 <= (1u << 24), KGX_ERR_ARG, "kgx_rmat_edges: a+b+c > 1");
  KGX_REQUIRE(e_count >= 0 && e_begin >= 0 && (e_count == 0 || (src && dst)), KGX_ERR_ARG,
              "kgx_rmat_edges: bad edge range");
  if (e_count == 0) return KGX_OK;
  Feistel fs;
  fs.hb = (scale + 1) / 2;
  fs.mask = (uint64_t(1) << fs.hb) - 1;
  for (int i = 0; i < 4; ++i) fs.keys[i] = splitmix64(seed ^ (0xA5A5A5A5A5A5A5A5ull + uint64_t(i)));
  const uint64_t base = splitmix64(seed);
  hipLaunchKernelGGL(rmat_kernel, dim3(grid_for(e_count, 16384)), dim3(kBlock), 0, stream, base, fs, scale,
                     uint64_t(n_nodes), a24, a24 + b24, a24 + b24 + c24, e_begin, e_count, src, dst);
  KGX_CHECK_LAUNCH();
  return KGX_OK;
}

extern "C" int kgx_select_workspace_bytes(int64_t n, size_t* bytes) {
  KGX_REQUIRE(bytes && n >= 0, KGX_ERR_ARG, "kgx_select_workspace_bytes: bad arguments");
  size_t scb = 0;
  const int32_t* si = nullptr;
  int32_t* so = nullptr;
  (void)rocprim::exclusive_scan(nullptr, scb, si, so, 0, (size_t)(n > 0 ? n : 1), rocprim::plus<int32_t>(), 0,
                          false);
  Carve c(nullptr, ~size_t(0));
  c.take<int32_t>(n);
  c.take<int32_t>(n);
  c.take<unsigned long long>(1);
  c.take<char>(scb);
  *bytes = c.used();
  return KGX_OK;
}

extern "C" int kgx_select_dst_range(const int32_t* src, const int32_t* dst, int64_t n, int64_t lo, int64_t hi,
                                    int32_t* src_out, int32_t* dst_out, void* workspace, size_t workspace_bytes,
                                    int64_t* n_out, kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(n >= 0 && n < (int64_t(1) << 31) && n_out, KGX_ERR_ARG, "kgx_select_dst_range: bad arguments");
  if (n == 0) {
    *n_out = 0;
    return KGX_OK;
  }
  size_t need = 0;
  kgx_select_workspace_bytes(n, &need);
  KGX_REQUIRE(workspace && workspace_bytes >= need, KGX_ERR_ARG, "kgx_select_dst_range: workspace too small");
  Carve c(workspace, workspace_bytes);
  int32_t* flags = c.take<int32_t>(n);
  int32_t* pos = c.take<int32_t>(n);
  unsigned long long* cnt = c.take<unsigned long long>(1);
  size_t scb = workspace_bytes - c.used();
  void* tmp = c.take<char>(0);
  const unsigned g = grid_for(n, 8192);
  hipLaunchKernelGGL(range_flags_kernel, dim3(g), dim3(kBlock), 0, stream, dst, n, lo, hi, flags);
  KGX_CHECK_LAUNCH();
  KGX_CHECK_HIP(rocprim::exclusive_scan(tmp, scb, (const int32_t*)flags, pos, 0, (size_t)n,
                                        rocprim::plus<int32_t>(), stream, false));
  hipLaunchKernelGGL(range_scatter_kernel, dim3(g), dim3(kBlock), 0, stream, src, dst, flags, pos, n, src_out,
                     dst_out, cnt);
  KGX_CHECK_LAUNCH();
  unsigned long long h = 0;
  KGX_CHECK_HIP(hipMemcpyAsync(&h, cnt, sizeof(h), hipMemcpyDeviceToHost, stream));
  KGX_CHECK_HIP(hipStreamSynchronize(stream));
  *n_out = int64_t(h);
  return KGX_OK;
}

extern "C" int kgx_gather_rows(const float* table, int64_t ld_table, const int32_t* rows, int64_t n, int64_t F,
                               float* out, int64_t ld_out, kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(n >= 0 && F >= 0, KGX_ERR_ARG, "kgx_gather_rows: bad sizes");
  if (n == 0 || F == 0) return KGX_OK;
  KGX_REQUIRE(table && rows && out, KGX_ERR_ARG, "kgx_gather_rows: null pointer");
  const bool v4 = (F % 4 == 0) && (ld_table % 4 == 0) && (ld_out % 4 == 0) &&
                  (reinterpret_cast<uintptr_t>(table) % 16 == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0);
  if (v4) {
    hipLaunchKernelGGL(gather_rows_kernel<4>, dim3(grid_for(n * (F / 4))), dim3(kBlock), 0, stream, table,
                       ld_table, rows, n, F, out, ld_out);
  } else {
    hipLaunchKernelGGL(gather_rows_kernel<1>, dim3(grid_for(n * F)), dim3(kBlock), 0, stream, table, ld_table,
                       rows, n, F, out, ld_out);
  }
  KGX_CHECK_LAUNCH();
  return KGX_OK;
}

extern "C" int kgx_scatter_f32(const float* in, const int32_t* perm, int64_t n, float* out,
                               kgx_stream_t stream_) {
  hipStream_t stream = as_stream(stream_);
  KGX_REQUIRE(n >= 0, KGX_ERR_ARG, "kgx_scatter_f32: bad size");
  if (n == 0) return KGX_OK;
  KGX_REQUIRE(in && perm && out, KGX_ERR_ARG, "kgx_scatter_f32: null pointer");
  hipLaunchKernelGGL(scatter_f32_kernel, dim3(grid_for(n)), dim3(kBlock), 0, stream, in, perm, n, out);
  KGX_CHECK_LAUNCH();
  return KGX_OK;
}

extern "C" int kgx_gcn_dinv(const int32_t* deg, int64_t n, float* dinv, kgx_stream_t stream_) {
  KGX_REQUIRE(n >= 0 && (n == 0 || (deg && dinv)), KGX_ERR_ARG, "kgx_gcn_dinv: bad arguments");
  if (n == 0) return KGX_OK;
  hipLaunchKernelGGL(gcn_dinv_kernel, dim3(grid_for(n, 8192)), dim3(kBlock), 0, as_stream(stream_), deg, n, dinv);
  KGX_CHECK_LAUNCH();
  return KGX_OK;
}

extern "C" int kgx_gcn_dinv_table(const int32_t* deg, int64_t n, const float* table, int64_t table_len, float* dinv,
                                  kgx_stream_t stream_) {
  KGX_REQUIRE(n >= 0 && (n == 0 || (deg && dinv && table && table_len > 0)), KGX_ERR_ARG,
              "kgx_gcn_dinv_table: bad arguments");
  if (n == 0) return KGX_OK;
  hipLaunchKernelGGL(gcn_dinv_table_kernel, dim3(grid_for(n, 8192)), dim3(kBlock), 0, as_stream(stream_), deg, n,
                     table, table_len, dinv);
  KGX_CHECK_LAUNCH();
  return KGX_OK;
}

extern "C" int kgx_gcn_edge_norm(const int32_t* rowptr, const int32_t* col, int64_t n_dst, const float* dinv_dst,
                                 const float* dinv_src, float* w, kgx_stream_t stream_) {
  KGX_REQUIRE(n_dst >= 0 && (n_dst == 0 || (rowptr && col && dinv_dst && dinv_src && w)), KGX_ERR_ARG,
              "kgx_gcn_edge_norm: bad arguments");
  if (n_dst == 0) return KGX_OK;
  hipStream_t s = as_stream(stream_);
  hipLaunchKernelGGL(gcn_edge_norm_kernel, dim3(grid_for(n_dst * 8, 8192)), dim3(kBlock), 0, s, rowptr, col, n_dst,
                     dinv_dst, dinv_src, w);
  KGX_CHECK_LAUNCH();
  hipLaunchKernelGGL(gcn_edge_norm_long_kernel, dim3(grid_for(n_dst, 8192)), dim3(kBlock), 0, s, rowptr, col,
                     n_dst, dinv_dst, dinv_src, w);
  KGX_CHECK_LAUNCH();
  return KGX_OK;
}

extern "C" int kgx_cu_split_layout_ok(int cus, int xccs, const char* arch) {
  return cu_split_layout_ok(cus, xccs, arch) ? 1 : 0;
}

extern "C" int kgx_cu_split_supported(int device) {
  int n = 0;
  KGX_CHECK_HIP(hipGetDeviceCount(&n));
  KGX_REQUIRE(device >= 0 && device < n, KGX_ERR_ARG, "kgx_cu_split_supported: no device %d", device);
  return cu_split_device_ok(device) ? 1 : 0;
}

namespace kgx {
namespace {
// where block b ran: (XCC << 8) | (SE << 5) | (SH << 4) | CU, from HW_REG_HW_ID (gfx9 layout:
// CU_ID [11:8], SH_ID [12], SE_ID [15:13]) and HW_REG_XCC_ID; each block stays ~20 us so the
// dispatcher spreads the grid over every CU its stream's mask allows
__global__ void cu_census_kernel(int32_t* __restrict__ ids, int64_t n) {
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const int64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < 2000) __builtin_amdgcn_s_sleep(8);  // 100 MHz ticks: ~20 us
  if (threadIdx.x == 0 && int64_t(blockIdx.x) < n)
    ids[blockIdx.x] = int32_t(((xcc & 0xf) << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xf));
}
}  // namespace
}  // namespace kgx

extern "C" int kgx_cu_split_census(int per32, int64_t n_blocks, int32_t* head_ids, int32_t* tail_ids, int* n_cus,
                                   kgx_stream_t stream_) {
  KGX_REQUIRE(per32 > 0 && per32 < 32 && n_blocks > 0 && n_blocks <= (1 << 20) && head_ids && tail_ids && n_cus,
              KGX_ERR_ARG, "kgx_cu_split_census: bad arguments");
  hipStream_t s = as_stream(stream_);
  CuSplit* cs = cu_split(per32, s);
  KGX_REQUIRE(cs != nullptr, KGX_ERR_UNSUPPORTED, "kgx_cu_split_census: no CU split on this device / stream");
  KGX_CHECK_HIP(hipEventRecord(cs->fork, s));
  KGX_CHECK_HIP(hipStreamWaitEvent(cs->head, cs->fork, 0));
  KGX_CHECK_HIP(hipStreamWaitEvent(cs->tail, cs->fork, 0));
  hipLaunchKernelGGL(cu_census_kernel, dim3(unsigned(n_blocks)), dim3(64), 0, cs->head, head_ids, n_blocks);
  KGX_CHECK_LAUNCH();
  hipLaunchKernelGGL(cu_census_kernel, dim3(unsigned(n_blocks)), dim3(64), 0, cs->tail, tail_ids, n_blocks);
  KGX_CHECK_LAUNCH();
  KGX_CHECK_HIP(hipEventRecord(cs->jh, cs->head));
  KGX_CHECK_HIP(hipEventRecord(cs->jt, cs->tail));
  KGX_CHECK_HIP(hipStreamWaitEvent(s, cs->jh, 0));
  KGX_CHECK_HIP(hipStreamWaitEvent(s, cs->jt, 0));
  KGX_CHECK_HIP(hipStreamSynchronize(s));
  n_cus[0] = cs->n_head;
  n_cus[1] = cs->n_tail;
  return KGX_OK;
}

// ---------------------------------------------------------------------------
// Schedule tails (graph.short_suffix_start / tiny.tiny_suffix_start) and the
// tiny-row records (tiny.tiny_pack) on the device: one pass each instead of a
// dozen torch ops with their host syncs (NS graph build: ~1.8 ms of 10).
// ---------------------------------------------------------------------------
namespace kgx {
namespace {

// out[0] = 1 + the last item that is split (slot >= 0) or longer than short_max,
// out[1] = the same for tiny_max (0: none) -- the suffix of short / tiny rows starts there
__global__ void sched_suffix_kernel(const int4* __restrict__ items, int64_t n, int short_max, int tiny_max,
                                    unsigned long long* __restrict__ out) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  unsigned long long ls = 0, lt = 0;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int4 v = items[i];
    const int len = v.z - v.y;
    if (v.w >= 0 || len > short_max) ls = (unsigned long long)(i + 1);
    if (v.w >= 0 || len > tiny_max) lt = (unsigned long long)(i + 1);
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a = __shfl_xor(ls, o, 64), b = __shfl_xor(lt, o, 64);
    ls = a > ls ? a : ls;
    lt = b > lt ? b : lt;
  }
  // one atomic pair per block, not per wave: 16K waves' atomics on two addresses serialised
  // at the L2 (0.38 ms per call at NS)
  __shared__ unsigned long long red[2][kBlock / 64];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wv] = ls;
    red[1][wv] = lt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < kBlock / 64; ++k) {
      ls = red[0][k] > ls ? red[0][k] : ls;
      lt = red[1][k] > lt ? red[1][k] : lt;
    }
    if (ls) atomicMax(&out[0], ls);
    if (lt) atomicMax(&out[1], lt);
  }
}

// record i of the tail items [start, start + n): {row, degree, col0, col1} and {w0, w1}
// (tiny.py's layout: col1 = col0 for degree 1, both 0 for degree 0, weights 0 where absent);
// st[0] counts the degree-2 records, st[1] = 1 + the last degree-2 record
__global__ void tiny_pack_kernel(const int4* __restrict__ items, int64_t start, int64_t n,
                                 const int32_t* __restrict__ col, const float* __restrict__ w, int64_t n_col,
                                 int4* __restrict__ pack, float2* __restrict__ tw, unsigned long long* __restrict__ st) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  unsigned long long cnt = 0, last2 = 0;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int4 v = items[start + i];
    const int deg = v.z - v.y;
    const int64_t last = n_col - 1;
    const int64_t i0 = v.y < last ? v.y : last;
    const int64_t i1b = int64_t(v.y) + (deg > 1 ? 1 : 0);
    const int64_t i1 = i1b < last ? i1b : last;
    const int32_t c0 = deg > 0 ? col[i0] : 0, c1 = deg > 0 ? col[i1] : 0;
    pack[i] = make_int4(v.x, deg, c0, c1);
    if (tw) tw[i] = make_float2(deg > 0 ? w[i0] : 0.0f, deg > 1 ? w[i1] : 0.0f);
    if (deg == 2) {
      ++cnt;
      last2 = (unsigned long long)(i + 1);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o, 64);
    const unsigned long long b = __shfl_xor(last2, o, 64);
    last2 = b > last2 ? b : last2;
  }
  __shared__ unsigned long long red[2][kBlock / 64];  // one atomic pair per block (sched_suffix_kernel)
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wv] = cnt;
    red[1][wv] = last2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < kBlock / 64; ++k) {
      cnt += red[0][k];
      last2 = red[1][k] > last2 ? red[1][k] : last2;
    }
    if (cnt) atomicAdd(&st[0], cnt);
    if (last2) atomicMax(&st[1], last2);
  }
}

}  // namespace
}  // namespace kgx

extern "C" int kgx_schedule_suffixes(const int32_t* items, int64_t n_items, int short_max, int tiny_max,
                                     void* workspace, int64_t* out, kgx_stream_t stream_) {
  KGX_REQUIRE(n_items >= 0 && out && workspace && (n_items == 0 || items), KGX_ERR_ARG,
              "kgx_schedule_suffixes: bad arguments");
  hipStream_t s = as_stream(stream_);
  auto* st = static_cast<unsigned long long*>(workspace);
  KGX_CHECK_HIP(hipMemsetAsync(st, 0, 2 * sizeof(unsigned long long), s));
  if (n_items > 0) {
    hipLaunchKernelGGL(sched_suffix_kernel, dim3(grid_for(n_items, 1024)), dim3(kBlock), 0, s,
                       reinterpret_cast<const int4*>(items), n_items, short_max, tiny_max, st);
    KGX_CHECK_LAUNCH();
  }
  unsigned long long h[2];
  KGX_CHECK_HIP(hipMemcpyAsync(h, st, sizeof(h), hipMemcpyDeviceToHost, s));
  KGX_CHECK_HIP(hipStreamSynchronize(s));
  out[0] = int64_t(h[0]);
  out[1] = int64_t(h[1]);
  return KGX_OK;
}

extern "C" int kgx_tiny_pack(const int32_t* items, int64_t start, int64_t n, const int32_t* col, const float* w,
                             int64_t n_col, int32_t* pack, float* tw, void* workspace, int64_t* out,
                             kgx_stream_t stream_) {
  KGX_REQUIRE(start >= 0 && n >= 0 && n_col > 0 && items && col && pack && workspace && out && (!tw || w),
              KGX_ERR_ARG, "kgx_tiny_pack: bad arguments");
  hipStream_t s = as_stream(stream_);
  auto* st = static_cast<unsigned long long*>(workspace);
  KGX_CHECK_HIP(hipMemsetAsync(st, 0, 2 * sizeof(unsigned long long), s));
  if (n > 0) {
    hipLaunchKernelGGL(tiny_pack_kernel, dim3(grid_for(n, 2048)), dim3(kBlock), 0, s,
                       reinterpret_cast<const int4*>(items), start, n, col, tw ? w : nullptr, n_col,
                       reinterpret_cast<int4*>(pack), reinterpret_cast<float2*>(tw), st);
    KGX_CHECK_LAUNCH();
  }
  unsigned long long h[2];
  KGX_CHECK_HIP(hipMemcpyAsync(h, st, sizeof(h), hipMemcpyDeviceToHost, s));
  KGX_CHECK_HIP(hipStreamSynchronize(s));
  out[0] = int64_t(h[0]);
  out[1] = int64_t(h[1]);
  return KGX_OK;
}
