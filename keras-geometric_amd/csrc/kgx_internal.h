// Internal helpers shared by the kgx HIP translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include <cstdlib>

#include "kgx.h"

namespace kgx {

void set_error(const char* fmt, ...);

inline hipStream_t as_stream(kgx_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline int ceil_log2_u64(uint64_t v) {
  int b = 0;
  while ((uint64_t(1) << b) < v) ++b;
  return b;
}

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Bump allocator over a caller-provided workspace.
struct Carve {
  char* base;
  size_t cap;
  size_t off = 0;
  Carve(void* b, size_t c) : base(static_cast<char*>(b)), cap(c) {}
  template <typename T>
  T* take(size_t count) {
    off = align_up(off, 256);
    T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
    off += count * sizeof(T);
    return p;
  }
  size_t used() const { return align_up(off, 256); }
};

constexpr int kBlock = 256;  // 4 waves of 64 lanes

// Grid for a grid-stride launch: enough blocks to fill 256 CUs x 8 blocks, never
// more than the work needs.
inline unsigned grid_for(int64_t work_threads, int64_t cap_blocks = 2048) {
  int64_t b = (work_threads + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > cap_blocks) b = cap_blocks;
  return static_cast<unsigned>(b);
}

// Grid for a persistent grid-stride launch: as many blocks as are resident at
// once (occupancy x CUs), never more than the work needs.
inline int cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

template <typename Kern>
unsigned resident_grid(Kern kernel, int64_t groups_needed, int G) {
  const int cus = cu_count();
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess || per_cu <= 0)
    per_cu = 4;
  const int64_t cap = int64_t(per_cu) * cus;
  const int64_t need = (groups_needed * G + kBlock - 1) / kBlock;
  const int64_t g = need < cap ? need : cap;
  return unsigned(g < 1 ? 1 : g);
}

// A launch that shares the GPU with a concurrent stream (KGX_FUSED_SHARE_GPU)
// takes (den - 1) / den of its resident grid: den = KGX_SHARE_DEN (default 8).
inline int64_t shared_cap(int64_t full) {
  const char* h = getenv("KGX_SHARE_DEN");  // read per launch: measurement sweeps change it in-process
  const int v = h ? atoi(h) : 8;
  const int den = v >= 2 ? v : 8;
  const int64_t c = full * (den - 1) / den;
  return c > 0 ? c : 1;
}

// A per-host-thread side stream and fork / join events, one set per
// translation unit (each .hip file's launches fork onto its own stream).
// Thread-local: concurrent launches from several host threads (one rank per
// thread in the tests) never share events.
struct ForkJoin {
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  int device = -1;
};
namespace {
inline ForkJoin& fork_join() {
  thread_local ForkJoin fj;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (fj.device != dev) {
    (void)hipStreamCreateWithFlags(&fj.side, hipStreamNonBlocking);
    (void)hipEventCreateWithFlags(&fj.fork, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&fj.join, hipEventDisableTiming);
    fj.device = dev;
  }
  return fj;
}
}  // namespace

// Joins a forked side stream back into the caller's stream on every return
// after the fork, so no error path leaves the caller's stream unordered
// against the forked kernel (whose outputs the caching allocator could
// otherwise hand out again while it still writes them).
struct JoinGuard {
  ForkJoin* fj = nullptr;
  hipStream_t s = nullptr;
  ~JoinGuard() {
    if (fj) (void)hipStreamWaitEvent(s, fj->join, 0);
  }
};

inline int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}
inline int log2i(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

}  // namespace kgx

#define KGX_CHECK_HIP(expr)                                                      \
  do {                                                                           \
    hipError_t kgx_e_ = (expr);                                                  \
    if (kgx_e_ != hipSuccess) {                                                  \
      kgx::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #expr,          \
                     hipGetErrorString(kgx_e_));                                 \
      return KGX_ERR_HIP;                                                        \
    }                                                                            \
  } while (0)

#define KGX_CHECK_LAUNCH() KGX_CHECK_HIP(hipGetLastError())

#define KGX_REQUIRE(cond, code, ...)                                             \
  do {                                                                           \
    if (!(cond)) {                                                               \
      kgx::set_error(__VA_ARGS__);                                               \
      return (code);                                                             \
    }                                                                            \
  } while (0)
