// Internal helpers shared by the kgx HIP translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

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
// takes (den - 1) / den of its resident grid: den = KGX_SHARE_DEN (default 32:
// the sharded GCN step with light rows and pruned pulls, simulated at 400 GB/s
// on three boxes, measured 11.72-11.79 ms at 32 against 11.80-11.84 at 16; 8
// and 64 were slower in round 5, 12.31-12.36 and 13.07-13.13 ms).
inline int64_t shared_cap(int64_t full) {
  const char* h = getenv("KGX_SHARE_DEN");  // read per launch: measurement sweeps change it in-process
  const int v = h ? atoi(h) : 32;
  const int den = v >= 2 ? v : 32;
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

// Spatial split of the GPU for one fused launch: two CU-masked streams
// (hipExtStreamCreateWithCUMask) per (host thread, device, split), "tail" over
// per32 of every 32 CUs and "head" over the rest; launches on them are forked
// from and joined back into the caller's stream, each grid sized to its CU set.
struct CuSplit {
  hipStream_t head = nullptr, tail = nullptr;
  hipEvent_t fork = nullptr, jh = nullptr, jt = nullptr;
  int device = -1, per32 = -1, n_head = 0, n_tail = 0;
};


// Every CU-masked stream and its events are destroyed by an atexit handler,
// which runs before the HIP runtime's own teardown (it is registered after the
// runtime initialised): left to the runtime, a process exit under rocprofv3's
// kernel trace crashed in __cxa_finalize once the masked streams existed.
inline void cu_split_registry(const CuSplit* add) {
  static std::mutex mu;
  static std::vector<CuSplit> all;
  static bool hooked = false;
  std::lock_guard<std::mutex> lock(mu);
  if (add) {
    all.push_back(*add);
    if (!hooked) {
      hooked = true;
      std::atexit([] { cu_split_registry(nullptr); });
    }
    return;
  }
  for (const CuSplit& c : all) {  // exit: drain and release
    (void)hipStreamSynchronize(c.head);
    (void)hipStreamSynchronize(c.tail);
    (void)hipStreamDestroy(c.head);
    (void)hipStreamDestroy(c.tail);
    (void)hipEventDestroy(c.fork);
    (void)hipEventDestroy(c.jh);
    (void)hipEventDestroy(c.jt);
  }
  all.clear();
}

// The layout the CU split was measured and validated on: gfx950
// with 256 CUs in 8 XCDs (one partition, SPX).  The split's tail set is "the
// first per32 of every 32 mask bits", which on that layout is one block of CUs
// per XCD; other splits of the mask measured 30-300 % slower there, so on any
// other CU count, XCD count or architecture (another partition mode, a
// harvested part, a larger chip) the launches run unsplit.
inline bool cu_split_layout_ok(int cus, int xccs, const char* arch) {
  return cus == 256 && xccs == 8 && arch && std::strncmp(arch, "gfx950", 6) == 0;
}

// per device, once per process: does it have the validated layout?  A device
// that does not gets a one-time note on stderr the first time a split is asked for.
inline bool cu_split_device_ok(int dev) {
  static std::mutex mu;
  static signed char known[64];  // 0 unknown, 1 ok, -1 not
  if (dev < 0 || dev >= 64) return false;
  std::lock_guard<std::mutex> lock(mu);
  if (known[dev] == 0) {
    int cus = 0, xccs = 0;
    hipDeviceProp_t prop;
    const bool got = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                     hipDeviceGetAttribute(&xccs, hipDeviceAttributeNumberOfXccs, dev) == hipSuccess &&
                     hipGetDeviceProperties(&prop, dev) == hipSuccess;
    const bool ok = got && cu_split_layout_ok(cus, xccs, prop.gcnArchName);
    known[dev] = ok ? 1 : -1;
    if (!ok)
      std::fprintf(stderr,
                   "kgx: device %d (%d CUs, %d XCDs, %s) is not the layout the CU split was validated on "
                   "(gfx950, 256 CUs, 8 XCDs): fused launches run unsplit\n",
                   dev, cus, xccs, got ? prop.gcnArchName : "?");
  }
  return known[dev] > 0;
}

// per (host thread, device, split): streams and events made once and kept for
// the process, like the library's other side streams (a small per-thread cache:
// a split is never re-created, so streams are not leaked by alternating splits).
// The device is the caller stream's; a stream on a device other than the
// current one runs unsplit (the masked streams are created on the current
// device).  The pair is shared by every caller stream of the thread, so two
// CU-split launches from different caller streams of one thread are ordered
// through it: the split assumes one caller stream per host thread (the
// layers' and bench.py's case; the sharded passes run unsplit).
inline CuSplit* cu_split(int per32, hipStream_t caller) {
  constexpr int kCache = 8;
  thread_local CuSplit cache[kCache];
  thread_local int used = 0;
  int dev = 0, sdev = 0;
  if (per32 <= 0 || per32 >= 32 || hipGetDevice(&dev) != hipSuccess) return nullptr;
  if (caller && (hipStreamGetDevice(caller, &sdev) != hipSuccess || sdev != dev)) return nullptr;
  for (int i = 0; i < used; ++i)
    if (cache[i].device == dev && cache[i].per32 == per32) return &cache[i];
  if (used == kCache || !cu_split_device_ok(dev)) return nullptr;
  const int cus = cu_count();
  uint32_t mh[8] = {0}, mt[8] = {0};
  int nh = 0, nt = 0;
  for (int c = 0; c < cus && c < 256; ++c) {
    if ((c % 32) < per32) {
      mt[c / 32] |= 1u << (c % 32);
      ++nt;
    } else {
      mh[c / 32] |= 1u << (c % 32);
      ++nh;
    }
  }
  if (nh == 0 || nt == 0) return nullptr;
  CuSplit n;
  const bool ok = hipExtStreamCreateWithCUMask(&n.head, 8, mh) == hipSuccess &&
                  hipExtStreamCreateWithCUMask(&n.tail, 8, mt) == hipSuccess &&
                  hipEventCreateWithFlags(&n.fork, hipEventDisableTiming) == hipSuccess &&
                  hipEventCreateWithFlags(&n.jh, hipEventDisableTiming) == hipSuccess &&
                  hipEventCreateWithFlags(&n.jt, hipEventDisableTiming) == hipSuccess;
  if (!ok) {  // release whatever was made: run unsplit
    if (n.head) (void)hipStreamDestroy(n.head);
    if (n.tail) (void)hipStreamDestroy(n.tail);
    if (n.fork) (void)hipEventDestroy(n.fork);
    if (n.jh) (void)hipEventDestroy(n.jh);
    if (n.jt) (void)hipEventDestroy(n.jt);
    return nullptr;
  }
  n.device = dev;
  n.per32 = per32;
  n.n_head = nh;
  n.n_tail = nt;
  cache[used] = n;
  ++used;
  cu_split_registry(&cache[used - 1]);
  return &cache[used - 1];
}

// joins both CU-masked streams back into the caller's stream on every return
struct SplitJoin {
  CuSplit* cs = nullptr;
  hipStream_t s = nullptr;
  ~SplitJoin() {
    if (cs) {
      (void)hipEventRecord(cs->jh, cs->head);
      (void)hipEventRecord(cs->jt, cs->tail);
      (void)hipStreamWaitEvent(s, cs->jh, 0);
      (void)hipStreamWaitEvent(s, cs->jt, 0);
    }
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
