// dmem.h -- lifetimes of device buffers made during setup (device.hip,
// gsetup.hip).
//
// Every kernel, fill and copy of the GPU setup and of the apply-layout
// builder runs on the null stream, and so do the temporaries' lifetimes:
//  * temporaries (Scratch, TmpPool, GHier, the seed-ring blocks) come from a
//    per-device cache of hipMalloc'd blocks (tmp_malloc / tmp_free).  A freed
//    block goes back to the cache at once and the next tmp_malloc may hand it
//    out again: its new users are queued on the null stream behind every
//    kernel that read it before -- no drain of the device and no reuse under
//    a running reader.  The cache is emptied at the end of every setup
//    (tmp_trim, after the null stream has drained);
//  * a long-lived (hipMalloc) array replaced during setup (operator re-homing,
//    K region candidates) is freed after an event recorded on the null stream
//    behind its last reader has completed (ordered_free): a wait on that one
//    stream, not on the device.
// Round 4 found (bench/contig_alias.hip) that the
// runtime's stream-ordered pool (hipMallocAsync) hands out blocks that share
// physical memory with other live blocks of the same pool: a block of a few
// MiB read back another live block's words.  Rounds 3-4 took the setup's
// temporaries from that pool; the intermittent wrong operators (whole lines
// of a conversion's output replaced by other data) were that aliasing.  No
// buffer of the library comes from hipMallocAsync any more.
// Round 3 drained the whole device before every hipFree instead (free-after-
// drain); DESIGN.md section 4.1 records what the round-4 diagnosis
// (bench/free_race.hip, scripts/gpu_freediag.sh) measured about hipFree.
// Diagnosis build only (make diag -> libmamg_diag.so, -DMAMG_DIAG=1; the
// product library reads none of these):
//   MAMG_FREE_MODE=drain   round 3's drain + hipFree
//   MAMG_FREE_MODE=plain   hipMalloc / hipFree with no ordering of our own
//                          (the round-2 code)
//   MAMG_ALLOC_LOG=<file>  every device allocation and free of the library,
//                          one line each ("M ptr bytes kind" / "F ptr"),
//                          replayed by bench/alloc_replay.hip
//   MAMG_DIAG_CONTIG=1     re-homed streams in physically contiguous
//                          allocations (rounds 2-4)
//   MAMG_DEBUG_PTRS=1      every setup temporary checked, when handed out,
//                          to be the start of a live runtime allocation at
//                          least as large (hipMemGetAddressRange), and the
//                          transpose's sort permutation checked before the
//                          gather that indexes with it (gsetup.hip)
#pragma once
#ifndef MAMG_DIAG
#define MAMG_DIAG 0
#endif
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <unordered_map>

namespace mamg {

// Device fills and device-to-device copies by the library's own kernels
// instead of hipMemset / hipMemcpy(DeviceToDevice) (same stream semantics:
// ordered on stream s, asynchronous to the host).  Round 4 moved every fill
// and device copy here while it chased the wrong operators of section 4.1;
// the cause turned out to be elsewhere (the pool aliasing above), but one
// code path for all of them is kept: the fills and copies are plain
// streaming kernels at HBM rate.
namespace detail {
template <class T>
__global__ __launch_bounds__(256) void fill_words_kernel(T* __restrict__ p, T v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}
template <class T>
__global__ __launch_bounds__(256) void copy_words_kernel(T* __restrict__ d, const T* __restrict__ s, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) d[i] = s[i];
}
inline unsigned words_grid(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
}
}  // namespace detail

inline hipError_t dev_memset(void* p, int v, size_t bytes, hipStream_t s = nullptr) {
  if (!bytes) return hipSuccess;
  const uint32_t b = (uint8_t)v, w = b * 0x01010101u;
  const uintptr_t a = (uintptr_t)p;
  if (a % 16 == 0 && bytes % 16 == 0) {
    const int64_t n = (int64_t)(bytes / 16);
    detail::fill_words_kernel<uint4><<<detail::words_grid(n), 256, 0, s>>>((uint4*)p, make_uint4(w, w, w, w), n);
  } else if (a % 8 == 0 && bytes % 8 == 0) {
    const int64_t n = (int64_t)(bytes / 8);
    detail::fill_words_kernel<uint64_t><<<detail::words_grid(n), 256, 0, s>>>((uint64_t*)p,
                                                                               ((uint64_t)w << 32) | w, n);
  } else if (a % 4 == 0 && bytes % 4 == 0) {
    const int64_t n = (int64_t)(bytes / 4);
    detail::fill_words_kernel<uint32_t><<<detail::words_grid(n), 256, 0, s>>>((uint32_t*)p, w, n);
  } else {
    const int64_t n = (int64_t)bytes;
    detail::fill_words_kernel<uint8_t><<<detail::words_grid(n), 256, 0, s>>>((uint8_t*)p, (uint8_t)b, n);
  }
  return hipGetLastError();
}

inline hipError_t dev_copy(void* d, const void* src, size_t bytes, hipStream_t s = nullptr) {
  if (!bytes) return hipSuccess;
  const uintptr_t a = (uintptr_t)d | (uintptr_t)src;
  if (a % 16 == 0 && bytes % 16 == 0) {
    const int64_t n = (int64_t)(bytes / 16);
    detail::copy_words_kernel<uint4><<<detail::words_grid(n), 256, 0, s>>>((uint4*)d, (const uint4*)src, n);
  } else if (a % 8 == 0 && bytes % 8 == 0) {
    const int64_t n = (int64_t)(bytes / 8);
    detail::copy_words_kernel<uint64_t><<<detail::words_grid(n), 256, 0, s>>>((uint64_t*)d, (const uint64_t*)src, n);
  } else if (a % 4 == 0 && bytes % 4 == 0) {
    const int64_t n = (int64_t)(bytes / 4);
    detail::copy_words_kernel<uint32_t><<<detail::words_grid(n), 256, 0, s>>>((uint32_t*)d, (const uint32_t*)src, n);
  } else {
    const int64_t n = (int64_t)bytes;
    detail::copy_words_kernel<uint8_t><<<detail::words_grid(n), 256, 0, s>>>((uint8_t*)d, (const uint8_t*)src, n);
  }
  return hipGetLastError();
}

// ---- allocation log (diagnosis build) --------------------------------------
namespace detail {
inline FILE* alloc_log() {
#if MAMG_DIAG
  static FILE* f = [] {
    const char* e = std::getenv("MAMG_ALLOC_LOG");
    return e && *e ? std::fopen(e, "w") : (FILE*)nullptr;
  }();
  return f;
#else
  return nullptr;
#endif
}
inline std::mutex& alloc_log_mu() {
  static std::mutex m;
  return m;
}
}  // namespace detail

// every device allocation and free of the library goes through these two
// (kind: tmp = setup temporary, long = handle-owned array, place = re-homed
// stream, pre = the layout reservation, scratch = scan/sort storage)
inline hipError_t raw_malloc(void** p, size_t b, const char* kind) {
  hipError_t e;
#if MAMG_DIAG
  static const bool contig = [] {
    const char* v = std::getenv("MAMG_DIAG_CONTIG");
    return v && std::atoi(v) == 1;
  }();
  if (contig && std::strcmp(kind, "place") == 0) {
    e = hipExtMallocWithFlags(p, b, hipDeviceMallocContiguous);
    if (e != hipSuccess) { (void)hipGetLastError(); e = hipMalloc(p, b); }
  } else {
    e = hipMalloc(p, b);
  }
#else
  e = hipMalloc(p, b);
#endif
  if (FILE* f = detail::alloc_log(); f && e == hipSuccess) {
    std::lock_guard<std::mutex> g(detail::alloc_log_mu());
    int d = 0;
    (void)hipGetDevice(&d);
    std::fprintf(f, "M %p %zu %s %d\n", *p, b, kind, d);
    std::fflush(f);
  }
  return e;
}
inline hipError_t raw_free(void* p) {
  if (FILE* f = detail::alloc_log(); f && p) {
    std::lock_guard<std::mutex> g(detail::alloc_log_mu());
    std::fprintf(f, "F %p\n", p);
    std::fflush(f);
  }
  return hipFree(p);
}

// diagnosis build: MAMG_DEBUG_PTRS checks (false in the product)
inline bool debug_ptrs() {
#if MAMG_DIAG
  static const bool on = [] {
    const char* e = std::getenv("MAMG_DEBUG_PTRS");
    return e && std::atoi(e) != 0;
  }();
  return on;
#else
  return false;
#endif
}

// p must start a live runtime allocation of at least b bytes
inline void check_block(const void* p, size_t b, const char* what) {
  if (!debug_ptrs() || !p) return;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  const hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p);
  if (e != hipSuccess || base != (hipDeviceptr_t)p || size < b) {
    (void)hipGetLastError();
    std::fprintf(stderr, "[mamg debug] %s %p (%zu B): %s, allocation base %p size %zu\n", what, p, b,
                 e != hipSuccess ? hipGetErrorString(e) : "not the start of a large enough allocation", (void*)base,
                 size);
  }
}

// 0: null-stream ordered (the product), 1: drain + hipFree, 2: plain
// hipFree (diagnosis build only); read once per process (a block must be
// freed the way it was allocated)
inline int free_mode() {
#if MAMG_DIAG
  static const int m = [] {
    const char* e = std::getenv("MAMG_FREE_MODE");
    if (e && std::strcmp(e, "drain") == 0) return 1;
    if (e && std::strcmp(e, "plain") == 0) return 2;
    return 0;
  }();
  return m;
#else
  return 0;
#endif
}

namespace detail {
// hipMalloc'd setup temporaries: every block the cache made, with its device
// (so a block freed while another device is current goes back to its own
// device's idle list), and the idle blocks of each device by size
struct TmpBlock {
  size_t bytes;
  int dev;
  bool idle;
};
struct TmpCache {
  std::mutex m;
  std::unordered_map<void*, TmpBlock> made;
  std::multimap<size_t, void*> idle[64];
};
inline TmpCache& tmp_cache() {
  static TmpCache c;
  return c;
}
inline int cur_device() {
  int d = 0;
  (void)hipGetDevice(&d);
  return d & 63;
}
// 4 KiB granules up to 1 MiB, 2 MiB granules above
inline size_t tmp_round(size_t b) {
  b = std::max<size_t>(b, 1);
  return b <= ((size_t)1 << 20) ? (b + 4095) & ~(size_t)4095 : (b + ((size_t)2 << 20) - 1) & ~(((size_t)2 << 20) - 1);
}
}  // namespace detail

// ---- the SpGEMM staging block (gsetup.hip spgemm_gl) ------------------------
// One block per device, allocated at its first use and kept, like the idle
// temporaries, until the cache is released (tmp_trim_dev): a large block
// allocated late, in a heap that earlier handles have fragmented, was written
// ~50x slower (profiles/r05_spgemm_stage_pool.txt).  A product holds it for
// the whole call (busy): a second host thread's setup on the same device
// meanwhile gets none and runs the unstaged two-pass product (same bits).
namespace detail {
struct StagePool {
  void* p = nullptr;
  size_t bytes = 0;
  bool busy = false;
};
inline std::mutex& stage_mu() {
  static std::mutex m;
  return m;
}
inline StagePool* stage_pools() {
  static StagePool s[64];
  return s;
}
}  // namespace detail

// free device d's staging block unless a product holds it (the caller has
// drained d's null stream, where its last users were queued)
inline void stage_free_dev(int d) {
  std::lock_guard<std::mutex> g(detail::stage_mu());
  detail::StagePool& sp = detail::stage_pools()[d & 63];
  if (!sp.p || sp.busy) return;
  (void)raw_free(sp.p);
  sp.p = nullptr;
  sp.bytes = 0;
}

// hipFree every idle cached block of device d and its staging block (after
// d's null stream has drained: the last users of an idle block were queued
// there); the current device is put back
inline void tmp_trim_dev(int d) {
  auto& c = detail::tmp_cache();
  bool stage;
  {
    std::lock_guard<std::mutex> g(detail::stage_mu());
    const detail::StagePool& sp = detail::stage_pools()[d & 63];
    stage = sp.p && !sp.busy;
  }
  std::lock_guard<std::mutex> g(c.m);
  auto& idle = c.idle[d & 63];
  if (idle.empty() && !stage) return;
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) { (void)hipGetLastError(); return; }
  if (cur != d && hipSetDevice(d) != hipSuccess) { (void)hipGetLastError(); return; }
  (void)hipStreamSynchronize(nullptr);
  for (auto& kv : idle) {
    (void)raw_free(kv.second);
    c.made.erase(kv.second);
  }
  idle.clear();
  if (stage) stage_free_dev(d);
  if (cur != d) (void)hipSetDevice(cur);
}

// the current device's idle blocks
inline void tmp_trim() { tmp_trim_dev(detail::cur_device()); }

// every device's idle blocks and staging blocks (mamg_release_setup_cache)
inline void tmp_trim_all() {
  for (int d = 0; d < 64; ++d) {
    bool any;
    {
      auto& c = detail::tmp_cache();
      std::lock_guard<std::mutex> g(c.m);
      any = !c.idle[d].empty();
    }
    {
      std::lock_guard<std::mutex> g(detail::stage_mu());
      any = any || detail::stage_pools()[d].p != nullptr;
    }
    if (any) tmp_trim_dev(d);
  }
}

// Bound of the idle cache (bytes per device) kept after a setup: the idle
// blocks above it are freed at the end of every setup, largest first, so the
// next setup of the process still finds the common sizes.  < 0: the default,
// an eighth of the device's HBM (36 GB on an MI355X); 0: everything released
// at the end of every setup (mamg_set_setup_cache_limit).
namespace detail {
inline int64_t& cache_limit() {
  static int64_t v = -1;
  return v;
}
}  // namespace detail
inline void set_cache_limit(int64_t bytes) { detail::cache_limit() = bytes; }
inline int64_t cache_limit_dev(int d) {
  const int64_t v = detail::cache_limit();
  if (v >= 0) return v;
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, d) != hipSuccess) { (void)hipGetLastError(); return 0; }
  return (int64_t)(pr.totalGlobalMem / 8);
}

// idle bytes cached on device d (tests, the bound)
inline int64_t tmp_idle_bytes(int d) {
  auto& c = detail::tmp_cache();
  std::lock_guard<std::mutex> g(c.m);
  int64_t b = 0;
  for (auto& kv : c.idle[d & 63]) b += (int64_t)kv.first;
  return b;
}

// the end of a setup: every device's idle cache down to the bound (the
// staging block is counted against it too; above the bound it is freed first)
inline void tmp_trim_to_limit_all() {
  for (int d = 0; d < 64; ++d) {
    auto& c = detail::tmp_cache();
    int64_t idle_b = 0;
    size_t stage_b = 0;
    {
      std::lock_guard<std::mutex> g(c.m);
      for (auto& kv : c.idle[d]) idle_b += (int64_t)kv.first;
    }
    {
      std::lock_guard<std::mutex> g(detail::stage_mu());
      const detail::StagePool& sp = detail::stage_pools()[d];
      if (sp.p && !sp.busy) stage_b = sp.bytes;
    }
    if (idle_b == 0 && stage_b == 0) continue;
    const int64_t lim = cache_limit_dev(d);
    if (idle_b + (int64_t)stage_b <= lim) continue;
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) { (void)hipGetLastError(); continue; }
    if (cur != d && hipSetDevice(d) != hipSuccess) { (void)hipGetLastError(); continue; }
    (void)hipStreamSynchronize(nullptr);
    if (lim == 0 || (int64_t)stage_b > lim) {
      stage_free_dev(d);
      stage_b = 0;
    }
    {
      std::lock_guard<std::mutex> g(c.m);
      auto& idle = c.idle[d];
      int64_t tot = 0;
      for (auto& kv : idle) tot += (int64_t)kv.first;
      while (!idle.empty() && tot + (int64_t)stage_b > lim) {
        auto it = std::prev(idle.end());   // the largest idle block
        tot -= (int64_t)it->first;
        (void)raw_free(it->second);
        c.made.erase(it->second);
        idle.erase(it);
      }
    }
    if (cur != d) (void)hipSetDevice(cur);
  }
}

// the staging block of the current device for one product: its size and
// pointer (0 / nullptr when none fits or another product holds it); the
// product releases it when done (StageLease)
inline size_t stage_acquire(size_t cap_bytes, void** p) {
  const int d = detail::cur_device();
  std::lock_guard<std::mutex> g(detail::stage_mu());
  detail::StagePool& sp = detail::stage_pools()[d];
  *p = nullptr;
  if (sp.busy) return 0;
  if (!sp.p && cap_bytes > 0) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
      const size_t b = (size_t)std::min((double)cap_bytes, 0.25 * (double)fr) & ~(((size_t)2 << 20) - 1);
      if (b >= ((size_t)64 << 20) && raw_malloc(&sp.p, b, "scratch") == hipSuccess) sp.bytes = b;
      else sp.p = nullptr;
    }
    (void)hipGetLastError();
  }
  if (!sp.p) return 0;
  sp.busy = true;
  *p = sp.p;
  return sp.bytes;
}
inline void stage_release(int d) {
  std::lock_guard<std::mutex> g(detail::stage_mu());
  detail::stage_pools()[d & 63].busy = false;
}
// the staging block held for one product (released when it goes out of scope)
struct StageLease {
  int dev = 0;
  void* p = nullptr;
  size_t bytes = 0;
  explicit StageLease(size_t cap_bytes) : dev(detail::cur_device()) { bytes = stage_acquire(cap_bytes, &p); }
  ~StageLease() {
    if (p) stage_release(dev);
  }
  StageLease(const StageLease&) = delete;
  StageLease& operator=(const StageLease&) = delete;
};

// hipMalloc for the library's long-lived arrays: when HBM runs out while the
// setup temporaries' cache holds idle blocks, the cache is emptied and the
// allocation tried once more
inline hipError_t dev_malloc(void** p, size_t b, const char* kind = "long") {
  hipError_t e = raw_malloc(p, b, kind);
  if (e == hipErrorOutOfMemory) {
    (void)hipGetLastError();
    tmp_trim();
    e = raw_malloc(p, b, kind);
  }
  return e;
}

// a setup temporary of b bytes (null-stream ordered): an idle cached block
// of the current device of at most 5/4 of the rounded size, else a new
// hipMalloc (the idle blocks are released and the allocation tried again
// when HBM runs out)
inline hipError_t tmp_malloc(void** p, size_t b) {
  if (free_mode() != 0) return raw_malloc(p, b, "tmp");
  auto& c = detail::tmp_cache();
  const int d = detail::cur_device();
  const size_t r = detail::tmp_round(b);
  {
    std::lock_guard<std::mutex> g(c.m);
    auto& idle = c.idle[d];
    auto it = idle.lower_bound(r);
    if (it != idle.end() && it->first <= r + r / 4) {
      *p = it->second;
      idle.erase(it);
      c.made[*p].idle = false;
      check_block(*p, r, "tmp_malloc (cached)");
      return hipSuccess;
    }
  }
  hipError_t e = raw_malloc(p, r, "tmp");
  if (e == hipErrorOutOfMemory) {
    (void)hipGetLastError();
    tmp_trim();
    e = raw_malloc(p, r, "tmp");
  }
  if (e != hipSuccess) return e;
  check_block(*p, r, "tmp_malloc (new)");
  std::lock_guard<std::mutex> g(c.m);
  c.made[*p] = detail::TmpBlock{r, d, false};
  return hipSuccess;
}

// back to the idle list of the block's own device, whatever device is current
inline void tmp_free(void* p) {
  if (!p) return;
  switch (free_mode()) {
    case 0: {
      auto& c = detail::tmp_cache();
      std::lock_guard<std::mutex> g(c.m);
      auto it = c.made.find(p);
      if (it == c.made.end() || it->second.idle) {   // not a live cached block: a bug of the caller
        std::fprintf(stderr, "[mamg] tmp_free(%p): %s\n", p, it == c.made.end() ? "unknown block" : "freed twice");
        break;
      }
      it->second.idle = true;
      c.idle[it->second.dev].emplace(it->second.bytes, p);
      break;
    }
    case 1: (void)hipDeviceSynchronize(); (void)raw_free(p); break;
    default: (void)raw_free(p); break;
  }
}

// cached temporaries of device d: (live, idle) block counts (tests)
inline void tmp_counts(int d, int64_t* live, int64_t* idle) {
  auto& c = detail::tmp_cache();
  std::lock_guard<std::mutex> g(c.m);
  *live = *idle = 0;
  for (auto& kv : c.made)
    if (kv.second.dev == (d & 63)) ++(kv.second.idle ? *idle : *live);
}

// a hipMalloc'd array whose last reader is queued on the null stream
inline void ordered_free(void* p) {
  if (!p) return;
  const int m = free_mode();
  if (m == 0) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) {
      (void)hipEventRecord(e, nullptr);
      (void)hipEventSynchronize(e);
      (void)hipEventDestroy(e);
    }
  } else if (m == 1) {
    (void)hipDeviceSynchronize();
  }
  (void)raw_free(p);
}

}  // namespace mamg
