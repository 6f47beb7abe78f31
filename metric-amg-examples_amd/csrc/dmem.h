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

// hipFree every idle cached block of device d (after d's null stream has
// drained: the last users of an idle block were queued there); the current
// device is put back
inline void tmp_trim_dev(int d) {
  auto& c = detail::tmp_cache();
  std::lock_guard<std::mutex> g(c.m);
  auto& idle = c.idle[d & 63];
  if (idle.empty()) return;
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) { (void)hipGetLastError(); return; }
  if (cur != d && hipSetDevice(d) != hipSuccess) { (void)hipGetLastError(); return; }
  (void)hipStreamSynchronize(nullptr);
  for (auto& kv : idle) {
    (void)raw_free(kv.second);
    c.made.erase(kv.second);
  }
  idle.clear();
  if (cur != d) (void)hipSetDevice(cur);
}

// the current device's idle blocks
inline void tmp_trim() { tmp_trim_dev(detail::cur_device()); }

// every device's idle blocks (the end of a setup)
inline void tmp_trim_all() {
  for (int d = 0; d < 64; ++d) {
    bool any;
    {
      auto& c = detail::tmp_cache();
      std::lock_guard<std::mutex> g(c.m);
      any = !c.idle[d].empty();
    }
    if (any) tmp_trim_dev(d);
  }
}

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
