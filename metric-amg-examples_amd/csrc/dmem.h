// dmem.h -- lifetimes of device buffers made during setup (device.hip,
// gsetup.hip).
//
// Every kernel, memset and copy of the GPU setup and of the apply-layout
// builder runs on the null stream, and so do the temporaries' lifetimes:
//  * temporaries (Scratch, TmpPool, GHier, the seed-ring blocks) come from
//    hipMallocAsync and go back with hipFreeAsync on the null stream.  The
//    pool hands a freed block to a later allocation only once the stream has
//    passed the free, i.e. after every kernel queued before it that reads the
//    block -- no drain of the device, and no reuse under a running reader;
//  * a long-lived (hipMalloc) array replaced during setup (operator re-homing,
//    K region candidates) is freed after an event recorded on the null stream
//    behind its last reader has completed (ordered_free): a wait on that one
//    stream, not on the device.
// Round 3 drained the whole device before every hipFree instead (free-after-
// drain); DESIGN.md section 4.1 records what the round-4 diagnosis
// (bench/free_race.hip, scripts/gpu_freediag.sh) measured about hipFree.
//   MAMG_FREE_MODE=drain   round 3's drain + hipFree (diagnosis only)
//   MAMG_FREE_MODE=plain   hipMalloc / hipFree with no ordering of our own
//                          (the round-2 code; diagnosis only)
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>

namespace mamg {

// Device fills and device-to-device copies by the library's own kernels
// instead of hipMemset / hipMemcpy(DeviceToDevice).  Round 4 traced the
// intermittent wrong operators to whole 128-byte
// lines of a kernel's output that still held the bytes an earlier runtime
// fill had left in the same recycled memory (zeros, or the NaN pattern of a
// diagnosis fill) after the kernel had written them: the runtime's fill /
// copy kernels' writes surfaced over later data.  Every fill and device
// copy of the setup, the layout builder and the apply goes through these
// (same stream semantics: ordered on stream s, asynchronous to the host).
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

// write back and invalidate every XCD's L2 (a system-scope fence in
// workgroups spread over all CUs); ordered on stream s
namespace detail {
template <int N>   // a template: one definition however many units include this
__global__ __launch_bounds__(64) void l2_flush_kernel() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, ""); }
}  // namespace detail
inline hipError_t l2_flush(hipStream_t s = nullptr) {
  detail::l2_flush_kernel<0><<<2048, 64, 0, s>>>();
  return hipGetLastError();
}

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

// 0: stream-ordered (default), 1: drain + hipFree, 2: plain hipFree; read
// once per process (a block must be freed the way it was allocated)
inline int free_mode() {
  static const int m = [] {
    const char* e = std::getenv("MAMG_FREE_MODE");
    if (e && std::strcmp(e, "drain") == 0) return 1;
    if (e && std::strcmp(e, "plain") == 0) return 2;
    return 0;
  }();
  return m;
}

// a setup temporary of b bytes (null-stream ordered)
inline hipError_t tmp_malloc(void** p, size_t b) {
  if (free_mode() != 0) return hipMalloc(p, b);
  return hipMallocAsync(p, b, nullptr);
}

inline void tmp_free(void* p) {
  if (!p) return;
  switch (free_mode()) {
    case 0: (void)hipFreeAsync(p, nullptr); break;
    case 1: (void)hipDeviceSynchronize(); (void)hipFree(p); break;
    default: (void)hipFree(p); break;
  }
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
  (void)hipFree(p);
}

}  // namespace mamg
