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

#include <cstdlib>
#include <cstring>

namespace mamg {

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
