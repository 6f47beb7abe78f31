// dmem.h -- freeing device temporaries (device.hip, gsetup.hip).
//
// Round-3 intermittent wrong operators were cured by draining the device
// before every free (VERDICT r03 "next round" #1).  This header funnels every
// such free through one function so that the mechanism can be measured:
//   MAMG_DRAIN=0    free without the device-wide drain (diagnosis only)
//   MAMG_FREELOG=1  print every free issued while null-stream work is still
//                   pending, with the time the hipFree call itself took
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

namespace mamg {

inline void free_after_drain(void* p, const char* site) {
  if (!p) return;
  const char* lg = std::getenv("MAMG_FREELOG");
  const bool log = lg && *lg == '1';
  bool pending = false;
  if (log) {
    pending = hipStreamQuery(nullptr) == hipErrorNotReady;
    (void)hipGetLastError();
  }
  const char* d = std::getenv("MAMG_DRAIN");
  if (!d || std::atoi(d) != 0) (void)hipDeviceSynchronize();
  const auto t0 = std::chrono::steady_clock::now();
  (void)hipFree(p);
  if (log && pending) {
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const bool still = hipStreamQuery(nullptr) == hipErrorNotReady;
    (void)hipGetLastError();
    std::fprintf(stderr, "[mamg freelog] %s: %p freed with null-stream work pending; hipFree %.3f ms; pending after: %d\n",
                 site, p, ms, (int)still);
  }
}

}  // namespace mamg
