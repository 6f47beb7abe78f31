// dprims.hip -- device scan / stable radix sort (hipCUB) behind plain
// functions, kept in their own translation unit so the template-heavy library
// is compiled once.  Used by the GPU setup and the device layout builder.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <mutex>
#include <vector>

#include "dmem.h"
#include "gsetup.h"

namespace mamg {

namespace {
int hip_fail(hipError_t e, const char* what, std::string* err) {
  *err = std::string(what) + ": " + hipGetErrorString(e);
  return MAMG_ERR_HIP;
}

// Temporary storage of the scans and sorts: hipMalloc'd blocks kept for
// these primitives only, per device, never returned to the allocator that
// serves the setup's data arrays.  A block is reused
// in null-stream order: every user issues on the null stream and returns
// the block behind its last kernel.
struct ScratchBlock {
  int dev;
  void* p;
  size_t bytes;
  bool busy;
};
std::mutex g_scratch_mu;
std::vector<ScratchBlock> g_scratch;

void* scratch_get(size_t bytes, hipError_t* e) {
  int dev = 0;
  if ((*e = hipGetDevice(&dev)) != hipSuccess) return nullptr;
  {
    std::lock_guard<std::mutex> g(g_scratch_mu);
    for (auto& b : g_scratch)
      if (!b.busy && b.dev == dev && b.bytes >= bytes) {
        b.busy = true;
        return b.p;
      }
  }
  const size_t n = std::max<size_t>(bytes, (size_t)1 << 20);
  void* p = nullptr;
  if ((*e = dev_malloc(&p, n, "scratch")) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> g(g_scratch_mu);
  g_scratch.push_back({dev, p, n, true});
  return p;
}

void scratch_put(void* p) {
  std::lock_guard<std::mutex> g(g_scratch_mu);
  for (auto& b : g_scratch)
    if (b.p == p) b.busy = false;
}
}  // namespace

void dprims_warm(void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int64_t* buf = nullptr;
  size_t bytes = 0;
  if (hipcub::DeviceScan::InclusiveSum(nullptr, bytes, buf, buf, (size_t)1, s) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  void* p = nullptr;   // two words + the scan's storage, kept for the process (no hipFree here)
  if (dev_malloc(&p, 64 + bytes, "scratch") != hipSuccess) { (void)hipGetLastError(); return; }
  buf = (int64_t*)p;
  if (hipMemsetAsync(buf, 0, 16, s) != hipSuccess ||
      hipcub::DeviceScan::InclusiveSum((char*)p + 64, bytes, buf, buf + 1, (size_t)1, s) != hipSuccess)
    (void)hipGetLastError();
}

// out[i] = in[0] + ... + in[i]  (in == out allowed)
int dscan_incl_i64(const int64_t* in, int64_t* out, int64_t n, void* stream, std::string* err) {
  if (n <= 0) return MAMG_OK;
  hipStream_t s = (hipStream_t)stream;
  size_t bytes = 0;
  hipError_t e = hipcub::DeviceScan::InclusiveSum(nullptr, bytes, in, out, (size_t)n, s);
  if (e != hipSuccess) return hip_fail(e, "DeviceScan::InclusiveSum(size)", err);
  void* tmp = scratch_get(bytes + 16, &e);
  if (!tmp) return hip_fail(e, "hipMalloc(scan scratch)", err);
  e = hipcub::DeviceScan::InclusiveSum(tmp, bytes, in, out, (size_t)n, s);
  scratch_put(tmp);
  if (e != hipSuccess) return hip_fail(e, "DeviceScan::InclusiveSum", err);
  return MAMG_OK;
}

namespace {
template <class K>
int sort_pairs(const K* kin, K* kout, const int64_t* vin, int64_t* vout, int64_t n, int key_bits,
               void* stream, std::string* err) {
  if (n <= 0) return MAMG_OK;
  hipStream_t s = (hipStream_t)stream;
  size_t bytes = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, kin, kout, vin, vout, (size_t)n, 0,
                                                    key_bits, s);
  if (e != hipSuccess) return hip_fail(e, "DeviceRadixSort::SortPairs(size)", err);
  void* tmp = scratch_get(bytes + 16, &e);
  if (!tmp) return hip_fail(e, "hipMalloc(sort scratch)", err);
  e = hipcub::DeviceRadixSort::SortPairs(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0, key_bits, s);
  scratch_put(tmp);
  if (e != hipSuccess) return hip_fail(e, "DeviceRadixSort::SortPairs", err);
  return MAMG_OK;
}
}  // namespace

// the same for 64-bit keys (composite (row, column) keys of the GPU setup)
int dsort_pairs_u64_i64(const uint64_t* kin, uint64_t* kout, const int64_t* vin, int64_t* vout,
                        int64_t n, int key_bits, void* stream, std::string* err) {
  return sort_pairs(kin, kout, vin, vout, n, key_bits, stream, err);
}

// stable LSD radix sort of (key, value) pairs on the low key_bits of the key
int dsort_pairs_i32_i64(const int32_t* kin, int32_t* kout, const int64_t* vin, int64_t* vout,
                        int64_t n, int key_bits, void* stream, std::string* err) {
  return sort_pairs(kin, kout, vin, vout, n, key_bits, stream, err);
}

}  // namespace mamg
