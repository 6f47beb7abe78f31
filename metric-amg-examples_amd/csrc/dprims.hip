// dprims.hip -- device scan / stable radix sort (hipCUB) behind plain
// functions, kept in their own translation unit so the template-heavy library
// is compiled once.  Used by the GPU setup and the device layout builder.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "gsetup.h"

namespace mamg {

namespace {
int hip_fail(hipError_t e, const char* what, std::string* err) {
  *err = std::string(what) + ": " + hipGetErrorString(e);
  return MAMG_ERR_HIP;
}
}  // namespace

// out[i] = in[0] + ... + in[i]  (in == out allowed)
int dscan_incl_i64(const int64_t* in, int64_t* out, int64_t n, void* stream, std::string* err) {
  if (n <= 0) return MAMG_OK;
  hipStream_t s = (hipStream_t)stream;
  size_t bytes = 0;
  hipError_t e = hipcub::DeviceScan::InclusiveSum(nullptr, bytes, in, out, (size_t)n, s);
  if (e != hipSuccess) return hip_fail(e, "DeviceScan::InclusiveSum(size)", err);
  void* tmp = nullptr;
  if ((e = hipMallocAsync(&tmp, bytes + 16, s)) != hipSuccess) return hip_fail(e, "hipMallocAsync(scan)", err);
  e = hipcub::DeviceScan::InclusiveSum(tmp, bytes, in, out, (size_t)n, s);
  hipError_t e2 = hipFreeAsync(tmp, s);
  if (e != hipSuccess) return hip_fail(e, "DeviceScan::InclusiveSum", err);
  if (e2 != hipSuccess) return hip_fail(e2, "hipFreeAsync(scan)", err);
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
  void* tmp = nullptr;
  if ((e = hipMallocAsync(&tmp, bytes + 16, s)) != hipSuccess) return hip_fail(e, "hipMallocAsync(sort)", err);
  e = hipcub::DeviceRadixSort::SortPairs(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0, key_bits, s);
  hipError_t e2 = hipFreeAsync(tmp, s);
  if (e != hipSuccess) return hip_fail(e, "DeviceRadixSort::SortPairs", err);
  if (e2 != hipSuccess) return hip_fail(e2, "hipFreeAsync(sort)", err);
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
