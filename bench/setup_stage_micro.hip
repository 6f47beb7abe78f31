// setup_stage_micro.hip -- why do the level-0 setup merges (block_rho,
// node_graph_fill, csr2bsr_fill) and the SpGEMM pair check run at ~0.1-1 TB/s
// on the nrefs=6 matrix (17 M nodes, ~30 entries per scalar row, 12 GB of
// field-major CSR)?  Synthetic matrix of that shape built on the device;
// times (a) the row staging loop one load per iteration (rowstage.h before
// round 5's batching) vs batched, (b) the sampled pair check.
//
//   hipcc -O3 --offload-arch=gfx950 bench/setup_stage_micro.hip -o /tmp/setup_stage_micro
//   /tmp/setup_stage_micro [nodes=16974593] [node_cols=15]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

constexpr int CAP = 2048;

// row r = f nv + I holds node columns I + o (o in [-w/2, w/2], clipped) of
// both fields: 2 m entries, m the clipped count
__global__ void build_kernel(int64_t nv, int w, int64_t* ptr, int32_t* col, double* val) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= 2 * nv) return;
  const int64_t I = r % nv;
  const int64_t lo = I - w / 2 < 0 ? 0 : I - w / 2, hi = I + w / 2 >= nv ? nv - 1 : I + w / 2;
  const int64_t m = hi - lo + 1;
  // entries before row r: rows are 2 m' long; full rows have 2 (w/2*2+1)
  const int64_t full = 2 * (2 * (w / 2) + 1);
  int64_t before = (r - r / nv * nv) * full + (r / nv) * nv * full;   // approximate layout: fixed stride
  ptr[r] = before;
  for (int64_t k = 0; k < 2 * m; ++k) {
    const int64_t j = k < m ? lo + k : nv + lo + (k - m);
    col[before + k] = (int32_t)j;
    val[before + k] = 1.0 + 1e-3 * (double)(k & 7);
  }
  for (int64_t k = 2 * m; k < full; ++k) {   // pad clipped rows with repeats of the last column
    col[before + k] = col[before + 2 * m - 1];
    val[before + k] = 0.0;
  }
  if (r == 2 * nv - 1) ptr[2 * nv] = before + full;
}

template <int U>
__global__ __launch_bounds__(64) void stage_kernel(int64_t nv, const int64_t* __restrict__ ptr,
                                                   const int32_t* __restrict__ col, const double* __restrict__ val,
                                                   double* out) {
  __shared__ int32_t c[2][CAP];
  __shared__ double v[2][CAP];
  const int lane = threadIdx.x;
  const int64_t I0 = (int64_t)blockIdx.x * 64, I1 = I0 + 64 < nv ? I0 + 64 : nv;
  int64_t b[2], n[2];
  for (int f = 0; f < 2; ++f) {
    b[f] = ptr[f * nv + I0];
    n[f] = ptr[f * nv + I1] - b[f];
  }
  if (n[0] > CAP || n[1] > CAP) return;
  if (U == 1) {
    for (int f = 0; f < 2; ++f)
      for (int64_t t = lane; t < n[f]; t += 64) {
        c[f][t] = col[b[f] + t];
        v[f][t] = val[b[f] + t];
      }
  } else {
    for (int f = 0; f < 2; ++f)
      for (int64_t t0 = 0; t0 < n[f]; t0 += 64 * U) {
        int32_t cc[U];
        double vv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t t = t0 + u * 64 + lane;
          if (t < n[f]) { cc[u] = col[b[f] + t]; vv[u] = val[b[f] + t]; }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t t = t0 + u * 64 + lane;
          if (t < n[f]) { c[f][t] = cc[u]; v[f][t] = vv[u]; }
        }
      }
  }
  __syncthreads();
  // a light per-lane use of the staged rows (sum of the node's row)
  const int64_t I = I0 + lane;
  if (I >= nv) return;
  double s = 0.0;
  for (int64_t k = ptr[I]; k < ptr[I + 1]; ++k) s += v[0][k - b[0]] * (double)(c[0][k - b[0]] & 1);
  out[I] = s;
}

constexpr int64_t PAIR_SAMPLE = 61;
__global__ __launch_bounds__(256) void pair_diff_kernel(int64_t h, const int64_t* __restrict__ aptr,
                                                        const int32_t* __restrict__ acol, unsigned long long* diff) {
  const int64_t p = ((int64_t)blockIdx.x * 256 + threadIdx.x) * PAIR_SAMPLE;
  bool d = false;
  if (p < h) {
    const int64_t p0 = aptr[p], p1 = aptr[p + h], L = aptr[p + 1] - p0;
    d = aptr[p + h + 1] - p1 != L;
    for (int64_t t = 0; !d && t < L; ++t) d = acol[p0 + t] != acol[p1 + t];
  }
  const unsigned long long b = __ballot(d);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(diff + (blockIdx.x & 63) * 16, (unsigned long long)__popcll(b));
}

int main(int argc, char** argv) {
  const int64_t nv = argc > 1 ? std::atoll(argv[1]) : 16974593;
  const int w = argc > 2 ? std::atoi(argv[2]) : 15;
  const int64_t full = 2 * (2 * (w / 2) + 1), nnz = 2 * nv * full;
  int64_t* ptr;
  int32_t* col;
  double *val, *out;
  unsigned long long* diff;
  CK(hipMalloc(&ptr, (2 * nv + 1) * sizeof(int64_t)));
  CK(hipMalloc(&col, nnz * sizeof(int32_t)));
  CK(hipMalloc(&val, nnz * sizeof(double)));
  CK(hipMalloc(&out, nv * sizeof(double)));
  CK(hipMalloc(&diff, 64 * 16 * sizeof(unsigned long long)));
  build_kernel<<<(unsigned)((2 * nv + 255) / 256), 256>>>(nv, w, ptr, col, val);
  CK(hipDeviceSynchronize());
  std::printf("nodes %lld, %lld entries per row, %.2f GB of CSR\n", (long long)nv, (long long)full, nnz * 12e-9);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double gb, auto&& fn) {
    fn();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0));
      fn();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    std::printf("%-28s %8.3f ms  %7.0f GB/s\n", name, best, gb / best * 1e3);
  };
  const unsigned g = (unsigned)((nv + 63) / 64);
  const double gb = nnz * 12e-9;
  timeit("stage, 1 load per iter", gb, [&] { stage_kernel<1><<<g, 64>>>(nv, ptr, col, val, out); });
  timeit("stage, 4 loads batched", gb, [&] { stage_kernel<4><<<g, 64>>>(nv, ptr, col, val, out); });
  timeit("stage, 8 loads batched", gb, [&] { stage_kernel<8><<<g, 64>>>(nv, ptr, col, val, out); });
  const int64_t ns = (nv + PAIR_SAMPLE - 1) / PAIR_SAMPLE;
  timeit("pair_diff (sampled)", ns * full * 8e-9, [&] {
    CK(hipMemset(diff, 0, 64 * 16 * sizeof(unsigned long long)));
    pair_diff_kernel<<<(unsigned)((ns + 255) / 256), 256>>>(nv, ptr, col, diff);
  });
  CK(hipGetLastError());
  return 0;
}
