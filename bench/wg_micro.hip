// wg_micro.hip -- cost of one step of a single-workgroup persistent loop
// (the coarse tail, device.hip tail_kernel): per iteration wall-clock time of
// a barrier alone, LDS / global read-modify-writes, dependent global gathers
// and flat (generic-pointer) accesses to LDS, at 1024 and 256 threads.
// Build: hipcc -O3 --offload-arch=gfx950 wg_micro.hip -o wg_micro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// MODE 0: barrier only; 1: LDS x[i] += 1 then barrier; 2: global x[i] += 1
// then barrier; 3: dependent chain idx -> val -> x gather (global) then
// barrier; 4: mode 1 through a generic pointer (flat); 5: mode 3 with x in
// LDS; 6: global store only (no read) then barrier
template <int MODE>
__global__ void step_kernel(int iters, double* __restrict__ g, const int* __restrict__ idx,
                            const double* __restrict__ val, uint64_t* __restrict__ out, int n, int flatsel) {
  __shared__ double sx[4096];
  const int t = threadIdx.x;
  for (int i = t; i < 4096; i += blockDim.x) sx[i] = 0.0;
  __syncthreads();
  double* fp = flatsel ? sx : g;   // generic pointer: LDS or global by a runtime flag
  const uint64_t t0 = wall_clock64(), c0 = clock64();
  double acc = 0.0;
  for (int it = 0; it < iters; ++it) {
    const int i = (int)(((long long)t * 131 + (long long)it * 1031) % n);
    if (MODE == 1) sx[i] += 1.0;
    if (MODE == 2) g[i] += 1.0;
    if (MODE == 3) { const int c = idx[i]; acc += val[i] * g[c]; if (t == 0) g[n + (it & 63)] = acc; }
    if (MODE == 4) fp[i] += 1.0;
    if (MODE == 5) { const int c = idx[i]; acc += val[i] * sx[c & 4095]; if (t == 0) sx[(it & 63)] = acc; }
    if (MODE == 6) g[i] = (double)it;
    __syncthreads();
  }
  const uint64_t t1 = wall_clock64(), c1 = clock64();
  if (t == 0) { out[0] = t1 - t0; out[1] = c1 - c0; }
  if (acc == 12345.0) g[0] = acc;
}

template <int MODE>
double run(int threads, int iters, double* g, int* idx, double* val, uint64_t* out, int n, int flatsel) {
  step_kernel<MODE><<<1, threads>>>(iters, g, idx, val, out, n, flatsel);
  CK(hipDeviceSynchronize());
  step_kernel<MODE><<<1, threads>>>(iters, g, idx, val, out, n, flatsel);
  CK(hipDeviceSynchronize());
  uint64_t ticks[2] = {0, 0};
  CK(hipMemcpy(ticks, out, 16, hipMemcpyDeviceToHost));
  if (MODE == 3) printf("[shader clock during mode 3: %.0f MHz] ", 100.0 * ticks[1] / ticks[0]);
  return ticks[0] * 10.0 / iters;   // 100 MHz -> ns per iteration
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 2048, iters = 20000;
  double *g, *val;
  int* idx;
  uint64_t* out;
  CK(hipMalloc(&g, (n + 64) * sizeof(double)));
  CK(hipMalloc(&val, n * sizeof(double)));
  CK(hipMalloc(&idx, n * sizeof(int)));
  CK(hipMalloc(&out, 16));
  std::vector<int> hi(n);
  for (int i = 0; i < n; ++i) hi[i] = (int)(((long long)i * 97 + 13) % n);
  printf("working set: %d doubles + %d ints (%.1f KB)\n", n, n, n * 12.0 / 1024);
  CK(hipMemcpy(idx, hi.data(), n * sizeof(int), hipMemcpyHostToDevice));
  CK(hipMemset(g, 0, (n + 64) * sizeof(double)));
  CK(hipMemset(val, 0, n * sizeof(double)));
  for (int threads : {1024, 256, 64}) {
    printf("threads %4d: barrier %.0f ns | LDS rmw %.0f | global rmw %.0f | global chain %.0f | "
           "flat->LDS rmw %.0f | flat->global rmw %.0f | chain, x in LDS %.0f | global store %.0f\n",
           threads, run<0>(threads, iters, g, idx, val, out, n, 0), run<1>(threads, iters, g, idx, val, out, n, 0),
           run<2>(threads, iters, g, idx, val, out, n, 0), run<3>(threads, iters, g, idx, val, out, n, 0),
           run<4>(threads, iters, g, idx, val, out, n, 1), run<4>(threads, iters, g, idx, val, out, n, 0),
           run<5>(threads, iters, g, idx, val, out, n, 0), run<6>(threads, iters, g, idx, val, out, n, 0));
  }
  return 0;
}
