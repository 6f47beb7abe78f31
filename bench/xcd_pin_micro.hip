// xcd_pin_micro.hip -- does pinning a chain of tiny dependent kernels to one
// XCD (8x the workgroups, the ones not on XCD 0 exit at once, HW_REG_XCC_ID)
// make them cheaper, by keeping their working set warm in that XCD's L2?
// The coarse levels of the reference family's W-cycle are ~12 k launches
// per apply of kernels like this.
//
//   hipcc -O3 --offload-arch=gfx950 bench/xcd_pin_micro.hip -o /tmp/xcd_pin_micro
//   /tmp/xcd_pin_micro [rows=1400] [nnz_per_row=30] [launches=4000]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

__device__ __forceinline__ unsigned xcc_id() {
  return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);   // HW_REG_XCC_ID, bits 3:0
}

// one Jacobi-like row update: x_new[i] = b[i] - sum_j a_ij x[j] over a
// colour's rows (the rows [r0, r1)), 4 lanes per row
template <bool PIN>
__global__ __launch_bounds__(256) void step_kernel(int r0, int r1, const int* __restrict__ ptr, const int* __restrict__ col,
                                                   const double* __restrict__ val, const double* __restrict__ b,
                                                   double* x) {
  int blk = blockIdx.x;
  if (PIN) {
    if (xcc_id() != 0) return;
    blk = blockIdx.x >> 3;
  }
  const int t = blk * 256 + threadIdx.x, r = r0 + t / 4, l = t & 3;
  double s = 0.0;
  if (r < r1)
    for (int k = ptr[r] + l; k < ptr[r + 1]; k += 4) s += val[k] * x[col[k]];
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  if (r < r1 && l == 0) x[r] = 0.5 * (b[r] - s) + 0.5 * x[r];
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 1400;
  const int w = argc > 2 ? std::atoi(argv[2]) : 30;
  const int L = argc > 3 ? std::atoi(argv[3]) : 4000;
  std::vector<int> ptr(n + 1), col((size_t)n * w);
  std::vector<double> val((size_t)n * w), b(n, 1.0), x(n, 0.0);
  srand(7);
  for (int i = 0; i <= n; ++i) ptr[i] = i * w;
  for (size_t k = 0; k < col.size(); ++k) { col[k] = rand() % n; val[k] = 1e-3 * (rand() % 100); }
  int *dptr, *dcol;
  double *dval, *db, *dx;
  CK(hipMalloc(&dptr, (n + 1) * sizeof(int)));
  CK(hipMalloc(&dcol, col.size() * sizeof(int)));
  CK(hipMalloc(&dval, val.size() * sizeof(double)));
  CK(hipMalloc(&db, n * sizeof(double)));
  CK(hipMalloc(&dx, n * sizeof(double)));
  CK(hipMemcpy(dptr, ptr.data(), ptr.size() * sizeof(int), hipMemcpyHostToDevice));
  CK(hipMemcpy(dcol, col.data(), col.size() * sizeof(int), hipMemcpyHostToDevice));
  CK(hipMemcpy(dval, val.data(), val.size() * sizeof(double), hipMemcpyHostToDevice));
  CK(hipMemcpy(db, b.data(), n * sizeof(double), hipMemcpyHostToDevice));
  CK(hipMemcpy(dx, x.data(), n * sizeof(double), hipMemcpyHostToDevice));
  const int colours = 12, per = (n + colours - 1) / colours;
  const int wg = (per * 4 + 255) / 256;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("rows %d, %d entries per row (%.0f KB of matrix), %d colours, %d workgroup(s) per step, %d launches\n", n,
              w, (double)n * w * 12 / 1024, colours, wg, L);
  for (int rep = 0; rep < 3; ++rep)
    for (int pin = 0; pin < 2; ++pin) {
      for (int graph = 0; graph < 2; ++graph) {
        auto issue = [&]() {
          for (int k = 0; k < L; ++k) {
            const int c = k % colours, r0 = c * per, r1 = std::min(n, r0 + per);
            if (pin) step_kernel<true><<<8 * wg, 256, 0, s>>>(r0, r1, dptr, dcol, dval, db, dx);
            else step_kernel<false><<<wg, 256, 0, s>>>(r0, r1, dptr, dcol, dval, db, dx);
          }
        };
        float ms = 0.f;
        if (!graph) {
          issue();   // warm
          CK(hipStreamSynchronize(s));
          CK(hipEventRecord(e0, s));
          issue();
          CK(hipEventRecord(e1, s));
        } else {
          hipGraph_t g;
          hipGraphExec_t ge;
          CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
          issue();
          CK(hipStreamEndCapture(s, &g));
          CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
          CK(hipGraphLaunch(ge, s));
          CK(hipStreamSynchronize(s));
          CK(hipEventRecord(e0, s));
          CK(hipGraphLaunch(ge, s));
          CK(hipEventRecord(e1, s));
          CK(hipStreamSynchronize(s));
          CK(hipGraphExecDestroy(ge));
          CK(hipGraphDestroy(g));
        }
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("rep %d %s %s: %.2f us per step\n", rep, pin ? "pinned to XCD 0" : "plain          ",
                    graph ? "graph" : "eager", 1e3 * ms / L);
      }
    }
  CK(hipGetLastError());
  return 0;
}
