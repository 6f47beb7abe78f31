// spmv_micro.hip -- kernel-variant microbenchmark for the level-0 operator
// (bidomain 3-D, nrefs=6: N = 34M, nnz = 1.0e9).  Times CSR and 2x2-BSR SpMV
// variants with HIP events and checks each against the CSR result.
// Build: make -C bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "mamg.h"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// ---------------- CSR, VL lanes per row, unroll U ------------------------------
template <int VL, int U, bool NT>
__global__ __launch_bounds__(256) void csr_k(int64_t n, const int64_t* __restrict__ ptr,
                                             const int32_t* __restrict__ col,
                                             const double* __restrict__ val,
                                             const double* __restrict__ x, double* __restrict__ y) {
  const int lane = threadIdx.x & (VL - 1);
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / VL;
  double s[U];
#pragma unroll
  for (int u = 0; u < U; ++u) s[u] = 0.0;
  if (row < n) {
    const int64_t p0 = ptr[row], p1 = ptr[row + 1];
    int64_t k = p0 + lane;
    for (; k + (U - 1) * VL < p1; k += U * VL) {
      int32_t c[U];
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (NT) {
          c[u] = __builtin_nontemporal_load(col + k + u * VL);
          v[u] = __builtin_nontemporal_load(val + k + u * VL);
        } else {
          c[u] = col[k + u * VL];
          v[u] = val[k + u * VL];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) s[u] += v[u] * x[c[u]];
    }
    for (; k < p1; k += VL) s[0] += val[k] * x[col[k]];
  }
  double t = 0.0;
#pragma unroll
  for (int u = 0; u < U; ++u) t += s[u];
#pragma unroll
  for (int off = VL / 2; off > 0; off >>= 1) t += __shfl_xor(t, off, VL);
  if (row < n && lane == 0) y[row] = t;
}

typedef double dv4 __attribute__((ext_vector_type(4)));
// ---------------- BSR 2x2, node-major, interleaved vectors -----------------------
// bptr[nv+1], bcol[nb] (node index J), bval[4*nb] = (a00, a01, a10, a11)
// x2/y2 interleaved: x2[2J+f]
template <int VL, bool NT>
__global__ __launch_bounds__(256) void bsr_k(int64_t nv, const int64_t* __restrict__ bptr,
                                             const int32_t* __restrict__ bcol,
                                             const dv4* __restrict__ bval,
                                             const double2* __restrict__ x2,
                                             double2* __restrict__ y2) {
  const int lane = threadIdx.x & (VL - 1);
  const int64_t node = ((int64_t)blockIdx.x * 256 + threadIdx.x) / VL;
  double s0 = 0.0, s1 = 0.0, t0 = 0.0, t1 = 0.0;
  if (node < nv) {
    const int64_t p0 = bptr[node], p1 = bptr[node + 1];
    int64_t k = p0 + lane;
    for (; k + VL < p1; k += 2 * VL) {
      int32_t c0, c1;
      dv4 v0, v1;
      if (NT) {
        c0 = __builtin_nontemporal_load(bcol + k);
        c1 = __builtin_nontemporal_load(bcol + k + VL);
        v0 = __builtin_nontemporal_load(bval + k);
        v1 = __builtin_nontemporal_load(bval + k + VL);
      } else {
        c0 = bcol[k]; c1 = bcol[k + VL];
        v0 = bval[k]; v1 = bval[k + VL];
      }
      const double2 a = x2[c0], b = x2[c1];
      s0 += v0.x * a.x; s0 += v0.y * a.y;
      s1 += v0.z * a.x; s1 += v0.w * a.y;
      t0 += v1.x * b.x; t0 += v1.y * b.y;
      t1 += v1.z * b.x; t1 += v1.w * b.y;
    }
    if (k < p1) {
      const int32_t c0 = bcol[k];
      const dv4 v0 = bval[k];
      const double2 a = x2[c0];
      s0 += v0.x * a.x; s0 += v0.y * a.y;
      s1 += v0.z * a.x; s1 += v0.w * a.y;
    }
  }
  s0 += t0;
  s1 += t1;
#pragma unroll
  for (int off = VL / 2; off > 0; off >>= 1) {
    s0 += __shfl_xor(s0, off, VL);
    s1 += __shfl_xor(s1, off, VL);
  }
  if (node < nv && lane == 0) y2[node] = make_double2(s0, s1);
}

// BSR with split value arrays (SoA: 4 planes) -- alternative coalescing
template <int VL>
__global__ __launch_bounds__(256) void bsr_soa_k(int64_t nv, const int64_t* __restrict__ bptr,
                                                 const int32_t* __restrict__ bcol,
                                                 const double2* __restrict__ vtop,
                                                 const double2* __restrict__ vbot,
                                                 const double2* __restrict__ x2,
                                                 double2* __restrict__ y2) {
  const int lane = threadIdx.x & (VL - 1);
  const int64_t node = ((int64_t)blockIdx.x * 256 + threadIdx.x) / VL;
  double s0 = 0.0, s1 = 0.0;
  if (node < nv) {
    const int64_t p0 = bptr[node], p1 = bptr[node + 1];
    for (int64_t k = p0 + lane; k < p1; k += VL) {
      const int32_t c = bcol[k];
      const double2 a = x2[c];
      const double2 u = vtop[k], w = vbot[k];
      s0 += u.x * a.x; s0 += u.y * a.y;
      s1 += w.x * a.x; s1 += w.y * a.y;
    }
  }
#pragma unroll
  for (int off = VL / 2; off > 0; off >>= 1) {
    s0 += __shfl_xor(s0, off, VL);
    s1 += __shfl_xor(s1, off, VL);
  }
  if (node < nv && lane == 0) y2[node] = make_double2(s0, s1);
}

// FETCH_SIZE calibration: stream-read n elements of width W bytes per lane
// (exactly n*W bytes), write one value per block
template <class T>
__global__ __launch_bounds__(256) void calib_read_k(int64_t n, const T* __restrict__ a,
                                                    double* __restrict__ out) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const T v = a[i];
#pragma unroll
    for (int w = 0; w < (int)(sizeof(T) / 4); ++w) s += (double)reinterpret_cast<const int*>(&v)[w];
  }
  if (s == 1234.5) out[blockIdx.x] = s;   // practically never: keeps the loads live
}

// WRITE_SIZE calibration: stream-write n elements of T (exactly n*sizeof(T)
// bytes); HALF: only the first 64 B of every 128 B line (partial-line writes,
// the pattern of a field-major epilogue store) -> n*sizeof(T)/2 bytes
template <class T, bool HALF>
__global__ __launch_bounds__(256) void calib_write_k(int64_t n, T* __restrict__ a) {
  constexpr int64_t per_half_line = 64 / sizeof(T);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if (HALF && ((i / per_half_line) & 1)) continue;
    a[i] = T{};
  }
}

// plain copy for the achievable-bandwidth reference
__global__ __launch_bounds__(256) void copy_k(int64_t n4, const double4* __restrict__ a,
                                              double4* __restrict__ b) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    b[i] = a[i];
}

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int calib(int reps) {
  // 2 GiB buffer, far above the 256 MiB MALL: every byte comes from HBM
  const int64_t bytes = (int64_t)2 << 30;
  char* a;
  double* out;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(a, 1, bytes));
  printf("calibration: each kernel reads exactly %ld bytes (compare FETCH_SIZE*1024)\n", (long)bytes);
#define CAL(T, name)                                                                       \
  {                                                                                        \
    const int64_t n = bytes / (int64_t)sizeof(T);                                          \
    float ms = timeit([&] { hipLaunchKernelGGL(calib_read_k<T>, dim3(256 * 16), dim3(256), 0, 0, n, (const T*)a, out); }, reps); \
    printf("calib %-8s (%2d B/lane): %.3f ms %.0f GB/s\n", name, (int)sizeof(T), ms, bytes / ms / 1e6); \
  }
  CAL(int, "int32") CAL(double, "f64") CAL(double2, "f64x2") CAL(dv4, "f64x4")
#define CALW(T, H, name)                                                                   \
  {                                                                                        \
    const int64_t n = bytes / (int64_t)sizeof(T);                                          \
    float ms = timeit([&] { hipLaunchKernelGGL((calib_write_k<T, H>), dim3(256 * 16), dim3(256), 0, 0, n, (T*)a); }, reps); \
    printf("calibw %-8s (%2d B/lane, %s): writes %ld bytes, %.3f ms\n", name, (int)sizeof(T),   \
           H ? "half lines" : "full lines", (long)(H ? bytes / 2 : bytes), ms);              \
  }
  CALW(double, false, "f64") CALW(double2, false, "f64x2") CALW(double, true, "f64") CALW(double2, true, "f64x2")
  CK(hipFree(a));
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "calib") return calib(argc > 2 ? atoi(argv[2]) : 3);
  const int n = argc > 1 ? atoi(argv[1]) : 256;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  int64_t N, nnz;
  mamg_gen_bidomain_size(3, n, &N, &nnz);
  std::vector<int64_t> ptr(N + 1);
  std::vector<int32_t> col(nnz);
  std::vector<double> val(nnz);
  mamg_gen_bidomain(3, n, 1e6, 2.0, 3.0, ptr.data(), col.data(), val.data());
  const int64_t nv = N / 2;
  printf("N=%ld nnz=%ld\n", (long)N, (long)nnz);
  // BSR 2x2 node-major
  std::vector<int64_t> bptr(nv + 1, 0);
  std::vector<int32_t> bcol;
  std::vector<double> bval;
  bcol.reserve(nnz / 4 + nv);
  bval.reserve(nnz + 4 * nv);
  struct E { int32_t J; int q; double v; };
  std::vector<E> ent;
  for (int64_t I = 0; I < nv; ++I) {
    ent.clear();
    for (int f = 0; f < 2; ++f) {       // rows I (f=0) and I+nv (f=1)
      const int64_t r = f * nv + I;
      for (int64_t k = ptr[r]; k < ptr[r + 1]; ++k)
        ent.push_back({(int32_t)(col[k] % nv), f * 2 + (int)(col[k] / nv), val[k]});
    }
    std::sort(ent.begin(), ent.end(), [](const E& a, const E& b) { return a.J < b.J; });
    for (size_t t = 0; t < ent.size();) {
      const int32_t J = ent[t].J;
      double b4[4] = {0, 0, 0, 0};
      for (; t < ent.size() && ent[t].J == J; ++t) b4[ent[t].q] = ent[t].v;
      bcol.push_back(J);
      for (int q = 0; q < 4; ++q) bval.push_back(b4[q]);
    }
    bptr[I + 1] = (int64_t)bcol.size();
  }
  const int64_t nb = (int64_t)bcol.size();
  printf("blocks=%ld (%.2f per node), explicit-zero fill %.3f%%\n", (long)nb, (double)nb / nv,
         100.0 * (4.0 * nb - nnz) / (4.0 * nb));
  std::vector<double> x(N);
  for (int64_t i = 0; i < N; ++i) x[i] = std::sin(0.001 * i) + 0.5;
  std::vector<double> x2(N);
  for (int64_t I = 0; I < nv; ++I) { x2[2 * I] = x[I]; x2[2 * I + 1] = x[nv + I]; }
  std::vector<double> vtop(2 * nb), vbot(2 * nb);
  for (int64_t k = 0; k < nb; ++k) {
    vtop[2 * k] = bval[4 * k]; vtop[2 * k + 1] = bval[4 * k + 1];
    vbot[2 * k] = bval[4 * k + 2]; vbot[2 * k + 1] = bval[4 * k + 3];
  }
  int64_t *dptr, *dbptr;
  int32_t *dcol, *dbcol;
  double *dval, *dbval, *dx, *dx2, *dy, *dy2, *dref, *dvt, *dvb;
  CK(hipMalloc(&dptr, (N + 1) * 8));
  CK(hipMalloc(&dcol, nnz * 4));
  CK(hipMalloc(&dval, nnz * 8));
  CK(hipMalloc(&dbptr, (nv + 1) * 8));
  CK(hipMalloc(&dbcol, nb * 4));
  CK(hipMalloc(&dbval, nb * 32));
  CK(hipMalloc(&dvt, nb * 16));
  CK(hipMalloc(&dvb, nb * 16));
  CK(hipMalloc(&dx, N * 8));
  CK(hipMalloc(&dx2, N * 8));
  CK(hipMalloc(&dy, N * 8));
  CK(hipMalloc(&dy2, N * 8));
  CK(hipMalloc(&dref, N * 8));
  CK(hipMemcpy(dptr, ptr.data(), (N + 1) * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dcol, col.data(), nnz * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dval, val.data(), nnz * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dbptr, bptr.data(), (nv + 1) * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dbcol, bcol.data(), nb * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dbval, bval.data(), nb * 32, hipMemcpyHostToDevice));
  CK(hipMemcpy(dvt, vtop.data(), nb * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(dvb, vbot.data(), nb * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(dx, x.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dx2, x2.data(), N * 8, hipMemcpyHostToDevice));

  const double csr_bytes = 12.0 * nnz + 8.0 * (N + 1) + 16.0 * N;
  const double bsr_bytes = 36.0 * nb + 8.0 * (nv + 1) + 16.0 * N;
  std::vector<double> ref(N), got(N), got2(N);
  // reference: CSR VL=16 U=2
  hipLaunchKernelGGL((csr_k<16, 2, false>), dim3((N * 16 + 255) / 256), dim3(256), 0, 0, N, dptr, dcol, dval, dx, dref);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(ref.data(), dref, N * 8, hipMemcpyDeviceToHost));
  auto check_csr = [&]() {
    CK(hipMemcpy(got.data(), dy, N * 8, hipMemcpyDeviceToHost));
    double m = 0, r = 0;
    for (int64_t i = 0; i < N; ++i) { m = std::max(m, std::fabs(got[i] - ref[i])); r = std::max(r, std::fabs(ref[i])); }
    return m / r;
  };
  auto check_bsr = [&]() {
    CK(hipMemcpy(got2.data(), dy2, N * 8, hipMemcpyDeviceToHost));
    double m = 0, r = 0;
    for (int64_t I = 0; I < nv; ++I)
      for (int f = 0; f < 2; ++f) {
        m = std::max(m, std::fabs(got2[2 * I + f] - ref[f * nv + I]));
        r = std::max(r, std::fabs(ref[f * nv + I]));
      }
    return m / r;
  };
#define RUN_CSR(VL, U, NT)                                                                 \
  {                                                                                        \
    float ms = timeit([&] { hipLaunchKernelGGL((csr_k<VL, U, NT>), dim3((N * VL + 255) / 256), dim3(256), 0, 0, N, dptr, dcol, dval, dx, dy); }, reps); \
    printf("csr VL=%2d U=%d nt=%d : %.3f ms  %.0f GB/s  err %.1e\n", VL, U, (int)NT, ms, csr_bytes / ms / 1e6, check_csr()); \
  }
  RUN_CSR(4, 2, false) RUN_CSR(4, 4, false) RUN_CSR(8, 1, false) RUN_CSR(8, 2, false) RUN_CSR(8, 4, false)
  RUN_CSR(16, 1, false) RUN_CSR(16, 2, false) RUN_CSR(32, 1, false) RUN_CSR(8, 2, true) RUN_CSR(16, 2, true)
#define RUN_BSR(VL, NT)                                                                    \
  {                                                                                        \
    float ms = timeit([&] { hipLaunchKernelGGL((bsr_k<VL, NT>), dim3((nv * VL + 255) / 256), dim3(256), 0, 0, nv, dbptr, dbcol, (const dv4*)dbval, (const double2*)dx2, (double2*)dy2); }, reps); \
    printf("bsr VL=%2d nt=%d    : %.3f ms  %.0f GB/s (bsr bytes) = %.0f GB/s csr-equiv  err %.1e\n", VL, (int)NT, ms, bsr_bytes / ms / 1e6, csr_bytes / ms / 1e6, check_bsr()); \
  }
  RUN_BSR(2, false) RUN_BSR(4, false) RUN_BSR(8, false) RUN_BSR(16, false) RUN_BSR(4, true) RUN_BSR(8, true)
#define RUN_SOA(VL)                                                                        \
  {                                                                                        \
    float ms = timeit([&] { hipLaunchKernelGGL((bsr_soa_k<VL>), dim3((nv * VL + 255) / 256), dim3(256), 0, 0, nv, dbptr, dbcol, (const double2*)dvt, (const double2*)dvb, (const double2*)dx2, (double2*)dy2); }, reps); \
    printf("bsr-soa VL=%2d      : %.3f ms  %.0f GB/s (bsr bytes)  err %.1e\n", VL, ms, bsr_bytes / ms / 1e6, check_bsr()); \
  }
  RUN_SOA(4) RUN_SOA(8) RUN_SOA(16)
  {
    const int64_t n4 = nnz / 4;
    float ms = timeit([&] { hipLaunchKernelGGL(copy_k, dim3(256 * 16), dim3(256), 0, 0, n4, (const double4*)dval, (double4*)dbval); }, reps);
    printf("copy %.2f GB: %.3f ms %.0f GB/s\n", 2.0 * n4 * 32 / 1e9, ms, 2.0 * n4 * 32 / ms / 1e6);
  }
  return 0;
}
