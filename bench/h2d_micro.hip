// h2d_micro.hip -- host-to-device upload of a pageable host array of A_0's
// size (upload_A0 took 338-415 ms for 12.3 GB): the
// runtime's pageable hipMemcpy, staged copies through pinned buffers filled
// by OpenMP threads (chunk size x buffers x threads), and page-locking the
// source in place (hipHostRegister) before a direct copy.
//
//   hipcc -O3 -fopenmp --offload-arch=gfx950 bench/h2d_micro.hip -o bench/h2d_micro
//   bench/h2d_micro [GB=12]
#include <hip/hip_runtime.h>
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void par_memcpy(void* d, const void* s, size_t b, int threads, size_t piece) {
  const long np = (long)((b + piece - 1) / piece);
#pragma omp parallel for schedule(static) num_threads(threads)
  for (long k = 0; k < np; ++k) {
    const size_t o = (size_t)k * piece;
    std::memcpy((char*)d + o, (const char*)s + o, std::min(piece, b - o));
  }
}

static double staged(void* dst, const char* src, size_t bytes, size_t ch, int nb, int threads, size_t piece) {
  std::vector<void*> buf(nb);
  for (auto& p : buf) CK(hipHostMalloc(&p, ch, hipHostMallocDefault));
  std::vector<hipEvent_t> ev(nb);
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipDeviceSynchronize());
  const double t0 = now();
  size_t k = 0;
  for (size_t off = 0; off < bytes; off += ch, ++k) {
    const int b = (int)(k % nb);
    const size_t len = std::min(ch, bytes - off);
    if (k >= (size_t)nb) CK(hipEventSynchronize(ev[b]));
    par_memcpy(buf[b], src + off, len, threads, piece);
    CK(hipMemcpyAsync((char*)dst + off, buf[b], len, hipMemcpyHostToDevice, s));
    CK(hipEventRecord(ev[b], s));
  }
  CK(hipStreamSynchronize(s));
  const double t = now() - t0;
  for (auto& p : buf) CK(hipHostFree(p));
  for (auto& e : ev) CK(hipEventDestroy(e));
  CK(hipStreamDestroy(s));
  return t;
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? std::atof(argv[1]) : 12.0;
  const size_t bytes = (size_t)(gb * 1e9) & ~(size_t)4095;
  char* src = (char*)std::aligned_alloc(4096, bytes);
#pragma omp parallel for schedule(static)
  for (long i = 0; i < (long)(bytes / 8); ++i) ((double*)src)[i] = (double)i;
  void* dst = nullptr;
  CK(hipMalloc(&dst, bytes));
  CK(hipMemcpy(dst, src, 1 << 20, hipMemcpyHostToDevice));   // warm the runtime
  std::printf("bytes %.2f GB, omp max threads %d\n", bytes / 1e9, omp_get_max_threads());
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipDeviceSynchronize());
    double t0 = now();
    CK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    double t = now() - t0;
    std::printf("pageable hipMemcpy: %.1f ms, %.1f GB/s\n", t * 1e3, bytes / t / 1e9);
  }
  // is the first copy's extra time the destination's first touch?  a fresh
  // destination copied into directly, and one written by a device memset first
  for (int rep = 0; rep < 2; ++rep) {
    for (int pre : {0, 1}) {
      void* d2 = nullptr;
      CK(hipMalloc(&d2, bytes));
      CK(hipDeviceSynchronize());
      double t0 = now();
      if (pre) CK(hipMemsetAsync(d2, 0, bytes, nullptr));
      CK(hipDeviceSynchronize());
      double t1 = now();
      CK(hipMemcpy(d2, src, bytes, hipMemcpyHostToDevice));
      double t2 = now();
      std::printf("fresh destination%s: memset %.1f ms + pageable copy %.1f ms (%.1f GB/s)\n",
                  pre ? " + device memset first" : "", (t1 - t0) * 1e3, (t2 - t1) * 1e3, bytes / (t2 - t1) / 1e9);
      CK(hipFree(d2));
    }
  }
  // fresh sources through the staged path, pinned buffers' allocation timed
  // too (what the library pays once per process)
  for (int rep = 0; rep < 2; ++rep) {
    char* s3 = (char*)std::aligned_alloc(4096, bytes);
#pragma omp parallel for schedule(static)
    for (long i = 0; i < (long)(bytes / 8); ++i) ((double*)s3)[i] = (double)i;
    const size_t ch = (size_t)64 << 20;
    double t0 = now();
    void* pb[4];
    for (auto& p : pb) CK(hipHostMalloc(&p, ch, hipHostMallocDefault));
    double t1 = now();
    for (auto& p : pb) CK(hipHostFree(p));
    const double t = staged(dst, s3, bytes, ch, 4, omp_get_max_threads(), (size_t)64 << 10);
    std::printf("fresh source, staged 64 MiB x 4, %d threads: %.1f ms (%.1f GB/s); 4 x 64 MiB hipHostMalloc %.1f ms\n",
                omp_get_max_threads(), t * 1e3, bytes / t / 1e9, (t1 - t0) * 1e3);
    std::free(s3);
  }
  // and a fresh source (the generator's just-written arrays) into the touched dst
  {
    char* s2 = (char*)std::aligned_alloc(4096, bytes);
#pragma omp parallel for schedule(static)
    for (long i = 0; i < (long)(bytes / 8); ++i) ((double*)s2)[i] = (double)i;
    CK(hipDeviceSynchronize());
    double t0 = now();
    CK(hipMemcpy(dst, s2, bytes, hipMemcpyHostToDevice));
    double t = now() - t0;
    std::printf("fresh source, touched destination: %.1f ms, %.1f GB/s\n", t * 1e3, bytes / t / 1e9);
    std::free(s2);
  }
  // a reference: device copy rate from a pinned buffer (PCIe ceiling)
  {
    void* pin = nullptr;
    const size_t pb = (size_t)1 << 30;
    CK(hipHostMalloc(&pin, pb, hipHostMallocDefault));
    std::memset(pin, 1, pb);
    CK(hipDeviceSynchronize());
    double t0 = now();
    for (int r = 0; r < 4; ++r) CK(hipMemcpy(dst, pin, pb, hipMemcpyHostToDevice));
    double t = now() - t0;
    std::printf("pinned hipMemcpy (4 x 1 GiB): %.1f GB/s\n", 4.0 * pb / t / 1e9);
    t0 = now();
    par_memcpy(pin, src, pb, omp_get_max_threads(), (size_t)64 << 10);
    t = now() - t0;
    std::printf("host memcpy pageable -> pinned 1 GiB, %d threads: %.1f GB/s\n", omp_get_max_threads(), pb / t / 1e9);
    CK(hipHostFree(pin));
  }
  const int tmax = omp_get_max_threads();
  for (size_t ch : {(size_t)16 << 20, (size_t)64 << 20, (size_t)256 << 20})
    for (int nb : {2, 4})
      for (int th : {tmax / 2, tmax}) {
        const double t = staged(dst, src, bytes, ch, nb, std::max(1, th), (size_t)64 << 10);
        std::printf("staged chunk %zu MiB x %d buffers, %d threads: %.1f ms, %.1f GB/s\n", ch >> 20, nb, th, t * 1e3,
                    bytes / t / 1e9);
      }
  {
    CK(hipDeviceSynchronize());
    double t0 = now();
    CK(hipHostRegister(src, bytes, hipHostRegisterDefault));
    double t1 = now();
    CK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    double t2 = now();
    CK(hipHostUnregister(src));
    double t3 = now();
    std::printf("hipHostRegister %.1f ms + copy %.1f ms (%.1f GB/s) + unregister %.1f ms = %.1f ms\n",
                (t1 - t0) * 1e3, (t2 - t1) * 1e3, bytes / (t2 - t1) / 1e9, (t3 - t2) * 1e3, (t3 - t0) * 1e3);
  }
  CK(hipFree(dst));
  std::free(src);
  return 0;
}
