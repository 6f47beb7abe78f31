// contig_alias.hip -- do physically contiguous allocations
// (hipExtMallocWithFlags(hipDeviceMallocContiguous)) share memory with other
// live allocations?  
//
// Interleaves allocations and frees of three kinds -- contiguous, plain
// hipMalloc, stream-ordered hipMallocAsync -- with sizes like the setup's
// (4 KiB .. 8 MiB), fills every new buffer with a pattern of its own (seed,
// index), and checks every live buffer's pattern every `check_every`
// operations and at the end.  A live buffer whose words changed was written
// through another allocation: the two share physical memory.
//
//   hipcc -O2 --offload-arch=gfx950 bench/contig_alias.hip -o build/contig_alias
//   build/contig_alias [ops=4000] [kinds=7] [check_every=50] [rng=1234567] [max_shift=11]
// kinds: bit 0 contiguous, bit 1 hipMalloc, bit 2 hipMallocAsync
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                             \
    }                                                                           \
  } while (0)

// a word names its buffer and index: a changed word names its writer
__device__ __host__ inline uint64_t pat(uint64_t seed, uint64_t i) { return (seed << 32) | (i & 0xffffffffull); }

__global__ void fill_kernel(uint64_t* p, int64_t n, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = pat(seed, (uint64_t)i);
}

// counts the words that differ and keeps the first differing index
__global__ void check_kernel(const uint64_t* p, int64_t n, uint64_t seed, unsigned long long* bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (p[i] != pat(seed, (uint64_t)i)) {
      atomicAdd(&bad[0], 1ull);
      atomicMin(&bad[1], (unsigned long long)i);
    }
}

struct Buf {
  uint64_t* p;
  int64_t n;
  uint64_t seed;
  int kind;  // 0 contiguous, 1 hipMalloc, 2 hipMallocAsync
  int born;
  int died;
};

static const char* kname(int k) { return k == 0 ? "contig" : k == 1 ? "malloc" : "async"; }

static uint64_t rng = 0x1234567ull;
static uint64_t rnd() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return rng;
}

int main(int argc, char** argv) {
  const int ops = argc > 1 ? std::atoi(argv[1]) : 4000;
  const int kinds = argc > 2 ? std::atoi(argv[2]) : 7;
  const int check_every = argc > 3 ? std::atoi(argv[3]) : 50;
  if (argc > 4) rng = std::strtoull(argv[4], nullptr, 10);
  const int max_shift = argc > 5 ? std::atoi(argv[5]) : 11;   // sizes 4 KiB << [0, max_shift]
  std::vector<Buf> all;   // every allocation made, by seed - 1
  unsigned long long* bad = nullptr;
  CK(hipMalloc(&bad, 2 * sizeof(unsigned long long)));
  std::vector<Buf> live;
  uint64_t seed = 1;
  long corrupt = 0, checks = 0;
  auto check_all = [&](int op) {
    bool first = true;
    for (const Buf& b : live) {
      const unsigned long long init[2] = {0ull, ~0ull};
      CK(hipMemcpy(bad, init, sizeof(init), hipMemcpyHostToDevice));
      check_kernel<<<1024, 256>>>(b.p, b.n, b.seed, bad);
      unsigned long long h[2];
      CK(hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost));
      ++checks;
      if (h[0]) {
        ++corrupt;
        if (first) {
          long long lb[3] = {0, 0, 0};
          for (const Buf& c : live) lb[c.kind] += c.n * 8;
          std::printf("op %d: live MiB contig %.1f malloc %.1f async %.1f\n", op, lb[0] / 1048576.0,
                      lb[1] / 1048576.0, lb[2] / 1048576.0);
          first = false;
        }
        std::printf("op %d: %s buffer %p (%lld bytes, made at op %d): %llu of %lld words changed, first at +%llu\n",
                    op, kname(b.kind), (void*)b.p, (long long)b.n * 8, b.born, h[0], (long long)b.n, h[1] * 8);
        uint64_t w = 0;
        CK(hipMemcpy(&w, b.p + h[1], 8, hipMemcpyDeviceToHost));
        const uint64_t ws = w >> 32, wi = w & 0xffffffffull;
        if (ws >= 1 && ws <= all.size()) {
          const Buf& o = all[ws - 1];
          std::printf("   the word there is word %llu of %s buffer %p (%lld bytes, made at op %d, %s at op %d)\n",
                      (unsigned long long)wi, kname(o.kind), (void*)o.p, (long long)o.n * 8, o.born,
                      o.died >= 0 ? "freed" : "live", o.died);
        } else {
          std::printf("   the word there is %016llx (no buffer's pattern)\n", (unsigned long long)w);
        }
        // refill, so that one event is reported once
        fill_kernel<<<1024, 256>>>(b.p, b.n, b.seed);
      }
    }
    CK(hipDeviceSynchronize());
  };
  int nalloc[3] = {0, 0, 0};
  for (int op = 0; op < ops; ++op) {
    const bool do_free = !live.empty() && (rnd() % 100) < (live.size() > 200 ? 60 : 40);
    if (do_free) {
      const size_t i = rnd() % live.size();
      Buf b = live[i];
      all[b.seed - 1].died = op;
      live[i] = live.back();
      live.pop_back();
      if (b.kind == 2) CK(hipFreeAsync(b.p, nullptr));
      else CK(hipFree(b.p));
    } else {
      int kind = (int)(rnd() % 3);
      while (!((kinds >> kind) & 1)) kind = (kind + 1) % 3;
      const int64_t bytes = (int64_t)4096 << (rnd() % (max_shift + 1));
      const int64_t n = bytes / 8 - (int64_t)(rnd() % 64);
      void* p = nullptr;
      if (kind == 0) CK(hipExtMallocWithFlags(&p, (size_t)n * 8, hipDeviceMallocContiguous));
      else if (kind == 1) CK(hipMalloc(&p, (size_t)n * 8));
      else CK(hipMallocAsync(&p, (size_t)n * 8, nullptr));
      ++nalloc[kind];
      Buf b{(uint64_t*)p, n, seed++, kind, op, -1};
      all.push_back(b);
      fill_kernel<<<1024, 256>>>(b.p, b.n, b.seed);
      live.push_back(b);
    }
    if ((op + 1) % check_every == 0) check_all(op);
  }
  check_all(ops);
  std::printf("ops %d (contig %d, malloc %d, async %d allocations), %zu live, %ld checks, %ld corrupted buffers\n",
              ops, nalloc[0], nalloc[1], nalloc[2], live.size(), checks, corrupt);
  for (const Buf& b : live) {
    if (b.kind == 2) CK(hipFreeAsync(b.p, nullptr));
    else CK(hipFree(b.p));
  }
  CK(hipDeviceSynchronize());
  CK(hipFree(bad));
  return corrupt ? 1 : 0;
}
