// device.hip -- CDNA4 (gfx950) apply path of the metric-AMG preconditioner.
//
// Replaces the HAZmath multigrid cycle behind `BB * r` (cbc.block operator,
// one cycle per call: `maxit: 1` /root/reference/src/amg_parameters.py:71,
// called by ConjGrad /root/reference/src/bidomain_3d.py:149-150) and the
// cbc.block PCG loop itself (mamg_pcg_device).
//
// Two device layouts of the same hierarchy (chosen at upload):
//  * CSR (general): every level as CSR {int64 rowptr, int32 col, fp64 val},
//    vectors in the caller's dof order.  Kernel: csr_kernel<VL,EPI,TAG>.
//  * BSR2 (nodal hierarchies, num_functions == 2, block-aligned smoother):
//    every level as 2x2 block CSR, node-major {int64 bptr, int32 node col,
//    4 fp64 per block}; internal vectors node-interleaved (x[2I+f]) so one
//    16-byte load gathers a node's pair; the level-0 block-Jacobi smoother is
//    kept as one 2x2 block per node and fused into the SpMV epilogue
//    (x' = x + W_I (b_I - (A x)_I)).  The caller's r / z stay field-major
//    ([u1; u2], src/bidomain_3d.py:124,138): level-0 kernels read/write them
//    with a field stride.  Index bytes drop from 4 per value to 1, gathers
//    halve; measured 2.2x faster level-0 SpMV than CSR (bench/spmv_micro.hip).
//
// Kernels (all HBM-bound, ~0.17 flop/B): VL lanes per
// row (node), VL a power of two chosen from the mean row length; lanes stride
// the row's contiguous block window (coalesced 32-byte block loads), x
// gathered through L2/MALL, partial sums reduced with wavefront shuffles, and
// a fused epilogue.  One apply = a fixed schedule of launches captured into a
// hipGraph; each launch carries its algorithmic bytes (roofline from the
// hierarchy, not from counters).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <map>
#include <numeric>
#include <vector>

#include "device.h"
#include "dmem.h"
#include "opts.h"
#include "rowstage.h"

#include <pthread.h>

namespace mamg {

// hipGraphInstantiate on a thread whose stack fits the graph.  The runtime
// walks a captured graph recursively at instantiation, one 64-byte frame per
// node of its longest dependency chain (a stream capture is one chain): the
// 8 virtual ranks' lockstep apply of the reference preset at nrefs=5 overflowed
// the 8 MiB main-thread stack after 130,903 frames and crashed the process
// (SIGSEGV on the guard page inside hipGraphInstantiate; diagnosis-build tracer,
// profiles/r06_graph_segv.txt).  Graphs of up to
// GRAPH_INSTANTIATE_INLINE nodes instantiate on the caller's thread (at most
// 1 MiB of its stack); larger ones on a helper thread with 256 B of stack per
// node (4x the measured frame) + 16 MiB, reserved, touched only as deep as the
// walk goes.
constexpr size_t GRAPH_INSTANTIATE_INLINE = 16384;

// Held across every stream capture of the library and every setup (capi.cpp
// TmpTrim): the HIP runtime invalidates a capture when another host thread
// issues legacy null-stream work meanwhile (the setups' synchronous copies),
// and refuses that work ("would make the legacy stream depend on a capturing
// blocking stream"), thread-local capture mode notwithstanding (two threads
// setting up and applying at once, tests/test_gpu_setup.py).  Setups of one
// process therefore run one at a time.
std::recursive_mutex& capture_mutex() {
  static std::recursive_mutex m;
  return m;
}
hipError_t graph_instantiate(hipGraphExec_t* ex, hipGraph_t g) {
  size_t nodes = 0;
  hipError_t e = hipGraphGetNodes(g, nullptr, &nodes);
  if (e != hipSuccess) return e;
  if (nodes <= GRAPH_INSTANTIATE_INLINE) return hipGraphInstantiate(ex, g, nullptr, nullptr, 0);
  struct Job {
    hipGraphExec_t* ex;
    hipGraph_t g;
    int dev;
    hipError_t e;
  } job{ex, g, 0, hipSuccess};
  if ((e = hipGetDevice(&job.dev)) != hipSuccess) return e;
  pthread_attr_t a;
  if (pthread_attr_init(&a) != 0) return hipErrorOutOfMemory;
  const size_t stack = ((nodes * 256 + ((size_t)16 << 20)) + 4095) & ~(size_t)4095;
  pthread_t t;
  int rc = pthread_attr_setstacksize(&a, stack);
  if (rc == 0)
    rc = pthread_create(&t, &a, [](void* p) -> void* {
      Job* j = static_cast<Job*>(p);
      j->e = hipSetDevice(j->dev);
      if (j->e == hipSuccess) j->e = hipGraphInstantiate(j->ex, j->g, nullptr, nullptr, 0);
      return nullptr;
    }, &job);
  pthread_attr_destroy(&a);
  if (rc != 0) return hipErrorOutOfMemory;
  pthread_join(t, nullptr);
  return job.e;
}

namespace {

#define HIPCHK(expr)                                                                 \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess) {                                                          \
      *err = std::string(#expr) + ": " + hipGetErrorString(e_);                      \
      return MAMG_ERR_HIP;                                                           \
    }                                                                                \
  } while (0)

// epilogues: y = s | y = y0 + s | r = b - s | x' = x + w (b - s) (point) |
// x' = x + W_I (b_I - s_I) (2x2 block, BSR only) |
// z = x1_I + W_I r1_I + s_I with s = K e, K = P - W (A P) (BSR only: the
// prolongation fused with the first post sweep through one operator)
enum Epi { EPI_Y = 0, EPI_YADD = 1, EPI_RESID = 2, EPI_JACOBI = 3, EPI_BJAC = 4, EPI_KPOST = 5, EPI_YBD = 6 };
// EPI_YBD (bsr2_kernel only): out = A x as EPI_Y, and the next level's first
// sweep from x = 0 in the same pass, y <- W out (the restriction b_c = R r
// writing x1_c = W_c b_c: one launch and one b_c read fewer per coarse level;
// the same two products as bd2_kernel, so the same bits)

typedef double dv4 __attribute__((ext_vector_type(4)));
typedef double dv2 __attribute__((ext_vector_type(2)));

constexpr int SCALE_BLOCKS = 256;   // partial-sum blocks of the coarse-scaling dots

// ---------------------------------------------------------------------------
// CSR kernels (general layout)
// ---------------------------------------------------------------------------
template <int VL, int EPI, int TAG>
__global__ __launch_bounds__(256) void csr_kernel(
    int64_t n, const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
    const double* __restrict__ val, const double* __restrict__ x,
    const double* y, const double* __restrict__ b, const double* __restrict__ w,
    double* out) {
  const int lane = threadIdx.x & (VL - 1);
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / VL;
  double s0 = 0.0, s1 = 0.0;
  if (row < n) {
    const int64_t p0 = ptr[row], p1 = ptr[row + 1];
    int64_t k = p0 + lane;
    for (; k + VL < p1; k += 2 * VL) {
      const int32_t c0 = col[k], c1 = col[k + VL];
      const double v0 = val[k], v1 = val[k + VL];
      s0 += v0 * x[c0];
      s1 += v1 * x[c1];
    }
    if (k < p1) s0 += val[k] * x[col[k]];
  }
  double s = s0 + s1;
#pragma unroll
  for (int off = VL / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, VL);
  if (row < n && lane == 0) {
    if (EPI == EPI_Y) out[row] = s;
    else if (EPI == EPI_YADD) out[row] = y[row] + s;
    else if (EPI == EPI_RESID) out[row] = b[row] - s;
    else out[row] = y[row] + w[row] * (b[row] - s);
  }
}

// ---------------------------------------------------------------------------
// BSR2 kernels (nodal layout).  Vector element (node I, field f):
//   node-major:  v[2I + f]          (stride argument 0)
//   field-major: v[f * stride + I]  (the caller's [u1; u2] order)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double vget(const double* v, int64_t stride, int64_t I, int f) {
  return stride ? v[f * stride + I] : v[2 * I + f];
}
__device__ __forceinline__ void vset(double* v, int64_t stride, int64_t I, int f, double a) {
  if (stride) v[f * stride + I] = a; else v[2 * I + f] = a;
}

// XCD-aware row order: the dispatcher hands workgroup b to XCD b % 8, so
// consecutive workgroups (neighbouring rows, which gather the same x entries)
// would land in 8 different L2s.  Renumber so that every XCD walks one
// contiguous range of rows (bijective for any grid size).
// W_I b_I with the contraction spelled out (fma of the first product onto
// the second), so that bd2_kernel and the restriction's EPI_YBD epilogue,
// compiled in different contexts, produce the same bits
__device__ __forceinline__ double2 wmul(const dv4& w, double b0, double b1) {
  return double2{__builtin_fma(w.x, b0, w.y * b1), __builtin_fma(w.z, b0, w.w * b1)};
}

__device__ __forceinline__ int64_t row_block_of(uint32_t b, uint32_t G, int remap) {
  if (!remap) return b;
  const uint32_t q = G >> 3, r = G & 7, x = b & 7;
  return (int64_t)(x * q + (x < r ? x : r) + (b >> 3));
}
__device__ __forceinline__ int64_t row_block(int remap) { return row_block_of(blockIdx.x, gridDim.x, remap); }

// block k of a BSR2 value array: 4 doubles (0,0) (0,1) (1,0) (1,1) per block,
// or in the symmetric-block format (SYM) two aligned streams: the diagonal
// pairs {(0,0), (1,1)} (16 B per block) then the off-diagonals (0,1) = (1,0)
// (8 B per block) starting at v + 2 nb
// NT: non-temporal (streaming) loads, so the matrix stream does not evict
// the gathered vector from L2
template <bool NT, class T>
__device__ __forceinline__ T ldg(const T* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}

template <bool SYM, bool NT = false>
__device__ __forceinline__ dv4 blk(const double* __restrict__ v, const double* __restrict__ off,
                                   int64_t k) {
  if (SYM) {
    const dv2 d = ldg<NT>(reinterpret_cast<const dv2*>(v) + k);
    const double b = ldg<NT>(off + k);
    return dv4{d.x, b, b, d.y};
  }
  return ldg<NT>(reinterpret_cast<const dv4*>(v) + k);
}

// x(node c) as a pair: node-interleaved (one 16-byte load) or field-major
template <bool XFM>
__device__ __forceinline__ double2 xget(const double* x, int64_t xs, int32_t c) {
  if (XFM) return double2{x[c], x[xs + c]};
  return reinterpret_cast<const double2*>(x)[c];
}

template <int VL, int EPI, bool XFM, bool SYM, int TAG, bool NT = false>
__global__ __launch_bounds__(256) void bsr2_kernel(
    int64_t nr, const int64_t* __restrict__ bptr, const int32_t* __restrict__ bcol,
    const double* __restrict__ bval, const double* __restrict__ x, int64_t xs,
    const double* y, const double* __restrict__ b, int64_t bs,
    const dv4* __restrict__ W, double* out, int64_t os, int remap, const int32_t* __restrict__ sched,
    int64_t rb0 = 0) {
  const int lane = threadIdx.x & (VL - 1);
  // rb0: first workgroup of a row-range launch (rows from 256 rb0 / VL)
  const int64_t node = ((sched ? (int64_t)sched[blockIdx.x] : rb0 + row_block(remap)) * 256 + threadIdx.x) / VL;
  const double* offd = SYM ? bval + 2 * bptr[nr] : nullptr;
  double s0 = 0.0, s1 = 0.0, t0 = 0.0, t1 = 0.0;
  // EPI_YBD's W block loaded with the row, not after the reduction (a
  // dependent load at the end of every row measured +36 us on level 0's R)
  const dv4 wy = (EPI == EPI_YBD && node < nr && lane == 0) ? W[node] : dv4{0.0, 0.0, 0.0, 0.0};
  if (node < nr) {
    // chunks of 2 VL blocks, branch-free: every lane issues both loads of a
    // chunk at once (index clamped into the row, contribution selected away),
    // so a row costs one load -> gather chain per chunk instead of a loop
    // chain followed by a divergent tail chain
    const int64_t p0 = bptr[node], p1 = bptr[node + 1];
    for (int64_t base = p0; base < p1; base += 2 * VL) {
      const int64_t ka = base + lane, kb = ka + VL;
      const bool ha = ka < p1, hb = kb < p1;
      const int64_t la = ha ? ka : p1 - 1, lb = hb ? kb : p1 - 1;
      const int32_t c0 = ldg<NT>(bcol + la), c1 = ldg<NT>(bcol + lb);
      const dv4 v0 = blk<SYM, NT>(bval, offd, la), v1 = blk<SYM, NT>(bval, offd, lb);
      const double2 a = xget<XFM>(x, xs, c0), e = xget<XFM>(x, xs, c1);
      s0 += ha ? v0.x * a.x + v0.y * a.y : 0.0;
      s1 += ha ? v0.z * a.x + v0.w * a.y : 0.0;
      t0 += hb ? v1.x * e.x + v1.y * e.y : 0.0;
      t1 += hb ? v1.z * e.x + v1.w * e.y : 0.0;
    }
  }
  s0 += t0;
  s1 += t1;
#pragma unroll
  for (int off = VL / 2; off > 0; off >>= 1) {
    s0 += __shfl_xor(s0, off, VL);
    s1 += __shfl_xor(s1, off, VL);
  }
  if (node < nr && lane == 0) {
    double o0, o1;
    if (EPI == EPI_Y) {
      o0 = s0; o1 = s1;
    } else if (EPI == EPI_YBD) {
      o0 = s0; o1 = s1;
      const double2 wb = wmul(wy, o0, o1);
      double* x1 = const_cast<double*>(y);
      x1[2 * node] = wb.x;
      x1[2 * node + 1] = wb.y;
    } else if (EPI == EPI_YADD) {
      o0 = y[2 * node] + s0; o1 = y[2 * node + 1] + s1;
    } else if (EPI == EPI_RESID) {
      o0 = vget(b, bs, node, 0) - s0; o1 = vget(b, bs, node, 1) - s1;
    } else if (EPI == EPI_KPOST) {
      const double r0 = vget(b, bs, node, 0), r1 = vget(b, bs, node, 1);
      const dv4 w = W[node];
      o0 = y[2 * node] + (w.x * r0 + w.y * r1) + s0;
      o1 = y[2 * node + 1] + (w.z * r0 + w.w * r1) + s1;
    } else {  // EPI_BJAC
      const double r0 = vget(b, bs, node, 0) - s0, r1 = vget(b, bs, node, 1) - s1;
      const dv4 w = W[node];
      o0 = y[2 * node] + (w.x * r0 + w.y * r1);
      o1 = y[2 * node + 1] + (w.z * r0 + w.w * r1);
    }
    vset(out, os, node, 0, o0);
    vset(out, os, node, 1, o1);
  }
}

// prolongation fused into the first post-smoothing sweep (post_fusion):
//   out(I) = x1(I) + (P e)(I) + W_I (r1(I) - (AP e)(I))
// which equals x2 + W (b - A x2) for x2 = x1 + P e, since r1 = b - A x1 and
// A x2 = A x1 + (AP) e.  Row I of the merged matrix holds P's blocks in
// [mptr[2I], mptr[2I+1]) then AP's in [mptr[2I+1], mptr[2I+2]): one contiguous
// window per node, both sums gathered from the same coarse vector e.
// The row's epilogue operands (x1, r1, W) are loaded by lane 0 before the
// block loop, so their latency overlaps the loop instead of following it.
template <int VL, bool NT, int TAG>
__global__ __launch_bounds__(256) void bsr2_post_kernel(
    int64_t nr, const int64_t* __restrict__ mptr, const int32_t* __restrict__ bcol,
    const double* __restrict__ bval, const double* __restrict__ e, const double* __restrict__ x1,
    const double* __restrict__ r1, const dv4* __restrict__ W, double* out, int64_t os, int remap) {
  const int lane = threadIdx.x & (VL - 1);
  const int64_t node = (row_block(remap) * 256 + threadIdx.x) / VL;
  const double2* e2 = reinterpret_cast<const double2*>(e);
  double p0 = 0.0, p1 = 0.0, q0 = 0.0, q1 = 0.0;
  dv4 w = {0.0, 0.0, 0.0, 0.0};
  double2 xx = {0.0, 0.0}, rr = {0.0, 0.0};
  if (node < nr && lane == 0) {
    w = W[node];
    xx = reinterpret_cast<const double2*>(x1)[node];
    rr = reinterpret_cast<const double2*>(r1)[node];
  }
  if (node < nr) {   // branch-free chunks of 2 VL blocks (see bsr2_kernel)
    const int64_t k0 = mptr[2 * node], km = mptr[2 * node + 1], k1 = mptr[2 * node + 2];
    for (int64_t base = k0; base < k1; base += 2 * VL) {
      const int64_t ka = base + lane, kb = ka + VL;
      const bool ha = ka < k1, hb = kb < k1;
      const int64_t la = ha ? ka : k1 - 1, lb = hb ? kb : k1 - 1;
      const int32_t c0 = ldg<NT>(bcol + la), c1 = ldg<NT>(bcol + lb);
      const dv4 v0 = blk<false, NT>(bval, nullptr, la), v1 = blk<false, NT>(bval, nullptr, lb);
      const double2 a = e2[c0], b = e2[c1];
      const double u0 = ha ? v0.x * a.x + v0.y * a.y : 0.0, u1 = ha ? v0.z * a.x + v0.w * a.y : 0.0;
      const double w0 = hb ? v1.x * b.x + v1.y * b.y : 0.0, w1 = hb ? v1.z * b.x + v1.w * b.y : 0.0;
      const bool pa = ka < km, pb = kb < km;
      p0 += pa ? u0 : 0.0; p1 += pa ? u1 : 0.0; q0 += pa ? 0.0 : u0; q1 += pa ? 0.0 : u1;
      p0 += pb ? w0 : 0.0; p1 += pb ? w1 : 0.0; q0 += pb ? 0.0 : w0; q1 += pb ? 0.0 : w1;
    }
  }
#pragma unroll
  for (int off = VL / 2; off > 0; off >>= 1) {
    p0 += __shfl_xor(p0, off, VL);
    p1 += __shfl_xor(p1, off, VL);
    q0 += __shfl_xor(q0, off, VL);
    q1 += __shfl_xor(q1, off, VL);
  }
  if (node < nr && lane == 0) {
    const double d0 = rr.x - q0, d1 = rr.y - q1;
    vset(out, os, node, 0, xx.x + p0 + (w.x * d0 + w.y * d1));
    vset(out, os, node, 1, xx.y + p1 + (w.z * d0 + w.w * d1));
  }
}

// ---------------------------------------------------------------------------
// Sliced-ELL variant of BSR2 (SELL-64) for the large short-row level-0
// operators (A_0: ~15 blocks per node, [P | AP]: ~13).  One lane per node;
// slice s = nodes [64 s, 64 s + 64) = one wavefront; block j of the slice's
// lane l sits at soff[s] + 64 j + l, so every load of the row loop is one
// fully coalesced 64-lane access (2 KB of blocks, 256 B of columns) with no
// cross-lane reduction.  meta[I] = row length | (P-part length << 16) (the
// split is used by the fused post kernel only).  Each lane loops only to its
// own length; padding is storage, never loaded.  Sums run in block order.
// ---------------------------------------------------------------------------
constexpr int SELL_C = 64;
constexpr int SELL_U = 4;     // blocks in flight per lane

// SPL: general blocks stored as two 16-byte streams per slot, the (0,0)(0,1)
// pairs at bval[2k] and the (1,0)(1,1) pairs at bval[2 nbs + 2k]: each load
// instruction reads 1 KB contiguous instead of 16 B of every 32 B over 2 KB
__device__ __forceinline__ dv4 blk_split(const double* __restrict__ v, int64_t nbs, int64_t k) {
  const dv2 a = reinterpret_cast<const dv2*>(v)[k];
  const dv2 b = reinterpret_cast<const dv2*>(v + 2 * nbs)[k];
  return dv4{a.x, a.y, b.x, b.y};
}
// split inside each 64-slot SELL slot row: the row's 64 (0,0)(0,1) pairs
// (1 KB) then its 64 (1,0)(1,1) pairs, so a 16-byte-per-lane load of
// consecutive slots reads one contiguous piece and the slot row stays 2 KB
__device__ __forceinline__ dv4 blk_split_local(const double* __restrict__ v, int64_t k) {
  const int64_t r = k & ~(int64_t)63, i = k & 63;
  const dv2 a = reinterpret_cast<const dv2*>(v + 4 * r)[i];
  const dv2 b = reinterpret_cast<const dv2*>(v + 4 * r + 128)[i];
  return dv4{a.x, a.y, b.x, b.y};
}
template <int SPL>
__device__ __forceinline__ dv4 blk_any(const double* __restrict__ v, int64_t nbs, int64_t k) {
  if (SPL == 1) return blk_split(v, nbs, k);
  if (SPL == 2) return blk_split_local(v, k);
  return reinterpret_cast<const dv4*>(v)[k];
}

template <int EPI, bool XFM, bool SYM, int U, bool SPL, int TAG>
__global__ __launch_bounds__(256) void sell2_kernel(
    int64_t nr, const int64_t* __restrict__ soff, const int32_t* __restrict__ meta,
    const int32_t* __restrict__ bcol, const double* __restrict__ bval, int64_t nbs,
    const double* __restrict__ x, int64_t xs, const double* y, const double* __restrict__ b,
    int64_t bs, const dv4* __restrict__ W, double* out, int64_t os, int remap,
    const int32_t* __restrict__ sched, int lsort) {
  const int64_t slot = (sched ? (int64_t)sched[blockIdx.x] : row_block(remap)) * 256 + threadIdx.x;
  if (slot >= nr) return;
  const double* offd = SYM ? bval + 2 * nbs : nullptr;
  const int m = meta[slot];
  const int len = m & 0xffff;
  int64_t k = soff[slot / SELL_C] + (slot & (SELL_C - 1));
  // the row this slot holds (DBsr::lsort: rows sorted by length in the slice)
  const int64_t node = lsort ? (slot & ~(int64_t)(SELL_C - 1)) | ((m >> 16) & (SELL_C - 1)) : slot;
  double s0 = 0.0, s1 = 0.0;
  // chunks of U blocks, branch-free (slot clamped into the row, contribution
  // selected away): one load -> gather chain per chunk
  for (int j = 0; j < len; j += U) {
    int32_t c[U];
    dv4 v[U];
    double2 a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t kk = k + (int64_t)SELL_C * (j + u < len ? j + u : len - 1);
      c[u] = bcol[kk];
      v[u] = SPL ? blk_split(bval, nbs, kk) : blk<SYM>(bval, offd, kk);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = xget<XFM>(x, xs, c[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = j + u < len;
      s0 += ok ? v[u].x * a[u].x + v[u].y * a[u].y : 0.0;
      s1 += ok ? v[u].z * a[u].x + v[u].w * a[u].y : 0.0;
    }
  }
  // epilogue operands after the loop (measured: loading them first is slower)
  double2 bb = {0.0, 0.0}, yy = {0.0, 0.0};
  dv4 w = {0.0, 0.0, 0.0, 0.0};
  if (EPI == EPI_RESID || EPI == EPI_BJAC || EPI == EPI_KPOST)
    bb = double2{vget(b, bs, node, 0), vget(b, bs, node, 1)};
  if (EPI == EPI_YADD || EPI == EPI_BJAC || EPI == EPI_KPOST) yy = reinterpret_cast<const double2*>(y)[node];
  if (EPI == EPI_BJAC || EPI == EPI_KPOST) w = W[node];
  double o0, o1;
  if (EPI == EPI_Y) {
    o0 = s0; o1 = s1;
  } else if (EPI == EPI_YADD) {
    o0 = yy.x + s0; o1 = yy.y + s1;
  } else if (EPI == EPI_RESID) {
    o0 = bb.x - s0; o1 = bb.y - s1;
  } else if (EPI == EPI_KPOST) {
    o0 = yy.x + (w.x * bb.x + w.y * bb.y) + s0;
    o1 = yy.y + (w.z * bb.x + w.w * bb.y) + s1;
  } else {  // EPI_BJAC
    const double r0 = bb.x - s0, r1 = bb.y - s1;
    o0 = yy.x + (w.x * r0 + w.y * r1);
    o1 = yy.y + (w.z * r0 + w.w * r1);
  }
  vset(out, os, node, 0, o0);
  vset(out, os, node, 1, o1);
}

// SELL-64 operator with LPR lanes per node row (multi-lane SELL).  A wavefront
// takes 64 / LPR rows of a 64-row slice; part q < LPR - 1 of a row takes its
// blocks [q U, (q + 1) U), the last part the rest in chunks of U, so a row of
// up to LPR U blocks is one load -> gather round trip per lane instead of a
// chain of chunks on one lane.  For a fixed chunk slot the lanes of one part
// read 64 / LPR consecutive slots.  The parts' sums meet by a __shfl_xor
// butterfly (addition commutes: every lane of a row ends with the same bits),
// then part f < 2 writes field f; its epilogue operands are loaded before
// the block loop.  Used for the level-0 fused post operator
// z = x1 + W r1 + K e (EPI_KPOST, LPR 2, U 5: K 1.69 -> 1.54 ms on one
// upload) and the SELL-stored coarse operators.
template <int LPR, int U, int EPI, bool XFM, bool SYM, int SPL, int TAG, int PROBE = 0, bool C16 = false>
__global__ __launch_bounds__(256) void msell_kernel(
    int64_t nr, const int64_t* __restrict__ soff, const int32_t* __restrict__ meta,
    const int32_t* __restrict__ bcol, const double* __restrict__ bval, int64_t nbs,
    const double* __restrict__ x, int64_t xs, const double* y, const double* __restrict__ b, int64_t bs,
    const dv4* __restrict__ W, double* out, int64_t os, int remap, int lsort, int64_t rb0,
    const uint16_t* __restrict__ c16, const int32_t* __restrict__ cbase) {
  constexpr int RW = 64 / LPR;                          // rows per wavefront
  const int lane = threadIdx.x & 63, q = lane / RW;
  // rb0: first workgroup of a row-range launch (rows [256 rb0 / LPR, ...))
  const int64_t slot = (rb0 + row_block(remap)) * (4 * RW) + (threadIdx.x >> 6) * RW + (lane & (RW - 1));
  const bool live = slot < nr;
  const int64_t ns = live ? slot : nr - 1;            // dead lanes mirror the last slot, write nothing
  const int m = meta[ns];
  const int len = m & 0xffff;
  const int64_t k = soff[ns / SELL_C] + (ns & (SELL_C - 1));
  // the row this slot holds (DBsr::lsort: rows sorted by length in the slice)
  const int64_t node = lsort ? (ns & ~(int64_t)(SELL_C - 1)) | ((m >> 16) & (SELL_C - 1)) : ns;
  const int64_t nd = node;
  const double* offd = SYM ? bval + 2 * nbs : nullptr;
  const int f = q & 1;
  const bool wr = q < 2;
  constexpr bool NB = EPI == EPI_RESID || EPI == EPI_BJAC || EPI == EPI_KPOST;
  constexpr bool NY = EPI == EPI_YADD || EPI == EPI_BJAC || EPI == EPI_KPOST;
  constexpr bool NW = EPI == EPI_BJAC || EPI == EPI_KPOST;
  const double yf = NY && wr ? y[2 * nd + f] : 0.0;
  const dv2 wf = NW && wr ? reinterpret_cast<const dv2*>(W + nd)[f] : dv2{0.0, 0.0};
  const double2 bb = NB && wr ? double2{vget(b, bs, nd, 0), vget(b, bs, nd, 1)} : double2{0.0, 0.0};
  double s0 = 0.0, s1 = 0.0;
  const int j0 = q * U, j1 = q == LPR - 1 ? len : (len < j0 + U ? len : j0 + U);
  const int32_t cb0 = C16 ? cbase[ns / SELL_C] : 0;
  for (int j = j0; j < j1; j += U) {
    int32_t c[U];
    dv4 v[U];
    double2 a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t kk = k + (int64_t)SELL_C * (j + u < j1 ? j + u : j1 - 1);
      if constexpr (C16) c[u] = cb0 + (int32_t)c16[kk];
      else c[u] = PROBE == 2 ? __builtin_nontemporal_load(bcol + kk) : bcol[kk];
      v[u] = SPL ? blk_any<SPL>(bval, nbs, kk) : blk<SYM, (PROBE >= 2)>(bval, offd, kk);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)   // PROBE 1 (A/B only, wrong results): no gather, the column as the value
      a[u] = PROBE == 1 ? double2{(double)c[u], 1.0} : xget<XFM>(x, xs, c[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = j + u < j1;
      s0 += ok ? v[u].x * a[u].x + v[u].y * a[u].y : 0.0;
      s1 += ok ? v[u].z * a[u].x + v[u].w * a[u].y : 0.0;
    }
  }
#pragma unroll
  for (int off = RW; off < 64; off <<= 1) {
    s0 += __shfl_xor(s0, off);
    s1 += __shfl_xor(s1, off);
  }
  if (!live || !wr) return;
  const double sf = f ? s1 : s0;
  double o;
  if (EPI == EPI_Y) {
    o = sf;
  } else if (EPI == EPI_YADD) {
    o = yf + sf;
  } else if (EPI == EPI_RESID) {
    o = (f ? bb.y : bb.x) - sf;
  } else if (EPI == EPI_KPOST) {
    o = yf + (wf.x * bb.x + wf.y * bb.y) + sf;
  } else {  // EPI_BJAC
    const double r0 = bb.x - s0, r1 = bb.y - s1;
    o = yf + (wf.x * r0 + wf.y * r1);
  }
  vset(out, os, node, f, o);
}

// ---------------------------------------------------------------------------
// Half-symmetric ELL-64 for a symmetric A0 (A_JI = A_IJ^T bitwise and every
// block symmetric, so A_JI = A_IJ): only the upper part J >= I is streamed
// (28 B per block with its column); a lower entry J < I is a 4-byte slot
// pointer to its mirror (J, I) in the upper part, whose row J the sweep
// streamed a few MB earlier, so the re-read is served by L2 / the 256 MB
// MALL instead of HBM.  The ELL slot p of upper block j of row J is
// (J / 64) 64 hwu + 64 j + J % 64, so J = 64 (p / (64 hwu)) + p % 64 needs no
// column.  For a translation-invariant stencil the 64 lanes' mirror slots
// are 64 consecutive rows of one slot: the gathers are coalesced too.
// Sums run lower part then upper part, each in column order: the full row's
// block order, so the result is bitwise that of sell2_kernel.
// ---------------------------------------------------------------------------
// streams of hsell2_kernel touched once: row meta, lower slot pointers and
// upper columns (level 1), and the b loads / output stores (level 2) are
// non-temporal, so that they do not displace from L2 the upper values the
// mirrors re-read.  Round 4 A/B at nrefs=6 (profiles/r04_hsell_nt.txt):
// residual L2-miss bytes 6.30 -> 6.03 (1) -> 5.87 GB (2) per launch,
// 1.077 -> 1.070 ms.  Build switch (0 = plain loads), default 2.
#ifndef MAMG_HSELL_NT
#define MAMG_HSELL_NT 2
#endif
template <class T>
__device__ __forceinline__ T ld_once(const T* p) {
  if constexpr (MAMG_HSELL_NT != 0) return __builtin_nontemporal_load(p);
  else return *p;
}

template <int EPI, bool XFM, int U, bool GH, int TAG>
__global__ __launch_bounds__(256) void hsell2_kernel(
    int64_t row0, int64_t nr, const int32_t* __restrict__ meta, const int32_t* __restrict__ ucol,
    const double* __restrict__ uval, int64_t nbs, int hwu, const int32_t* __restrict__ lptr, int hwl,
    const int64_t* __restrict__ gsoff, const int32_t* __restrict__ gcol, const double* __restrict__ gval,
    int64_t ngs, const double* __restrict__ x, int64_t xs, const double* y, const double* __restrict__ b,
    int64_t bs, const dv4* __restrict__ W, double* out, int64_t os, int remap,
    const int32_t* __restrict__ sched) {
  const int64_t blk0 = sched ? (int64_t)sched[blockIdx.x] : row_block(remap);
  const int64_t node = row0 + blk0 * 256 + threadIdx.x;   // rows [row0, nr)
  if (node >= nr) return;
  const double* offd = uval + 2 * nbs;
  const int m = ld_once(meta + node);
  const int ulen = m & 0xff, llen = (m >> 8) & 0xff;
  const uint32_t urow = 64u * (uint32_t)hwu;
  double s0 = 0.0, s1 = 0.0;
  {
    const int64_t k = (node >> 6) * (int64_t)(64 * hwl) + (node & 63);
    for (int j = 0; j < llen; j += U) {
      uint32_t p[U];
      dv4 v[U];
      double2 a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) p[u] = (uint32_t)ld_once(lptr + k + (int64_t)SELL_C * (j + u < llen ? j + u : llen - 1));
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int32_t c = (int32_t)((p[u] / urow) * 64u + (p[u] & 63u));
        v[u] = blk<true>(uval, offd, p[u]);
        a[u] = xget<XFM>(x, xs, c);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = j + u < llen;
        s0 += ok ? v[u].x * a[u].x + v[u].y * a[u].y : 0.0;
        s1 += ok ? v[u].z * a[u].x + v[u].w * a[u].y : 0.0;
      }
    }
  }
  {
    const int64_t k = (node >> 6) * (int64_t)urow + (node & 63);
    for (int j = 0; j < ulen; j += U) {
      int32_t c[U];
      dv4 v[U];
      double2 a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t kk = k + (int64_t)SELL_C * (j + u < ulen ? j + u : ulen - 1);
        c[u] = ld_once(ucol + kk);
        v[u] = blk<true>(uval, offd, kk);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] = xget<XFM>(x, xs, c[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = j + u < ulen;
        s0 += ok ? v[u].x * a[u].x + v[u].y * a[u].y : 0.0;
        s1 += ok ? v[u].z * a[u].x + v[u].w * a[u].y : 0.0;
      }
    }
  }
  if (GH) {   // ghost columns (after every owned column in the row's order)
    const int glen = m >> 16;
    const int64_t k = gsoff[node >> 6] + (node & 63);
    const double* goff = gval + 2 * ngs;
    for (int j = 0; j < glen; j += U) {
      int32_t c[U];
      dv4 v[U];
      double2 a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t kk = k + (int64_t)SELL_C * (j + u < glen ? j + u : glen - 1);
        c[u] = gcol[kk];
        v[u] = blk<true>(gval, goff, kk);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] = xget<XFM>(x, xs, c[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = j + u < glen;
        s0 += ok ? v[u].x * a[u].x + v[u].y * a[u].y : 0.0;
        s1 += ok ? v[u].z * a[u].x + v[u].w * a[u].y : 0.0;
      }
    }
  }
  double2 bb = {0.0, 0.0}, yy = {0.0, 0.0};
  dv4 w = {0.0, 0.0, 0.0, 0.0};
  if (EPI == EPI_RESID || EPI == EPI_BJAC)
    bb = MAMG_HSELL_NT >= 2 ? double2{ld_once(b + (bs ? node : 2 * node)), ld_once(b + (bs ? bs + node : 2 * node + 1))}
                            : double2{vget(b, bs, node, 0), vget(b, bs, node, 1)};
  if (EPI == EPI_YADD || EPI == EPI_BJAC) yy = reinterpret_cast<const double2*>(y)[node];
  if (EPI == EPI_BJAC) w = W[node];
  double o0, o1;
  if (EPI == EPI_Y) {
    o0 = s0; o1 = s1;
  } else if (EPI == EPI_YADD) {
    o0 = yy.x + s0; o1 = yy.y + s1;
  } else if (EPI == EPI_RESID) {
    o0 = bb.x - s0; o1 = bb.y - s1;
  } else {  // EPI_BJAC
    const double r0 = bb.x - s0, r1 = bb.y - s1;
    o0 = yy.x + (w.x * r0 + w.y * r1);
    o1 = yy.y + (w.z * r0 + w.w * r1);
  }
  if constexpr (MAMG_HSELL_NT >= 2) {
    __builtin_nontemporal_store(o0, out + (os ? node : 2 * node));
    __builtin_nontemporal_store(o1, out + (os ? os + node : 2 * node + 1));
  } else {
    vset(out, os, node, 0, o0);
    vset(out, os, node, 1, o1);
  }
}

// fused prolongation + first post sweep on a SELL-64 [P | AP] (see
// bsr2_post_kernel).  Rows are sorted by length inside windows of
// SELL_SIGMA rows (slot i holds row perm[i]) so a wavefront's lanes have
// near-equal trip counts; blocks [0, plen) of a row are P's, [plen, len) AP's,
// selected per block (one loop, no divergence between the two parts).
constexpr int SELL_SIGMA = 4096;

template <int TAG>
__global__ __launch_bounds__(256) void sell2_post_kernel(
    int64_t nr, const int64_t* __restrict__ soff, const int32_t* __restrict__ meta,
    const int32_t* __restrict__ perm, const int32_t* __restrict__ bcol,
    const double* __restrict__ bval, const double* __restrict__ e, const double* __restrict__ x1,
    const double* __restrict__ r1, const dv4* __restrict__ W, double* out, int64_t os) {
  const int64_t slot = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (slot >= nr) return;
  const int64_t node = perm[slot];
  const int32_t m = meta[slot];
  const int len = m & 0xffff, plen = m >> 16;
  int64_t k = soff[slot / SELL_C] + (slot & (SELL_C - 1));
  double p0 = 0.0, p1 = 0.0, q0 = 0.0, q1 = 0.0;
  int j = 0;
  for (; j + SELL_U <= len; j += SELL_U, k += SELL_U * SELL_C) {
    int32_t c[SELL_U];
    dv4 v[SELL_U];
    double2 a[SELL_U];
#pragma unroll
    for (int u = 0; u < SELL_U; ++u) { c[u] = bcol[k + u * SELL_C]; v[u] = blk<false>(bval, nullptr, k + u * SELL_C); }
#pragma unroll
    for (int u = 0; u < SELL_U; ++u) a[u] = xget<false>(e, 0, c[u]);
#pragma unroll
    for (int u = 0; u < SELL_U; ++u) {
      const double u0 = v[u].x * a[u].x + v[u].y * a[u].y, u1 = v[u].z * a[u].x + v[u].w * a[u].y;
      const bool isp = j + u < plen;
      p0 += isp ? u0 : 0.0; p1 += isp ? u1 : 0.0; q0 += isp ? 0.0 : u0; q1 += isp ? 0.0 : u1;
    }
  }
  for (; j < len; ++j, k += SELL_C) {
    const dv4 v = blk<false>(bval, nullptr, k);
    const double2 a = xget<false>(e, 0, bcol[k]);
    const double u0 = v.x * a.x + v.y * a.y, u1 = v.z * a.x + v.w * a.y;
    const bool isp = j < plen;
    p0 += isp ? u0 : 0.0; p1 += isp ? u1 : 0.0; q0 += isp ? 0.0 : u0; q1 += isp ? 0.0 : u1;
  }
  const dv4 w = W[node];
  const double d0 = r1[2 * node] - q0, d1 = r1[2 * node + 1] - q1;
  vset(out, os, node, 0, x1[2 * node] + p0 + (w.x * d0 + w.y * d1));
  vset(out, os, node, 1, x1[2 * node + 1] + p1 + (w.z * d0 + w.w * d1));
}

// block-diagonal apply: out(I) = [y(I) +] W_I b(I)
template <bool ADD>
__global__ __launch_bounds__(256) void bd2_kernel(int64_t nv, const dv4* __restrict__ W,
                                                  const double* __restrict__ b, int64_t bs,
                                                  const double* y, double* out, int64_t os) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nv) return;
  const double b0 = vget(b, bs, I, 0), b1 = vget(b, bs, I, 1);
  const double2 wb = wmul(W[I], b0, b1);
  double o0 = wb.x, o1 = wb.y;
  if (ADD) { o0 += y[2 * I]; o1 += y[2 * I + 1]; }
  vset(out, os, I, 0, o0);
  vset(out, os, I, 1, o1);
}

__global__ __launch_bounds__(256) void scale_kernel(int64_t n, const double* __restrict__ w,
                                                    const double* __restrict__ b,
                                                    double* __restrict__ x) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] = w[i] * b[i];
}

// out = w * in (SMOOTHER_POLY step smoothers w_k W, built once at upload)
__global__ __launch_bounds__(256) void wscale_kernel(int64_t n, double w, const double* __restrict__ in,
                                                     double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = w * in[i];
}

__global__ __launch_bounds__(256) void axpy_kernel(int64_t n, const double* __restrict__ e,
                                                   double* x) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] = x[i] + e[i];
}

// coarsest level: x = Ainv b, one wave per row
__global__ __launch_bounds__(256) void gemv_kernel(int64_t n, const double* __restrict__ Ainv,
                                                   const double* __restrict__ b,
                                                   double* __restrict__ x) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + wave;
  double s = 0.0;
  if (row < n) {
    const double* a = Ainv + row * n;
    for (int64_t j = lane; j < n; j += 64) s += a[j] * b[j];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (row < n && lane == 0) x[row] = s;
}

// ---- CG vector kernels ------------------------------------------------------
constexpr int DOT_BLOCKS = 1024;

__global__ __launch_bounds__(256) void dot_partial_kernel(int64_t n, const double* __restrict__ a,
                                                          const double* __restrict__ b,
                                                          double* __restrict__ part) {
  __shared__ double red[4];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    s += a[i] * b[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---- device-resident PCG state (dev_pcg): the scalars of cbc.block's
// ConjGrad live in HBM, so an iteration is one replayable hipGraph and the
// host only polls the state one iteration behind the GPU
struct PcgState {
  double rz, dq, alpha, beta, tol;
  int it, maxiter, active, run, status;   // status: PCG_* below
};
enum { PCG_RUNNING = 0, PCG_STOPPED = 1, PCG_DQ_ZERO = 2, PCG_RZ_NEG = 3, PCG_NOT_POS = 4 };

__device__ double block_sum256(double s) {   // 256 threads -> thread 0
  __shared__ double red[4];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// rz = <r, z> (partials) -> residuals[0], tolerance, first active flag
__global__ __launch_bounds__(256) void pcg_init_kernel(int nb, const double* __restrict__ part, PcgState* st,
                                                       double tol, int relconv, int maxiter, double* res) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) s += part[i];
  s = block_sum256(s);
  if (threadIdx.x) return;
  st->it = 0; st->maxiter = maxiter; st->run = 0; st->alpha = 0.0; st->beta = 0.0; st->dq = 0.0;
  st->rz = s;
  if (s < 0.0) { st->active = 0; st->status = PCG_NOT_POS; st->tol = tol; res[0] = 0.0; return; }
  const double r0 = sqrt(s);
  res[0] = r0;
  st->tol = relconv ? tol * r0 : tol;
  st->active = (r0 > st->tol && maxiter > 0) ? 1 : 0;
  st->status = st->active ? PCG_RUNNING : PCG_STOPPED;
}

// dq = <d, A d>; alpha = rz / dq (the host loop's breakdown on dq == 0)
__global__ __launch_bounds__(256) void pcg_alpha_kernel(int nb, const double* __restrict__ part, PcgState* st) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) s += part[i];
  s = block_sum256(s);
  if (threadIdx.x) return;
  st->run = st->active;
  if (!st->active) return;
  st->dq = s;
  if (s == 0.0) { st->active = 0; st->status = PCG_DQ_ZERO; return; }
  st->alpha = st->rz / s;
}

__global__ __launch_bounds__(256) void pcg_xr_kernel(int64_t n, const PcgState* __restrict__ st,
                                                     const double* __restrict__ d, const double* __restrict__ q,
                                                     double* __restrict__ x, double* __restrict__ r) {
  if (!st->active) return;
  const double alpha = st->alpha;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    x[i] = x[i] + alpha * d[i];
    r[i] = r[i] - alpha * q[i];
  }
}

// rz' = <r, B r>: beta, residuals[it + 1], stop test (tolerance / maxiter)
__global__ __launch_bounds__(256) void pcg_beta_kernel(int nb, const double* __restrict__ part, PcgState* st,
                                                       double* res, double* alphas, double* betas) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) s += part[i];
  s = block_sum256(s);
  if (threadIdx.x) return;
  if (!st->active) return;
  if (s < 0.0) { st->active = 0; st->status = PCG_RZ_NEG; return; }
  const double beta = s / st->rz;
  const int k = st->it;
  st->beta = beta;
  st->rz = s;
  res[k + 1] = sqrt(s);
  alphas[k] = st->alpha;
  betas[k] = beta;
  st->it = k + 1;
  if (!(res[k + 1] > st->tol) || k + 1 >= st->maxiter) { st->active = 0; st->status = PCG_STOPPED; }
}

// d = z + beta d; on <r, Br> < 0 this iteration's x update is undone instead
// (cbc.block restores x before breaking)
__global__ __launch_bounds__(256) void pcg_d_kernel(int64_t n, const PcgState* __restrict__ st,
                                                    const double* __restrict__ z, double* __restrict__ d,
                                                    double* __restrict__ x) {
  if (!st->run || st->status == PCG_DQ_ZERO) return;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (st->status == PCG_RZ_NEG) x[i] = x[i] - st->alpha * d[i];
  else d[i] = z[i] + st->beta * d[i];
}

// field-major [v0; v1] (stride bs) -> node-interleaved pairs
__global__ __launch_bounds__(256) void interleave2_kernel(int64_t n, const double* __restrict__ in, int64_t bs,
                                                          double* __restrict__ out) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I < n) reinterpret_cast<double2*>(out)[I] = double2{in[I], in[bs + I]};
}

// node-interleaved pairs -> out (field stride os, or node-interleaved if os == 0)
__global__ __launch_bounds__(256) void deinterleave2_kernel(int64_t n, const double* __restrict__ in,
                                                            double* __restrict__ out, int64_t os) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= n) return;
  const double2 v = reinterpret_cast<const double2*>(in)[I];
  vset(out, os, I, 0, v.x);
  vset(out, os, I, 1, v.y);
}

// ---------------------------------------------------------------------------
// Multicolour node-block Gauss-Seidel (SMOOTHER_SGS / SMOOTHER_GS): the
// reference's SGS (src/amg_parameters.py:72) and its level-0 multiplicative
// Schwarz on the seed blocks (src/utils.py:84) in a parallel order.  The
// nodes are coloured (jp_round_kernel) so that no two nodes of a colour are
// adjacent; G = A_l with its node rows permuted colour by colour, so one
// colour is one contiguous row range [c0, c1) and one launch:
//   x(I) <- x(I) + D_i (b(I) - (A x)(I)),   I = perm[i],
// in place (a lane never reads an x(J) another lane of the launch writes).
// D_i = the unscaled inverse of node I's smoother block (permuted order).
// Lane groups of VL per row as bsr2_kernel; x node-interleaved; b with field
// stride bs (the caller's [u1; u2] r on level 0).  Oracle:
// mamg_oracle.Level.gs_sweep.
// ---------------------------------------------------------------------------
template <int VL, bool SYM>
__global__ __launch_bounds__(256) void gs2_kernel(
    int64_t c0, int64_t c1, const int32_t* __restrict__ perm, const int64_t* __restrict__ bptr,
    const int32_t* __restrict__ bcol, const double* __restrict__ bval, int64_t nbt,
    const dv4* __restrict__ D, double* x, const double* __restrict__ b, int64_t bs) {
  const int lane = threadIdx.x & (VL - 1);
  const int64_t i = c0 + ((int64_t)blockIdx.x * 256 + threadIdx.x) / VL;
  const double* offd = SYM ? bval + 2 * nbt : nullptr;
  const double2* x2 = reinterpret_cast<const double2*>(x);
  double s0 = 0.0, s1 = 0.0, t0 = 0.0, t1 = 0.0;
  if (i < c1) {
    const int64_t p0 = bptr[i], p1 = bptr[i + 1];
    for (int64_t base = p0; base < p1; base += 2 * VL) {
      const int64_t ka = base + lane, kb = ka + VL;
      const bool ha = ka < p1, hb = kb < p1;
      const int64_t la = ha ? ka : p1 - 1, lb = hb ? kb : p1 - 1;
      const int32_t ca = bcol[la], cb = bcol[lb];
      const dv4 v0 = blk<SYM>(bval, offd, la), v1 = blk<SYM>(bval, offd, lb);
      const double2 a = x2[ca], e = x2[cb];
      s0 += ha ? v0.x * a.x + v0.y * a.y : 0.0;
      s1 += ha ? v0.z * a.x + v0.w * a.y : 0.0;
      t0 += hb ? v1.x * e.x + v1.y * e.y : 0.0;
      t1 += hb ? v1.z * e.x + v1.w * e.y : 0.0;
    }
  }
  s0 += t0;
  s1 += t1;
#pragma unroll
  for (int off = VL / 2; off > 0; off >>= 1) {
    s0 += __shfl_xor(s0, off, VL);
    s1 += __shfl_xor(s1, off, VL);
  }
  if (i < c1 && lane == 0 && perm[i] >= 0) {
    const int64_t I = perm[i];
    const double r0 = vget(b, bs, I, 0) - s0, r1 = vget(b, bs, I, 1) - s1;
    const dv4 d = D[i];
    const double2 xi = x2[I];
    reinterpret_cast<double2*>(x)[I] = double2{xi.x + (d.x * r0 + d.y * r1), xi.y + (d.z * r0 + d.w * r1)};
  }
}

// ---------------------------------------------------------------------------
// Coarse tail: the whole cycle of the levels from tail_level down (the
// recursion below one coarse level, V or W), run by ONE workgroup of 512
// threads that walks the same op list the launch path would launch, with a
// workgroup barrier between ops instead of a kernel boundary.  Each op
// computes every row exactly as its kernel does (same lane groups, chunks,
// shuffle order; runtime lane count), so the results equal the launch path's
// up to FMA contraction.  For the deep levels of the reference family's
// W-cycle (HEM ratio ~4, levels visited 2^l times, one launch per colour)
// this replaces tens of thousands of ~5 us launches per apply.
// ---------------------------------------------------------------------------
enum TKind { T_BSR = 0, T_BD = 1, T_GEMV = 2, T_AXPY = 3, T_ZERO = 4, T_GS = 5, T_DOT2 = 6, T_CSCALE = 7,
             T_COPY = 8, T_RLOAD = 9 };
// LDS residency (tail_lds_plan): the program itself and every work vector of
// the tail levels live in the workgroup's LDS for the whole launch; a vector
// field of a TOp then holds (byte offset in the dynamic LDS) | 1 instead of a
// global pointer (doubles are 8-aligned, so bit 0 tags it), resolved per op.
// T_COPY ops at the ends move the vectors read before written in, and the
// written ones out.  The colour steps' dependent chain becomes LDS op
// descriptor (scalar loads) -> global (L2) row pointers, columns, values ->
// LDS x gathers.
// Register residency (tail_kernel RES, tail_res_plan): the rows of the tail
// levels' operators are spread over the workgroup's threads, one row per
// thread, and held in registers for the whole launch (T_RLOAD ops at the
// start load them).  An op with res = 1 on such a matrix: thread t computes
// row t - rbase if that lies in the op's (compact) row range [r0, r1), from
// registers; ridx maps compact rows to the matrix's rows (a GS layout pads
// each colour to whole 64-row slices).  A colour step is then LDS descriptor
// -> LDS x gathers -> LDS store, with no global round trip.
struct TOp {
  int kind = 0, epi = 0, vl = 1, sym = 0, res = 0, rbase = 0;
  int64_t n = 0, r0 = 0, r1 = 0, nb = 0;
  const int64_t* ptr = nullptr;
  const int32_t* col = nullptr;
  const double* val = nullptr;
  const double *x = nullptr, *y = nullptr, *b = nullptr, *w = nullptr;
  const dv4* W = nullptr;
  double* out = nullptr;
  const int32_t* perm = nullptr;
  double* part = nullptr;
  const int32_t* ridx = nullptr;
};
// 512 threads: 256 VGPRs per lane (1024 would cap them at 128 and spill the
// interpreter's loop state to scratch); the tail's ops hold a few hundred
// rows x <= 4 lanes, so one or two passes either way
constexpr int TAIL_THREADS = 512;


// v + (v of the lane M away) inside groups of 4 lanes, by DPP quad
// permutations (one VALU op per 32-bit half) instead of an LDS-routed
// ds_bpermute; the same value and sum as __shfl_xor(v, M, 4)
template <int M>
__device__ __forceinline__ double quad_xor(double v) {
  constexpr int ctrl = M == 1 ? 0xB1 : 0x4E;   // quad_perm [1,0,3,2] / [2,3,0,1]
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, ctrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), ctrl, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// a load from an operand that is always in global memory (the tail's
// matrices): the TOp fields are generic pointers (a vector field may hold an
// LDS address), so without the cast every load would be a flat load
template <class T>
__device__ __forceinline__ T gload(const T* p) {
  return *(const __attribute__((address_space(1))) T*)p;
}
template <bool SYM>
__device__ __forceinline__ dv4 tail_blk(const double* v, const double* off, int k) {
  if (SYM) {
    const dv2 d = gload(reinterpret_cast<const dv2*>(v) + k);
    const double b = gload(off + k);
    return dv4{d.x, b, b, d.y};
  }
  return gload(reinterpret_cast<const dv4*>(v) + k);
}

#define AS1 __attribute__((address_space(1)))
#define AS3 __attribute__((address_space(3)))

// A vector operand of a tail op: in the workgroup's LDS (a tagged offset,
// tail_lds_plan) or in global memory, known per op (uniform).  Every access
// is a typed ds_ / global_ instruction, never a FLAT access through a generic
// pointer (FLAT loads of LDS data returned zeros intermittently in the row
// merges; rowstage.h).
struct TVec {
  double* g = nullptr;
  AS3 double* l = nullptr;
  bool lds = false;
  __device__ __forceinline__ double ld(int64_t i) const { return lds ? l[i] : *(const AS1 double*)(g + i); }
  __device__ __forceinline__ void st(int64_t i, double v) const {
    if (lds) l[i] = v;
    else *(AS1 double*)(g + i) = v;
  }
};
__device__ __forceinline__ TVec tvec(const double* p, char* lds) {
  const uintptr_t u = (uintptr_t)p;
  TVec v;
  v.lds = (u & 1) != 0;
  if (v.lds) v.l = (AS3 double*)(lds + (u & ~(uintptr_t)1));
  else v.g = const_cast<double*>(p);
  return v;
}
struct TOpnd {   // the vector operands of one op
  TVec x, y, b, out, part;
};

// x(c) as a pair; XL: x is in LDS for every op of the program (no branch)
template <bool XL>
__device__ __forceinline__ double2 tail_x(const TVec& x, int c) {
  if (XL || x.lds) {
    const dv2 v = ((const AS3 dv2*)x.l)[c];
    return double2{v.x, v.y};
  }
  const dv2 v = ((const AS1 dv2*)x.g)[c];
  return double2{v.x, v.y};
}

// the matrix side of a tail SpMV / GS op (global arrays, typed loads)
struct TailMat {
  const TOp& o;
  const double* offd;
  __device__ explicit TailMat(const TOp& op) : o(op), offd(op.sym ? op.val + 2 * op.nb : nullptr) {}
  __device__ int P(int i) const { return (int)gload(o.ptr + i); }
  __device__ int32_t perm(int i) const { return gload(o.perm + i); }
  __device__ dv4 W(int i) const { return gload(o.W + i); }
  __device__ int32_t C(int k) const { return gload(o.col + k); }
  __device__ dv4 V(int k) const { return o.sym ? tail_blk<true>(o.val, offd, k) : tail_blk<false>(o.val, nullptr, k); }
};
// rows of a lane-group BSR2 op (bsr2_kernel's per-row code, node-major
// vectors); GS: rows [r0, r1) of the colour-permuted matrix, update in place.
// XL: the gathered vector x lives in LDS
// LIGHT (the register-resident kernel, whose generic ops are the few
// non-resident transfers): no first-chunk prefetch, fewer live registers
template <bool XL, bool LIGHT = false>
__device__ void tail_bsr(const TOp& o, const TOpnd& V, bool gs) {
  const TailMat M(o);
  // 32-bit row arithmetic (tail levels are small) and shifts by log2(VL):
  // a 64-bit division per row chunk cost more than the chunk's loads
  const int VL = o.vl, lvl = 31 - __builtin_clz(VL);
  const int lane = threadIdx.x & (VL - 1);
  const int rows = (int)(gs ? o.r1 - o.r0 : o.n);
  const int row0 = gs ? (int)o.r0 : 0;
  const TVec& X = V.x;
  for (int base = 0; base < (rows << lvl); base += TAIL_THREADS) {   // uniform trip count
    const int v = base + (int)threadIdx.x;
    const int node = row0 + (v >> lvl);
    const bool live = (v >> lvl) < rows;
    double s0 = 0.0, s1 = 0.0, t0 = 0.0, t1 = 0.0;
    // GS: the row's own operands loaded before the block loop (its latency
    // overlaps the gathers; x(I) is not written by this colour step's other rows)
    // every lane issues its row's pointer, permutation and block-inverse
    // loads together, branch-free (a dead lane reads row row0 and drops it),
    // so they form one round trip instead of a chain behind a branch
    const int nodec = live ? node : row0;
    const int p0 = M.P(nodec), p1 = live ? M.P(nodec + 1) : p0;
    int gI = -1;
    dv4 gd = {0.0, 0.0, 0.0, 0.0};
    if (gs) {
      gI = live ? M.perm(nodec) : -1;
      gd = M.W(nodec);
    }
    const int gIc = gI >= 0 ? gI : 0;
    double gb0 = 0.0, gb1 = 0.0;
    double2 gx = {0.0, 0.0};
    if (gs) {
      gb0 = V.b.ld(2 * gIc);
      gb1 = V.b.ld(2 * gIc + 1);
      gx = tail_x<XL>(X, gIc);
    }
    if (!LIGHT && p1 > p0) {
      // the first two chunks: all column and value loads issued before any
      // gather, so a row of up to 4 VL blocks is one load -> gather round trip
      {
        int kk[4], ll[4];
        bool hh[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          kk[q] = p0 + lane + q * VL;
          hh[q] = kk[q] < p1;
          ll[q] = hh[q] ? kk[q] : p1 - 1;
        }
        int32_t cc[4];
        dv4 vv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          cc[q] = M.C(ll[q]);
          vv[q] = M.V(ll[q]);
        }
        double2 xa[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) xa[q] = tail_x<XL>(X, cc[q]);
#pragma unroll
        for (int q = 0; q < 4; q += 2) {
          s0 += hh[q] ? vv[q].x * xa[q].x + vv[q].y * xa[q].y : 0.0;
          s1 += hh[q] ? vv[q].z * xa[q].x + vv[q].w * xa[q].y : 0.0;
          t0 += hh[q + 1] ? vv[q + 1].x * xa[q + 1].x + vv[q + 1].y * xa[q + 1].y : 0.0;
          t1 += hh[q + 1] ? vv[q + 1].z * xa[q + 1].x + vv[q + 1].w * xa[q + 1].y : 0.0;
        }
      }
    }
    if (p1 > p0) {
      for (int kb0 = LIGHT ? p0 : p0 + 4 * VL; kb0 < p1; kb0 += 2 * VL) {
        const int ka = kb0 + lane, kb = ka + VL;
        const bool ha = ka < p1, hb = kb < p1;
        const int la = ha ? ka : p1 - 1, lb = hb ? kb : p1 - 1;
        const int32_t c0 = M.C(la), c1 = M.C(lb);
        const dv4 v0 = M.V(la);
        const dv4 v1 = M.V(lb);
        const double2 a = tail_x<XL>(X, c0), e = tail_x<XL>(X, c1);
        s0 += ha ? v0.x * a.x + v0.y * a.y : 0.0;
        s1 += ha ? v0.z * a.x + v0.w * a.y : 0.0;
        t0 += hb ? v1.x * e.x + v1.y * e.y : 0.0;
        t1 += hb ? v1.z * e.x + v1.w * e.y : 0.0;
      }
    }
    s0 += t0;
    s1 += t1;
    if (VL <= 4) {   // the tail's lane counts (MAMG_TAIL_VL <= 4): xor 2, then xor 1, as below
      if (VL == 4) {
        s0 += quad_xor<2>(s0);
        s1 += quad_xor<2>(s1);
      }
      if (VL >= 2) {
        s0 += quad_xor<1>(s0);
        s1 += quad_xor<1>(s1);
      }
    } else {
      for (int off = VL / 2; off > 0; off >>= 1) {
        s0 += __shfl_xor(s0, off, VL);
        s1 += __shfl_xor(s1, off, VL);
      }
    }
    if (!live || lane != 0) continue;
    if (gs) {
      if (gI < 0) continue;
      const double r0 = gb0 - s0, r1 = gb1 - s1;
      V.out.st(2 * gI, gx.x + (gd.x * r0 + gd.y * r1));
      V.out.st(2 * gI + 1, gx.y + (gd.z * r0 + gd.w * r1));
      continue;
    }
    double o0, o1;
    if (o.epi == EPI_Y) {
      o0 = s0; o1 = s1;
    } else if (o.epi == EPI_YADD) {
      o0 = V.y.ld(2 * node) + s0; o1 = V.y.ld(2 * node + 1) + s1;
    } else if (o.epi == EPI_RESID) {
      o0 = V.b.ld(2 * node) - s0; o1 = V.b.ld(2 * node + 1) - s1;
    } else if (o.epi == EPI_KPOST) {
      const double r0 = V.b.ld(2 * node), r1 = V.b.ld(2 * node + 1);
      const dv4 w = M.W(node);
      o0 = V.y.ld(2 * node) + (w.x * r0 + w.y * r1) + s0;
      o1 = V.y.ld(2 * node + 1) + (w.z * r0 + w.w * r1) + s1;
    } else {  // EPI_BJAC
      const double r0 = V.b.ld(2 * node) - s0, r1 = V.b.ld(2 * node + 1) - s1;
      const dv4 w = M.W(node);
      o0 = V.y.ld(2 * node) + (w.x * r0 + w.y * r1);
      o1 = V.y.ld(2 * node + 1) + (w.z * r0 + w.w * r1);
    }
    V.out.st(2 * node, o0);
    V.out.st(2 * node + 1, o1);
  }
}

// a thread's register-resident row (see TOp): up to RES_RB blocks; the rest
// of a longer row in the LDS region (values at ovv, 16-bit columns at ovc,
// the GS block inverse at gdo; byte offsets)
constexpr int RES_RB = 12;
struct TRes {
  int len = 0, gI = -1, ovv = 0, ovc = 0, gdo = 0;
  uint32_t c[RES_RB / 2];   // two 16-bit node columns (the tail levels have < 2^16 nodes)
  dv4 v[RES_RB];
  __device__ __forceinline__ int col(int k) const { return (int)((c[k >> 1] >> (16 * (k & 1))) & 0xffffu); }
};

// T_RLOAD: every resident row of the program from an image built at plan
// time (tail_res_plan): its blocks slot-major (val: dv4 [RES_RB][TAIL_THREADS],
// col: packed 16-bit column pairs [RES_RB / 2][TAIL_THREADS]), its header
// (ridx: length, node, first overflow block; [3][TAIL_THREADS]) and the LDS
// region's bytes (b: n bytes -> LDS byte r0: the GS block inverses, one per
// thread (TAIL_THREADS x 32 B), r1 overflow blocks' values (32 B), their
// 16-bit columns).  One coalesced round trip instead of the chain row index
// -> row pointer -> columns and values.
__device__ __forceinline__ void tail_rload(const TOp& o, TRes& R, char* lds) {
  const int t = (int)threadIdx.x;
  {   // the LDS region first (fewer live registers than after the rows' loads)
    const dv2* src = reinterpret_cast<const dv2*>(o.b);
    AS3 dv2* dst = (AS3 dv2*)(lds + o.r0);
    const int n16 = (int)(o.n / 16);
    for (int i0 = t; i0 < n16; i0 += 2 * TAIL_THREADS) {   // two 16-byte loads in flight per lane
      const bool h1 = i0 + TAIL_THREADS < n16;
      const dv2 w0 = gload(src + i0), w1 = h1 ? gload(src + i0 + TAIL_THREADS) : dv2{0.0, 0.0};
      dst[i0] = w0;
      if (h1) dst[i0 + TAIL_THREADS] = w1;
    }
  }
  const dv4* iv = reinterpret_cast<const dv4*>(o.val);
  const uint32_t* ic = reinterpret_cast<const uint32_t*>(o.col);
  R.len = gload(o.ridx + t);
  R.gI = gload(o.ridx + TAIL_THREADS + t);
  const int ovs = gload(o.ridx + 2 * TAIL_THREADS + t);
#pragma unroll
  for (int k = 0; k < RES_RB; ++k) R.v[k] = gload(iv + k * TAIL_THREADS + t);
#pragma unroll
  for (int k = 0; k < RES_RB / 2; ++k) R.c[k] = gload(ic + k * TAIL_THREADS + t);
  const int ovb = (int)o.r0 + 32 * TAIL_THREADS;
  R.ovv = ovb + 32 * ovs;
  R.ovc = ovb + 32 * (int)o.r1 + 2 * ovs;
  R.gdo = (int)o.r0 + 32 * t;
}

// a row of a T_BSR / T_GS op from the thread's resident row (tail_bsr's
// operations at node gI; one lane per row, blocks summed in row order over
// two alternating accumulators)
template <bool XL>
__device__ __forceinline__ void tail_res(const TOp& o, const TOpnd& V, const TRes& R, bool gs, const char* lds) {
  const int j = (int)threadIdx.x - o.rbase;
  if (j < (int)o.r0 || j >= (int)o.r1) return;
  const int node = R.gI;
  const TVec& X = V.x;
  double gb0 = 0.0, gb1 = 0.0;
  double2 gx = {0.0, 0.0};
  if (gs) {
    gb0 = V.b.ld(2 * node);
    gb1 = V.b.ld(2 * node + 1);
    gx = tail_x<XL>(X, node);
  }
  double s0 = 0.0, s1 = 0.0, t0 = 0.0, t1 = 0.0;
  constexpr int GQ = RES_RB / 2;   // gathers in flight
#pragma unroll
  for (int k0 = 0; k0 < RES_RB; k0 += GQ) {
    double2 xa[GQ];
#pragma unroll
    for (int q = 0; q < GQ; ++q) xa[q] = tail_x<XL>(X, R.col(k0 + q));
    // blocks past the row's length are zero (tail_rload) and gather x(0):
    // no predicate, 0 * x(0) adds +-0
#pragma unroll
    for (int q = 0; q < GQ; q += 2) {   // fused multiply-adds into four accumulators
      const int k = k0 + q;
      s0 = fma(R.v[k].y, xa[q].y, fma(R.v[k].x, xa[q].x, s0));
      s1 = fma(R.v[k].w, xa[q].y, fma(R.v[k].z, xa[q].x, s1));
      t0 = fma(R.v[k + 1].y, xa[q + 1].y, fma(R.v[k + 1].x, xa[q + 1].x, t0));
      t1 = fma(R.v[k + 1].w, xa[q + 1].y, fma(R.v[k + 1].z, xa[q + 1].x, t1));
    }
  }
  // a long row's remaining blocks, from the LDS region, four at a time:
  // their column, value and x loads issued together (two LDS round trips
  // per four blocks, not two per block); past the row's end: column 0, zero
  // values (tail_rload pads the region's last row to a multiple of 4)
  for (int k0 = 0; k0 < R.len - RES_RB; k0 += 4) {
    int c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = (int)*(const AS3 uint16_t*)(lds + R.ovc + 2 * (k0 + q));
    dv4 v[4];
    double2 a[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = *(const AS3 dv4*)(lds + R.ovv + 32 * (k0 + q));
      a[q] = tail_x<XL>(X, c[q]);
    }
#pragma unroll
    for (int q = 0; q < 4; q += 2) {
      s0 = fma(v[q].y, a[q].y, fma(v[q].x, a[q].x, s0));
      s1 = fma(v[q].w, a[q].y, fma(v[q].z, a[q].x, s1));
      t0 = fma(v[q + 1].y, a[q + 1].y, fma(v[q + 1].x, a[q + 1].x, t0));
      t1 = fma(v[q + 1].w, a[q + 1].y, fma(v[q + 1].z, a[q + 1].x, t1));
    }
  }
  s0 += t0;
  s1 += t1;
  if (gs) {
    const double r0 = gb0 - s0, r1 = gb1 - s1;
    const dv4 gd = *(const AS3 dv4*)(lds + R.gdo);
    V.out.st(2 * node, gx.x + (gd.x * r0 + gd.y * r1));
    V.out.st(2 * node + 1, gx.y + (gd.z * r0 + gd.w * r1));
    return;
  }
  double o0, o1;
  if (o.epi == EPI_Y) {
    o0 = s0; o1 = s1;
  } else if (o.epi == EPI_YADD) {
    o0 = V.y.ld(2 * node) + s0; o1 = V.y.ld(2 * node + 1) + s1;
  } else if (o.epi == EPI_RESID) {
    o0 = V.b.ld(2 * node) - s0; o1 = V.b.ld(2 * node + 1) - s1;
  } else if (o.epi == EPI_KPOST) {
    const double r0 = V.b.ld(2 * node), r1 = V.b.ld(2 * node + 1);
    const dv4 w = gload(o.W + node);
    o0 = V.y.ld(2 * node) + (w.x * r0 + w.y * r1) + s0;
    o1 = V.y.ld(2 * node + 1) + (w.z * r0 + w.w * r1) + s1;
  } else {  // EPI_BJAC
    const double r0 = V.b.ld(2 * node) - s0, r1 = V.b.ld(2 * node + 1) - s1;
    const dv4 w = gload(o.W + node);
    o0 = V.y.ld(2 * node) + (w.x * r0 + w.y * r1);
    o1 = V.y.ld(2 * node + 1) + (w.z * r0 + w.w * r1);
  }
  V.out.st(2 * node, o0);
  V.out.st(2 * node + 1, o1);
}

// STAMP: thread 0 records the 100 MHz wall clock at the start and after every
// op's barrier (stamps[0..nops]; MAMG_TAIL_PROFILE diagnosis, dev_time_apply)
// dynamic LDS: the tail levels' work vectors (tail_lds_plan)
extern __shared__ double tail_lds[];

// XL: every SpMV / GS op of the program gathers from an LDS-resident x
// (tail_lds_plan placed all of them), so the gathers are ds_reads
// RES: the program has register-resident rows (T_RLOAD, res ops)
template <bool STAMP, bool XL, bool RES>
__global__ __launch_bounds__(TAIL_THREADS) void tail_kernel(const TOp* __restrict__ gprog, int nops, int prog_lds,
                                                           uint64_t* __restrict__ stamps) {
  __shared__ double red[TAIL_THREADS / 64][2];
  TRes R;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  char* lds = reinterpret_cast<char*>(tail_lds);
  if (STAMP && t == 0) { stamps[0] = wall_clock64(); stamps[nops + 1] = clock64(); }
  // the op descriptors: copied whole into the dynamic LDS at prog_lds (>= 0)
  // once, so an op starts on LDS reads, with no global round trip on the
  // way from one op to the next; else read from global memory per op
  constexpr int TW = (int)(sizeof(TOp) / 8);
  const uint64_t* gw = reinterpret_cast<const uint64_t*>(gprog);
  const AS3 uint64_t* lw = (const AS3 uint64_t*)(lds + (prog_lds > 0 ? prog_lds : 0));
  if (prog_lds >= 0) {
    AS3 uint64_t* dst = (AS3 uint64_t*)(lds + prog_lds);
    const int nw = nops * TW;
    for (int i0 = t; i0 < nw; i0 += 8 * TAIL_THREADS) {   // 8 loads in flight per lane
      uint64_t v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = i0 + q * TAIL_THREADS < nw ? gload(gw + i0 + q * TAIL_THREADS) : 0;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (i0 + q * TAIL_THREADS < nw) dst[i0 + q * TAIL_THREADS] = v[q];
    }
    __syncthreads();
  }
  for (int k = 0; k < nops; ++k) {
    TOp od;
    if (prog_lds >= 0) {
      uint64_t w[TW];
#pragma unroll
      for (int q = 0; q < TW; ++q) {
        // the descriptor is uniform: into scalar registers, not 2 VGPRs per word
        const uint64_t v = lw[k * TW + q];
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
        w[q] = ((uint64_t)hi << 32) | lo;
      }
      __builtin_memcpy(&od, w, sizeof(TOp));
    } else {
      od = gprog[k];
    }
    const TOp& o = od;   // uniform; matrices global, vectors through V
    TOpnd V;
    V.x = tvec(od.x, lds);
    V.y = tvec(od.y, lds);
    V.b = tvec(od.b, lds);
    V.out = tvec(od.out, lds);
    V.part = tvec(od.part, lds);
    switch (o.kind) {
      case T_COPY:
        for (int64_t i = t; i < o.n; i += TAIL_THREADS) V.out.st(i, V.x.ld(i));
        break;
      case T_BSR:
        if (RES && o.res) tail_res<XL>(o, V, R, false, lds);
        else tail_bsr<XL, RES>(o, V, false);
        break;
      case T_GS:
        if (RES && o.res) tail_res<XL>(o, V, R, true, lds);
        else tail_bsr<XL, RES>(o, V, true);
        break;
      case T_RLOAD:
        if (RES) tail_rload(o, R, lds);
        break;
      case T_BD:
        for (int64_t I = t; I < o.n; I += TAIL_THREADS) {
          const double b0 = V.b.ld(2 * I), b1 = V.b.ld(2 * I + 1);
          const dv4 w = gload(o.W + I);
          V.out.st(2 * I, w.x * b0 + w.y * b1);
          V.out.st(2 * I + 1, w.z * b0 + w.w * b1);
        }
        break;
      case T_AXPY:
        for (int64_t i = t; i < o.n; i += TAIL_THREADS) V.out.st(i, V.out.ld(i) + V.x.ld(i));
        break;
      case T_ZERO:
        for (int64_t i = t; i < o.n; i += TAIL_THREADS) V.out.st(i, 0.0);
        break;
      case T_GEMV:   // gemv_kernel: one wave per row; small: one thread per row
        if (o.n <= TAIL_THREADS) {   // no shuffle tree on the dependent chain
          if (t < o.n) {
            double s0 = 0.0, s1 = 0.0;
            int j = 0;
            if ((uintptr_t)o.w & 1) {   // the matrix in the resident rows' LDS region (tail_res_plan)
              const AS3 double* a = (const AS3 double*)(lds + ((uintptr_t)o.w & ~(uintptr_t)1)) + (int64_t)t * o.n;
              for (; j + 1 < (int)o.n; j += 2) { s0 += a[j] * V.x.ld(j); s1 += a[j + 1] * V.x.ld(j + 1); }
              if (j < (int)o.n) s0 += a[j] * V.x.ld(j);
            } else {
              const double* a = o.w + (int64_t)t * o.n;
              for (; j + 1 < (int)o.n; j += 2) { s0 += gload(a + j) * V.x.ld(j); s1 += gload(a + j + 1) * V.x.ld(j + 1); }
              if (j < (int)o.n) s0 += gload(a + j) * V.x.ld(j);
            }
            V.out.st(t, s0 + s1);
          }
          break;
        }
        for (int64_t row0 = 0; row0 < o.n; row0 += TAIL_THREADS / 64) {
          const int64_t row = row0 + wave;
          double sum = 0.0;
          if (row < o.n) {
            const double* a = o.w + row * o.n;
            for (int64_t j = lane; j < o.n; j += 64) sum += gload(a + j) * V.x.ld(j);
          }
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
          if (row < o.n && lane == 0) V.out.st(row, sum);
        }
        break;
      case T_DOT2: {   // dot2_partial_kernel's SCALE_BLOCKS blocks, four at a time
        // blocks past the data hold (0 + 0) + (0 + 0) = +0.0 in the launch
        // path: written directly, so only the blocks with rows loop and sync
        const int nbl = (int)std::min<int64_t>(SCALE_BLOCKS, (o.n + 255) / 256);
        for (int i = nbl + t; i < SCALE_BLOCKS; i += TAIL_THREADS) {
          V.part.st(2 * i, 0.0);
          V.part.st(2 * i + 1, 0.0);
        }
        for (int vb0 = 0; vb0 < nbl; vb0 += TAIL_THREADS / 256) {
          const int vb = vb0 + (t >> 8), tt = t & 255;
          double a = 0.0, c = 0.0;
          for (int64_t i = (int64_t)vb * 256 + tt; i < o.n; i += (int64_t)SCALE_BLOCKS * 256) {
            a += V.b.ld(i) * V.x.ld(i);
            c += V.y.ld(i) * V.x.ld(i);
          }
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) {
            a += __shfl_xor(a, off, 64);
            c += __shfl_xor(c, off, 64);
          }
          if (lane == 0) { red[wave][0] = a; red[wave][1] = c; }
          __syncthreads();
          if (tt == 0 && vb < nbl) {
            const int w0 = (t >> 8) * 4;
            V.part.st(2 * vb, (red[w0][0] + red[w0 + 1][0]) + (red[w0 + 2][0] + red[w0 + 3][0]));
            V.part.st(2 * vb + 1, (red[w0][1] + red[w0 + 1][1]) + (red[w0 + 2][1] + red[w0 + 3][1]));
          }
          __syncthreads();
        }
        break;
      }
      case T_CSCALE: {   // cscale_kernel: alpha from the partials (one block's order), then scale
        __shared__ double alpha;
        if (t < 256) {
          double a = 0.0, c = 0.0;
          for (int i = t; i < SCALE_BLOCKS; i += 256) { a += V.part.ld(2 * i); c += V.part.ld(2 * i + 1); }
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) {
            a += __shfl_xor(a, off, 64);
            c += __shfl_xor(c, off, 64);
          }
          if (lane == 0) { red[wave][0] = a; red[wave][1] = c; }
        }
        __syncthreads();
        if (t == 0) {
          const double num = (red[0][0] + red[1][0]) + (red[2][0] + red[3][0]);
          const double den = (red[0][1] + red[1][1]) + (red[2][1] + red[3][1]);
          alpha = den > 0.0 ? num / den : 1.0;
        }
        __syncthreads();
        const double al = alpha;
        for (int64_t i = t; i < o.n; i += TAIL_THREADS) V.out.st(i, al * V.out.ld(i));
        break;
      }
      default: break;
    }
    __syncthreads();   // the next op reads what this one wrote (workgroup-scope visibility)
    if (STAMP && t == 0) { stamps[k + 1] = wall_clock64(); stamps[nops + 2 + k] = clock64(); }
  }
}

// one tail_kernel launch; flags bit 0: XL, bit 1: RES
template <bool STAMP>
void tail_launch(int flags, const TOp* prog, int n, int prog_lds, size_t lds, uint64_t* stamps, hipStream_t s) {
  switch (flags & 3) {
    case 0: tail_kernel<STAMP, false, false><<<1, TAIL_THREADS, lds, s>>>(prog, n, prog_lds, stamps); break;
    case 1: tail_kernel<STAMP, true, false><<<1, TAIL_THREADS, lds, s>>>(prog, n, prog_lds, stamps); break;
    case 2: tail_kernel<STAMP, false, true><<<1, TAIL_THREADS, lds, s>>>(prog, n, prog_lds, stamps); break;
    default: tail_kernel<STAMP, true, true><<<1, TAIL_THREADS, lds, s>>>(prog, n, prog_lds, stamps); break;
  }
}

__device__ __forceinline__ uint32_t hash32_dev(uint64_t i, int level) {   // = host.h hash32
  uint32_t x = (uint32_t)(i & 0xFFFFFFFFu);
  const uint32_t lv = (uint32_t)(((uint64_t)(int64_t)level * 0x85EBCA77ull) & 0xFFFFFFFFull);
  x = x * 0x9E3779B1u + lv;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint64_t colour_key(int64_t I, int level) {
  return ((uint64_t)hash32_dev((uint64_t)I, level + 0x4000) << 32) | (uint64_t)(uint32_t)I;
}

// one round of the Jones-Plassmann colouring (mamg_oracle.jp_colouring): an
// uncoloured node whose key beats every uncoloured neighbour's takes the
// smallest colour no coloured neighbour holds.  Reads the previous round's
// colours (cin), writes the next (cout): winners of a round are never
// adjacent, so the result is independent of the visiting order.
__global__ __launch_bounds__(256) void jp_round_kernel(int64_t nr, const int64_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ col, int level,
                                                       const int8_t* __restrict__ cin, int8_t* __restrict__ cout,
                                                       unsigned long long* nleft, int* toomany) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nr) return;
  const int8_t ci = cin[I];
  if (ci >= 0) { cout[I] = ci; return; }
  const uint64_t key = colour_key(I, level);
  uint64_t nbmax = 0, mask = 0;
  for (int64_t k = ptr[I]; k < ptr[I + 1]; ++k) {
    const int32_t J = col[k];
    if (J == I) continue;
    const int8_t cj = cin[J];
    if (cj < 0) {
      const uint64_t kj = colour_key(J, level);
      nbmax = kj > nbmax ? kj : nbmax;
    } else {
      mask |= 1ull << cj;
    }
  }
  if (key > nbmax) {
    if (~mask == 0ull) { *toomany = 1; cout[I] = 0; }
    else cout[I] = (int8_t)(__ffsll((long long)~mask) - 1);
  } else {
    cout[I] = -1;
    atomicAdd(nleft, 1ull);
  }
}

// the colouring needs an undirected node graph: every block (I, J) must have
// its mirror (J, I) (binary search in row J)
__global__ __launch_bounds__(256) void pattern_sym_kernel(int64_t nr, const int64_t* __restrict__ ptr,
                                                          const int32_t* __restrict__ col, int* bad) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nr) return;
  for (int64_t k = ptr[I]; k < ptr[I + 1]; ++k) {
    const int32_t J = col[k];
    int64_t lo = ptr[J], hi = ptr[J + 1];
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (col[m] < I) lo = m + 1; else hi = m;
    }
    if (lo >= ptr[J + 1] || col[lo] != I) { *bad = 1; return; }
  }
}

__global__ __launch_bounds__(256) void colour_count_kernel(int64_t nr, const int8_t* __restrict__ c,
                                                           int32_t* __restrict__ ci, int64_t* __restrict__ iota,
                                                           unsigned long long* cnt) {
  __shared__ unsigned int hist[64];
  if (threadIdx.x < 64) hist[threadIdx.x] = 0;
  __syncthreads();
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I < nr) {
    ci[I] = c[I];
    iota[I] = I;
    atomicAdd(&hist[c[I]], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 64 && hist[threadIdx.x]) atomicAdd(cnt + threadIdx.x, (unsigned long long)hist[threadIdx.x]);
}

// sorted position k (colour c = cs[k]) -> padded permuted row pcs[c] + k - gcs[c]
__global__ __launch_bounds__(256) void perm_place_kernel(int64_t nr, const int32_t* __restrict__ cs,
                                                         const int64_t* __restrict__ sorted,
                                                         const int64_t* __restrict__ gcs,
                                                         const int64_t* __restrict__ pcs, int32_t* __restrict__ perm) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= nr) return;
  const int c = cs[k];
  perm[pcs[c] + k - gcs[c]] = (int32_t)sorted[k];
}

__global__ __launch_bounds__(256) void perm_len_kernel(int64_t nrp, const int32_t* __restrict__ perm,
                                                       const int64_t* __restrict__ ptr, int64_t* __restrict__ gptr) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nrp) return;
  const int32_t I = perm[i];
  gptr[i + 1] = I < 0 ? 0 : ptr[I + 1] - ptr[I];
}

// ---------------------------------------------------------------------------
// Multiplicative node-patch Schwarz on level 0 (Schwarz_type PATCHES): the
// reference's level-0 smoother, symmetric multiplicative Schwarz on one block
// per seed = seed + its 1-ring (src/amg_parameters.py:83-87, src/utils.py:84)
// with exact local solves.  With a seed on every node (the bidomain's u2
// dofs, src/bidomain_3d.py:138) the block of node I is both fields of the
// closed neighbourhood N[I] = row I of A_0's node pattern.  Parallel order:
// patches coloured at distance 3 (two patch centres of one colour are >= 4
// hops apart: no patch of a launch reads an x another one writes).
// Oracle: mamg_oracle.Patches (colouring, inverses, sweep).
// ---------------------------------------------------------------------------
constexpr int PATCH_MAX_NODES = 16;
constexpr int PATCH_WORDS = 4;          // 256 colours

__device__ __forceinline__ uint64_t patch_key_dev(int64_t I) {
  return ((uint64_t)hash32_dev((uint64_t)I, 0x5000) << 32) | (uint64_t)(uint32_t)I;
}

// k[I] = key(I) while I is uncoloured, else 0
__global__ __launch_bounds__(256) void pkey_init_kernel(int64_t nr, const int16_t* __restrict__ c, uint64_t* __restrict__ k) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I < nr) k[I] = c[I] < 0 ? patch_key_dev(I) : 0ull;
}

// out[I] = max of in over row I's node columns and I itself (one hop)
__global__ __launch_bounds__(256) void pkey_max_kernel(int64_t nr, const int64_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ col, const uint64_t* __restrict__ in,
                                                       uint64_t* __restrict__ out) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nr) return;
  uint64_t m = in[I];
  for (int64_t k = ptr[I]; k < ptr[I + 1]; ++k) {
    const uint64_t v = in[col[k]];
    m = v > m ? v : m;
  }
  out[I] = m;
}

// ---- distance-3 Jones-Plassmann colouring (mamg_oracle.patch_colouring) -----
// Round-synchronous: an uncoloured node whose key is the largest uncoloured
// key within 3 hops takes the lowest colour absent within 3 hops.  That
// colours a node once every higher-keyed node within 3 hops is coloured, so
// the result is the greedy colouring in descending key order whatever the
// schedule.  Rounds 2-4 recomputed every node's 3-hop maxima and 256-bit
// colour masks each round by three full key-max and three full mask-or passes
// (12 ms per round, 341 rounds at nrefs=6: 4.2 s of the patch layout).  Since
// round 5 each round keeps, per node, the 1-, 2- and
// 3-hop maxima m1, m2, m3 of the uncoloured keys and a 1-hop colour mask:
//  * a maximum changes only when the node it names (the key's low 32 bits)
//    gets coloured, so each round re-derives just those entries (lazy refresh,
//    one level from the one below, closed neighbourhoods);
//  * a winner (m3 == own key) ORs the 1-hop masks of its 2-hop ball (= the
//    colours within 3 hops) and adds its colour bit to its neighbours' 1-hop
//    masks: two winners are > 3 hops apart, so no winner sees another's bit.
// Same keys, same rounds, same colours (tests/test_gpu_patch.py).

// m[I] refreshed from src (src == nullptr: the keys of uncoloured nodes):
// kept unless the node it names was coloured.  FIND (the 3-hop level, 1024
// threads): only uncoloured nodes, and those whose maximum is their own key
// are appended to the winner list, one atomic per workgroup.  No winner means
// no uncoloured node (the largest uncoloured key always wins).
// whether node x is coloured: one bit per node (round 6), so the lookups of
// the nodes the maxima name hit the 2 MB bitmap in L2 instead of gathering
// 2-byte colours from a 34 MB array (the same tests, the same colours)
__device__ __forceinline__ bool coloured(const uint32_t* __restrict__ cb, int64_t x) {
  return (cb[x >> 5] >> (x & 31)) & 1u;
}

template <bool FIND>
__global__ __launch_bounds__(FIND ? 1024 : 256) void pkey_refresh_kernel(
    int64_t nr, const int64_t* __restrict__ ptr, const int32_t* __restrict__ col, const uint32_t* __restrict__ cb,
    const uint64_t* __restrict__ src, uint64_t* __restrict__ m, int32_t* __restrict__ win,
    unsigned int* __restrict__ nwin) {
  constexpr int NT = FIND ? 1024 : 256;
  const int64_t I = (int64_t)blockIdx.x * NT + threadIdx.x;
  bool w = false;
  if (I < nr) {
    const bool unc = !coloured(cb, I);
    uint64_t v = m[I];
    if ((!FIND || unc) && v != 0 && coloured(cb, (uint32_t)v)) {   // its maximum was coloured: recompute
      // rows hold <= PATCH_MAX_NODES columns (build_patches checks): every
      // column load, then every gather, in flight together
      v = src ? src[I] : (unc ? patch_key_dev(I) : 0ull);
      const int64_t k0 = ptr[I];
      const int len = (int)(ptr[I + 1] - k0);
      int32_t J[PATCH_MAX_NODES];
#pragma unroll
      for (int q = 0; q < PATCH_MAX_NODES; ++q) J[q] = q < len ? col[k0 + q] : (int32_t)I;
#pragma unroll
      for (int q = 0; q < PATCH_MAX_NODES; ++q) {
        const uint64_t u = src ? src[J[q]] : (!coloured(cb, J[q]) ? patch_key_dev(J[q]) : 0ull);
        v = u > v ? u : v;
      }
      m[I] = v;
    }
    w = FIND && unc && v == patch_key_dev(I);
  }
  if constexpr (FIND) {   // workgroup-aggregated list appends
    __shared__ unsigned int wc[NT / 64 + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long bw = __ballot(w);
    if (lane == 0) wc[wv] = (unsigned int)__popcll(bw);
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned int t = 0;
      for (int k = 0; k < NT / 64; ++k) { const unsigned int x = wc[k]; wc[k] = t; t += x; }
      wc[NT / 64] = t ? atomicAdd(nwin, t) : 0u;
    }
    __syncthreads();
    if (w) win[wc[NT / 64] + wc[wv] + __popcll(bw & ((1ull << lane) - 1))] = (int32_t)I;
  }
}

// one wave per winner: the colours within 3 hops = OR of the 1-hop masks over
// the closed 2-hop ball; the lowest free colour; the colour bit into the
// 1-hop masks of the closed 1-ring
__global__ __launch_bounds__(256) void patch_win_kernel(int64_t nwin, const int32_t* __restrict__ win,
                                                        const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
                                                        int16_t* __restrict__ c, uint32_t* __restrict__ cb,
                                                        unsigned long long* __restrict__ mask1, int* toomany) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= nwin) return;
  const int64_t I = win[t];
  const int64_t p0 = ptr[I];
  const int d1 = (int)(ptr[I + 1] - p0) + 1;     // closed 1-ring: row I's columns, then I
  // lane a < d1 holds the ring's a-th member u and u's row range
  int64_t u = I, q0 = 0;
  int lu = 0;
  if (lane < d1) {
    if (lane + 1 < d1) u = col[p0 + lane];
    q0 = ptr[u];
    lu = (int)(ptr[u + 1] - q0) + 1;             // closed: u's columns, then u
  }
  unsigned long long mk[PATCH_WORDS] = {0ull, 0ull, 0ull, 0ull};
  // (a, b) pairs, 4 members of the ring at a time and 16 lanes per member
  for (int a0 = 0; a0 < d1; a0 += 4) {
    const int a = a0 + (lane >> 4);
    const int64_t ua = __shfl(u, a & 63), qa = __shfl(q0, a & 63);
    const int la = __shfl(lu, a & 63);
    if (a < d1)
      for (int b = lane & 15; b < la; b += 16) {
        const int64_t x = b + 1 < la ? (int64_t)col[qa + b] : ua;
#pragma unroll
        for (int w = 0; w < PATCH_WORDS; ++w) mk[w] |= mask1[PATCH_WORDS * x + w];
      }
  }
#pragma unroll
  for (int w = 0; w < PATCH_WORDS; ++w)
    for (int o = 32; o > 0; o >>= 1) mk[w] |= __shfl_xor(mk[w], o);
  int cc = -1;
  for (int w = 0; w < PATCH_WORDS && cc < 0; ++w)
    if (~mk[w]) cc = 64 * w + __ffsll((long long)~mk[w]) - 1;
  if (cc < 0) {
    if (lane == 0) *toomany = 1;
    cc = 0;
  }
  if (lane == 0) {
    c[I] = (int16_t)cc;
    atomicOr(&cb[I >> 5], 1u << (I & 31));
  }
  if (lane < d1) atomicOr(&mask1[PATCH_WORDS * u + cc / 64], 1ull << (cc % 64));
}

__global__ __launch_bounds__(256) void pcolour_count_kernel(int64_t nr, const int16_t* __restrict__ c,
                                                            int32_t* __restrict__ ci, int64_t* __restrict__ iota,
                                                            unsigned long long* cnt) {
  __shared__ unsigned int hist[64 * PATCH_WORDS];
  hist[threadIdx.x] = 0;
  __syncthreads();
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I < nr) {
    ci[I] = c[I];
    iota[I] = I;
    atomicAdd(&hist[c[I]], 1u);
  }
  __syncthreads();
  if (hist[threadIdx.x]) atomicAdd(cnt + threadIdx.x, (unsigned long long)hist[threadIdx.x]);
}

__global__ __launch_bounds__(256) void patch_rowlen_kernel(int64_t nr, const int64_t* __restrict__ ptr, int* maxlen) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I < nr) atomicMax(maxlen, (int)(ptr[I + 1] - ptr[I]));
}

__global__ __launch_bounds__(256) void i64_to_i32_kernel(int64_t n, const int64_t* __restrict__ a, int32_t* __restrict__ b) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) b[i] = (int32_t)a[i];
}

// column-packed upper triangle: U(i, j), i <= j, at j (j + 1) / 2 + i
__device__ __forceinline__ int upk(int i, int j) { return i <= j ? j * (j + 1) / 2 + i : i * (i + 1) / 2 + j; }

// lane src's double (src may differ per lane): two ds_bpermute_b32
__device__ __forceinline__ double bperm_f64(double v, int src) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)(unsigned)u);
  const int hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// lane l's double, broadcast to the wave (l wave-uniform)
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Patch inverses, one wave per patch (4 per workgroup).  Lane j < 2d holds
// column j of the augmented [A_p | I] (d = 2 m <= 32 rows in registers; local
// dof i = 2 a + f, a = the node's position in row I, f = field).  Gauss-Jordan
// without pivoting in mamg_oracle.batched_inverse's operation order (row k
// divided by the pivot, then M_i -= M_ik M_k, no contraction); the packed
// upper triangle of the inverse is stored (the oracle symmetrises the same).
// gcol: the rows' columns as global node ids, sorted per row (the search
// keys; = col on one GPU, the rank-local rows keep the global column order
// with local indices in col on N GPUs)
__global__ __launch_bounds__(256) void patch_inv_kernel(int64_t np, const int32_t* __restrict__ perm,
                                                        const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
                                                        const int32_t* __restrict__ gcol,
                                                        const dv4* __restrict__ val, int64_t ustride, double* __restrict__ U,
                                                        int* bad) {
#pragma clang fp contract(off)
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + wv;
  if (i >= np) return;
  const int32_t I = perm[i];
  const int64_t q0 = ptr[I];
  const int m = (int)(ptr[I + 1] - q0);
  const int d = 2 * m;
  double M[2 * PATCH_MAX_NODES];
#pragma unroll
  for (int r = 0; r < 2 * PATCH_MAX_NODES; ++r) M[r] = 0.0;
  if (lane < d) {
    const int32_t Jb = gcol[q0 + (lane >> 1)];
    const int g = lane & 1;
#pragma unroll
    for (int a = 0; a < PATCH_MAX_NODES; ++a) {
      if (a < m) {
        const int32_t Ja = col[q0 + a];
        int64_t lo = ptr[Ja], hi = ptr[Ja + 1];
        while (lo < hi) {
          const int64_t md = (lo + hi) >> 1;
          if (gcol[md] < Jb) lo = md + 1; else hi = md;
        }
        if (lo < ptr[Ja + 1] && gcol[lo] == Jb) {
          const dv4 v = val[lo];
          M[2 * a] = g ? v.y : v.x;
          M[2 * a + 1] = g ? v.w : v.z;
        }
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < 2 * PATCH_MAX_NODES; ++r) M[r] = (lane - d == r) ? 1.0 : 0.0;
  }
  // pivots unrolled (k a constant: no register selects), the pivot column's
  // entries broadcast from lane k by v_readlane rather than LDS permutes: the
  // same operations on the same values as the loop of rounds 2-4
  // (300 -> see DESIGN.md 2.11 for the measured time)
#pragma unroll
  for (int k = 0; k < 2 * PATCH_MAX_NODES; ++k) {
    if (k < d) {
      const double p = readlane_f64(M[k], k);
      if (!(p > 0.0)) { if (lane == 0) atomicOr(bad, 1); return; }
      const double mk = M[k] / p;
#pragma unroll
      for (int r = 0; r < 2 * PATCH_MAX_NODES; ++r) {
        if (r == k) continue;
        const double f = readlane_f64(M[r], k);
        const double t = f * mk;
        M[r] = M[r] - t;
      }
      M[k] = mk;
    }
  }
  if (lane >= d && lane < 2 * d) {
    const int jj = lane - d;
    double* Up = U + i * ustride + jj * (jj + 1) / 2;
#pragma unroll
    for (int r = 0; r < 2 * PATCH_MAX_NODES; ++r)
      if (r <= jj) Up[r] = M[r];
  }
}

// ---- patch matrices through LDS (round 6): the assembly and the packed
// store of the patch inverse kernels.  A patch's 32 x 32 matrix (zero past
// d, the identity on the padded diagonal when `pad`) sits column-major with
// stride PATCH_LD doubles (33: the tile reads of patch_inv3_kernel hit 32
// banks).
constexpr int PATCH_LD = 33;

// Assembly by rows: the patch's nl lanes take its row nodes, L = nl / 16
// lanes per row node a (Ja = the centre row's a-th column) and the patch
// nodes b = q, q + L, .. of lane q; each lane loads Ja's <= 16 keys at once,
// finds its nodes' keys among them by comparisons in registers, then loads
// the found blocks at once: three dependent loads instead of one five-step
// binary search per (row, column) pair.  A pair absent from Ja's row stays 0.
// The values are copies: the assembled matrix is the one the searches built.
template <int L>
__device__ __forceinline__ void patch_assemble(double* S, int sub, int q0i, int64_t q0, int m, bool pad,
                                               const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
                                               const int32_t* __restrict__ gcol, const dv4* __restrict__ val) {
  (void)q0i;
  constexpr int nl = 16 * L, NB = PATCH_MAX_NODES / L;
  const int d = 2 * m;
  for (int k = sub; k < 32 * PATCH_LD; k += nl) {
    const int j = k / PATCH_LD, r = k - j * PATCH_LD;
    S[k] = (pad && r == j && j >= d) ? 1.0 : 0.0;
  }
  const int a = sub / L, q = sub % L;
  if (a >= m) return;
  const int32_t Ja = col[q0 + a];
  const int64_t p0 = ptr[Ja];
  const int n = (int)(ptr[Ja + 1] - p0);
  int32_t kr[PATCH_MAX_NODES], kb[NB];
#pragma unroll
  for (int k = 0; k < PATCH_MAX_NODES; ++k) kr[k] = k < n ? gcol[p0 + k] : -1;
#pragma unroll
  for (int t = 0; t < NB; ++t) kb[t] = q + L * t < m ? gcol[q0 + q + L * t] : -2;
  int pos[NB];
#pragma unroll
  for (int t = 0; t < NB; ++t) {
    int x = -1;
#pragma unroll
    for (int k = 0; k < PATCH_MAX_NODES; ++k) x = kr[k] == kb[t] ? k : x;
    pos[t] = x;
  }
  dv4 v[NB];
#pragma unroll
  for (int t = 0; t < NB; ++t) v[t] = pos[t] >= 0 ? val[p0 + pos[t]] : dv4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int t = 0; t < NB; ++t)
    if (pos[t] >= 0) {
      const int b = q + L * t;
      double* c0 = S + (2 * b) * PATCH_LD + 2 * a;
      double* c1 = c0 + PATCH_LD;
      c0[0] = v[t].x; c1[0] = v[t].y; c0[1] = v[t].z; c1[1] = v[t].w;
    }
}

// the packed upper triangle (column j: rows 0 .. j, at j (j + 1) / 2) of
// sign * the LDS matrix, written by nl lanes with consecutive addresses
__device__ __forceinline__ void patch_store(const double* S, int sub, int nl, int d, double sign, double* __restrict__ Up) {
  const int nt = d * (d + 1) / 2;
  for (int k = sub; k < nt; k += nl) {
    int j = (int)((sqrtf(8.0f * (float)k + 1.0f) - 1.0f) * 0.5f);
    j += (j + 1) * (j + 2) / 2 <= k ? 1 : 0;
    j -= j * (j + 1) / 2 > k ? 1 : 0;
    Up[k] = sign * S[j * PATCH_LD + (k - j * (j + 1) / 2)];
  }
}

// Patch inverses, two patches per wave (round 6): the same
// operations on the same values as patch_inv_kernel, so the same bits, with
// half the instructions per patch.
//  * In place: half-wave h (lanes 32 h .. 32 h + 31) holds one patch, lane j
//    < d column j of A_p (d = 2 m <= 32).  At pivot k, column k of the
//    augmented [A_p | I] becomes e_k and identity column k is e_k until then
//    (exactly: every update of it adds -(f x +0) = +0), so lane k takes
//    over identity column k: row k = 1 / p, row r = 0 - f_r (1 / p), the
//    augmented code's own operations on it.  The other lanes update as
//    before (row k divided by the pivot, then M_r -= f_r M_k, no
//    contraction); f_r = column k's row r, broadcast within the half by
//    ds_bpermute (one instruction serves both patches) before lane k
//    overwrites it.
//  * Assembly: each lane's block searches in the patch rows run as
//    PATCH_MAX_NODES independent branch-free binary searches (5 steps for
//    rows of <= 16 blocks, every load in bounds), one straight-line block
//    whose loads overlap, instead of one data-dependent loop per row after
//    another.
//  * The pivot and row loops are fully unrolled (a partly rolled loop put M
//    in scratch: 272 B per lane, 1.8 s at nrefs=6).
__global__ __launch_bounds__(256) void patch_inv2_kernel(int64_t np, const int32_t* __restrict__ perm,
                                                         const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
                                                         const int32_t* __restrict__ gcol,
                                                         const dv4* __restrict__ val, int64_t ustride, double* __restrict__ U,
                                                         int* bad) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63, hl = lane & 31, hb = lane & 32;
  const int64_t i = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 6) * 2 + (lane >> 5);
  const bool live = i < np;
  const int32_t I = live ? perm[i] : 0;
  const int64_t q0 = ptr[I];
  const int m = live ? (int)(ptr[I + 1] - q0) : 0;
  const int d = 2 * m;
  double M[2 * PATCH_MAX_NODES];
#pragma unroll
  for (int r = 0; r < 2 * PATCH_MAX_NODES; ++r) M[r] = 0.0;
  if (hl < d) {
    const int32_t Jb = gcol[q0 + (hl >> 1)];
    const int g = hl & 1;
    // each row's lower bound of Jb by a branch-free 5-step binary search
    // (rows of <= 16 blocks), every load in bounds, so the rows' searches
    // form one straight-line block and their loads overlap
#pragma unroll
    for (int a = 0; a < PATCH_MAX_NODES; ++a) {
      const bool va = a < m;
      const int32_t Ja = va ? col[q0 + a] : I;
      const int64_t p0 = ptr[Ja];
      const int n = va ? (int)(ptr[Ja + 1] - p0) : 0;
      int64_t b = p0;
      int l = n;
#pragma unroll
      for (int st = 0; st < 5; ++st) {
        const int h = l >> 1;
        const bool lt = gcol[l > 0 ? b + h : p0] < Jb;
        b = (l > 0 && lt) ? b + h + 1 : b;
        l = l > 0 ? (lt ? l - h - 1 : h) : 0;
      }
      if (va && b < p0 + n && gcol[b] == Jb) {
        const dv4 v = val[b];
        M[2 * a] = g ? v.y : v.x;
        M[2 * a + 1] = g ? v.w : v.z;
      }
    }
  }
  bool ok = true;
#pragma clang loop unroll(full)
  for (int k = 0; k < 2 * PATCH_MAX_NODES; ++k) {
    // every lane takes part in the broadcasts (the other half may have k < d)
    const double p = bperm_f64(M[k], hb + k);
    const bool act = k < d && ok;
    if (act && !(p > 0.0)) ok = false;
    const bool upd = act && ok && hl < d;
    const bool own = hl == k;
    const double mk = own ? 1.0 / p : M[k] / p;
#pragma clang loop unroll(full)
    for (int r = 0; r < 2 * PATCH_MAX_NODES; ++r) {
      if (r == k) continue;
      const double f = bperm_f64(M[r], hb + k);
      const double t = f * mk;
      if (upd) M[r] = (own ? 0.0 : M[r]) - t;
    }
    if (upd) M[k] = mk;
  }
  if (!ok && hl == 0) atomicOr(bad, 1);
  if (live && ok && hl < d) {
    double* Up = U + i * ustride + hl * (hl + 1) / 2;
#pragma unroll
    for (int r = 0; r < 2 * PATCH_MAX_NODES; ++r)
      if (r <= hl) Up[r] = M[r];
  }
}

// Patch inverses on the matrix cores (round 6):
// one patch per wave, the 32 x 32 (zero-padded to the identity past d)
// patch matrix as four 16 x 16 f64 tiles in the v_mfma_f64_16x16x4 C/D
// layout (lane l, register r: row 16a + (l >> 4) + 4r, column 16b + (l & 15)),
// inverted by the symmetric block sweep on 4 x 4 pivot blocks K:
//   P = M(K, K), R = M(K, :), S = P^-1 R               (one MFMA per tile column)
//   M(i, j) -= S(:, i)^T R(:, j)  for all i, j          (four MFMAs: the A operand
//                                                        is S itself, the B operand R
//                                                        itself -- no data movement)
//   M(K, :) = S, M(:, K) = S^T (ds_bpermute), M(K, K) = -P^-1,
// which leaves M = -A_p^-1 after the eight blocks (Goodnight's sweep;
// symmetry is what makes the column panel S^T, so the row panel alone feeds
// both operands).  A_p is SPD, so no pivoting: a non-positive pivot of a 4 x 4
// block sets *bad as the scalar kernels do.  Assembly as patch_inv2_kernel
// (lane j < 32 builds column j), then an LDS transpose into the tile layout.
// The rounding differs from the scalar Gauss-Jordan: the inverses equal
// patch_inv2_kernel's to ~1e-14 relative (tests/test_gpu_patch.py).
// PART (diagnosis build only, MAMG_PATCH_INV 4 / 5): 1 = assembly and
// stores without the sweep, 2 = the sweep on the identity without assembly
// Waves take patches in colour order, so the 4.2 KB inverses are written in
// address order.  (Node order -- neighbouring patches, whose rows overlap,
// assembled together from L2 -- was 1.3 ms faster in a fresh process but
// 2.9 s slower in a process that had just freed another 63 GB inverse array:
// writes scattered over 72 GB)
template <int PART = 0>
__global__ __launch_bounds__(256, 4) void patch_inv3_kernel(int64_t np, const int32_t* __restrict__ perm,
                                                         const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
                                                         const int32_t* __restrict__ gcol,
                                                         const dv4* __restrict__ val, int64_t ustride, double* __restrict__ U,
                                                         int* bad) {
  constexpr int LD = PATCH_LD;
  __shared__ double sm[4][32 * LD];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane >> 4, lc = lane & 15;
  const int64_t i = (int64_t)blockIdx.x * 4 + w;
  const bool live = i < np;
  const int32_t I = live ? perm[i] : 0;
  const int64_t q0 = ptr[I];
  const int m = live ? (int)(ptr[I + 1] - q0) : 0;
  const int d = 2 * m;
  double* S = sm[w];
  if (PART == 2) {   // diagnosis: the identity
    for (int k = lane; k < 32 * LD; k += 64) S[k] = (k % LD == k / LD) ? 1.0 : 0.0;
  } else {
    patch_assemble<4>(S, lane, 0, q0, m, true, ptr, col, gcol, val);
  }
  __syncthreads();
  dv4 T[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) T[a][b][r] = S[(16 * b + lc) * LD + 16 * a + lr + 4 * r];
  bool ok = true;
#pragma unroll
  for (int K = 0; K < (PART == 1 ? 0 : 8); ++K) {
    const int t = K >> 2, rr = K & 3;
    // the pivot block spread over 16 lanes: lane l holds Q(l & 15, l >> 4)
    // for (l & 15) < 4 (P(kk, c) sits in lane 16 kk + 4 rr + c of T[t][t][rr]),
    // swept in place (Q <- -P^-1): per pivot one broadcast and two permutes
    const bool qv = lc < 4;
    double Q = bperm_f64(T[t][t][rr], qv ? 16 * lc + 4 * rr + lr : lane);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const double dp = readlane_f64(Q, 17 * p);
      ok = ok && dp > 0.0;
      // 1 / dp: v_rcp_f64 and two Newton steps (the IEEE division sequence
      // is a 10-deep dependent chain, four per block)
      double inv = __builtin_amdgcn_rcp(dp);
      inv = fma(inv, fma(-dp, inv, 1.0), inv);
      inv = fma(inv, fma(-dp, inv, 1.0), inv);
      const double qrp = bperm_f64(Q, 16 * p + lc), qpc = bperm_f64(Q, 16 * lr + p);
      const bool rp = lc == p, cp = lr == p;
      // every candidate computed, then selected (no divergent branches)
      const double upd = Q - qrp * qpc * inv, scl = Q * inv;
      const double q1 = (rp || cp) ? scl : upd;
      Q = (rp && cp) ? -inv : q1;
    }
    // A operand of S = P^-1 R: lane l holds (P^-1)(l & 15, l >> 4) for (l & 15) < 4, else 0
    const double pa = qv ? -Q : 0.0;
    const double R0 = T[t][0][rr], R1 = T[t][1][rr];
    const dv4 z = {0.0, 0.0, 0.0, 0.0};
    const double S0 = __builtin_amdgcn_mfma_f64_16x16x4f64(pa, R0, z, 0, 0, 0)[0];   // S(lr, lc) of column tile 0
    const double S1 = __builtin_amdgcn_mfma_f64_16x16x4f64(pa, R1, z, 0, 0, 0)[0];
    // M -= S^T R on every tile (rows and columns K are rewritten below)
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const double sa = a ? -S1 : -S0;
      T[a][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(sa, R0, T[a][0], 0, 0, 0);
      T[a][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(sa, R1, T[a][1], 0, 0, 0);
    }
    // row panel K <- S (the same lanes), column panel K <- S^T
    T[t][0][rr] = S0;
    T[t][1][rr] = S1;
    const bool inK = lc >= 4 * rr && lc < 4 * rr + 4;
    const int kk = inK ? lc - 4 * rr : 0;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double v = bperm_f64(a ? S1 : S0, 16 * kk + lr + 4 * r);
        T[a][t][r] = inK ? v : T[a][t][r];
      }
    // pivot block K <- -P^-1 (= Q): (lr, kk) from lane 16 kk + lr
    const double qk = bperm_f64(Q, 16 * kk + lr);
    T[t][t][rr] = inK ? qk : T[t][t][rr];
  }
  if (!ok && lane == 0 && live) atomicOr(bad, 1);
  // M = -A_p^-1: the tiles back into LDS, then the packed upper triangle of -M
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) S[(16 * b + lc) * LD + 16 * a + lr + 4 * r] = T[a][b][r];
  __syncthreads();
  if (live && ok) patch_store(S, lane, 64, d, -1.0, U + i * ustride);
}

// MAMG_PATCH_INV: 1 the round-5 kernel (one patch per wave), 2 two patches
// per wave (bitwise the same), default 3 the matrix-core block sweep
int patch_inv_version() {
  const char* e = opt("MAMG_PATCH_INV");
  const int v = e ? std::atoi(e) : 3;
#if MAMG_DIAG
  if (v == 4 || v == 5) return v;
#endif
  return v == 1 || v == 2 ? v : 3;
}

void launch_patch_inv(int64_t np, const int32_t* perm, const int64_t* ptr, const int32_t* col, const int32_t* gcol,
                      const dv4* val, int64_t ustride, double* U, int* bad) {
  if (np <= 0) return;
  switch (patch_inv_version()) {
    case 1: patch_inv_kernel<<<(unsigned)((np + 3) / 4), 256>>>(np, perm, ptr, col, gcol, val, ustride, U, bad); break;
    case 2: patch_inv2_kernel<<<(unsigned)((np + 7) / 8), 256>>>(np, perm, ptr, col, gcol, val, ustride, U, bad); break;
#if MAMG_DIAG
    case 4: patch_inv3_kernel<1><<<(unsigned)((np + 3) / 4), 256>>>(np, perm, ptr, col, gcol, val, ustride, U, bad); break;
    case 5: patch_inv3_kernel<2><<<(unsigned)((np + 3) / 4), 256>>>(np, perm, ptr, col, gcol, val, ustride, U, bad); break;
#endif
    default: patch_inv3_kernel<<<(unsigned)((np + 3) / 4), 256>>>(np, perm, ptr, col, gcol, val, ustride, U, bad); break;
  }
}

// One colour of a patch sweep, one wave per patch (4 per workgroup), in place
// on x (node-interleaved):  x|_p += Minv_p (b - A x)|_p.  The patch's node rows
// are reduced by 4 lanes each (lanes 4a..4a+3 = node a); lane i < d then forms
// delta_i = sum_j U(min, max) r_j and updates its own dof.  b has field stride
// bs (the caller's [u1; u2] r on level 0).
__global__ __launch_bounds__(256) void patch_kernel(int64_t c0, int64_t c1, const int32_t* __restrict__ perm,
                                                    const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
                                                    const dv4* __restrict__ val, const double* __restrict__ U,
                                                    int64_t ustride, double* x, const double* __restrict__ b, int64_t bs) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t i = c0 + (int64_t)blockIdx.x * 4 + wv;
  if (i >= c1) return;
  const int32_t I = perm[i];
  const int64_t q0 = ptr[I];
  const int m = (int)(ptr[I + 1] - q0);
  const int a = lane >> 2, q = lane & 3;
  const double2* x2 = reinterpret_cast<const double2*>(x);
  // this lane's row of the packed inverse, loaded up front: it does not
  // depend on the residual, so its latency overlaps the row gathers
  const double* Up = U + i * ustride;
  const int li = lane < 2 * m ? lane : 0;
  double u[2 * PATCH_MAX_NODES];
#pragma unroll
  for (int j = 0; j < 2 * PATCH_MAX_NODES; ++j) u[j] = j < 2 * m ? Up[upk(li, j)] : 0.0;
  // node a's row, blocks q, q + 4, q + 8, q + 12 (a row has <= PATCH_MAX_NODES
  // blocks): loads first, then gathers, then the sums in block order
  double s0 = 0.0, s1 = 0.0;
  int32_t J = 0;
  if (a < m) {
    J = col[q0 + a];
    const int64_t p0 = ptr[J], p1 = ptr[J + 1];
    int32_t c[PATCH_MAX_NODES / 4];
    dv4 v[PATCH_MAX_NODES / 4];
    double2 xc[PATCH_MAX_NODES / 4];
#pragma unroll
    for (int t = 0; t < PATCH_MAX_NODES / 4; ++t) {
      const int64_t k = p0 + q + 4 * t;
      const int64_t kk = k < p1 ? k : p0;
      c[t] = col[kk];
      v[t] = val[kk];
    }
#pragma unroll
    for (int t = 0; t < PATCH_MAX_NODES / 4; ++t) xc[t] = x2[c[t]];
#pragma unroll
    for (int t = 0; t < PATCH_MAX_NODES / 4; ++t)
      if (p0 + q + 4 * t < p1) {
        s0 += v[t].x * xc[t].x + v[t].y * xc[t].y;
        s1 += v[t].z * xc[t].x + v[t].w * xc[t].y;
      }
  }
  s0 += __shfl_xor(s0, 1);
  s1 += __shfl_xor(s1, 1);
  s0 += __shfl_xor(s0, 2);
  s1 += __shfl_xor(s1, 2);
  double r0 = 0.0, r1 = 0.0;
  if (a < m) {
    r0 = vget(b, bs, J, 0) - s0;
    r1 = vget(b, bs, J, 1) - s1;
  }
  double delta = 0.0;
#pragma unroll
  for (int jn = 0; jn < PATCH_MAX_NODES; ++jn) {
    const double a0 = __shfl(r0, 4 * jn), a1 = __shfl(r1, 4 * jn);
    if (jn < m) delta += u[2 * jn] * a0 + u[2 * jn + 1] * a1;
  }
  if (lane < 2 * m) {
    const int64_t Ji = col[q0 + (lane >> 1)];
    x[2 * Ji + (lane & 1)] += delta;
  }
}

// ---------------------------------------------------------------------------
// Multiplicative seed-ring Schwarz (Schwarz_type RINGS, level 0): the
// reference's SCHWARZ_SYMMETRIC on one block per seed = the seed and its
// breadth-first Schwarz_maxlvl ring (src/utils.py:60-86), exact local solves.
// Blocks of one colour share no member and read no x another one writes, so
// a colour is one launch, one 128-thread workgroup per block:
//   r|_k = b|_k - (A x)|_k  (one thread per member: the member's field row of
//   A_0's node BSR2 row), then x|_k += Minv_k r|_k  (thread a: sum over c of
//   Minv(a, c) r_c from the transposed inverse, coalesced over the threads).
// x node-interleaved; b with field stride bs.  Oracle: mamg_oracle.Rings.sweep.
constexpr int RING_THREADS = 128;
__global__ __launch_bounds__(RING_THREADS) void ring_kernel(int64_t k0, const int64_t* __restrict__ mo,
                                                         const int32_t* __restrict__ mem,
                                                         const int64_t* __restrict__ io,
                                                         const double* __restrict__ minvT,
                                                         const int64_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ col,
                                                         const dv4* __restrict__ val, double* x,
                                                         const double* __restrict__ b, int64_t bs) {
  __shared__ double res[RING_MAX_DOFS];
  const int64_t k = k0 + blockIdx.x;
  const int64_t m0 = mo[k];
  const int d = (int)(mo[k + 1] - m0);
  const double* T = minvT + io[k];
  const double2* x2 = reinterpret_cast<const double2*>(x);
  for (int a = threadIdx.x; a < d; a += RING_THREADS) {
    const int32_t g = mem[m0 + a];
    const int32_t I = g >> 1;
    const int f = g & 1;
    double s = 0.0;
    const int64_t p1 = ptr[I + 1];
    for (int64_t q = ptr[I]; q < p1; ++q) {
      const dv4 v = val[q];
      const double2 xj = x2[col[q]];
      s += f ? v.z * xj.x + v.w * xj.y : v.x * xj.x + v.y * xj.y;
    }
    res[a] = vget(b, bs, I, f) - s;
  }
  __syncthreads();
  for (int a = threadIdx.x; a < d; a += RING_THREADS) {
    double dl = 0.0;
    for (int c = 0; c < d; ++c) dl += T[(int64_t)c * d + a] * res[c];
    x[mem[m0 + a]] += dl;
  }
}

// block j of the colour order <- block ord[j] of ring_blocks_dev's output:
// its inverse transposed into rinv at rio[j]
__global__ __launch_bounds__(256) void ring_perm_inv_kernel(int64_t nb, const int32_t* __restrict__ ord,
                                                            const int64_t* __restrict__ blen,
                                                            const int64_t* __restrict__ sq,
                                                            const double* __restrict__ inv,
                                                            const int64_t* __restrict__ rio, double* __restrict__ rinv) {
  const int64_t j = blockIdx.x;
  if (j >= nb) return;
  const int64_t o = ord[j], d = blen[o];
  const double* src = inv + (o ? sq[o - 1] : 0);
  double* dst = rinv + rio[j];
  for (int64_t t = threadIdx.x; t < d * d; t += 256) {
    const int64_t a = t / d, c = t - a * d;
    dst[c * d + a] = src[t];
  }
}

// the rest's GS (RINGS): node blocks with one covered dof become split
// (diagonal) smoother blocks, so gs_layout inverts them as two 1x1 blocks;
// cov[I]: bit f = dof f of node I lies in a seed block
__global__ __launch_bounds__(256) void rest_w_kernel(int64_t nv, const dv4* __restrict__ W,
                                                     const uint8_t* __restrict__ cov, dv4* __restrict__ Wp) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nv) return;
  const dv4 w = W[I];
  const uint8_t c = cov[I];
  Wp[I] = (c == 1 || c == 2) ? dv4{w.x, 0.0, 0.0, w.w} : w;
}

// ... and the covered dofs take no update: their rows / columns of D zeroed
__global__ __launch_bounds__(256) void rest_mask_kernel(int64_t nr, const int32_t* __restrict__ perm,
                                                        const uint8_t* __restrict__ cov, dv4* __restrict__ D) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nr || perm[i] < 0) return;
  const uint8_t c = cov[perm[i]];
  const dv4 d = D[i];
  if (c == 3) D[i] = dv4{0.0, 0.0, 0.0, 0.0};
  else if (c == 1) D[i] = dv4{0.0, 0.0, 0.0, d.w};
  else if (c == 2) D[i] = dv4{d.x, 0.0, 0.0, 0.0};
}

// 2x2 Gauss-Jordan without pivoting in mamg_oracle.batched_inverse's
// operation order (no contraction), on node I's diagonal block; the
// off-diagonals are dropped when I's two dofs are separate smoother blocks
// (W_I diagonal), which gives exactly the two 1x1 inverses
__device__ dv4 gj2_inverse(double a00, double a01, double a10, double a11, int* bad) {
#pragma clang fp contract(off)
  if (!(a00 > 0.0)) { *bad = 1; return dv4{0.0, 0.0, 0.0, 0.0}; }
  const double p = a00;
  const double r01 = a01 / p, r02 = 1.0 / p, r03 = 0.0 / p;
  const double f1 = a10;
  double m11 = a11 - f1 * r01, m12 = 0.0 - f1 * r02, m13 = 1.0 - f1 * r03;
  if (!(m11 > 0.0)) { *bad = 1; return dv4{0.0, 0.0, 0.0, 0.0}; }
  const double q = m11;
  m12 = m12 / q;
  m13 = m13 / q;
  const double f0 = r01;
  const double n02 = r02 - f0 * m12, n03 = r03 - f0 * m13;
  return dv4{n02, n03, m12, m13};
}

__global__ __launch_bounds__(256) void perm_fill_kernel(int64_t nr, const int32_t* __restrict__ perm,
                                                        const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
                                                        const dv4* __restrict__ val, const dv4* __restrict__ W,
                                                        const int64_t* __restrict__ gptr, int32_t* __restrict__ gcol,
                                                        dv4* __restrict__ gval, dv4* __restrict__ Dg, int* bad) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nr) return;
  if (perm[i] < 0) { Dg[i] = dv4{0.0, 0.0, 0.0, 0.0}; return; }
  const int64_t I = perm[i];
  int64_t o = gptr[i];
  dv4 dg = {0.0, 0.0, 0.0, 0.0};
  bool has = false;
  for (int64_t k = ptr[I]; k < ptr[I + 1]; ++k, ++o) {
    gcol[o] = col[k];
    gval[o] = val[k];
    if (col[k] == I) { dg = val[k]; has = true; }
  }
  if (!has) { *bad = 1; return; }
  const dv4 w = W[I];
  const bool split = w.y == 0.0 && w.z == 0.0;
  Dg[i] = gj2_inverse(dg.x, split ? 0.0 : dg.y, split ? 0.0 : dg.z, dg.w, bad);
}

// coarse-grid correction scaling (coarse_scaling ON, src/amg_parameters.py:78):
// alpha = <b_c, e> / <A_c e, e> (= <r, P e> / <A P e, P e> for A_c = P^T A P),
// e <- alpha e; alpha = 1 if the denominator is not positive.  Partial sums
// per block, then every block of the scaling launch reduces the partials in
// the same fixed order (so all agree on alpha).  Oracle: mamg_oracle.coarse_scale.
__global__ __launch_bounds__(256) void dot2_partial_kernel(int64_t n, const double* __restrict__ bc,
                                                           const double* __restrict__ e,
                                                           const double* __restrict__ q,
                                                           double* __restrict__ part) {
  __shared__ double red[8];
  double s = 0.0, t = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    s += bc[i] * e[i];
    t += q[i] * e[i];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, 64);
    t += __shfl_xor(t, off, 64);
  }
  if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = s; red[4 + (threadIdx.x >> 6)] = t; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
    part[2 * blockIdx.x + 1] = (red[4] + red[5]) + (red[6] + red[7]);
  }
}

__global__ __launch_bounds__(256) void cscale_kernel(int64_t n, int nb, const double* __restrict__ part,
                                                     double* __restrict__ e) {
  __shared__ double red[8];
  __shared__ double alpha;
  double s = 0.0, t = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) { s += part[2 * i]; t += part[2 * i + 1]; }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, 64);
    t += __shfl_xor(t, off, 64);
  }
  if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = s; red[4 + (threadIdx.x >> 6)] = t; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double num = (red[0] + red[1]) + (red[2] + red[3]);
    const double den = (red[4] + red[5]) + (red[6] + red[7]);
    alpha = den > 0.0 ? num / den : 1.0;
  }
  __syncthreads();
  const double a = alpha;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) e[i] = a * e[i];
}

inline unsigned nblocks(int64_t work) { return (unsigned)((work + 255) / 256); }

// Tuning knobs (environment, read at upload), kept
// because a test or an A/B needs them:
//   MAMG_SELL_MIN_ROWS  node rows from which a level-0-class operator is stored
//                       SELL-64 / half-symmetric (default 2^20; tests lower it
//                       to exercise those formats on small problems)
//   MAMG_MSELL_MIN_ROWS node rows from which a coarse level's A and K are stored
//                       SELL-64 with several lanes per row (msell_kernel; off by
//                       default: slower than the lane-group BSR kernels there)
//   MAMG_HALF           0: SELL-64 instead of the half-symmetric ELL-64 A0 (1)
//   MAMG_HALF_BANDS     band schedule of the half-symmetric kernel: sub-bands per
//                       XCD (1; 0 = row order)
//   MAMG_R_BANDS        plane-band schedule of the level-0 restriction: sub-bands
//                       per XCD (1; 0 = XCD-contiguous rows)
//   MAMG_K_SORT         level-0 K's rows sorted by length inside each SELL slice
//                       (1; 0 = row order; sort_sell_slices)
//   MAMG_POST_K         0: fused post sweep over [P | AP] instead of K = P - W A P (1)
//   multi-GPU (mamg_setup_dist): MAMG_OVERLAP 0 = no interior-row launch during
//   the forward halo (1); MAMG_DIST_TEST=dry: a virtual rank skips its exchanges
//   (compute-only timing; results meaningless); setup: MAMG_PRERESERVE_B_PER_NNZ
// Fixed by measurement (round 1 A/Bs; the variants
// measured slower were removed in round 2): XCD-contiguous restriction rows,
// SELL chunks of 8 blocks (K: 6), half-symmetric chunks of 4 with
// XCD-contiguous rows, symmetric-block packing, lane counts from the mean row
// length.
constexpr int g_sell_u = 8;
constexpr int g_post_u = 6;
constexpr int64_t g_sell_max_len = 40;
int g_half = 1;
int g_half_bands = 1;
int g_r_bands = 1;
int g_k_sort = 1;
int g_post_k = 1;
int g_kvar = 0;
int g_k_c16 = 1;   // MAMG_K_COL16: level-0 K's columns as 16-bit offsets from a per-slice base
__global__ void warm_kernel() {}

// MAMG_FUSE_RBD: which restrictions write the next level's first sweep
// (EPI_YBD): 2 those below level 0 (default), 1 all, 0 none.  A/B at
// nrefs=6 (profiles/r05_fuse_rbd_ab.txt, 3 x 3 alternating runs): coarse
// levels 0.400 -> 0.386 ms with 2; with 1 also level 0's restriction,
// 0.461 -> 0.490 ms, a net loss
int g_fuse_rbd = 2;
int64_t g_sell_min_rows = 1 << 20;
int64_t g_msell_min_rows = (int64_t)1 << 40;
int64_t g_tail_nodes = 0;
bool g_tail_set = false;   // MAMG_TAIL_NODES given: applies to every smoother (tests)   // off: coarse levels 0.41 -> 0.50 ms
int g_tail_vl = 4;           // lanes per row cap inside the coarse tail (MAMG_TAIL_VL; 1/2/4/8/64 measured)
void read_knobs() {
  const char* e = nullptr;
#if MAMG_DIAG
  e = std::getenv("MAMG_K_VARIANT");   // the level-0 K kernel (diagnosis build: tests, A/Bs; read at upload)
  g_kvar = e ? std::atoi(e) : 0;
#endif
  e = opt("MAMG_POST_K");
  g_post_k = e ? std::atoi(e) : 1;   // 0: [P | AP]; 1: K (one block per slot); 2: K, split layout forced
  e = opt("MAMG_SELL_MIN_ROWS");
  g_sell_min_rows = e ? std::atoll(e) : (1 << 20);
  e = opt("MAMG_TAIL_NODES");
  g_tail_nodes = e ? std::atoll(e) : 0;
  g_tail_set = e != nullptr;
  e = opt("MAMG_TAIL_VL");
  g_tail_vl = e ? std::max(1, std::min(64, std::atoi(e))) : 4;
  e = opt("MAMG_MSELL_MIN_ROWS");
  g_msell_min_rows = e ? std::atoll(e) : ((int64_t)1 << 40);
  e = opt("MAMG_HALF");
  g_half = e ? std::atoi(e) != 0 : 1;
  e = opt("MAMG_HALF_BANDS");
  g_half_bands = e ? std::atoi(e) : 1;
  e = opt("MAMG_R_BANDS");
  g_r_bands = e ? std::atoi(e) : 1;
  e = opt("MAMG_K_SORT");
  g_k_sort = e ? std::atoi(e) : 1;
  e = opt("MAMG_FUSE_RBD");
  g_fuse_rbd = e ? std::atoi(e) : 2;
  e = opt("MAMG_K_COL16");
  g_k_c16 = e ? std::atoi(e) : 1;
}

// every block symmetric (bitwise): then 3 doubles per block carry it exactly
bool blocks_symmetric(const HBsr& B) {
  const int64_t nb = B.ptr[B.nr];
  int64_t bad = 0;
  for (int64_t k = 0; k < nb; ++k)
    bad |= std::memcmp(&B.val[4 * k + 1], &B.val[4 * k + 2], sizeof(double)) != 0;
  return bad == 0;
}
void pack_sym(const HBsr& B, std::vector<double>* v3) {
  const int64_t nb = B.ptr[B.nr];
  v3->resize(3 * nb);
  for (int64_t k = 0; k < nb; ++k) {
    (*v3)[2 * k] = B.val[4 * k];
    (*v3)[2 * k + 1] = B.val[4 * k + 3];
    (*v3)[2 * nb + k] = B.val[4 * k + 1];
  }
}

// ---------------------------------------------------------------------------
// device structures
// ---------------------------------------------------------------------------
struct DCsr {
  int64_t n = 0, m = 0, nnz = 0;
  int64_t* ptr = nullptr;
  int32_t* col = nullptr;
  double* val = nullptr;
  int lanes = 8;
};

struct DBsr {              // 2x2 blocks, node-major
  int64_t nr = 0, nc = 0, nb = 0;
  int64_t* ptr = nullptr;
  int32_t* col = nullptr;
  double* val = nullptr;   // 4 doubles per block, 3 if sym
  int lanes = 8;
  bool sym = false;        // symmetric-block format (every block has (0,1) == (1,0))
  // SELL-64 storage (sell == true): ptr unused; soff per slice, meta per row,
  // col / val hold nbs (>= nb, padded) slots
  bool sell = false;
  int split = 0;            // SELL general blocks as two 16-byte streams (1: two global streams,
                            // 2: split inside each slot row; sell2_kernel / msell_kernel SPL)
  int lpr = 1;              // SELL lanes per row: 1 sell2_kernel, > 1 msell_kernel
  int64_t nbs = 0;
  int64_t* soff = nullptr;
  int32_t* meta = nullptr;
  int32_t* perm = nullptr;  // SELL-C-sigma: row held by each slot (merged matrices)
  bool lsort = false;       // SELL rows sorted by length inside each slice: meta is per slot,
                            // length | (row - slice start) << 16 (sort_sell_slices)
  // SELL columns as 16-bit offsets from a per-slice base (level-0 K, round
  // 6: compress_sell_cols); col is kept for the layout code, the kernel reads
  // col16 + cbase
  uint16_t* col16 = nullptr;
  int32_t* cbase = nullptr;
  // half-symmetric ELL-64 (half == true, A symmetric bitwise): col / val hold
  // the upper part I <= J < nr, hwu slots per row; lptr holds,
  // per lower entry J < I, the slot of the mirror block (J, I) in the upper
  // part, hwl slots per row; ghost columns (>= nr, multi-GPU rank-local A)
  // in their own SELL-64 part (gsoff per slice, zero width where a slice has
  // none); meta = upper length | lower length << 8 | ghost length << 16
  bool half = false;
  int hwu = 0, hwl = 0;
  int64_t nlo = 0;          // lower entries (nb = upper + ghost entries + nlo)
  int32_t* lptr = nullptr;
  int64_t ngs = 0;          // ghost-part slots (0: no ghost part)
  int64_t* gsoff = nullptr;
  int32_t* gcol = nullptr;
  double* gval = nullptr;
  // band schedule of the half-symmetric kernel (full-range launches):
  // workgroup b processes 256-row block sched[b] (nullptr: row_block order)
  int32_t* sched = nullptr;
  int64_t nsched = 0;
  int64_t band_stride = 0;  // plane stride S in rows (0: no band schedule)
  // band schedule of one sub-range launch [sr0, sr1) (multi-GPU interior rows)
  int32_t* sched_r = nullptr;
  int64_t nsched_r = 0, sr0 = 0, sr1 = 0;
  // plane-band schedule of a lane-group BSR launch with rsched_vl lanes per
  // row (the level-0 restriction): workgroup b processes row block rsched[b]
  int32_t* rsched = nullptr;
  int64_t nrsched = 0;
  int rsched_vl = 0;
};

struct DLevel {
  int64_t n = 0;           // dofs
  bool coarsest = false;
  DCsr A, P, R, WB;        // CSR layout
  DBsr Ab, Pb, Rb;         // BSR2 layout
  DBsr PAb;                // BSR2 post fusion: merged [P | AP] rows (ptr: 2 nr + 1)
  DBsr KPb;                // BSR2 post fusion: K = P - W (A P), one operator (default)
  dv4* Wd = nullptr;       // BSR2 layout: 2x2 smoother block per node
  double* winv = nullptr;
  // SMOOTHER_POLY: the step smoothers w_k W, k = 1..m (BSR2: Wk; CSR: WBk
  // sharing WB's pattern, or winvk); empty for the Jacobi smoothers
  std::vector<dv4*> Wk;
  std::vector<DCsr> WBk;
  std::vector<double*> winvk;
  double* Ainv = nullptr;
  double *b = nullptr, *x = nullptr, *t = nullptr, *t2 = nullptr, *r = nullptr,
         *c = nullptr, *e = nullptr;
  // multicolour Gauss-Seidel (SMOOTHER_SGS / SMOOTHER_GS, BSR2 layout): A_l's
  // node rows permuted colour by colour (Gb, lane groups), the node of each
  // permuted row (gperm), the unscaled smoother-block inverses in that order
  // (Gd), colour c = permuted rows [gcs[c], gcs[c + 1])
  DBsr Gb;
  int32_t* gperm = nullptr;
  dv4* Gd = nullptr;
  std::vector<int64_t> gcs, gbk;     // colour row starts / block starts (+ end)
  // level-0 node-patch Schwarz (Schwarz_type PATCHES): A_0 as plain BSR2 in
  // node order (Sptr, Scol, Sval: the patch rows), the patch centres colour by
  // colour (pperm), colour c = patches [pcs[c], pcs[c + 1]), the packed upper
  // triangles of the patch inverses (pu, stride pus doubles per patch)
  int64_t* Sptr = nullptr;
  int32_t* Scol = nullptr;
  dv4* Sval = nullptr;
  int64_t Snb = 0;
  int32_t* pperm = nullptr;
  double* pu = nullptr;
  int64_t pus = 0;
  std::vector<int64_t> pcs;
  // level-0 seed-ring Schwarz (Schwarz_type RINGS): the blocks colour by
  // colour (colour c = blocks [rcs[c], rcs[c + 1])), block k's members as
  // node-interleaved dof indices 2 I + f at rmem[rmo[k] .. rmo[k + 1]), its
  // Gauss-Jordan inverse transposed (column-major d x d) at rinv + rio[k];
  // A_0's rows in Sptr / Scol / Sval; the rest's GS in Gb / gperm / Gd / gcs
  // (covered dofs masked out of Gd)
  int64_t* rmo = nullptr;
  int32_t* rmem = nullptr;
  int64_t* rio = nullptr;
  double* rinv = nullptr;
  std::vector<int64_t> rcs;
  int64_t rnm = 0;          // members of all blocks
  double rinv_n = 0.0;      // inverse entries of all blocks
  // coarse-grid correction scaling of the correction computed ON this level:
  // q = A_l e, partial sums of <b, e>, <q, e>
  double* q = nullptr;
  double* part2 = nullptr;
};

enum OpKind { OP_CSR = 0, OP_SCALE = 1, OP_GEMV = 2, OP_AXPY = 3, OP_BSR = 4, OP_BD = 5, OP_POST = 6, OP_ILV = 7,
              OP_GS = 8, OP_ZERO = 9, OP_DOT2 = 10, OP_CSCALE = 11, OP_PATCH = 12, OP_TAIL = 13, OP_RING = 14 };
// kernel classes (kernel_ms / class_bytes slots)
enum Cls {
  C_L0_RESID = 0,   // dominant: r = b - A0 x (once per apply)
  C_L0_SMOOTH = 1,  // post-smooth SpMV on A0 (fused Jacobi / block Jacobi)
  C_L0_WB = 2,      // level-0 smoother application outside an SpMV
  C_L0_R = 3,       // level-0 restriction
  C_L0_P = 4,       // level-0 prolongation
  C_COARSE = 5,     // all SpMV-class launches on levels >= 1
  C_DENSE = 6,      // coarsest dense solve
  C_MISC = 7,       // W-cycle / maxit corrections
  C_COMM = 8,       // multi-GPU: halo pack/unpack + RCCL exchanges
  NCLS = 8
};

struct Op {
  int kind = OP_CSR, epi = EPI_Y, cls = 0, tag = 1;
  const DCsr* M = nullptr;
  const DBsr* Mb = nullptr;
  int64_t n = 0;
  const double *x = nullptr, *y = nullptr, *b = nullptr, *w = nullptr;
  const dv4* W = nullptr;
  double* out = nullptr;
  int64_t xs = 0, bs = 0, os = 0;   // BSR2 field strides (0 = node-major)
  bool xfm = false;
  int remap = 0;                    // XCD-contiguous row order (restriction ops)
  int64_t r0 = 0, r1 = -1;          // row range [r0, r1) (half-symmetric ops, GS colours; r1 < 0: all rows)
  const int32_t* perm = nullptr;    // GS: node of each permuted row
  double* part = nullptr;           // DOT2 / CSCALE partial sums
  const struct DLevel* lev = nullptr;   // PATCH: the level's patch data
  const TOp* prog = nullptr;        // TAIL: the device op list (n ops)
  int tail_pl = -1;                 // TAIL: the program's LDS byte offset (-1: read from global memory)
  double bytes = 0.0;
};

inline int remap_of(const Op& o) { return o.remap; }

struct Graph {
  const double* r = nullptr;
  double* z = nullptr;
  hipGraphExec_t exec = nullptr;
  hipGraph_t graph = nullptr;
};

// one PCG iteration captured for a solution vector x and a history length
// (dev_pcg): reused by later solves into the same x (drivers, gamma sweeps)
struct PcgGraph {
  double* x = nullptr;
  int maxiter = 0;
  hipGraphExec_t exec = nullptr;
  hipGraph_t graph = nullptr;
  double* hist = nullptr;          // residuals[maxiter + 1], alphas[maxiter], betas[maxiter]
  hipEvent_t ev[2] = {nullptr, nullptr};
  void release() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
    for (hipEvent_t e : ev) if (e) (void)hipEventDestroy(e);
    if (hist) (void)raw_free(hist);
    *this = PcgGraph();
  }
};

}  // namespace

struct DeviceHandle {
  mamg_params p;
  int device = 0;
  bool bsr = false;
  std::vector<DLevel> L;
  std::vector<void*> allocs;
  char* arena = nullptr;           // pre-reserved HBM, bump-allocated (dev_prereserve)
  size_t arena_left = 0;
  char* arena0 = nullptr;          // the reservation's range [arena0, arena1)
  char* arena1 = nullptr;
  hipStream_t cap = nullptr;
  std::vector<Graph> graphs;
  std::vector<PcgGraph> pcgs;
  // coarse tail (tail_kernel): first level run by it (0 = off) and the
  // device op lists built so far, one per (b, x) entry of that level
  int tail_level = 0;
  std::vector<double> kregion_ms;  // select_k_region: K ms per candidate region, the one kept
  int kregion_best = -1;
  struct TailProg { const double* b; double* x; TOp* prog; int n; double bytes; int64_t lds; bool xl; int prog_lds; bool res; };
  mutable std::vector<TailProg> tails;
  double* hr = nullptr;            // host-apply staging (device)
  double* hz = nullptr;
  double *cr = nullptr, *cz = nullptr, *cd = nullptr, *cq = nullptr;  // PCG
  double* part = nullptr;
  double* dres = nullptr;
  double* hres = nullptr;          // pinned host scalar
  double apply_bytes = 0.0;
  double setup_ms[8] = {};         // GPU setup phase timings (dev_from_ghier)
  double layout_ms[4] = {};        // apply-layout phases: build, K region trials, re-homing, finish (LT_*)
  // every piece of work on the handle's scratch buffers (apply, host apply,
  // spmv, PCG, timing) waits for this event on its stream and re-records it
  // afterwards: work on one handle is serialized across streams
  hipEvent_t last = nullptr;
  ~DeviceHandle() {
    if (last) (void)hipEventDestroy(last);
    for (auto& g : graphs) {
      if (g.exec) (void)hipGraphExecDestroy(g.exec);
      if (g.graph) (void)hipGraphDestroy(g.graph);
    }
    for (auto& g : pcgs) g.release();
    for (auto& t : tails) (void)raw_free(t.prog);
    for (void* a : allocs) (void)raw_free(a);
    if (hres) (void)hipHostFree(hres);
    if (cap) (void)hipStreamDestroy(cap);
  }
};

namespace {

enum { LT_BUILD = 0, LT_KREGION = 1, LT_REHOME = 2, LT_FINISH = 3 };

// MAMG_POISON=1 (tests): every double array a handle or the layout builder
// allocates starts as NaN bytes instead of whatever the memory held, so a
// read of a value nothing wrote shows in the result (index arrays are left
// alone: a poisoned index would fault instead of showing)
template <class T>
void poison_doubles(T* p, size_t bytes) {
  if constexpr (std::is_same<T, double>::value) {
    const char* e = opt("MAMG_POISON");
    if (e && std::atoi(e) != 0) (void)dev_memset(p, 0xff, bytes);
  }
}

// free a handle-owned (hipMalloc) array replaced during the upload, behind
// its last reader on the null stream (dmem.h ordered_free)
inline void drained_free(void* p) { ordered_free(p); }

// wait for the layout builder's queued work (all of it on the null stream)
inline hipError_t null_sync() { return hipStreamSynchronize(nullptr); }

// device allocation owned by a handle (single-GPU or multi-GPU: both keep `allocs`)
template <class HT, class T>
int dalloc(HT* h, T** p, int64_t count, std::string* err) {
  *p = nullptr;
  if (count <= 0) return MAMG_OK;
  const size_t bytes = ((size_t)count * sizeof(T) + 4095) & ~(size_t)4095;
  if (h->arena && bytes <= h->arena_left) {
    *p = (T*)h->arena;
    h->arena += bytes;
    h->arena_left -= bytes;
    poison_doubles(*p, bytes);
    return MAMG_OK;
  }
  void* q = nullptr;
  // a very large long-lived array (the node patches' inverses: 63 GB at
  // nrefs=6) is placed after the idle setup cache is released, so it is not
  // laid out around the cached blocks (with them kept, the patch layout build
  // took 2.2-2.8 s instead of 0.68 s, BENCH_r05 / profiles/r05_bench_g.json)
  if ((size_t)count * sizeof(T) >= ((size_t)8 << 30)) tmp_trim();
  HIPCHK(dev_malloc(&q, (size_t)count * sizeof(T)));
  h->allocs.push_back(q);
  *p = (T*)q;
  poison_doubles(*p, (size_t)count * sizeof(T));
  return MAMG_OK;
}

// lanes per row: ~3 entries per lane (bench/spmv_micro.hip: 8 lanes best for
// the ~30 nnz CSR rows and the ~15 block BSR rows of the level-0 operator)
int pick_lanes(int64_t n, int64_t nnz) {
  const double avg = n ? (double)nnz / (double)n : 1.0;
  int l = 2;
  while (l < 64 && 3.0 * (2 * l) <= avg + 1e-9) l *= 2;
  return l;
}

int upload_csr(DeviceHandle* h, const CsrView& M, DCsr* D, int lanes, std::string* err) {
  D->n = M.n;
  D->m = M.m;
  D->nnz = M.nnz();
  D->lanes = lanes > 0 ? lanes : pick_lanes(M.n, D->nnz);
  int rc;
  if ((rc = dalloc(h, &D->ptr, M.n + 1, err))) return rc;
  if ((rc = dalloc(h, &D->col, std::max<int64_t>(D->nnz, 1), err))) return rc;
  if ((rc = dalloc(h, &D->val, std::max<int64_t>(D->nnz, 1), err))) return rc;
  HIPCHK(hipMemcpy(D->ptr, M.ptr, (M.n + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if (D->nnz) {
    HIPCHK(hipMemcpy(D->col, M.col, D->nnz * sizeof(int32_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(D->val, M.val, D->nnz * sizeof(double), hipMemcpyHostToDevice));
  }
  return MAMG_OK;
}

// a device CSR (GPU setup output) copied into the handle's memory
int adopt_csr(DeviceHandle* h, const DevMat& M, DCsr* D, int lanes, std::string* err) {
  D->n = M.n;
  D->m = M.m;
  D->nnz = M.nnz;
  D->lanes = lanes > 0 ? lanes : pick_lanes(M.n, D->nnz);
  int rc;
  if ((rc = dalloc(h, &D->ptr, M.n + 1, err))) return rc;
  if ((rc = dalloc(h, &D->col, std::max<int64_t>(D->nnz, 1), err))) return rc;
  if ((rc = dalloc(h, &D->val, std::max<int64_t>(D->nnz, 1), err))) return rc;
  HIPCHK(dev_copy(D->ptr, M.ptr, (M.n + 1) * sizeof(int64_t)));
  if (D->nnz) {
    HIPCHK(dev_copy(D->col, M.col, D->nnz * sizeof(int32_t)));
    HIPCHK(dev_copy(D->val, M.val, D->nnz * sizeof(double)));
  }
  return MAMG_OK;
}

// lanes per node row for 2x2 blocks: ~2 blocks per lane (VL = 8 for the
// ~15-block level-0 rows: 1.87 ms vs 2.00 ms at VL = 4, bench/spmv_micro.hip;
// round 3 at nrefs=6: 1/4, 1/2 and 2x these lanes on the coarse levels were
// 0.419-0.527 ms vs 0.421 ms, profiles/r03_ab_coarse_lanes.txt)
int pick_lanes_bsr(int64_t nr, int64_t nb) {
  const double avg = nr ? (double)nb / (double)nr : 1.0;
  int l = 2;
  while (l < 64 && 2.0 * (2 * l) <= 2.0 * avg) l *= 2;
  return l;
}

// SELL-64 copy of a BSR2 matrix (host packing: convert.cpp to_sell)
template <class HT>
int upload_sell(HT* h, const HBsr& B, DBsr* D, std::string* err) {
  HSell S;
  const bool merged = (int64_t)B.ptr.size() == 2 * B.nr + 1;
  int rc = to_sell(B, D->sym, SELL_C, merged ? SELL_SIGMA : 1, &S, err);
  if (rc) return rc;
  const int64_t ns = (int64_t)S.soff.size() - 1;
  const int per = D->sym ? 3 : 4;
  D->sell = true;
  D->nbs = S.nbs;
  if ((rc = dalloc(h, &D->soff, ns + 1, err))) return rc;
  if ((rc = dalloc(h, &D->meta, std::max<int64_t>(S.nr, 1), err))) return rc;
  if ((rc = dalloc(h, &D->col, std::max<int64_t>(S.nbs, 1), err))) return rc;
  if ((rc = dalloc(h, &D->val, std::max<int64_t>(per * S.nbs, 1), err))) return rc;
  HIPCHK(hipMemcpy(D->soff, S.soff.data(), (ns + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if (S.nr) HIPCHK(hipMemcpy(D->meta, S.meta.data(), S.nr * sizeof(int32_t), hipMemcpyHostToDevice));
  if (!S.perm.empty()) {
    if ((rc = dalloc(h, &D->perm, S.nr, err))) return rc;
    HIPCHK(hipMemcpy(D->perm, S.perm.data(), S.nr * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  if (S.nbs) {
    HIPCHK(hipMemcpy(D->col, S.col.data(), S.nbs * sizeof(int32_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(D->val, S.val.data(), per * S.nbs * sizeof(double), hipMemcpyHostToDevice));
  }
  return MAMG_OK;
}

// (also uploads a merged [P | AP] matrix: then B.ptr has 2 nr + 1 entries)
template <class HT>
int upload_bsr(HT* h, const HBsr& B, DBsr* D, int lanes, std::string* err,
               bool sym = false) {
  const int64_t np = (int64_t)B.ptr.size();
  D->nr = B.nr;
  D->nc = B.nc;
  D->nb = B.ptr[np - 1];
  D->lanes = lanes > 0 ? lanes : pick_lanes_bsr(B.nr, D->nb);
  int rc;
  // SELL-64 for many short rows (one lane per row needs >> 256 CUs x 64 rows)
  const bool merged_rows = np == 2 * B.nr + 1;
  if (B.nr >= g_sell_min_rows && D->nb <= g_sell_max_len * B.nr && !merged_rows) {
    D->sym = sym && np == B.nr + 1 && blocks_symmetric(B);
    return upload_sell(h, B, D, err);
  }
  if ((rc = dalloc(h, &D->ptr, np, err))) return rc;
  if ((rc = dalloc(h, &D->col, std::max<int64_t>(D->nb, 1), err))) return rc;
  D->sym = sym && np == B.nr + 1 && blocks_symmetric(B);
  const int per = D->sym ? 3 : 4;
  if ((rc = dalloc(h, &D->val, std::max<int64_t>(per * D->nb, 1), err))) return rc;
  HIPCHK(hipMemcpy(D->ptr, B.ptr.data(), np * sizeof(int64_t), hipMemcpyHostToDevice));
  if (D->nb) {
    HIPCHK(hipMemcpy(D->col, B.col.data(), D->nb * sizeof(int32_t), hipMemcpyHostToDevice));
    if (D->sym) {
      std::vector<double> v3;
      pack_sym(B, &v3);
      HIPCHK(hipMemcpy(D->val, v3.data(), D->nb * 3 * sizeof(double), hipMemcpyHostToDevice));
    } else {
      HIPCHK(hipMemcpy(D->val, B.val.data(), D->nb * 4 * sizeof(double), hipMemcpyHostToDevice));
    }
  }
  return MAMG_OK;
}

// ---------------------------------------------------------------------------
// Device-side layout construction: field-major CSR already in HBM (GPU setup
// output, or host CSR copied up) -> the BSR2 / symmetric / SELL-64 / merged
// [P | AP] apply layouts.  Same layouts as the host conversions in
// convert.cpp (to_bsr2, merge_bsr_rows, to_sell with sigma = 1, pack_sym);
// pure data movement, so the apply sees identical bits either way.
// ---------------------------------------------------------------------------
// node I's four sorted column segments (rowstage.h stage_segs): q = 2 f + g
// holds the entries of row f nr + I whose column lies in field g (node
// column = col - g nc)
template <bool FILL, int CAP = RS_CAP>
__global__ __launch_bounds__(64) void csr2bsr_kernel(int64_t nr, int64_t nc, const int64_t* __restrict__ ptr,
                                                     const int32_t* __restrict__ col,
                                                     const double* __restrict__ val, int64_t* bptr,
                                                     int32_t* __restrict__ bcol, dv4* __restrict__ bval) {
  __shared__ RowStageT<FILL, CAP> S;   // rowstage.h: the wave's rows staged through LDS
  const int64_t I0 = (int64_t)blockIdx.x * RS_NODES, I = I0 + threadIdx.x;
  RowView vw[2];
  stage_rows<FILL>(S, ptr, col, val, nr, I0, vw);
  if (I >= nr) return;
  Seg4 g;
  stage_segs(ptr, vw, nr, nc, I, g.k, g.e);
  g.init(vw, nc);
  int64_t o = FILL ? bptr[I] : 0;
  for (;;) {
    const int64_t J = g.next();
    if (J == INT64_MAX) break;
    dv4 v = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (g.c[q] == J) {
        if (FILL) v[q] = vw[q >> 1].val(g.k[q]);
        ++g.k[q];
        g.head(vw, nc, q);
      }
    if (FILL) {
      bval[o] = v;
      bcol[o] = (int32_t)J;
    }
    ++o;
  }
  if (!FILL) bptr[I + 1] = o;
}

// The fill pass with columns only in LDS (16 KB, ~10 waves per CU instead
// of 3 with the 48 KB column + value staging): each lane's merge writes, in
// place of every staged column, the entry's slot in the output (4 (o - o0) + q,
// o0 the workgroup's first block) and the zeros of its blocks' missing
// components; then the wave sweeps the value ranges with coalesced loads and
// stores each value into its slot.  Same blocks, same bits.  Ranges over
// CAP (not staged) merge from global memory as in csr2bsr_kernel.
template <int CAP>
__global__ __launch_bounds__(64) void csr2bsr_fill_kernel(int64_t nr, int64_t nc, const int64_t* __restrict__ ptr,
                                                          const int32_t* __restrict__ col,
                                                          const double* __restrict__ val, const int64_t* bptr,
                                                          int32_t* __restrict__ bcol, dv4* __restrict__ bval) {
  __shared__ RowStageT<false, CAP> S;   // columns, then each entry's slot
  const int64_t I0 = (int64_t)blockIdx.x * RS_NODES, I = I0 + threadIdx.x;
  RowView vw[2];
  stage_rows<false>(S, ptr, col, val, nr, I0, vw);
  const bool lds = vw[0].lds;      // uniform over the workgroup
  if (!lds) {                      // long ranges: values from global memory
    if (I >= nr) return;
    Seg4 g;
    stage_segs(ptr, vw, nr, nc, I, g.k, g.e);
    g.init(vw, nc);
    int64_t o = bptr[I];
    for (;;) {
      const int64_t J = g.next();
      if (J == INT64_MAX) break;
      dv4 v = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (g.c[q] == J) {
          v[q] = vw[q >> 1].val(g.k[q]);
          ++g.k[q];
          g.head(vw, nc, q);
        }
      bval[o] = v;
      bcol[o] = (int32_t)J;
      ++o;
    }
    return;
  }
  const int64_t o0 = bptr[I0];
  double* bv = reinterpret_cast<double*>(bval + o0);
  if (I < nr) {
    Seg4 g;
    stage_segs(ptr, vw, nr, nc, I, g.k, g.e);
    g.init(vw, nc);
    int64_t o = bptr[I];
    for (;;) {
      const int64_t J = g.next();
      if (J == INT64_MAX) break;
      const int32_t rel = (int32_t)(o - o0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (g.c[q] == J) {
          S.c[q >> 1][g.k[q] - vw[q >> 1].off] = 4 * rel + q;   // this entry's slot (its column was read)
          ++g.k[q];
          g.head(vw, nc, q);
        } else {
          bv[4 * rel + q] = 0.0;
        }
      }
      bcol[o] = (int32_t)J;
      ++o;
    }
  }
  __syncthreads();
  const int64_t I1 = I0 + RS_NODES < nr ? I0 + RS_NODES : nr;
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int64_t b = ptr[f * nr + I0], n = ptr[f * nr + I1] - b;
    scatter_staged(S.c[f], val, b, n, bv);
  }
}

// *bad = 1 when some block has a01 != a10 (bitwise).  Grid-stride over at most
// SYM_CHECK_BLOCKS workgroups, one atomic per workgroup: with one atomic per
// mismatching wave, a non-symmetric level-1 operator (25.8 M blocks, nearly
// all mismatching) serialised ~400 K atomics on one word (4.6 ms)
constexpr unsigned SYM_CHECK_BLOCKS = 16384;
__global__ __launch_bounds__(256) void sym_check_kernel(int64_t nb, const dv4* __restrict__ v, int* bad) {
  int d = 0;
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < nb; k += (int64_t)gridDim.x * 256)
    d |= __double_as_longlong(v[k].y) != __double_as_longlong(v[k].z);
  if (__syncthreads_or(d) && threadIdx.x == 0) atomicOr(bad, 1);
}

__global__ __launch_bounds__(256) void pack_sym_kernel(int64_t nb, const dv4* __restrict__ v,
                                                       double* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= nb) return;
  const dv4 a = v[k];
  out[2 * k] = a.x;
  out[2 * k + 1] = a.w;
  out[2 * nb + k] = a.y;
}

// merged [P | Q] row pointers: lengths at 2I+1, 2I+2 (scanned afterwards)
__global__ __launch_bounds__(256) void merge_len_kernel(int64_t nr, const int64_t* __restrict__ pp,
                                                        const int64_t* __restrict__ qp, int64_t* mptr) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nr) return;
  mptr[2 * I + 1] = pp[I + 1] - pp[I];
  mptr[2 * I + 2] = qp[I + 1] - qp[I];
  if (I == 0) mptr[0] = 0;
}

__global__ __launch_bounds__(256) void merge_fill_kernel(int64_t nr, const int64_t* __restrict__ pp,
                                                         const int32_t* __restrict__ pc, const dv4* __restrict__ pv,
                                                         const int64_t* __restrict__ qp, const int32_t* __restrict__ qc,
                                                         const dv4* __restrict__ qv, const int64_t* __restrict__ mptr,
                                                         int32_t* __restrict__ mc, dv4* __restrict__ mv) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nr) return;
  int64_t d = mptr[2 * I];
  for (int64_t k = pp[I]; k < pp[I + 1]; ++k, ++d) { mc[d] = pc[k]; mv[d] = pv[k]; }
  for (int64_t k = qp[I]; k < qp[I + 1]; ++k, ++d) { mc[d] = qc[k]; mv[d] = qv[k]; }
}

// K = P - W_I (A P) row by row on the union of P's and AP's block patterns
// (the fused post-smoothing operator: x1 + P e + W (r1 - AP e) = x1 + W r1 + K e);
// a block absent from one operand contributes exact zeros
template <bool FILL>
__global__ __launch_bounds__(256) void kmerge_kernel(int64_t nr, const int64_t* __restrict__ pp,
                                                     const int32_t* __restrict__ pc, const dv4* __restrict__ pv,
                                                     const int64_t* __restrict__ qp, const int32_t* __restrict__ qc,
                                                     const dv4* __restrict__ qv, const dv4* __restrict__ W,
                                                     int64_t* kp, int32_t* __restrict__ kc, dv4* __restrict__ kv) {
#pragma clang fp contract(off)   // the host's kmerge_rows (dist.cpp, -ffp-contract=off) bit for bit
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nr) return;
  int64_t a = pp[I], ae = pp[I + 1], b = qp[I], be = qp[I + 1];
  int64_t o = FILL ? kp[I] : 0;
  const dv4 w = FILL ? W[I] : dv4{0.0, 0.0, 0.0, 0.0};
  const dv4 zero = {0.0, 0.0, 0.0, 0.0};
  while (a < ae || b < be) {
    const int32_t ja = a < ae ? pc[a] : INT32_MAX, jb = b < be ? qc[b] : INT32_MAX;
    const int32_t j = min(ja, jb);
    if (FILL) {
      const dv4 p = ja == j ? pv[a] : zero, q = jb == j ? qv[b] : zero;
      dv4 k;   // blocks (0,0) (0,1) (1,0) (1,1) = x y z w;  (W q)_ab = W_a0 q_0b + W_a1 q_1b
      k.x = p.x - (w.x * q.x + w.y * q.z);
      k.y = p.y - (w.x * q.y + w.y * q.w);
      k.z = p.z - (w.z * q.x + w.w * q.z);
      k.w = p.w - (w.z * q.y + w.w * q.w);
      kc[o] = j;
      kv[o] = k;
    }
    if (ja == j) ++a;
    if (jb == j) ++b;
    ++o;
  }
  if (!FILL) kp[I + 1] = o;
}

// SELL-64: slice widths and per-row meta (length | first-part length << 16)
__global__ __launch_bounds__(256) void sell_meta_kernel(int64_t nr, const int64_t* __restrict__ bptr, int merged,
                                                        int32_t* __restrict__ meta, int64_t* __restrict__ soff,
                                                        int* bad) {
  const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t ns = (nr + SELL_C - 1) / SELL_C;
  if (s >= ns) return;
  int64_t w = 0;
  for (int64_t I = s * SELL_C; I < min(nr, (s + 1) * SELL_C); ++I) {
    const int64_t a = merged ? bptr[2 * I] : bptr[I];
    const int64_t m = merged ? bptr[2 * I + 1] : a;
    const int64_t e = merged ? bptr[2 * I + 2] : bptr[I + 1];
    if (e - a >= 0xffff) { atomicOr(bad, 1); continue; }
    meta[I] = (int32_t)((e - a) | ((m - a) << 16));
    w = max(w, e - a);
  }
  soff[s + 1] = (int64_t)SELL_C * w;
  if (s == 0) soff[0] = 0;
}

__global__ __launch_bounds__(256) void sell_fill_kernel(int64_t nr, const int64_t* __restrict__ bptr, int merged,
                                                        const int32_t* __restrict__ bcol, const dv4* __restrict__ bval,
                                                        const int64_t* __restrict__ soff, int64_t nbs, int sym,
                                                        int32_t* __restrict__ scol, double* __restrict__ sval) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nr) return;
  const int64_t a = merged ? bptr[2 * I] : bptr[I];
  const int64_t e = merged ? bptr[2 * I + 2] : bptr[I + 1];
  int64_t kk = soff[I / SELL_C] + (I % SELL_C);
  for (int64_t k = a; k < e; ++k, kk += SELL_C) {
    scol[kk] = bcol[k];
    const dv4 v = bval[k];
    if (sym) {
      sval[2 * kk] = v.x;
      sval[2 * kk + 1] = v.w;
      sval[2 * nbs + kk] = v.y;
    } else {
      reinterpret_cast<dv4*>(sval)[kk] = v;
    }
  }
}

// SELL-64 rows sorted by length inside each slice (DBsr::lsort): one 64-lane
// workgroup per slice; lane i's rank = rows longer than row i + equal rows
// before it (stable, longest first).  nmeta[slot] = length | (row offset << 16),
// src[slot] = the row offset the slot takes its blocks from.
__global__ __launch_bounds__(64) void sell_sort_kernel(int64_t nr, const int32_t* __restrict__ meta,
                                                      int32_t* __restrict__ nmeta, int32_t* __restrict__ src) {
  __shared__ int len[SELL_C];
  const int64_t r0 = (int64_t)blockIdx.x * SELL_C;
  const int i = threadIdx.x;
  const int cnt = (int)min((int64_t)SELL_C, nr - r0);
  const int li = i < cnt ? meta[r0 + i] & 0xffff : -1;
  len[i] = li;
  __syncthreads();
  if (i >= cnt) return;
  int rank = 0;
  for (int j = 0; j < cnt; ++j) rank += (len[j] > li) || (len[j] == li && j < i);
  nmeta[r0 + rank] = li | (i << 16);
  src[r0 + rank] = i;
}

// the slot arrays re-ordered to the sorted rows: slot p of slice s takes the
// blocks of slot src[p] (width = the slice's, so every block moves whole)
__global__ __launch_bounds__(64) void sell_permute_kernel(int64_t nr, const int64_t* __restrict__ soff,
                                                         const int32_t* __restrict__ src, int64_t nbs, int per,
                                                         const int32_t* __restrict__ col, const double* __restrict__ val,
                                                         int32_t* __restrict__ ncol, double* __restrict__ nval) {
  const int64_t s = blockIdx.x, r0 = s * SELL_C;
  const int p = threadIdx.x;
  if (r0 + p >= nr) return;
  const int64_t w = (soff[s + 1] - soff[s]) / SELL_C;
  const int64_t d0 = soff[s] + p, s0 = soff[s] + src[r0 + p];
  for (int64_t j = 0; j < w; ++j) {
    const int64_t d = d0 + SELL_C * j, o = s0 + SELL_C * j;
    ncol[d] = col[o];
    if (per == 4) {
      reinterpret_cast<dv4*>(nval)[d] = reinterpret_cast<const dv4*>(val)[o];
    } else {
      reinterpret_cast<dv2*>(nval)[d] = reinterpret_cast<const dv2*>(val)[o];
      nval[2 * nbs + d] = val[2 * nbs + o];
    }
  }
}

// half-symmetric ELL-64: per-row lower / upper / ghost counts (meta),
// widths (max), lower-entry total.  Grid-stride over at most HALF_META_BLOCKS
// workgroups, reduced in the workgroup, one atomic per counter per workgroup:
// three one-word atomics per wave serialised on their words (6.1 ms at A_0)
constexpr unsigned HALF_META_BLOCKS = 4096;
__global__ __launch_bounds__(256) void half_meta_kernel(int64_t nr, const int64_t* __restrict__ bptr,
                                                        const int32_t* __restrict__ bcol,
                                                        int32_t* __restrict__ meta, int* wmax,
                                                        unsigned long long* nlo) {
  unsigned long long snl = 0;
  int mu = 0, ml = 0, bad = 0;
  for (int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x; I < nr; I += (int64_t)gridDim.x * 256) {
    const int64_t a = bptr[I], e = bptr[I + 1];
    int64_t lo = a, hi = e;
    while (lo < hi) {            // first column >= I
      const int64_t mid = (lo + hi) >> 1;
      if (bcol[mid] < I) lo = mid + 1; else hi = mid;
    }
    const int64_t nl = lo - a;
    hi = e;
    while (lo < hi) {            // first column >= nr (ghosts)
      const int64_t mid = (lo + hi) >> 1;
      if (bcol[mid] < nr) lo = mid + 1; else hi = mid;
    }
    const int64_t ng = e - lo, nu = e - a - nl - ng;
    if (nu > 0xff || nl > 0xff || ng > 0x7fff) { bad = 1; continue; }
    snl += (unsigned long long)nl;
    meta[I] = (int32_t)(nu | (nl << 8) | (ng << 16));
    mu = max(mu, (int)nu);
    ml = max(ml, (int)nl);
  }
  for (int o = 32; o > 0; o >>= 1) {
    snl += __shfl_xor(snl, o);
    mu = max(mu, __shfl_xor(mu, o));
    ml = max(ml, __shfl_xor(ml, o));
    bad |= __shfl_xor(bad, o);
  }
  __shared__ unsigned long long ws[4];
  __shared__ int wu[4], wl[4], wb[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { ws[w] = snl; wu[w] = mu; wl[w] = ml; wb[w] = bad; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; ++k) {
      snl += ws[k];
      mu = max(mu, wu[k]);
      ml = max(ml, wl[k]);
      bad |= wb[k];
    }
    if (snl) atomicAdd(nlo, snl);
    if (mu) atomicMax(wmax, mu);
    if (ml) atomicMax(wmax + 1, ml);
    if (bad) atomicOr(wmax + 2, 1);
  }
}

// ghost-part slice widths (slot counts, scanned into gsoff afterwards)
__global__ __launch_bounds__(256) void half_gwidth_kernel(int64_t nr, const int32_t* __restrict__ meta,
                                                          int64_t* __restrict__ gsoff) {
  const int64_t sl = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t ns = (nr + SELL_C - 1) / SELL_C;
  if (sl >= ns) return;
  int w = 0;
  for (int64_t I = sl * SELL_C; I < min(nr, (sl + 1) * SELL_C); ++I) w = max(w, meta[I] >> 16);
  gsoff[sl + 1] = (int64_t)SELL_C * w;
  if (sl == 0) gsoff[0] = 0;
}

// upper blocks into their ELL slots, ghost blocks into the ghost SELL part
// (symmetric-block packing); every lower block (I, J) must have a
// bitwise-equal mirror (J, I), whose upper slot it records
__global__ __launch_bounds__(256) void half_fill_kernel(int64_t nr, const int64_t* __restrict__ bptr,
                                                        const int32_t* __restrict__ bcol, const dv4* __restrict__ bval,
                                                        const int32_t* __restrict__ meta, int hwu, int hwl, int64_t nbs,
                                                        int32_t* __restrict__ ucol, double* __restrict__ uval,
                                                        int32_t* __restrict__ lptr, const int64_t* __restrict__ gsoff,
                                                        int64_t ngs, int32_t* __restrict__ gcol,
                                                        double* __restrict__ gval, int* bad, int check_only) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nr) return;
  const int mI = meta[I];
  const int64_t a = bptr[I], e = bptr[I + 1], nl = (mI >> 8) & 0xff, ng = mI >> 16;
  const int64_t ubase = (I >> 6) * (int64_t)(64 * hwu) + (I & 63);
  for (int64_t k = a + nl, j = 0; k < e - ng && !check_only; ++k, ++j) {
    const int64_t kk = ubase + 64 * j;
    const dv4 v = bval[k];
    ucol[kk] = bcol[k];
    uval[2 * kk] = v.x;
    uval[2 * kk + 1] = v.w;
    uval[2 * nbs + kk] = v.y;
  }
  if (ng && !check_only) {
    const int64_t gbase = gsoff[I >> 6] + (I & 63);
    for (int64_t k = e - ng, j = 0; k < e; ++k, ++j) {
      const int64_t kk = gbase + 64 * j;
      const dv4 v = bval[k];
      gcol[kk] = bcol[k];
      gval[2 * kk] = v.x;
      gval[2 * kk + 1] = v.w;
      gval[2 * ngs + kk] = v.y;
    }
  }
  const int64_t lbase = (I >> 6) * (int64_t)(64 * hwl) + (I & 63);
  for (int64_t k = a, j = 0; k < a + nl; ++k, ++j) {
    const int64_t J = bcol[k];
    const int mJ = meta[J];
    const int64_t uJ = bptr[J] + ((mJ >> 8) & 0xff), eJ = uJ + (mJ & 0xff);
    int64_t lo = uJ, hi = eJ;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (bcol[mid] < I) lo = mid + 1; else hi = mid;
    }
    const dv4 v = bval[k];
    bool ok = lo < eJ && bcol[lo] == I;
    if (ok) {
      const dv4 t = bval[lo];
      ok = __double_as_longlong(v.x) == __double_as_longlong(t.x) &&
           __double_as_longlong(v.y) == __double_as_longlong(t.z) &&
           __double_as_longlong(v.z) == __double_as_longlong(t.y) &&
           __double_as_longlong(v.w) == __double_as_longlong(t.w);
    }
    if (!ok) { atomicOr(bad, 1); return; }
    if (check_only) continue;
    const int64_t jj = lo - uJ;
    lptr[lbase + 64 * j] = (int32_t)((J >> 6) * (int64_t)(64 * hwu) + 64 * jj + (J & 63));
  }
}

// coarsest inverse, dof order -> node-interleaved order
__global__ __launch_bounds__(256) void permute_dense_kernel(int64_t n, const double* __restrict__ in,
                                                            double* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * n) return;
  const int64_t i = t / n, j = t % n, nv = n / 2;
  out[(2 * (i % nv) + i / nv) * n + (2 * (j % nv) + j / nv)] = in[t];
}

// raw device BSR2 (4 doubles per block); merged: ptr has 2 nr + 1 entries
struct TBsr {
  int64_t nr = 0, nc = 0, nb = 0;
  bool merged = false;
  int64_t* ptr = nullptr;
  int32_t* col = nullptr;
  dv4* val = nullptr;
};

// scoped temporaries of the layout builder, null-stream ordered (dmem.h):
// the layout kernels that read them are queued on the null stream, and a
// block handed out again is used only by work queued behind them
struct TmpPool {
  std::vector<void*> v;
  ~TmpPool() {
    for (void* p : v) tmp_free(p);
  }
  template <class T>
  int alloc(T** p, int64_t count, std::string* err) {
    void* q = nullptr;
    HIPCHK(tmp_malloc(&q, (size_t)std::max<int64_t>(count, 1) * sizeof(T)));
    v.push_back(q);
    *p = (T*)q;
    poison_doubles(*p, (size_t)std::max<int64_t>(count, 1) * sizeof(T));
    return MAMG_OK;
  }
  void release(void* p) {
    for (auto& q : v)
      if (q == p) {
        tmp_free(q);
        q = nullptr;
      }
  }
};

int dev_csr_to_bsr(TmpPool* T, const DevMat& M, int64_t nr, int64_t nc, TBsr* B, std::string* err) {
  int rc;
  B->nr = nr; B->nc = nc; B->merged = false;
  if ((rc = T->alloc(&B->ptr, nr + 1, err))) return rc;
  HIPCHK(dev_memset(B->ptr, 0, sizeof(int64_t)));
  // rows whose wave ranges average over RS_CAP (the coarse Galerkin products;
  // A_0 averages ~1900) stage through the 64 KB column-only RS_CAP_LONG
  // variant: 2 waves per CU, but coalesced (level 1: 14.9 -> 12.2 ms)
  const unsigned g = (unsigned)((nr + RS_NODES - 1) / RS_NODES);
  const bool lng = nr && (double)M.nnz / (double)(2 * nr) * RS_NODES > RS_CAP;
  if (nr && lng) csr2bsr_kernel<false, RS_CAP_LONG><<<g, RS_NODES>>>(nr, nc, M.ptr, M.col, M.val, B->ptr, nullptr, nullptr);
  else if (nr) csr2bsr_kernel<false><<<g, RS_NODES>>>(nr, nc, M.ptr, M.col, M.val, B->ptr, nullptr, nullptr);
  HIPCHK(hipGetLastError());
  if ((rc = dscan_incl_i64(B->ptr, B->ptr, nr + 1, nullptr, err))) return rc;
  HIPCHK(hipMemcpy(&B->nb, B->ptr + nr, sizeof(int64_t), hipMemcpyDeviceToHost));
  if ((rc = T->alloc(&B->col, B->nb, err))) return rc;
  if ((rc = T->alloc(&B->val, B->nb, err))) return rc;
  // MAMG_CSR2BSR_FILL=0: the column + value staged fill (csr2bsr_kernel<true>; tests, A/B)
  const char* fe = opt("MAMG_CSR2BSR_FILL");
  const bool f2 = fe ? std::atoi(fe) != 0 : true;
  if (nr && f2 && lng)
    csr2bsr_fill_kernel<RS_CAP_LONG><<<g, RS_NODES>>>(nr, nc, M.ptr, M.col, M.val, B->ptr, B->col, B->val);
  else if (nr && f2)
    csr2bsr_fill_kernel<RS_CAP><<<g, RS_NODES>>>(nr, nc, M.ptr, M.col, M.val, B->ptr, B->col, B->val);
  else if (nr)
    csr2bsr_kernel<true><<<g, RS_NODES>>>(nr, nc, M.ptr, M.col, M.val, B->ptr, B->col, B->val);
  HIPCHK(hipGetLastError());
  return MAMG_OK;
}

int dev_merge_rows(TmpPool* T, const TBsr& P, const TBsr& Q, TBsr* M, std::string* err) {
  int rc;
  const int64_t nr = P.nr;
  M->nr = nr; M->nc = P.nc; M->merged = true;
  if ((rc = T->alloc(&M->ptr, 2 * nr + 1, err))) return rc;
  if (nr) merge_len_kernel<<<nblocks(nr), 256>>>(nr, P.ptr, Q.ptr, M->ptr);
  HIPCHK(hipGetLastError());
  if ((rc = dscan_incl_i64(M->ptr, M->ptr, 2 * nr + 1, nullptr, err))) return rc;
  M->nb = P.nb + Q.nb;
  if ((rc = T->alloc(&M->col, M->nb, err))) return rc;
  if ((rc = T->alloc(&M->val, M->nb, err))) return rc;
  if (nr) merge_fill_kernel<<<nblocks(nr), 256>>>(nr, P.ptr, P.col, P.val, Q.ptr, Q.col, Q.val, M->ptr, M->col, M->val);
  HIPCHK(hipGetLastError());
  return MAMG_OK;
}

int dev_kmerge(TmpPool* T, const TBsr& P, const TBsr& Q, const double* W, TBsr* K, std::string* err) {
  int rc;
  const int64_t nr = P.nr;
  K->nr = nr; K->nc = P.nc; K->merged = false;
  if ((rc = T->alloc(&K->ptr, nr + 1, err))) return rc;
  HIPCHK(dev_memset(K->ptr, 0, sizeof(int64_t)));
  const dv4* Wv = reinterpret_cast<const dv4*>(W);
  if (nr) kmerge_kernel<false><<<nblocks(nr), 256>>>(nr, P.ptr, P.col, P.val, Q.ptr, Q.col, Q.val, Wv, K->ptr,
                                                      nullptr, nullptr);
  HIPCHK(hipGetLastError());
  if ((rc = dscan_incl_i64(K->ptr, K->ptr, nr + 1, nullptr, err))) return rc;
  HIPCHK(hipMemcpy(&K->nb, K->ptr + nr, sizeof(int64_t), hipMemcpyDeviceToHost));
  if ((rc = T->alloc(&K->col, K->nb, err))) return rc;
  if ((rc = T->alloc(&K->val, K->nb, err))) return rc;
  if (nr) kmerge_kernel<true><<<nblocks(nr), 256>>>(nr, P.ptr, P.col, P.val, Q.ptr, Q.col, Q.val, Wv, K->ptr,
                                                     K->col, K->val);
  HIPCHK(hipGetLastError());
  return MAMG_OK;
}

// the schedule of G 256-row blocks for plane stride S (empty: keep row order)
std::vector<int32_t> band_sched(int64_t G, int64_t S, int nsub) {
  std::vector<int32_t> sched;
  const int64_t Pb = std::max<int64_t>(1, (S + 128) / 256), nb = 8 * (int64_t)nsub;
  if (nsub <= 0 || G < 64 || Pb < 4 * nb) return sched;
  std::vector<std::vector<int32_t>> L(8);
  for (int x = 0; x < 8; ++x)
    for (int sb = 0; sb < nsub; ++sb) {
      const int64_t band = (int64_t)x * nsub + sb, c0 = band * Pb / nb, c1 = (band + 1) * Pb / nb;
      for (int64_t p0 = 0; p0 < G; p0 += Pb)
        for (int64_t c = c0; c < c1 && p0 + c < G; ++c) L[x].push_back((int32_t)(p0 + c));
    }
  // balance to the round-robin dispatch: XCD x runs ceil / floor(G / 8)
  // workgroups; surplus tails move to the short lists
  std::vector<int32_t> spill;
  for (int x = 0; x < 8; ++x) {
    const size_t want = (size_t)(G / 8 + (x < G % 8 ? 1 : 0));
    while (L[x].size() > want) { spill.push_back(L[x].back()); L[x].pop_back(); }
  }
  for (int x = 0; x < 8; ++x) {
    const size_t want = (size_t)(G / 8 + (x < G % 8 ? 1 : 0));
    while (L[x].size() < want) { L[x].push_back(spill.back()); spill.pop_back(); }
  }
  sched.resize(G);
  std::vector<char> seen(G, 0);
  for (int64_t b = 0; b < G; ++b) {
    sched[b] = L[b % 8][b / 8];
    if (sched[b] < 0 || sched[b] >= G || seen[sched[b]]++) return std::vector<int32_t>();
  }
  return sched;
}

template <class HT>
int upload_sched(HT* h, const std::vector<int32_t>& sched, int32_t** d, int64_t* n, std::string* err) {
  int rc;
  if ((rc = dalloc(h, d, (int64_t)sched.size(), err))) return rc;
  HIPCHK(hipMemcpy(*d, sched.data(), sched.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  *n = (int64_t)sched.size();
  return MAMG_OK;
}

// Band schedule for the half-symmetric kernel.  A lower block (I, J < I) is
// re-read from row J's upper part; with the rows of a structured 3-D mesh in
// lexicographic order the farthest mirror sits one plane (stride S rows)
// back.  Row order alone puts a whole plane (~16 MB at n = 256) between the
// two reads, more than an XCD's 4 MB L2.  The schedule cuts each plane of
// 256-row blocks into 8 x nsub bands, gives XCD x (workgroups b = x mod 8)
// the bands x nsub .. x nsub + nsub - 1 and walks each band plane by plane,
// so the mirror was streamed one band (S / (8 nsub) rows) earlier on the same
// XCD.  S = the median, over sampled rows, of the distance to the row's first
// (smallest) column.  The schedule only permutes which workgroup computes
// which rows: every row is still summed by one lane in its own order, so the
// result is bitwise that of any other order.  Unstructured or narrow-band
// matrices (< 4 blocks per band) keep the row_block order.
template <class HT>
int build_band_sched(HT* h, const TBsr& B, DBsr* D, std::string* err) {
  const int64_t nr = B.nr, G = (nr + 255) / 256;
  if (g_half_bands <= 0 || G < 64) return MAMG_OK;
  const int ns = 257;
  std::vector<int64_t> off;
  for (int i = 0; i < ns; ++i) {
    const int64_t I = nr / 4 + (nr / 2) * i / ns;
    int64_t p = 0;
    int32_t c = 0;
    HIPCHK(hipMemcpy(&p, B.ptr + I, sizeof(int64_t), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&c, B.col + p, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (c < I) off.push_back(I - c);
  }
  if (off.size() < ns / 2) return MAMG_OK;
  std::nth_element(off.begin(), off.begin() + off.size() / 2, off.end());
  const std::vector<int32_t> sched = band_sched(G, off[off.size() / 2], g_half_bands);
  if (sched.empty()) return MAMG_OK;
  D->band_stride = off[off.size() / 2];
  return upload_sched(h, sched, &D->sched, &D->nsched, err);
}

// the same for the launch over rows [r0, r1) only (block b covers rows
// r0 + 256 b ..): the multi-GPU interior run
template <class HT>
int build_band_sched_range(HT* h, DBsr* D, int64_t r0, int64_t r1, std::string* err) {
  if (!D->half || D->band_stride <= 0 || r1 <= r0) return MAMG_OK;
  const std::vector<int32_t> sched = band_sched((r1 - r0 + 255) / 256, D->band_stride, g_half_bands);
  if (sched.empty()) return MAMG_OK;
  D->sr0 = r0;
  D->sr1 = r1;
  return upload_sched(h, sched, &D->sched_r, &D->nsched_r, err);
}

// first column of the first non-empty row of each group of rpw rows (-1: none)
__global__ void wg_first_col_kernel(int64_t G, int rpw, int64_t nr, const int64_t* __restrict__ ptr,
                                    const int32_t* __restrict__ col, int32_t* __restrict__ out) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= G) return;
  int32_t c = -1;
  for (int64_t i = b * rpw; i < nr && i < (b + 1) * rpw; ++i)
    if (ptr[i] < ptr[i + 1]) { c = col[ptr[i]]; break; }
  out[b] = c;
}

// Plane-band schedule of the level-0 restriction R_0 (coarse rows, fine
// columns).  A coarse row gathers r_1 over its smoothed aggregate, ~5 fine
// planes deep; coarse rows come in aggregate order, i.e. coarse plane after
// coarse plane, so a fine plane is gathered again by the next coarse plane's
// rows -- one coarse plane of R_0 (~30 MB at n = 256) later, long gone from
// an XCD's 4 MB L2 when each XCD walks whole planes.  Here a workgroup's key
// is the in-plane position (first column mod the fine plane stride Sf) of its
// first row: the plane is cut into 8 nsub bands, XCD x (workgroups b = x mod
// 8) takes the bands x nsub .. x nsub + nsub - 1 and walks each through all
// planes, so the re-gather is one band-plane of R_0 later and still in L2.
// Only which workgroup computes which rows changes: results are bitwise.
std::vector<int32_t> rest_band_sched(const std::vector<int32_t>& c0, int64_t Sf, int nsub) {
  std::vector<int32_t> sched;
  const int64_t G = (int64_t)c0.size(), nb = 8 * (int64_t)nsub;
  if (nsub <= 0 || Sf <= 0 || G < 64 * nb) return sched;
  std::vector<std::vector<int32_t>> L(8);
  std::vector<std::vector<int32_t>> band(nb);
  int64_t last = 0;
  for (int64_t b = 0; b < G; ++b) {
    const int64_t c = c0[b] >= 0 ? c0[b] : last;
    last = c;
    band[std::min<int64_t>(nb - 1, (c % Sf) * nb / Sf)].push_back((int32_t)b);
  }
  for (int64_t k = 0; k < nb; ++k) L[k / nsub].insert(L[k / nsub].end(), band[k].begin(), band[k].end());
  std::vector<int32_t> spill;   // balance to the round-robin dispatch, as band_sched
  for (int x = 0; x < 8; ++x) {
    const size_t want = (size_t)(G / 8 + (x < G % 8 ? 1 : 0));
    while (L[x].size() > want) { spill.push_back(L[x].back()); L[x].pop_back(); }
  }
  for (int x = 0; x < 8; ++x) {
    const size_t want = (size_t)(G / 8 + (x < G % 8 ? 1 : 0));
    while (L[x].size() < want && !spill.empty()) { L[x].push_back(spill.back()); spill.pop_back(); }
  }
  sched.resize(G);
  std::vector<char> seen(G, 0);
  for (int64_t b = 0; b < G; ++b) {
    if ((size_t)(b / 8) >= L[b % 8].size()) return std::vector<int32_t>();
    sched[b] = L[b % 8][b / 8];
    if (sched[b] < 0 || sched[b] >= G || seen[sched[b]]++) return std::vector<int32_t>();
  }
  return sched;
}

// the schedule for D (a lane-group BSR, not SELL / merged) given the fine
// plane stride Sf of its columns
template <class HT>
int build_rest_sched(HT* h, TmpPool* T, DBsr* D, int64_t Sf, std::string* err) {
  if (g_r_bands <= 0 || Sf <= 0 || D->sell || D->half || !D->ptr || D->lanes <= 0) return MAMG_OK;
  const int rpw = 256 / D->lanes;
  const int64_t G = (D->nr * (int64_t)D->lanes + 255) / 256;
  if (G < 64 * 8 * (int64_t)g_r_bands || G >= ((int64_t)1 << 31)) return MAMG_OK;
  int rc;
  int32_t* c0 = nullptr;
  if ((rc = T->alloc(&c0, G, err))) return rc;
  wg_first_col_kernel<<<nblocks(G), 256>>>(G, rpw, D->nr, D->ptr, D->col, c0);
  HIPCHK(hipGetLastError());
  std::vector<int32_t> hc(G);
  HIPCHK(hipMemcpy(hc.data(), c0, G * sizeof(int32_t), hipMemcpyDeviceToHost));
  T->release(c0);
  const std::vector<int32_t> sched = rest_band_sched(hc, Sf, g_r_bands);
  if (sched.empty()) return MAMG_OK;
  if ((rc = upload_sched(h, sched, &D->rsched, &D->nrsched, err))) return rc;
  D->rsched_vl = D->lanes;
  return MAMG_OK;
}

// half-symmetric ELL-64 for a symmetric-block A whose owned part (columns
// < nr) is symmetric bitwise; columns >= nr (ghosts of a rank-local A) go to
// the ghost part (hsell2_kernel).  Returns MAMG_OK with D->half set, or
// MAMG_OK with D->half false when a mirror is missing or differs, a row part
// is too long, or the ELL padding would exceed ~30 % (the caller then builds
// SELL-64); temporaries of a rejected attempt are freed with the pool.
template <class HT>
int try_half(HT* h, TmpPool* T, const TBsr& B, DBsr* D, std::string* err) {
  int rc;
  const int64_t nr = B.nr, ns = (nr + SELL_C - 1) / SELL_C;
  int* wm = nullptr;   // [0] max upper, [1] max lower, [2] part too long, [3] not symmetric
  int32_t* meta = nullptr;
  unsigned long long* nlod = nullptr;
  int64_t* gsoff = nullptr;
  if ((rc = T->alloc(&wm, 4, err))) return rc;
  if ((rc = T->alloc(&meta, nr, err))) return rc;
  if ((rc = T->alloc(&nlod, 1, err))) return rc;
  if ((rc = T->alloc(&gsoff, ns + 1, err))) return rc;
  HIPCHK(dev_memset(wm, 0, 4 * sizeof(int)));
  HIPCHK(dev_memset(nlod, 0, sizeof(unsigned long long)));
  half_meta_kernel<<<std::min(nblocks(nr), HALF_META_BLOCKS), 256>>>(nr, B.ptr, B.col, meta, wm, nlod);
  HIPCHK(hipGetLastError());
  int hw[4] = {0, 0, 0, 0};
  unsigned long long nloh = 0;
  HIPCHK(hipMemcpy(hw, wm, 4 * sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(&nloh, nlod, sizeof(nloh), hipMemcpyDeviceToHost));
  if (hw[2]) return MAMG_OK;
  half_gwidth_kernel<<<nblocks(ns), 256>>>(nr, meta, gsoff);
  HIPCHK(hipGetLastError());
  if ((rc = dscan_incl_i64(gsoff, gsoff, ns + 1, nullptr, err))) return rc;
  int64_t ngs = 0;
  HIPCHK(hipMemcpy(&ngs, gsoff + ns, sizeof(int64_t), hipMemcpyDeviceToHost));
  const int64_t nlo = (int64_t)nloh;
  const int64_t su = 64 * ns * (int64_t)hw[0], sl = 64 * ns * (int64_t)hw[1];
  const int64_t nup = B.nb - nlo;   // upper + ghost entries
  if (su >= (int64_t)1 << 31 || (double)(su + ngs) > 1.3 * nup + 4096 || (double)sl > 1.3 * nlo + 4096)
    return MAMG_OK;
  half_fill_kernel<<<nblocks(nr), 256>>>(nr, B.ptr, B.col, B.val, meta, hw[0], hw[1], su, nullptr, nullptr,
                                         nullptr, nullptr, 0, nullptr, nullptr, wm + 3, 1);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(&hw[3], wm + 3, sizeof(int), hipMemcpyDeviceToHost));
  if (hw[3]) return MAMG_OK;   // a mirror is missing or differs
  if ((rc = dalloc(h, &D->meta, std::max<int64_t>(nr, 1), err))) return rc;
  if ((rc = dalloc(h, &D->col, std::max<int64_t>(su, 1), err))) return rc;
  if ((rc = dalloc(h, &D->val, std::max<int64_t>(3 * su, 1), err))) return rc;
  if ((rc = dalloc(h, &D->lptr, std::max<int64_t>(sl, 1), err))) return rc;
  if (ngs) {
    if ((rc = dalloc(h, &D->gsoff, ns + 1, err))) return rc;
    if ((rc = dalloc(h, &D->gcol, ngs, err))) return rc;
    if ((rc = dalloc(h, &D->gval, 3 * ngs, err))) return rc;
    HIPCHK(dev_copy(D->gsoff, gsoff, (ns + 1) * sizeof(int64_t)));
    HIPCHK(dev_memset(D->gcol, 0, ngs * sizeof(int32_t)));
    HIPCHK(dev_memset(D->gval, 0, 3 * ngs * sizeof(double)));
  }
  HIPCHK(dev_copy(D->meta, meta, nr * sizeof(int32_t)));
  HIPCHK(dev_memset(D->col, 0, std::max<int64_t>(su, 1) * sizeof(int32_t)));
  HIPCHK(dev_memset(D->val, 0, std::max<int64_t>(3 * su, 1) * sizeof(double)));
  HIPCHK(dev_memset(D->lptr, 0, std::max<int64_t>(sl, 1) * sizeof(int32_t)));
  half_fill_kernel<<<nblocks(nr), 256>>>(nr, B.ptr, B.col, B.val, meta, hw[0], hw[1], su, D->col, D->val, D->lptr,
                                         D->gsoff, ngs, D->gcol, D->gval, wm + 3, 0);
  HIPCHK(hipGetLastError());
  D->half = true;
  D->hwu = hw[0];
  D->hwl = hw[1];
  D->nbs = su;
  D->nlo = nlo;
  D->ngs = ngs;
  return build_band_sched(h, B, D, err);
}

// host BSR2 (multi-GPU rank-local level-0 A: owned rows, [owned | ghost]
// columns) -> half-symmetric ELL-64 when its owned part is symmetric bitwise,
// else upload_bsr (SELL-64 / lane groups)
template <class HT>
int upload_half_or_bsr(HT* h, const HBsr& B, DBsr* D, std::string* err) {
  const int64_t np = (int64_t)B.ptr.size();
  if (g_half && B.nr >= g_sell_min_rows && np == B.nr + 1 && blocks_symmetric(B)) {
    int rc;
    TmpPool T;
    TBsr tb;
    tb.nr = B.nr; tb.nc = B.nc; tb.nb = B.ptr[B.nr];
    if ((rc = T.alloc(&tb.ptr, np, err))) return rc;
    if ((rc = T.alloc(&tb.col, tb.nb, err))) return rc;
    if ((rc = T.alloc(&tb.val, tb.nb, err))) return rc;
    HIPCHK(hipMemcpy(tb.ptr, B.ptr.data(), np * sizeof(int64_t), hipMemcpyHostToDevice));
    if (tb.nb) {
      HIPCHK(hipMemcpy(tb.col, B.col.data(), tb.nb * sizeof(int32_t), hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(tb.val, B.val.data(), tb.nb * sizeof(dv4), hipMemcpyHostToDevice));
    }
    D->nr = B.nr;
    D->nc = B.nc;
    D->nb = tb.nb;
    D->lanes = pick_lanes_bsr(B.nr, D->nb);
    D->sym = true;
    if ((rc = try_half(h, &T, tb, D, err))) return rc;
    if (D->half) return MAMG_OK;
  }
  return upload_bsr(h, B, D, 0, err, true);
}

// final apply layout from a raw device BSR (the device-side counterpart of
// upload_bsr): SELL-64 for large short-row plain matrices, symmetric-block
// packing where every block has (0,1) == (1,0) bitwise, else 4 doubles/block
template <class HT>
int finalize_bsr(HT* h, TmpPool* T, TBsr& B, DBsr* D, int lanes, bool sym_ok, std::string* err,
                 bool allow_sell = true, bool allow_half = false, bool allow_msell = false) {
  int rc;
  const int64_t nr = B.nr, np = B.merged ? 2 * nr + 1 : nr + 1;
  D->nr = nr;
  D->nc = B.nc;
  D->nb = B.nb;
  D->lanes = lanes > 0 ? lanes : pick_lanes_bsr(nr, D->nb);
  bool sym = false;
  if (sym_ok && !B.merged && B.nb > 0) {
    int* bad = nullptr;
    if ((rc = T->alloc(&bad, 1, err))) return rc;
    HIPCHK(dev_memset(bad, 0, sizeof(int)));
    sym_check_kernel<<<std::min(nblocks(B.nb), SYM_CHECK_BLOCKS), 256>>>(B.nb, B.val, bad);
    int hb = 1;
    HIPCHK(hipMemcpy(&hb, bad, sizeof(int), hipMemcpyDeviceToHost));
    sym = hb == 0;
  }
  D->sym = sym;
  const int per = sym ? 3 : 4;
  // multi-lane SELL (msell_kernel) for the coarse levels' A and K: lanes per
  // row from the mean row length, chunks of 5 blocks per lane
  const bool msell = allow_sell && allow_msell && !B.merged && nr >= g_msell_min_rows && nr < g_sell_min_rows;
  if (msell) {
    const double mean = nr ? (double)D->nb / (double)nr : 0.0;
    D->lpr = mean <= 10.0 ? 2 : mean <= 20.0 ? 4 : mean <= 40.0 ? 8 : 16;
  }
  if (allow_sell && ((nr >= g_sell_min_rows && D->nb <= g_sell_max_len * nr) || msell) && !B.merged) {
    if (allow_half && g_half && sym && nr == B.nc) {
      if ((rc = try_half(h, T, B, D, err))) return rc;
      if (D->half) return MAMG_OK;
    }
    const int64_t ns = (nr + SELL_C - 1) / SELL_C;
    int* bad = nullptr;
    if ((rc = T->alloc(&bad, 1, err))) return rc;
    HIPCHK(dev_memset(bad, 0, sizeof(int)));
    D->sell = true;
    if ((rc = dalloc(h, &D->soff, ns + 1, err))) return rc;
    if ((rc = dalloc(h, &D->meta, std::max<int64_t>(nr, 1), err))) return rc;
    sell_meta_kernel<<<nblocks(ns), 256>>>(nr, B.ptr, 0, D->meta, D->soff, bad);
    HIPCHK(hipGetLastError());
    int hb = 0;
    HIPCHK(hipMemcpy(&hb, bad, sizeof(int), hipMemcpyDeviceToHost));
    if (hb) { *err = "SELL: row longer than 65534 blocks"; return MAMG_ERR_UNSUPPORTED; }
    if ((rc = dscan_incl_i64(D->soff, D->soff, ns + 1, nullptr, err))) return rc;
    HIPCHK(hipMemcpy(&D->nbs, D->soff + ns, sizeof(int64_t), hipMemcpyDeviceToHost));
    if ((rc = dalloc(h, &D->col, std::max<int64_t>(D->nbs, 1), err))) return rc;
    if ((rc = dalloc(h, &D->val, std::max<int64_t>(per * D->nbs, 1), err))) return rc;
    HIPCHK(dev_memset(D->col, 0, std::max<int64_t>(D->nbs, 1) * sizeof(int32_t)));
    HIPCHK(dev_memset(D->val, 0, std::max<int64_t>(per * D->nbs, 1) * sizeof(double)));
    sell_fill_kernel<<<nblocks(nr), 256>>>(nr, B.ptr, 0, B.col, B.val, D->soff, D->nbs, sym ? 1 : 0, D->col, D->val);
    HIPCHK(hipGetLastError());
    return MAMG_OK;
  }
  if ((rc = dalloc(h, &D->ptr, np, err))) return rc;
  if ((rc = dalloc(h, &D->col, std::max<int64_t>(D->nb, 1), err))) return rc;
  if ((rc = dalloc(h, &D->val, std::max<int64_t>(per * D->nb, 1), err))) return rc;
  HIPCHK(dev_copy(D->ptr, B.ptr, np * sizeof(int64_t)));
  if (D->nb) {
    HIPCHK(dev_copy(D->col, B.col, D->nb * sizeof(int32_t)));
    if (sym) pack_sym_kernel<<<nblocks(D->nb), 256>>>(D->nb, B.val, D->val);
    else HIPCHK(dev_copy(D->val, B.val, D->nb * sizeof(dv4)));
    HIPCHK(hipGetLastError());
  }
  return MAMG_OK;
}

// Level-0 K's rows sorted by length inside each SELL slice (MAMG_K_SORT, default
// on).  A 128-byte line of one block slot holds 4 neighbouring rows' blocks;
// in row order their lengths differ, so the last slots of the longer rows pull
// whole lines whose other quarters are padding: 13 % more line bytes than
// stored blocks for the bidomain K.  Sorted, the rows sharing a line have equal
// or neighbouring lengths (1.9 %).  Each row keeps its blocks and their order:
// results are bitwise those of row order (test_k_row_sort_bitwise).
template <class HT>
int sort_sell_slices(HT* h, TmpPool* T, DBsr* D, std::string* err) {
  int rc;
  if (!D->sell || D->split || D->nr == 0) return MAMG_OK;
  const int64_t ns = (D->nr + SELL_C - 1) / SELL_C, per = D->sym ? 3 : 4;
  int32_t *nmeta = nullptr, *src = nullptr, *ncol = nullptr;
  double* nval = nullptr;
  if ((rc = T->alloc(&nmeta, D->nr, err)) || (rc = T->alloc(&src, D->nr, err)) ||
      (rc = T->alloc(&ncol, std::max<int64_t>(D->nbs, 1), err)) ||
      (rc = T->alloc(&nval, std::max<int64_t>(per * D->nbs, 1), err)))
    return rc;
  HIPCHK(dev_memset(ncol, 0, std::max<int64_t>(D->nbs, 1) * sizeof(int32_t)));
  HIPCHK(dev_memset(nval, 0, std::max<int64_t>(per * D->nbs, 1) * sizeof(double)));
  sell_sort_kernel<<<(unsigned)ns, SELL_C>>>(D->nr, D->meta, nmeta, src);
  HIPCHK(hipGetLastError());
  sell_permute_kernel<<<(unsigned)ns, SELL_C>>>(D->nr, D->soff, src, D->nbs, (int)per, D->col, D->val, ncol, nval);
  HIPCHK(hipGetLastError());
  HIPCHK(dev_copy(D->meta, nmeta, D->nr * sizeof(int32_t)));
  HIPCHK(dev_copy(D->col, ncol, D->nbs * sizeof(int32_t)));
  HIPCHK(dev_copy(D->val, nval, per * D->nbs * sizeof(double)));
  T->release(nmeta); T->release(src); T->release(ncol); T->release(nval);
  D->lsort = true;
  return MAMG_OK;
}

// SELL columns as 16-bit offsets from a per-slice base (round 6, level-0 K:
// MAMG_K_COL16, default on).  K's columns are coarse node ids; the 64 rows of
// a slice reach the aggregates of a few neighbouring planes, so every slice's
// columns span far less than 2^16 (at nrefs=6: 4-byte columns are 11 % of K's
// stream).  cbase[s] = the slice's smallest column; a matrix with any slice
// spanning more keeps its 32-bit columns (then nothing changes).  The kernel
// adds the base back: the same columns, the same sums, bitwise the 32-bit
// layout (tests/test_gpu.py::test_k_col16_bitwise).
__global__ __launch_bounds__(64) void sell_span_kernel(int64_t nr, const int64_t* __restrict__ soff,
                                                       const int32_t* __restrict__ meta,
                                                       const int32_t* __restrict__ col, int32_t* __restrict__ cbase,
                                                       int* wide) {
  const int64_t s = blockIdx.x, slot = s * SELL_C + threadIdx.x;
  int32_t lo = INT32_MAX, hi = INT32_MIN;
  if (slot < nr) {
    const int len = meta[slot] & 0xffff;
    const int64_t k = soff[s] + threadIdx.x;
    for (int j = 0; j < len; ++j) {
      const int32_t c = col[k + (int64_t)SELL_C * j];
      lo = c < lo ? c : lo;
      hi = c > hi ? c : hi;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t a = __shfl_xor(lo, o), b = __shfl_xor(hi, o);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if (threadIdx.x == 0) {
    cbase[s] = lo == INT32_MAX ? 0 : lo;
    if (hi != INT32_MIN && (int64_t)hi - (int64_t)lo > 65535) atomicOr(wide, 1);
  }
}
__global__ __launch_bounds__(64) void sell_col16_kernel(int64_t nr, const int64_t* __restrict__ soff,
                                                        const int32_t* __restrict__ meta,
                                                        const int32_t* __restrict__ col,
                                                        const int32_t* __restrict__ cbase, uint16_t* __restrict__ c16) {
  const int64_t s = blockIdx.x, slot = s * SELL_C + threadIdx.x;
  if (slot >= nr) return;
  const int len = meta[slot] & 0xffff;
  const int64_t k = soff[s] + threadIdx.x;
  const int32_t b = cbase[s];
  for (int j = 0; j < len; ++j) c16[k + (int64_t)SELL_C * j] = (uint16_t)(col[k + (int64_t)SELL_C * j] - b);
}
template <class HT>
int compress_sell_cols(HT* h, TmpPool* T, DBsr* D, std::string* err) {
  int rc;
  if (!D->sell || D->half || D->nr == 0 || D->nbs == 0) return MAMG_OK;
  const int64_t ns = (D->nr + SELL_C - 1) / SELL_C;
  int32_t* base = nullptr;
  int* wide = nullptr;
  if ((rc = T->alloc(&wide, 1, err))) return rc;
  HIPCHK(dev_memset(wide, 0, sizeof(int)));
  if ((rc = dalloc(h, &base, ns, err))) return rc;
  sell_span_kernel<<<(unsigned)ns, SELL_C>>>(D->nr, D->soff, D->meta, D->col, base, wide);
  HIPCHK(hipGetLastError());
  int hw = 1;
  HIPCHK(hipMemcpy(&hw, wide, sizeof(int), hipMemcpyDeviceToHost));
  T->release(wide);
  if (hw) return MAMG_OK;   // a slice spans more than 16 bits: 32-bit columns (base stays unused)
  uint16_t* c16 = nullptr;
  if ((rc = dalloc(h, &c16, D->nbs, err))) return rc;
  HIPCHK(dev_memset(c16, 0, D->nbs * sizeof(uint16_t)));
  sell_col16_kernel<<<(unsigned)ns, SELL_C>>>(D->nr, D->soff, D->meta, D->col, base, c16);
  HIPCHK(hipGetLastError());
  D->col16 = c16;
  D->cbase = base;
  return MAMG_OK;
}

// one BSR2 level from device-resident field-major CSRs (AP.n == 0: no fusion)
struct LevelSrc {
  DevMat A, P, AP, R;
  const double* W = nullptr;      // 4 nv node blocks (device)
  const double* Ainv = nullptr;   // coarsest: n x n dof order (device)
  const std::vector<int32_t>* seeds = nullptr;   // level 0, SCHWARZ_RINGS
};

inline bool gs_smoother(const mamg_params& p) {
  return p.smoother == MAMG_SMOOTHER_SGS || p.smoother == MAMG_SMOOTHER_GS;
}

// smoothing step s of a sweep sequence: the Jacobi smoothers take W every
// step; SMOOTHER_POLY takes w_1 W .. w_m W before the coarse correction and
// w_m W .. w_1 W after it (mamg_oracle.Hierarchy.cycle), repeated per sweep
inline int step_index(int m, int s, bool pre) {
  const int k = s % m;
  return pre ? k : m - 1 - k;
}
const dv4* step_wd(const DLevel& L, int s, bool pre) {
  return L.Wk.empty() ? L.Wd : L.Wk[step_index((int)L.Wk.size(), s, pre)];
}
const DCsr& step_wb(const DLevel& L, int s, bool pre) {
  return L.WBk.empty() ? L.WB : L.WBk[step_index((int)L.WBk.size(), s, pre)];
}
const double* step_winv(const DLevel& L, int s, bool pre) {
  return L.winvk.empty() ? L.winv : L.winvk[step_index((int)L.winvk.size(), s, pre)];
}

// SMOOTHER_POLY step smoothers w_k W of n doubles each (device copies)
int poly_scaled(DeviceHandle* h, const double* W, int64_t n, std::vector<double*>* out, std::string* err) {
  double w[MAMG_POLY_MAX];
  const int m = poly_weights(h->p, w);
  for (int k = 0; k < m; ++k) {
    double* o = nullptr;
    int rc = dalloc(h, &o, n, err);
    if (rc) return rc;
    if (n) wscale_kernel<<<nblocks(n), 256>>>(n, w[k], W, o);
    HIPCHK(hipGetLastError());
    out->push_back(o);
  }
  return MAMG_OK;
}

// Jones-Plassmann colouring of the node graph of B (every node of the level;
// jp_round_kernel rounds, one 8-byte readback each): *ca (TmpPool-owned, nr
// bytes) = colour per node, *ncol = colours used
int gs_colour(TmpPool* T, const TBsr& B, int level, int8_t** ca_out, int* ncol_out, std::string* err) {
  int rc;
  const int64_t nr = B.nr;
  int* flags = nullptr;                 // [0] asymmetric pattern, [1] > 64 colours
  unsigned long long* left = nullptr;
  unsigned long long* cnt = nullptr;
  int8_t *ca = nullptr, *cb = nullptr;
  if ((rc = T->alloc(&flags, 4, err))) return rc;
  if ((rc = T->alloc(&left, 1, err))) return rc;
  if ((rc = T->alloc(&cnt, 64, err))) return rc;
  if ((rc = T->alloc(&ca, nr, err))) return rc;
  if ((rc = T->alloc(&cb, nr, err))) return rc;
  HIPCHK(dev_memset(flags, 0, 4 * sizeof(int)));
  HIPCHK(dev_memset(cnt, 0, 64 * sizeof(unsigned long long)));
  pattern_sym_kernel<<<nblocks(nr), 256>>>(nr, B.ptr, B.col, flags);
  HIPCHK(hipGetLastError());
  int hf[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpy(hf, flags, 4 * sizeof(int), hipMemcpyDeviceToHost));
  if (hf[0]) { *err = "multicolour GS: node pattern of level " + std::to_string(level) + " not symmetric"; return MAMG_ERR_UNSUPPORTED; }
  HIPCHK(dev_memset(ca, 0xff, nr));
  for (int round = 0;; ++round) {
    unsigned long long nl = 0;
    HIPCHK(dev_memset(left, 0, sizeof(unsigned long long)));
    jp_round_kernel<<<nblocks(nr), 256>>>(nr, B.ptr, B.col, level, ca, cb, left, flags + 1);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(&nl, left, sizeof(nl), hipMemcpyDeviceToHost));
    std::swap(ca, cb);
    if (nl == 0) break;
    if (round > 100000) { *err = "multicolour GS: colouring did not finish"; return MAMG_ERR_SETUP; }
  }
  HIPCHK(hipMemcpy(hf, flags, 4 * sizeof(int), hipMemcpyDeviceToHost));
  if (hf[1]) { *err = "multicolour GS: more than 64 colours on level " + std::to_string(level); return MAMG_ERR_UNSUPPORTED; }
  int32_t* ci = nullptr;
  int64_t* iota = nullptr;
  if ((rc = T->alloc(&ci, nr, err))) return rc;
  if ((rc = T->alloc(&iota, nr, err))) return rc;
  colour_count_kernel<<<nblocks(nr), 256>>>(nr, ca, ci, iota, cnt);
  HIPCHK(hipGetLastError());
  unsigned long long hc[64];
  HIPCHK(hipMemcpy(hc, cnt, sizeof(hc), hipMemcpyDeviceToHost));
  int ncol = 0;
  for (int c = 0; c < 64; ++c)
    if (hc[c]) ncol = c + 1;
  for (void* q : {(void*)cb, (void*)ci, (void*)iota}) T->release(q);
  *ca_out = ca;
  *ncol_out = ncol;
  return MAMG_OK;
}

// GS layout of the rows of B with colours ca (ncol colours; a colour may have
// no rows here, as on one rank of a multi-GPU level): permutation by a stable
// radix sort of the rows by colour (ascending row within a colour), the
// permuted BSR2 copy, its block inverses (node blocks from W's pattern) and
// the colour ranges (each colour padded to whole 64-row slices)
template <class HT>
int gs_layout(HT* h, TmpPool* T, const TBsr& B, const double* W, const int8_t* ca, int ncol, int level,
              DBsr* Gb, int32_t** gperm, dv4** Gd, std::vector<int64_t>* gcs_out, std::vector<int64_t>* gbk,
              std::string* err) {
  int rc;
  const int64_t nr = B.nr;
  int* flags = nullptr;
  unsigned long long* cnt = nullptr;
  int32_t *ci = nullptr, *cs = nullptr;
  int64_t *iota = nullptr, *sorted = nullptr;
  if ((rc = T->alloc(&flags, 4, err))) return rc;
  if ((rc = T->alloc(&cnt, 64, err))) return rc;
  if ((rc = T->alloc(&ci, nr, err))) return rc;
  if ((rc = T->alloc(&cs, nr, err))) return rc;
  if ((rc = T->alloc(&iota, nr, err))) return rc;
  if ((rc = T->alloc(&sorted, nr, err))) return rc;
  HIPCHK(dev_memset(flags, 0, 4 * sizeof(int)));
  HIPCHK(dev_memset(cnt, 0, 64 * sizeof(unsigned long long)));
  if (nr) colour_count_kernel<<<nblocks(nr), 256>>>(nr, ca, ci, iota, cnt);
  HIPCHK(hipGetLastError());
  if ((rc = dsort_pairs_i32_i64(ci, cs, iota, sorted, nr, 6, nullptr, err))) return rc;
  unsigned long long hc[64];
  HIPCHK(hipMemcpy(hc, cnt, sizeof(hc), hipMemcpyDeviceToHost));
  // colour c: sorted positions [gcs[c], gcs[c+1]); permuted rows from pcs[c],
  // each colour padded to whole 64-row slices
  std::vector<int64_t> gcs(65, 0), pcs(65, 0);
  for (int c = 0; c < ncol; ++c) {
    gcs[c + 1] = gcs[c] + (int64_t)hc[c];
    pcs[c + 1] = pcs[c] + ((int64_t)hc[c] + SELL_C - 1) / SELL_C * SELL_C;
  }
  const int64_t nrp = pcs[ncol];
  int64_t *gcs_d = nullptr, *pcs_d = nullptr;
  if ((rc = T->alloc(&gcs_d, 65, err))) return rc;
  if ((rc = T->alloc(&pcs_d, 65, err))) return rc;
  HIPCHK(hipMemcpy(gcs_d, gcs.data(), 65 * sizeof(int64_t), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(pcs_d, pcs.data(), 65 * sizeof(int64_t), hipMemcpyHostToDevice));
  gcs_out->assign(pcs.begin(), pcs.begin() + ncol + 1);
  TBsr G;
  G.nr = nrp; G.nc = B.nc; G.nb = B.nb;
  if ((rc = T->alloc(&G.ptr, nrp + 1, err))) return rc;
  HIPCHK(dev_memset(G.ptr, 0, sizeof(int64_t)));
  if ((rc = dalloc(h, gperm, std::max<int64_t>(nrp, 1), err))) return rc;
  if ((rc = dalloc(h, Gd, std::max<int64_t>(nrp, 1), err))) return rc;
  HIPCHK(dev_memset(*gperm, 0xff, std::max<int64_t>(nrp, 1) * sizeof(int32_t)));
  if (nr) perm_place_kernel<<<nblocks(nr), 256>>>(nr, cs, sorted, gcs_d, pcs_d, *gperm);
  HIPCHK(hipGetLastError());
  if (nrp) perm_len_kernel<<<nblocks(nrp), 256>>>(nrp, *gperm, B.ptr, G.ptr);
  HIPCHK(hipGetLastError());
  if ((rc = dscan_incl_i64(G.ptr, G.ptr, nrp + 1, nullptr, err))) return rc;
  if ((rc = T->alloc(&G.col, G.nb, err))) return rc;
  if ((rc = T->alloc(&G.val, G.nb, err))) return rc;
  if (nrp)
    perm_fill_kernel<<<nblocks(nrp), 256>>>(nrp, *gperm, B.ptr, B.col, B.val, reinterpret_cast<const dv4*>(W),
                                            G.ptr, G.col, G.val, *Gd, flags + 2);
  HIPCHK(hipGetLastError());
  int hf[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpy(hf, flags, 4 * sizeof(int), hipMemcpyDeviceToHost));
  if (hf[2]) { *err = "multicolour GS: a smoother block is missing or not SPD on level " + std::to_string(level); return MAMG_ERR_SETUP; }
  gbk->assign(ncol + 1, 0);
  for (int c = 0; c <= ncol; ++c) HIPCHK(hipMemcpy(&(*gbk)[c], G.ptr + (*gcs_out)[c], sizeof(int64_t), hipMemcpyDeviceToHost));
  // lane groups, not SELL-64: one lane per row over a colour's rows measured
  // 19.7 vs 11.5 ms for the four level-0 sweeps at nrefs=6
  if ((rc = finalize_bsr(h, T, G, Gb, 0, true, err, false))) return rc;
  for (void* q : {(void*)ci, (void*)cs, (void*)iota, (void*)sorted, (void*)G.ptr, (void*)G.col, (void*)G.val})
    T->release(q);
  return MAMG_OK;
}

// Multicolour GS layout of one level from A_l's device BSR2 B and the
// level's (scaled) smoother blocks W (only their pattern is used: a node
// whose W block is diagonal has two 1x1 smoother blocks)
template <class HT>
int build_gs(HT* h, TmpPool* T, const TBsr& B, const double* W, int level, DLevel* D, std::string* err) {
  int8_t* ca = nullptr;
  int ncol = 0;
  int rc = gs_colour(T, B, level, &ca, &ncol, err);
  if (rc) return rc;
  rc = gs_layout(h, T, B, W, ca, ncol, level, &D->Gb, &D->gperm, &D->Gd, &D->gcs, &D->gbk, err);
  T->release(ca);
  // the colour steps of small coarse levels (<= 20000 node rows: a launch of
  // a few hundred rows, bound by its dependent load chain) take the largest
  // power of two <= 1.25 x the mean row length as lanes per row (about one
  // block per lane) instead of the SpMV rule's ~two: the reference family at
  // nrefs=6, level 7 8 -> 16 lanes, 142.4 -> 139.9 ms per apply
  // (profiles/r06_ab_misc.txt)
  if (rc == MAMG_OK && level > 0 && B.nr <= 20000 && D->Gb.nr > 0) {
    const double avg = (double)D->Gb.nb / (double)std::max<int64_t>(1, (int64_t)(B.nr));
    int l = 2;
    while (l < 64 && (double)(2 * l) <= 1.25 * avg) l *= 2;
    D->Gb.lanes = l;
  }
#if MAMG_DIAG   // diagnosis: lanes per row of the launched colour steps on levels of <= 20000 node rows
  if (const char* e = std::getenv("MAMG_GS_LANES"))
    if (rc == MAMG_OK && level > 0 && B.nr <= 20000 && std::atoi(e) > 0) D->Gb.lanes = std::atoi(e);
#endif
  return rc;
}

__global__ __launch_bounds__(256) void split_blocks_kernel(int64_t nbs, const dv4* __restrict__ in, dv2* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= nbs) return;
  const dv4 v = in[k];
  out[k] = dv2{v.x, v.y};
  out[nbs + k] = dv2{v.z, v.w};
}

__global__ __launch_bounds__(256) void split_local_kernel(int64_t nbs, const dv4* __restrict__ in, double* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= nbs) return;
  const dv4 v = in[k];
  const int64_t r = k & ~(int64_t)63, i = k & 63;
  reinterpret_cast<dv2*>(out + 4 * r)[i] = dv2{v.x, v.y};
  reinterpret_cast<dv2*>(out + 4 * r + 128)[i] = dv2{v.z, v.w};
}
__global__ __launch_bounds__(256) void unsplit_local_kernel(int64_t nbs, const double* __restrict__ in, dv4* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= nbs) return;
  out[k] = blk_split_local(in, k);
}
// SELL slice s (64 w_s slots) moved from soff_old[s] to soff_new[s] (one workgroup per slice)
__global__ __launch_bounds__(256) void unsplit_blocks_kernel(int64_t nbs, const dv2* __restrict__ in, dv4* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= nbs) return;
  const dv2 a = in[k], b = in[nbs + k];
  out[k] = dv4{a.x, a.y, b.x, b.y};
}

inline bool patch_schwarz(const mamg_params& p) {
  return p.Schwarz_levels >= 1 && p.Schwarz_type == MAMG_SCHWARZ_PATCHES;
}

// the distance-3 colouring of the node graph of B (c[I], device, from T), its
// colour count bound check and the longest row (node patches: <= 16 nodes)
int patch_colour(TmpPool* T, const TBsr& B, int16_t** cout, int* maxlen, std::string* err) {
  int rc;
  const int64_t nr = B.nr;
  int* flags = nullptr;                 // [0] asymmetric pattern, [1] > 256 colours, [3] max row length
  if ((rc = T->alloc(&flags, 4, err))) return rc;
  HIPCHK(dev_memset(flags, 0, 4 * sizeof(int)));
  pattern_sym_kernel<<<nblocks(nr), 256>>>(nr, B.ptr, B.col, flags);
  patch_rowlen_kernel<<<nblocks(nr), 256>>>(nr, B.ptr, flags + 3);
  HIPCHK(hipGetLastError());
  int hf[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpy(hf, flags, 4 * sizeof(int), hipMemcpyDeviceToHost));
  if (hf[0]) { *err = "node patches: node pattern of level 0 not symmetric"; return MAMG_ERR_UNSUPPORTED; }
  if (hf[3] > PATCH_MAX_NODES) {
    *err = "node patches: a node has " + std::to_string(hf[3]) + " neighbours (at most " +
           std::to_string(PATCH_MAX_NODES) + " nodes per patch)";
    return MAMG_ERR_UNSUPPORTED;
  }
  *maxlen = hf[3];
  int16_t* c = nullptr;
  uint64_t *m1 = nullptr, *m2 = nullptr, *m3 = nullptr;
  unsigned long long* mask1 = nullptr;
  int32_t* win = nullptr;
  unsigned int* wcnt = nullptr;                // winners of the round
  uint32_t* cb = nullptr;                      // coloured nodes, one bit each
  if ((rc = T->alloc(&c, nr, err))) return rc;
  if ((rc = T->alloc(&cb, nr / 32 + 1, err))) return rc;
  HIPCHK(dev_memset(cb, 0, (nr / 32 + 1) * sizeof(uint32_t)));
  if ((rc = T->alloc(&m1, nr, err))) return rc;
  if ((rc = T->alloc(&m2, nr, err))) return rc;
  if ((rc = T->alloc(&m3, nr, err))) return rc;
  if ((rc = T->alloc(&mask1, PATCH_WORDS * nr, err))) return rc;
  if ((rc = T->alloc(&win, nr, err))) return rc;
  if ((rc = T->alloc(&wcnt, 1, err))) return rc;
  HIPCHK(dev_memset(c, 0xff, nr * sizeof(int16_t)));
  HIPCHK(dev_memset(mask1, 0, PATCH_WORDS * nr * sizeof(unsigned long long)));
  // the 3-hop maxima of all keys (three full passes), then the winner list
  pkey_init_kernel<<<nblocks(nr), 256>>>(nr, c, m3);
  pkey_max_kernel<<<nblocks(nr), 256>>>(nr, B.ptr, B.col, m3, m1);
  pkey_max_kernel<<<nblocks(nr), 256>>>(nr, B.ptr, B.col, m1, m2);
  pkey_max_kernel<<<nblocks(nr), 256>>>(nr, B.ptr, B.col, m2, m3);
  const unsigned g1k = (unsigned)((nr + 1023) / 1024);
  HIPCHK(dev_memset(wcnt, 0, sizeof(unsigned int)));
  pkey_refresh_kernel<true><<<g1k, 1024>>>(nr, B.ptr, B.col, cb, m2, m3, win, wcnt);
  HIPCHK(hipGetLastError());
  for (int round = 0;; ++round) {
    unsigned int nw = 0;
    HIPCHK(hipMemcpy(&nw, wcnt, sizeof(nw), hipMemcpyDeviceToHost));
    if (nw == 0) break;                        // every node coloured
    if (round > 100000) { *err = "node patches: colouring did not finish"; return MAMG_ERR_SETUP; }
    patch_win_kernel<<<(unsigned)((nw + 3) / 4), 256>>>(nw, win, B.ptr, B.col, c, cb, mask1, flags + 1);
    pkey_refresh_kernel<false><<<nblocks(nr), 256>>>(nr, B.ptr, B.col, cb, nullptr, m1, nullptr, nullptr);
    pkey_refresh_kernel<false><<<nblocks(nr), 256>>>(nr, B.ptr, B.col, cb, m1, m2, nullptr, nullptr);
    HIPCHK(dev_memset(wcnt, 0, sizeof(unsigned int)));
    pkey_refresh_kernel<true><<<g1k, 1024>>>(nr, B.ptr, B.col, cb, m2, m3, win, wcnt);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipMemcpy(hf, flags, 4 * sizeof(int), hipMemcpyDeviceToHost));
  if (hf[1]) { *err = "node patches: more than 256 colours"; return MAMG_ERR_UNSUPPORTED; }
  T->release(m1); T->release(m2); T->release(m3); T->release(mask1); T->release(win); T->release(wcnt);
  T->release(flags); T->release(cb);
  *cout = c;
  return MAMG_OK;
}

// Node-patch Schwarz data of level 0 from A_0's device BSR2 B: the distance-3
// colouring (patch_colour), patches sorted by colour (stable radix sort,
// ascending centre within a colour), A_0 kept as plain BSR2 for the patch
// rows, and the patch inverses (patch_inv_kernel).
int build_patches(DeviceHandle* h, TmpPool* T, const TBsr& B, DLevel* D, std::string* err) {
  int rc;
  const int64_t nr = B.nr;
  int* flags = nullptr;                 // [2] bad pivot
  unsigned long long* cnt = nullptr;
  if ((rc = T->alloc(&flags, 4, err))) return rc;
  if ((rc = T->alloc(&cnt, 64 * PATCH_WORDS, err))) return rc;
  HIPCHK(dev_memset(flags, 0, 4 * sizeof(int)));
  HIPCHK(dev_memset(cnt, 0, 64 * PATCH_WORDS * sizeof(unsigned long long)));
  int16_t* c = nullptr;
  int hf[4] = {0, 0, 0, 0};
  if ((rc = patch_colour(T, B, &c, &hf[3], err))) return rc;
  int32_t *ci = nullptr, *cs = nullptr;
  int64_t *iota = nullptr, *sorted = nullptr;
  if ((rc = T->alloc(&ci, nr, err))) return rc;
  if ((rc = T->alloc(&cs, nr, err))) return rc;
  if ((rc = T->alloc(&iota, nr, err))) return rc;
  if ((rc = T->alloc(&sorted, nr, err))) return rc;
  pcolour_count_kernel<<<nblocks(nr), 256>>>(nr, c, ci, iota, cnt);
  HIPCHK(hipGetLastError());
  if ((rc = dsort_pairs_i32_i64(ci, cs, iota, sorted, nr, 8, nullptr, err))) return rc;
  std::vector<unsigned long long> hc(64 * PATCH_WORDS);
  HIPCHK(hipMemcpy(hc.data(), cnt, hc.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  int ncol = 0;
  for (int k = 0; k < 64 * PATCH_WORDS; ++k)
    if (hc[k]) ncol = k + 1;
  D->pcs.assign(ncol + 1, 0);
  for (int k = 0; k < ncol; ++k) D->pcs[k + 1] = D->pcs[k] + (int64_t)hc[k];
  if ((rc = dalloc(h, &D->pperm, nr, err))) return rc;
  i64_to_i32_kernel<<<nblocks(nr), 256>>>(nr, sorted, D->pperm);
  HIPCHK(hipGetLastError());
  for (void* q : {(void*)c, (void*)ci, (void*)cs, (void*)iota, (void*)sorted}) T->release(q);
  // A_0's patch rows: plain BSR2 in node order
  D->Snb = B.nb;
  if ((rc = dalloc(h, &D->Sptr, nr + 1, err))) return rc;
  if ((rc = dalloc(h, &D->Scol, B.nb, err))) return rc;
  if ((rc = dalloc(h, &D->Sval, B.nb, err))) return rc;
  HIPCHK(dev_copy(D->Sptr, B.ptr, (nr + 1) * sizeof(int64_t)));
  HIPCHK(dev_copy(D->Scol, B.col, B.nb * sizeof(int32_t)));
  HIPCHK(dev_copy(D->Sval, B.val, B.nb * sizeof(dv4)));
  const int64_t dmax = 2 * (int64_t)hf[3];
  D->pus = dmax * (dmax + 1) / 2;
  if ((rc = dalloc(h, &D->pu, nr * D->pus, err))) return rc;
  launch_patch_inv(nr, D->pperm, D->Sptr, D->Scol, D->Scol, D->Sval, D->pus, D->pu, flags + 2);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(hf, flags, 4 * sizeof(int), hipMemcpyDeviceToHost));
  if (hf[2]) { *err = "node patches: a patch matrix is not SPD (non-positive Gauss-Jordan pivot)"; return MAMG_ERR_SETUP; }
  return MAMG_OK;
}

inline bool rings_schwarz(const mamg_params& p) {
  return p.Schwarz_levels >= 1 && p.Schwarz_type == MAMG_SCHWARZ_RINGS;
}

// Seed-ring Schwarz data of level 0 (Schwarz_type RINGS) from A_0's device
// CSR S.A and node BSR2 B: the blocks and their inverses on the device
// (ring_blocks_dev: the additive form's breadth-first rings and Gauss-Jordan
// kernels), the greedy conflict colouring on the host (setup.cpp
// ring_colouring, in seed order: the sequential step, as VMB's), the blocks
// re-ordered colour by colour with their inverses transposed, A_0's plain
// BSR2 copy for the block rows, and the rest's multicolour node-block GS with
// the covered dofs masked out (mamg_oracle.rest_gs_inverse).
int build_rings(DeviceHandle* h, TmpPool* T, const TBsr& B, const LevelSrc& S, DLevel* D, std::string* err) {
  const mamg_params& p = h->p;
  if (!S.seeds || S.seeds->empty()) { *err = "seed rings: no seeds"; return MAMG_ERR_ARG; }
  const int64_t n = S.A.n, nv = n / 2, ns = (int64_t)S.seeds->size();
  const auto t0 = std::chrono::steady_clock::now();
  auto ms_since = [](std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  };
  RingBlocks RB;
  int rc = ring_blocks_dev(S.A, S.seeds->data(), ns, p.Schwarz_maxlvl, p.Schwarz_mmsize, &RB, err);
  if (rc) return rc;
  struct Guard { RingBlocks* r; ~Guard() { ring_blocks_free(r); } } guard{&RB};
  const int mm = RB.mm;
  std::vector<int32_t> blk((size_t)ns * mm);
  std::vector<int64_t> blen(ns), sq(ns);
  HIPCHK(hipMemcpy(blk.data(), RB.blk, blk.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(blen.data(), RB.blen, ns * sizeof(int64_t), hipMemcpyDeviceToHost));
  std::vector<int64_t> bptr(ns + 1, 0);
  for (int64_t k = 0; k < ns; ++k) bptr[k + 1] = bptr[k] + blen[k];
  std::vector<int32_t> mem(bptr[ns]);
  for (int64_t k = 0; k < ns; ++k) std::copy(blk.begin() + k * mm, blk.begin() + k * mm + blen[k], mem.begin() + bptr[k]);
  // A_0's pattern for the conflict graph
  std::vector<int64_t> aptr(n + 1);
  std::vector<int32_t> acol(S.A.nnz);
  HIPCHK(hipMemcpy(aptr.data(), S.A.ptr, (n + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(acol.data(), S.A.col, S.A.nnz * sizeof(int32_t), hipMemcpyDeviceToHost));
  CsrView Av;
  Av.n = Av.m = n; Av.ptr = aptr.data(); Av.col = acol.data();
  std::vector<int32_t> colour;
  const double t_blocks = ms_since(t0);
  const auto t1 = std::chrono::steady_clock::now();
  ring_colouring(Av, bptr, mem, &colour);
  const double t_colour = ms_since(t1);
  std::vector<int32_t>().swap(acol);
  int ncol = 0;
  for (int32_t c : colour) ncol = std::max(ncol, c + 1);
  if (p.print_level >= 1)   // what the seed rings cost at the drivers' sizes
    std::fprintf(stderr, "[mamg] seed rings: %lld blocks, %lld member dofs (max %d per block), %d colours, "
                 "blocks + inverses %.1f ms, host colouring %.1f ms, %.3f GB of inverses\n",
                 (long long)ns, (long long)bptr[ns], mm, ncol, t_blocks, t_colour,
                 [&] { double q = 0; for (int64_t k = 0; k < ns; ++k) q += (double)blen[k] * blen[k]; return 8e-9 * q; }());
  std::vector<int32_t> ord(ns);
  std::iota(ord.begin(), ord.end(), 0);
  std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return colour[a] < colour[b]; });
  D->rcs.assign(ncol + 1, 0);
  for (int32_t c : colour) D->rcs[c + 1]++;
  for (int c = 0; c < ncol; ++c) D->rcs[c + 1] += D->rcs[c];
  std::vector<int64_t> mo(ns + 1, 0), io(ns + 1, 0);
  std::vector<int32_t> rm;
  rm.reserve(mem.size());
  std::vector<uint8_t> cov(nv, 0);
  for (int64_t j = 0; j < ns; ++j) {
    const int64_t o = ord[j], d = blen[o];
    mo[j + 1] = mo[j] + d;
    io[j + 1] = io[j] + d * d;
    for (int64_t t = bptr[o]; t < bptr[o + 1]; ++t) {
      const int64_t g = mem[t], I = g % nv, f = g / nv;
      rm.push_back((int32_t)(2 * I + f));
      cov[I] |= (uint8_t)(1u << f);
    }
  }
  D->rnm = mo[ns];
  D->rinv_n = (double)io[ns];
  if ((rc = dalloc(h, &D->rmo, ns + 1, err))) return rc;
  if ((rc = dalloc(h, &D->rio, ns + 1, err))) return rc;
  if ((rc = dalloc(h, &D->rmem, std::max<int64_t>(D->rnm, 1), err))) return rc;
  if ((rc = dalloc(h, &D->rinv, std::max<int64_t>(io[ns], 1), err))) return rc;
  HIPCHK(hipMemcpy(D->rmo, mo.data(), (ns + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(D->rio, io.data(), (ns + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(D->rmem, rm.data(), rm.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  int32_t* dord = nullptr;
  if ((rc = T->alloc(&dord, ns, err))) return rc;
  HIPCHK(hipMemcpy(dord, ord.data(), ns * sizeof(int32_t), hipMemcpyHostToDevice));
  ring_perm_inv_kernel<<<(unsigned)ns, 256>>>(ns, dord, RB.blen, RB.sq, RB.inv, D->rio, D->rinv);
  HIPCHK(hipGetLastError());
  // A_0's block rows: plain BSR2 in node order
  D->Snb = B.nb;
  if ((rc = dalloc(h, &D->Sptr, B.nr + 1, err))) return rc;
  if ((rc = dalloc(h, &D->Scol, B.nb, err))) return rc;
  if ((rc = dalloc(h, &D->Sval, B.nb, err))) return rc;
  HIPCHK(dev_copy(D->Sptr, B.ptr, (B.nr + 1) * sizeof(int64_t)));
  HIPCHK(dev_copy(D->Scol, B.col, B.nb * sizeof(int32_t)));
  HIPCHK(dev_copy(D->Sval, B.val, B.nb * sizeof(dv4)));
  // the rest's GS: multicolour node-block GS, covered dofs masked
  uint8_t* dcov = nullptr;
  dv4* Wp = nullptr;
  if ((rc = T->alloc(&dcov, nv, err))) return rc;
  if ((rc = T->alloc(&Wp, nv, err))) return rc;
  HIPCHK(hipMemcpy(dcov, cov.data(), nv, hipMemcpyHostToDevice));
  rest_w_kernel<<<nblocks(nv), 256>>>(nv, reinterpret_cast<const dv4*>(S.W), dcov, Wp);
  HIPCHK(hipGetLastError());
  if ((rc = build_gs(h, T, B, reinterpret_cast<const double*>(Wp), 0, D, err))) return rc;
  const int64_t nrp = D->gcs.empty() ? 0 : D->gcs.back();
  if (nrp) rest_mask_kernel<<<nblocks(nrp), 256>>>(nrp, D->gperm, dcov, D->Gd);
  HIPCHK(hipGetLastError());
  return MAMG_OK;   // ring_blocks_dev's buffers: freed by the guard, null-stream ordered
}

int build_bsr_level(DeviceHandle* h, int l, const LevelSrc& S, int64_t nvc, int lanesA, std::string* err) {
  DLevel& D = h->L[l];
  const mamg_params& p = h->p;
  const int64_t nv = D.n / 2;
  int rc;
  TmpPool T;
  if (D.coarsest) {
    if ((rc = dalloc(h, &D.Ainv, D.n * D.n, err))) return rc;
    permute_dense_kernel<<<nblocks(D.n * D.n), 256>>>(D.n, S.Ainv, D.Ainv);
    HIPCHK(hipGetLastError());
    TBsr B;
    if ((rc = dev_csr_to_bsr(&T, S.A, nv, nv, &B, err))) return rc;
    return finalize_bsr(h, &T, B, &D.Ab, 0, false, err);
  }
  {
    TBsr B;
    if ((rc = dev_csr_to_bsr(&T, S.A, nv, nv, &B, err))) return rc;
    if ((rc = finalize_bsr(h, &T, B, &D.Ab, lanesA, true, err, true, l == 0, l > 0)))
      return rc;
    const bool patches = l == 0 && patch_schwarz(p);
    const bool rings = l == 0 && rings_schwarz(p) && S.seeds && !S.seeds->empty();
    if (gs_smoother(p) && !patches && !rings)
      if ((rc = build_gs(h, &T, B, S.W, l, &D, err))) return rc;
    if (patches)
      if ((rc = build_patches(h, &T, B, &D, err))) return rc;
    if (rings)
      if ((rc = build_rings(h, &T, B, S, &D, err))) return rc;
    T.release(B.ptr); T.release(B.col); T.release(B.val);
  }
  if ((rc = dalloc(h, &D.Wd, nv, err))) return rc;
  HIPCHK(dev_copy(D.Wd, S.W, 4 * nv * sizeof(double)));
  if (p.smoother == MAMG_SMOOTHER_POLY) {
    std::vector<double*> wk;
    if ((rc = poly_scaled(h, S.W, 4 * nv, &wk, err))) return rc;
    for (double* q : wk) D.Wk.push_back(reinterpret_cast<dv4*>(q));
  }
  if (p.post_fusion && p.postsmooth_iter >= 1 && S.AP.n == D.n && !gs_smoother(p) &&
      !(l == 0 && (patch_schwarz(p) || rings_schwarz(p)))) {
    TBsr Pb, Qb, M;
    if ((rc = dev_csr_to_bsr(&T, S.P, nv, nvc, &Pb, err))) return rc;
    if ((rc = dev_csr_to_bsr(&T, S.AP, nv, nvc, &Qb, err))) return rc;
    if (g_post_k) {   // one operator K = P - W (A P) on AP's pattern,
                      // W = the first post-smoothing step's smoother
      const double* Wpost = reinterpret_cast<const double*>(step_wd(D, 0, false));
      if ((rc = dev_kmerge(&T, Pb, Qb, Wpost, &M, err))) return rc;
    } else {          // P and AP blocks side by side in one row window
      if ((rc = dev_merge_rows(&T, Pb, Qb, &M, err))) return rc;
    }
    T.release(Pb.ptr); T.release(Pb.col); T.release(Pb.val);
    T.release(Qb.ptr); T.release(Qb.col); T.release(Qb.val);
    // K: SELL-64 with 4-block chunks (K rows hold ~9 blocks at level 0; A/B in
    // DESIGN.md section 4), lane-group BSR if MAMG_POST_SELL=0; the merged
    // window is never SELL on this path
    if ((rc = finalize_bsr(h, &T, M, g_post_k ? &D.KPb : &D.PAb, 0, false, err, g_post_k != 0, false,
                           l > 0 && g_post_k != 0)))
      return rc;
    if (l == 0 && g_post_k && g_k_sort && D.KPb.sell && D.KPb.lpr <= 1)
      if ((rc = sort_sell_slices(h, &T, &D.KPb, err))) return rc;
    if (l == 0 && g_post_k && D.KPb.sell && g_k_c16)
      if ((rc = compress_sell_cols(h, &T, &D.KPb, err))) return rc;
  } else {
    TBsr Pb;
    if ((rc = dev_csr_to_bsr(&T, S.P, nv, nvc, &Pb, err))) return rc;
    if ((rc = finalize_bsr(h, &T, Pb, &D.Pb, 0, false, err))) return rc;
  }
  {
    TBsr Rb;
    if ((rc = dev_csr_to_bsr(&T, S.R, nvc, nv, &Rb, err))) return rc;
    if ((rc = finalize_bsr(h, &T, Rb, &D.Rb, 0, false, err))) return rc;
    if (l == 0 && (rc = build_rest_sched(h, &T, &D.Rb, D.Ab.band_stride, err))) return rc;
  }
  return MAMG_OK;
}

// host CSR -> temporary device CSR
int upload_tmp(TmpPool* T, const CsrView& M, DevMat* D, std::string* err) {
  int rc;
  D->n = M.n; D->m = M.m; D->nnz = M.nnz();
  if ((rc = T->alloc(&D->ptr, M.n + 1, err))) return rc;
  if ((rc = T->alloc(&D->col, D->nnz, err))) return rc;
  if ((rc = T->alloc(&D->val, D->nnz, err))) return rc;
  HIPCHK(hipMemcpy(D->ptr, M.ptr, (M.n + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if (D->nnz) {
    HIPCHK(hipMemcpy(D->col, M.col, D->nnz * sizeof(int32_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(D->val, M.val, D->nnz * sizeof(double), hipMemcpyHostToDevice));
  }
  return MAMG_OK;
}

// ---- algorithmic bytes (per layout) ------------------------------
double csr_bytes(const DCsr& M, int epi) {
  double b = 12.0 * M.nnz + 8.0 * (M.n + 1) + 8.0 * M.m + 8.0 * M.n;  // A, x, out
  if (epi == EPI_YADD) b += 8.0 * M.n;
  if (epi == EPI_RESID) b += 8.0 * M.n;
  if (epi == EPI_JACOBI) b += 16.0 * M.n;
  return b;
}

double index_bytes(const DBsr& M, int64_t ptr_entries) {
  return M.sell ? 4.0 * M.nr + 8.0 * (M.nr / SELL_C + 2) : 8.0 * ptr_entries;
}

double bsr_bytes(const DBsr& M, int epi) {
  // half-symmetric: upper blocks (28 B with column) + 4-byte mirror slot per
  // lower block + row meta; the mirrors' values are re-reads, not counted
  double b = M.half ? 28.0 * (M.nb - M.nlo) + 4.0 * M.nlo + 4.0 * M.nr + (M.ngs ? 8.0 * (M.nr / SELL_C + 2) : 0.0) +
                          16.0 * M.nc + 16.0 * M.nr
                    : (M.sym ? 28.0 : M.col16 ? 34.0 : 36.0) * M.nb + index_bytes(M, M.nr + 1) +
                          (M.col16 ? 4.0 * (M.nr / SELL_C + 1) : 0.0) + 16.0 * M.nc + 16.0 * M.nr;
  if (epi == EPI_YADD) b += 16.0 * M.nr;
  if (epi == EPI_RESID) b += 16.0 * M.nr;
  if (epi == EPI_BJAC || epi == EPI_KPOST) b += 16.0 * M.nr + 16.0 * M.nr + 32.0 * M.nr;   // y, b, W
  return b;
}

Op csr_op(const DCsr& M, int epi, int cls, int tag, const double* x, const double* y,
          const double* b, const double* w, double* out) {
  Op o;
  o.kind = OP_CSR; o.epi = epi; o.cls = cls; o.tag = tag; o.M = &M; o.n = M.n;
  o.x = x; o.y = y; o.b = b; o.w = w; o.out = out;
  o.bytes = csr_bytes(M, epi);
  return o;
}

Op bsr_op(const DBsr& M, int epi, int cls, int tag, const double* x, int64_t xs, const double* y,
          const double* b, int64_t bs, const dv4* W, double* out, int64_t os) {
  Op o;
  o.kind = OP_BSR; o.epi = epi; o.cls = cls; o.tag = tag; o.Mb = &M; o.n = M.nr;
  o.x = x; o.xs = xs; o.xfm = xs != 0; o.y = y; o.b = b; o.bs = bs; o.W = W; o.out = out; o.os = os;
  o.bytes = bsr_bytes(M, epi);
  return o;
}

// merged [P | AP] blocks + 2 nr + 1 pointers, e gathered once, x1 r1 W out
Op post_op(const DBsr& M, const double* r1, const dv4* W, int cls, int tag, const double* e,
           const double* x1, double* out, int64_t os) {
  Op o;
  o.kind = OP_POST; o.cls = cls; o.tag = tag; o.Mb = &M; o.n = M.nr;
  o.x = e; o.y = x1; o.b = r1; o.W = W; o.out = out; o.os = os;
  o.bytes = 36.0 * M.nb + index_bytes(M, 2 * M.nr + 1) + 16.0 * M.nc + 16.0 * M.nr * 3 + 32.0 * M.nr;
  return o;
}

Op gemv_op(const DLevel& L, const double* b, double* out) {
  Op o;
  o.kind = OP_GEMV; o.cls = C_DENSE; o.n = L.n; o.x = b; o.w = L.Ainv; o.out = out;
  o.bytes = 8.0 * L.n * L.n + 16.0 * L.n;
  return o;
}

Op axpy_op(int64_t n, const double* e, double* x) {
  Op o;
  o.kind = OP_AXPY; o.cls = C_MISC; o.n = n; o.x = e; o.out = x; o.bytes = 24.0 * n;
  return o;
}

void scale_ops(const DeviceHandle* h, int lc, std::vector<Op>* ops);

// ---- CSR layout: cycle from zero initial guess: xout = MG_l(b) --------------
void cycle_ops_csr(const DeviceHandle* h, int l, const double* b, double* xout, std::vector<Op>* ops) {
  const DLevel& L = h->L[l];
  const mamg_params& p = h->p;
  const bool l0 = l == 0;
  if (L.coarsest) { ops->push_back(gemv_op(L, b, xout)); return; }
  const DLevel& C = h->L[l + 1];
  const bool blk = L.WB.n > 0;
  const int tagA = l0 ? 0 : 1;
  const int clsS = l0 ? C_L0_SMOOTH : C_COARSE;
  const int clsW = l0 ? C_L0_WB : C_COARSE;
  double* X = L.t;
  double* X2 = L.t2;
  const int steps = smoother_steps(p);
  const int npre = p.presmooth_iter * steps, npost = p.postsmooth_iter * steps;
  if (blk) {
    ops->push_back(csr_op(step_wb(L, 0, true), EPI_Y, clsW, tagA, b, nullptr, nullptr, nullptr, X));
  } else {
    Op o;
    o.kind = OP_SCALE; o.cls = clsW; o.n = L.n; o.w = step_winv(L, 0, true); o.x = b; o.out = X;
    o.bytes = 24.0 * L.n;
    ops->push_back(o);
  }
  for (int s = 1; s < npre; ++s) {
    if (blk) {
      ops->push_back(csr_op(L.A, EPI_RESID, clsS, tagA, X, nullptr, b, nullptr, L.r));
      ops->push_back(csr_op(step_wb(L, s, true), EPI_YADD, clsW, tagA, L.r, X, nullptr, nullptr, X2));
    } else {
      ops->push_back(csr_op(L.A, EPI_JACOBI, clsS, tagA, X, X, b, step_winv(L, s, true), X2));
    }
    std::swap(X, X2);
  }
  ops->push_back(csr_op(L.A, EPI_RESID, l0 ? C_L0_RESID : C_COARSE, tagA, X, nullptr, b, nullptr, L.r));
  ops->push_back(csr_op(L.R, EPI_Y, l0 ? C_L0_R : C_COARSE, tagA, L.r, nullptr, nullptr, nullptr, C.b));
  cycle_ops_csr(h, l + 1, C.b, C.x, ops);
  if (p.cycle_type == MAMG_W_CYCLE && !C.coarsest) {
    ops->push_back(csr_op(C.A, EPI_RESID, C_MISC, 1, C.x, nullptr, C.b, nullptr, C.c));
    cycle_ops_csr(h, l + 1, C.c, C.e, ops);
    ops->push_back(axpy_op(C.n, C.e, C.x));
  }
  if (p.coarse_scaling) scale_ops(h, l + 1, ops);
  ops->push_back(csr_op(L.P, EPI_YADD, l0 ? C_L0_P : C_COARSE, tagA, C.x, X, nullptr, nullptr, X));
  for (int s = 0; s < npost; ++s) {
    double* out = (s == npost - 1) ? xout : X2;
    if (blk) {
      ops->push_back(csr_op(L.A, EPI_RESID, clsS, tagA, X, nullptr, b, nullptr, L.r));
      ops->push_back(csr_op(step_wb(L, s, false), EPI_YADD, clsW, tagA, L.r, X, nullptr, nullptr, out));
    } else {
      ops->push_back(csr_op(L.A, EPI_JACOBI, clsS, tagA, X, X, b, step_winv(L, s, false), out));
    }
    if (out == X2) std::swap(X, X2);
  }
}

// ---- BSR2 layout.  b / xout of level 0 are the caller's field-major vectors
// (stride nv0); all other vectors are node-interleaved (stride 0).
// one multicolour GS sweep (colours ascending if fwd, else descending) in place on x
template <class LV>
Op gs_op(const LV& L, int c, double* x, const double* b, int64_t bs, int cls) {
  Op o;
  o.kind = OP_GS; o.cls = cls; o.Mb = &L.Gb; o.perm = L.gperm; o.W = L.Gd;
  o.x = x; o.out = x; o.b = b; o.bs = bs;
  o.r0 = L.gcs[c]; o.r1 = L.gcs[c + 1]; o.n = o.r1 - o.r0;
  const double rows = (double)o.n, ncol = (double)(L.gcs.size() - 1);
  // blocks + pointers + perm + D + b + own x read/write + the gathered x
  // (every node's pair once per sweep, spread over the colours)
  o.bytes = (L.Gb.sym ? 28.0 : 36.0) * (double)(L.gbk[c + 1] - L.gbk[c]) + 8.0 * (rows + 1) + 4.0 * rows +
            32.0 * rows + 16.0 * rows + 32.0 * rows + 16.0 * (double)L.Gb.nc / ncol;
  return o;
}

// one colour of a node-patch sweep: per patch its packed inverse, its node
// rows (blocks + pointers), b and x read/write for its dofs, the gathered x
Op patch_op(const DLevel& L, int c, double* x, const double* b, int64_t bs, int cls) {
  Op o;
  o.kind = OP_PATCH; o.cls = cls; o.lev = &L;
  o.out = x; o.b = b; o.bs = bs;
  o.r0 = L.pcs[c]; o.r1 = L.pcs[c + 1]; o.n = o.r1 - o.r0;
  const double np = (double)o.n, nv = (double)(L.n / 2);
  const double mavg = nv > 0 ? (double)L.Snb / nv : 0.0;   // nodes per patch = blocks per row
  o.bytes = np * (8.0 * (double)L.pus + mavg * (36.0 * mavg + 8.0) + mavg * (16.0 + 32.0) + 12.0);
  return o;
}

// one colour of a seed-ring sweep: per block its transposed inverse, its
// members' rows of A_0 (blocks + pointers), b and x read/write for its
// members, the gathered x
Op ring_op(const DLevel& L, int c, double* x, const double* b, int64_t bs, int cls) {
  Op o;
  o.kind = OP_RING; o.cls = cls; o.lev = &L;
  o.out = x; o.b = b; o.bs = bs;
  o.r0 = L.rcs[c]; o.r1 = L.rcs[c + 1]; o.n = o.r1 - o.r0;
  const double nb = (double)(L.rcs.back()), frac = nb > 0 ? (double)o.n / nb : 0.0;
  const double nv = (double)(L.n / 2), bpr = nv > 0 ? (double)L.Snb / nv : 0.0;   // blocks per node row
  const double m = frac * (double)L.rnm;                                          // members of this colour
  o.bytes = frac * 8.0 * L.rinv_n + m * (bpr * 36.0 + 16.0 + 4.0 + 8.0 + 16.0 + bpr * 16.0) + 16.0 * o.n;
  return o;
}

void ring_sweep_ops(const DLevel& L, bool fwd, double* x, const double* b, int64_t bs, int cls, std::vector<Op>* ops) {
  const int nc = (int)L.rcs.size() - 1;
  for (int k = 0; k < nc; ++k) {
    const int c = fwd ? k : nc - 1 - k;
    if (L.rcs[c + 1] > L.rcs[c]) ops->push_back(ring_op(L, c, x, b, bs, cls));
  }
}

void patch_sweep_ops(const DLevel& L, bool fwd, double* x, const double* b, int64_t bs, int cls, std::vector<Op>* ops) {
  const int nc = (int)L.pcs.size() - 1;
  for (int k = 0; k < nc; ++k) {
    const int c = fwd ? k : nc - 1 - k;
    if (L.pcs[c + 1] > L.pcs[c]) ops->push_back(patch_op(L, c, x, b, bs, cls));
  }
}

void gs_sweep_ops(const DLevel& L, bool fwd, double* x, const double* b, int64_t bs, int cls, std::vector<Op>* ops) {
  const int nc = (int)L.gcs.size() - 1;
  for (int k = 0; k < nc; ++k) {
    const int c = fwd ? k : nc - 1 - k;
    if (L.gcs[c + 1] > L.gcs[c]) ops->push_back(gs_op(L, c, x, b, bs, cls));
  }
}

// coarse-grid correction scaling of level lc's correction e = C.x against its
// right-hand side C.b: q = A_c e, then alpha and e <- alpha e
void scale_ops(const DeviceHandle* h, int lc, std::vector<Op>* ops) {
  const DLevel& C = h->L[lc];
  if (h->bsr) ops->push_back(bsr_op(C.Ab, EPI_Y, C_MISC, 1, C.x, 0, nullptr, nullptr, 0, nullptr, C.q, 0));
  else ops->push_back(csr_op(C.A, EPI_Y, C_MISC, 1, C.x, nullptr, nullptr, nullptr, C.q));
  Op d;
  d.kind = OP_DOT2; d.cls = C_MISC; d.n = C.n; d.b = C.b; d.x = C.x; d.y = C.q; d.part = C.part2;
  d.bytes = 24.0 * C.n;
  ops->push_back(d);
  Op sc;
  sc.kind = OP_CSCALE; sc.cls = C_MISC; sc.n = C.n; sc.part = C.part2; sc.out = C.x; sc.bytes = 16.0 * C.n;
  ops->push_back(sc);
}

// ---- BSR2 layout.  b / xout of level 0 are the caller's field-major vectors
// (stride nv0); all other vectors are node-interleaved (stride 0).
// one op of the launch path as a coarse-tail op (tail_kernel); false if
// the tail cannot express it (level-0 formats and strides, patches, CSR)
bool to_tail(const Op& o, TOp* t) {
  *t = TOp();
  switch (o.kind) {
    case OP_BSR:
    case OP_GS: {
      const DBsr& M = *o.Mb;
      if (M.sell || M.half || M.split || o.xs || o.bs || o.os || o.xfm || M.lanes < 1 || M.lanes > 64) return false;
      t->kind = o.kind == OP_GS ? T_GS : T_BSR;
      t->epi = o.epi; t->vl = std::min(M.lanes, g_tail_vl); t->sym = M.sym ? 1 : 0; t->n = M.nr; t->nb = M.nb;
      t->ptr = M.ptr; t->col = M.col; t->val = M.val;
      t->x = o.kind == OP_GS ? o.out : o.x; t->y = o.y; t->b = o.b; t->W = o.W; t->out = o.out;
      t->r0 = o.r0; t->r1 = o.r1; t->perm = o.perm;
      return true;
    }
    case OP_BD:
      if (o.bs || o.os) return false;
      t->kind = T_BD; t->n = o.n; t->W = o.W; t->b = o.b; t->out = o.out;
      return true;
    case OP_GEMV: t->kind = T_GEMV; t->n = o.n; t->w = o.w; t->x = o.x; t->out = o.out; return true;
    case OP_AXPY: t->kind = T_AXPY; t->n = o.n; t->x = o.x; t->out = o.out; return true;
    case OP_ZERO: t->kind = T_ZERO; t->n = o.n; t->out = o.out; return true;
    case OP_DOT2: t->kind = T_DOT2; t->n = o.n; t->b = o.b; t->x = o.x; t->y = o.y; t->part = o.part; return true;
    case OP_CSCALE: t->kind = T_CSCALE; t->n = o.n; t->part = o.part; t->out = o.out; return true;
    default: return false;
  }
}

void cycle_ops_bsr(const DeviceHandle* h, int l, const double* b, int64_t bs, double* xout,
                   int64_t os, std::vector<Op>* ops, bool tail_ok = true, bool x1_ready = false);

static_assert(sizeof(TOp) % 8 == 0, "TOp is copied into LDS as 8-byte words");
constexpr int64_t TAIL_LDS_MAX = 160 * 1024 - 1024;   // gfx950: 160 KB per workgroup, minus the static arrays

// LDS residency of a coarse-tail program (see T_COPY): every work vector of
// levels >= l the program touches gets an LDS slot; the fields are rewritten
// to tagged LDS offsets, vectors read before written are copied in first and
// written ones copied out last.  Returns the dynamic LDS bytes, or 0 (program
// unchanged: global vectors) when the plan exceeds the LDS.
int64_t tail_lds_plan(const DeviceHandle* h, int l, std::vector<TOp>* prog, int64_t reserve = 0) {
  if (const char* e = opt("MAMG_TAIL_LDS"))
    if (std::atoi(e) == 0) return 0;
  struct Vec {
    double* base;
    int64_t n;
    bool used = false, in = false, out = false, seen = false, lds = false;
    int64_t off = 0, uses = 0;
  };
  std::vector<Vec> vecs;
  for (size_t ll = l; ll < h->L.size(); ++ll) {
    const DLevel& L = h->L[ll];
    for (double* v : {L.b, L.x, L.t, L.t2, L.r, L.c, L.e, L.q})
      if (v) vecs.push_back({v, L.n});
    if (L.part2) vecs.push_back({L.part2, 2 * SCALE_BLOCKS});
  }
  auto find = [&](const double* p) -> Vec* {
    for (auto& v : vecs)
      if (p >= v.base && p < v.base + v.n) return &v;
    return nullptr;
  };
  auto touch = [&](const double* p, bool write) {
    Vec* v = find(p);
    if (!v) return;
    v->used = true;
    ++v->uses;
    if (!v->seen && !write) v->in = true;
    v->seen = true;
    if (write) v->out = true;
  };
  for (const TOp& o : *prog) {   // reads of an op before its writes
    const bool rmw = o.kind == T_GS || o.kind == T_AXPY || o.kind == T_CSCALE;
    for (const double* r : {o.x, o.y, o.b}) if (r) touch(r, false);
    if (o.part) touch(o.part, o.kind != T_CSCALE ? true : false);
    if (o.out) { if (rmw) touch(o.out, false); touch(o.out, true); }
  }
  // the most-used bytes first (the deepest levels: small and visited most
  // often) until the LDS is full; the rest stay global
  std::vector<Vec*> order;
  for (auto& v : vecs)
    if (v.used) order.push_back(&v);
  std::stable_sort(order.begin(), order.end(),
                   [](const Vec* a, const Vec* b) { return a->uses * b->n > b->uses * a->n; });
  int64_t off = 0;
  for (Vec* v : order) {
    const int64_t sz = (v->n * 8 + 15) / 16 * 16;
    if (off + sz > TAIL_LDS_MAX - reserve) continue;
    v->lds = true;
    v->off = off;
    off += sz;
  }
  if (off == 0) return 0;
  static std::atomic<uint64_t> attr_devices{0};   // the attribute is set once per device
  const int dev = h->device & 63;
  if (!(attr_devices >> dev & 1)) {
    const void* fns[] = {(const void*)tail_kernel<false, false, false>, (const void*)tail_kernel<false, true, false>,
                         (const void*)tail_kernel<false, false, true>, (const void*)tail_kernel<false, true, true>,
#if MAMG_DIAG   // the stamped (profiling) variants
                         (const void*)tail_kernel<true, false, false>, (const void*)tail_kernel<true, true, false>,
                         (const void*)tail_kernel<true, false, true>, (const void*)tail_kernel<true, true, true>,
#endif
    };
    bool ok = true;
    for (const void* f : fns)
      ok = ok && hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)TAIL_LDS_MAX) == hipSuccess;
    if (!ok) {
      (void)hipGetLastError();
      return 0;                        // no large dynamic LDS: keep the global-vector program
    }
    attr_devices.fetch_or(1ull << dev);
  }
  auto tag = [&](const double* p) -> double* {
    Vec* v = find(p);
    if (!v || !v->lds) return const_cast<double*>(p);
    return reinterpret_cast<double*>((uintptr_t)(v->off + 8 * (p - v->base)) | 1);
  };
  for (TOp& o : *prog) {
    o.x = tag(o.x); o.y = tag(o.y); o.b = tag(o.b); o.out = tag(o.out); o.part = tag(o.part);
  }
  std::vector<TOp> full;
  for (const auto& v : vecs)
    if (v.lds && v.in) {
      TOp c;
      c.kind = T_COPY; c.n = v.n; c.x = v.base; c.out = reinterpret_cast<double*>((uintptr_t)v.off | 1);
      full.push_back(c);
    }
  full.insert(full.end(), prog->begin(), prog->end());
  for (const auto& v : vecs)
    if (v.lds && v.out) {
      TOp c;
      c.kind = T_COPY; c.n = v.n; c.x = reinterpret_cast<double*>((uintptr_t)v.off | 1); c.out = v.base;
      full.push_back(c);
    }
  prog->swap(full);
  return off;
}

// Register residency of a coarse-tail program (TOp, tail_kernel RES): the
// operators of levels l, l + 1, .. get one row per thread, while their rows
// fit the workgroup.  A level with a multicolour GS layout holds it (Gb:
// colour-permuted, each colour padded to 64-row slices); the level's other
// ops on A (residual, scaling) then read Gb's row i at node perm(i) -- the
// same blocks in the same order as A's row.  One T_RLOAD op in front loads
// every resident row from an image (see tail_rload) built here from the
// matrices; img holds it, and the T_RLOAD's val / col / ridx / b fields hold
// (byte offset in img + 1) until the caller sets device pointers, its r0 / r1
// the LDS region's place once the LDS plan is known.  Returns false when
// nothing is resident.
bool tail_res_plan(const DeviceHandle* h, int l, std::vector<TOp>* prog, std::vector<char>* img, int64_t* nov) {
  *nov = 0;
  if (const char* e = opt("MAMG_TAIL_RES"))
    if (std::atoi(e) == 0) return false;
  constexpr int T = TAIL_THREADS;
  std::vector<dv4> iv((size_t)RES_RB * T, dv4{0.0, 0.0, 0.0, 0.0});
  std::vector<uint32_t> ic((size_t)RES_RB / 2 * T, 0u);
  std::vector<int32_t> hdr((size_t)3 * T, 0);
  std::vector<dv4> gd(T, dv4{0.0, 0.0, 0.0, 0.0});
  std::vector<dv4> ovv;
  std::vector<uint16_t> ovc;
  auto get = [](void* dst, const void* src, size_t bytes) {
    if (hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess) return true;
    (void)hipGetLastError();
    return false;
  };
  int rbase = 0;
  for (size_t ll = (size_t)l; ll < h->L.size(); ++ll) {
    const DLevel& L = h->L[ll];
    const bool hasg = L.gcs.size() > 1;
    const DBsr& M = hasg ? L.Gb : L.Ab;
    if (!M.ptr || M.sell || M.half || M.split || M.nr <= 0 || M.nc > 65536) continue;
    std::vector<int32_t> pm(hasg ? M.nr : 0);
    std::vector<int64_t> ptr(M.nr + 1);
    if ((hasg && !get(pm.data(), L.gperm, M.nr * sizeof(int32_t))) ||
        !get(ptr.data(), M.ptr, (M.nr + 1) * sizeof(int64_t)))
      return false;
    std::vector<int64_t> comp(M.nr + 1, 0);   // rows before -> compact rows before
    std::vector<int32_t> rows;                // compact -> M row
    for (int64_t i = 0; i < M.nr; ++i) {
      if (!hasg || pm[i] >= 0) rows.push_back((int32_t)i);
      comp[i + 1] = (int64_t)rows.size();
    }
    const int n = (int)rows.size();
    if (rbase + n > T) continue;   // a deeper level may still fit
    const int64_t nb = M.nb;
    std::vector<int32_t> col(nb);
    std::vector<double> val((size_t)(M.sym ? 3 : 4) * nb);
    std::vector<dv4> W(hasg ? M.nr : 0);
    if (!get(col.data(), M.col, nb * sizeof(int32_t)) || !get(val.data(), M.val, val.size() * sizeof(double)) ||
        (hasg && !get(W.data(), L.Gd, M.nr * sizeof(dv4))))
      return false;
    auto blk = [&](int64_t k) {
      if (!M.sym) return dv4{val[4 * k], val[4 * k + 1], val[4 * k + 2], val[4 * k + 3]};
      const double b = val[2 * nb + k];
      return dv4{val[2 * k], b, b, val[2 * k + 1]};
    };
    for (int j = 0; j < n; ++j) {
      const int t = rbase + j, i = rows[j];
      const int64_t p0 = ptr[i], len = ptr[i + 1] - p0;
      hdr[t] = (int)len;
      hdr[T + t] = hasg ? pm[i] : i;
      hdr[2 * T + t] = (int)ovv.size();
      for (int k = 0; k < RES_RB && k < len; ++k) {
        iv[(size_t)k * T + t] = blk(p0 + k);
        ic[(size_t)(k / 2) * T + t] |= (uint32_t)col[p0 + k] << (16 * (k & 1));
      }
      if (len > RES_RB) {   // whole fours (tail_res), zero-padded
        const int64_t nk = (len - RES_RB + 3) / 4 * 4;
        for (int64_t k = 0; k < nk; ++k) {
          const bool in = RES_RB + k < len;
          ovv.push_back(in ? blk(p0 + RES_RB + k) : dv4{0.0, 0.0, 0.0, 0.0});
          ovc.push_back(in ? (uint16_t)col[p0 + RES_RB + k] : (uint16_t)0);
        }
      }
      if (hasg) gd[t] = W[i];
    }
    for (TOp& t : *prog) {
      if (t.kind == T_GS && hasg && t.ptr == L.Gb.ptr) {
        t.res = 1; t.rbase = rbase; t.r0 = comp[t.r0]; t.r1 = comp[t.r1];
      } else if (t.kind == T_BSR && t.ptr == L.Ab.ptr) {
        t.res = 1; t.rbase = rbase; t.r0 = 0; t.r1 = n;
        t.ptr = M.ptr; t.col = M.col; t.val = M.val; t.sym = M.sym ? 1 : 0; t.nb = M.nb;
        t.perm = hasg ? L.gperm : nullptr;
      }
    }
    rbase += n;
  }
  if (rbase == 0) return false;
  *nov = (int64_t)ovv.size();
  // the image: values, columns, header, then the LDS region's bytes (block
  // inverses, overflow values, overflow columns padded to 16 B)
  auto put = [&](const void* p, size_t bytes) {
    const size_t off = img->size();
    img->insert(img->end(), static_cast<const char*>(p), static_cast<const char*>(p) + bytes);
    img->resize((img->size() + 15) / 16 * 16, 0);
    return off;
  };
  TOp ld;
  ld.kind = T_RLOAD; ld.r0 = -1; ld.r1 = *nov;
  // the coarsest level's dense inverse (T_GEMV, n <= 64) joins the region:
  // its op's w becomes (offset in the region + 1) with res = 2, turned into
  // a tagged LDS address with the region's (tail_ops)
  std::vector<double> dense;
  std::vector<std::pair<const double*, size_t>> dmap;
  for (TOp& t : *prog) {
    if (t.kind != T_GEMV || !t.w || t.n > 64 || t.n <= 0) continue;
    size_t at = SIZE_MAX;
    for (const auto& q : dmap)
      if (q.first == t.w) at = q.second;
    if (at == SIZE_MAX) {
      at = dense.size();
      dense.resize(at + (size_t)(t.n * t.n));
      if (!get(dense.data() + at, t.w, (size_t)(t.n * t.n) * sizeof(double))) return false;
      dmap.push_back({t.w, at});
    }
    t.res = 2;
    t.w = reinterpret_cast<const double*>((uintptr_t)at);   // doubles into the dense part
  }
  const size_t ov = put(iv.data(), iv.size() * sizeof(dv4));
  const size_t oc = put(ic.data(), ic.size() * sizeof(uint32_t));
  const size_t oh = put(hdr.data(), hdr.size() * sizeof(int32_t));
  const size_t og = put(gd.data(), gd.size() * sizeof(dv4));
  if (!ovv.empty()) put(ovv.data(), ovv.size() * sizeof(dv4));
  if (!ovc.empty()) put(ovc.data(), ovc.size() * sizeof(uint16_t));
  const size_t odn = img->size();
  if (!dense.empty()) put(dense.data(), dense.size() * sizeof(double));
  for (TOp& t : *prog)   // byte offset of each dense matrix in the region
    if (t.kind == T_GEMV && t.res == 2) t.w = reinterpret_cast<const double*>((uintptr_t)(odn - og + 8 * (uintptr_t)t.w));
  ld.n = (int64_t)(img->size() - og);   // the LDS region's bytes (a multiple of 16)
  ld.val = reinterpret_cast<const double*>((uintptr_t)ov + 1);
  ld.col = reinterpret_cast<const int32_t*>((uintptr_t)oc + 1);
  ld.ridx = reinterpret_cast<const int32_t*>((uintptr_t)oh + 1);
  ld.b = reinterpret_cast<const double*>((uintptr_t)og + 1);
  prog->insert(prog->begin(), ld);
  return true;
}

// the cycle of level l and everything below as one tail_kernel launch; the
// device op list is built once per (b, x) and kept on the handle
bool tail_ops(const DeviceHandle* h, int l, const double* b, double* xout, std::vector<Op>* ops) {
  const DeviceHandle::TailProg* tp = nullptr;
  for (const auto& t : h->tails)
    if (t.b == b && t.x == xout) tp = &t;
  if (!tp) {
    std::vector<Op> sub;
    cycle_ops_bsr(h, l, b, 0, xout, 0, &sub, false);
    std::vector<TOp> prog(sub.size());
    double bytes = 0.0;
    for (size_t k = 0; k < sub.size(); ++k) {
      if (!to_tail(sub[k], &prog[k])) return false;
      bytes += sub[k].bytes;
    }
    std::vector<char> img;
    int64_t nov = 0;
    const std::vector<TOp> plain = prog;
    bool res = tail_res_plan(h, l, &prog, &img, &nov);
    int64_t region = 0;   // the resident rows' LDS region, kept free of vectors
    for (const TOp& t : prog)
      if (t.kind == T_RLOAD) region = t.n;
    int64_t lds = tail_lds_plan(h, l, &prog, region + 16);
    bool xl = lds > 0;   // every gathered x in LDS: the ds_read variant of the kernel
    for (const TOp& t : prog)
      if ((t.kind == T_BSR || t.kind == T_GS) && !((uintptr_t)t.x & 1)) xl = false;
    // the program itself into the LDS after the vectors when it fits
    // (TAIL_LDS_MAX); the dynamic LDS then covers both
    int prog_lds = -1;
    int64_t pbytes = (int64_t)(prog.size() * sizeof(TOp));
    const char* pl_opt = opt("MAMG_TAIL_PROG_LDS");
    // default: scalar loads (s_load of a uniform descriptor: 795 vs 1262
    // cycles per empty op)
    const bool prog_in_lds = pl_opt ? std::atoi(pl_opt) != 0 : false;
    if (lds > 0 && prog_in_lds) {
      const int64_t off = (lds + 15) / 16 * 16;
      if (off + pbytes <= TAIL_LDS_MAX) {
        prog_lds = (int)off;
        lds = off + pbytes;
      }
    }
    // the resident rows' LDS region (block inverses, overflow blocks) after
    // both; without room for it (or for the program) the tail keeps its
    // operators in global memory
    if (res) {
      int64_t need = 0;   // the T_RLOAD's LDS region bytes
      for (const TOp& t : prog)
        if (t.kind == T_RLOAD) need = t.n;
      const int64_t off = (lds + 15) / 16 * 16;
      if (lds > 0 && off + need <= TAIL_LDS_MAX) {
        for (TOp& t : prog) {
          if (t.kind == T_RLOAD) { t.r0 = off; t.r1 = nov; }
          if (t.kind == T_GEMV && t.res == 2)   // its matrix in the region: a tagged LDS address
            t.w = reinterpret_cast<const double*>((uintptr_t)(off + (uintptr_t)t.w) | 1);
        }
        lds = off + need;
      } else {
        res = false;
        img.clear();
        prog = plain;
        lds = tail_lds_plan(h, l, &prog);
        prog_lds = -1;
        pbytes = (int64_t)(prog.size() * sizeof(TOp));
        if (lds > 0 && prog_in_lds) {
          const int64_t o2 = (lds + 15) / 16 * 16;
          if (o2 + pbytes <= TAIL_LDS_MAX) {
            prog_lds = (int)o2;
            lds = o2 + pbytes;
          }
        }
      }
    }
    void* d = nullptr;
    const int64_t ioff = (pbytes + 15) / 16 * 16;
    const size_t tbytes = img.size();
    if (raw_malloc(&d, (size_t)ioff + tbytes, "long") != hipSuccess) { (void)hipGetLastError(); return false; }
    char* dimg = static_cast<char*>(d) + ioff;
    auto fix = [&](auto*& f) {
      if (f) f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dimg + ((uintptr_t)f - 1));
    };
    for (TOp& t : prog)
      if (t.kind == T_RLOAD) { fix(t.val); fix(t.col); fix(t.ridx); fix(t.b); }
    if (hipMemcpy(d, prog.data(), prog.size() * sizeof(TOp), hipMemcpyHostToDevice) != hipSuccess ||
        (tbytes && hipMemcpy(dimg, img.data(), tbytes, hipMemcpyHostToDevice) != hipSuccess)) {
      (void)hipGetLastError();
      (void)raw_free(d);
      return false;
    }
    h->tails.push_back({b, xout, (TOp*)d, (int)prog.size(), bytes, lds, xl, prog_lds, res});
    tp = &h->tails.back();
  }
  Op o;
  o.kind = OP_TAIL; o.cls = C_COARSE; o.prog = tp->prog; o.n = tp->n; o.bytes = tp->bytes;
  o.r0 = tp->lds;   // dynamic LDS bytes (0: the program reads global vectors)
  o.r1 = (tp->xl ? 1 : 0) | (tp->res ? 2 : 0);
  o.tail_pl = tp->prog_lds;
  ops->push_back(o);
  return true;
}

// level l's cycle (launch path) begins with the first sweep X = W b into L.t
// (OP_BD): the restriction into l may then write it (EPI_YBD)
bool starts_with_bd(const DeviceHandle* h, int l) {
  const DLevel& L = h->L[l];
  return l > 0 && l != h->tail_level && !L.coarsest && L.gcs.size() <= 1 && L.pcs.size() <= 1 &&
         L.rcs.size() <= 1;
}

// x1_ready: X = W b is already in L.t (written by the restriction's EPI_YBD)
void cycle_ops_bsr(const DeviceHandle* h, int l, const double* b, int64_t bs, double* xout,
                   int64_t os, std::vector<Op>* ops, bool tail_ok, bool x1_ready) {
  if (tail_ok && l > 0 && l == h->tail_level && bs == 0 && os == 0 && tail_ops(h, l, b, xout, ops)) return;
  const DLevel& L = h->L[l];
  const mamg_params& p = h->p;
  const bool l0 = l == 0;
  if (L.coarsest) { ops->push_back(gemv_op(L, b, xout)); return; }   // l > 0 here
  const DLevel& C = h->L[l + 1];
  const int64_t nv = L.n / 2;
  const int tagA = l0 ? 0 : 1;
  const int clsS = l0 ? C_L0_SMOOTH : C_COARSE;
  const int clsW = l0 ? C_L0_WB : C_COARSE;
  const bool pat = L.pcs.size() > 1;                      // node-patch Schwarz on this level
  const bool rng = L.rcs.size() > 1;                      // seed-ring Schwarz + the rest's GS
  const bool gs = L.gcs.size() > 1 || pat || rng;         // multicolour GS on this level
  const bool sgs = p.smoother == MAMG_SMOOTHER_SGS || pat || rng;
  auto sweep = [&](bool fwd, double* x) {
    if (pat) {
      patch_sweep_ops(L, fwd, x, b, bs, clsS, ops);
    } else if (rng) {   // one symmetric step = rings fwd, rest fwd | rest bwd, rings bwd (mamg_oracle.rings_step)
      if (fwd) { ring_sweep_ops(L, true, x, b, bs, clsS, ops); gs_sweep_ops(L, true, x, b, bs, clsS, ops); }
      else { gs_sweep_ops(L, false, x, b, bs, clsS, ops); ring_sweep_ops(L, false, x, b, bs, clsS, ops); }
    } else {
      gs_sweep_ops(L, fwd, x, b, bs, clsS, ops);
    }
  };
  const int steps = smoother_steps(p);
  const int npre = p.presmooth_iter * steps, npost = p.postsmooth_iter * steps;
  double* X = (gs && os == 0) ? xout : L.t;               // GS sweeps in place
  double* X2 = L.t2;
  if (gs) {   // pre: from x = 0, forward (SGS: then backward) sweeps
    Op z;
    z.kind = OP_ZERO; z.cls = clsW; z.n = L.n; z.out = X; z.bytes = 8.0 * L.n;
    ops->push_back(z);
    for (int s = 0; s < p.presmooth_iter; ++s) {
      sweep(true, X);
      if (sgs) sweep(false, X);
    }
  } else {    // first sweep from x = 0: X = W b (POLY: w_1 W b)
    Op o;
    o.kind = OP_BD; o.cls = clsW; o.n = nv; o.W = step_wd(L, 0, true); o.b = b; o.bs = bs; o.out = X;
    o.bytes = 32.0 * nv + 16.0 * nv + 16.0 * nv;
    if (!x1_ready) ops->push_back(o);
    for (int s = 1; s < npre; ++s) {
      ops->push_back(bsr_op(L.Ab, EPI_BJAC, clsS, tagA, X, 0, X, b, bs, step_wd(L, s, true), X2, 0));
      std::swap(X, X2);
    }
  }
  ops->push_back(bsr_op(L.Ab, EPI_RESID, l0 ? C_L0_RESID : C_COARSE, tagA, X, 0, nullptr, b, bs,
                        nullptr, L.r, 0));
  ops->push_back(bsr_op(L.Rb, EPI_Y, l0 ? C_L0_R : C_COARSE, tagA, L.r, 0, nullptr, nullptr, 0,
                        nullptr, C.b, 0));
  ops->back().remap = 1;
  // the coarse level's first sweep in the restriction's epilogue (launch path,
  // bsr2_kernel layouts only; the tail programs keep their own T_BD)
  const bool ybd = (g_fuse_rbd == 1 || (g_fuse_rbd == 2 && l > 0)) && tail_ok && starts_with_bd(h, l + 1) &&
                   !L.Rb.sell && !L.Rb.half && !L.Rb.sym && !L.Rb.split;
  if (ybd) {
    Op& r = ops->back();
    r.epi = EPI_YBD;
    r.W = step_wd(C, 0, true);
    r.y = C.t;
    r.bytes += 48.0 * (double)(C.n / 2);   // W_c read, x1_c written
  }
  cycle_ops_bsr(h, l + 1, C.b, 0, C.x, 0, ops, tail_ok, ybd);
  if (p.cycle_type == MAMG_W_CYCLE && !C.coarsest) {
    ops->push_back(bsr_op(C.Ab, EPI_RESID, C_MISC, 1, C.x, 0, nullptr, C.b, 0, nullptr, C.c, 0));
    cycle_ops_bsr(h, l + 1, C.c, 0, C.e, 0, ops, tail_ok);
    ops->push_back(axpy_op(C.n, C.e, C.x));
  }
  if (p.coarse_scaling) scale_ops(h, l + 1, ops);
  if (gs) {   // prolongate, then backward (SGS: forward then backward) sweeps
    ops->push_back(bsr_op(L.Pb, EPI_YADD, l0 ? C_L0_P : C_COARSE, tagA, C.x, 0, X, nullptr, 0, nullptr, X, 0));
    for (int s = 0; s < p.postsmooth_iter; ++s) {
      if (sgs) sweep(true, X);
      sweep(false, X);
    }
    if (X != xout) {
      Op o;
      o.kind = OP_ILV; o.epi = 1; o.cls = clsW; o.n = nv; o.b = X; o.out = xout; o.os = os;
      o.bytes = 32.0 * nv;
      ops->push_back(o);
    }
    return;
  }
  int s0 = 0;
  if (L.KPb.nr > 0 && npost >= 1) {   // z = x1 + W r1 + K e (one operator, K built with this W)
    const bool last = npost == 1;
    ops->push_back(bsr_op(L.KPb, EPI_KPOST, clsS, tagA, C.x, 0, X, L.r, 0, step_wd(L, 0, false),
                          last ? xout : X2, last ? os : 0));
    if (!last) std::swap(X, X2);
    s0 = 1;
  } else if (L.PAb.nr > 0 && npost >= 1) {   // prolongation + first post sweep
    const bool last = npost == 1;
    ops->push_back(post_op(L.PAb, L.r, step_wd(L, 0, false), clsS, tagA, C.x, X, last ? xout : X2,
                           last ? os : 0));
    if (!last) std::swap(X, X2);
    s0 = 1;
  } else {
    ops->push_back(bsr_op(L.Pb, EPI_YADD, l0 ? C_L0_P : C_COARSE, tagA, C.x, 0, X, nullptr, 0,
                          nullptr, X, 0));
  }
  for (int s = s0; s < npost; ++s) {
    const bool last = s == npost - 1;
    double* out = last ? xout : X2;
    ops->push_back(bsr_op(L.Ab, EPI_BJAC, clsS, tagA, X, 0, X, b, bs, step_wd(L, s, false), out,
                          last ? os : 0));
    if (!last) std::swap(X, X2);
  }
}

void apply_ops(const DeviceHandle* h, const double* r, double* z, std::vector<Op>* ops) {
  ops->clear();
  const DLevel& L0 = h->L[0];
  if (h->bsr && !L0.coarsest) {
    const int64_t nv = L0.n / 2;
    cycle_ops_bsr(h, 0, r, nv, z, nv, ops);
    for (int it = 1; it < h->p.maxit; ++it) {   // z += MG(r - A z), field-major
      ops->push_back(bsr_op(L0.Ab, EPI_RESID, C_MISC, 1, z, nv, nullptr, r, nv, nullptr, L0.c, nv));
      cycle_ops_bsr(h, 0, L0.c, nv, L0.e, nv, ops);
      ops->push_back(axpy_op(L0.n, L0.e, z));
    }
    return;
  }
  cycle_ops_csr(h, 0, r, z, ops);
  for (int it = 1; it < h->p.maxit; ++it) {
    ops->push_back(csr_op(L0.A, EPI_RESID, C_MISC, 1, z, nullptr, r, nullptr, L0.c));
    cycle_ops_csr(h, 0, L0.c, L0.e, ops);
    ops->push_back(axpy_op(L0.n, L0.e, z));
  }
}

// y = A0 x / r = b - A0 x on caller-layout vectors (PCG, spmv)
Op a0_op(const DeviceHandle* h, int epi, const double* x, const double* b, double* out) {
  const DLevel& L0 = h->L[0];
  if (h->bsr && L0.Ab.nr > 0) {
    const int64_t nv = L0.n / 2;
    return bsr_op(L0.Ab, epi, C_MISC, 1, x, nv, nullptr, b, nv, nullptr, out, nv);
  }
  return csr_op(L0.A, epi, C_MISC, 1, x, nullptr, b, nullptr, out);
}

template <int VL, int TAG>
void launch_csr_vl(const Op& o, hipStream_t s) {
  const DCsr& M = *o.M;
  const unsigned g = nblocks(M.n * (int64_t)VL);
  if (g == 0) return;
  switch (o.epi) {
    case EPI_Y:
      csr_kernel<VL, EPI_Y, TAG><<<g, 256, 0, s>>>(M.n, M.ptr, M.col, M.val, o.x, o.y, o.b, o.w, o.out);
      break;
    case EPI_YADD:
      csr_kernel<VL, EPI_YADD, TAG><<<g, 256, 0, s>>>(M.n, M.ptr, M.col, M.val, o.x, o.y, o.b, o.w, o.out);
      break;
    case EPI_RESID:
      csr_kernel<VL, EPI_RESID, TAG><<<g, 256, 0, s>>>(M.n, M.ptr, M.col, M.val, o.x, o.y, o.b, o.w, o.out);
      break;
    default:
      csr_kernel<VL, EPI_JACOBI, TAG><<<g, 256, 0, s>>>(M.n, M.ptr, M.col, M.val, o.x, o.y, o.b, o.w, o.out);
      break;
  }
}

template <int TAG>
void launch_csr_tag(const Op& o, hipStream_t s) {
  switch (o.M->lanes) {
    case 2: launch_csr_vl<2, TAG>(o, s); break;
    case 4: launch_csr_vl<4, TAG>(o, s); break;
    case 8: launch_csr_vl<8, TAG>(o, s); break;
    case 16: launch_csr_vl<16, TAG>(o, s); break;
    case 32: launch_csr_vl<32, TAG>(o, s); break;
    default: launch_csr_vl<64, TAG>(o, s); break;
  }
}

// rows [o.r0, o.r1) when o.r1 >= 0 (the distributed K's overlap split: r0 a
// multiple of 256, r1 too or = nr, so each workgroup's rows lie in the range)
template <int VL, bool XFM, bool SYM, int TAG>
void launch_bsr_x(const Op& o, hipStream_t s) {
  const DBsr& M = *o.Mb;
  const bool rng = o.r1 >= 0;
  const int64_t r0 = rng ? o.r0 : 0, r1 = rng ? o.r1 : M.nr;
  if (r1 <= r0) return;
  const int64_t b0 = r0 * VL / 256;
  const unsigned g = (unsigned)(nblocks(r1 * (int64_t)VL) - b0);
#define BSR_ARGS r1, M.ptr, M.col, M.val, o.x, o.xs, o.y, o.b, o.bs, o.W, o.out, o.os, remap_of(o), \
    (!rng && M.rsched && M.rsched_vl == VL && (int64_t)g == M.nrsched) ? M.rsched : nullptr, b0
  switch (o.epi) {
    case EPI_Y: bsr2_kernel<VL, EPI_Y, XFM, SYM, TAG><<<g, 256, 0, s>>>(BSR_ARGS); break;
    case EPI_YBD:   // restrictions only: node-interleaved, never symmetric
      if constexpr (!XFM && !SYM) bsr2_kernel<VL, EPI_YBD, false, false, TAG><<<g, 256, 0, s>>>(BSR_ARGS);
      break;
    case EPI_YADD: bsr2_kernel<VL, EPI_YADD, XFM, SYM, TAG><<<g, 256, 0, s>>>(BSR_ARGS); break;
    case EPI_RESID: bsr2_kernel<VL, EPI_RESID, XFM, SYM, TAG><<<g, 256, 0, s>>>(BSR_ARGS); break;
    case EPI_KPOST:   // K is never symmetric and e is node-major
      if constexpr (!XFM && !SYM) bsr2_kernel<VL, EPI_KPOST, false, false, TAG><<<g, 256, 0, s>>>(BSR_ARGS);
      break;
    default: bsr2_kernel<VL, EPI_BJAC, XFM, SYM, TAG><<<g, 256, 0, s>>>(BSR_ARGS); break;
  }
#undef BSR_ARGS
}

template <bool XFM, bool SYM, int U, bool NT, int TAG>
void launch_sell_u(const Op& o, hipStream_t s) {
  const DBsr& M = *o.Mb;
  const unsigned g = nblocks(M.nr);
  if (g == 0) return;
#define SELL_ARGS M.nr, M.soff, M.meta, M.col, M.val, M.nbs, o.x, o.xs, o.y, o.b, o.bs, o.W, o.out, o.os, \
    0, \
    ((int64_t)g == M.nsched ? M.sched : nullptr), M.lsort ? 1 : 0
  switch (o.epi) {
    case EPI_Y: sell2_kernel<EPI_Y, XFM, SYM, U, NT, TAG><<<g, 256, 0, s>>>(SELL_ARGS); break;
    case EPI_YADD: sell2_kernel<EPI_YADD, XFM, SYM, U, NT, TAG><<<g, 256, 0, s>>>(SELL_ARGS); break;
    case EPI_RESID: sell2_kernel<EPI_RESID, XFM, SYM, U, NT, TAG><<<g, 256, 0, s>>>(SELL_ARGS); break;
    case EPI_KPOST:
      if constexpr (!XFM && !SYM) sell2_kernel<EPI_KPOST, false, false, U, NT, TAG><<<g, 256, 0, s>>>(SELL_ARGS);
      break;
    default: sell2_kernel<EPI_BJAC, XFM, SYM, U, NT, TAG><<<g, 256, 0, s>>>(SELL_ARGS); break;
  }
#undef SELL_ARGS
}

// rows [o.r0, o.r1) when o.r1 >= 0: the bounds are multiples of 256 (or
// r1 = nr), so every workgroup of every LPR covers whole 64-row slices of
// the range (dist K_ROWS_ALIGN)
template <int LPR, int U, bool XFM, bool SYM, int SPL, int TAG, int PROBE = 0>
void launch_msell(const Op& o, hipStream_t s) {
  const DBsr& M = *o.Mb;
  const int64_t rows = 256 / LPR;
  const int64_t r0 = o.r1 < 0 ? 0 : o.r0, r1 = o.r1 < 0 ? M.nr : o.r1;
  if (r1 <= r0) return;
  const int64_t b0 = r0 / rows;
  const unsigned g = (unsigned)((r1 + rows - 1) / rows - b0);
#define MSELL_ARGS r1, M.soff, M.meta, M.col, M.val, M.nbs, o.x, o.xs, o.y, o.b, o.bs, o.W, o.out, o.os, \
    (TAG == 0 && g_kvar == 3) ? 1 : 0, M.lsort ? 1 : 0, b0, M.col16, M.cbase
  switch (o.epi) {
    case EPI_Y: msell_kernel<LPR, U, EPI_Y, XFM, SYM, SPL, TAG, PROBE><<<g, 256, 0, s>>>(MSELL_ARGS); break;
    case EPI_YADD: msell_kernel<LPR, U, EPI_YADD, XFM, SYM, SPL, TAG, PROBE><<<g, 256, 0, s>>>(MSELL_ARGS); break;
    case EPI_RESID: msell_kernel<LPR, U, EPI_RESID, XFM, SYM, SPL, TAG, PROBE><<<g, 256, 0, s>>>(MSELL_ARGS); break;
    case EPI_KPOST:
      if constexpr (!XFM && !SYM) {
        if (TAG == 0 && PROBE == 0 && M.col16)   // level-0 K with 16-bit columns (compress_sell_cols)
          msell_kernel<LPR, U, EPI_KPOST, false, false, SPL, TAG, 0, true><<<g, 256, 0, s>>>(MSELL_ARGS);
        else
          msell_kernel<LPR, U, EPI_KPOST, false, false, SPL, TAG, PROBE><<<g, 256, 0, s>>>(MSELL_ARGS);
      }
      break;
    default: msell_kernel<LPR, U, EPI_BJAC, XFM, SYM, SPL, TAG, PROBE><<<g, 256, 0, s>>>(MSELL_ARGS); break;
  }
#undef MSELL_ARGS
}

// the level-0 K kernel (MAMG_K_VARIANT for A/Bs, read at upload and by
// mamg_time_apply): 0 two lanes per row, chunks of 5 (default); 1 one lane
// per row, chunks of 6 (sell2_kernel, round 2); 2 four lanes per row, chunks
// of 3; 4 / 5 the default with non-temporal loads of the columns and values /
// the values only (the K stream kept from evicting the gathered e from L2);
// 9 a probe without the e gathers (wrong results, timing only)
template <int SPL>
bool launch_kvariant(const Op& o, hipStream_t s) {
  switch (g_kvar) {
    case 4: launch_msell<2, 5, false, false, SPL, 0, 2>(o, s); return true;
    case 5: launch_msell<2, 5, false, false, SPL, 0, 3>(o, s); return true;
    case 1: return SPL == 2 ? (launch_msell<1, 6, false, false, SPL, 0>(o, s), true) : false;
    case 2: launch_msell<4, 3, false, false, SPL, 0>(o, s); return true;
    case 3: launch_msell<2, 5, false, false, SPL, 0>(o, s); return true;   // XCD-contiguous rows
    case 9: launch_msell<2, 5, false, false, SPL, 0, 1>(o, s); return true;
    default: launch_msell<2, 5, false, false, SPL, 0>(o, s); return true;
  }
}

// whether the level-0 K launch honours an op's row range [r0, r1) (the
// multi-lane SELL and lane-group kernels do; launch_sell_u, reached only with
// the diagnosis build's MAMG_K_VARIANT=1 on a K not split in two streams,
// does not): the distributed apply splits K around the coarse halo only then
// 
bool k_ranges_ok(const DBsr& K) { return !K.sell || !(g_kvar == 1 && K.split != 2); }

template <bool XFM, bool SYM, int TAG>
void launch_sell_x(const Op& o, hipStream_t s) {
  // level-0 K operator: two lanes per row (launch_kvariant); multi-lane SELL
  // coarse operators: lanes per row from the mean row length; everything else
  // one lane, chunks of 8
  if constexpr (TAG == 0 && !XFM && !SYM) {
    if (o.epi == EPI_KPOST && (o.Mb->split == 2   ? launch_kvariant<2>(o, s)
                               : o.Mb->split ? launch_kvariant<1>(o, s)
                                             : launch_kvariant<0>(o, s)))
      return;
  }
  if constexpr (!XFM) {
    if (o.Mb->lpr > 1 && !o.Mb->split) {
      switch (o.Mb->lpr) {
        case 2: launch_msell<2, 5, false, SYM, false, TAG>(o, s); return;
        case 4: launch_msell<4, 5, false, SYM, false, TAG>(o, s); return;
        case 8: launch_msell<8, 5, false, SYM, false, TAG>(o, s); return;
        default: launch_msell<16, 5, false, SYM, false, TAG>(o, s); return;
      }
    }
  }
  if (o.Mb->split && TAG == 0) launch_sell_u<XFM, SYM, g_post_u, true, TAG>(o, s);
  else if (o.Mb->split) launch_sell_u<XFM, SYM, g_sell_u, true, TAG>(o, s);
  else if (TAG == 0 && o.epi == EPI_KPOST) launch_sell_u<XFM, SYM, g_post_u, false, TAG>(o, s);
  else launch_sell_u<XFM, SYM, g_sell_u, false, TAG>(o, s);
}

template <int TAG>
void launch_sell(const Op& o, hipStream_t s) {
  if (o.Mb->sym) {
    if (o.xfm) launch_sell_x<true, true, TAG>(o, s); else launch_sell_x<false, true, TAG>(o, s);
  } else {
    if (o.xfm) launch_sell_x<true, false, TAG>(o, s); else launch_sell_x<false, false, TAG>(o, s);
  }
}

template <int VL, int TAG>
void launch_bsr_vl(const Op& o, hipStream_t s) {
  if (o.Mb->sym) {
    if (o.xfm) launch_bsr_x<VL, true, true, TAG>(o, s); else launch_bsr_x<VL, false, true, TAG>(o, s);
  } else {
    if (o.xfm) launch_bsr_x<VL, true, false, TAG>(o, s); else launch_bsr_x<VL, false, false, TAG>(o, s);
  }
}

template <int VL, int TAG>
void launch_post_vl(const Op& o, hipStream_t s) {
  const DBsr& M = *o.Mb;
  const unsigned g = nblocks(M.nr * (int64_t)VL);
  if (g == 0) return;
  bsr2_post_kernel<VL, false, TAG><<<g, 256, 0, s>>>(M.nr, M.ptr, M.col, M.val, o.x, o.y, o.b, o.W,
                                                       o.out, o.os, remap_of(o));
}

template <int TAG>
void launch_post_tag(const Op& o, hipStream_t s) {
  if (o.Mb->sell) {
    const DBsr& M = *o.Mb;
    if (M.nr)
      sell2_post_kernel<TAG><<<nblocks(M.nr), 256, 0, s>>>(M.nr, M.soff, M.meta, M.perm, M.col, M.val,
                                                           o.x, o.y, o.b, o.W, o.out, o.os);
    return;
  }
  switch (o.Mb->lanes) {
    case 2: launch_post_vl<2, TAG>(o, s); break;
    case 4: launch_post_vl<4, TAG>(o, s); break;
    case 8: launch_post_vl<8, TAG>(o, s); break;
    case 16: launch_post_vl<16, TAG>(o, s); break;
    case 32: launch_post_vl<32, TAG>(o, s); break;
    default: launch_post_vl<64, TAG>(o, s); break;
  }
}

template <bool XFM, int U, bool GH, int TAG>
void launch_half_u(const Op& o, hipStream_t s) {
  const DBsr& M = *o.Mb;
  const int64_t r0 = o.r1 < 0 ? 0 : o.r0, r1 = o.r1 < 0 ? M.nr : o.r1;
  const unsigned g = nblocks(r1 - r0);
  if (r1 <= r0) return;
#define HALF_ARGS r0, r1, M.meta, M.col, M.val, M.nbs, M.hwu, M.lptr, M.hwl, M.gsoff, M.gcol, M.gval, M.ngs, \
    o.x, o.xs, o.y, o.b, o.bs, o.W, o.out, o.os, 1, \
    (r0 == 0 && r1 == M.nr && (int64_t)g == M.nsched) ? M.sched \
    : (r0 == M.sr0 && r1 == M.sr1 && (int64_t)g == M.nsched_r) ? M.sched_r : nullptr
  switch (o.epi) {
    case EPI_Y: hsell2_kernel<EPI_Y, XFM, U, GH, TAG><<<g, 256, 0, s>>>(HALF_ARGS); break;
    case EPI_YADD: hsell2_kernel<EPI_YADD, XFM, U, GH, TAG><<<g, 256, 0, s>>>(HALF_ARGS); break;
    case EPI_RESID: hsell2_kernel<EPI_RESID, XFM, U, GH, TAG><<<g, 256, 0, s>>>(HALF_ARGS); break;
    case EPI_KPOST: break;   // A is never the K operator
    default: hsell2_kernel<EPI_BJAC, XFM, U, GH, TAG><<<g, 256, 0, s>>>(HALF_ARGS); break;
  }
#undef HALF_ARGS
}

template <bool XFM, bool GH, int TAG>
void launch_half_x(const Op& o, hipStream_t s) {
  launch_half_u<XFM, 4, GH, TAG>(o, s);
}

template <int TAG>
void launch_half(const Op& o, hipStream_t s) {
  const bool gh = o.Mb->ngs > 0;
  if (o.xfm) {
    if (gh) launch_half_x<true, true, TAG>(o, s); else launch_half_x<true, false, TAG>(o, s);
  } else {
    if (gh) launch_half_x<false, true, TAG>(o, s); else launch_half_x<false, false, TAG>(o, s);
  }
}

template <int TAG>
void launch_bsr_tag(const Op& o, hipStream_t s) {
  if (o.Mb->half) { launch_half<TAG>(o, s); return; }
  if (o.Mb->sell) { launch_sell<TAG>(o, s); return; }
  switch (o.Mb->lanes) {
    case 2: launch_bsr_vl<2, TAG>(o, s); break;
    case 4: launch_bsr_vl<4, TAG>(o, s); break;
    case 8: launch_bsr_vl<8, TAG>(o, s); break;
    case 16: launch_bsr_vl<16, TAG>(o, s); break;
    case 32: launch_bsr_vl<32, TAG>(o, s); break;
    default: launch_bsr_vl<64, TAG>(o, s); break;
  }
}

template <int VL>
void launch_gs_vl(const Op& o, hipStream_t s) {
  const DBsr& M = *o.Mb;
  const unsigned g = nblocks(o.n * (int64_t)VL);
  if (M.sym)
    gs2_kernel<VL, true><<<g, 256, 0, s>>>(o.r0, o.r1, o.perm, M.ptr, M.col, M.val, M.nb, o.W, o.out, o.b, o.bs);
  else
    gs2_kernel<VL, false><<<g, 256, 0, s>>>(o.r0, o.r1, o.perm, M.ptr, M.col, M.val, M.nb, o.W, o.out, o.b, o.bs);
}

void launch_gs(const Op& o, hipStream_t s) {
  switch (o.Mb->lanes) {
    case 2: launch_gs_vl<2>(o, s); break;
    case 4: launch_gs_vl<4>(o, s); break;
    case 8: launch_gs_vl<8>(o, s); break;
    case 16: launch_gs_vl<16>(o, s); break;
    case 32: launch_gs_vl<32>(o, s); break;
    default: launch_gs_vl<64>(o, s); break;
  }
}

void launch(const Op& o, hipStream_t s) {
  switch (o.kind) {
    case OP_CSR:
      if (o.tag == 0) launch_csr_tag<0>(o, s); else launch_csr_tag<1>(o, s);
      break;
    case OP_BSR:
      if (o.tag == 0) launch_bsr_tag<0>(o, s); else launch_bsr_tag<1>(o, s);
      break;
    case OP_POST:
      if (o.tag == 0) launch_post_tag<0>(o, s); else launch_post_tag<1>(o, s);
      break;
    case OP_BD:
      if (o.n) bd2_kernel<false><<<nblocks(o.n), 256, 0, s>>>(o.n, o.W, o.b, o.bs, nullptr, o.out, 0);
      break;
    case OP_SCALE:
      if (o.n) scale_kernel<<<nblocks(o.n), 256, 0, s>>>(o.n, o.w, o.x, o.out);
      break;
    case OP_AXPY:
      if (o.n) axpy_kernel<<<nblocks(o.n), 256, 0, s>>>(o.n, o.x, o.out);
      break;
    case OP_GEMV:
      if (o.n) gemv_kernel<<<(unsigned)((o.n + 3) / 4), 256, 0, s>>>(o.n, o.w, o.x, o.out);
      break;
    case OP_ILV:
      if (o.n && o.epi == 1) deinterleave2_kernel<<<nblocks(o.n), 256, 0, s>>>(o.n, o.b, o.out, o.os);
      else if (o.n) interleave2_kernel<<<nblocks(o.n), 256, 0, s>>>(o.n, o.b, o.bs, o.out);
      break;
    case OP_GS:
      if (o.n > 0) launch_gs(o, s);
      break;
    case OP_PATCH:
      if (o.n > 0)
        patch_kernel<<<(unsigned)((o.n + 3) / 4), 256, 0, s>>>(o.r0, o.r1, o.lev->pperm, o.lev->Sptr, o.lev->Scol,
                                                                o.lev->Sval, o.lev->pu, o.lev->pus, o.out, o.b, o.bs);
      break;
    case OP_RING:
      if (o.n > 0)
        ring_kernel<<<(unsigned)o.n, RING_THREADS, 0, s>>>(o.r0, o.lev->rmo, o.lev->rmem, o.lev->rio, o.lev->rinv,
                                                          o.lev->Sptr, o.lev->Scol, o.lev->Sval, o.out, o.b, o.bs);
      break;
    case OP_ZERO:
      if (o.n) (void)dev_memset(o.out, 0, o.n * sizeof(double), s);
      break;
    case OP_DOT2:
      if (o.n) dot2_partial_kernel<<<SCALE_BLOCKS, 256, 0, s>>>(o.n, o.b, o.x, o.y, o.part);
      break;
    case OP_TAIL:   // r1: bit 0 = every gathered x in LDS, bit 1 = register-resident rows
      if (o.n) tail_launch<false>((int)o.r1, o.prog, (int)o.n, o.tail_pl, (size_t)o.r0, nullptr, s);
      break;
    case OP_CSCALE:
      if (o.n) cscale_kernel<<<(unsigned)std::min<int64_t>(SCALE_BLOCKS, nblocks(o.n)), 256, 0, s>>>(o.n, SCALE_BLOCKS, o.part, o.out);
      break;
  }
}

// handle ordering (DeviceHandle::last)
int order_begin(DeviceHandle* h, hipStream_t s, std::string* err) {
  if (!h->last) HIPCHK(hipEventCreateWithFlags(&h->last, hipEventDisableTiming));
  HIPCHK(hipStreamWaitEvent(s, h->last, 0));
  return MAMG_OK;
}
int order_end(DeviceHandle* h, hipStream_t s, std::string* err) {
  if (!h->last) HIPCHK(hipEventCreateWithFlags(&h->last, hipEventDisableTiming));   // the upload's own mark
  HIPCHK(hipEventRecord(h->last, s));
  return MAMG_OK;
}

int get_graph(DeviceHandle* h, const double* r, double* z, hipGraphExec_t* exec, std::string* err) {
  for (auto& g : h->graphs)
    if (g.r == r && g.z == z) { *exec = g.exec; return MAMG_OK; }
  if (h->graphs.size() >= 16) {   // evict oldest, after every launch on the handle finished
    if (h->last) HIPCHK(hipEventSynchronize(h->last));
    auto& g = h->graphs.front();
    (void)hipGraphExecDestroy(g.exec);
    (void)hipGraphDestroy(g.graph);
    h->graphs.erase(h->graphs.begin());
  }
  std::vector<Op> ops;
  apply_ops(h, r, z, &ops);
  Graph g;
  g.r = r; g.z = z;
  std::lock_guard<std::recursive_mutex> capture_lock(capture_mutex());
  HIPCHK(hipStreamBeginCapture(h->cap, hipStreamCaptureModeThreadLocal));
  for (const Op& o : ops) launch(o, h->cap);
  HIPCHK(hipStreamEndCapture(h->cap, &g.graph));
  HIPCHK(graph_instantiate(&g.exec, g.graph));
  h->graphs.push_back(g);
  *exec = g.exec;
  return MAMG_OK;
}

// BSR2 layout usable: 2 fields, every level's smoother node-block diagonal
bool bsr_eligible(const Hierarchy& H, const CsrView& A0, const mamg_params& p) {
  if (p.num_functions != 2) return false;
  for (size_t l = 0; l < H.levels.size(); ++l) {
    const HostLevel& hl = H.levels[l];
    if (hl.n % 2) return false;
    if (hl.coarsest) continue;
    if (hl.WB.n == 0) return false;                     // point smoother: CSR path
    std::vector<double> blk;
    if (!node_blocks_of(hl.WB.view(), hl.n / 2, &blk)) return false;
  }
  (void)A0;
  return true;
}

}  // namespace

// ---------------------------------------------------------------------------
// Re-home the level-0 streams -- K values and columns (6.4 GB at nrefs=6),
// A_0's upper values and columns (4.3 GB), R_0's values (2.3 GB) -- and the
// coarser levels' operators into fresh allocations once the setup's
// temporaries are gone.  The kernels' DRAM rate depends on where these arrays
// land, for the same bytes and the same PMC traffic: as built in the
// pre-reserved arena K ran 1.59-1.71 ms; re-homed into plain allocations
// 1.48-1.68 ms (residual 1.06-1.09 vs 1.09-1.10 ms, restriction 0.51 vs
// 0.53 ms) (profiles/r02_rehome_level0.txt).  Same data:
// results are bitwise equal.
// A fresh allocation for a re-homed stream (plain hipMalloc).  Rounds 2-4
// took these from hipExtMallocWithFlags(hipDeviceMallocContiguous); with the
// setup temporaries in the library's own block cache (dmem.h), a setup made
// after a handle with contiguous re-homed arrays faulted in its first
// kernels on every run, so contiguous allocations are
// no longer made.  The K region search (select_k_region) keeps its value:
// distinct plain allocations still differ by a few percent.
void* placement_alloc(size_t b) {
  void* r = nullptr;
  if (dev_malloc(&r, b, "place") != hipSuccess) { (void)hipGetLastError(); r = nullptr; }
  return r;
}

void rehome_array(DeviceHandle* h, void** ptr, size_t b) {
  if (!*ptr || b == 0) return;
  void* r = placement_alloc(b);
  if (!r) return;
  if (dev_copy(r, *ptr, b) != hipSuccess) {
    (void)hipGetLastError();
    (void)raw_free(r);
    return;
  }
  void* old = *ptr;
  h->allocs.push_back(r);
  *ptr = r;
  const bool in_arena = (char*)old >= h->arena0 && (char*)old < h->arena1;
  auto it = std::find(h->allocs.begin(), h->allocs.end(), old);
  if (!in_arena && it != h->allocs.end()) {
    drained_free(old);
    h->allocs.erase(it);
  }
}

// values and columns of one operator (half-symmetric: the upper part)
void rehome_bsr(DeviceHandle* h, DBsr& M) {
  if (M.nr == 0) return;
  const int64_t slots = (M.sell || M.half) ? M.nbs : M.nb;
  rehome_array(h, (void**)&M.val, (size_t)slots * ((M.sym || M.half) ? 3 : 4) * sizeof(double));
  rehome_array(h, (void**)&M.col, (size_t)slots * sizeof(int32_t));
}

// Level-0 K values placed by measurement.  The K
// kernel's time follows the physical memory region its value stream (5.7 GB at
// nrefs=6) lands in: 1.37 vs 1.55 ms for the same bytes, layout and kernel,
// with identical fabric request counts and no TLB misses (bench/kplace.py,
// profiles/r03_k_placement.txt); slice order, split layouts and XCD row order
// do not remove it.  So the values are copied into up to MAMG_KREGION_TRIES
// (4) distinct fresh allocations, K is timed in each (one warm + three launches), and the fastest
// region is kept.  Same bytes: results are bitwise equal.
// Bounded (round 4): candidates are tried one at a time while the search has
// spent less than MAMG_KREGION_BUDGET_MS (200) and a quarter of the HBM stays
// free after the next copy (a co-resident caller keeps its memory); the
// losers are freed at the end (kept until then so that every candidate is a
// distinct region).
void select_k_region(DeviceHandle* h) {
  DLevel& L = h->L[0];
  DBsr& K = L.KPb;
  const size_t bytes = (size_t)K.nbs * 4 * sizeof(double);
  const char* e = opt("MAMG_KREGION_TRIES");
  const int tries = e ? std::atoi(e) : 4;
  const char* eb = opt("MAMG_KREGION_BUDGET_MS");
  const double budget = eb ? std::atof(eb) : 200.0;
  if (tries <= 1 || K.sym || !L.r || !L.t || !L.Wd || !h->L[1].x) {
    rehome_array(h, (void**)&K.val, bytes);
    return;
  }
  double* out = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (raw_malloc((void**)&out, L.n * sizeof(double), "tmp") != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
      hipEventCreate(&e1) != hipSuccess) {
    (void)hipGetLastError();
    if (out) (void)raw_free(out);
    rehome_array(h, (void**)&K.val, bytes);
    return;
  }
  const auto t0 = std::chrono::steady_clock::now();
  void* old = K.val;
  const Op op = bsr_op(K, EPI_KPOST, C_L0_SMOOTH, 0, h->L[1].x, 0, L.t, L.r, 0, L.Wd, out, L.n / 2);
  std::vector<void*> bufs;
  std::vector<float> ms;
  size_t best = 0;
  for (int t = 0; t < tries; ++t) {
    const double spent = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (t > 0 && spent > budget) break;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) { (void)hipGetLastError(); break; }
    if (fr < bytes + tot / 4) break;
    void* r = placement_alloc(bytes);
    if (!r) break;
    bufs.push_back(r);
    (void)dev_copy(r, old, bytes);
    K.val = (double*)r;
    launch(op, nullptr);
    (void)hipEventRecord(e0, nullptr);
    for (int k = 0; k < 3; ++k) launch(op, nullptr);
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float m = 1e30f;
    (void)hipEventElapsedTime(&m, e0, e1);
    ms.push_back(m);
    if (ms.back() < ms[best]) best = bufs.size() - 1;
  }
  if (bufs.empty()) {
    K.val = (double*)old;
    (void)raw_free(out);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipGetLastError();
    return;
  }
  K.val = (double*)bufs[best];
  h->allocs.push_back(bufs[best]);
  for (size_t i = 0; i < bufs.size(); ++i)
    if (i != best) drained_free(bufs[i]);
  const bool in_arena = (char*)old >= h->arena0 && (char*)old < h->arena1;
  auto it = std::find(h->allocs.begin(), h->allocs.end(), old);
  if (!in_arena && it != h->allocs.end()) {
    drained_free(old);
    h->allocs.erase(it);
  }
  drained_free(out);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipGetLastError();
  if (h->p.print_level >= 2) {
    std::fprintf(stderr, "[mamg] K value regions (ms per K launch):");
    for (float m : ms) std::fprintf(stderr, " %.4f", m / 3);
    std::fprintf(stderr, " -> %zu\n", best);
  }
  h->kregion_ms.assign(ms.begin(), ms.end());
  for (auto& m : h->kregion_ms) m /= 3.0;
  h->kregion_best = (int)best;
}

void rehome_operators(DeviceHandle* h) {
  const char* e = opt("MAMG_REHOME");   // 0: keep the operators where the layout builder put them (tests)
  if (e && std::atoi(e) == 0) return;
  if (!h->bsr || h->L.size() < 2 || h->L[0].KPb.nr < g_sell_min_rows || !h->L[0].KPb.sell) return;
  DLevel& L = h->L[0];
  auto lap = [t = std::chrono::steady_clock::now()]() mutable {
    const auto n = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(n - t).count();
    t = n;
    return ms;
  };
  select_k_region(h);            // the largest stream first, placed by measurement
  h->layout_ms[LT_KREGION] = lap();
  if (L.KPb.col16) rehome_array(h, (void**)&L.KPb.col16, (size_t)L.KPb.nbs * sizeof(uint16_t));
  else rehome_array(h, (void**)&L.KPb.col, (size_t)L.KPb.nbs * sizeof(int32_t));
  if (L.Ab.half) rehome_bsr(h, L.Ab);
  if (!L.Rb.sell && !L.Rb.sym)
    rehome_array(h, (void**)&L.Rb.val, (size_t)L.Rb.nb * 4 * sizeof(double));
  // the coarser levels' operators too (coarse levels 0.41 -> 0.395 ms per apply)
  for (size_t l = 1; l < h->L.size(); ++l) {
    DLevel& D = h->L[l];
    if (D.coarsest) break;
    for (DBsr* M : {&D.Ab, &D.KPb, &D.Rb, &D.Pb})
      if (!M->half) rehome_bsr(h, *M);
  }
  h->layout_ms[LT_REHOME] = lap();
}

// Block layout of a SELL-stored K's values: one 32-byte block per slot, or two
// 16-byte streams per slot (SPL: each wave load reads contiguous pairs).  The
// arithmetic is the same, so results are bitwise equal either way
// (test_k_block_layouts_bitwise).  Rearranged in place through a temporary.
void set_k_split(DBsr& K, int mode) {
  if (!K.sell || K.sym || K.split == mode || K.nbs == 0 || (K.nbs & 63)) return;
  void* t = nullptr;
  if (raw_malloc((void**)&t, (size_t)K.nbs * sizeof(dv4), "tmp") != hipSuccess) { (void)hipGetLastError(); return; }
  const size_t bytes = (size_t)K.nbs * sizeof(dv4);
  if (K.split) {   // back to one block per slot first
    if (K.split == 2) unsplit_local_kernel<<<nblocks(K.nbs), 256>>>(K.nbs, K.val, (dv4*)t);
    else unsplit_blocks_kernel<<<nblocks(K.nbs), 256>>>(K.nbs, reinterpret_cast<const dv2*>(K.val), (dv4*)t);
    (void)dev_copy(K.val, t, bytes);
    K.split = 0;
  }
  if (mode == 1) split_blocks_kernel<<<nblocks(K.nbs), 256>>>(K.nbs, reinterpret_cast<const dv4*>(K.val), (dv2*)t);
  if (mode == 2) split_local_kernel<<<nblocks(K.nbs), 256>>>(K.nbs, reinterpret_cast<const dv4*>(K.val), (double*)t);
  if (mode) (void)dev_copy(K.val, t, bytes);
  drained_free(t);
  K.split = mode;
}

// Round 2 chose the layout per box by timing both at upload (split 1.57 vs
// 1.71 ms on one box, the opposite on another).  With the two-lanes-per-row
// K kernel (msell_kernel) the one-block layout is kept everywhere
// (DESIGN.md section 4); MAMG_POST_K=2 forces the split layout on every
// SELL-stored K (tests), MAMG_K_LAYOUT=split|block switches level 0 at
// mamg_time_apply (A/Bs on one upload).
// the coarse tail (tail_kernel) takes over from the first level with at most
// MAMG_TAIL_NODES node rows (0 = off).  Default: off for the Jacobi-family
// smoothers and 1024 for the multicolour GS smoothers; a coarsest level alone
// stays a launch.  Measured at nrefs=6 in the bench's timed loop (DESIGN.md
// section 4.2, profiles/r03_ab_tail.txt): the Jacobi V-cycle 276.1-276.3 vs
// 277.5-277.7 applies/s without it (2-D nrefs=6: 4601 vs 4971), because one
// tail op costs ~2 us, more than the kernel boundary it replaces; the
// reference family's W-cycle, whose colour steps are the launches, 196.7 ->
// 182.5 ms per apply with it (PCG graph replay).
void set_tail_level(DeviceHandle* h) {
  h->tail_level = 0;
  const int64_t nodes = g_tail_set ? g_tail_nodes : (gs_smoother(h->p) ? 1024 : 0);
  if (!h->bsr || nodes <= 0) return;
  for (int l = 1; l < (int)h->L.size(); ++l) {
    if (h->L[l].coarsest) return;
    if (h->L[l].n / 2 <= nodes) { h->tail_level = l; return; }
  }
}

void apply_k_layout_knob(DeviceHandle* h) {
  if (!h->bsr || h->L.size() < 2 || g_post_k != 2) return;
  for (DLevel& D : h->L)
    if (!D.coarsest) set_k_split(D.KPb, 1);
}

void debug_sums(DeviceHandle* h, const char* stage, bool konly);

std::string layout_error(const mamg_params& p) {
  if (patch_schwarz(p))
    return "SCHWARZ_PATCHES needs the BSR2 layout (num_functions 2, node-block smoothers on every level)";
  if (rings_schwarz(p))
    return "SCHWARZ_RINGS needs the BSR2 layout (num_functions 2, node-block smoothers on every level)";
  return "multicolour GS/SGS smoothers need the BSR2 layout (num_functions 2, node-aligned smoother blocks)";
}

int dev_upload(const Hierarchy& H, const CsrView& A0, const mamg_params& p, DeviceHandle** out,
               std::string* err) {
  const auto t0 = std::chrono::steady_clock::now();
  std::unique_ptr<DeviceHandle> h(new DeviceHandle());
  h->p = p;
  h->device = p.device;
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (ndev <= 0) { *err = "no HIP device"; return MAMG_ERR_HIP; }
  HIPCHK(hipSetDevice(p.device));
  HIPCHK(hipStreamCreateWithFlags(&h->cap, hipStreamNonBlocking));
  const int nl = (int)H.levels.size();
  h->L.resize(nl);
  h->bsr = bsr_eligible(H, A0, p);
  read_knobs();
  if ((gs_smoother(p) || patch_schwarz(p) || rings_schwarz(p)) && !h->bsr) {
    *err = layout_error(p);
    return MAMG_ERR_UNSUPPORTED;
  }
  int rc;
  for (int l = 0; l < nl; ++l) {
    const HostLevel& hl = H.levels[l];
    DLevel& D = h->L[l];
    D.n = hl.n;
    D.coarsest = hl.coarsest;
    const CsrView Al = l == 0 ? A0 : H.A(l);
    const int lanesA = l == 0 ? p.spmv_lanes : 0;
    if (h->bsr && !(l == 0 && D.coarsest)) {
      // copy the level's CSRs up once and build the apply layouts on the device
      TmpPool T;
      LevelSrc S;
      if ((rc = upload_tmp(&T, Al, &S.A, err))) return rc;
      if (D.coarsest) {
        double* dA = nullptr;
        if ((rc = T.alloc(&dA, D.n * D.n, err))) return rc;
        HIPCHK(hipMemcpy(dA, hl.Ainv.data(), D.n * D.n * sizeof(double), hipMemcpyHostToDevice));
        S.Ainv = dA;
        if ((rc = build_bsr_level(h.get(), l, S, 0, 0, err))) return rc;
      } else {
        const int64_t nv = D.n / 2, nvc = H.levels[l + 1].n / 2;
        if ((rc = upload_tmp(&T, hl.P.view(), &S.P, err))) return rc;
        if ((rc = upload_tmp(&T, hl.R.view(), &S.R, err))) return rc;
        if (p.post_fusion && p.postsmooth_iter >= 1 && hl.AP.n == hl.n)
          if ((rc = upload_tmp(&T, hl.AP.view(), &S.AP, err))) return rc;
        std::vector<double> blk;
        node_blocks_of(hl.WB.view(), nv, &blk);
        double* dW = nullptr;
        if ((rc = T.alloc(&dW, 4 * nv, err))) return rc;
        HIPCHK(hipMemcpy(dW, blk.data(), 4 * nv * sizeof(double), hipMemcpyHostToDevice));
        S.W = dW;
        S.seeds = &H.seeds;
        if ((rc = build_bsr_level(h.get(), l, S, nvc, lanesA, err))) return rc;
      }
    } else if (D.coarsest) {     // CSR layout, or a single-level hierarchy
      if ((rc = dalloc(h.get(), &D.Ainv, D.n * D.n, err))) return rc;
      HIPCHK(hipMemcpy(D.Ainv, hl.Ainv.data(), D.n * D.n * sizeof(double), hipMemcpyHostToDevice));
      if ((rc = upload_csr(h.get(), Al, &D.A, lanesA, err))) return rc;
    } else {
      if ((rc = upload_csr(h.get(), Al, &D.A, lanesA, err))) return rc;
      if ((rc = upload_csr(h.get(), hl.P.view(), &D.P, 0, err))) return rc;
      if ((rc = upload_csr(h.get(), hl.R.view(), &D.R, 0, err))) return rc;
      if (hl.WB.n > 0) {
        if ((rc = upload_csr(h.get(), hl.WB.view(), &D.WB, 0, err))) return rc;
      } else {
        if ((rc = dalloc(h.get(), &D.winv, D.n, err))) return rc;
        HIPCHK(hipMemcpy(D.winv, hl.winv.data(), D.n * sizeof(double), hipMemcpyHostToDevice));
      }
      if (p.smoother == MAMG_SMOOTHER_POLY) {   // step smoothers w_k W (values only)
        std::vector<double*> wk;
        if ((rc = poly_scaled(h.get(), hl.WB.n > 0 ? D.WB.val : D.winv, hl.WB.n > 0 ? D.WB.nnz : D.n, &wk,
                              err)))
          return rc;
        for (double* q : wk) {
          if (hl.WB.n > 0) {
            DCsr c = D.WB;
            c.val = q;
            D.WBk.push_back(c);
          } else {
            D.winvk.push_back(q);
          }
        }
      }
    }
    double** vecs[] = {&D.b, &D.x, &D.t, &D.t2, &D.r, &D.c, &D.e};
    for (double** v : vecs)
      if ((rc = dalloc(h.get(), v, D.n, err))) return rc;
    if (p.coarse_scaling) {
      if ((rc = dalloc(h.get(), &D.q, D.n, err))) return rc;
      if ((rc = dalloc(h.get(), &D.part2, 2 * SCALE_BLOCKS, err))) return rc;
    }
  }
  const int64_t n0 = h->L[0].n;
  double** v0[] = {&h->hr, &h->hz};
  for (double** v : v0)
    if ((rc = dalloc(h.get(), v, n0, err))) return rc;
  std::vector<Op> ops;
  apply_ops(h.get(), h->hr, h->hz, &ops);
  for (const Op& o : ops) h->apply_bytes += o.bytes;
  HIPCHK(null_sync());
  const auto t1 = std::chrono::steady_clock::now();
  h->layout_ms[LT_BUILD] = std::chrono::duration<double, std::milli>(t1 - t0).count();
  debug_sums(h.get(), "pre-rehome", true);
  rehome_operators(h.get());
  debug_sums(h.get(), "post-rehome", true);
  const auto t2 = std::chrono::steady_clock::now();
  apply_k_layout_knob(h.get());
  set_tail_level(h.get());
  // every layout kernel and device-to-device copy (null stream) ordered
  // before the handle's first use on any stream (order_begin waits on it)
  if ((rc = order_end(h.get(), nullptr, err))) return rc;
  HIPCHK(hipEventSynchronize(h->last));
  debug_sums(h.get(), "upload", false);
  h->layout_ms[LT_FINISH] =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t2).count();
  *out = h.release();
  return MAMG_OK;
}

// HBM reserved before the GPU setup churns memory: the apply layout is then
// bump-allocated from it (dev_from_ghier / dist_upload adopt it).  Measured at
// nrefs=6, fresh processes: K kernel 1.47-1.50 ms from the reservation vs
// 1.61-1.71 ms from hipMallocs made after the setup's alloc/free churn
// (profiles/r01_bench_prereserve_ab.log).  Bytes per A0
// entry: MAMG_PRERESERVE_B_PER_NNZ (default 20, ~16.5 used at nrefs=6; 0 = off);
// a rank of N reserves 1.25 x that / N + 0.5.
// one pending reservation per host thread (setups in different threads, e.g.
// virtual ranks or several devices, never see each other's), tagged with its
// device: a handle on another device does not adopt it
static thread_local void* g_pre = nullptr;
static thread_local size_t g_pre_bytes = 0;
static thread_local int g_pre_dev = -1;
void dev_prereserve(int device, int64_t nnz, int nranks) {
  const char* e = opt("MAMG_PRERESERVE_B_PER_NNZ");
  double b = e ? std::atof(e) : 20.0;
  if (nranks > 1) b = 1.25 * b / nranks + 0.5;
  dev_prereserve_release();
  if (b <= 0 || nnz <= 0) return;
  if (hipSetDevice(device) != hipSuccess) { (void)hipGetLastError(); return; }
  const size_t bytes = ((size_t)(b * (double)nnz) + (1 << 21)) & ~(size_t)((1 << 21) - 1);
  if (raw_malloc(&g_pre, bytes, "pre") == hipSuccess) { g_pre_bytes = bytes; g_pre_dev = device; }
  else { (void)hipGetLastError(); g_pre = nullptr; }
}
void dev_prereserve_release() {
  if (g_pre) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(g_pre_dev);
    (void)raw_free(g_pre);
    (void)hipSetDevice(cur);
  }
  g_pre = nullptr;
  g_pre_bytes = 0;
  g_pre_dev = -1;
}
template <class HT>
void adopt_prereserve(HT* h) {
  if (!g_pre || g_pre_dev != h->device) { dev_prereserve_release(); return; }
  h->allocs.push_back(g_pre);
  h->arena = (char*)g_pre;
  h->arena_left = g_pre_bytes;
  if constexpr (std::is_same<HT, DeviceHandle>::value) {
    h->arena0 = (char*)g_pre;
    h->arena1 = (char*)g_pre + g_pre_bytes;
  }
  g_pre = nullptr;
  g_pre_bytes = 0;
  g_pre_dev = -1;
}

int dev_from_ghier(GHier* G, const DevMat& A0, const mamg_params& p, DeviceHandle** out,
                   std::string* err) {
  const auto t0 = std::chrono::steady_clock::now();
  std::unique_ptr<DeviceHandle> h(new DeviceHandle());
  h->p = p;
  h->device = p.device;
  adopt_prereserve(h.get());
  HIPCHK(hipSetDevice(p.device));
  HIPCHK(hipStreamCreateWithFlags(&h->cap, hipStreamNonBlocking));
  read_knobs();
  h->bsr = !G->generic;   // a general block or point smoother: the CSR layout (as dev_upload)
  if ((gs_smoother(p) || patch_schwarz(p) || rings_schwarz(p)) && !h->bsr) {
    *err = layout_error(p);
    return MAMG_ERR_UNSUPPORTED;
  }
  const int nl = (int)G->levels.size();
  h->L.resize(nl);
  int rc;
  for (int l = 0; l < nl; ++l) {
    GLevel& g = G->levels[l];
    DLevel& D = h->L[l];
    D.n = g.n;
    D.coarsest = g.coarsest;
    if (!h->bsr) {                       // CSR layout from the device CSRs (dev_upload's CSR branch)
      if ((rc = adopt_csr(h.get(), l == 0 ? A0 : g.A, &D.A, l == 0 ? p.spmv_lanes : 0, err))) return rc;
      if (D.coarsest) {
        if ((rc = dalloc(h.get(), &D.Ainv, D.n * D.n, err))) return rc;
        HIPCHK(dev_copy(D.Ainv, g.Ainv, D.n * D.n * sizeof(double)));
      } else {
        if ((rc = adopt_csr(h.get(), g.P, &D.P, 0, err))) return rc;
        if ((rc = adopt_csr(h.get(), g.R, &D.R, 0, err))) return rc;
        if (g.WB.n > 0) {
          if ((rc = adopt_csr(h.get(), g.WB, &D.WB, 0, err))) return rc;
        } else {
          if ((rc = dalloc(h.get(), &D.winv, D.n, err))) return rc;
          HIPCHK(dev_copy(D.winv, g.winv, D.n * sizeof(double)));
        }
        if (p.smoother == MAMG_SMOOTHER_POLY) {   // step smoothers w_k W (values only)
          std::vector<double*> wk;
          const bool blk = g.WB.n > 0;
          if ((rc = poly_scaled(h.get(), blk ? D.WB.val : D.winv, blk ? D.WB.nnz : D.n, &wk, err))) return rc;
          for (double* q : wk) {
            if (blk) {
              DCsr c = D.WB;
              c.val = q;
              D.WBk.push_back(c);
            } else {
              D.winvk.push_back(q);
            }
          }
        }
      }
    } else if (l == 0 && D.coarsest) {          // single-level hierarchy: CSR A0 + dense inverse
      if ((rc = dalloc(h.get(), &D.Ainv, D.n * D.n, err))) return rc;
      HIPCHK(dev_copy(D.Ainv, g.Ainv, D.n * D.n * sizeof(double)));
      D.A.n = A0.n; D.A.m = A0.m; D.A.nnz = A0.nnz;
      D.A.lanes = p.spmv_lanes > 0 ? p.spmv_lanes : pick_lanes(A0.n, A0.nnz);
      if ((rc = dalloc(h.get(), &D.A.ptr, A0.n + 1, err))) return rc;
      if ((rc = dalloc(h.get(), &D.A.col, std::max<int64_t>(A0.nnz, 1), err))) return rc;
      if ((rc = dalloc(h.get(), &D.A.val, std::max<int64_t>(A0.nnz, 1), err))) return rc;
      HIPCHK(dev_copy(D.A.ptr, A0.ptr, (A0.n + 1) * sizeof(int64_t)));
      if (A0.nnz) {
        HIPCHK(dev_copy(D.A.col, A0.col, A0.nnz * sizeof(int32_t)));
        HIPCHK(dev_copy(D.A.val, A0.val, A0.nnz * sizeof(double)));
      }
    } else {
      LevelSrc S;
      S.A = l == 0 ? A0 : g.A;
      S.P = g.P; S.R = g.R; S.AP = g.AP; S.W = g.W; S.Ainv = g.Ainv;
      S.seeds = &G->seeds;
      const int64_t nvc = D.coarsest ? 0 : G->levels[l + 1].n / 2;
      if ((rc = build_bsr_level(h.get(), l, S, nvc, l == 0 ? p.spmv_lanes : 0, err))) return rc;
    }
    {
      char st[32];
      std::snprintf(st, sizeof st, "built-L%d", l);
      debug_sums(h.get(), st, true);
    }
    // the level's GPU-setup buffers are no longer needed (A_l stays for l+1's
    // Galerkin product only, which is done)
    for (void* q : {(void*)g.P.ptr, (void*)g.P.col, (void*)g.P.val, (void*)g.R.ptr, (void*)g.R.col,
                    (void*)g.R.val, (void*)g.AP.ptr, (void*)g.AP.col, (void*)g.AP.val, (void*)g.W,
                    (void*)g.Ainv, (void*)g.WB.ptr, (void*)g.WB.col, (void*)g.WB.val, (void*)g.winv})
      if (q) G->release(q);
    if (l > 0)
      for (void* q : {(void*)g.A.ptr, (void*)g.A.col, (void*)g.A.val})
        if (q) G->release(q);
    g.P = g.R = g.AP = g.WB = DevMat();
    g.W = g.Ainv = g.winv = nullptr;
    if (l > 0) g.A = DevMat();
    double** vecs[] = {&D.b, &D.x, &D.t, &D.t2, &D.r, &D.c, &D.e};
    for (double** v : vecs)
      if ((rc = dalloc(h.get(), v, D.n, err))) return rc;
    if (p.coarse_scaling) {
      if ((rc = dalloc(h.get(), &D.q, D.n, err))) return rc;
      if ((rc = dalloc(h.get(), &D.part2, 2 * SCALE_BLOCKS, err))) return rc;
    }
  }
  const int64_t n0 = h->L[0].n;
  double** v0[] = {&h->hr, &h->hz};
  for (double** v : v0)
    if ((rc = dalloc(h.get(), v, n0, err))) return rc;
  std::vector<Op> ops;
  apply_ops(h.get(), h->hr, h->hz, &ops);
  for (const Op& o : ops) h->apply_bytes += o.bytes;
  for (int k = 0; k < 8; ++k) h->setup_ms[k] = G->phase_ms[k];
  HIPCHK(null_sync());
  const auto t1 = std::chrono::steady_clock::now();
  h->layout_ms[LT_BUILD] = std::chrono::duration<double, std::milli>(t1 - t0).count();
  debug_sums(h.get(), "pre-rehome", true);
  rehome_operators(h.get());
  debug_sums(h.get(), "post-rehome", true);
  const auto t2 = std::chrono::steady_clock::now();
  apply_k_layout_knob(h.get());
  set_tail_level(h.get());
  if ((rc = order_end(h.get(), nullptr, err))) return rc;   // as in dev_upload
  HIPCHK(hipEventSynchronize(h->last));
  debug_sums(h.get(), "upload", false);
  const auto t3 = std::chrono::steady_clock::now();
  h->layout_ms[LT_FINISH] = std::chrono::duration<double, std::milli>(t3 - t2).count();
  h->setup_ms[GS_LAYOUT] = std::chrono::duration<double, std::milli>(t3 - t0).count();
  *out = h.release();
  return MAMG_OK;
}

void dev_setup_ms(const DeviceHandle* h, double* ms8) {
  for (int k = 0; k < 8; ++k) ms8[k] = h->setup_ms[k];
}
void dev_layout_ms(const DeviceHandle* h, double* ms4) {
  for (int k = 0; k < 4; ++k) ms4[k] = h->layout_ms[k];
}

void dev_tmp_trim() { tmp_trim_all(); }
void dev_tmp_trim_to_limit() { tmp_trim_to_limit_all(); }
void dev_set_cache_limit(int64_t bytes) { set_cache_limit(bytes); }
int64_t dev_cache_limit(int device) { return cache_limit_dev(device); }
int64_t dev_cache_idle_bytes(int device) {
  int64_t b = tmp_idle_bytes(device);
  std::lock_guard<std::mutex> g(detail::stage_mu());
  return b + (int64_t)detail::stage_pools()[device & 63].bytes;
}

void dev_destroy(DeviceHandle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  // every use of the handle (applies, PCG, timing, host applies) recorded
  // h->last on its stream: wait for that, not for the device
  if (h->last) (void)hipEventSynchronize(h->last);
  if (h->cap) (void)hipStreamSynchronize(h->cap);
  delete h;
}

int64_t dev_nrows(const DeviceHandle* h) { return h->L[0].n; }
int dev_num_levels(const DeviceHandle* h) { return (int)h->L.size(); }
double dev_apply_bytes(const DeviceHandle* h) { return h->apply_bytes; }
int dev_layout(const DeviceHandle* h) { return h->bsr ? 1 : 0; }
int dev_level_format(const DeviceHandle* h, int level) {
  const DLevel& L = h->L[level];
  return (L.Ab.sell ? MAMG_FMT_SELL : 0) | (L.Ab.sym ? MAMG_FMT_SYM : 0) | (L.Ab.half ? MAMG_FMT_HALF : 0) |
         (L.PAb.nr > 0 || L.KPb.nr > 0 ? MAMG_FMT_POST_FUSED : 0) | (L.KPb.nr > 0 ? MAMG_FMT_POST_K : 0) |
         (L.KPb.sell ? MAMG_FMT_POST_SELL : 0) | (L.Ab.nsched > 0 || L.Ab.nsched_r > 0 ? MAMG_FMT_BANDS : 0) |
         (L.pcs.size() > 1 ? MAMG_FMT_PATCHES : 0) | (L.gcs.size() > 1 ? MAMG_FMT_GS : 0) |
         (L.rcs.size() > 1 ? MAMG_FMT_RINGS : 0) | (L.Rb.nrsched > 0 ? MAMG_FMT_R_BANDS : 0) |
         (L.KPb.col16 ? MAMG_FMT_K_COL16 : 0);
}

mamg_params dev_params(const DeviceHandle* h) { return h->p; }
void dev_kregion(const DeviceHandle* h, std::vector<double>* ms, int* kept) {
  *ms = h->kregion_ms;
  *kept = h->kregion_best;
}

// MAMG_DEBUG_SUMS=1 (diagnosis): a 64-bit FNV-1a hash of every operator
// array of the handle, per level, printed to stderr at the end of the upload
// and before each apply, so two handles of one problem (which must hold the
// same bytes wherever they live) name the array that differs
void debug_sums(DeviceHandle* h, const char* stage, bool konly) {
#if MAMG_DIAG
  static const bool on = [] {
    const char* e = std::getenv("MAMG_DEBUG_SUMS");
    return e && std::atoi(e) != 0;
  }();
#else
  constexpr bool on = false;   // diagnosis build only
#endif
  if (!on) return;
  // no device-wide sync: the copies below are ordered on the null stream,
  // as every layout-builder step is
  auto hash = [](const void* p, size_t b) -> unsigned long long {
    if (!p || !b) return 0ull;
    std::vector<unsigned char> v(b);
    if (hipMemcpy(v.data(), p, b, hipMemcpyDeviceToHost) != hipSuccess) { (void)hipGetLastError(); return 1ull; }
    unsigned long long x = 1469598103934665603ull;
    for (unsigned char c : v) x = (x ^ c) * 1099511628211ull;
    return x;
  };
  std::string line;
  char buf[160];
  if (konly) {   // level 0's K values and where they live (build-time trace)
    const DBsr& K = h->L[0].KPb;
    const int64_t slots = (K.sell || K.half) ? K.nbs : K.nb;
    const int per = (K.sym || K.half) ? 3 : 4;
    const bool ar = (char*)K.val >= h->arena0 && (char*)K.val < h->arena1;
    std::fprintf(stderr, "[mamg sums] %s L0.K val %016llx at %p (%s, %lld B)\n", stage,
                 hash(K.val, (size_t)slots * per * 8), (void*)K.val, ar ? "arena" : "own", (long long)(slots * per * 8));
    return;
  }
  for (size_t l = 0; l < h->L.size(); ++l) {
    const DLevel& L = h->L[l];
    const std::pair<const char*, const DBsr*> ms[] = {{"A", &L.Ab}, {"K", &L.KPb}, {"PA", &L.PAb}, {"P", &L.Pb},
                                                      {"R", &L.Rb}, {"G", &L.Gb}};
    for (const auto& m : ms) {
      const DBsr& M = *m.second;
      if (!M.nr) continue;
      const int per = (M.sym || M.half) ? 3 : 4;
      const int64_t slots = (M.sell || M.half) ? M.nbs : M.nb;
      std::snprintf(buf, sizeof buf, " L%zu.%s val %016llx col %016llx", l, m.first,
                    hash(M.val, (size_t)slots * per * 8), hash(M.col, (size_t)slots * 4));
      line += buf;
    }
    if (L.Wd) {
      std::snprintf(buf, sizeof buf, " L%zu.W %016llx", l, hash(L.Wd, (size_t)(L.n / 2) * 32));
      line += buf;
    }
    if (L.Ainv) {
      std::snprintf(buf, sizeof buf, " L%zu.Ainv %016llx", l, hash(L.Ainv, (size_t)L.n * L.n * 8));
      line += buf;
    }
  }
  std::fprintf(stderr, "[mamg sums] %s%s\n", stage, line.c_str());
}

int dev_apply(DeviceHandle* h, const double* d_r, double* d_z, void* stream, std::string* err) {
  if (d_r == d_z) { *err = "r and z must not alias"; return MAMG_ERR_ARG; }
  debug_sums(h, "apply", false);
  HIPCHK(hipSetDevice(h->device));
  hipGraphExec_t exec;
  int rc = get_graph(h, d_r, d_z, &exec, err);
  if (rc) return rc;
  if ((rc = order_begin(h, (hipStream_t)stream, err))) return rc;
  HIPCHK(hipGraphLaunch(exec, (hipStream_t)stream));
  return order_end(h, (hipStream_t)stream, err);
}

int dev_apply_host(DeviceHandle* h, const double* r, double* z, std::string* err) {
  HIPCHK(hipSetDevice(h->device));
  const int64_t n = h->L[0].n;
  hipGraphExec_t exec;
  int rc = get_graph(h, h->hr, h->hz, &exec, err);
  if (rc) return rc;
  if ((rc = order_begin(h, h->cap, err))) return rc;   // after queued device-pointer applies
  HIPCHK(hipMemcpyAsync(h->hr, r, n * sizeof(double), hipMemcpyHostToDevice, h->cap));
  HIPCHK(hipGraphLaunch(exec, h->cap));
  HIPCHK(hipMemcpyAsync(z, h->hz, n * sizeof(double), hipMemcpyDeviceToHost, h->cap));
  if ((rc = order_end(h, h->cap, err))) return rc;
  HIPCHK(hipStreamSynchronize(h->cap));
  return MAMG_OK;
}

int dev_spmv(DeviceHandle* h, const double* d_x, double* d_y, void* stream, std::string* err) {
  HIPCHK(hipSetDevice(h->device));
  int rc = order_begin(h, (hipStream_t)stream, err);
  if (rc) return rc;
  launch(a0_op(h, EPI_Y, d_x, nullptr, d_y), (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return order_end(h, (hipStream_t)stream, err);
}


int dev_pcg(DeviceHandle* h, const double* d_b, double* d_x, double tol, int maxiter,
            int relativeconv, double* residuals, double* alphas, double* betas, int* niters,
            void* stream, std::string* err) {
  // cbc.block ConjGrad (mamg_oracle.pcg) with every scalar in HBM: one
  // iteration = one hipGraph (q = A d, <d,q>, alpha, x/r update, z = B r,
  // <r,z>, beta, stop test, d update).  The host keeps one iteration queued
  // ahead and polls the state of the previous one, so the GPU never waits
  // for a host round trip; the queued iteration after the stopping one
  // finds the state inactive and leaves x untouched.
  HIPCHK(hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = h->L[0].n;
  int rc;
  if (maxiter < 0) { *err = "maxiter must be >= 0"; return MAMG_ERR_ARG; }
  if (!h->cr) {
    double** v[] = {&h->cr, &h->cz, &h->cd, &h->cq};
    for (double** q : v)
      if ((rc = dalloc(h, q, n, err))) return rc;
    if ((rc = dalloc(h, &h->part, DOT_BLOCKS, err))) return rc;
    if ((rc = dalloc(h, &h->dres, (int64_t)((sizeof(PcgState) + 7) / 8), err))) return rc;
    HIPCHK(hipHostMalloc((void**)&h->hres, 2 * sizeof(PcgState), hipHostMallocDefault));
  }
  PcgState* st = reinterpret_cast<PcgState*>(h->dres);
  PcgState* hst = reinterpret_cast<PcgState*>(h->hres);
  const unsigned g = nblocks(n);
  if ((rc = order_begin(h, s, err))) return rc;
  // the iteration graph for (x, maxiter), captured once and kept on the
  // handle (at most 4; the oldest evicted after the handle's work is done)
  PcgGraph* pg = nullptr;
  for (auto& q : h->pcgs)
    if (q.x == d_x && q.maxiter == maxiter) pg = &q;
  if (!pg) {
    if (h->pcgs.size() >= 4) {
      if (h->last) HIPCHK(hipEventSynchronize(h->last));
      HIPCHK(hipStreamSynchronize(s));
      h->pcgs.front().release();
      h->pcgs.erase(h->pcgs.begin());
    }
    PcgGraph q;
    q.x = d_x;
    q.maxiter = maxiter;
    if (raw_malloc((void**)&q.hist, (3 * (size_t)maxiter + 1) * sizeof(double), "long") != hipSuccess) {
      (void)hipGetLastError();
      *err = "PCG history allocation failed";
      return MAMG_ERR_HIP;
    }
    double *dres = q.hist, *dal = q.hist + maxiter + 1, *dbe = dal + maxiter;
    std::vector<Op> ops;
    apply_ops(h, h->cr, h->cz, &ops);
    std::lock_guard<std::recursive_mutex> capture_lock(capture_mutex());
    hipError_t e = hipStreamBeginCapture(h->cap, hipStreamCaptureModeThreadLocal);
    if (e == hipSuccess) {
      launch(a0_op(h, EPI_Y, h->cd, nullptr, h->cq), h->cap);           // q = A d
      dot_partial_kernel<<<DOT_BLOCKS, 256, 0, h->cap>>>(n, h->cd, h->cq, h->part);
      pcg_alpha_kernel<<<1, 256, 0, h->cap>>>(DOT_BLOCKS, h->part, st);
      pcg_xr_kernel<<<g, 256, 0, h->cap>>>(n, st, h->cd, h->cq, d_x, h->cr);
      for (const Op& o : ops) launch(o, h->cap);                          // z = B r
      dot_partial_kernel<<<DOT_BLOCKS, 256, 0, h->cap>>>(n, h->cr, h->cz, h->part);
      pcg_beta_kernel<<<1, 256, 0, h->cap>>>(DOT_BLOCKS, h->part, st, dres, dal, dbe);
      pcg_d_kernel<<<g, 256, 0, h->cap>>>(n, st, h->cz, h->cd, d_x);
      e = hipStreamEndCapture(h->cap, &q.graph);
    }
    if (e == hipSuccess) e = graph_instantiate(&q.exec, q.graph);
    for (hipEvent_t& x : q.ev)
      if (e == hipSuccess) e = hipEventCreateWithFlags(&x, hipEventDisableTiming);
    if (e != hipSuccess) {
      q.release();
      *err = std::string("PCG graph: ") + hipGetErrorString(e);
      return MAMG_ERR_HIP;
    }
    h->pcgs.push_back(q);
    pg = &h->pcgs.back();
  }
  double *dres = pg->hist, *dal = pg->hist + maxiter + 1, *dbe = dal + maxiter;
  launch(a0_op(h, EPI_RESID, d_x, d_b, h->cr), s);                 // r = b - A x
  if ((rc = dev_apply(h, h->cr, h->cz, s, err))) return rc;         // z = B r
  HIPCHK(dev_copy(h->cd, h->cz, n * sizeof(double), s));
  dot_partial_kernel<<<DOT_BLOCKS, 256, 0, s>>>(n, h->cr, h->cz, h->part);
  pcg_init_kernel<<<1, 256, 0, s>>>(DOT_BLOCKS, h->part, st, tol, relativeconv, maxiter, dres);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(&hst[0], st, sizeof(PcgState), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (hst[0].status == PCG_NOT_POS) {
    *err = "Matrix is not positive";
    *niters = 0;
    (void)order_end(h, s, err);
    return MAMG_ERR_BREAKDOWN;
  }
  if (hst[0].active) {
    // iteration k's state lands in hst[k & 1]; iteration k + 1 is queued
    // before the host waits for iteration k
    for (int k = 0; k < maxiter; ++k) {
      HIPCHK(hipGraphLaunch(pg->exec, s));
      HIPCHK(hipMemcpyAsync(&hst[k & 1], st, sizeof(PcgState), hipMemcpyDeviceToHost, s));
      HIPCHK(hipEventRecord(pg->ev[k & 1], s));
      if (k == 0) continue;
      HIPCHK(hipEventSynchronize(pg->ev[(k - 1) & 1]));
      if (!hst[(k - 1) & 1].active) break;
    }
  }
  HIPCHK(hipMemcpyAsync(&hst[0], st, sizeof(PcgState), hipMemcpyDeviceToHost, s));
  if ((rc = order_end(h, s, err))) return rc;
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipGetLastError());
  const PcgState fin = hst[0];
  const int it = fin.it;
  HIPCHK(hipMemcpy(residuals, dres, (it + 1) * sizeof(double), hipMemcpyDeviceToHost));
  if (it > 0) {
    HIPCHK(hipMemcpy(alphas, dal, it * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(betas, dbe, it * sizeof(double), hipMemcpyDeviceToHost));
  }
  *niters = it;
  if (fin.status == PCG_DQ_ZERO) {   // the host loop's breakdown flag (krylov.py): same status here
    *err = "ConjGrad stopped: <d,Ad> = 0";
    return MAMG_ERR_BREAKDOWN;
  }
  if (fin.status == PCG_RZ_NEG) {
    *err = "ConjGrad breakdown (<r,Br> < 0)";
    return MAMG_ERR_BREAKDOWN;
  }
  return MAMG_OK;
}

int dev_time_apply(DeviceHandle* h, const double* d_r, double* d_z, int reps, int mode, double* ms,
                   double* kernel_ms, double* class_bytes, void* stream, std::string* err) {
  HIPCHK(hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  int rc = order_begin(h, s, err);
  if (rc) return rc;
  std::vector<Op> ops;
  apply_ops(h, d_r, d_z, &ops);
  if (class_bytes) {
    for (int c = 0; c < 16; ++c) class_bytes[c] = 0.0;
    for (const Op& o : ops) class_bytes[o.cls] += o.bytes;
  }
  if (reps <= 0) { *ms = 0.0; return MAMG_OK; }
  // events: per rep, per instrumented op, one (start, end) pair
  std::vector<int> inst;
  for (size_t k = 0; k < ops.size(); ++k)
    if (mode == 1 || ops[k].cls == C_L0_RESID || ops[k].cls == C_L0_SMOOTH) inst.push_back((int)k);
  std::vector<hipEvent_t> ev(2 * inst.size() * (size_t)reps + 2);
  for (auto& e : ev) HIPCHK(hipEventCreate(&e));
  HIPCHK(hipEventRecord(ev[0], s));
  size_t q = 2;
  for (int rp = 0; rp < reps; ++rp) {
    size_t ii = 0;
    for (size_t k = 0; k < ops.size(); ++k) {
      const bool timed = ii < inst.size() && inst[ii] == (int)k;
      if (timed) HIPCHK(hipEventRecord(ev[q], s));
      launch(ops[k], s);
      if (timed) { HIPCHK(hipEventRecord(ev[q + 1], s)); q += 2; ++ii; }
    }
  }
  HIPCHK(hipEventRecord(ev[1], s));
  if ((rc = order_end(h, s, err))) return rc;
  HIPCHK(hipEventSynchronize(ev[1]));
  HIPCHK(hipGetLastError());
  float tot = 0.f;
  HIPCHK(hipEventElapsedTime(&tot, ev[0], ev[1]));
  *ms = tot / reps;
  if (kernel_ms) {
    for (int c = 0; c < 16; ++c) kernel_ms[c] = 0.0;
    q = 2;
    for (int rp = 0; rp < reps; ++rp)
      for (size_t ii = 0; ii < inst.size(); ++ii) {
        float t = 0.f;
        HIPCHK(hipEventElapsedTime(&t, ev[q], ev[q + 1]));
        kernel_ms[ops[inst[ii]].cls] += t / reps;
        q += 2;
      }
  }
#if MAMG_DIAG
  if (mode == 1 && std::getenv("MAMG_OP_PROFILE")) {
    // diagnosis: event time per (op kind, rows) summed over one apply
    std::map<std::pair<int, int64_t>, std::pair<int, double>> acc;
    q = 2;
    for (int rp = 0; rp < reps; ++rp)
      for (size_t ii = 0; ii < inst.size(); ++ii) {
        float t = 0.f;
        HIPCHK(hipEventElapsedTime(&t, ev[q], ev[q + 1]));
        const Op& o = ops[inst[ii]];
        auto& a = acc[{o.kind, o.Mb ? o.Mb->nr : (o.M ? o.M->n : o.n)}];
        a.first += 1;
        a.second += t;
        q += 2;
      }
    for (const auto& kv : acc)
      std::fprintf(stderr, "[mamg op] kind %d rows %lld launches/apply %.1f ms/apply %.4f us/launch %.2f\n",
                   kv.first.first, (long long)kv.first.second, kv.second.first / (double)reps,
                   kv.second.second / reps, 1e3 * kv.second.second / kv.second.first);
  }
  if (std::getenv("MAMG_TAIL_PROFILE")) {
    // diagnosis: the interpreter's cost per op with nothing to do (200 ops
    // with no rows), the program in LDS and in global memory
    {
      const int nn = 200;
      std::vector<TOp> np(nn);
      for (auto& t : np) { t.kind = T_ZERO; t.n = 0; }
      TOp* dp = nullptr;
      uint64_t* dst = nullptr;
      HIPCHK(raw_malloc((void**)&dp, nn * sizeof(TOp), "tmp"));
      HIPCHK(raw_malloc((void**)&dst, 2 * (nn + 1) * sizeof(uint64_t), "tmp"));
      HIPCHK(hipMemcpy(dp, np.data(), nn * sizeof(TOp), hipMemcpyHostToDevice));
      std::vector<uint64_t> st(2 * (nn + 1));
      for (int pl : {0, -1}) {
        for (int rep = 0; rep < 3; ++rep) tail_launch<true>(0, dp, nn, pl, pl == 0 ? nn * sizeof(TOp) : 0, dst, s);
        HIPCHK(hipStreamSynchronize(s));
        HIPCHK(hipMemcpy(st.data(), dst, st.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
        std::fprintf(stderr, "[mamg tail] %d empty ops, program in %s: %.3f us/op, %.0f cycles/op\n", nn,
                     pl == 0 ? "LDS" : "global", (double)(st[nn] - st[0]) * 0.01 / nn,
                     (double)(st[2 * nn + 1] - st[nn + 1]) / nn);
      }
      // without stamps: event time of 200 vs 2000 empty ops, 512 and 64 threads
      {
        const int nb = 2000;
        std::vector<TOp> nq(nb);
        for (auto& t : nq) { t.kind = T_ZERO; t.n = 0; }
        TOp* dq = nullptr;
        HIPCHK(raw_malloc((void**)&dq, nb * sizeof(TOp), "tmp"));
        HIPCHK(hipMemcpy(dq, nq.data(), nb * sizeof(TOp), hipMemcpyHostToDevice));
        hipEvent_t e0, e1;
        HIPCHK(hipEventCreate(&e0));
        HIPCHK(hipEventCreate(&e1));
        for (int th : {TAIL_THREADS, 64}) {
          float tt[2] = {0.f, 0.f};
          for (int v = 0; v < 2; ++v) {
            const int cnt = v ? nb : nn;
            tail_kernel<false, false, false><<<1, th, 0, s>>>(dq, cnt, -1, nullptr);
            HIPCHK(hipEventRecord(e0, s));
            for (int rep = 0; rep < 10; ++rep) tail_kernel<false, false, false><<<1, th, 0, s>>>(dq, cnt, -1, nullptr);
            HIPCHK(hipEventRecord(e1, s));
            HIPCHK(hipEventSynchronize(e1));
            HIPCHK(hipEventElapsedTime(&tt[v], e0, e1));
          }
          std::fprintf(stderr, "[mamg tail] empty op without stamps, %d threads: %.3f us/op\n", th,
                       1e3 * (tt[1] - tt[0]) / 10.0 / (nb - nn));
        }
        HIPCHK(hipEventDestroy(e0));
        HIPCHK(hipEventDestroy(e1));
        (void)raw_free(dq);
      }
      (void)raw_free(dp);
      (void)raw_free(dst);
    }
    // diagnosis: wall-clock stamps after every op of each coarse-tail program
    for (const auto& tp : h->tails) {
      std::vector<TOp> prog(tp.n);
      std::vector<uint64_t> st(2 * (tp.n + 1));   // 100 MHz stamps, then shader-clock stamps
      uint64_t* dst = nullptr;
      HIPCHK(raw_malloc((void**)&dst, 2 * (tp.n + 1) * sizeof(uint64_t), "tmp"));
      HIPCHK(hipMemcpy(prog.data(), tp.prog, tp.n * sizeof(TOp), hipMemcpyDeviceToHost));
      for (int rep = 0; rep < 2; ++rep)
        tail_launch<true>((tp.xl ? 1 : 0) | (tp.res ? 2 : 0), tp.prog, tp.n, tp.prog_lds, (size_t)tp.lds, dst, s);
      HIPCHK(hipStreamSynchronize(s));
      HIPCHK(hipMemcpy(st.data(), dst, 2 * (tp.n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost));
      (void)raw_free(dst);
      std::map<std::pair<int, int64_t>, std::pair<int, double>> acc;
      for (int k = 0; k < tp.n; ++k) {
        auto& a = acc[{prog[k].kind, prog[k].n}];
        a.first += 1;
        a.second += (double)(st[k + 1] - st[k]) * 0.01;   // 100 MHz ticks -> us
      }
      const double us = (double)(st[tp.n] - st[0]) * 0.01, cyc = (double)(st[2 * tp.n + 1] - st[tp.n + 1]);
      std::fprintf(stderr, "[mamg tail] program of %d ops: %.1f us, %.0f shader cycles (%.0f MHz)\n", tp.n, us, cyc,
                   us > 0 ? cyc / us : 0.0);
      if (std::atoi(std::getenv("MAMG_TAIL_PROFILE")) > 1)
        for (int k = 0; k < tp.n; ++k)
          std::fprintf(stderr, "[mamg tail op] %d kind %d n %lld rows [%lld, %lld) vl %d lds %d us %.2f\n", k,
                       prog[k].kind, (long long)prog[k].n, (long long)prog[k].r0, (long long)prog[k].r1,
                       prog[k].vl, (int)(((uintptr_t)prog[k].x | (uintptr_t)prog[k].out) & 1),
                       (double)(st[k + 1] - st[k]) * 0.01);
      for (const auto& kv : acc)
        std::fprintf(stderr, "[mamg tail] kind %d rows %lld ops %d us %.1f us/op %.3f\n", kv.first.first,
                     (long long)kv.first.second, kv.second.first, kv.second.second,
                     kv.second.second / kv.second.first);
    }
  }
#endif  // MAMG_DIAG
  for (auto& e : ev) (void)hipEventDestroy(e);
  return MAMG_OK;
}

}  // namespace mamg

// ===========================================================================
// Multi-GPU V-cycle (row-partitioned, RCCL over xGMI).  Plan: dist.cpp.
// ===========================================================================
#include <rccl/rccl.h>

#include "dist.h"

namespace mamg {
namespace {

#define NCCLCHK(expr)                                                                \
  do {                                                                               \
    ncclResult_t r_ = (expr);                                                        \
    if (r_ != ncclSuccess) {                                                         \
      *err = std::string(#expr) + ": " + ncclGetErrorString(r_);                     \
      return MAMG_ERR_HIP;                                                           \
    }                                                                                \
  } while (0)

__global__ __launch_bounds__(256) void pack2_kernel(int64_t n, const int64_t* __restrict__ idx,
                                                    const double* __restrict__ x,
                                                    double* __restrict__ buf) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < n) {
    const double2 v = reinterpret_cast<const double2*>(x)[idx[k]];
    reinterpret_cast<double2*>(buf)[k] = v;
  }
}

// ghost slots idx[k] of x (after the nloc owned nodes) <- buf pairs
__global__ __launch_bounds__(256) void unpack2_kernel(int64_t n, const int64_t* __restrict__ idx, int64_t nloc,
                                                      const double* __restrict__ buf, double* x) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < n) reinterpret_cast<double2*>(x)[nloc + idx[k]] = reinterpret_cast<const double2*>(buf)[k];
}

__global__ __launch_bounds__(256) void addidx2_kernel(int64_t n, const int64_t* __restrict__ idx,
                                                      const double* __restrict__ buf, double* x) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < n) {
    double2* px = reinterpret_cast<double2*>(x) + idx[k];
    const double2 a = *px, v = reinterpret_cast<const double2*>(buf)[k];
    *px = make_double2(a.x + v.x, a.y + v.y);
  }
}

struct DDLevel {
  int64_t nv = 0, nloc = 0, ng = 0;
  bool replicated = false, coarsest = false;
  DBsr A, P, R;
  DBsr PA;                 // post fusion: merged [P_loc | AP_loc]
  DBsr K;                  // post fusion: K_loc = P_loc - W (AP)_loc (default)
  dv4* W = nullptr;
  std::vector<dv4*> Wk;    // SMOOTHER_POLY step smoothers w_k W (empty: Jacobi)
  double* Ainv = nullptr;
  double *b = nullptr, *x = nullptr, *t = nullptr, *t2 = nullptr, *r = nullptr;
  double *c = nullptr, *e = nullptr;     // W-cycle: second visit's right-hand side / correction
  double *q = nullptr, *part2 = nullptr; // coarse scaling of this level's correction: A e, dot partials
  double* spx = nullptr;   // level 0: [owned | ghost] operand of the standalone SpMV
  int64_t ib0 = 0, ib1 = 0;  // longest run of A_loc rows without ghost columns
  int64_t kb0 = 0, kb1 = 0;  // the same for K (coarse ghost columns), bounds multiples of K_ROWS_ALIGN or nloc
  int64_t* send_idx = nullptr;
  double *sendbuf = nullptr, *recvbuf = nullptr;
  std::vector<int64_t> send_off, ghost_off;
  // multicolour GS (SMOOTHER_GS / SGS): the owned rows permuted colour by
  // colour (gs_layout; the level's global colouring, so every rank has the
  // same colours), and each colour's halo: its send nodes and ghost slots per
  // peer, offsets cs_off / cg_off[c (P + 1) + q]
  DBsr Gb;
  int32_t* gperm = nullptr;
  dv4* Gd = nullptr;
  std::vector<int64_t> gcs, gbk;
  int64_t *csend_idx = nullptr, *cghost_idx = nullptr;
  std::vector<int64_t> cs_off, cg_off;
  // level-0 node-patch Schwarz on N ranks (dist_patches): the ghost region is
  // the 3-hop ball of the owned nodes; the rank computes every patch centred
  // within 1 hop of its nodes (pl: the patch rows of the nodes within 2 hops,
  // columns local in the global column order, centres colour by colour,
  // inverses); cs_off / cg_off above hold each colour's halo of the nodes
  // its patches write; pb = b interleaved over [owned | ghost]
  bool patches = false;
  DLevel pl;
  int32_t* Sgcol = nullptr;
  double* pb = nullptr;
  // level-0 seed-ring Schwarz on N ranks (dist_rings): the rank's blocks
  // (rl: rcs, rmo, rmem, rio, rinv; the block rows Sptr / Scol / Sval over
  // the local nodes), the ring colours' halos at cs_off / cg_off indices
  // [0, nrc), the rest GS's colours at [nrc, nrc + gcs.size() - 1)
  bool rings = false;
  int nrc = 0;
  DLevel rl;
  uint8_t* rcov = nullptr;   // covered dofs of the owned nodes (bit f)
};

// D_CHALO: the forward halo of one colour's nodes (after that colour's GS step)
enum DKind { D_OP = 0, D_HALO = 1, D_REVERSE = 2, D_ALLREDUCE = 3, D_OVERLAP = 4, D_CHALO = 5 };

struct DOp {
  int dk = D_OP;
  Op op;
  int level = 0;
  int colour = 0;            // D_CHALO
  double* buf = nullptr;
  int64_t count = 0;
  double bytes = 0.0;
  int cls = 0;
};

}  // namespace

struct DistHandle {
  mamg_params p;
  int rank = 0, nranks = 1, device = 0;
  ncclComm_t comm = nullptr;
  std::vector<DDLevel> L;
  std::vector<void*> allocs;
  char* arena = nullptr;
  size_t arena_left = 0;
  double apply_bytes = 0.0;
  int64_t nv0 = 0, o0 = 0, o1 = 0;
  bool overlap = true;                 // MAMG_OVERLAP: interior rows during the forward halo
  bool dry = false;                    // MAMG_DIST_TEST=dry: virtual rank skips its exchanges (timing only)
  hipStream_t side = nullptr;          // stream of the interior rows
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  hipEvent_t last = nullptr;           // recorded after every apply / spmv / timing (dist_destroy waits)
  // host-staged exchange backend (mamg_dist_set_exchange): pinned staging
  // per level (sends, ghost payloads, receives of the reverse-add) and one
  // all-reduce buffer
  bool host_ex = false;
  mamg_exchange ex{};
  std::vector<double*> hsend, hghost, hrecv;
  double* hred = nullptr;
  std::vector<void*> pinned;
  // the apply replayed as a hipGraph (dist_apply_graph): one per (r, z) pair,
  // captured on `cap` with the RCCL calls inside; graph_err set when a
  // capture failed (the handle then stays eager)
  struct Graph {
    const double* r;
    double* z;
    hipGraph_t g;
    hipGraphExec_t e;
  };
  std::vector<Graph> graphs;
  hipStream_t cap = nullptr;
  std::string graph_err;
  void drop_graphs() {
    for (auto& g : graphs) {
      (void)hipGraphExecDestroy(g.e);
      (void)hipGraphDestroy(g.g);
    }
    graphs.clear();
  }
  ~DistHandle() {
    if (last) (void)hipEventSynchronize(last);
    drop_graphs();
    if (cap) (void)hipStreamDestroy(cap);
    for (void* q : pinned) (void)hipHostFree(q);
    if (ev_in) (void)hipEventDestroy(ev_in);
    if (ev_out) (void)hipEventDestroy(ev_out);
    if (last) (void)hipEventDestroy(last);
    if (side) (void)hipStreamDestroy(side);
    for (void* a : allocs) (void)raw_free(a);
    if (comm) (void)ncclCommDestroy(comm);
  }
};

namespace {

template <class T>
int ddalloc(DistHandle* h, T** p, int64_t count, std::string* err) {
  *p = nullptr;
  if (count <= 0) return MAMG_OK;
  void* q = nullptr;
  HIPCHK(dev_malloc(&q, (size_t)count * sizeof(T)));
  HIPCHK(dev_memset(q, 0, (size_t)count * sizeof(T)));
  h->allocs.push_back(q);
  *p = (T*)q;
  return MAMG_OK;
}


DOp wrap(const Op& o) {
  DOp d;
  d.dk = D_OP; d.op = o; d.bytes = o.bytes; d.cls = o.cls;
  return d;
}

DOp halo_op(int level, double* x, const DDLevel& D, int cls) {
  DOp d;
  d.dk = D_HALO; d.level = level; d.buf = x; d.cls = cls;
  const int64_t ns = D.send_off.empty() ? 0 : D.send_off.back();
  d.bytes = 8.0 * ns + 16.0 * ns * 2 + 16.0 * D.ng;   // idx, pack r/w, ghost writes
  return d;
}

// forward halo of x followed by the SpMV `op` on A_loc: with the
// half-symmetric A, the ghost-free row run [ib0, ib1) (maybe empty) runs on the
// side stream while the halo is in flight (one D_OVERLAP), the rest after it.
// Every row is computed by the same kernel code either way (same bits).
void halo_residual(const DistHandle* h, int l, double* x, const Op& op, std::vector<DOp>* ops) {
  const DDLevel& D = h->L[l];
  if (!(h->overlap && D.A.half)) {
    ops->push_back(halo_op(l, x, D, C_COMM));
    ops->push_back(wrap(op));
    return;
  }
  const double f = (double)(D.ib1 - D.ib0) / (double)std::max<int64_t>(D.nloc, 1);
  DOp ov = halo_op(l, x, D, op.cls);   // timed and counted with the SpMV's class
  ov.dk = D_OVERLAP;
  ov.op = op;
  ov.op.r0 = D.ib0;
  ov.op.r1 = D.ib1;
  ov.op.bytes = op.bytes * f;
  ov.bytes += ov.op.bytes;
  ops->push_back(ov);
  const int64_t lo[2] = {0, D.ib1}, hi[2] = {D.ib0, D.nloc};
  for (int k = 0; k < 2; ++k) {   // both always emitted (possibly empty): one schedule on every rank
    Op b = op;
    b.r0 = lo[k];
    b.r1 = hi[k];
    b.bytes = op.bytes * (double)std::max<int64_t>(hi[k] - lo[k], 0) / (double)std::max<int64_t>(D.nloc, 1);
    ops->push_back(wrap(b));
  }
}

// coarse-grid correction scaling of level lc's correction C.x against C.b on
// N ranks: halo of C.x (distributed level), q = A_c x on the owned rows,
// partial sums of <b, x>, <q, x> over the owned rows, one all-reduce of the
// partials (distributed level), alpha = num / den on every rank, x <- alpha x
// on the owned rows and the ghosts (so the post step needs no second halo)
void dscale_ops(const DistHandle* h, int lc, std::vector<DOp>* ops) {
  const DDLevel& C = h->L[lc];
  const Op q = bsr_op(C.A, EPI_Y, C_MISC, 1, C.x, 0, nullptr, nullptr, 0, nullptr, C.q, 0);
  if (C.replicated) ops->push_back(wrap(q)); else halo_residual(h, lc, C.x, q, ops);
  Op d;
  d.kind = OP_DOT2; d.cls = C_MISC; d.n = 2 * C.nloc; d.b = C.b; d.x = C.x; d.y = C.q; d.part = C.part2;
  d.bytes = 24.0 * d.n;
  ops->push_back(wrap(d));
  if (!C.replicated) {
    DOp a;
    a.dk = D_ALLREDUCE; a.cls = C_COMM; a.buf = C.part2; a.count = 2 * SCALE_BLOCKS; a.bytes = 16.0 * SCALE_BLOCKS;
    ops->push_back(a);
  }
  Op sc;
  sc.kind = OP_CSCALE; sc.cls = C_MISC; sc.n = 2 * (C.nloc + C.ng); sc.part = C.part2; sc.out = C.x;
  sc.bytes = 16.0 * sc.n;
  ops->push_back(wrap(sc));
}

void dcycle_ops(const DistHandle* h, int l, const double* b, int64_t bs, double* xout, int64_t os,
                std::vector<DOp>* ops);

// coarse-grid correction of level l from its residual D.r: partial
// restriction, reverse-add (or all-reduce into a replicated level), the
// coarse cycle (W: twice), scaling, and the halo of the correction C.x
// (left to the caller when defer_halo: it overlaps that halo with K)
void dcoarse_ops(const DistHandle* h, int l, std::vector<DOp>* ops, bool defer_halo = false) {
  const DDLevel& D = h->L[l];
  const DDLevel& C = h->L[l + 1];
  const bool l0 = l == 0;
  const int tagA = l0 ? 0 : 1;
  ops->push_back(wrap(bsr_op(D.R, EPI_Y, l0 ? C_L0_R : C_COARSE, tagA, D.r, 0, nullptr, nullptr, 0,
                             nullptr, C.b, 0)));
  ops->back().op.remap = 1;
  if (!D.replicated) {
    DOp d;
    d.cls = C_COMM;
    if (C.replicated) {
      d.dk = D_ALLREDUCE; d.buf = C.b; d.count = 2 * C.nv; d.bytes = 16.0 * C.nv * 2;
    } else {
      d.dk = D_REVERSE; d.level = l + 1; d.buf = C.b;
      const int64_t ns = C.send_off.back();
      d.bytes = 16.0 * C.ng + 16.0 * ns * 3 + 8.0 * ns;
    }
    ops->push_back(d);
  }
  dcycle_ops(h, l + 1, C.b, 0, C.x, 0, ops);
  if (h->p.cycle_type == MAMG_W_CYCLE && !C.coarsest) {   // second visit on the updated residual
    const Op res = bsr_op(C.A, EPI_RESID, C_MISC, 1, C.x, 0, nullptr, C.b, 0, nullptr, C.c, 0);
    if (C.replicated) ops->push_back(wrap(res)); else halo_residual(h, l + 1, C.x, res, ops);
    dcycle_ops(h, l + 1, C.c, 0, C.e, 0, ops);
    ops->push_back(wrap(axpy_op(2 * C.nloc, C.e, C.x)));
  }
  if (h->p.coarse_scaling) dscale_ops(h, l + 1, ops);      // ghosts of C.x scaled too
  else if (!C.replicated && !defer_halo) ops->push_back(halo_op(l + 1, C.x, C, C_COMM));
}

// level 0's K with the coarse-e halo in flight: rows [kb0, kb1) (no coarse
// ghost columns) on the side stream during the halo (one D_OVERLAP), the
// rest after it; the same kernel code computes every row either way
void k_overlap(const DistHandle* h, const Op& k, std::vector<DOp>* ops) {
  const DDLevel& D = h->L[0];
  const DDLevel& C = h->L[1];
  const double n = (double)std::max<int64_t>(D.nloc, 1);
  DOp ov = halo_op(1, C.x, C, k.cls);   // timed and counted with K's class
  ov.dk = D_OVERLAP;
  ov.op = k;
  ov.op.r0 = D.kb0;
  ov.op.r1 = D.kb1;
  ov.op.bytes = k.bytes * (double)(D.kb1 - D.kb0) / n;
  ov.bytes += ov.op.bytes;
  ops->push_back(ov);
  const int64_t lo[2] = {0, D.kb1}, hi[2] = {D.kb0, D.nloc};
  for (int q = 0; q < 2; ++q) {   // both always emitted (possibly empty): one schedule on every rank
    Op b = k;
    b.r0 = lo[q];
    b.r1 = hi[q];
    b.bytes = k.bytes * (double)std::max<int64_t>(hi[q] - lo[q], 0) / n;
    ops->push_back(wrap(b));
  }
}

DOp chalo_op(int level, int c, double* x, const DDLevel& D, int P) {
  DOp d;
  d.dk = D_CHALO; d.level = level; d.colour = c; d.buf = x; d.cls = C_COMM;
  const int64_t ns = D.cs_off[(size_t)(c + 1) * (P + 1) - 1] - D.cs_off[(size_t)c * (P + 1)];
  const int64_t ng = D.cg_off[(size_t)(c + 1) * (P + 1) - 1] - D.cg_off[(size_t)c * (P + 1)];
  d.bytes = 8.0 * ns + 32.0 * ns + 8.0 * ng + 32.0 * ng;   // indices, pack, unpack
  return d;
}

// one multicolour GS sweep on the owned rows, each colour's step followed by
// that colour's halo so the next colour reads current ghosts; every rank
// emits the same exchanges, also for colours it has no rows of
void dgs_sweep(const DistHandle* h, int l, bool fwd, double* x, const double* b, int64_t bs, int cls,
               std::vector<DOp>* ops) {
  const DDLevel& D = h->L[l];
  const int nc = (int)D.gcs.size() - 1;
  for (int k = 0; k < nc; ++k) {
    const int c = fwd ? k : nc - 1 - k;
    ops->push_back(wrap(gs_op(D, c, x, b, bs, cls)));   // empty here: not launched (same schedule on every rank)
    if (!D.replicated) ops->push_back(chalo_op(l, c, x, D, h->nranks));
  }
}

// multi-GPU cycle with multicolour GS / SGS (cycle_ops_bsr's GS branch): from
// x = 0, pre sweeps, residual (ghosts current), coarse correction, x += P e,
// halo, post sweeps; X holds [owned | ghost]
void dcycle_gs(const DistHandle* h, int l, const double* b, int64_t bs, double* xout, int64_t os,
               std::vector<DOp>* ops) {
  const DDLevel& D = h->L[l];
  const DDLevel& C = h->L[l + 1];
  const bool l0 = l == 0;
  const int tagA = l0 ? 0 : 1;
  const int clsS = l0 ? C_L0_SMOOTH : C_COARSE;
  const int clsW = l0 ? C_L0_WB : C_COARSE;
  const bool sgs = h->p.smoother == MAMG_SMOOTHER_SGS;
  double* X = os == 0 ? xout : D.t;
  {
    Op z;
    z.kind = OP_ZERO; z.cls = clsW; z.n = 2 * (D.nloc + D.ng); z.out = X; z.bytes = 8.0 * z.n;
    ops->push_back(wrap(z));
  }
  for (int s = 0; s < h->p.presmooth_iter; ++s) {
    dgs_sweep(h, l, true, X, b, bs, clsS, ops);
    if (sgs) dgs_sweep(h, l, false, X, b, bs, clsS, ops);
  }
  ops->push_back(wrap(bsr_op(D.A, EPI_RESID, l0 ? C_L0_RESID : C_COARSE, tagA, X, 0, nullptr, b, bs, nullptr,
                             D.r, 0)));
  dcoarse_ops(h, l, ops);
  ops->push_back(wrap(bsr_op(D.P, EPI_YADD, l0 ? C_L0_P : C_COARSE, tagA, C.x, 0, X, nullptr, 0, nullptr, X, 0)));
  if (!D.replicated) ops->push_back(halo_op(l, X, D, C_COMM));
  for (int s = 0; s < h->p.postsmooth_iter; ++s) {
    if (sgs) dgs_sweep(h, l, true, X, b, bs, clsS, ops);
    dgs_sweep(h, l, false, X, b, bs, clsS, ops);
  }
  if (X != xout) {
    Op o;
    o.kind = OP_ILV; o.epi = 1; o.cls = clsW; o.n = D.nloc; o.b = X; o.out = xout; o.os = os;
    o.bytes = 32.0 * D.nloc;
    ops->push_back(wrap(o));
  }
}

// one node-patch sweep of level 0 on N ranks: per colour the rank's patches
// of that colour, then that colour's halo (the written nodes within 3 hops);
// every rank emits every colour's exchange, also without patches of its own
void dpatch_sweep(const DistHandle* h, bool fwd, double* x, std::vector<DOp>* ops) {
  const DDLevel& D = h->L[0];
  const int nc = (int)D.pl.pcs.size() - 1;
  for (int k = 0; k < nc; ++k) {
    const int c = fwd ? k : nc - 1 - k;
    ops->push_back(wrap(patch_op(D.pl, c, x, D.pb, 0, C_L0_SMOOTH)));   // empty: not launched
    ops->push_back(chalo_op(0, c, x, D, h->nranks));
  }
}

// multi-GPU level-0 cycle with the node-patch Schwarz (cycle_ops_bsr's
// patch branch): b interleaved over [owned | ghost] + its halo; x = 0; pre
// sweeps forward then backward; residual (ghosts current); the coarse
// correction; x += P e and its halo; post sweeps forward then backward
void dcycle_patch(const DistHandle* h, const double* b, int64_t bs, double* xout, int64_t os,
                  std::vector<DOp>* ops) {
  const DDLevel& D = h->L[0];
  const DDLevel& C = h->L[1];
  double* X = D.t;
  {
    Op o;
    o.kind = OP_ILV; o.cls = C_L0_WB; o.n = D.nloc; o.b = b; o.bs = bs; o.out = D.pb;
    o.bytes = 32.0 * D.nloc;
    ops->push_back(wrap(o));
    ops->push_back(halo_op(0, D.pb, D, C_COMM));
    Op z;
    z.kind = OP_ZERO; z.cls = C_L0_WB; z.n = 2 * (D.nloc + D.ng); z.out = X; z.bytes = 8.0 * z.n;
    ops->push_back(wrap(z));
  }
  for (int s = 0; s < h->p.presmooth_iter; ++s) {
    dpatch_sweep(h, true, X, ops);
    dpatch_sweep(h, false, X, ops);
  }
  ops->push_back(wrap(bsr_op(D.A, EPI_RESID, C_L0_RESID, 0, X, 0, nullptr, b, bs, nullptr, D.r, 0)));
  dcoarse_ops(h, 0, ops);
  ops->push_back(wrap(bsr_op(D.P, EPI_YADD, C_L0_P, 0, C.x, 0, X, nullptr, 0, nullptr, X, 0)));
  ops->push_back(halo_op(0, X, D, C_COMM));
  for (int s = 0; s < h->p.postsmooth_iter; ++s) {
    dpatch_sweep(h, true, X, ops);
    dpatch_sweep(h, false, X, ops);
  }
  Op o;
  o.kind = OP_ILV; o.epi = 1; o.cls = C_L0_WB; o.n = D.nloc; o.b = X; o.out = xout; o.os = os;
  o.bytes = 32.0 * D.nloc;
  ops->push_back(wrap(o));
}

// one symmetric level-0 seed-ring step on N ranks (the single-GPU sweep of
// cycle_ops_bsr, mamg_oracle.rings_step): forward = ring colours ascending,
// then the rest's GS colours ascending; backward = the rest descending, then
// the rings descending; each colour's step followed by its halo (every rank
// emits every exchange, also for colours it has no work in)
void dring_sweep(const DistHandle* h, bool fwd, double* x, std::vector<DOp>* ops) {
  const DDLevel& D = h->L[0];
  const int nrc = D.nrc, ngc = (int)D.gcs.size() - 1, P = h->nranks;
  auto rings = [&](bool f) {
    for (int k = 0; k < nrc; ++k) {
      const int c = f ? k : nrc - 1 - k;
      ops->push_back(wrap(ring_op(D.rl, c, x, D.pb, 0, C_L0_SMOOTH)));   // empty: not launched
      ops->push_back(chalo_op(0, c, x, D, P));
    }
  };
  auto rest = [&](bool f) {
    for (int k = 0; k < ngc; ++k) {
      const int c = f ? k : ngc - 1 - k;
      ops->push_back(wrap(gs_op(D, c, x, D.pb, 0, C_L0_SMOOTH)));
      ops->push_back(chalo_op(0, nrc + c, x, D, P));
    }
  };
  if (fwd) { rings(true); rest(true); } else { rest(false); rings(false); }
}

// multi-GPU level-0 cycle with the seed-ring Schwarz (cycle_ops_bsr's ring
// branch): b interleaved over [owned | ghost] + its halo; x = 0; pre steps
// forward then backward; residual; the coarse correction; x += P e and its
// halo; post steps forward then backward
void dcycle_rings(const DistHandle* h, const double* b, int64_t bs, double* xout, int64_t os,
                  std::vector<DOp>* ops) {
  const DDLevel& D = h->L[0];
  const DDLevel& C = h->L[1];
  double* X = D.t;
  {
    Op o;
    o.kind = OP_ILV; o.cls = C_L0_WB; o.n = D.nloc; o.b = b; o.bs = bs; o.out = D.pb;
    o.bytes = 32.0 * D.nloc;
    ops->push_back(wrap(o));
    ops->push_back(halo_op(0, D.pb, D, C_COMM));
    Op z;
    z.kind = OP_ZERO; z.cls = C_L0_WB; z.n = 2 * (D.nloc + D.ng); z.out = X; z.bytes = 8.0 * z.n;
    ops->push_back(wrap(z));
  }
  for (int s = 0; s < h->p.presmooth_iter; ++s) {
    dring_sweep(h, true, X, ops);
    dring_sweep(h, false, X, ops);
  }
  ops->push_back(wrap(bsr_op(D.A, EPI_RESID, C_L0_RESID, 0, X, 0, nullptr, b, bs, nullptr, D.r, 0)));
  dcoarse_ops(h, 0, ops);
  ops->push_back(wrap(bsr_op(D.P, EPI_YADD, C_L0_P, 0, C.x, 0, X, nullptr, 0, nullptr, X, 0)));
  ops->push_back(halo_op(0, X, D, C_COMM));
  for (int s = 0; s < h->p.postsmooth_iter; ++s) {
    dring_sweep(h, true, X, ops);
    dring_sweep(h, false, X, ops);
  }
  Op o;
  o.kind = OP_ILV; o.epi = 1; o.cls = C_L0_WB; o.n = D.nloc; o.b = X; o.out = xout; o.os = os;
  o.bytes = 32.0 * D.nloc;
  ops->push_back(wrap(o));
}

// multi-GPU cycle from x = 0 (V or W, nu1 / nu2 sweeps, optional coarse-grid
// scaling): see dist.cpp / dist_ref.py
void dcycle_ops(const DistHandle* h, int l, const double* b, int64_t bs, double* xout, int64_t os,
                std::vector<DOp>* ops) {
  if (l == 0 && h->L[0].patches) { dcycle_patch(h, b, bs, xout, os, ops); return; }
  if (l == 0 && h->L[0].rings) { dcycle_rings(h, b, bs, xout, os, ops); return; }
  if (!h->L[l].coarsest && h->L[l].gcs.size() > 1) { dcycle_gs(h, l, b, bs, xout, os, ops); return; }
  const DDLevel& D = h->L[l];
  const bool l0 = l == 0;
  const int tagA = l0 ? 0 : 1;
  if (D.coarsest) {
    Op o;
    o.kind = OP_GEMV; o.cls = C_DENSE; o.n = 2 * D.nv; o.x = b; o.w = D.Ainv; o.out = xout;
    o.bytes = 8.0 * o.n * o.n + 16.0 * o.n;
    ops->push_back(wrap(o));
    return;
  }
  const DDLevel& C = h->L[l + 1];
  const int m = smoother_steps(h->p);   // steps per smoothing (POLY: Chebyshev degree)
  const int npre = h->p.presmooth_iter * m, npost = h->p.postsmooth_iter * m;
  auto wk = [&](int s, bool pre) -> const dv4* { return D.Wk.empty() ? D.W : D.Wk[step_index(m, s, pre)]; };
  const int clsS = l0 ? C_L0_SMOOTH : C_COARSE;
  double* X = D.t;
  double* X2 = D.t2;
  {
    Op o;
    o.kind = OP_BD; o.cls = l0 ? C_L0_WB : C_COARSE; o.n = D.nloc; o.W = wk(0, true); o.b = b; o.bs = bs;
    o.out = X; o.bytes = 64.0 * D.nloc;
    ops->push_back(wrap(o));
  }
  for (int s = 1; s < npre; ++s) {   // further pre steps: halo of X, then x + w_s W (b - A x)
    const Op bj = bsr_op(D.A, EPI_BJAC, clsS, tagA, X, 0, X, b, bs, wk(s, true), X2, 0);
    if (D.replicated) ops->push_back(wrap(bj)); else halo_residual(h, l, X, bj, ops);
    std::swap(X, X2);
  }
  {
    const Op res = bsr_op(D.A, EPI_RESID, l0 ? C_L0_RESID : C_COARSE, tagA, X, 0, nullptr, b, bs, nullptr, D.r, 0);
    if (D.replicated) {
      ops->push_back(wrap(res));
    } else {
      halo_residual(h, l, X, res, ops);
    }
  }
  // K on its ghost-free rows while the coarse-e halo is in flight (level 0,
  // no coarse scaling); the schedule's shape is the same on every rank (the
  // overlap and both remainder launches are emitted, maybe empty)
  const bool kov = l == 0 && h->overlap && D.K.nr > 0 && !C.replicated && !h->p.coarse_scaling && npost >= 1 &&
                   k_ranges_ok(D.K);
  dcoarse_ops(h, l, ops, kov);
  int s0 = 0;
  if (D.K.nr > 0 || D.PA.nr > 0) {   // fused first post step (K built with its smoother), operands local
    const bool last = npost == 1;
    if (D.K.nr > 0) { // X + W r + K e
      const Op k = bsr_op(D.K, EPI_KPOST, clsS, tagA, C.x, 0, X, D.r, 0, wk(0, false), last ? xout : X2,
                          last ? os : 0);
      if (kov) k_overlap(h, k, ops); else ops->push_back(wrap(k));
    } else            // X + P e + W (r - AP e)
      ops->push_back(wrap(post_op(D.PA, D.r, wk(0, false), clsS, tagA, C.x, X, last ? xout : X2,
                                  last ? os : 0)));
    if (last) return;
    std::swap(X, X2);
    s0 = 1;
  } else {
    ops->push_back(wrap(bsr_op(D.P, EPI_YADD, l0 ? C_L0_P : C_COARSE, tagA, C.x, 0, X, nullptr, 0,
                               nullptr, X, 0)));
  }
  for (int s = s0; s < npost; ++s) {   // halo of the iterate, then x + w W (b - A x)
    const bool last = s == npost - 1;
    const Op bj = bsr_op(D.A, EPI_BJAC, clsS, tagA, X, 0, X, b, bs, wk(s, false), last ? xout : X2,
                         last ? os : 0);
    if (D.replicated) ops->push_back(wrap(bj)); else halo_residual(h, l, X, bj, ops);
    std::swap(X, X2);
  }
}

// one exchange through the host callbacks: device payloads staged in pinned
// memory around the callback (stream synchronised first), the same pack /
// unpack / rank-ordered reverse-add kernels as the RCCL branch of run_dop
int run_dop_host(DistHandle* h, const DOp& d, hipStream_t s, std::string* err) {
  const int P = h->nranks;
  std::vector<double*> snd(P, nullptr), rcv(P, nullptr);
  std::vector<int64_t> sc(P, 0), rc(P, 0);
  if (d.dk == D_ALLREDUCE) {
    HIPCHK(hipMemcpyAsync(h->hred, d.buf, d.count * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (h->ex.allreduce(h->ex.ctx, h->hred, d.count)) { *err = "exchange allreduce callback failed"; return MAMG_ERR_HIP; }
    HIPCHK(hipMemcpyAsync(d.buf, h->hred, d.count * sizeof(double), hipMemcpyHostToDevice, s));
    return MAMG_OK;
  }
  const DDLevel& D = h->L[d.level];
  const int64_t ns = D.send_off.back();
  if (d.dk == D_OVERLAP) {   // interior rows on the side stream, host halo on s, join
    HIPCHK(hipEventRecord(h->ev_in, s));
    HIPCHK(hipStreamWaitEvent(h->side, h->ev_in, 0));
    launch(d.op, h->side);
    HIPCHK(hipEventRecord(h->ev_out, h->side));
    DOp hd = d;
    hd.dk = D_HALO;
    int r = run_dop_host(h, hd, s, err);
    HIPCHK(hipStreamWaitEvent(s, h->ev_out, 0));
    return r;
  }
  double* hs = h->hsend[d.level];
  double* hg = h->hghost[d.level];
  double* hr = h->hrecv[d.level];
  if (d.dk == D_CHALO) {
    const size_t b0 = (size_t)d.colour * (P + 1);
    const int64_t s0 = D.cs_off[b0], s1 = D.cs_off[b0 + P], g0 = D.cg_off[b0], g1 = D.cg_off[b0 + P];
    for (int q = 0; q < P; ++q) {
      if (q == h->rank) continue;
      snd[q] = hs + 2 * D.cs_off[b0 + q]; sc[q] = 2 * (D.cs_off[b0 + q + 1] - D.cs_off[b0 + q]);
      rcv[q] = hg + 2 * D.cg_off[b0 + q]; rc[q] = 2 * (D.cg_off[b0 + q + 1] - D.cg_off[b0 + q]);
    }
    if (s1 > s0) {
      pack2_kernel<<<nblocks(s1 - s0), 256, 0, s>>>(s1 - s0, D.csend_idx + s0, d.buf, D.sendbuf + 2 * s0);
      HIPCHK(hipMemcpyAsync(hs + 2 * s0, D.sendbuf + 2 * s0, 2 * (s1 - s0) * sizeof(double), hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    if (h->ex.sendrecv(h->ex.ctx, P, snd.data(), sc.data(), rcv.data(), rc.data())) {
      *err = "exchange sendrecv callback failed";
      return MAMG_ERR_HIP;
    }
    if (g1 > g0) {
      HIPCHK(hipMemcpyAsync(D.recvbuf + 2 * g0, hg + 2 * g0, 2 * (g1 - g0) * sizeof(double), hipMemcpyHostToDevice, s));
      unpack2_kernel<<<nblocks(g1 - g0), 256, 0, s>>>(g1 - g0, D.cghost_idx + g0, D.nloc, D.recvbuf + 2 * g0, d.buf);
    }
    return MAMG_OK;
  }
  for (int q = 0; q < P; ++q) {
    if (q == h->rank) continue;
    const int64_t sq = D.send_off[q + 1] - D.send_off[q], gq = D.ghost_off[q + 1] - D.ghost_off[q];
    if (d.dk == D_HALO) {   // my owned values they ghost -> their ghosts of mine
      snd[q] = hs + 2 * D.send_off[q]; sc[q] = 2 * sq;
      rcv[q] = hg + 2 * D.ghost_off[q]; rc[q] = 2 * gq;
    } else {                // D_REVERSE: my ghost partials -> their owned rows
      snd[q] = hg + 2 * D.ghost_off[q]; sc[q] = 2 * gq;
      rcv[q] = hr + 2 * D.send_off[q]; rc[q] = 2 * sq;
    }
  }
  if (d.dk == D_HALO) {
    if (ns) {
      pack2_kernel<<<nblocks(ns), 256, 0, s>>>(ns, D.send_idx, d.buf, D.sendbuf);
      HIPCHK(hipMemcpyAsync(hs, D.sendbuf, 2 * ns * sizeof(double), hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    if (h->ex.sendrecv(h->ex.ctx, P, snd.data(), sc.data(), rcv.data(), rc.data())) {
      *err = "exchange sendrecv callback failed";
      return MAMG_ERR_HIP;
    }
    if (D.ng)
      HIPCHK(hipMemcpyAsync(d.buf + 2 * D.nloc, hg, 2 * D.ng * sizeof(double), hipMemcpyHostToDevice, s));
    return MAMG_OK;
  }
  // D_REVERSE
  if (D.ng) HIPCHK(hipMemcpyAsync(hg, d.buf + 2 * D.nloc, 2 * D.ng * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (h->ex.sendrecv(h->ex.ctx, P, snd.data(), sc.data(), rcv.data(), rc.data())) {
    *err = "exchange sendrecv callback failed";
    return MAMG_ERR_HIP;
  }
  if (ns) HIPCHK(hipMemcpyAsync(D.recvbuf, hr, 2 * ns * sizeof(double), hipMemcpyHostToDevice, s));
  for (int q = 0; q < P; ++q) {
    const int64_t sq = D.send_off[q + 1] - D.send_off[q];
    if (q == h->rank || !sq) continue;
    addidx2_kernel<<<nblocks(sq), 256, 0, s>>>(sq, D.send_idx + D.send_off[q], D.recvbuf + 2 * D.send_off[q], d.buf);
  }
  return MAMG_OK;
}

int run_dop(DistHandle* h, const DOp& d, hipStream_t s, std::string* err) {
  if (d.dk == D_OP) {
    launch(d.op, s);
    return MAMG_OK;
  }
  if (h->nranks == 1 && !h->comm) {     // no peers: halos empty, sums over one rank
    if (d.dk == D_OVERLAP) launch(d.op, s);
    return MAMG_OK;
  }
  // (a 1-rank RCCL communicator takes the RCCL path below: empty send /
  // receive groups, an all-reduce over one rank, the side-stream fork; the
  // one-GPU tests exercise those calls, eager and inside a graph capture)
  if (!h->comm && h->dry) {            // compute-only timing of one rank (results meaningless)
    if (d.dk == D_OVERLAP) launch(d.op, s);
    return MAMG_OK;
  }
  if (!h->comm && h->host_ex) return run_dop_host(h, d, s, err);
  if (!h->comm) {
    *err = "virtual rank handle (no communicator): use mamg_dist_virtual_apply / _spmv";
    return MAMG_ERR_ARG;
  }
  if (d.dk == D_ALLREDUCE) {
    NCCLCHK(ncclAllReduce(d.buf, d.buf, d.count, ncclDouble, ncclSum, h->comm, s));
    return MAMG_OK;
  }
  const DDLevel& D = h->L[d.level];
  const int64_t ns = D.send_off.back();
  if (d.dk == D_OVERLAP) {   // interior rows on the side stream, halo on s, join
    HIPCHK(hipEventRecord(h->ev_in, s));
    HIPCHK(hipStreamWaitEvent(h->side, h->ev_in, 0));
    launch(d.op, h->side);
    HIPCHK(hipEventRecord(h->ev_out, h->side));
    DOp hd = d;
    hd.dk = D_HALO;
    int rc = run_dop(h, hd, s, err);
    HIPCHK(hipStreamWaitEvent(s, h->ev_out, 0));
    return rc;
  }
  if (d.dk == D_CHALO) {      // one colour's nodes: pack, send / receive, unpack into the ghost slots
    const int P = h->nranks;
    const size_t b0 = (size_t)d.colour * (P + 1);
    const int64_t s0 = D.cs_off[b0], s1 = D.cs_off[b0 + P], g0 = D.cg_off[b0], g1 = D.cg_off[b0 + P];
    if (s1 > s0) pack2_kernel<<<nblocks(s1 - s0), 256, 0, s>>>(s1 - s0, D.csend_idx + s0, d.buf, D.sendbuf + 2 * s0);
    NCCLCHK(ncclGroupStart());
    for (int q = 0; q < P; ++q) {
      if (q == h->rank) continue;
      const int64_t sc = D.cs_off[b0 + q + 1] - D.cs_off[b0 + q], gc = D.cg_off[b0 + q + 1] - D.cg_off[b0 + q];
      if (sc) NCCLCHK(ncclSend(D.sendbuf + 2 * D.cs_off[b0 + q], 2 * sc, ncclDouble, q, h->comm, s));
      if (gc) NCCLCHK(ncclRecv(D.recvbuf + 2 * D.cg_off[b0 + q], 2 * gc, ncclDouble, q, h->comm, s));
    }
    NCCLCHK(ncclGroupEnd());
    if (g1 > g0) unpack2_kernel<<<nblocks(g1 - g0), 256, 0, s>>>(g1 - g0, D.cghost_idx + g0, D.nloc, D.recvbuf + 2 * g0, d.buf);
    return MAMG_OK;
  }
  if (d.dk == D_HALO) {
    if (ns) pack2_kernel<<<nblocks(ns), 256, 0, s>>>(ns, D.send_idx, d.buf, D.sendbuf);
    NCCLCHK(ncclGroupStart());
    for (int q = 0; q < h->nranks; ++q) {
      if (q == h->rank) continue;
      const int64_t sc = D.send_off[q + 1] - D.send_off[q];
      const int64_t gc = D.ghost_off[q + 1] - D.ghost_off[q];
      if (sc) NCCLCHK(ncclSend(D.sendbuf + 2 * D.send_off[q], 2 * sc, ncclDouble, q, h->comm, s));
      if (gc) NCCLCHK(ncclRecv(d.buf + 2 * (D.nloc + D.ghost_off[q]), 2 * gc, ncclDouble, q, h->comm, s));
    }
    NCCLCHK(ncclGroupEnd());
    return MAMG_OK;
  }
  // D_REVERSE: ghost partials -> owners; owners add in rank order
  NCCLCHK(ncclGroupStart());
  for (int q = 0; q < h->nranks; ++q) {
    if (q == h->rank) continue;
    const int64_t sc = D.send_off[q + 1] - D.send_off[q];
    const int64_t gc = D.ghost_off[q + 1] - D.ghost_off[q];
    if (gc) NCCLCHK(ncclSend(d.buf + 2 * (D.nloc + D.ghost_off[q]), 2 * gc, ncclDouble, q, h->comm, s));
    if (sc) NCCLCHK(ncclRecv(D.recvbuf + 2 * D.send_off[q], 2 * sc, ncclDouble, q, h->comm, s));
  }
  NCCLCHK(ncclGroupEnd());
  for (int q = 0; q < h->nranks; ++q) {
    const int64_t sc = D.send_off[q + 1] - D.send_off[q];
    if (q == h->rank || !sc) continue;
    addidx2_kernel<<<nblocks(sc), 256, 0, s>>>(sc, D.send_idx + D.send_off[q],
                                               D.recvbuf + 2 * D.send_off[q], d.buf);
  }
  return MAMG_OK;
}

void dapply_ops(const DistHandle* h, const double* r, double* z, std::vector<DOp>* ops) {
  ops->clear();
  const int64_t nloc = h->L[0].nloc;
  dcycle_ops(h, 0, r, nloc, z, nloc, ops);
}

// y = A x on the rank's rows (field-major local slices): interleave x into
// the [owned | ghost] buffer, forward halo, SpMV with A_loc (PCG operator)
void dspmv_ops(const DistHandle* h, const double* x, double* y, std::vector<DOp>* ops) {
  ops->clear();
  const DDLevel& D = h->L[0];
  Op o;
  o.kind = OP_ILV; o.cls = C_MISC; o.n = D.nloc; o.b = x; o.bs = D.nloc; o.out = D.spx;
  o.bytes = 32.0 * D.nloc;
  ops->push_back(wrap(o));
  const Op mv = bsr_op(D.A, EPI_Y, C_L0_RESID, 0, D.spx, 0, nullptr, nullptr, 0, nullptr, y, D.nloc);
  if (D.replicated) ops->push_back(wrap(mv)); else halo_residual(h, 0, D.spx, mv, ops);
}

}  // namespace

void device_warm(void* stream) {
  warm_kernel<<<1, 64, 0, (hipStream_t)stream>>>();
  (void)hipGetLastError();
}

int dist_get_unique_id(void* id, std::string* err) {
  ncclUniqueId u;
  NCCLCHK(ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof(u));
  return MAMG_OK;
}

// ---------------------------------------------------------------------------
// Rank-local operators built in HBM from the GPU hierarchy (mamg_setup_dist's
// default): the device restatement of build_dist_plan's conversions, so no
// matrix of the hierarchy crosses PCIe.  Row slices are gathered from the
// field-major CSRs, converted by the single-GPU csr2bsr kernel, and their
// columns renumbered [owned | ghost] (owned first, each part in global order:
// dist.cpp remap_cols); K by kmerge_kernel, the partial restriction from R's
// rows (R = P^T exactly, so its blocks are transpose_bsr's).  Bitwise the
// host plan's operators (tests/test_gpu_dist.py::test_rank_slice_download_bitwise).
// ---------------------------------------------------------------------------
namespace {

// rows f m + i of the gathered CSR = rows f nvr + row(i) of M, row(i) =
// rows[i] or r0 + i
__global__ __launch_bounds__(256) void rowlen_gather_kernel(int64_t m, int64_t nvr, const int64_t* __restrict__ rows,
                                                            int64_t r0, const int64_t* __restrict__ ptr,
                                                            int64_t* __restrict__ len) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= 2 * m) return;
  const int64_t f = i / m, k = i - f * m;
  const int64_t src = f * nvr + (rows ? rows[k] : r0 + k);
  len[i + 1] = ptr[src + 1] - ptr[src];
}

__global__ __launch_bounds__(256) void rowcopy_gather_kernel(int64_t m, int64_t nvr, const int64_t* __restrict__ rows,
                                                             int64_t r0, const int64_t* __restrict__ ptr,
                                                             const int32_t* __restrict__ col,
                                                             const double* __restrict__ val,
                                                             const int64_t* __restrict__ optr,
                                                             int32_t* __restrict__ ocol, double* __restrict__ oval) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= 2 * m) return;
  const int64_t f = i / m, k = i - f * m;
  const int64_t src = f * nvr + (rows ? rows[k] : r0 + k);
  int64_t o = optr[i];
  for (int64_t q = ptr[src]; q < ptr[src + 1]; ++q, ++o) {
    ocol[o] = col[q];
    oval[o] = val[q];
  }
}

// node columns -> local [owned | ghost] numbering: owned blocks first, then
// ghosts, each in the row's (global) order
__global__ __launch_bounds__(256) void map_part_kernel(int64_t nr, const int64_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ col, const dv4* __restrict__ val,
                                                       const int32_t* __restrict__ map, int32_t nown,
                                                       int32_t* __restrict__ ocol, dv4* __restrict__ oval) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nr) return;
  int64_t o = ptr[I];
  for (int part = 0; part < 2; ++part)
    for (int64_t k = ptr[I]; k < ptr[I + 1]; ++k) {
      const int32_t c = map[col[k]];
      if ((c < nown) == (part == 0)) { ocol[o] = c; oval[o] = val[k]; ++o; }
    }
}

// keep the blocks whose column lies in [w0, w1), renumbered from w0
__global__ __launch_bounds__(256) void window_len_kernel(int64_t nr, const int64_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ col, int64_t w0, int64_t w1,
                                                         int64_t* __restrict__ len) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nr) return;
  int64_t c = 0;
  for (int64_t k = ptr[I]; k < ptr[I + 1]; ++k) c += col[k] >= w0 && col[k] < w1;
  len[I + 1] = c;
}

__global__ __launch_bounds__(256) void window_fill_kernel(int64_t nr, const int64_t* __restrict__ ptr,
                                                          const int32_t* __restrict__ col,
                                                          const dv4* __restrict__ val, int64_t w0, int64_t w1,
                                                          const int64_t* __restrict__ optr,
                                                          int32_t* __restrict__ ocol, dv4* __restrict__ oval) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nr) return;
  int64_t o = optr[I];
  for (int64_t k = ptr[I]; k < ptr[I + 1]; ++k)
    if (col[k] >= w0 && col[k] < w1) { ocol[o] = (int32_t)(col[k] - w0); oval[o] = val[k]; ++o; }
}

__global__ __launch_bounds__(256) void map_fill_kernel(int64_t n, int64_t first, int32_t base,
                                                       const int64_t* __restrict__ ids, int32_t* __restrict__ map) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  map[ids ? ids[k] : first + k] = base + (int32_t)k;
}

__global__ __launch_bounds__(256) void ghost_row_kernel(int64_t nr, const int64_t* __restrict__ ptr,
                                                        const int32_t* __restrict__ col, int32_t nown,
                                                        uint8_t* __restrict__ flag) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nr) return;
  uint8_t g = 0;
  for (int64_t k = ptr[I]; k < ptr[I + 1]; ++k) g |= col[k] >= nown;
  flag[I] = g;
}

// a node split by seed blocks keeps the two diagonal entries of its block
__global__ __launch_bounds__(256) void unjoin_kernel(int64_t n, const uint8_t* __restrict__ joined, dv4* W) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I < n && !joined[I]) { W[I].y = 0.0; W[I].z = 0.0; }
}

// rows of a field-major CSR (node rows r0 + i, or rows[i]) as a BSR2 with
// global node columns
int dev_rows_to_bsr(TmpPool* T, const DevMat& M, int64_t nvr, int64_t nvc, int64_t m, const int64_t* rows,
                    int64_t r0, TBsr* B, std::string* err) {
  int rc;
  DevMat S;
  S.n = 2 * m;
  S.m = M.m;
  if ((rc = T->alloc(&S.ptr, 2 * m + 1, err))) return rc;
  HIPCHK(dev_memset(S.ptr, 0, sizeof(int64_t)));
  if (m) rowlen_gather_kernel<<<nblocks(2 * m), 256>>>(m, nvr, rows, r0, M.ptr, S.ptr);
  HIPCHK(hipGetLastError());
  if ((rc = dscan_incl_i64(S.ptr, S.ptr, 2 * m + 1, nullptr, err))) return rc;
  HIPCHK(hipMemcpy(&S.nnz, S.ptr + 2 * m, sizeof(int64_t), hipMemcpyDeviceToHost));
  if ((rc = T->alloc(&S.col, S.nnz, err))) return rc;
  if ((rc = T->alloc(&S.val, S.nnz, err))) return rc;
  if (m) rowcopy_gather_kernel<<<nblocks(2 * m), 256>>>(m, nvr, rows, r0, M.ptr, M.col, M.val, S.ptr, S.col, S.val);
  HIPCHK(hipGetLastError());
  return dev_csr_to_bsr(T, S, m, nvc, B, err);
}

// column map of a distributed level: owned J -> J - o0, ghost g_k -> nloc + k
int dev_col_map(TmpPool* T, const DistLevel& L, int32_t** map, std::string* err) {
  int rc;
  if ((rc = T->alloc(map, L.nv, err))) return rc;
  HIPCHK(dev_memset(*map, 0xff, L.nv * sizeof(int32_t)));
  if (L.nloc) map_fill_kernel<<<nblocks(L.nloc), 256>>>(L.nloc, L.o0, 0, nullptr, *map);
  const int64_t ng = (int64_t)L.ghosts.size();
  if (ng) {
    int64_t* g = nullptr;
    if ((rc = T->alloc(&g, ng, err))) return rc;
    HIPCHK(hipMemcpy(g, L.ghosts.data(), ng * sizeof(int64_t), hipMemcpyHostToDevice));
    map_fill_kernel<<<nblocks(ng), 256>>>(ng, 0, (int32_t)L.nloc, g, *map);
  }
  HIPCHK(hipGetLastError());
  return MAMG_OK;
}

// BSR2 columns renumbered by map, [owned | ghost] order; nc = local columns
int dev_map_cols(TmpPool* T, const TBsr& B, const int32_t* map, int64_t nown, int64_t nc, TBsr* O,
                 std::string* err) {
  int rc;
  *O = B;
  O->nc = nc;
  if ((rc = T->alloc(&O->col, B.nb, err))) return rc;
  if ((rc = T->alloc(&O->val, B.nb, err))) return rc;
  if (B.nr) map_part_kernel<<<nblocks(B.nr), 256>>>(B.nr, B.ptr, B.col, B.val, map, (int32_t)nown, O->col, O->val);
  HIPCHK(hipGetLastError());
  return MAMG_OK;
}

int dev_window_cols(TmpPool* T, const TBsr& B, int64_t w0, int64_t w1, TBsr* O, std::string* err) {
  int rc;
  O->nr = B.nr; O->nc = w1 - w0; O->merged = false;
  if ((rc = T->alloc(&O->ptr, B.nr + 1, err))) return rc;
  HIPCHK(dev_memset(O->ptr, 0, sizeof(int64_t)));
  if (B.nr) window_len_kernel<<<nblocks(B.nr), 256>>>(B.nr, B.ptr, B.col, w0, w1, O->ptr);
  HIPCHK(hipGetLastError());
  if ((rc = dscan_incl_i64(O->ptr, O->ptr, B.nr + 1, nullptr, err))) return rc;
  HIPCHK(hipMemcpy(&O->nb, O->ptr + B.nr, sizeof(int64_t), hipMemcpyDeviceToHost));
  if ((rc = T->alloc(&O->col, O->nb, err))) return rc;
  if ((rc = T->alloc(&O->val, O->nb, err))) return rc;
  if (B.nr) window_fill_kernel<<<nblocks(B.nr), 256>>>(B.nr, B.ptr, B.col, B.val, w0, w1, O->ptr, O->col, O->val);
  HIPCHK(hipGetLastError());
  return MAMG_OK;
}

// ---- node patches on N ranks (dist_patches) --------------------------------
// hop distance of every node from the owned range (0 owned, 1..3, 127 beyond)
__global__ __launch_bounds__(256) void hop_init_kernel(int64_t nv, int64_t o0, int64_t o1, int8_t* __restrict__ d) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I < nv) d[I] = (I >= o0 && I < o1) ? 0 : 127;
}
__global__ __launch_bounds__(256) void hop_step_kernel(int64_t nv, const int64_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ col, const int8_t* __restrict__ din,
                                                       int8_t* __restrict__ dout, int k) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nv) return;
  int8_t v = din[I];
  if (v == 127)
    for (int64_t q = ptr[I]; q < ptr[I + 1]; ++q)
      if (din[col[q]] == k - 1) { v = (int8_t)k; break; }
  dout[I] = v;
}
// global id of local node li ([owned | ghost])
__device__ __forceinline__ int64_t local_gid(int64_t li, int64_t nloc, int64_t o0, const int64_t* gh) {
  return li < nloc ? o0 + li : gh[li - nloc];
}
// the rank's patch / ring-block rows: local row li = B's row of its global
// node when that node is within hmax hops of the owned range, else empty
// (len[li + 1])
__global__ __launch_bounds__(256) void srow_len_kernel(int64_t nl, int64_t nloc, int64_t o0, const int64_t* __restrict__ gh,
                                                       const int8_t* __restrict__ hop, const int64_t* __restrict__ bptr,
                                                       int64_t* __restrict__ len, int hmax) {
  const int64_t li = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (li >= nl) return;
  const int64_t g = local_gid(li, nloc, o0, gh);
  len[li + 1] = hop[g] <= hmax ? bptr[g + 1] - bptr[g] : 0;
}
// ... its blocks in B's (global) column order: local columns (map) and the
// global ids (the inverse kernel's search keys)
__global__ __launch_bounds__(256) void srow_fill_kernel(int64_t nl, int64_t nloc, int64_t o0, const int64_t* __restrict__ gh,
                                                        const int64_t* __restrict__ bptr, const int32_t* __restrict__ bcol,
                                                        const dv4* __restrict__ bval, const int32_t* __restrict__ map,
                                                        const int64_t* __restrict__ sptr, int32_t* __restrict__ scol,
                                                        int32_t* __restrict__ sgcol, dv4* __restrict__ sval) {
  const int64_t li = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (li >= nl || sptr[li + 1] == sptr[li]) return;
  const int64_t g = local_gid(li, nloc, o0, gh);
  int64_t o = sptr[li];
  for (int64_t k = bptr[g]; k < bptr[g + 1]; ++k, ++o) {
    scol[o] = map[bcol[k]];
    sgcol[o] = bcol[k];
    sval[o] = bval[k];
  }
}
// per local node: its hop distance and colour (for the centre list)
__global__ __launch_bounds__(256) void local_hop_colour_kernel(int64_t nl, int64_t nloc, int64_t o0,
                                                               const int64_t* __restrict__ gh,
                                                               const int8_t* __restrict__ hop,
                                                               const int16_t* __restrict__ c, int8_t* __restrict__ lh,
                                                               int16_t* __restrict__ lc) {
  const int64_t li = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (li >= nl) return;
  const int64_t g = local_gid(li, nloc, o0, gh);
  lh[li] = hop[g];
  lc[li] = c[g];
}
// colours of the patches that write node J (the centres in J's closed
// neighbourhood), -1 padded: PATCH_MAX_NODES + 1 slots per node
__global__ __launch_bounds__(256) void cover_kernel(int64_t cnt, const int64_t* __restrict__ nodes,
                                                    const int64_t* __restrict__ bptr, const int32_t* __restrict__ bcol,
                                                    const int16_t* __restrict__ c, int16_t* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= cnt) return;
  const int64_t J = nodes[t];
  int16_t* o = out + t * (PATCH_MAX_NODES + 1);
  int k = 0;
  bool self = false;
  for (int64_t q = bptr[J]; q < bptr[J + 1] && k < PATCH_MAX_NODES + 1; ++q) {
    self |= bcol[q] == J;
    o[k++] = c[bcol[q]];
  }
  if (!self && k < PATCH_MAX_NODES + 1) o[k++] = c[J];
  for (; k < PATCH_MAX_NODES + 1; ++k) o[k] = -1;
}

// Level-0 node patches of a rank: the global distance-3
// colouring (every rank colours the whole level-0 graph, as the single-GPU
// build_patches, so all ranks hold the same colours); the centres within 1
// hop of the owned nodes (their patches write owned nodes; the owner of
// every written node computes the same patch from the same x, so its bits
// agree); their rows (nodes within 2 hops) with the global column order kept
// (the patch's local dof order, hence its Gauss-Jordan, equals the single
// GPU's); the inverses; and per colour the halo of the nodes its patches
// write (send: owned nodes in a peer's 3-hop region, receive: ghosts), so
// that the ghosts within 3 hops are current before the next colour.
int dist_patches(DistHandle* h, const DevMat& A0d, const DistLevel& P, DDLevel* D, std::string* err) {
  int rc;
  TmpPool T;
  const int64_t nv = P.nv, nloc = P.nloc, ng = (int64_t)P.ghosts.size(), nl = nloc + ng;
  const int R = h->nranks;
  TBsr B;
  if ((rc = dev_csr_to_bsr(&T, A0d, nv, nv, &B, err))) return rc;
  int16_t* c = nullptr;
  int maxlen = 0;
  if ((rc = patch_colour(&T, B, &c, &maxlen, err))) return rc;
  int16_t hcol_max = 0;
  {
    std::vector<int16_t> hc(nv);
    HIPCHK(hipMemcpy(hc.data(), c, nv * sizeof(int16_t), hipMemcpyDeviceToHost));
    for (int16_t v : hc) hcol_max = std::max(hcol_max, v);
  }
  const int ncol = hcol_max + 1;
  int8_t *hop = nullptr, *hop2 = nullptr;
  if ((rc = T.alloc(&hop, nv, err)) || (rc = T.alloc(&hop2, nv, err))) return rc;
  hop_init_kernel<<<nblocks(nv), 256>>>(nv, P.o0, P.o1, hop);
  for (int k = 1; k <= 3; ++k) {
    hop_step_kernel<<<nblocks(nv), 256>>>(nv, B.ptr, B.col, hop, hop2, k);
    std::swap(hop, hop2);
  }
  HIPCHK(hipGetLastError());
  int64_t* gh = nullptr;
  if ((rc = T.alloc(&gh, std::max<int64_t>(ng, 1), err))) return rc;
  if (ng) HIPCHK(hipMemcpy(gh, P.ghosts.data(), ng * sizeof(int64_t), hipMemcpyHostToDevice));
  int32_t* map = nullptr;
  if ((rc = dev_col_map(&T, P, &map, err))) return rc;
  // the patch rows
  DLevel& L = D->pl;
  if ((rc = ddalloc(h, &L.Sptr, nl + 1, err))) return rc;
  if (nl) srow_len_kernel<<<nblocks(nl), 256>>>(nl, nloc, P.o0, gh, hop, B.ptr, L.Sptr, 2);
  HIPCHK(hipGetLastError());
  if ((rc = dscan_incl_i64(L.Sptr, L.Sptr, nl + 1, nullptr, err))) return rc;
  HIPCHK(hipMemcpy(&L.Snb, L.Sptr + nl, sizeof(int64_t), hipMemcpyDeviceToHost));
  if ((rc = ddalloc(h, &L.Scol, std::max<int64_t>(L.Snb, 1), err))) return rc;
  if ((rc = ddalloc(h, &D->Sgcol, std::max<int64_t>(L.Snb, 1), err))) return rc;
  if ((rc = ddalloc(h, &L.Sval, std::max<int64_t>(L.Snb, 1), err))) return rc;
  if (nl) srow_fill_kernel<<<nblocks(nl), 256>>>(nl, nloc, P.o0, gh, B.ptr, B.col, B.val, map, L.Sptr, L.Scol, D->Sgcol,
                                                 L.Sval);
  HIPCHK(hipGetLastError());
  // the centres (within 1 hop), colour by colour, ascending global id inside a colour
  std::vector<int8_t> lh(nl);
  std::vector<int16_t> lc(nl);
  {
    int8_t* dlh = nullptr;
    int16_t* dlc = nullptr;
    if ((rc = T.alloc(&dlh, std::max<int64_t>(nl, 1), err)) || (rc = T.alloc(&dlc, std::max<int64_t>(nl, 1), err)))
      return rc;
    if (nl) local_hop_colour_kernel<<<nblocks(nl), 256>>>(nl, nloc, P.o0, gh, hop, c, dlh, dlc);
    HIPCHK(hipGetLastError());
    if (nl) {
      HIPCHK(hipMemcpy(lh.data(), dlh, nl, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(lc.data(), dlc, nl * sizeof(int16_t), hipMemcpyDeviceToHost));
    }
  }
  std::vector<std::pair<int64_t, int64_t>> cen;   // (colour << 40 | global id, local id)
  for (int64_t li = 0; li < nl; ++li)
    if (lh[li] <= 1) {
      const int64_t g = li < nloc ? P.o0 + li : P.ghosts[li - nloc];
      cen.push_back({((int64_t)lc[li] << 40) | g, li});
    }
  std::sort(cen.begin(), cen.end());
  const int64_t np = (int64_t)cen.size();
  L.pcs.assign(ncol + 1, 0);
  std::vector<int32_t> perm(np);
  for (int64_t i = 0; i < np; ++i) {
    perm[i] = (int32_t)cen[i].second;
    ++L.pcs[(cen[i].first >> 40) + 1];
  }
  for (int k = 0; k < ncol; ++k) L.pcs[k + 1] += L.pcs[k];
  L.n = 2 * np;
  if ((rc = ddalloc(h, &L.pperm, std::max<int64_t>(np, 1), err))) return rc;
  if (np) HIPCHK(hipMemcpy(L.pperm, perm.data(), np * sizeof(int32_t), hipMemcpyHostToDevice));
  // inverses
  const int64_t dmax = 2 * (int64_t)maxlen;
  L.pus = dmax * (dmax + 1) / 2;
  if ((rc = ddalloc(h, &L.pu, std::max<int64_t>(np * L.pus, 1), err))) return rc;
  int* bad = nullptr;
  if ((rc = T.alloc(&bad, 1, err))) return rc;
  HIPCHK(dev_memset(bad, 0, sizeof(int)));
  launch_patch_inv(np, L.pperm, L.Sptr, L.Scol, D->Sgcol, L.Sval, L.pus, L.pu, bad);
  HIPCHK(hipGetLastError());
  int hb = 0;
  HIPCHK(hipMemcpy(&hb, bad, sizeof(int), hipMemcpyDeviceToHost));
  if (hb) { *err = "node patches: a patch matrix is not SPD (non-positive Gauss-Jordan pivot)"; return MAMG_ERR_SETUP; }
  // each colour's halo: the listed nodes its patches write
  const int64_t ns = P.send_off.empty() ? 0 : P.send_off.back();
  std::vector<int64_t> lst(ns + ng);
  for (int64_t t = 0; t < ns; ++t) lst[t] = P.o0 + P.send_idx[t];
  for (int64_t g = 0; g < ng; ++g) lst[ns + g] = P.ghosts[g];
  constexpr int CW = PATCH_MAX_NODES + 1;
  std::vector<int16_t> cov((size_t)(ns + ng) * CW);
  if (ns + ng) {
    int64_t* dl = nullptr;
    int16_t* dc = nullptr;
    if ((rc = T.alloc(&dl, ns + ng, err)) || (rc = T.alloc(&dc, (ns + ng) * CW, err))) return rc;
    HIPCHK(hipMemcpy(dl, lst.data(), (ns + ng) * sizeof(int64_t), hipMemcpyHostToDevice));
    cover_kernel<<<nblocks(ns + ng), 256>>>(ns + ng, dl, B.ptr, B.col, c, dc);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(cov.data(), dc, cov.size() * sizeof(int16_t), hipMemcpyDeviceToHost));
  }
  auto covers = [&](int64_t t, int col) {
    for (int k = 0; k < CW; ++k)
      if (cov[(size_t)t * CW + k] == col) return true;
    return false;
  };
  std::vector<int64_t> cs, cg;
  D->cs_off.assign((size_t)ncol * (R + 1), 0);
  D->cg_off.assign((size_t)ncol * (R + 1), 0);
  for (int col = 0; col < ncol; ++col) {
    for (int q = 0; q < R; ++q) {
      D->cs_off[(size_t)col * (R + 1) + q] = (int64_t)cs.size();
      D->cg_off[(size_t)col * (R + 1) + q] = (int64_t)cg.size();
      for (int64_t t = P.send_off[q]; t < P.send_off[q + 1]; ++t)
        if (covers(t, col)) cs.push_back(P.send_idx[t]);
      for (int64_t g = P.ghost_off[q]; g < P.ghost_off[q + 1]; ++g)
        if (covers(ns + g, col)) cg.push_back(g);
    }
    D->cs_off[(size_t)col * (R + 1) + R] = (int64_t)cs.size();
    D->cg_off[(size_t)col * (R + 1) + R] = (int64_t)cg.size();
  }
  if (!cs.empty()) {
    if ((rc = ddalloc(h, &D->csend_idx, (int64_t)cs.size(), err))) return rc;
    HIPCHK(hipMemcpy(D->csend_idx, cs.data(), cs.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  if (!cg.empty()) {
    if ((rc = ddalloc(h, &D->cghost_idx, (int64_t)cg.size(), err))) return rc;
    HIPCHK(hipMemcpy(D->cghost_idx, cg.data(), cg.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  D->patches = true;
  if (h->p.print_level >= 2)
    std::fprintf(stderr, "[mamg] rank %d/%d node patches: %d colours, %lld centres (%lld owned), %lld ghost nodes "
                 "(3 hops), colour halos %lld sends / %lld receives in all\n", h->rank, R, ncol, (long long)np,
                 (long long)nloc, (long long)ng, (long long)cs.size(), (long long)cg.size());
  return MAMG_OK;
}

// Level-0 seed-ring Schwarz of a rank (SCHWARZ_RINGS on N GPUs, DESIGN.md
// 6.4): every rank builds the global blocks, inverses and
// conflict colouring (ring_blocks_dev + ring_colouring, the single-GPU
// build_rings' steps, so every rank holds the same blocks and colours) and
// keeps the blocks with a member node it owns -- the owner of every written
// node computes every block that writes it, from the same x, so its bits agree
// with one GPU's.  A block's members lie within 2 maxlvl hops of an owned node
// and its rows read x within 2 maxlvl + 1 hops: the ghost region.  The rest's
// multicolour GS runs on the owned rows with the covered dofs masked
// (dev_rank_ops, from *cov_owned).  One colour table serves both: ring colour
// c at index c (the nodes its blocks write), GS colour g at nrc + g (the nodes
// of that colour), each with the halo of those nodes in the send / ghost
// lists, so the exchange code is the multicolour GS's.
int dist_rings(DistHandle* h, const DevMat& A0d, const DistLevel& P, const std::vector<int32_t>& seeds,
               const int8_t* gcol, int ngc, DDLevel* D, uint8_t** cov_owned, std::string* err) {
  int rc;
  TmpPool T;
  const mamg_params& p = h->p;
  const int64_t nv = P.nv, nloc = P.nloc, ng = (int64_t)P.ghosts.size(), nl = nloc + ng, n = A0d.n;
  const int R = h->nranks, L = p.Schwarz_maxlvl;
  const int64_t ns = (int64_t)seeds.size();
  if (ns <= 0) { *err = "seed rings: no seeds"; return MAMG_ERR_ARG; }
  // the global blocks and their conflict colouring (build_rings)
  RingBlocks RB;
  if ((rc = ring_blocks_dev(A0d, seeds.data(), ns, L, p.Schwarz_mmsize, &RB, err))) return rc;
  struct Guard { RingBlocks* r; ~Guard() { ring_blocks_free(r); } } guard{&RB};
  const int mm = RB.mm;
  std::vector<int32_t> blk((size_t)ns * mm);
  std::vector<int64_t> blen(ns);
  HIPCHK(hipMemcpy(blk.data(), RB.blk, blk.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(blen.data(), RB.blen, ns * sizeof(int64_t), hipMemcpyDeviceToHost));
  std::vector<int64_t> bptr(ns + 1, 0);
  for (int64_t k = 0; k < ns; ++k) bptr[k + 1] = bptr[k] + blen[k];
  std::vector<int32_t> mem(bptr[ns]);
  for (int64_t k = 0; k < ns; ++k) std::copy(blk.begin() + k * mm, blk.begin() + k * mm + blen[k], mem.begin() + bptr[k]);
  std::vector<int32_t>().swap(blk);
  std::vector<int32_t> colour;
  {
    std::vector<int64_t> aptr(n + 1);
    std::vector<int32_t> acol(A0d.nnz);
    HIPCHK(hipMemcpy(aptr.data(), A0d.ptr, (n + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(acol.data(), A0d.col, A0d.nnz * sizeof(int32_t), hipMemcpyDeviceToHost));
    CsrView Av;
    Av.n = Av.m = n; Av.ptr = aptr.data(); Av.col = acol.data();
    ring_colouring(Av, bptr, mem, &colour);
  }
  int nrc = 0;
  for (int32_t c : colour) nrc = std::max(nrc, c + 1);
  std::vector<int32_t> ord(ns);
  std::iota(ord.begin(), ord.end(), 0);
  std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return colour[a] < colour[b]; });
  // local node ids (owned first, then ghosts), covered dofs, the colours
  // writing each node (one bit per ring colour)
  std::vector<int32_t> loc(nv, -1);
  for (int64_t i = 0; i < nloc; ++i) loc[P.o0 + i] = (int32_t)i;
  for (int64_t g = 0; g < ng; ++g) loc[P.ghosts[g]] = (int32_t)(nloc + g);
  const int CW = (nrc + 63) / 64;
  std::vector<uint64_t> wr((size_t)nv * std::max(CW, 1), 0);
  std::vector<uint8_t> cov(nv, 0);
  for (int64_t k = 0; k < ns; ++k)
    for (int64_t t = bptr[k]; t < bptr[k + 1]; ++t) {
      const int64_t gd = mem[t], I = gd % nv, f = gd / nv;
      cov[I] |= (uint8_t)(1u << f);
      wr[(size_t)I * CW + colour[k] / 64] |= 1ull << (colour[k] % 64);
    }
  // the rank's blocks: a member node owned, colour by colour (seed order inside)
  DLevel& RL = D->rl;
  RL.rcs.assign(nrc + 1, 0);
  std::vector<int32_t> mine;
  std::vector<int64_t> mo(1, 0), io(1, 0);
  std::vector<int32_t> rm;
  for (int64_t j = 0; j < ns; ++j) {
    const int32_t k = ord[j];
    bool own = false;
    for (int64_t t = bptr[k]; t < bptr[k + 1] && !own; ++t) {
      const int64_t I = mem[t] % nv;
      own = I >= P.o0 && I < P.o1;
    }
    if (!own) continue;
    for (int64_t t = bptr[k]; t < bptr[k + 1]; ++t) {
      const int64_t gd = mem[t], I = gd % nv, f = gd / nv;
      if (loc[I] < 0) {
        *err = "multi-GPU seed rings: a block member outside the rank's " + std::to_string(2 * L + 1) +
               "-hop ghost region";
        return MAMG_ERR_SETUP;
      }
      rm.push_back(2 * loc[I] + (int32_t)f);
    }
    mine.push_back(k);
    mo.push_back(mo.back() + blen[k]);
    io.push_back(io.back() + blen[k] * blen[k]);
    ++RL.rcs[colour[k] + 1];
  }
  for (int c = 0; c < nrc; ++c) RL.rcs[c + 1] += RL.rcs[c];
  const int64_t nb = (int64_t)mine.size();
  RL.n = 2 * nl;
  RL.rnm = mo.back();
  RL.rinv_n = (double)io.back();
  if ((rc = ddalloc(h, &RL.rmo, nb + 1, err)) || (rc = ddalloc(h, &RL.rio, nb + 1, err)) ||
      (rc = ddalloc(h, &RL.rmem, std::max<int64_t>(RL.rnm, 1), err)) ||
      (rc = ddalloc(h, &RL.rinv, std::max<int64_t>(io.back(), 1), err)))
    return rc;
  HIPCHK(hipMemcpy(RL.rmo, mo.data(), (nb + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(RL.rio, io.data(), (nb + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if (RL.rnm) HIPCHK(hipMemcpy(RL.rmem, rm.data(), rm.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  if (nb) {
    int32_t* dmine = nullptr;
    if ((rc = T.alloc(&dmine, nb, err))) return rc;
    HIPCHK(hipMemcpy(dmine, mine.data(), nb * sizeof(int32_t), hipMemcpyHostToDevice));
    ring_perm_inv_kernel<<<(unsigned)nb, 256>>>(nb, dmine, RB.blen, RB.sq, RB.inv, RL.rio, RL.rinv);
    HIPCHK(hipGetLastError());
  }
  // the block rows: A_0's node rows of the local nodes within 2 L hops,
  // local columns (the ring kernel reads x through them)
  TBsr B;
  if ((rc = dev_csr_to_bsr(&T, A0d, nv, nv, &B, err))) return rc;
  int8_t *hop = nullptr, *hop2 = nullptr;
  if ((rc = T.alloc(&hop, nv, err)) || (rc = T.alloc(&hop2, nv, err))) return rc;
  hop_init_kernel<<<nblocks(nv), 256>>>(nv, P.o0, P.o1, hop);
  for (int k = 1; k <= 2 * L; ++k) {
    hop_step_kernel<<<nblocks(nv), 256>>>(nv, B.ptr, B.col, hop, hop2, k);
    std::swap(hop, hop2);
  }
  HIPCHK(hipGetLastError());
  int64_t* gh = nullptr;
  if ((rc = T.alloc(&gh, std::max<int64_t>(ng, 1), err))) return rc;
  if (ng) HIPCHK(hipMemcpy(gh, P.ghosts.data(), ng * sizeof(int64_t), hipMemcpyHostToDevice));
  int32_t* map = nullptr;
  if ((rc = dev_col_map(&T, P, &map, err))) return rc;
  if ((rc = ddalloc(h, &RL.Sptr, nl + 1, err))) return rc;
  if (nl) srow_len_kernel<<<nblocks(nl), 256>>>(nl, nloc, P.o0, gh, hop, B.ptr, RL.Sptr, 2 * L);
  HIPCHK(hipGetLastError());
  if ((rc = dscan_incl_i64(RL.Sptr, RL.Sptr, nl + 1, nullptr, err))) return rc;
  HIPCHK(hipMemcpy(&RL.Snb, RL.Sptr + nl, sizeof(int64_t), hipMemcpyDeviceToHost));
  int32_t* sg = nullptr;
  if ((rc = ddalloc(h, &RL.Scol, std::max<int64_t>(RL.Snb, 1), err)) ||
      (rc = T.alloc(&sg, std::max<int64_t>(RL.Snb, 1), err)) ||
      (rc = ddalloc(h, &RL.Sval, std::max<int64_t>(RL.Snb, 1), err)))
    return rc;
  if (nl) srow_fill_kernel<<<nblocks(nl), 256>>>(nl, nloc, P.o0, gh, B.ptr, B.col, B.val, map, RL.Sptr, RL.Scol, sg,
                                                 RL.Sval);
  HIPCHK(hipGetLastError());
  // the covered dofs of the owned nodes (the rest's GS masks them)
  if ((rc = ddalloc(h, cov_owned, std::max<int64_t>(nloc, 1), err))) return rc;
  if (nloc) HIPCHK(hipMemcpy(*cov_owned, cov.data() + P.o0, nloc, hipMemcpyHostToDevice));
  // the colour table: ring colours, then the rest GS's node colours
  std::vector<int8_t> hc(nv);
  if (nv) HIPCHK(hipMemcpy(hc.data(), gcol, nv, hipMemcpyDeviceToHost));
  auto in = [&](int64_t I, int idx) {
    return idx < nrc ? ((wr[(size_t)I * CW + idx / 64] >> (idx % 64)) & 1ull) != 0 : hc[I] == idx - nrc;
  };
  const int nct = nrc + ngc;
  std::vector<int64_t> cs, cg;
  D->cs_off.assign((size_t)nct * (R + 1), 0);
  D->cg_off.assign((size_t)nct * (R + 1), 0);
  for (int idx = 0; idx < nct; ++idx) {
    for (int q = 0; q < R; ++q) {
      D->cs_off[(size_t)idx * (R + 1) + q] = (int64_t)cs.size();
      D->cg_off[(size_t)idx * (R + 1) + q] = (int64_t)cg.size();
      for (int64_t t = P.send_off[q]; t < P.send_off[q + 1]; ++t)
        if (in(P.o0 + P.send_idx[t], idx)) cs.push_back(P.send_idx[t]);
      for (int64_t g = P.ghost_off[q]; g < P.ghost_off[q + 1]; ++g)
        if (in(P.ghosts[g], idx)) cg.push_back(g);
    }
    D->cs_off[(size_t)idx * (R + 1) + R] = (int64_t)cs.size();
    D->cg_off[(size_t)idx * (R + 1) + R] = (int64_t)cg.size();
  }
  if (!cs.empty()) {
    if ((rc = ddalloc(h, &D->csend_idx, (int64_t)cs.size(), err))) return rc;
    HIPCHK(hipMemcpy(D->csend_idx, cs.data(), cs.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  if (!cg.empty()) {
    if ((rc = ddalloc(h, &D->cghost_idx, (int64_t)cg.size(), err))) return rc;
    HIPCHK(hipMemcpy(D->cghost_idx, cg.data(), cg.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  D->rings = true;
  D->nrc = nrc;
  if (p.print_level >= 2)
    std::fprintf(stderr, "[mamg] rank %d/%d seed rings: %lld of %lld blocks, %d ring colours + %d GS colours, "
                 "%lld ghost nodes (%d hops), colour halos %lld sends / %lld receives in all\n", h->rank, R,
                 (long long)nb, (long long)ns, nrc, ngc, (long long)ng, 2 * L + 1, (long long)cs.size(),
                 (long long)cg.size());
  return MAMG_OK;
}

// each colour's halo of a distributed level: colour c's nodes in every send
// list and ghost list, in list order (so the sender's subset and the
// receiver's subset match), offsets per (colour, peer); gcol = the level's
// global colouring on the device
int colour_halo_lists(DistHandle* h, const DistLevel& P, const int8_t* gcol, int ncol, DDLevel* D,
                      std::string* err) {
  const int R = h->nranks;
  std::vector<int8_t> hc(P.nv);
  if (P.nv) HIPCHK(hipMemcpy(hc.data(), gcol, P.nv, hipMemcpyDeviceToHost));
  std::vector<int64_t> cs, cg;
  D->cs_off.assign((size_t)ncol * (R + 1), 0);
  D->cg_off.assign((size_t)ncol * (R + 1), 0);
  for (int c = 0; c < ncol; ++c) {
    for (int q = 0; q < R; ++q) {
      D->cs_off[(size_t)c * (R + 1) + q] = (int64_t)cs.size();
      D->cg_off[(size_t)c * (R + 1) + q] = (int64_t)cg.size();
      for (int64_t t = P.send_off[q]; t < P.send_off[q + 1]; ++t)
        if (hc[P.o0 + P.send_idx[t]] == c) cs.push_back(P.send_idx[t]);
      for (int64_t g = P.ghost_off[q]; g < P.ghost_off[q + 1]; ++g)
        if (hc[P.ghosts[g]] == c) cg.push_back(g);
    }
    D->cs_off[(size_t)c * (R + 1) + R] = (int64_t)cs.size();
    D->cg_off[(size_t)c * (R + 1) + R] = (int64_t)cg.size();
  }
  int rc;
  if (!cs.empty()) {
    if ((rc = ddalloc(h, &D->csend_idx, (int64_t)cs.size(), err))) return rc;
    HIPCHK(hipMemcpy(D->csend_idx, cs.data(), cs.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  if (!cg.empty()) {
    if ((rc = ddalloc(h, &D->cghost_idx, (int64_t)cg.size(), err))) return rc;
    HIPCHK(hipMemcpy(D->cghost_idx, cg.data(), cg.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  return MAMG_OK;
}

// the longest run [*r0, *r1) of M's rows whose columns are all < nown (owned:
// no ghost), for the launches during a halo
constexpr int64_t K_ROWS_ALIGN = 256;   // launch_msell row ranges: whole workgroups of every LPR
int ghost_free_run(TmpPool* T, const TBsr& M, int64_t nown, int64_t* r0, int64_t* r1, std::string* err) {
  int rc;
  const int64_t n = M.nr;
  uint8_t* fl = nullptr;
  if ((rc = T->alloc(&fl, n, err))) return rc;
  if (n) ghost_row_kernel<<<nblocks(n), 256>>>(n, M.ptr, M.col, (int32_t)nown, fl);
  HIPCHK(hipGetLastError());
  std::vector<uint8_t> hf(n);
  if (n) HIPCHK(hipMemcpy(hf.data(), fl, n, hipMemcpyDeviceToHost));
  int64_t best0 = 0, best1 = 0, run0 = 0;
  for (int64_t I = 0; I <= n; ++I)
    if (I == n || hf[I]) {
      if (I - run0 > best1 - best0) { best0 = run0; best1 = I; }
      run0 = I + 1;
    }
  *r0 = best0;
  *r1 = best1;
  return MAMG_OK;
}

// level l's A_loc (+ overlap window, band schedule), K / [P | AP] / P, R_loc
// and W from the GPU hierarchy (the operator block of dist_upload)
int dev_rank_ops(DistHandle* h, const GHier& G, const DevMat& A0d, const DistPlan& plan, int l, double kw,
                 const int8_t* gcol, int ncol, std::string* err) {
  int rc;
  const DistLevel& P = plan.levels[l];
  const GLevel& g = G.levels[l];
  DDLevel& D = h->L[l];
  const int64_t nv = P.nv, nloc = P.nloc, nc = nloc + (int64_t)P.ghosts.size();
  TmpPool T;
  int32_t* map = nullptr;
  if (!P.replicated && (rc = dev_col_map(&T, P, &map, err))) return rc;
  // W (node blocks of the owned rows)
  if ((rc = ddalloc(h, &D.W, nloc, err))) return rc;
  if (nloc) {
    HIPCHK(dev_copy(D.W, reinterpret_cast<const dv4*>(g.W) + P.o0, nloc * sizeof(dv4)));
    if (g.joined) unjoin_kernel<<<nblocks(nloc), 256>>>(nloc, g.joined + P.o0, D.W);
    HIPCHK(hipGetLastError());
  }
  // A_loc (+ the multicolour GS layout of its rows, colours of the level's
  // global colouring gcol)
  {
    TBsr raw, tA;
    const DevMat& Am = l == 0 ? A0d : g.A;
    if ((rc = dev_rows_to_bsr(&T, Am, nv, nv, nloc, nullptr, P.o0, &raw, err))) return rc;
    if (P.replicated) tA = raw;
    else if ((rc = dev_map_cols(&T, raw, map, nloc, nc, &tA, err))) return rc;
    if (!P.replicated && (rc = ghost_free_run(&T, tA, nloc, &D.ib0, &D.ib1, err)))   // overlap window
      return rc;
    bool half = false;
    if (l == 0 && g_half && tA.nr >= g_sell_min_rows && tA.nb > 0) {   // upload_half_or_bsr
      int* bad = nullptr;
      if ((rc = T.alloc(&bad, 1, err))) return rc;
      HIPCHK(dev_memset(bad, 0, sizeof(int)));
      sym_check_kernel<<<std::min(nblocks(tA.nb), SYM_CHECK_BLOCKS), 256>>>(tA.nb, tA.val, bad);
      int hb = 1;
      HIPCHK(hipMemcpy(&hb, bad, sizeof(int), hipMemcpyDeviceToHost));
      if (hb == 0) {
        D.A.nr = tA.nr; D.A.nc = tA.nc; D.A.nb = tA.nb;
        D.A.lanes = pick_lanes_bsr(tA.nr, tA.nb);
        D.A.sym = true;
        if ((rc = try_half(h, &T, tA, &D.A, err))) return rc;
        half = D.A.half;
      }
    }
    if (!half && (rc = finalize_bsr(h, &T, tA, &D.A, 0, true, err))) return rc;
    if (l == 0 && (rc = build_band_sched_range(h, &D.A, D.ib0, D.ib1, err))) return rc;
    if (gcol) {
      // seed rings: the rest's GS, covered dofs masked (build_rings' rest_w /
      // rest_mask on the owned rows)
      const double* Wg = reinterpret_cast<const double*>(D.W);
      if (D.rcov && nloc) {
        dv4* Wp = nullptr;
        if ((rc = T.alloc(&Wp, nloc, err))) return rc;
        rest_w_kernel<<<nblocks(nloc), 256>>>(nloc, D.W, D.rcov, Wp);
        HIPCHK(hipGetLastError());
        Wg = reinterpret_cast<const double*>(Wp);
      }
      if ((rc = gs_layout(h, &T, tA, Wg, gcol + P.o0, ncol, l, &D.Gb, &D.gperm, &D.Gd, &D.gcs, &D.gbk, err)))
        return rc;
      const int64_t nrp = D.gcs.empty() ? 0 : D.gcs.back();
      if (D.rcov && nrp) rest_mask_kernel<<<nblocks(nrp), 256>>>(nrp, D.gperm, D.rcov, D.Gd);
      HIPCHK(hipGetLastError());
    }
  }
  // prolongation side (level l+1 numbering)
  const DistLevel& C = plan.levels[l + 1];
  const int64_t cnc = C.replicated ? C.nv : C.nloc + (int64_t)C.ghosts.size();
  int32_t* cmap = nullptr;
  if (!C.replicated && (rc = dev_col_map(&T, C, &cmap, err))) return rc;
  auto rows_c = [&](const DevMat& M, TBsr* O) -> int {   // rows [o0, o1) of a fine x coarse CSR
    TBsr raw;
    int r = dev_rows_to_bsr(&T, M, nv, C.nv, nloc, nullptr, P.o0, &raw, err);
    if (r) return r;
    if (C.replicated) { *O = raw; return MAMG_OK; }
    return dev_map_cols(&T, raw, cmap, C.nloc, cnc, O, err);
  };
  TBsr tP;
  if ((rc = rows_c(g.P, &tP))) return rc;
  if (plan.fuse) {
    TBsr tAP, tK;
    if ((rc = rows_c(g.AP, &tAP))) return rc;
    if (plan.kpost) {
      const double* Wk = reinterpret_cast<const double*>(D.W);
      if (kw != 1.0 && nloc) {
        double* q = nullptr;
        if ((rc = T.alloc(&q, 4 * nloc, err))) return rc;
        wscale_kernel<<<nblocks(4 * nloc), 256>>>(4 * nloc, kw, Wk, q);
        HIPCHK(hipGetLastError());
        Wk = q;
      }
      if ((rc = dev_kmerge(&T, tP, tAP, Wk, &tK, err))) return rc;
      if ((rc = finalize_bsr(h, &T, tK, &D.K, 0, false, err))) return rc;
      if (l == 0 && g_k_sort && D.K.sell && D.K.lpr <= 1)   // rows sorted inside slices (section 4.1)
        if ((rc = sort_sell_slices(h, &T, &D.K, err))) return rc;
      // K's rows without coarse ghost columns, run while the coarse-e halo is
      // in flight (level 0's SELL K: launch_msell takes row ranges)
      if (l == 0 && !P.replicated && !C.replicated) {
        int64_t k0 = 0, k1 = 0;
        if ((rc = ghost_free_run(&T, tK, C.nloc, &k0, &k1, err))) return rc;
        k0 = (k0 + K_ROWS_ALIGN - 1) / K_ROWS_ALIGN * K_ROWS_ALIGN;
        k1 = k1 == nloc ? nloc : k1 / K_ROWS_ALIGN * K_ROWS_ALIGN;
        if (k1 > k0) { D.kb0 = k0; D.kb1 = k1; }
      }
    } else {
      if ((rc = dev_merge_rows(&T, tP, tAP, &tK, err))) return rc;
      if ((rc = finalize_bsr(h, &T, tK, &D.PA, 0, false, err))) return rc;
    }
  } else if ((rc = finalize_bsr(h, &T, tP, &D.P, 0, false, err))) {
    return rc;
  }
  // partial restriction R_loc = P_loc^T: R's rows of the local coarse nodes
  // ([owned | ghost], or all when replicated), columns in [o0, o1)
  {
    std::vector<int64_t> rows;
    rows.reserve(cnc);
    if (C.replicated) {
      for (int64_t J = 0; J < C.nv; ++J) rows.push_back(J);
    } else {
      for (int64_t J = C.o0; J < C.o1; ++J) rows.push_back(J);
      rows.insert(rows.end(), C.ghosts.begin(), C.ghosts.end());
    }
    int64_t* drows = nullptr;
    if ((rc = T.alloc(&drows, cnc, err))) return rc;
    if (cnc) HIPCHK(hipMemcpy(drows, rows.data(), cnc * sizeof(int64_t), hipMemcpyHostToDevice));
    TBsr raw, tR;
    if ((rc = dev_rows_to_bsr(&T, g.R, C.nv, nv, cnc, drows, 0, &raw, err))) return rc;
    if ((rc = dev_window_cols(&T, raw, P.o0, P.o1, &tR, err))) return rc;
    if ((rc = finalize_bsr(h, &T, tR, &D.R, 0, false, err))) return rc;
  }
  return MAMG_OK;
}

}  // namespace

int dist_check(const mamg_params& p, std::string* err) {
  if (p.maxit != 1) {
    *err = "multi-GPU apply supports maxit 1 (one cycle per application, src/amg_parameters.py:71)";
    return MAMG_ERR_UNSUPPORTED;
  }
  return MAMG_OK;
}

int dist_upload(const Hierarchy& H, const CsrView& A0, const mamg_params& p, int rank, int nranks,
                const void* comm_id, int64_t rep_nodes, DistHandle** out, std::string* err,
                const GhostLists* ghosts, const GHier* G, const DevMat* A0d) {
  if (int rc = dist_check(p, err)) return rc;
  const bool gs = gs_smoother(p);
  const bool patches = patch_schwarz(p);
  const bool rings = rings_schwarz(p);
  if ((patches || rings) && !(G && A0d && ghosts)) {
    *err = std::string("multi-GPU ") + (patches ? "node patches need the rank operators and the 3-hop" :
           "seed rings need the rank operators and the (2 Schwarz_maxlvl + 1)-hop") +
           " ghost lists built from the GPU hierarchy (mamg_setup_dist with a GPU-setup profile)";
    return MAMG_ERR_UNSUPPORTED;
  }
  if (gs && !G) {
    *err = "multi-GPU multicolour GS needs the rank operators built from the GPU hierarchy (mamg_setup_dist "
           "with a GPU-setup profile)";
    return MAMG_ERR_UNSUPPORTED;
  }
  read_knobs();
  double pw[MAMG_POLY_MAX];
  const int pm = poly_weights(p, pw);
  DistPlan plan;
  const auto tp0 = std::chrono::steady_clock::now();
  const double kw = p.smoother == MAMG_SMOOTHER_POLY ? pw[pm - 1] : 1.0;
  bool fuse = p.post_fusion != 0 && !gs && !patches && !rings;   // GS / patches / rings post-smooth after x += P e (as on one GPU)
  if (G)                   // operators from the GPU hierarchy: fusion needs its A P on every level
    for (size_t l = 0; l + 1 < G->levels.size() && fuse; ++l)
      if (!G->levels[l].coarsest && G->levels[l].AP.n != G->levels[l].n) fuse = false;
  int rc = build_dist_plan(H, A0, rank, nranks, rep_nodes, fuse, &plan, err, g_post_k != 0, kw, ghosts,
                           G != nullptr);
  if (rc) return rc;
  if (p.print_level >= 2)
    std::fprintf(stderr, "[mamg] rank %d/%d setup:   of which host plan    %.3f s\n", rank, nranks,
                 std::chrono::duration<double>(std::chrono::steady_clock::now() - tp0).count());
  std::unique_ptr<DistHandle> h(new DistHandle());
  h->p = p;
  h->rank = rank;
  h->nranks = nranks;
  h->device = p.device;
  adopt_prereserve(h.get());
  HIPCHK(hipSetDevice(p.device));
  if (comm_id) {                         // RCCL communicator; NULL = virtual (tests)
    ncclUniqueId uid;
    std::memcpy(&uid, comm_id, sizeof(uid));
    NCCLCHK(ncclCommInitRank(&h->comm, nranks, uid, rank));
  }
  {
    const char* e = opt("MAMG_OVERLAP");
    h->overlap = e ? std::atoi(e) != 0 : true;
    e = opt("MAMG_DIST_TEST");
    h->dry = !comm_id && e && std::string(e) == "dry";
  }
  HIPCHK(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->ev_out, hipEventDisableTiming));
  const int nl = (int)plan.levels.size();
  h->L.resize(nl);
  for (int l = 0; l < nl; ++l) {
    DistLevel& P = plan.levels[l];
    DDLevel& D = h->L[l];
    D.nv = P.nv;
    D.nloc = P.nloc;
    D.ng = (int64_t)P.ghosts.size();
    D.replicated = P.replicated;
    D.coarsest = P.coarsest;
    D.send_off = P.send_off;
    D.ghost_off = P.ghost_off;
    if (D.coarsest) {
      const HostLevel& hl = H.levels[l];
      const int64_t n = hl.n, nv = n / 2;
      std::vector<double> Ap(n * n);
      auto pos = [nv](int64_t i) { return 2 * (i % nv) + i / nv; };
      for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n; ++j) Ap[pos(i) * n + pos(j)] = hl.Ainv[i * n + j];
      if ((rc = ddalloc(h.get(), &D.Ainv, n * n, err))) return rc;
      HIPCHK(hipMemcpy(D.Ainv, Ap.data(), n * n * sizeof(double), hipMemcpyHostToDevice));
    } else if (G) {
      // multicolour GS: the level's global colouring (every rank computes the
      // same one, as the single-GPU build_gs), then each colour's halo lists
      TmpPool TC;
      int8_t* gcol = nullptr;
      int ncol = 0;
      const bool rl0 = l == 0 && rings && !G->seeds.empty();   // level-0 seed rings + the rest's GS
      if ((gs || rl0) && !(l == 0 && patches)) {
        TBsr B;
        if ((rc = dev_csr_to_bsr(&TC, l == 0 ? *A0d : G->levels[l].A, D.nv, D.nv, &B, err))) return rc;
        if ((rc = gs_colour(&TC, B, l, &gcol, &ncol, err))) return rc;
        TC.release(B.ptr); TC.release(B.col); TC.release(B.val);
        if (rl0) {
          if ((rc = dist_rings(h.get(), *A0d, P, G->seeds, gcol, ncol, &D, &D.rcov, err))) return rc;
        } else if (!D.replicated && (rc = colour_halo_lists(h.get(), P, gcol, ncol, &D, err))) {
          return rc;
        }
      }
      if ((rc = dev_rank_ops(h.get(), *G, *A0d, plan, l, kw, gcol, ncol, err))) return rc;
      if (l == 0 && patches && !D.coarsest && (rc = dist_patches(h.get(), *A0d, P, &D, err))) return rc;
    } else {
      // longest run of rows without ghost columns (columns < nown): the
      // overlap windows, as ghost_free_run on the device path
      auto run_of = [](const HBsr& M, int64_t nown, int64_t* r0, int64_t* r1) {
        int64_t best0 = 0, best1 = 0, run0 = 0;
        for (int64_t I = 0; I <= M.nr; ++I) {
          bool ghost = I == M.nr;
          for (int64_t k = I < M.nr ? M.ptr[I] : 0; !ghost && k < M.ptr[I + 1]; ++k)
            ghost = M.col[k] >= nown;
          if (ghost) {
            if (I - run0 > best1 - best0) { best0 = run0; best1 = I; }
            run0 = I + 1;
          }
        }
        *r0 = best0;
        *r1 = best1;
      };
      if (!P.replicated) run_of(P.A, P.A.nr, &D.ib0, &D.ib1);
      if (l == 0 && !P.replicated && !plan.levels[1].replicated && P.K.nr > 0) {
        int64_t k0 = 0, k1 = 0;
        run_of(P.K, plan.levels[1].nloc, &k0, &k1);
        k0 = (k0 + K_ROWS_ALIGN - 1) / K_ROWS_ALIGN * K_ROWS_ALIGN;
        k1 = k1 == P.K.nr ? P.K.nr : k1 / K_ROWS_ALIGN * K_ROWS_ALIGN;
        if (k1 > k0) { D.kb0 = k0; D.kb1 = k1; }
      }
      if (l == 0) {
        if ((rc = upload_half_or_bsr(h.get(), P.A, &D.A, err))) return rc;
        if ((rc = build_band_sched_range(h.get(), &D.A, D.ib0, D.ib1, err))) return rc;
      } else if ((rc = upload_bsr(h.get(), P.A, &D.A, 0, err, true))) {
        return rc;
      }
      if (P.K.nr > 0) {
        if ((rc = upload_bsr(h.get(), P.K, &D.K, 0, err))) return rc;
      } else if (P.PA.nr > 0) {
        if ((rc = upload_bsr(h.get(), P.PA, &D.PA, 0, err))) return rc;
      } else {
        if ((rc = upload_bsr(h.get(), P.P, &D.P, 0, err))) return rc;
      }
      if ((rc = upload_bsr(h.get(), P.Rp, &D.R, 0, err))) return rc;
      if ((rc = ddalloc(h.get(), &D.W, D.nloc, err))) return rc;
      HIPCHK(hipMemcpy(D.W, P.W.data(), 4 * D.nloc * sizeof(double), hipMemcpyHostToDevice));
    }
    if (!D.coarsest) {
      if (p.smoother == MAMG_SMOOTHER_POLY) {   // w_k W as on one GPU (poly_scaled)
        for (int k = 0; k < pm; ++k) {
          dv4* q = nullptr;
          if ((rc = ddalloc(h.get(), &q, D.nloc, err))) return rc;
          if (D.nloc)
            wscale_kernel<<<nblocks(4 * D.nloc), 256>>>(4 * D.nloc, pw[k], reinterpret_cast<const double*>(D.W),
                                                         reinterpret_cast<double*>(q));
          HIPCHK(hipGetLastError());
          D.Wk.push_back(q);
        }
      }
    }
    const int64_t full = D.nloc + D.ng;
    if ((rc = ddalloc(h.get(), &D.b, 2 * full, err))) return rc;
    if ((rc = ddalloc(h.get(), &D.x, 2 * full, err))) return rc;
    if ((rc = ddalloc(h.get(), &D.t, 2 * full, err))) return rc;
    if ((rc = ddalloc(h.get(), &D.t2, 2 * full, err))) return rc;
    if ((rc = ddalloc(h.get(), &D.r, 2 * full, err))) return rc;
    if (l == 0 && !D.coarsest && (rc = ddalloc(h.get(), &D.spx, 2 * full, err))) return rc;
    if ((D.patches || D.rings) && (rc = ddalloc(h.get(), &D.pb, 2 * full, err))) return rc;
    if (l > 0 && p.cycle_type == MAMG_W_CYCLE) {
      if ((rc = ddalloc(h.get(), &D.c, 2 * full, err))) return rc;
      if ((rc = ddalloc(h.get(), &D.e, 2 * full, err))) return rc;
    }
    if (l > 0 && p.coarse_scaling) {
      if ((rc = ddalloc(h.get(), &D.q, 2 * full, err))) return rc;
      if ((rc = ddalloc(h.get(), &D.part2, 2 * SCALE_BLOCKS, err))) return rc;
    }
    const int64_t ns = P.send_idx.size();
    // colour halos: a node in the lists of every colour that writes it (node
    // patches), so their totals may exceed the plain lists
    const int64_t tcs = D.cs_off.empty() ? 0 : D.cs_off.back(), tcg = D.cg_off.empty() ? 0 : D.cg_off.back();
    if (ns) {
      if ((rc = ddalloc(h.get(), &D.send_idx, ns, err))) return rc;
      HIPCHK(hipMemcpy(D.send_idx, P.send_idx.data(), ns * sizeof(int64_t), hipMemcpyHostToDevice));
    }
    if (std::max(ns, tcs) > 0 && (rc = ddalloc(h.get(), &D.sendbuf, 2 * std::max(ns, tcs), err))) return rc;
    const int64_t nrcv = std::max(std::max(ns, D.ng), tcg);
    if (nrcv > 0 && (rc = ddalloc(h.get(), &D.recvbuf, 2 * nrcv, err))) return rc;
  }
  h->nv0 = plan.levels[0].nv;
  h->o0 = plan.levels[0].o0;
  h->o1 = plan.levels[0].o1;
  // the rank-local operators are not re-homed: they are plain allocations
  // made after the setup already, and a second copy measured 204-208 vs
  // 209-214 applies/s (2 ranks, one GPU, profiles/r02_bench_2rank_rehome_ab.txt)
  std::vector<DOp> ops;
  dapply_ops(h.get(), nullptr, nullptr, &ops);
  for (const DOp& d : ops) h->apply_bytes += d.bytes;
  HIPCHK(null_sync());
  *out = h.release();
  return MAMG_OK;
}

void dist_destroy(DistHandle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->last) (void)hipEventSynchronize(h->last);   // the last apply / spmv / timing on any stream
  if (h->side) (void)hipStreamSynchronize(h->side);
  delete h;
}

void dist_range(const DistHandle* h, int64_t* o0, int64_t* o1, int64_t* nv) {
  *o0 = h->o0; *o1 = h->o1; *nv = h->nv0;
}

double dist_apply_bytes(const DistHandle* h) { return h->apply_bytes; }

int dist_mark(DistHandle* h, hipStream_t s, std::string* err) {
  if (!h->last) HIPCHK(hipEventCreateWithFlags(&h->last, hipEventDisableTiming));
  HIPCHK(hipEventRecord(h->last, s));
  return MAMG_OK;
}

// What one distributed apply issues on a rank with P > 1 peers over RCCL
// (the same walk as run_dop, nothing launched): c[0] kernels, c[1] RCCL
// send / receive groups, c[2] point-to-point messages, c[3] all-reduces,
// c[4] stream forks (interior rows on the side stream).  With P == 1 only
// the kernels remain.
void dist_apply_launches(const DistHandle* h, int64_t c[5]) {
  for (int k = 0; k < 5; ++k) c[k] = 0;
  std::vector<DOp> ops;
  dapply_ops(h, nullptr, nullptr, &ops);
  const int P = h->nranks;
  for (const DOp& d : ops) {
    if (d.dk == D_OP || (P == 1 && d.dk == D_OVERLAP)) { ++c[0]; continue; }
    if (P == 1) continue;
    if (d.dk == D_ALLREDUCE) { ++c[3]; continue; }
    const DDLevel& D = h->L[d.level];
    const int64_t ns = D.send_off.back();
    if (d.dk == D_OVERLAP) { ++c[0]; ++c[4]; }
    if (d.dk == D_OVERLAP || d.dk == D_HALO) {
      if (ns) ++c[0];
      ++c[1];
      for (int q = 0; q < P; ++q) {
        if (q == h->rank) continue;
        c[2] += (D.send_off[q + 1] > D.send_off[q]) + (D.ghost_off[q + 1] > D.ghost_off[q]);
      }
    } else if (d.dk == D_CHALO) {
      const size_t b0 = (size_t)d.colour * (P + 1);
      c[0] += (D.cs_off[b0 + P] > D.cs_off[b0]) + (D.cg_off[b0 + P] > D.cg_off[b0]);
      ++c[1];
      for (int q = 0; q < P; ++q) {
        if (q == h->rank) continue;
        c[2] += (D.cs_off[b0 + q + 1] > D.cs_off[b0 + q]) + (D.cg_off[b0 + q + 1] > D.cg_off[b0 + q]);
      }
    } else {   // D_REVERSE
      ++c[1];
      for (int q = 0; q < P; ++q) {
        if (q == h->rank) continue;
        const bool sc = D.send_off[q + 1] > D.send_off[q], gc = D.ghost_off[q + 1] > D.ghost_off[q];
        c[2] += sc + gc;
        c[0] += sc;
      }
    }
  }
}

int dist_apply(DistHandle* h, const double* d_r, double* d_z, void* stream, std::string* err) {
  HIPCHK(hipSetDevice(h->device));
  std::vector<DOp> ops;
  dapply_ops(h, d_r, d_z, &ops);
  for (const DOp& d : ops) {
    int rc = run_dop(h, d, (hipStream_t)stream, err);
    if (rc) return rc;
  }
  HIPCHK(hipGetLastError());
  return dist_mark(h, (hipStream_t)stream, err);
}

int dist_spmv(DistHandle* h, const double* d_x, double* d_y, void* stream, std::string* err) {
  HIPCHK(hipSetDevice(h->device));
  if (h->L.empty() || h->L[0].coarsest) { *err = "single-level hierarchy: no distributed operator"; return MAMG_ERR_ARG; }
  std::vector<DOp> ops;
  dspmv_ops(h, d_x, d_y, &ops);
  for (const DOp& d : ops) {
    int rc = run_dop(h, d, (hipStream_t)stream, err);
    if (rc) return rc;
  }
  HIPCHK(hipGetLastError());
  return dist_mark(h, (hipStream_t)stream, err);
}

// The op list of one apply captured into a hipGraph on the handle's capture
// stream: kernels, the side-stream fork of the interior rows (events), and
// the RCCL send / receive groups and all-reduces inside the capture.  A
// failed capture leaves nothing behind and is reported (the caller stays
// eager).
int dist_capture(DistHandle* h, const std::vector<DOp>& ops, hipGraph_t* gr, hipGraphExec_t* ex, std::string* err) {
  *gr = nullptr;
  *ex = nullptr;
  std::lock_guard<std::recursive_mutex> capture_lock(capture_mutex());
  if (!h->cap) HIPCHK(hipStreamCreateWithFlags(&h->cap, hipStreamNonBlocking));
  HIPCHK(hipStreamBeginCapture(h->cap, hipStreamCaptureModeThreadLocal));
  int rc = MAMG_OK;
  for (const DOp& d : ops)
    if ((rc = run_dop(h, d, h->cap, err))) break;
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(h->cap, &g);
  if (rc || e != hipSuccess) {
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    if (!rc) *err = std::string("stream capture of the distributed apply: ") + hipGetErrorString(e);
    return rc ? rc : MAMG_ERR_HIP;
  }
  const hipError_t ei = graph_instantiate(ex, g);
  if (ei != hipSuccess) {
    (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    *err = std::string("hipGraphInstantiate of the distributed apply: ") + hipGetErrorString(ei);
    return MAMG_ERR_HIP;
  }
  *gr = g;
  return MAMG_OK;
}

int dist_graph_exec(DistHandle* h, const double* d_r, double* d_z, hipGraphExec_t* ex, std::string* err) {
  if (!h->comm && h->nranks > 1 && !h->dry) {
    *err = "graph replay needs an RCCL communicator (or one rank): host-staged and virtual exchanges run eagerly";
    return MAMG_ERR_UNSUPPORTED;
  }
  if (!h->graph_err.empty()) { *err = "graph capture failed on this handle: " + h->graph_err; return MAMG_ERR_UNSUPPORTED; }
  for (auto& g : h->graphs)
    if (g.r == d_r && g.z == d_z) { *ex = g.e; return MAMG_OK; }
  if (h->graphs.size() >= 16) {   // evict the oldest once every launch on the handle finished
    if (h->last) HIPCHK(hipEventSynchronize(h->last));
    (void)hipGraphExecDestroy(h->graphs.front().e);
    (void)hipGraphDestroy(h->graphs.front().g);
    h->graphs.erase(h->graphs.begin());
  }
  std::vector<DOp> ops;
  dapply_ops(h, d_r, d_z, &ops);
  DistHandle::Graph g{d_r, d_z, nullptr, nullptr};
  const int rc = dist_capture(h, ops, &g.g, &g.e, err);
  if (rc) {
    h->graph_err = *err;
    return rc;
  }
  h->graphs.push_back(g);
  *ex = g.e;
  return MAMG_OK;
}

int dist_graph_prepare(DistHandle* h, const double* d_r, double* d_z, std::string* err) {
  HIPCHK(hipSetDevice(h->device));
  hipGraphExec_t ex = nullptr;
  return dist_graph_exec(h, d_r, d_z, &ex, err);
}

int dist_apply_graph(DistHandle* h, const double* d_r, double* d_z, void* stream, std::string* err) {
  HIPCHK(hipSetDevice(h->device));
  hipGraphExec_t ex = nullptr;
  const int rc = dist_graph_exec(h, d_r, d_z, &ex, err);
  if (rc) return rc;
  HIPCHK(hipGraphLaunch(ex, (hipStream_t)stream));
  return dist_mark(h, (hipStream_t)stream, err);
}

int dist_time_apply(DistHandle* h, const double* d_r, double* d_z, int reps, int mode, double* ms,
                    double* kernel_ms, double* class_bytes, void* stream, std::string* err) {
  HIPCHK(hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  std::vector<DOp> ops;
  dapply_ops(h, d_r, d_z, &ops);
  if (class_bytes) {
    for (int c = 0; c < 16; ++c) class_bytes[c] = 0.0;
    for (const DOp& d : ops) class_bytes[d.cls] += d.bytes;
  }
  if (reps <= 0) { *ms = 0.0; return MAMG_OK; }
  if (mode == 2) {   // graph replays, events around the whole run only
    hipGraphExec_t ex = nullptr;
    int rc = dist_graph_exec(h, d_r, d_z, &ex, err);
    if (rc) return rc;
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, s));
    for (int rp = 0; rp < reps; ++rp) HIPCHK(hipGraphLaunch(ex, s));
    HIPCHK(hipEventRecord(e1, s));
    HIPCHK(hipEventSynchronize(e1));
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, e0, e1));
    *ms = t / reps;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (kernel_ms)
      for (int c = 0; c < 16; ++c) kernel_ms[c] = 0.0;
    return dist_mark(h, s, err);
  }
  std::vector<int> inst;
  for (size_t k = 0; k < ops.size(); ++k)
    if (mode == 1 || ops[k].cls == C_L0_RESID || ops[k].cls == C_L0_SMOOTH) inst.push_back((int)k);
  std::vector<hipEvent_t> ev(2 * inst.size() * (size_t)reps + 2);
  for (auto& e : ev) HIPCHK(hipEventCreate(&e));
  HIPCHK(hipEventRecord(ev[0], s));
  size_t q = 2;
  int rc;
  for (int rp = 0; rp < reps; ++rp) {
    size_t ii = 0;
    for (size_t k = 0; k < ops.size(); ++k) {
      const bool timed = ii < inst.size() && inst[ii] == (int)k;
      if (timed) HIPCHK(hipEventRecord(ev[q], s));
      if ((rc = run_dop(h, ops[k], s, err))) return rc;
      if (timed) { HIPCHK(hipEventRecord(ev[q + 1], s)); q += 2; ++ii; }
    }
  }
  HIPCHK(hipEventRecord(ev[1], s));
  HIPCHK(hipEventSynchronize(ev[1]));
  HIPCHK(hipGetLastError());
  float tot = 0.f;
  HIPCHK(hipEventElapsedTime(&tot, ev[0], ev[1]));
  *ms = tot / reps;
  if (kernel_ms) {
    for (int c = 0; c < 16; ++c) kernel_ms[c] = 0.0;
    q = 2;
    for (int rp = 0; rp < reps; ++rp)
      for (size_t ii = 0; ii < inst.size(); ++ii) {
        float t = 0.f;
        HIPCHK(hipEventElapsedTime(&t, ev[q], ev[q + 1]));
        kernel_ms[ops[inst[ii]].cls] += t / reps;
        q += 2;
      }
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  return MAMG_OK;
}

}  // namespace mamg

// ---------------------------------------------------------------------------
// Virtual communicator (tests on a single GPU): P rank handles on one device,
// executed in lockstep on one stream; exchanges are device copies between the
// ranks' buffers with exactly the counts/offsets the RCCL path uses.
// ---------------------------------------------------------------------------
namespace mamg {

__global__ __launch_bounds__(256) void vsum_kernel(int64_t n, const double* __restrict__ a,
                                                   double* acc) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) acc[i] = acc[i] + a[i];
}

// P ranks' op lists in lockstep on one stream
int virtual_run(const std::vector<DistHandle*>& hs, const std::vector<std::vector<DOp>>& ops, hipStream_t s,
                std::string* err, bool mark = true) {
  const int P = (int)hs.size();
  for (int p = 1; p < P; ++p)
    if (ops[p].size() != ops[0].size()) { *err = "rank schedules differ"; return MAMG_ERR_SETUP; }
  for (size_t k = 0; k < ops[0].size(); ++k) {
    const int dk = ops[0][k].dk;
    if (dk == D_OP) {
      for (int p = 0; p < P; ++p) launch(ops[p][k].op, s);
    } else if (dk == D_HALO || dk == D_OVERLAP) {
      if (dk == D_OVERLAP)
        for (int p = 0; p < P; ++p) launch(ops[p][k].op, s);
      for (int p = 0; p < P; ++p) {
        const DDLevel& D = hs[p]->L[ops[p][k].level];
        const int64_t ns = D.send_off.back();
        if (ns) pack2_kernel<<<nblocks(ns), 256, 0, s>>>(ns, D.send_idx, ops[p][k].buf, D.sendbuf);
      }
      for (int p = 0; p < P; ++p) {          // p receives from q
        const DDLevel& D = hs[p]->L[ops[p][k].level];
        for (int q = 0; q < P; ++q) {
          if (q == p) continue;
          const int64_t gc = D.ghost_off[q + 1] - D.ghost_off[q];
          if (!gc) continue;
          const DDLevel& Q = hs[q]->L[ops[q][k].level];
          const int64_t sc = Q.send_off[p + 1] - Q.send_off[p];
          if (sc != gc) { *err = "halo count mismatch"; return MAMG_ERR_SETUP; }
          HIPCHK(dev_copy(ops[p][k].buf + 2 * (D.nloc + D.ghost_off[q]), Q.sendbuf + 2 * Q.send_off[p], 2 * gc * sizeof(double), s));
        }
      }
    } else if (dk == D_CHALO) {
      const int c = ops[0][k].colour;
      const size_t b0 = (size_t)c * (P + 1);
      for (int p = 0; p < P; ++p) {
        const DDLevel& D = hs[p]->L[ops[p][k].level];
        const int64_t s0 = D.cs_off[b0], s1 = D.cs_off[b0 + P];
        if (s1 > s0)
          pack2_kernel<<<nblocks(s1 - s0), 256, 0, s>>>(s1 - s0, D.csend_idx + s0, ops[p][k].buf, D.sendbuf + 2 * s0);
      }
      for (int p = 0; p < P; ++p) {          // p receives colour c's ghosts from q
        const DDLevel& D = hs[p]->L[ops[p][k].level];
        for (int q = 0; q < P; ++q) {
          if (q == p) continue;
          const int64_t gc = D.cg_off[b0 + q + 1] - D.cg_off[b0 + q];
          const DDLevel& Q = hs[q]->L[ops[q][k].level];
          const int64_t sc = Q.cs_off[b0 + p + 1] - Q.cs_off[b0 + p];
          if (sc != gc) { *err = "colour halo count mismatch"; return MAMG_ERR_SETUP; }
          if (!gc) continue;
          HIPCHK(dev_copy(D.recvbuf + 2 * D.cg_off[b0 + q], Q.sendbuf + 2 * Q.cs_off[b0 + p], 2 * gc * sizeof(double), s));
        }
      }
      for (int p = 0; p < P; ++p) {
        const DDLevel& D = hs[p]->L[ops[p][k].level];
        const int64_t g0 = D.cg_off[b0], g1 = D.cg_off[b0 + P];
        if (g1 > g0)
          unpack2_kernel<<<nblocks(g1 - g0), 256, 0, s>>>(g1 - g0, D.cghost_idx + g0, D.nloc, D.recvbuf + 2 * g0,
                                                          ops[p][k].buf);
      }
    } else if (dk == D_REVERSE) {
      for (int q = 0; q < P; ++q) {          // owner q receives partials from p
        const DDLevel& Q = hs[q]->L[ops[q][k].level];
        for (int p = 0; p < P; ++p) {
          if (p == q) continue;
          const int64_t sc = Q.send_off[p + 1] - Q.send_off[p];
          if (!sc) continue;
          const DDLevel& D = hs[p]->L[ops[p][k].level];
          const int64_t gc = D.ghost_off[q + 1] - D.ghost_off[q];
          if (sc != gc) { *err = "reverse count mismatch"; return MAMG_ERR_SETUP; }
          HIPCHK(dev_copy(Q.recvbuf + 2 * Q.send_off[p], ops[p][k].buf + 2 * (D.nloc + D.ghost_off[q]), 2 * sc * sizeof(double), s));
        }
      }
      for (int q = 0; q < P; ++q) {
        const DDLevel& Q = hs[q]->L[ops[q][k].level];
        for (int p = 0; p < P; ++p) {
          const int64_t sc = Q.send_off[p + 1] - Q.send_off[p];
          if (p == q || !sc) continue;
          addidx2_kernel<<<nblocks(sc), 256, 0, s>>>(sc, Q.send_idx + Q.send_off[p],
                                                     Q.recvbuf + 2 * Q.send_off[p], ops[q][k].buf);
        }
      }
    } else {                                 // D_ALLREDUCE: sum in rank order
      const int64_t n = ops[0][k].count;
      for (int p = 1; p < P; ++p)
        vsum_kernel<<<nblocks(n), 256, 0, s>>>(n, ops[p][k].buf, ops[0][k].buf);
      for (int p = 1; p < P; ++p)
        HIPCHK(dev_copy(ops[p][k].buf, ops[0][k].buf, n * sizeof(double), s));
    }
  }
  HIPCHK(hipGetLastError());
  if (mark)
    for (DistHandle* h : hs) {
      const int rc = dist_mark(h, s, err);
      if (rc) return rc;
    }
  return MAMG_OK;
}

int dist_set_exchange(DistHandle* h, const mamg_exchange& ex, std::string* err) {
  if (h->comm) { *err = "handle has an RCCL communicator; the host exchange is for comm_id == NULL"; return MAMG_ERR_ARG; }
  HIPCHK(hipSetDevice(h->device));
  auto pin = [&](double** p, int64_t n) -> int {
    *p = nullptr;
    if (n <= 0) return MAMG_OK;
    void* q = nullptr;
    HIPCHK(hipHostMalloc(&q, n * sizeof(double), hipHostMallocDefault));
    h->pinned.push_back(q);
    *p = (double*)q;
    return MAMG_OK;
  };
  if (!h->host_ex) {
    int64_t red = 0;
    const int nl = (int)h->L.size();
    h->hsend.assign(nl, nullptr);
    h->hghost.assign(nl, nullptr);
    h->hrecv.assign(nl, nullptr);
    for (int l = 0; l < nl; ++l) {
      const DDLevel& D = h->L[l];
      const int64_t ns = D.send_off.empty() ? 0 : D.send_off.back();
      const int64_t tcs = D.cs_off.empty() ? 0 : D.cs_off.back(), tcg = D.cg_off.empty() ? 0 : D.cg_off.back();
      int rc;
      if ((rc = pin(&h->hsend[l], 2 * std::max(ns, tcs))) || (rc = pin(&h->hghost[l], 2 * std::max(D.ng, tcg))) ||
          (rc = pin(&h->hrecv[l], 2 * ns)))
        return rc;
      red = std::max(red, 2 * D.nv);
    }
    red = std::max<int64_t>(red, 2 * SCALE_BLOCKS);   // coarse scaling partials
    int rc = pin(&h->hred, red);
    if (rc) return rc;
  }
  h->ex = ex;
  h->host_ex = true;
  return MAMG_OK;
}

int dist_virtual_apply(const std::vector<DistHandle*>& hs, const std::vector<const double*>& r,
                       const std::vector<double*>& z, void* stream, std::string* err) {
  const int P = (int)hs.size();
  HIPCHK(hipSetDevice(hs[0]->device));
  std::vector<std::vector<DOp>> ops(P);
  for (int p = 0; p < P; ++p) dapply_ops(hs[p], r[p], z[p], &ops[p]);
  return virtual_run(hs, ops, (hipStream_t)stream, err);
}

// the virtual ranks' lockstep apply captured into one hipGraph (rank 0's
// capture stream), launched once and destroyed: the graph path's kernels,
// forks and exchange order, checked bitwise against the eager lockstep run
int dist_virtual_apply_graph(const std::vector<DistHandle*>& hs, const std::vector<const double*>& r,
                             const std::vector<double*>& z, void* stream, std::string* err) {
  const int P = (int)hs.size();
  HIPCHK(hipSetDevice(hs[0]->device));
  std::vector<std::vector<DOp>> ops(P);
  for (int p = 0; p < P; ++p) dapply_ops(hs[p], r[p], z[p], &ops[p]);
  DistHandle* h0 = hs[0];
  std::lock_guard<std::recursive_mutex> capture_lock(capture_mutex());
  if (!h0->cap) HIPCHK(hipStreamCreateWithFlags(&h0->cap, hipStreamNonBlocking));
  HIPCHK(hipStreamBeginCapture(h0->cap, hipStreamCaptureModeThreadLocal));
  int rc = virtual_run(hs, ops, h0->cap, err, false);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(h0->cap, &g);
  if (rc || e != hipSuccess) {
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    if (!rc) *err = std::string("stream capture of the virtual apply: ") + hipGetErrorString(e);
    return rc ? rc : MAMG_ERR_HIP;
  }
  hipGraphExec_t ex = nullptr;
  const hipError_t ei = graph_instantiate(&ex, g);
  if (ei != hipSuccess) {
    (void)hipGraphDestroy(g);
    *err = std::string("hipGraphInstantiate of the virtual apply: ") + hipGetErrorString(ei);
    return MAMG_ERR_HIP;
  }
  const hipError_t el = hipGraphLaunch(ex, (hipStream_t)stream);
  const hipError_t es = hipStreamSynchronize((hipStream_t)stream);
  (void)hipGraphExecDestroy(ex);
  (void)hipGraphDestroy(g);
  if (el != hipSuccess || es != hipSuccess) {
    *err = std::string("virtual apply graph launch: ") + hipGetErrorString(el != hipSuccess ? el : es);
    return MAMG_ERR_HIP;
  }
  for (DistHandle* h : hs)
    if ((rc = dist_mark(h, (hipStream_t)stream, err))) return rc;
  return MAMG_OK;
}

int dist_virtual_spmv(const std::vector<DistHandle*>& hs, const std::vector<const double*>& x,
                      const std::vector<double*>& y, void* stream, std::string* err) {
  const int P = (int)hs.size();
  HIPCHK(hipSetDevice(hs[0]->device));
  std::vector<std::vector<DOp>> ops(P);
  for (int p = 0; p < P; ++p) {
    if (hs[p]->L.empty() || hs[p]->L[0].coarsest) { *err = "single-level hierarchy"; return MAMG_ERR_ARG; }
    dspmv_ops(hs[p], x[p], y[p], &ops[p]);
  }
  return virtual_run(hs, ops, (hipStream_t)stream, err);
}

}  // namespace mamg
