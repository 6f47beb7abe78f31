// gsetup.hip -- GPU setup of the nodal smoothed-aggregation hierarchy.
//
// Replaces the HAZmath metric-AMG setup behind
//   metricAMG(A, W, idofs=interface_dofs, parameters=...)   src/utils.py:86
// for the bidomain profile (num_functions = 2, node-block smoothers, nodal SA;
// DESIGN.md section 2.2) with gfx950 kernels, starting from A0 already in HBM.
// It computes the same hierarchy as the host setup (setup.cpp) BIT FOR BIT:
// every value is the same sequence of IEEE binary64 operations (this file is
// compiled with -ffp-contract=off; device sqrt and division are correctly
// rounded), sums run in the host's (scipy SMMP / CSR) order, exact zeros are
// dropped by the same rules, and every integer decision (strength, MIS-2,
// aggregation, seed blocks) follows setup.cpp exactly.
//
// Per level (nv nodes, 2 fields, dof f nv + I):
//   node graph     s_IJ = ||A_IJ||_F          one thread per node: 4-way merge
//   strength       flags on the node graph, symmetrised via the mirror entry
//   MIS-2          round-synchronous 2-hop max of hash keys; roots by scan
//   aggregation    distance-1 joins, then strongest aggregated neighbour
//   smoothers      2x2 node-block (or level-0 seed-block) inverses, rho_B =
//                  max_i sum_j |(D_B^-1 A)_ij| by a 2-row merge per dof
//   prolongator    A T (wave-per-row hash SpGEMM), then P = T - w D_B^-1 (A T)
//                  fused into one 2-row merge per dof
//   Galerkin       R = P^T (stable radix sort), A P and R (A P) (hash SpGEMM)
//   coarsest       dense Gauss-Jordan (no pivoting), one pivot per 3 launches
//
// Hash SpGEMM (row i of C = A B): one wavefront per row; the LDS table
// accumulates sums[j] += a_ik b_kj exactly in scipy's order (A's entries in
// CSR order, each B row's entries once).  The wave takes A's entries in
// batches of 64 / GL: lane group g (GL lanes) loads entry kb + g and its B row,
// all groups insert their columns into the table at once, then the groups add
// their products one group after another (g ascending = CSR order; within a
// group the columns are distinct, so no two lanes touch one slot).  A batch
// with a B row longer than GL falls back to one entry at a time, 64 lanes over
// its B row.  GL is chosen per product from B's mean row length.  Rows run
// first in a 128-slot table, overflowing rows in 512 and then 2048 slots; a
// row with more distinct columns than that fails loudly
// (MAMG_ERR_UNSUPPORTED) instead of degrading.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <atomic>
#include <cstring>
#include <mutex>
#include <thread>

#include "dist.h"
#include "dmem.h"
#include "opts.h"
#include "gsetup.h"
#include "rowstage.h"

typedef double dv4_t __attribute__((ext_vector_type(4)));

namespace mamg {

// buffers are null-stream ordered (dmem.h): freed behind the kernels queued
// before the free, never under them
GHier::~GHier() {
  for (void* p : allocs)
    if (p) tmp_free(p);
}

void GHier::release(void* p) {
  for (auto& q : allocs)
    if (q == p) { tmp_free(q); q = nullptr; }
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

#define RCHK(expr)              \
  do {                          \
    int rc_ = (expr);           \
    if (rc_) return rc_;        \
  } while (0)

inline unsigned nblk(int64_t work, int per = 256) { return (unsigned)std::max<int64_t>(1, (work + per - 1) / per); }

constexpr uint64_t ST_OUT = 0, ST_UND = 1, ST_IN = 2;

// same arithmetic as host.h hash32 / oracle hash32
__device__ __forceinline__ uint32_t dhash32(uint64_t i, int level) {
  uint32_t x = (uint32_t)(i & 0xFFFFFFFFu);
  uint32_t lv = (uint32_t)(((uint64_t)(int64_t)level * 0x85EBCA77ull) & 0xFFFFFFFFull);
  x = x * 0x9E3779B1u + lv;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ int64_t dfind(const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
                                         int64_t i, int64_t j) {
  int64_t lo = ptr[i], hi = ptr[i + 1];
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (col[mid] < j) lo = mid + 1; else hi = mid;
  }
  return (lo < ptr[i + 1] && col[lo] == j) ? lo : -1;
}

// ---------------------------------------------------------------------------
// owned device buffers
// ---------------------------------------------------------------------------
struct Scratch {            // temporaries of one setup call
  std::vector<void*> v;
  ~Scratch() {
    for (void* p : v) if (p) tmp_free(p);
  }
  template <class T>
  int alloc(T** p, int64_t count, std::string* err) {
    void* q = nullptr;
    HIPCHK(tmp_malloc(&q, (size_t)std::max<int64_t>(count, 1) * sizeof(T)));
    v.push_back(q);
    *p = (T*)q;
    return MAMG_OK;
  }
  void release(void* p) {
    for (auto& q : v)
      if (q == p) { tmp_free(q); q = nullptr; }
  }
};

template <class T>
int galloc(GHier* G, T** p, int64_t count, std::string* err) {
  void* q = nullptr;
  HIPCHK(tmp_malloc(&q, (size_t)std::max<int64_t>(count, 1) * sizeof(T)));
  G->allocs.push_back(q);
  *p = (T*)q;
  return MAMG_OK;
}

template <class T>
int to_host(T* dst, const T* src, int64_t count, std::string* err) {
  if (count > 0) HIPCHK(hipMemcpy(dst, src, count * sizeof(T), hipMemcpyDeviceToHost));
  return MAMG_OK;
}

// ---------------------------------------------------------------------------
// node graph (setup.cpp node_graph, nf = 2): s_IJ = sqrt(sum of squares over
// the 2x2 block), accumulated over rows I then nv + I, each in CSR order
// ---------------------------------------------------------------------------
template <bool FILL, int CAP = RS_CAP>
__global__ __launch_bounds__(64) void node_graph_kernel(int64_t nv, const int64_t* __restrict__ ptr,
                                                        const int32_t* __restrict__ col,
                                                        const double* __restrict__ val, int64_t* gptr,
                                                        int32_t* __restrict__ gcol, double* __restrict__ gval) {
  __shared__ RowStageT<FILL, CAP> S;
  const int64_t I0 = (int64_t)blockIdx.x * RS_NODES, I = I0 + threadIdx.x;
  RowView vw[2];
  stage_rows<FILL>(S, ptr, col, val, nv, I0, vw);
  if (I >= nv) return;
  Seg4 g;
  stage_segs(ptr, vw, nv, nv, I, g.k, g.e);
  g.init(vw, nv);
  int64_t o = FILL ? gptr[I] : 0;
  for (;;) {
    const int64_t J = g.next();
    if (J == INT64_MAX) break;
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q)          // order (f0,g0) (f0,g1) (f1,g0) (f1,g1)
      if (g.c[q] == J) {
        if (FILL) {
          const double a = vw[q >> 1].val(g.k[q]);
          acc += a * a;
        }
        ++g.k[q];
        g.head(vw, nv, q);
      }
    if (FILL) { gcol[o] = (int32_t)J; gval[o] = sqrt(acc); }
    ++o;
  }
  if (!FILL) gptr[I + 1] = o;
}

// The fill pass with columns only in LDS (as device.hip csr2bsr_fill_kernel):
// each lane's merge writes gcol, every entry's slot 4 (o - o0) + q in place of
// its staged column and the zeros of its blocks' missing components into the
// block scratch T; the wave then stores the values into their slots with
// coalesced loads, and every block's sum of squares is taken in the order
// (f0,g0) (f0,g1) (f1,g0) (f1,g1) -- a missing component adds +0 to a sum >= +0,
// so the bits are those of node_graph_kernel<true>.  Ranges over RS_CAP: as
// node_graph_kernel<true>.
template <int CAP>
__global__ __launch_bounds__(64) void node_graph_fill_kernel(int64_t nv, const int64_t* __restrict__ ptr,
                                                             const int32_t* __restrict__ col,
                                                             const double* __restrict__ val,
                                                             const int64_t* __restrict__ gptr,
                                                             int32_t* __restrict__ gcol, double* __restrict__ gval,
                                                             double* __restrict__ T) {
  __shared__ RowStageT<false, CAP> S;
  const int64_t I0 = (int64_t)blockIdx.x * RS_NODES, I = I0 + threadIdx.x;
  RowView vw[2];
  stage_rows<false>(S, ptr, col, val, nv, I0, vw);
  if (!vw[0].lds) {
    if (I >= nv) return;
    Seg4 g;
    stage_segs(ptr, vw, nv, nv, I, g.k, g.e);
    g.init(vw, nv);
    int64_t o = gptr[I];
    for (;;) {
      const int64_t J = g.next();
      if (J == INT64_MAX) break;
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (g.c[q] == J) {
          const double a = vw[q >> 1].val(g.k[q]);
          acc += a * a;
          ++g.k[q];
          g.head(vw, nv, q);
        }
      gcol[o] = (int32_t)J;
      gval[o] = sqrt(acc);
      ++o;
    }
    return;
  }
  const int64_t o0 = gptr[I0];
  const int64_t I1 = I0 + RS_NODES < nv ? I0 + RS_NODES : nv;
  double* tb = T + 4 * o0;
  if (I < nv) {
    Seg4 g;
    stage_segs(ptr, vw, nv, nv, I, g.k, g.e);
    g.init(vw, nv);
    int64_t o = gptr[I];
    for (;;) {
      const int64_t J = g.next();
      if (J == INT64_MAX) break;
      const int32_t rel = (int32_t)(o - o0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (g.c[q] == J) {
          S.c[q >> 1][g.k[q] - vw[q >> 1].off] = 4 * rel + q;
          ++g.k[q];
          g.head(vw, nv, q);
        } else {
          tb[4 * rel + q] = 0.0;
        }
      }
      gcol[o] = (int32_t)J;
      ++o;
    }
  }
  __syncthreads();
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int64_t b = ptr[f * nv + I0], n = ptr[f * nv + I1] - b;
    scatter_staged(S.c[f], val, b, n, tb);
  }
  __syncthreads();
  const int64_t ob = gptr[I1] - o0;
  for (int64_t r = threadIdx.x; r < ob; r += 64) {
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double a = tb[4 * r + q];
      acc += a * a;
    }
    gval[o0 + r] = sqrt(acc);
  }
}

// |diagonal| of a square CSR (0 if absent)
__global__ __launch_bounds__(256) void absdiag_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                      const int32_t* __restrict__ col, const double* __restrict__ val,
                                                      double* __restrict__ d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t p = dfind(ptr, col, i, i);
  d[i] = p >= 0 ? fabs(val[p]) : 0.0;
}

// strength (setup.cpp strength): flag the entry and its mirror; a missing
// mirror (non-symmetric pattern) is counted and rejected by the caller
__global__ __launch_bounds__(256) void strength_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ col,
                                                       const double* __restrict__ val, const double* __restrict__ d,
                                                       double theta, int rowmax, uint8_t* flag, int* nextra) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double m = 0.0;   // the row's largest coupling: theta is relative to it
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
    if (col[k] != i) m = fmax(m, fabs(val[k]));
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) {
    const int64_t j = col[k];
    if (j == i) continue;
    const double av = fabs(val[k]);
    const double s = sqrt(d[i] * d[j]);
    if ((av >= theta * (rowmax ? m : s)) && (av > 1e-12 * s)) {
      flag[k] = 1;
      const int64_t q = dfind(ptr, col, j, i);
      if (q >= 0) flag[q] = 1;
      else atomicAdd(nextra, 1);
    }
  }
}

// ---------------------------------------------------------------------------
// Sharded single-word reductions: one atomic per wave on one word serialises
// at ~88 per microsecond (MI355X_MICROARCH.md, dequeue), so a 17 M-node grid's
// 265 K wave atomics took ~3 ms (the MIS-2 key kernel: 3.17 ms per round for
// 24 B per node).  The waves of block b add into shard b mod 64 (128 B
// apart); the host sums (or maxes) the 64 shards.
// ---------------------------------------------------------------------------
constexpr int CSH = 64, CSTR = 16;
__device__ __forceinline__ unsigned long long* shard_of(unsigned long long* c) {
  return c + (blockIdx.x & (CSH - 1)) * CSTR;
}

// ---------------------------------------------------------------------------
// MIS-2 aggregation (setup.cpp aggregate_mis2)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mis_init_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                       const uint8_t* __restrict__ flag, int level,
                                                       uint64_t* __restrict__ state, uint64_t* __restrict__ low,
                                                       uint8_t* __restrict__ nonisol) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  bool any = false;
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) any |= flag[k] != 0;
  nonisol[i] = any;
  state[i] = any ? ST_UND : ST_OUT;
  low[i] = ((uint64_t)(dhash32((uint64_t)i, level) & 0x7FFFFFFFu) << 31) | (uint64_t)i;
}

__global__ __launch_bounds__(256) void mis_key_kernel(int64_t n, const uint64_t* __restrict__ state,
                                                      const uint64_t* __restrict__ low, uint64_t* __restrict__ key,
                                                      unsigned long long* und) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool u = false;
  if (i < n) {
    key[i] = (state[i] << 62) | low[i];
    u = state[i] == ST_UND;
  }
  const unsigned long long b = __ballot(u);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(shard_of(und), (unsigned long long)__popcll(b));
}

__global__ __launch_bounds__(256) void mis_max_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                      const int32_t* __restrict__ col,
                                                      const uint8_t* __restrict__ flag,
                                                      const uint64_t* __restrict__ in, uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint64_t m = in[i];
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
    if (flag[k]) m = max(m, in[col[k]]);
  out[i] = m;
}

__global__ __launch_bounds__(256) void mis_update_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ col,
                                                         const uint8_t* __restrict__ flag,
                                                         const uint64_t* __restrict__ m1,
                                                         const uint64_t* __restrict__ key,
                                                         uint64_t* __restrict__ state) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n || state[i] != ST_UND) return;
  uint64_t m = m1[i];
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
    if (flag[k]) m = max(m, m1[col[k]]);
  if (m == key[i]) state[i] = ST_IN;
  else if ((m >> 62) == ST_IN) state[i] = ST_OUT;
}

// The same two maxima with the workgroup's rows staged (round 5): lane t
// loads entry b + t of the 256 nodes' contiguous entry range (coalesced col /
// flag reads, MM_BATCH gathers in flight) and stores flag ? x[col] : 0 into
// LDS; each node's lane then takes the max over its LDS range.  A max is
// exact in any order and 0 is its identity over keys, so the results are those
// of mis_max_kernel / mis_update_kernel (whose lane-per-row walks split every
// load into ~64 cache-line requests: 1.6 ms per level-0 round, ~16 rounds).
// Ranges over MM_CAP: the row walk.
constexpr int MM_CAP = 6144, MM_BATCH = 4;
template <bool UPDATE>
__global__ __launch_bounds__(256) void mis_staged_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ col,
                                                         const uint8_t* __restrict__ flag,
                                                         const uint64_t* __restrict__ x,
                                                         const uint64_t* __restrict__ key,
                                                         uint64_t* __restrict__ out) {
  __shared__ uint64_t L[MM_CAP];
  const int64_t i0 = (int64_t)blockIdx.x * 256, i1 = i0 + 256 < n ? i0 + 256 : n, i = i0 + threadIdx.x;
  const int64_t b = ptr[i0], m = ptr[i1] - b;
  if (m > MM_CAP) {
    if (i >= n || (UPDATE && out[i] != ST_UND)) return;
    uint64_t v = x[i];
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
      if (flag[k]) v = max(v, x[col[k]]);
    if (!UPDATE) out[i] = v;
    else if (v == key[i]) out[i] = ST_IN;
    else if ((v >> 62) == ST_IN) out[i] = ST_OUT;
    return;
  }
  for (int64_t t0 = 0; t0 < m; t0 += 256 * MM_BATCH) {
    int32_t c[MM_BATCH];
    uint8_t f[MM_BATCH];
#pragma unroll
    for (int u = 0; u < MM_BATCH; ++u) {
      const int64_t t = t0 + u * 256 + threadIdx.x;
      f[u] = 0;
      if (t < m) { c[u] = col[b + t]; f[u] = flag[b + t]; }
    }
    uint64_t v[MM_BATCH];
#pragma unroll
    for (int u = 0; u < MM_BATCH; ++u) v[u] = f[u] ? x[c[u]] : 0;
#pragma unroll
    for (int u = 0; u < MM_BATCH; ++u) {
      const int64_t t = t0 + u * 256 + threadIdx.x;
      if (t < m) L[t] = v[u];
    }
  }
  __syncthreads();
  if (i >= n || (UPDATE && out[i] != ST_UND)) return;
  uint64_t v = x[i];
  for (int64_t k = ptr[i] - b, e = ptr[i + 1] - b; k < e; ++k) v = max(v, L[k]);
  if (!UPDATE) out[i] = v;
  else if (v == key[i]) out[i] = ST_IN;
  else if ((v >> 62) == ST_IN) out[i] = ST_OUT;
}

__global__ __launch_bounds__(256) void root_flag_kernel(int64_t n, const uint64_t* __restrict__ state,
                                                        int64_t* __restrict__ f) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) f[i] = state[i] == ST_IN;
}

// agg = root number (inclusive scan - 1) for roots, -1 otherwise
__global__ __launch_bounds__(256) void root_number_kernel(int64_t n, const uint64_t* __restrict__ state,
                                                          const int64_t* __restrict__ scan, int64_t* __restrict__ agg) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) agg[i] = state[i] == ST_IN ? scan[i] - 1 : -1;
}

// phase 2: a non-root joins its (unique) strong root neighbour
__global__ __launch_bounds__(256) void agg_phase2_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ col,
                                                         const uint8_t* __restrict__ flag,
                                                         const uint64_t* __restrict__ state,
                                                         const int64_t* __restrict__ agg, int64_t* __restrict__ agg2) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int64_t a = agg[i];
  if (state[i] != ST_IN)
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
      if (flag[k] && state[col[k]] == ST_IN) a = agg[col[k]];
  agg2[i] = a;
}

// phase 3: remaining non-isolated nodes join the strongest aggregated
// neighbour (weight |s_IJ| * 1.0; ties: smallest aggregate id)
__global__ __launch_bounds__(256) void agg_phase3_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ col,
                                                         const double* __restrict__ val,
                                                         const uint8_t* __restrict__ flag,
                                                         const uint8_t* __restrict__ nonisol,
                                                         const int64_t* __restrict__ agg2, int64_t* __restrict__ agg3,
                                                         int* bad) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (!nonisol[i] || agg2[i] >= 0) { agg3[i] = agg2[i]; return; }
  double bw = -1.0;
  int64_t ba = -1;
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) {
    if (!flag[k]) continue;
    const double w = fabs(val[k]) * 1.0;
    if (w == 0.0) continue;
    const int64_t a = agg2[col[k]];
    if (a < 0) continue;
    if (w > bw || (w == bw && a < ba)) { bw = w; ba = a; }
  }
  if (ba < 0) atomicAdd(bad, 1);
  agg3[i] = ba;
}

// ---------------------------------------------------------------------------
// parallel heavy-edge matching (setup.cpp aggregate_hem / hem_match)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t dedge_hash(int64_t i, int64_t j, int lvl) {
  const int64_t a = i < j ? i : j, b = i < j ? j : i;
  return dhash32((uint64_t)a, 0x5000 + lvl) ^ dhash32((uint64_t)b, 0x6000 + lvl);
}

// compacted copy of a CSR: entries with flag (if given), off the diagonal
// (if nodiag), weight |v| * 1.0 (if absval) that is not 0.0; count / fill
template <bool FILL>
__global__ __launch_bounds__(256) void wgraph_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                     const int32_t* __restrict__ col, const double* __restrict__ val,
                                                     const uint8_t* __restrict__ flag, int absval,
                                                     int64_t* __restrict__ optr, int32_t* __restrict__ ocol,
                                                     double* __restrict__ oval) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int64_t o = FILL ? optr[i] : 0;
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) {
    if (flag && !flag[k]) continue;
    if (col[k] == i) continue;
    const double w = absval ? fabs(val[k]) * 1.0 : val[k];
    if (w == 0.0) continue;
    if (FILL) { ocol[o] = col[k]; oval[o] = w; }
    ++o;
  }
  if (!FILL) optr[i + 1] = o;
}

__global__ __launch_bounds__(256) void hem_pick_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ col,
                                                       const double* __restrict__ val,
                                                       const uint8_t* __restrict__ act,
                                                       const int64_t* __restrict__ mate, int lvl,
                                                       int64_t* __restrict__ choice) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int64_t best = -1;
  double bw = 0.0;
  uint32_t bh = 0;
  if (act[i] && mate[i] < 0)
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) {
      const int64_t j = col[k];
      if (j == i || !act[j] || mate[j] >= 0) continue;
      const double w = val[k];
      const uint32_t h = dedge_hash(i, j, lvl);
      if (best < 0 || w > bw || (w == bw && (h > bh || (h == bh && j < best)))) {
        best = j; bw = w; bh = h;
      }
    }
  choice[i] = best;
}

__global__ __launch_bounds__(256) void hem_mutual_kernel(int64_t n, const int64_t* __restrict__ choice,
                                                         int64_t* __restrict__ mate, unsigned long long* got) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool m = false;
  if (i < n) {
    const int64_t c = choice[i];
    if (c >= 0 && choice[c] == i) { mate[i] = c; m = true; }
  }
  const unsigned long long b = __ballot(m);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(shard_of(got), (unsigned long long)__popcll(b));
}

// root = smallest member of a pair (or the unmatched node itself)
__global__ __launch_bounds__(256) void hem_root_kernel(int64_t n, const uint8_t* __restrict__ act,
                                                       const int64_t* __restrict__ mate, int64_t* __restrict__ f) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) f[i] = act[i] && (mate[i] < 0 || i < mate[i]);
}

__global__ __launch_bounds__(256) void hem_number_kernel(int64_t n, const uint8_t* __restrict__ act,
                                                         const int64_t* __restrict__ mate,
                                                         const int64_t* __restrict__ scan, int64_t* __restrict__ a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (!act[i]) { a[i] = -1; return; }
  const int64_t r = (mate[i] >= 0 && mate[i] < i) ? mate[i] : i;
  a[i] = scan[r] - 1;
}

__global__ __launch_bounds__(256) void hem_compose_kernel(int64_t n, const int64_t* __restrict__ a,
                                                          int64_t* __restrict__ agg) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n && agg[i] >= 0) agg[i] = a[agg[i]];
}

// T of one pass: row i -> a[i] (value 1) where act[i]; ptr = inclusive scan of act
__global__ __launch_bounds__(256) void hem_t_kernel(int64_t n, const uint8_t* __restrict__ act,
                                                    const int64_t* __restrict__ a, int64_t* __restrict__ tptr,
                                                    int32_t* __restrict__ tcol, double* __restrict__ tval, int fill) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (!fill) { tptr[i + 1] = act[i] ? 1 : 0; return; }
  if (act[i]) { tcol[tptr[i]] = (int32_t)a[i]; tval[tptr[i]] = 1.0; }
}

__global__ __launch_bounds__(256) void agg_size_kernel(int64_t n, const int64_t* __restrict__ agg,
                                                       unsigned long long* __restrict__ size) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n && agg[i] >= 0) atomicAdd(size + agg[i], 1ull);
}

// a node alone in its aggregate joins the heaviest strong neighbour's
// aggregate of >= 2 members (ties: smallest id; setup.cpp aggregate_hem)
__global__ __launch_bounds__(256) void hem_absorb_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ col,
                                                         const double* __restrict__ val,
                                                         const int64_t* __restrict__ agg,
                                                         const unsigned long long* __restrict__ size,
                                                         int64_t* __restrict__ agg2, int64_t* __restrict__ used) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int64_t a0 = agg[i];
  if (a0 >= 0 && size[a0] == 1) {
    double bw = 0.0;
    int64_t ba = -1;
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) {
      const int64_t a = agg[col[k]];
      if (a < 0 || size[a] < 2) continue;
      const double w = val[k];
      if (ba < 0 || w > bw || (w == bw && a < ba)) { bw = w; ba = a; }
    }
    if (ba >= 0) a0 = ba;
  }
  agg2[i] = a0;
  if (a0 >= 0) used[a0] = 1;   // benign race: every writer stores 1
}

__global__ __launch_bounds__(256) void agg_remap_kernel(int64_t n, const int64_t* __restrict__ agg2,
                                                        const int64_t* __restrict__ scan, int64_t* __restrict__ agg) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) agg[i] = agg2[i] >= 0 ? scan[agg2[i]] - 1 : -1;
}

__global__ __launch_bounds__(256) void nonzero_flag_kernel(int64_t n, const int64_t* __restrict__ cnt,
                                                           uint8_t* __restrict__ act) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) act[i] = cnt[i + 1] > 0;
}

__global__ __launch_bounds__(256) void u8_fill_kernel(int64_t n, uint8_t v, uint8_t* __restrict__ p) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ __launch_bounds__(256) void iota_nonisol_kernel(int64_t n, const uint8_t* __restrict__ act,
                                                           int64_t* __restrict__ agg) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) agg[i] = act[i] ? i : -1;
}

// ---------------------------------------------------------------------------
// smoother / SA node blocks
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void seed_mark_kernel(int64_t m, const int32_t* __restrict__ idofs, int64_t n,
                                                        uint8_t* __restrict__ isseed, int* bad) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= m) return;
  const int32_t s = idofs[t];
  if (s < 0 || s >= n) { atomicAdd(bad, 1); return; }
  isseed[s] = 1;
}

// strongest seed neighbour of every non-seed dof (setup.cpp block_smoother):
// max |a_js| over seed columns s != j, ties to the smaller s.  Eight lanes per
// row, each over a strided part of it, then a butterfly of the eight
// candidates: the order (|a| desc, s asc) is total, so the result is the
// sequential scan's in any order (NaN entries never win either way)
__global__ __launch_bounds__(256) void best_seed_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                        const int32_t* __restrict__ col,
                                                        const double* __restrict__ val,
                                                        const uint8_t* __restrict__ isseed, int64_t* __restrict__ best) {
  const int lane = threadIdx.x & 7;
  const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 3;
  double bv = -1.0;
  int64_t bs = -1;
  if (j < n && !isseed[j])
    for (int64_t k = ptr[j] + lane; k < ptr[j + 1]; k += 8) {
      const int64_t s = col[k];
      if (s == j || !isseed[s]) continue;
      const double v = fabs(val[k]);
      if (v > bv || (v == bv && s < bs)) { bv = v; bs = s; }
    }
#pragma unroll
  for (int off = 4; off > 0; off >>= 1) {
    const double ov = __shfl_xor(bv, off, 8);
    const int64_t os = __shfl_xor(bs, off, 8);
    if (ov > bv || (ov == bv && os < bs && os >= 0)) { bv = ov; bs = os; }
  }
  if (j < n && lane == 0) best[j] = bs;
}

// fast test of the common case: every joiner's strongest seed is its own
// node's other dof (then each seed has at most that one joiner, and the
// blocks are node-aligned exactly as block_smoother builds them);
// joined[I]: dofs I and nv + I form one block (needs Schwarz_mmsize >= 2)
__global__ __launch_bounds__(256) void seed_align_kernel(int64_t nv, const uint8_t* __restrict__ isseed,
                                                         const int64_t* __restrict__ best, int mmsize,
                                                         uint8_t* __restrict__ joined, int* bad) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nv) return;
  bool j = false;
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int64_t d = f * nv + I, partner = (1 - f) * nv + I;
    if (isseed[d] || best[d] < 0) continue;
    if (best[d] != partner) { atomicAdd(bad, 1); continue; }
    j = j || mmsize >= 2;
  }
  joined[I] = j;
}

// 2x2 node-block inverse by Gauss-Jordan without pivoting (setup.cpp
// gauss_jordan on the block [[a00 a01] [a10 a11]]); a block split into two
// singletons (joined == 0) has its coupling entries set to 0, which gives the
// singleton inverses 1/a00, 1/a11 bit for bit
__device__ __forceinline__ double entry(const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
                                        const double* __restrict__ val, int64_t i, int64_t j) {
  const int64_t p = dfind(ptr, col, i, j);
  return p >= 0 ? val[p] : 0.0;
}

__global__ __launch_bounds__(256) void node_inverse_kernel(int64_t nv, const int64_t* __restrict__ ptr,
                                                           const int32_t* __restrict__ col,
                                                           const double* __restrict__ val,
                                                           const uint8_t* __restrict__ joined,
                                                           dv4_t* __restrict__ Dinv, int* bad) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nv) return;
  const bool jn = joined ? joined[I] != 0 : true;
  double M[2][4];
  M[0][0] = entry(ptr, col, val, I, I);
  M[0][1] = jn ? entry(ptr, col, val, I, nv + I) : 0.0;
  M[1][0] = jn ? entry(ptr, col, val, nv + I, I) : 0.0;
  M[1][1] = entry(ptr, col, val, nv + I, nv + I);
  M[0][2] = 1.0; M[0][3] = 0.0; M[1][2] = 0.0; M[1][3] = 1.0;
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const double p = M[k][k];
    if (!(p > 0.0)) ok = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) M[k][j] = M[k][j] / p;
    const int i = 1 - k;
    const double fi = M[i][k];
#pragma unroll
    for (int j = 0; j < 4; ++j) M[i][j] = M[i][j] - fi * M[k][j];
  }
  if (!ok) atomicAdd(bad, 1);
  Dinv[I] = dv4_t{M[0][2], M[0][3], M[1][2], M[1][3]};
}

// *split = 1 when some node's dofs are in different seed blocks
__global__ __launch_bounds__(256) void any_split_kernel(int64_t nv, const uint8_t* __restrict__ joined, int* split) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I < nv && !joined[I]) *split = 1;
}

// rho_B = max over dofs of sum_j |(D_B^-1 A)_ij| (SMMP order: row I's terms
// then row nv + I's; sorted-column abs sum of the nonzeros)
__global__ __launch_bounds__(64) void block_rho_kernel(int64_t nv, const int64_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ col,
                                                       const double* __restrict__ val,
                                                       const dv4_t* __restrict__ Dinv,
                                                       unsigned long long* rho_bits) {
  __shared__ RowStage S;
  const int64_t I0 = (int64_t)blockIdx.x * RS_NODES, I = I0 + threadIdx.x;
  RowView vw[2];
  stage_rows<true>(S, ptr, col, val, nv, I0, vw);
  double s = 0.0;
  if (I < nv) {
    const dv4_t D = Dinv[I];
    for (int f = 0; f < 2; ++f) {          // dof f nv + I
      const double d0 = f ? D.z : D.x, d1 = f ? D.w : D.y;
      int64_t a = ptr[I], ae = ptr[I + 1], b = ptr[nv + I], be = ptr[nv + I + 1];
      double sf = 0.0;
      while (a < ae || b < be) {
        const int64_t ja = a < ae ? vw[0].col(a) : INT64_MAX, jb = b < be ? vw[1].col(b) : INT64_MAX;
        const int64_t j = min(ja, jb);
        double v = 0.0;
        if (ja == j) { v = v + d0 * vw[0].val(a); ++a; }
        if (jb == j) { v = v + d1 * vw[1].val(b); ++b; }
        if (v != 0.0) sf += fabs(v) * 1.0;
      }
      s = fmax(s, sf);
    }
  }
  // wave max first (the sums are >= +0, so the max is exact in any order),
  // then one atomic per wave
  for (int o = 32; o > 0; o >>= 1) s = fmax(s, __shfl_xor(s, o));
  if ((threadIdx.x & 63) == 0) atomicMax(shard_of(rho_bits), (unsigned long long)__double_as_longlong(s));
}

__global__ __launch_bounds__(256) void scale_blocks_kernel(int64_t nv, double sc, const dv4_t* __restrict__ D,
                                                           dv4_t* __restrict__ W) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nv) return;
  const dv4_t d = D[I];
  W[I] = dv4_t{sc * d.x, sc * d.y, sc * d.z, sc * d.w};
}

// ---------------------------------------------------------------------------
// hash SpGEMM, C = A B, one wavefront per row (see file header)
// ---------------------------------------------------------------------------
struct BCsr {               // B given as CSR
  const int64_t* ptr;
  const int32_t* col;
  const double* val;
  __device__ __forceinline__ int64_t len(int64_t k) const { return ptr[k + 1] - ptr[k]; }
  __device__ __forceinline__ void get(int64_t k, int64_t t, int32_t* j, double* v) const {
    const int64_t q = ptr[k] + t;
    *j = col[q];
    *v = val[q];
  }
};

struct BTent {              // B = tentative prolongator: dof f nv + I -> f nagg + agg(I), 1.0
  const int64_t* agg;
  int64_t nv, nagg;
  __device__ __forceinline__ int64_t len(int64_t k) const { return agg[k % nv] >= 0 ? 1 : 0; }
  __device__ __forceinline__ void get(int64_t k, int64_t, int32_t* j, double* v) const {
    *j = (int32_t)((k / nv) * nagg + agg[k % nv]);
    *v = 1.0;
  }
};

// insert column j into a wave's table: its slot, or full = true
template <int TS>
__device__ __forceinline__ uint32_t hash_insert(int32_t* keys, int32_t j, bool* full) {
  uint32_t slot = ((uint32_t)j * 2654435761u) & (TS - 1);
  for (int probes = 0;;) {
    const int32_t cur = keys[slot];
    if (cur == j) return slot;
    if (cur == -1) {
      const int32_t old = atomicCAS(&keys[slot], -1, j);
      if (old == -1 || old == j) return slot;
    }
    slot = (slot + 1) & (TS - 1);
    if (++probes >= TS) { *full = true; return 0; }
  }
}

// one-pass staging of the count pass (spgemm_gl): a row of at most `stride`
// entries is written, rank-sorted, at row * stride (st[row] = 1) while its
// count is taken, so the fill pass only compacts it (stage_copy_kernel); a
// longer row is listed in ulist for the fill launch
struct SpStage {
  int32_t* col = nullptr;   // nullptr: no staging (two passes)
  double* val = nullptr;
  int64_t stride = 0;
  uint8_t* st = nullptr;
  int32_t* ulist = nullptr;
  int* uctr = nullptr;
};

template <int TS, int WPB, bool FILL, int GL, class BS>
__global__ __launch_bounds__(64 * WPB) void spgemm_kernel(
    int64_t nrows, const int32_t* __restrict__ rows, const int64_t* __restrict__ ub, int64_t lim,
    const int64_t* __restrict__ aptr, const int32_t* __restrict__ acol, const double* __restrict__ aval,
    BS B, int64_t* cptr, int32_t* __restrict__ ccol, double* __restrict__ cval, int* overflow,
    int32_t* spill, SpStage stg = SpStage()) {
  constexpr int NG = 64 / GL;
  __shared__ int32_t keys[WPB][TS];
  __shared__ double sums[WPB][TS];
  __shared__ int32_t ck[WPB][TS];
  __shared__ double cv[WPB][TS];
  __shared__ int cnt[WPB];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane / GL, sub = lane % GL;
  const int64_t nw = (int64_t)gridDim.x * WPB;
  for (int64_t r = (int64_t)blockIdx.x * WPB + w; r < nrows; r += nw) {
    const int64_t i = rows ? rows[r] : r;
    if (!rows && ub && ub[i] > lim) continue;    // binned to the large-table launch
    for (int s = lane; s < TS; s += 64) { keys[w][s] = -1; sums[w][s] = 0.0; }
    if (lane == 0) cnt[w] = 0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    bool full = false;
    const int64_t a1 = aptr[i + 1];
    for (int64_t kb = aptr[i]; kb < a1; kb += NG) {
      int64_t k = 0, len = 0;
      double a = 0.0;
      if (kb + g < a1) { k = acol[kb + g]; a = aval[kb + g]; len = B.len(k); }
      if (NG > 1 && !__any(len > GL)) {
        const bool act = sub < len;
        int32_t j = 0;
        double bv = 0.0;
        uint32_t slot = 0;
        if (act) {
          B.get(k, sub, &j, &bv);
          slot = hash_insert<TS>(keys[w], j, &full);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (__any(full)) break;
        for (int gg = 0; gg < NG; ++gg) {       // groups add in CSR order
          if (g == gg && act) sums[w][slot] = sums[w][slot] + a * bv;
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        continue;
      }
      for (int gg = 0; gg < NG && kb + gg < a1; ++gg) {   // one entry at a time
        const int64_t k1 = acol[kb + gg];
        const double a2 = aval[kb + gg];
        const int64_t len1 = B.len(k1);
        for (int64_t t0 = 0; t0 < len1; t0 += 64) {
          const int64_t t = t0 + lane;
          if (t < len1) {
            int32_t j;
            double bv;
            B.get(k1, t, &j, &bv);
            const uint32_t slot = hash_insert<TS>(keys[w], j, &full);
            if (!full) sums[w][slot] = sums[w][slot] + a2 * bv;
          }
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        if (__any(full)) break;
      }
      if (__any(full)) break;
    }
    if (__any(full)) {
      // table full: the row spills to the next tier's list (count pass) or
      // is skipped here because that tier fills it (fill pass); in the last
      // tier (no spill list) it is an error
      if (lane == 0) {
        if (!spill) atomicAdd(overflow + 1, 1);
        else if (!FILL) spill[atomicAdd(overflow, 1)] = (int32_t)i;
      }
      continue;
    }
    // nonzero entries (scipy drops exact zeros), appended in any order
    for (int s = lane; s < TS; s += 64) {
      if (keys[w][s] != -1 && sums[w][s] != 0.0) {
        const int q = atomicAdd(&cnt[w], 1);
        ck[w][q] = keys[w][s];
        cv[w][q] = sums[w][s];
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int m = cnt[w];
    int32_t* oc = ccol;
    double* ov = cval;
    int64_t base = 0;
    if (!FILL) {
      if (lane == 0) cptr[i + 1] = m;
      if (!stg.col) continue;
      if (m > stg.stride) {                  // too long to stage: the fill launch does it
        if (lane == 0) stg.ulist[atomicAdd(stg.uctr, 1)] = (int32_t)i;
        continue;
      }
      if (lane == 0) stg.st[i] = 1;
      oc = stg.col;
      ov = stg.val;
      base = i * stg.stride;
    } else {
      base = cptr[i];
    }
    for (int e = lane; e < m; e += 64) {     // rank sort by column
      const int32_t key = ck[w][e];
      int rank = 0;
      for (int t = 0; t < m; ++t) rank += ck[w][t] < key;
      oc[base + rank] = key;
      ov[base + rank] = cv[w][e];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------------------
// prolongator smoothing fused with the merge against T (setup.cpp
// smooth_prolongator_block + smooth_merge): row i = f nv + I of
// Y = D_B^-1 (A T) is the merge of (A T) rows I and nv + I (terms in that
// order), scaled by w, then P_i = T_i - Y_i with zeros dropped
// ---------------------------------------------------------------------------
template <bool FILL>
__global__ __launch_bounds__(256) void smooth_p_kernel(int64_t nv, const int64_t* __restrict__ tptr,
                                                       const int32_t* __restrict__ tcol,
                                                       const double* __restrict__ tval,
                                                       const dv4_t* __restrict__ Dinv, const int64_t* __restrict__ agg,
                                                       int64_t nagg, double w, int64_t* pptr,
                                                       int32_t* __restrict__ pcol, double* __restrict__ pval) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= 2 * nv) return;
  const int64_t I = i % nv, f = i / nv;
  const dv4_t D = Dinv[I];
  const double d0 = f ? D.z : D.x, d1 = f ? D.w : D.y;
  const bool ht = agg[I] >= 0;
  const int32_t tc = ht ? (int32_t)(f * nagg + agg[I]) : -1;
  bool tdone = !ht;
  int64_t o = FILL ? pptr[i] : 0;
  int64_t a = tptr[I], ae = tptr[I + 1], b = tptr[nv + I], be = tptr[nv + I + 1];
  while (a < ae || b < be) {
    const int64_t ja = a < ae ? tcol[a] : INT64_MAX, jb = b < be ? tcol[b] : INT64_MAX;
    const int64_t jj = min(ja, jb);
    double y = 0.0;
    if (ja == jj) { y = y + d0 * tval[a]; ++a; }
    if (jb == jj) { y = y + d1 * tval[b]; ++b; }
    if (y == 0.0) continue;                       // Y's exact zeros are dropped
    const int32_t j = (int32_t)jj;
    const double x = 1.0 * (w * y);
    if (!tdone && tc < j) {
      if (FILL) { pcol[o] = tc; pval[o] = 1.0; }
      ++o;
      tdone = true;
    }
    double r;
    if (x == 0.0) {
      if (!tdone && tc == j) { r = 1.0; tdone = true; } else continue;
    } else if (!tdone && tc == j) {
      r = 1.0 - x; tdone = true;
    } else {
      r = 0.0 - x;
    }
    if (r != 0.0) {
      if (FILL) { pcol[o] = j; pval[o] = r; }
      ++o;
    }
  }
  if (!tdone) {
    if (FILL) { pcol[o] = tc; pval[o] = 1.0; }
    ++o;
  }
  if (!FILL) pptr[i + 1] = o;
}

// unsmoothed aggregation: P = T
__global__ __launch_bounds__(256) void tent_kernel(int64_t n, int64_t nv, const int64_t* __restrict__ agg,
                                                   int64_t nagg, int64_t* __restrict__ pptr,
                                                   int32_t* __restrict__ pcol, double* __restrict__ pval, int pass) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t I = i % nv, f = i / nv;
  if (pass == 0) { pptr[i + 1] = agg[I] >= 0 ? 1 : 0; return; }
  if (agg[I] >= 0) { pcol[pptr[i]] = (int32_t)(f * nagg + agg[I]); pval[pptr[i]] = 1.0; }
}

// ---------------------------------------------------------------------------
// transpose helpers: row index of every entry, column counts, gather
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void entry_rows_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                         int64_t* __restrict__ idx, int64_t* __restrict__ colcnt,
                                                         const int32_t* __restrict__ col) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) {
    idx[k] = k;
    atomicAdd((unsigned long long*)&colcnt[col[k] + 1], 1ull);
  }
}

__global__ __launch_bounds__(256) void row_of_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                     int32_t* __restrict__ rowof) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) rowof[k] = (int32_t)i;
}

__global__ __launch_bounds__(256) void transpose_gather_kernel(int64_t nnz, const int64_t* __restrict__ perm,
                                                               const int32_t* __restrict__ rowof,
                                                               const double* __restrict__ val,
                                                               int32_t* __restrict__ rcol, double* __restrict__ rval) {
  const int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (d >= nnz) return;
  const int64_t k = perm[d];
  rcol[d] = rowof[k];
  rval[d] = val[k];
}

// ---------------------------------------------------------------------------
// coarsest level: dense matrix + Gauss-Jordan (setup.cpp gauss_jordan)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dense_init_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ col,
                                                         const double* __restrict__ val, double* __restrict__ M) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t w = 2 * n;
  for (int64_t j = 0; j < w; ++j) M[i * w + j] = 0.0;
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) M[i * w + col[k]] = val[k];
  M[i * w + n + i] = 1.0;
}

// pivot p = M[k][k] into f[n], multipliers f[i] = M[i][k] (f[k] = 0); rows
// i != k are untouched by the row-k scaling, so reading them first is exact
__global__ __launch_bounds__(256) void gj_col_kernel(int64_t n, int64_t k, const double* M, double* f) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) f[i] = i == k ? 0.0 : M[i * 2 * n + k];
  if (i == k) f[n] = M[k * 2 * n + k];
}

__global__ __launch_bounds__(256) void gj_scale_kernel(int64_t n, int64_t k, double* M, const double* f, int* bad) {
  const int64_t w = 2 * n;
  const double p = f[n];
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < w) {
    if (j == 0 && !(p > 0.0)) atomicAdd(bad, 1);
    M[k * w + j] = M[k * w + j] / p;
  }
}

__global__ __launch_bounds__(256) void gj_elim_kernel(int64_t n, int64_t k, double* M, const double* f) {
  const int64_t w = 2 * n;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * w) return;
  const int64_t i = t / w, j = t % w;
  if (i == k) return;
  M[i * w + j] = M[i * w + j] - f[i] * M[k * w + j];
}

__global__ __launch_bounds__(256) void gj_extract_kernel(int64_t n, const double* __restrict__ M,
                                                         double* __restrict__ inv) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * n) return;
  const int64_t i = t / n, j = t % n;
  inv[t] = M[i * 2 * n + n + j];
}

// ---------------------------------------------------------------------------
// point quantities (setup.cpp diag_of, abs_rowsum, rho_estimate, winv) and
// the point SA prolongator (smooth_prolongator + smooth_merge)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void point_diag_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ col,
                                                         const double* __restrict__ val, double* __restrict__ dg,
                                                         double* __restrict__ dinv, double* __restrict__ rs) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t p = dfind(ptr, col, i, i);
  const double d = p >= 0 ? val[p] : 0.0;
  dg[i] = d;
  dinv[i] = 1.0 / d;
  double s = 0.0;
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) s += fabs(val[k]) * 1.0;
  rs[i] = s;
}

// y_i = scale_i * sum_k a_ik x_k (sum in CSR order from 0.0; scale == nullptr: 1)
__global__ __launch_bounds__(256) void row_spmv_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ col,
                                                       const double* __restrict__ val,
                                                       const double* __restrict__ scale,
                                                       const double* __restrict__ x, double* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) s += val[k] * x[col[k]];
  y[i] = scale ? scale[i] * s : s;
}

// power-iteration start vector (setup.cpp rho_estimate / overlap_smoother)
__global__ __launch_bounds__(256) void hash_vec_kernel(int64_t n, double* __restrict__ v) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = ((double)dhash32((uint64_t)i, 977) / 4294967296.0) * 2.0 - 1.0;
}

// bits[0] = max |v_i|, bits[1] = max |w_i| (non-negative doubles order as
// their bit patterns, so the atomic max is exact in any order)
__global__ __launch_bounds__(256) void maxabs2_kernel(int64_t n, const double* __restrict__ v,
                                                      const double* __restrict__ w, unsigned long long* bits) {
  double a = 0.0, b = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    a = fmax(a, fabs(v[i]));
    b = fmax(b, fabs(w[i]));
  }
  for (int o = 32; o > 0; o >>= 1) {
    a = fmax(a, __shfl_xor(a, o));
    b = fmax(b, __shfl_xor(b, o));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(bits, (unsigned long long)__double_as_longlong(a));
    atomicMax(bits + 1, (unsigned long long)__double_as_longlong(b));
  }
}

// v = w / max|w| (the power iteration's normalisation)
__global__ __launch_bounds__(256) void vnorm_kernel(int64_t n, const double* __restrict__ w,
                                                    const unsigned long long* __restrict__ bits,
                                                    double* __restrict__ v) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = w[i] / __longlong_as_double((long long)bits[1]);
}

// max_i a_i b_i from -inf (Gershgorin bound; the products may be negative),
// one workgroup: fmax is exact and order-free for non-NaN values, and skips
// NaN as std::max(r, NaN) keeps r
__global__ __launch_bounds__(1024) void maxprod_kernel(int64_t n, const double* __restrict__ a,
                                                       const double* __restrict__ b, double* out) {
  __shared__ double red[16];
  double m = -INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += 1024) m = fmax(m, a[i] * b[i]);
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int t = 1; t < 16; ++t) m = fmax(m, red[t]);
    *out = m;
  }
}

// point smoother weights: relaxation / d, d = a_ii (JACOBI), sum |a_ij|
// (L1DIAG) or a_ii rho (JACOBI_RHO, POLY)
__global__ __launch_bounds__(256) void winv_kernel(int64_t n, int kind, double relax, double rho,
                                                   const double* __restrict__ dg, const double* __restrict__ rs,
                                                   double* __restrict__ winv) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double d = kind == 0 ? dg[i] : kind == 1 ? rs[i] : dg[i] * rho;
  winv[i] = relax / d;
}

// point SA: P_i = T_i - (w dinv_i) (A T)_i, merged as setup.cpp smooth_merge
// (T row i: column f nagg + agg(I) when aggregated)
template <bool FILL>
__global__ __launch_bounds__(256) void smooth_pt_kernel(int64_t n, int64_t nv, const int64_t* __restrict__ agg,
                                                        int64_t nagg, double w, const double* __restrict__ dinv,
                                                        const int64_t* __restrict__ aptr,
                                                        const int32_t* __restrict__ acol,
                                                        const double* __restrict__ aval, int64_t* pptr,
                                                        int32_t* __restrict__ pcol, double* __restrict__ pval) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t I = i % nv, f = i / nv;
  const bool ht = agg[I] >= 0;
  const int32_t tc = ht ? (int32_t)(f * nagg + agg[I]) : -1;
  bool tdone = !ht;
  const double ci = w * dinv[i];
  int64_t o = FILL ? pptr[i] : 0;
  for (int64_t k = aptr[i]; k < aptr[i + 1]; ++k) {
    const int32_t j = acol[k];
    const double x = ci * aval[k];
    if (!tdone && tc < j) {
      if (FILL) { pcol[o] = tc; pval[o] = 1.0; }
      ++o;
      tdone = true;
    }
    double r;
    if (x == 0.0) {
      if (!tdone && tc == j) { r = 1.0; tdone = true; } else continue;
    } else if (!tdone && tc == j) {
      r = 1.0 - x; tdone = true;
    } else {
      r = 0.0 - x;
    }
    if (r != 0.0) {
      if (FILL) { pcol[o] = j; pval[o] = r; }
      ++o;
    }
  }
  if (!tdone) {
    if (FILL) { pcol[o] = tc; pval[o] = 1.0; }
    ++o;
  }
  if (!FILL) pptr[i + 1] = o;
}

// ---------------------------------------------------------------------------
// general seed blocks (setup.cpp block_smoother / block_inverse / block_rho)
// ---------------------------------------------------------------------------
// sort key of every dof: its strongest seed, or n (no seed neighbour)
__global__ __launch_bounds__(256) void best_key_kernel(int64_t n, const int64_t* __restrict__ best,
                                                       int32_t* __restrict__ key, int64_t* __restrict__ idx) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  key[j] = best[j] >= 0 ? (int32_t)best[j] : (int32_t)n;
  idx[j] = j;
}

// joiners sorted by (seed, index): the first mmsize - 1 of each seed join it
// (setup.cpp: ascending j, cnt[s] < mmsize - 1), the others stay alone
__global__ __launch_bounds__(256) void owner_kernel(int64_t n, const int32_t* __restrict__ skey,
                                                    const int64_t* __restrict__ sidx, int mmsize,
                                                    int64_t* __restrict__ owner, uint8_t* __restrict__ isowner) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= n) return;
  const int32_t s = skey[q];
  const int64_t j = sidx[q];
  int64_t o = j;
  if (s < n) {
    int64_t lo = 0, hi = q;          // first position of key s
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (skey[mid] < s) lo = mid + 1; else hi = mid;
    }
    if (q - lo < (int64_t)mmsize - 1) o = s;
  }
  owner[j] = o;
  isowner[o] = 1;                    // benign race: every writer stores 1
}

__global__ __launch_bounds__(256) void u8_to_i64_kernel(int64_t n, const uint8_t* __restrict__ a,
                                                        int64_t* __restrict__ b) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) b[i] = a[i];
}

// block id = rank of the owner among the owners (ascending index)
__global__ __launch_bounds__(256) void bid_kernel(int64_t n, const int64_t* __restrict__ owner,
                                                  const int64_t* __restrict__ oscan, int64_t* __restrict__ bid,
                                                  int32_t* __restrict__ bkey, int64_t* __restrict__ idx,
                                                  unsigned long long* __restrict__ bcnt) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const int64_t b = oscan[owner[j]] - 1;
  bid[j] = b;
  bkey[j] = (int32_t)b;
  idx[j] = j;
  atomicAdd(bcnt + b + 1, 1ull);
}

// the blocks are node-aligned (convert.cpp node_blocks_of holds for the
// block CSR) iff every block is one dof or the two dofs of one node
__global__ __launch_bounds__(256) void align_kernel(int64_t nv, const int64_t* __restrict__ bid,
                                                    const int64_t* __restrict__ bptr,
                                                    uint8_t* __restrict__ joined, int* bad) {
  const int64_t I = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (I >= nv) return;
  const int64_t b0 = bid[I], b1 = bid[nv + I];
  const int64_t s0 = bptr[b0 + 1] - bptr[b0], s1 = bptr[b1 + 1] - bptr[b1];
  const bool j = b0 == b1;
  if (s0 > 2 || s1 > 2 || (s0 == 2 && !j) || (s1 == 2 && !j)) atomicAdd(bad, 1);
  joined[I] = j;
}

// member position inside its block, and the block CSR's row lengths
__global__ __launch_bounds__(256) void member_pos_kernel(int64_t n, const int64_t* __restrict__ mem,
                                                         const int64_t* __restrict__ bid,
                                                         const int64_t* __restrict__ bptr, int64_t* __restrict__ pos,
                                                         int64_t* __restrict__ dptr) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= n) return;
  const int64_t j = mem[q], b = bid[j];
  pos[j] = q - bptr[b];
  dptr[j + 1] = bptr[b + 1] - bptr[b];
}

// Gauss-Jordan without pivoting (setup.cpp gauss_jordan) of the s x 2s matrix
// M (row-major, [A | I]) by one workgroup of NT threads; F = s multipliers.
// Every element sees the host's operations in the host's order (row k scaled,
// then M_ij -= f_i M_kj with f read after the scaling), so the bits agree.
template <int NT>
__device__ bool block_gauss_jordan(double* M, double* F, int64_t s) {
  const int64_t w = 2 * s;
  const int tid = threadIdx.x;
  for (int64_t k = 0; k < s; ++k) {
    const double p = M[k * w + k];
    __syncthreads();
    if (!(p > 0.0)) return false;
    for (int64_t j = tid; j < w; j += NT) M[k * w + j] = M[k * w + j] / p;
    __syncthreads();
    for (int64_t i = tid; i < s; i += NT) F[i] = i == k ? 0.0 : M[i * w + k];
    __syncthreads();
    // every element, as the host does (x - f 0 can turn -0 into +0)
    for (int64_t t = tid; t < s * w; t += NT) {
      const int64_t i = t / w, j = t - i * w;
      if (i != k) M[i * w + j] = M[i * w + j] - F[i] * M[k * w + j];
    }
    __syncthreads();
  }
  return true;
}

// one-dof blocks: inverse 1 / a_ii (Gauss-Jordan on a 1 x 1 block)
__global__ __launch_bounds__(256) void blk_single_kernel(int64_t nb, const int64_t* __restrict__ bptr,
                                                         const int64_t* __restrict__ mem,
                                                         const int64_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ col,
                                                         const double* __restrict__ val,
                                                         const int64_t* __restrict__ dptr,
                                                         int32_t* __restrict__ dcol, double* __restrict__ dval,
                                                         int* bad) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nb || bptr[b + 1] - bptr[b] != 1) return;
  const int64_t i = mem[bptr[b]];
  const int64_t q = dfind(ptr, col, i, i);
  const double p = q >= 0 ? val[q] : 0.0;
  if (!(p > 0.0)) atomicAdd(bad, 1);
  dcol[dptr[i]] = (int32_t)i;
  dval[dptr[i]] = 1.0 / p;
}

__global__ __launch_bounds__(256) void multi_flag_kernel(int64_t nb, const int64_t* __restrict__ bptr,
                                                         int64_t* __restrict__ f) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b < nb) f[b] = bptr[b + 1] - bptr[b] >= 2;
}

// list of the blocks of >= 2 dofs and their Gauss-Jordan scratch (2 s^2 + s)
__global__ __launch_bounds__(256) void multi_list_kernel(int64_t nb, const int64_t* __restrict__ bptr,
                                                         const int64_t* __restrict__ fscan,
                                                         int64_t* __restrict__ list, int64_t* __restrict__ gj) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nb) return;
  const int64_t s = bptr[b + 1] - bptr[b];
  if (s < 2) return;
  const int64_t q = fscan[b] - 1;
  list[q] = b;
  gj[q] = 2 * s * s + s;
}

// blocks of >= 2 dofs, one wave each: dense block from A's rows (entries
// whose column lies in the block), Gauss-Jordan in scratch, rows of D_B^-1
__global__ __launch_bounds__(64) void blk_multi_kernel(const int64_t* __restrict__ list, int64_t nlist,
                                                       const int64_t* __restrict__ moff,
                                                       const int64_t* __restrict__ bptr,
                                                       const int64_t* __restrict__ mem,
                                                       const int64_t* __restrict__ bid,
                                                       const int64_t* __restrict__ pos,
                                                       const int64_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ col,
                                                       const double* __restrict__ val, double* scratch,
                                                       const int64_t* __restrict__ dptr, int32_t* __restrict__ dcol,
                                                       double* __restrict__ dval, int* bad) {
  const int64_t t0 = blockIdx.x;
  if (t0 >= nlist) return;
  const int64_t b = list[t0], s = bptr[b + 1] - bptr[b], w = 2 * s;
  const int64_t* m = mem + bptr[b];
  double* M = scratch + (t0 ? moff[t0 - 1] : 0);
  double* F = M + s * w;
  const int lane = threadIdx.x;
  for (int64_t t = lane; t < s * w; t += 64) M[t] = 0.0;
  __syncthreads();
  for (int64_t a = lane; a < s; a += 64) {
    const int64_t i = m[a];
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
      if (bid[col[k]] == b) M[a * w + pos[col[k]]] = val[k];
    M[a * w + s + a] = 1.0;
  }
  __syncthreads();
  if (!block_gauss_jordan<64>(M, F, s)) {
    if (lane == 0) atomicAdd(bad, 1);
    return;
  }
  for (int64_t t = lane; t < s * s; t += 64) {
    const int64_t a = t / s, c = t - a * s, i = m[a];
    dcol[dptr[i] + c] = (int32_t)m[c];
    dval[dptr[i] + c] = M[a * w + s + c];
  }
}

// max_i sum_j |C_ij| over a CSR with sorted columns and no exact zeros
__global__ __launch_bounds__(256) void rowabs_max_kernel(int64_t n, const int64_t* __restrict__ ptr,
                                                         const double* __restrict__ val, unsigned long long* bits) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  double s = 0.0;
  if (i < n)
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
      if (val[k] != 0.0) s += fabs(val[k]) * 1.0;
  for (int o = 32; o > 0; o >>= 1) s = fmax(s, __shfl_xor(s, o));
  if ((threadIdx.x & 63) == 0) atomicMax(shard_of(bits), (unsigned long long)__double_as_longlong(s));
}

__global__ __launch_bounds__(256) void scale_vals_kernel(int64_t n, double sc, double* __restrict__ v) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = sc * v[i];
}

// ---------------------------------------------------------------------------
// additive Schwarz on the seeds' overlapping rings (setup.cpp overlap_smoother)
// ---------------------------------------------------------------------------
// breadth-first ring of one seed, one wave: the visit order of the host's
// loop (neighbours in CSR order, at most mmsize dofs, depth <= maxlvl), the
// membership test spread over the lanes; then the members sorted
__global__ __launch_bounds__(64) void ring_bfs_kernel(int64_t ns, const int32_t* __restrict__ seeds,
                                                      const int64_t* __restrict__ ptr,
                                                      const int32_t* __restrict__ col, int maxlvl, int mm,
                                                      int32_t* __restrict__ blk, int64_t* __restrict__ blen) {
  extern __shared__ int32_t sh[];
  int32_t* order = sh;
  int32_t* depth = sh + mm;
  const int64_t k = blockIdx.x;
  const int lane = threadIdx.x;
  if (k >= ns) return;
  if (lane == 0) { order[0] = seeds[k]; depth[0] = 0; }
  __syncthreads();
  int size = 1, head = 0;
  while (head < size && size < mm) {
    const int32_t v = order[head];
    const int dv = depth[head];
    ++head;
    if (dv == maxlvl) continue;
    bool full = false;
    for (int64_t q = ptr[v]; q < ptr[v + 1] && !full; ++q) {
      const int32_t j = col[q];
      bool hit = false;
      for (int t = lane; t < size; t += 64) hit |= order[t] == j;
      if (__any(hit)) continue;
      if (lane == 0) { order[size] = j; depth[size] = dv + 1; }
      ++size;
      __syncthreads();
      full = size >= mm;
    }
  }
  __syncthreads();
  for (int e = lane; e < size; e += 64) {
    const int32_t key = order[e];
    int rank = 0;
    for (int t = 0; t < size; ++t) rank += order[t] < key;
    blk[k * mm + rank] = key;
  }
  if (lane == 0) blen[k] = size;
}

__global__ __launch_bounds__(256) void sq_len_kernel(int64_t ns, const int64_t* __restrict__ blen,
                                                     int64_t* __restrict__ sq, int64_t* __restrict__ gj) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= ns) return;
  const int64_t m = blen[k];
  sq[k] = m * m;
  gj[k] = 2 * m * m + m;
}

// dense ring block from A (binary searches), one workgroup of 256 threads
// (blocks of up to Schwarz_mmsize 200 dofs), its inverse into inv (row-major
// at the block's contribution offset), and the covered flags
__global__ __launch_bounds__(256) void ring_inv_kernel(int64_t ns, int mm, const int32_t* __restrict__ blk,
                                                      const int64_t* __restrict__ blen,
                                                      const int64_t* __restrict__ sqscan,
                                                      const int64_t* __restrict__ gjscan,
                                                      const int64_t* __restrict__ ptr,
                                                      const int32_t* __restrict__ col,
                                                      const double* __restrict__ val, double* scratch,
                                                      double* __restrict__ inv, uint8_t* __restrict__ cov, int* bad) {
  const int64_t k = blockIdx.x;
  if (k >= ns) return;
  const int64_t s = blen[k], w = 2 * s;
  const int32_t* b = blk + k * mm;
  double* M = scratch + (k ? gjscan[k - 1] : 0);
  double* F = M + s * w;
  double* out = inv + (k ? sqscan[k - 1] : 0);
  const int tid = threadIdx.x;
  for (int64_t t = tid; t < s * w; t += 256) {
    const int64_t a = t / w, c = t - a * w;
    double x = 0.0;
    if (c < s) {
      const int64_t q = dfind(ptr, col, b[a], b[c]);
      if (q >= 0) x = val[q];
    } else if (c - s == a) {
      x = 1.0;
    }
    M[t] = x;
  }
  for (int64_t a = tid; a < s; a += 256) cov[b[a]] = 1;
  __syncthreads();
  if (!block_gauss_jordan<256>(M, F, s)) {
    if (tid == 0) atomicAdd(bad, 1);
    return;
  }
  for (int64_t t = tid; t < s * s; t += 256) {
    const int64_t a = t / s, c = t - a * s;
    out[t] = M[a * w + s + c];
  }
}

// (row, column) keys of every block contribution, in block order, then one
// diagonal key per uncovered dof (source -1 - i: 1 / a_ii)
__global__ __launch_bounds__(64) void ring_keys_kernel(int64_t ns, int mm, int64_t n, const int32_t* __restrict__ blk,
                                                       const int64_t* __restrict__ blen,
                                                       const int64_t* __restrict__ sqscan, uint64_t* __restrict__ key,
                                                       int64_t* __restrict__ src) {
  const int64_t k = blockIdx.x;
  if (k >= ns) return;
  const int64_t s = blen[k], o = k ? sqscan[k - 1] : 0;
  const int32_t* b = blk + k * mm;
  for (int64_t t = threadIdx.x; t < s * s; t += 64) {
    const int64_t a = t / s, c = t - a * s;
    key[o + t] = (uint64_t)b[a] * (uint64_t)n + (uint64_t)b[c];
    src[o + t] = o + t;
  }
}

__global__ __launch_bounds__(256) void uncov_keys_kernel(int64_t n, const uint8_t* __restrict__ cov,
                                                         const int64_t* __restrict__ uscan, int64_t base,
                                                         uint64_t* __restrict__ key, int64_t* __restrict__ src) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n || cov[i]) return;
  const int64_t q = base + uscan[i] - 1;
  key[q] = (uint64_t)i * (uint64_t)n + (uint64_t)i;
  src[q] = -1 - i;
}

__global__ __launch_bounds__(256) void uncov_flag_kernel(int64_t n, const uint8_t* __restrict__ cov,
                                                         int64_t* __restrict__ f) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) f[i] = cov[i] ? 0 : 1;
}

__global__ __launch_bounds__(256) void run_flag_kernel(int64_t e, const uint64_t* __restrict__ key,
                                                       int64_t* __restrict__ f) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < e) f[t] = (t == 0 || key[t] != key[t - 1]) ? 1 : 0;
}

// run starts, column indices and row counts of the merged pattern
__global__ __launch_bounds__(256) void run_start_kernel(int64_t e, int64_t n, const uint64_t* __restrict__ key,
                                                        const int64_t* __restrict__ fscan,
                                                        int64_t* __restrict__ ustart, int32_t* __restrict__ wcol,
                                                        unsigned long long* __restrict__ wcnt) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= e || !(t == 0 || key[t] != key[t - 1])) return;
  const int64_t u = fscan[t] - 1;
  ustart[u] = t;
  wcol[u] = (int32_t)(key[t] % (uint64_t)n);
  atomicAdd(wcnt + key[t] / (uint64_t)n + 1, 1ull);
}

// each merged entry sums its run in block order from 0.0 (setup.cpp: W_ij +=
// inv in seed order), or is 1 / a_ii for an uncovered dof
__global__ __launch_bounds__(256) void run_sum_kernel(int64_t nu, int64_t e, const int64_t* __restrict__ ustart,
                                                      const int64_t* __restrict__ src, const double* __restrict__ inv,
                                                      const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
                                                      const double* __restrict__ val, double* __restrict__ wval) {
  const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (u >= nu) return;
  const int64_t t1 = u + 1 < nu ? ustart[u + 1] : e;
  double s = 0.0;
  for (int64_t t = ustart[u]; t < t1; ++t) {
    const int64_t q = src[t];
    if (q >= 0) {
      s += inv[q];
    } else {
      const int64_t i = -1 - q, p = dfind(ptr, col, i, i);
      s = 1.0 / (p >= 0 ? val[p] : 0.0);
    }
  }
  wval[u] = s;
}

// 2x2 node blocks as the host's block CSR (ghier_download's rule: rows
// {I, nv + I}, or the diagonal alone where seed blocks split the node)
__global__ __launch_bounds__(256) void node_wb_kernel(int64_t nv, const dv4_t* __restrict__ W,
                                                      const uint8_t* __restrict__ joined, int64_t* __restrict__ ptr,
                                                      int32_t* __restrict__ col, double* __restrict__ val, int fill) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= 2 * nv) return;
  const int64_t I = i % nv, f = i / nv;
  const bool jn = joined ? joined[I] != 0 : true;
  if (!fill) { ptr[i + 1] = jn ? 2 : 1; return; }
  const dv4_t w = W[I];
  const int64_t o = ptr[i];
  if (jn) {
    col[o] = (int32_t)I; val[o] = f ? w.z : w.x;
    col[o + 1] = (int32_t)(nv + I); val[o + 1] = f ? w.w : w.y;
  } else {
    col[o] = (int32_t)i; val[o] = f ? w.w : w.x;
  }
}

// input check (setup.cpp host_setup): monotone row pointers, columns in
// range and strictly increasing within each row; eight lanes per row (a
// wave reads its rows' columns contiguously), one flag per failing wave
__global__ __launch_bounds__(256) void validate_kernel(int64_t n, int64_t m, const int64_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ col, int* bad) {
  const int lane = threadIdx.x & 7;
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 3;
  int nb = 0;
  if (i < n) {
    const int64_t a = ptr[i], b = ptr[i + 1];
    nb = b < a;
    for (int64_t k = a + lane; k < b && !nb; k += 8) {
      const int32_t c = col[k];
      nb |= (c < 0 || c >= m || (k > a && c <= col[k - 1]));
    }
  }
  if (__any(nb) && (threadIdx.x & 63) == 0) atomicAdd(bad, 1);
}

// ---------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------
struct Clock {
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  double lap() {
    const auto t = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(t - t0).count();
    t0 = t;
    return ms;
  }
};

int read_int(const int* d, int* h, std::string* err) { return to_host(h, d, 1, err); }

// a sharded counter (shard_of): allocate / zero, then read its sum or max
int shards_alloc(Scratch* S, unsigned long long** c, std::string* err) {
  RCHK(S->alloc(c, CSH * CSTR, err));
  HIPCHK(dev_memset(*c, 0, CSH * CSTR * sizeof(unsigned long long)));
  return MAMG_OK;
}
int shards_zero(unsigned long long* c) {
  return dev_memset(c, 0, CSH * CSTR * sizeof(unsigned long long)) == hipSuccess ? MAMG_OK : MAMG_ERR_HIP;
}
int shards_read(const unsigned long long* c, bool max, unsigned long long* out, std::string* err) {
  unsigned long long h[CSH * CSTR];
  RCHK(to_host(h, c, CSH * CSTR, err));
  unsigned long long r = 0;
  for (int k = 0; k < CSH; ++k) r = max ? std::max(r, h[k * CSTR]) : r + h[k * CSTR];
  *out = r;
  return MAMG_OK;
}

// The count + staging pass over row pairs (i, i + h) of a field-major
// 2-function matrix (round 5): when the two rows hold the same columns (the
// 2 x 2 node blocks of A_l, and of R = P^T), the wave loads each B row once
// for both, inserts its columns once, and accumulates two sums per slot.
// Each sum takes exactly its scalar row's terms in the same order (the same
// batches, the same group-serialised adds), the table holds the same keys
// (so the same tier), and each row is extracted and staged as alone: the
// bits of spgemm_kernel row by row.  Pairs whose columns differ are listed
// (mism) for spgemm_kernel; a full table spills both rows.
template <int TS, int WPB, int GL, class BS>
__global__ __launch_bounds__(64 * WPB) void spgemm_pair_kernel(
    int64_t h, const int64_t* __restrict__ aptr, const int32_t* __restrict__ acol, const double* __restrict__ aval,
    BS B, int64_t* cptr, int* overflow, int32_t* spill, SpStage stg, int32_t* mism, int* nmism) {
  constexpr int NG = 64 / GL;
  __shared__ int32_t keys[WPB][TS];
  __shared__ double sums[WPB][2][TS];
  __shared__ int32_t ck[WPB][TS];
  __shared__ double cv[WPB][TS];
  __shared__ int cnt[WPB];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane / GL, sub = lane % GL;
  const int64_t nw = (int64_t)gridDim.x * WPB;
  for (int64_t pr = (int64_t)blockIdx.x * WPB + w; pr < h; pr += nw) {
    const int64_t i0 = pr, i1 = pr + h;
    const int64_t p0 = aptr[i0], p1 = aptr[i1], L = aptr[i0 + 1] - p0;
    bool diff = aptr[i1 + 1] - p1 != L;
    if (!diff) {
      bool d = false;
      for (int64_t t = lane; t < L; t += 64) d |= acol[p0 + t] != acol[p1 + t];
      diff = __any(d);
    }
    if (diff) {
      if (lane == 0) {
        const int q = atomicAdd(nmism, 2);
        mism[q] = (int32_t)i0;
        mism[q + 1] = (int32_t)i1;
      }
      continue;
    }
    for (int s = lane; s < TS; s += 64) { keys[w][s] = -1; sums[w][0][s] = 0.0; sums[w][1][s] = 0.0; }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    bool full = false;
    for (int64_t kb = 0; kb < L; kb += NG) {
      int64_t k = 0, len = 0;
      double a0 = 0.0, a1 = 0.0;
      if (kb + g < L) { k = acol[p0 + kb + g]; a0 = aval[p0 + kb + g]; a1 = aval[p1 + kb + g]; len = B.len(k); }
      if (NG > 1 && !__any(len > GL)) {
        const bool act = sub < len;
        int32_t j = 0;
        double bv = 0.0;
        uint32_t slot = 0;
        if (act) {
          B.get(k, sub, &j, &bv);
          slot = hash_insert<TS>(keys[w], j, &full);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (__any(full)) break;
        for (int gg = 0; gg < NG; ++gg) {       // groups add in CSR order
          if (g == gg && act) {
            sums[w][0][slot] = sums[w][0][slot] + a0 * bv;
            sums[w][1][slot] = sums[w][1][slot] + a1 * bv;
          }
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        continue;
      }
      for (int gg = 0; gg < NG && kb + gg < L; ++gg) {   // one entry at a time
        const int64_t k1 = acol[p0 + kb + gg];
        const double x0 = aval[p0 + kb + gg], x1 = aval[p1 + kb + gg];
        const int64_t len1 = B.len(k1);
        for (int64_t t0 = 0; t0 < len1; t0 += 64) {
          const int64_t t = t0 + lane;
          if (t < len1) {
            int32_t j;
            double bv;
            B.get(k1, t, &j, &bv);
            const uint32_t slot = hash_insert<TS>(keys[w], j, &full);
            if (!full) {
              sums[w][0][slot] = sums[w][0][slot] + x0 * bv;
              sums[w][1][slot] = sums[w][1][slot] + x1 * bv;
            }
          }
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        if (__any(full)) break;
      }
      if (__any(full)) break;
    }
    if (__any(full)) {   // both rows to the next tier
      if (lane == 0) {
        const int q = atomicAdd(overflow, 2);
        spill[q] = (int32_t)i0;
        spill[q + 1] = (int32_t)i1;
      }
      continue;
    }
    for (int r = 0; r < 2; ++r) {
      const int64_t i = r ? i1 : i0;
      if (lane == 0) cnt[w] = 0;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      for (int s = lane; s < TS; s += 64) {   // nonzero entries (scipy drops exact zeros)
        if (keys[w][s] != -1 && sums[w][r][s] != 0.0) {
          const int q = atomicAdd(&cnt[w], 1);
          ck[w][q] = keys[w][s];
          cv[w][q] = sums[w][r][s];
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      const int m = cnt[w];
      if (lane == 0) cptr[i + 1] = m;
      if (m > stg.stride) {
        if (lane == 0) stg.ulist[atomicAdd(stg.uctr, 1)] = (int32_t)i;
      } else {
        if (lane == 0) stg.st[i] = 1;
        const int64_t base = i * stg.stride;
        for (int e = lane; e < m; e += 64) {     // rank sort by column
          const int32_t key = ck[w][e];
          int rank = 0;
          for (int t = 0; t < m; ++t) rank += ck[w][t] < key;
          stg.col[base + rank] = key;
          stg.val[base + rank] = cv[w][e];
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
  }
}

// *diff += pairs (i, i + h) whose rows hold different columns (a pair kernel
// would hand every such pair to the row kernel: for UA's R = T^T all of
// them, since row J holds field-0 columns and row nc + J field-1 columns)
// (a sample: every PAIR_SAMPLE-th pair; the decision needs a fraction, and the
// full check, one lane walking both rows, cost 3 ms per level-0 product)
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
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(shard_of(diff), (unsigned long long)__popcll(b));
}

// staged rows into place: row i's m = ptr[i + 1] - ptr[i] entries from
// scol / sval at i * S (S lanes per row)
template <int S>
__global__ __launch_bounds__(256) void stage_copy_kernel(int64_t n, const uint8_t* __restrict__ st,
                                                         const int32_t* __restrict__ scol,
                                                         const double* __restrict__ sval,
                                                         const int64_t* __restrict__ ptr, int32_t* __restrict__ col,
                                                         double* __restrict__ val) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t i = t / S;
  const int e = (int)(t % S);
  if (i >= n || !st[i]) return;
  const int64_t p0 = ptr[i];
  if (e < ptr[i + 1] - p0) {
    col[p0 + e] = scol[i * S + e];
    val[p0 + e] = sval[i * S + e];
  }
}

// exact output size + row pointers + entries of C = A B (hash SpGEMM).
// Optimistic tiering: every row first runs in a 128-slot table (4 waves per
// block, 12 KB of LDS, so LDS no longer caps the waves per CU); a row whose
// distinct columns overflow it spills to a list that the 512-slot launch
// redoes, whose overflow the 2048-slot launch (1 wave per block) redoes.  A
// row's tier depends only on its distinct-column count, so the count and fill
// passes agree.  Each slot accumulates its products in A-row order whatever
// the table size, so every tier gives the same bits.  (Binning by the
// product-count upper bound sent most Galerkin rows, whose product counts far
// exceed their distinct counts, to the slow large-table launch.)
// One pass for most rows (round 5): the tier-0 count pass also writes each
// row of at most `stride` entries into a staging area (SpStage), and the fill
// pass compacts those instead of recomputing them; the rows above `stride`
// (ulist) and the spilled tiers keep the count + fill passes.  The staging
// area is n * stride entries, stride the largest of 128 / 64 / 32 / 16 within
// MAMG_SPGEMM_STAGE_GB (default 16; 0: two passes everywhere) and a quarter
// of the free HBM (MAMG_SPGEMM_STAGE_STRIDE caps it: tests of the long-row
// list).  Same kernel code, same rank sort: the same bits.
// MAMG_SPGEMM_PAIR=0: the staged count pass row by row (A/B, tests)
bool spgemm_pair_on() {
  const char* e = opt("MAMG_SPGEMM_PAIR");
  return e ? std::atoi(e) != 0 : true;
}

// The staging area is the per-device staging block of dmem.h (StageLease),
// at most min(MAMG_SPGEMM_STAGE_GB, a quarter of the free HBM), kept for the
// process until the setup cache is released; used in null-stream order, as
// the setup temporaries are, and held by one product at a time.
size_t stage_cap_bytes() {
  const char* e = opt("MAMG_SPGEMM_STAGE_GB");
  const double cap_gb = e ? std::atof(e) : 16.0;
  return cap_gb > 0.0 ? (size_t)(cap_gb * 1e9) : 0;
}

int64_t spgemm_stage_stride(int64_t n, size_t pool) {
  const char* e = opt("MAMG_SPGEMM_STAGE_GB");
  if (e && std::atof(e) <= 0.0) return 0;
  e = opt("MAMG_SPGEMM_STAGE_STRIDE");
  const int64_t smax = e ? std::atoll(e) : 128;
  if (n <= 0) return 0;
  for (int64_t s : {128, 64, 32, 16})
    if (s <= smax && (double)n * (double)s * 12.0 <= (double)pool) return s;
  return 0;
}

// pair: A is a field-major 2-function matrix (rows i, i + n / 2 of node i):
// the staged count pass runs over row pairs (spgemm_pair_kernel)
template <int GL, class BS>
int spgemm_gl(GHier* G, const DevMat& A, BS B, int64_t ncols, DevMat* C, std::string* err, bool pair) {
#if MAMG_DIAG
  // MAMG_SPGEMM_TRACE (diagnosis build): one line per product on stderr
  const bool trace = std::getenv("MAMG_SPGEMM_TRACE") != nullptr;
  if (trace) (void)hipDeviceSynchronize();
  const auto tr0 = std::chrono::steady_clock::now();
#endif
  constexpr int TS0 = 128, TS1 = 512, TS2 = 2048;
  const int64_t n = A.n;
  Scratch S;
  int32_t *l1 = nullptr, *l2 = nullptr;
  int* ctr = nullptr;   // [0] rows spilled by tier 0, [1] tier-2 overflow, [2] rows spilled by tier 1, [3] fill
  RCHK(S.alloc(&l1, n, err));
  RCHK(S.alloc(&l2, n, err));
  RCHK(S.alloc(&ctr, 5, err));
  HIPCHK(dev_memset(ctr, 0, 5 * sizeof(int)));
  SpStage stg;
  StageLease lease(stage_cap_bytes());     // held until the product returns
  void* pool = lease.p;
  stg.stride = pool ? spgemm_stage_stride(n, lease.bytes) : 0;
  int32_t* l3 = nullptr;
  int n3 = 0;
  if (stg.stride) {   // values first (8-byte aligned), then the columns
    stg.val = reinterpret_cast<double*>(pool);
    stg.col = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(pool) + (size_t)n * stg.stride * sizeof(double));
    RCHK(S.alloc(&stg.st, n, err));
    RCHK(S.alloc(&l3, n, err));
    HIPCHK(dev_memset(stg.st, 0, (size_t)n));
    stg.ulist = l3;
    stg.uctr = ctr + 4;
  }
#if MAMG_DIAG
  const auto tr1 = std::chrono::steady_clock::now();   // after the staging allocations
#endif
  C->n = n;
  C->m = ncols;
  RCHK(galloc(G, &C->ptr, n + 1, err));
  HIPCHK(dev_memset(C->ptr, 0, (n + 1) * sizeof(int64_t)));
  const unsigned g0 = (unsigned)std::min<int64_t>(std::max<int64_t>(1, (n + 3) / 4), 65536);
  int n1 = 0, n2 = 0;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1) {
      RCHK(dscan_incl_i64(C->ptr, C->ptr, n + 1, nullptr, err));
      RCHK(to_host(&C->nnz, C->ptr + n, 1, err));
      RCHK(galloc(G, &C->col, C->nnz, err));
      RCHK(galloc(G, &C->val, C->nnz, err));
    }
    int64_t* cp = C->ptr;
    int32_t* cc = pass ? C->col : nullptr;
    double* cv = pass ? C->val : nullptr;
    if (pass == 0) {
      if (pair && stg.stride && n % 2 == 0 && spgemm_pair_on()) {   // only when most pairs agree
        unsigned long long* dc = nullptr;
        RCHK(shards_alloc(&S, &dc, err));
        const int64_t ns = (n / 2 + PAIR_SAMPLE - 1) / PAIR_SAMPLE;   // pairs sampled
        pair_diff_kernel<<<nblk(ns), 256>>>(n / 2, A.ptr, A.col, dc);
        HIPCHK(hipGetLastError());
        unsigned long long nd = 0;
        RCHK(shards_read(dc, false, &nd, err));
        pair = nd * 8 <= (unsigned long long)ns;
      }
      if (pair && stg.stride && n % 2 == 0 && spgemm_pair_on()) {
        int32_t* lm = nullptr;
        int* nm = nullptr;
        RCHK(S.alloc(&lm, n, err));
        RCHK(S.alloc(&nm, 1, err));
        HIPCHK(dev_memset(nm, 0, sizeof(int)));
        const unsigned gp = (unsigned)std::min<int64_t>(std::max<int64_t>(1, (n / 2 + 3) / 4), 65536);
        spgemm_pair_kernel<TS0, 4, GL><<<gp, 256>>>(n / 2, A.ptr, A.col, A.val, B, cp, ctr, l1, stg, lm, nm);
        HIPCHK(hipGetLastError());
        int hm = 0;
        RCHK(read_int(nm, &hm, err));
        if (hm)   // pairs with different columns: row by row
          spgemm_kernel<TS0, 4, false, GL><<<(unsigned)std::min<int64_t>((hm + 3) / 4, 65536), 256>>>(
              hm, lm, nullptr, 0, A.ptr, A.col, A.val, B, cp, cc, cv, ctr, l1, stg);
      } else {
        spgemm_kernel<TS0, 4, false, GL><<<g0, 256>>>(n, nullptr, nullptr, 0, A.ptr, A.col, A.val, B, cp, cc, cv,
                                                  ctr, l1, stg);
      }
      HIPCHK(hipGetLastError());
      RCHK(read_int(ctr, &n1, err));
      if (stg.stride) RCHK(read_int(ctr + 4, &n3, err));
      if (n1) {
        const unsigned g1 = (unsigned)std::min<int64_t>((n1 + 3) / 4, 65536);
        spgemm_kernel<TS1, 4, false, GL><<<g1, 256>>>(n1, l1, nullptr, 0, A.ptr, A.col, A.val, B, cp, cc, cv,
                                                  ctr + 2, l2);
        HIPCHK(hipGetLastError());
        RCHK(read_int(ctr + 2, &n2, err));
      }
      if (n2)
        spgemm_kernel<TS2, 1, false, GL><<<(unsigned)std::min<int64_t>(n2, 65536), 64>>>(
            n2, l2, nullptr, 0, A.ptr, A.col, A.val, B, cp, cc, cv, ctr, nullptr);
    } else {
      if (!stg.stride) {
        spgemm_kernel<TS0, 4, true, GL><<<g0, 256>>>(n, nullptr, nullptr, 0, A.ptr, A.col, A.val, B, cp, cc, cv,
                                                 ctr + 3, l1);
      } else {
        const unsigned gs = (unsigned)((n * stg.stride + 255) / 256);
        switch (stg.stride) {
          case 128: stage_copy_kernel<128><<<gs, 256>>>(n, stg.st, stg.col, stg.val, cp, cc, cv); break;
          case 64: stage_copy_kernel<64><<<gs, 256>>>(n, stg.st, stg.col, stg.val, cp, cc, cv); break;
          case 32: stage_copy_kernel<32><<<gs, 256>>>(n, stg.st, stg.col, stg.val, cp, cc, cv); break;
          default: stage_copy_kernel<16><<<gs, 256>>>(n, stg.st, stg.col, stg.val, cp, cc, cv); break;
        }
        if (n3)   // tier-0 rows longer than the stride
          spgemm_kernel<TS0, 4, true, GL><<<(unsigned)std::min<int64_t>((n3 + 3) / 4, 65536), 256>>>(
              n3, l3, nullptr, 0, A.ptr, A.col, A.val, B, cp, cc, cv, ctr + 3, l1);
      }
      if (n1)
        spgemm_kernel<TS1, 4, true, GL><<<(unsigned)std::min<int64_t>((n1 + 3) / 4, 65536), 256>>>(
            n1, l1, nullptr, 0, A.ptr, A.col, A.val, B, cp, cc, cv, ctr + 3, l2);
      if (n2)
        spgemm_kernel<TS2, 1, true, GL><<<(unsigned)std::min<int64_t>(n2, 65536), 64>>>(
            n2, l2, nullptr, 0, A.ptr, A.col, A.val, B, cp, cc, cv, ctr, nullptr);
    }
    HIPCHK(hipGetLastError());
    int ovf = 0;
    RCHK(read_int(ctr + 1, &ovf, err));
    if (ovf) {
      *err = "GPU SpGEMM: " + std::to_string(ovf) + " row(s) with more than 2048 distinct columns "
             "(use the host setup, mamg_setup)";
      return MAMG_ERR_UNSUPPORTED;
    }
  }
#if MAMG_DIAG
  if (trace) {
    (void)hipDeviceSynchronize();
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    const auto tr2 = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[mamg spgemm] n %lld nnz %lld stride %lld pair %d: allocations %.2f ms, products %.2f ms, free %.1f GB\n",
                 (long long)n, (long long)C->nnz, (long long)stg.stride, (int)pair,
                 std::chrono::duration<double, std::milli>(tr1 - tr0).count(),
                 std::chrono::duration<double, std::milli>(tr2 - tr1).count(), fr / 1e9);
  }
#endif
  return MAMG_OK;
}

// lane-group width from B's mean row length (most B rows fit one group)
template <class BS>
int spgemm(GHier* G, const DevMat& A, BS B, int64_t ncols, DevMat* C, std::string* err, double blen,
           bool pair = false) {
  if (blen <= 1.5) return spgemm_gl<2>(G, A, B, ncols, C, err, pair);
  if (blen <= 5.0) return spgemm_gl<8>(G, A, B, ncols, C, err, pair);
  if (blen <= 11.0) return spgemm_gl<16>(G, A, B, ncols, C, err, pair);
  return spgemm_gl<32>(G, A, B, ncols, C, err, pair);
}

// R = P^T (setup.cpp transpose: counting order == stable sort by column)
int transpose(GHier* G, const DevMat& P, DevMat* R, std::string* err) {
  Scratch S;
  const int64_t nnz = P.nnz;
  R->n = P.m;
  R->m = P.n;
  R->nnz = nnz;
  RCHK(galloc(G, &R->ptr, P.m + 1, err));
  RCHK(galloc(G, &R->col, nnz, err));
  RCHK(galloc(G, &R->val, nnz, err));
  HIPCHK(dev_memset(R->ptr, 0, (P.m + 1) * sizeof(int64_t)));
  int64_t *idx = nullptr, *perm = nullptr;
  int32_t *keys = nullptr, *rowof = nullptr;
  RCHK(S.alloc(&idx, nnz, err));
  RCHK(S.alloc(&perm, nnz, err));
  RCHK(S.alloc(&keys, nnz, err));
  RCHK(S.alloc(&rowof, nnz, err));
  entry_rows_kernel<<<nblk(P.n), 256>>>(P.n, P.ptr, idx, R->ptr, P.col);
  row_of_kernel<<<nblk(P.n), 256>>>(P.n, P.ptr, rowof);
  HIPCHK(hipGetLastError());
  RCHK(dscan_incl_i64(R->ptr, R->ptr, P.m + 1, nullptr, err));
  int bits = 1;
  while ((int64_t(1) << bits) < P.m && bits < 32) ++bits;
  RCHK(dsort_pairs_i32_i64(P.col, keys, idx, perm, nnz, bits, nullptr, err));
  if (debug_ptrs()) {   // diagnosis build: the gather below indexes with perm
    for (const void* q : {(const void*)perm, (const void*)rowof, (const void*)P.val, (const void*)R->col,
                          (const void*)R->val})
      check_block(q, 1, "transpose operand");
    std::vector<int64_t> hp(nnz);
    RCHK(to_host(hp.data(), perm, nnz, err));
    std::vector<char> seen(nnz, 0);
    for (int64_t d = 0; d < nnz; ++d) {
      if (hp[d] < 0 || hp[d] >= nnz || seen[hp[d]]) {
        *err = "debug: the transpose's sort permutation is not a permutation (entry " + std::to_string(d) + " = " +
               std::to_string(hp[d]) + ")";
        return MAMG_ERR_SETUP;
      }
      seen[hp[d]] = 1;
    }
  }
  transpose_gather_kernel<<<nblk(nnz), 256>>>(nnz, perm, rowof, P.val, R->col, R->val);
  HIPCHK(hipGetLastError());
  return MAMG_OK;
}

// W = (relax / rho_B) D_B^-1 and rho_B for node blocks D
int block_rho(const DevMat& A, int64_t nv, const dv4_t* D, double* rho, std::string* err) {
  Scratch S;
  unsigned long long* rb = nullptr;
  RCHK(shards_alloc(&S, &rb, err));
  block_rho_kernel<<<(unsigned)((nv + RS_NODES - 1) / RS_NODES), RS_NODES>>>(nv, A.ptr, A.col, A.val, D, rb);
  HIPCHK(hipGetLastError());
  unsigned long long h = 0;
  RCHK(shards_read(rb, true, &h, err));
  std::memcpy(rho, &h, sizeof(double));
  return MAMG_OK;
}

int node_inverse(const DevMat& A, int64_t nv, const uint8_t* joined, dv4_t* D, const char* what,
                 std::string* err) {
  Scratch S;
  int* bad = nullptr;
  RCHK(S.alloc(&bad, 1, err));
  HIPCHK(dev_memset(bad, 0, sizeof(int)));
  node_inverse_kernel<<<nblk(nv), 256>>>(nv, A.ptr, A.col, A.val, joined, D, bad);
  HIPCHK(hipGetLastError());
  int hb = 0;
  RCHK(read_int(bad, &hb, err));
  if (hb) { *err = std::string(what) + " block not SPD (non-positive pivot)"; return MAMG_ERR_SETUP; }
  return MAMG_OK;
}

// compacted weighted graph of M (flagged, off-diagonal, non-zero entries)
int wgraph(const DevMat& M, const uint8_t* flag, int absval, Scratch* S, DevMat* W, std::string* err) {
  const int64_t n = M.n;
  W->n = W->m = n;
  RCHK(S->alloc(&W->ptr, n + 1, err));
  HIPCHK(dev_memset(W->ptr, 0, sizeof(int64_t)));
  wgraph_kernel<false><<<nblk(n), 256>>>(n, M.ptr, M.col, M.val, flag, absval, W->ptr, nullptr, nullptr);
  HIPCHK(hipGetLastError());
  RCHK(dscan_incl_i64(W->ptr, W->ptr, n + 1, nullptr, err));
  RCHK(to_host(&W->nnz, W->ptr + n, 1, err));
  RCHK(S->alloc(&W->col, W->nnz, err));
  RCHK(S->alloc(&W->val, W->nnz, err));
  wgraph_kernel<true><<<nblk(n), 256>>>(n, M.ptr, M.col, M.val, flag, absval, W->ptr, W->col, W->val);
  HIPCHK(hipGetLastError());
  return MAMG_OK;
}

// parallel heavy-edge matching on the strong node graph (setup.cpp
// aggregate_hem): HEM passes of handshake rounds; pass k + 1 on T^T W T
int aggregate_hem_dev(GHier* G, const DevMat& Gr, const uint8_t* flag, int level, int64_t** agg_out,
                      int64_t* nagg_out, std::string* err) {
  constexpr int PASSES = 2, MAX_ROUNDS = 64;
  Scratch S;
  const int64_t n = Gr.n;
  DevMat W;
  RCHK(wgraph(Gr, flag, 1, &S, &W, err));
  const DevMat W1 = W;   // pass-1 graph (Scratch-owned until return)
  uint8_t* act = nullptr;
  RCHK(S.alloc(&act, n, err));
  {   // active = any strong neighbour
    int64_t* cnt = nullptr;
    RCHK(S.alloc(&cnt, n + 1, err));
    HIPCHK(dev_memset(cnt, 0, sizeof(int64_t)));
    wgraph_kernel<false><<<nblk(n), 256>>>(n, Gr.ptr, Gr.col, Gr.val, flag, 2, cnt, nullptr, nullptr);
    nonzero_flag_kernel<<<nblk(n), 256>>>(n, cnt, act);
    HIPCHK(hipGetLastError());
  }
  int64_t* agg = nullptr;
  RCHK(galloc(G, &agg, n, err));
  iota_nonisol_kernel<<<nblk(n), 256>>>(n, act, agg);
  int64_t nagg = n;
  unsigned long long* got = nullptr;
  RCHK(shards_alloc(&S, &got, err));
  for (int ps = 0; ps < PASSES; ++ps) {
    const int64_t m = W.n;
    int64_t *mate = nullptr, *choice = nullptr, *f = nullptr, *a = nullptr;
    RCHK(S.alloc(&mate, m, err));
    RCHK(S.alloc(&choice, m, err));
    RCHK(S.alloc(&f, m, err));
    RCHK(S.alloc(&a, m, err));
    HIPCHK(dev_memset(mate, 0xff, m * sizeof(int64_t)));
    for (int round = 0; round < MAX_ROUNDS; ++round) {
      RCHK(shards_zero(got));
      hem_pick_kernel<<<nblk(m), 256>>>(m, W.ptr, W.col, W.val, act, mate, 16 * level + ps, choice);
      hem_mutual_kernel<<<nblk(m), 256>>>(m, choice, mate, got);
      HIPCHK(hipGetLastError());
      unsigned long long hg = 0;
      RCHK(shards_read(got, false, &hg, err));
      if (!hg) break;
    }
    hem_root_kernel<<<nblk(m), 256>>>(m, act, mate, f);
    RCHK(dscan_incl_i64(f, f, m, nullptr, err));
    RCHK(to_host(&nagg, f + m - 1, 1, err));
    hem_number_kernel<<<nblk(m), 256>>>(m, act, mate, f, a);
    hem_compose_kernel<<<nblk(n), 256>>>(n, a, agg);
    HIPCHK(hipGetLastError());
    if (nagg == 0) {   // no strong edge on this level (theta > 0): no aggregates, every agg[i] = -1
      *agg_out = agg;
      *nagg_out = 0;
      return MAMG_OK;
    }
    if (ps + 1 == PASSES) break;
    DevMat T, Tt, WT, C;   // W_next = T^T W T without its diagonal
    T.n = m; T.m = nagg;
    RCHK(S.alloc(&T.ptr, m + 1, err));
    HIPCHK(dev_memset(T.ptr, 0, sizeof(int64_t)));
    hem_t_kernel<<<nblk(m), 256>>>(m, act, a, T.ptr, nullptr, nullptr, 0);
    RCHK(dscan_incl_i64(T.ptr, T.ptr, m + 1, nullptr, err));
    RCHK(to_host(&T.nnz, T.ptr + m, 1, err));
    RCHK(S.alloc(&T.col, T.nnz, err));
    RCHK(S.alloc(&T.val, T.nnz, err));
    hem_t_kernel<<<nblk(m), 256>>>(m, act, a, T.ptr, T.col, T.val, 1);
    HIPCHK(hipGetLastError());
    RCHK(spgemm(G, W, BTent{a, m, nagg}, nagg, &WT, err, 1.0));
    RCHK(transpose(G, T, &Tt, err));
    RCHK(spgemm(G, Tt, BCsr{WT.ptr, WT.col, WT.val}, nagg, &C, err,
                WT.n ? (double)WT.nnz / (double)WT.n : 1.0));
    for (void* q : {(void*)WT.ptr, (void*)WT.col, (void*)WT.val, (void*)Tt.ptr, (void*)Tt.col, (void*)Tt.val})
      G->release(q);
    DevMat W2;
    RCHK(wgraph(C, nullptr, 0, &S, &W2, err));
    for (void* q : {(void*)C.ptr, (void*)C.col, (void*)C.val}) G->release(q);
    W = W2;
    RCHK(S.alloc(&act, nagg, err));
    u8_fill_kernel<<<nblk(nagg), 256>>>(nagg, 1, act);
    HIPCHK(hipGetLastError());
  }
  {   // absorption of the nodes left alone, then compact ids
    unsigned long long* size = nullptr;
    int64_t *agg2 = nullptr, *used = nullptr;
    RCHK(S.alloc(&size, nagg, err));
    RCHK(S.alloc(&agg2, n, err));
    RCHK(S.alloc(&used, nagg, err));
    HIPCHK(dev_memset(size, 0, std::max<int64_t>(nagg, 1) * sizeof(unsigned long long)));
    HIPCHK(dev_memset(used, 0, std::max<int64_t>(nagg, 1) * sizeof(int64_t)));
    agg_size_kernel<<<nblk(n), 256>>>(n, agg, size);
    hem_absorb_kernel<<<nblk(n), 256>>>(n, W1.ptr, W1.col, W1.val, agg, size, agg2, used);
    HIPCHK(hipGetLastError());
    RCHK(dscan_incl_i64(used, used, nagg, nullptr, err));
    int64_t nused = 0;
    if (nagg) RCHK(to_host(&nused, used + nagg - 1, 1, err));
    agg_remap_kernel<<<nblk(n), 256>>>(n, agg2, used, agg);
    HIPCHK(hipGetLastError());
    nagg = nused;
  }
  *agg_out = agg;
  *nagg_out = nagg;
  return MAMG_OK;
}

// aggregation of the node graph of A (setup.cpp node_graph + strength +
// aggregate_mis2 / aggregate_hem); scalar: of A itself (num_functions 1)
int aggregate(GHier* G, const DevMat& A, int64_t nv, int level, double theta, bool scalar, int64_t** agg_out,
              int64_t* nagg_out, std::string* err) {
  Scratch S;
  DevMat Gr;
  if (scalar) {
    Gr = A;
  } else {
    Gr.n = Gr.m = nv;
    RCHK(S.alloc(&Gr.ptr, nv + 1, err));
    HIPCHK(dev_memset(Gr.ptr, 0, sizeof(int64_t)));
    // long rows (coarse levels): the 64 KB column-only staging (device.hip dev_csr_to_bsr)
    const unsigned g = (unsigned)((nv + RS_NODES - 1) / RS_NODES);
    const bool lng = (double)A.nnz / (double)std::max<int64_t>(1, 2 * nv) * RS_NODES > RS_CAP;
    if (lng) node_graph_kernel<false, RS_CAP_LONG><<<g, RS_NODES>>>(nv, A.ptr, A.col, A.val, Gr.ptr, nullptr, nullptr);
    else node_graph_kernel<false><<<g, RS_NODES>>>(nv, A.ptr, A.col, A.val, Gr.ptr, nullptr, nullptr);
    HIPCHK(hipGetLastError());
    RCHK(dscan_incl_i64(Gr.ptr, Gr.ptr, nv + 1, nullptr, err));
    RCHK(to_host(&Gr.nnz, Gr.ptr + nv, 1, err));
    RCHK(S.alloc(&Gr.col, Gr.nnz, err));
    RCHK(S.alloc(&Gr.val, Gr.nnz, err));
    const char* fe = opt("MAMG_CSR2BSR_FILL");   // 0: the column + value staged merge (tests, A/B)
    if (fe && std::atoi(fe) == 0) {
      node_graph_kernel<true><<<g, RS_NODES>>>(nv, A.ptr, A.col, A.val, Gr.ptr, Gr.col, Gr.val);
    } else {
      Scratch TS;
      double* T = nullptr;
      RCHK(TS.alloc(&T, 4 * std::max<int64_t>(Gr.nnz, 1), err));
      if (lng) node_graph_fill_kernel<RS_CAP_LONG><<<g, RS_NODES>>>(nv, A.ptr, A.col, A.val, Gr.ptr, Gr.col, Gr.val, T);
      else node_graph_fill_kernel<RS_CAP><<<g, RS_NODES>>>(nv, A.ptr, A.col, A.val, Gr.ptr, Gr.col, Gr.val, T);
      HIPCHK(hipGetLastError());
    }
  }
  double* d = nullptr;
  uint8_t *flag = nullptr, *nonisol = nullptr;
  int* ctr = nullptr;
  RCHK(S.alloc(&d, nv, err));
  RCHK(S.alloc(&flag, Gr.nnz, err));
  RCHK(S.alloc(&nonisol, nv, err));
  RCHK(S.alloc(&ctr, 2, err));
  HIPCHK(dev_memset(flag, 0, std::max<int64_t>(Gr.nnz, 1)));
  HIPCHK(dev_memset(ctr, 0, 2 * sizeof(int)));
  absdiag_kernel<<<nblk(nv), 256>>>(nv, Gr.ptr, Gr.col, Gr.val, d);
  strength_kernel<<<nblk(nv), 256>>>(nv, Gr.ptr, Gr.col, Gr.val, d, theta,
                                     G->params.strength_measure == MAMG_STRENGTH_ROWMAX, flag, ctr);
  HIPCHK(hipGetLastError());
  int nextra = 0;
  RCHK(read_int(ctr, &nextra, err));
  if (nextra) {
    *err = "GPU setup: strength graph has entries without a mirror (non-symmetric sparsity "
           "pattern); use the host setup (mamg_setup)";
    return MAMG_ERR_UNSUPPORTED;
  }
  if (G->params.aggregation_type == MAMG_HEM) return aggregate_hem_dev(G, Gr, flag, level, agg_out, nagg_out, err);
  if (G->params.aggregation_type == MAMG_VMB) {
    // sequential by definition: the strong graph built here goes to the
    // host, setup.cpp's aggregate_vmb (bitwise the host setup's, which
    // builds the same graph and flags) numbers the aggregates, and they come
    // back; every other setup step stays on the device
    std::vector<int64_t> hptr(nv + 1);
    std::vector<int32_t> hcol(Gr.nnz);
    std::vector<double> hval(Gr.nnz);
    std::vector<uint8_t> hflag(Gr.nnz);
    RCHK(to_host(hptr.data(), Gr.ptr, nv + 1, err));
    if (Gr.nnz) {
      RCHK(to_host(hcol.data(), Gr.col, Gr.nnz, err));
      RCHK(to_host(hval.data(), Gr.val, Gr.nnz, err));
      RCHK(to_host(hflag.data(), flag, Gr.nnz, err));
    }
    CsrView V;
    V.n = V.m = nv;
    V.ptr = hptr.data();
    V.col = hcol.data();
    V.val = hval.data();
    std::vector<int64_t> hagg;
    int64_t nagg = 0;
    int rc = aggregate_vmb_flags(V, hflag.data(), &hagg, &nagg, err);
    if (rc) return rc;
    int64_t* agg = nullptr;
    RCHK(galloc(G, &agg, nv, err));
    HIPCHK(hipMemcpy(agg, hagg.data(), nv * sizeof(int64_t), hipMemcpyHostToDevice));
    *agg_out = agg;
    *nagg_out = nagg;
    return MAMG_OK;
  }
  uint64_t *state = nullptr, *low = nullptr, *key = nullptr, *m1 = nullptr;
  unsigned long long* und = nullptr;
  RCHK(S.alloc(&state, nv, err));
  RCHK(S.alloc(&low, nv, err));
  RCHK(S.alloc(&key, nv, err));
  RCHK(S.alloc(&m1, nv, err));
  RCHK(shards_alloc(&S, &und, err));
  mis_init_kernel<<<nblk(nv), 256>>>(nv, Gr.ptr, flag, level, state, low, nonisol);
  const char* ms = opt("MAMG_MIS_STAGED");   // 0: the lane-per-row walks (tests, A/B)
  const bool mis_staged = ms ? std::atoi(ms) != 0 : true;
  for (int rounds = 0;; ++rounds) {
    if (rounds > 10000) { *err = "mis2 did not converge"; return MAMG_ERR_SETUP; }
    RCHK(shards_zero(und));
    mis_key_kernel<<<nblk(nv), 256>>>(nv, state, low, key, und);
    HIPCHK(hipGetLastError());
    unsigned long long hu = 0;
    RCHK(shards_read(und, false, &hu, err));
    if (hu == 0) break;
    if (mis_staged) {   // the update stages every entry: only while many nodes are undecided
      mis_staged_kernel<false><<<nblk(nv), 256>>>(nv, Gr.ptr, Gr.col, flag, key, nullptr, m1);
      if (hu * 4 > (unsigned long long)nv)
        mis_staged_kernel<true><<<nblk(nv), 256>>>(nv, Gr.ptr, Gr.col, flag, m1, key, state);
      else
        mis_update_kernel<<<nblk(nv), 256>>>(nv, Gr.ptr, Gr.col, flag, m1, key, state);
    } else {
      mis_max_kernel<<<nblk(nv), 256>>>(nv, Gr.ptr, Gr.col, flag, key, m1);
      mis_update_kernel<<<nblk(nv), 256>>>(nv, Gr.ptr, Gr.col, flag, m1, key, state);
    }
  }
  int64_t *f = nullptr, *agg = nullptr, *agg2 = nullptr, *agg3 = nullptr;
  RCHK(S.alloc(&f, nv, err));
  RCHK(S.alloc(&agg, nv, err));
  RCHK(S.alloc(&agg2, nv, err));
  RCHK(galloc(G, &agg3, nv, err));
  root_flag_kernel<<<nblk(nv), 256>>>(nv, state, f);
  RCHK(dscan_incl_i64(f, f, nv, nullptr, err));
  int64_t nroots = 0;
  RCHK(to_host(&nroots, f + nv - 1, 1, err));
  root_number_kernel<<<nblk(nv), 256>>>(nv, state, f, agg);
  agg_phase2_kernel<<<nblk(nv), 256>>>(nv, Gr.ptr, Gr.col, flag, state, agg, agg2);
  agg_phase3_kernel<<<nblk(nv), 256>>>(nv, Gr.ptr, Gr.col, Gr.val, flag, nonisol, agg2, agg3, ctr + 1);
  HIPCHK(hipGetLastError());
  int bad = 0;
  RCHK(read_int(ctr + 1, &bad, err));
  if (bad) { *err = "aggregation left a non-isolated node unassigned"; return MAMG_ERR_SETUP; }
  *agg_out = agg3;
  *nagg_out = nroots;
  return MAMG_OK;
}

int coarsest_inverse(GHier* G, const DevMat& A, double** inv_out, std::string* err) {
  Scratch S;
  const int64_t n = A.n, w = 2 * n;
  double *M = nullptr, *f = nullptr, *inv = nullptr;
  int* bad = nullptr;
  RCHK(S.alloc(&M, n * w, err));
  RCHK(S.alloc(&f, n + 1, err));
  RCHK(S.alloc(&bad, 1, err));
  RCHK(galloc(G, &inv, n * n, err));
  HIPCHK(dev_memset(bad, 0, sizeof(int)));
  dense_init_kernel<<<nblk(n), 256>>>(n, A.ptr, A.col, A.val, M);
  for (int64_t k = 0; k < n; ++k) {
    gj_col_kernel<<<nblk(n), 256>>>(n, k, M, f);
    gj_scale_kernel<<<nblk(w), 256>>>(n, k, M, f, bad);
    gj_elim_kernel<<<nblk(n * w), 256>>>(n, k, M, f);
  }
  gj_extract_kernel<<<nblk(n * n), 256>>>(n, M, inv);
  HIPCHK(hipGetLastError());
  int hb = 0;
  RCHK(read_int(bad, &hb, err));
  if (hb) { *err = "coarsest matrix not SPD"; return MAMG_ERR_SETUP; }
  *inv_out = inv;
  return MAMG_OK;
}

int bits_for(int64_t v) {   // key bits covering 0..v
  int b = 1;
  while (b < 63 && (int64_t(1) << b) <= v) ++b;
  return b;
}

// point quantities of one level (setup.cpp host_setup: dg, dinv, rs, rho)
struct PointLevel {
  double *dg = nullptr, *dinv = nullptr, *rs = nullptr;
  double rho = 0.0;
};

// rho_estimate: Gershgorin bound (iters 0) or inf-norm power iterations of
// D^-1 A; the maxima are exact, each row sums in CSR order
int rho_estimate_dev(const DevMat& A, const PointLevel& P, int iters, Scratch* S, double* rho, std::string* err) {
  const int64_t n = A.n;
  if (iters == 0) {
    double* m = nullptr;
    RCHK(S->alloc(&m, 1, err));
    maxprod_kernel<<<1, 1024>>>(n, P.dinv, P.rs, m);
    HIPCHK(hipGetLastError());
    return to_host(rho, m, 1, err);
  }
  double *v = nullptr, *w = nullptr;
  unsigned long long* bits = nullptr;
  RCHK(S->alloc(&v, n, err));
  RCHK(S->alloc(&w, n, err));
  RCHK(S->alloc(&bits, 2, err));
  hash_vec_kernel<<<nblk(n), 256>>>(n, v);
  const unsigned gm = (unsigned)std::min<int64_t>(nblk(n), 1024);
  for (int it = 0; it < iters; ++it) {
    row_spmv_kernel<<<nblk(n), 256>>>(n, A.ptr, A.col, A.val, P.dinv, v, w);
    HIPCHK(dev_memset(bits, 0, 2 * sizeof(unsigned long long), nullptr));
    maxabs2_kernel<<<gm, 256>>>(n, v, w, bits);
    vnorm_kernel<<<nblk(n), 256>>>(n, w, bits, v);
  }
  HIPCHK(hipGetLastError());
  unsigned long long hb[2] = {0, 0};
  RCHK(to_host(hb, bits, 2, err));
  double mv, mw;
  std::memcpy(&mv, &hb[0], sizeof(double));
  std::memcpy(&mw, &hb[1], sizeof(double));
  *rho = mw / mv;
  return MAMG_OK;
}

int point_level(const DevMat& A, const mamg_params& p, bool need_rho, Scratch* S, PointLevel* P,
                std::string* err) {
  const int64_t n = A.n;
  RCHK(S->alloc(&P->dg, n, err));
  RCHK(S->alloc(&P->dinv, n, err));
  RCHK(S->alloc(&P->rs, n, err));
  point_diag_kernel<<<nblk(n), 256>>>(n, A.ptr, A.col, A.val, P->dg, P->dinv, P->rs);
  HIPCHK(hipGetLastError());
  P->rho = 0.0;
  if (need_rho) RCHK(rho_estimate_dev(A, *P, p.rho_iters, S, &P->rho, err));
  return MAMG_OK;
}

// seed blocks (setup.cpp block_smoother): every non-seed dof joins its
// strongest seed neighbour, at most Schwarz_mmsize - 1 joiners per seed (the
// lowest indices); blocks numbered by their owner's index.  bid: block of
// every dof, bptr: block offsets of the members mem (ascending in a block)
struct SeedBlocks {
  int64_t *bid = nullptr, *bptr = nullptr, *mem = nullptr;
  int64_t nb = 0;
};

int seed_blocks_dev(const DevMat& A, const int32_t* idofs, int64_t n_idofs, int mmsize, Scratch* S,
                    SeedBlocks* B, std::string* err) {
  const int64_t n = A.n;
  int32_t* di = nullptr;
  uint8_t *isseed = nullptr, *isowner = nullptr;
  int64_t *best = nullptr, *idx = nullptr, *sidx = nullptr, *owner = nullptr, *oscan = nullptr;
  int32_t *key = nullptr, *skey = nullptr;
  int* bad = nullptr;
  RCHK(S->alloc(&di, n_idofs, err));
  RCHK(S->alloc(&isseed, n, err));
  RCHK(S->alloc(&isowner, n, err));
  RCHK(S->alloc(&best, n, err));
  RCHK(S->alloc(&idx, n, err));
  RCHK(S->alloc(&sidx, n, err));
  RCHK(S->alloc(&owner, n, err));
  RCHK(S->alloc(&oscan, n, err));
  RCHK(S->alloc(&key, n, err));
  RCHK(S->alloc(&skey, n, err));
  RCHK(S->alloc(&bad, 1, err));
  HIPCHK(hipMemcpy(di, idofs, n_idofs * sizeof(int32_t), hipMemcpyHostToDevice));
  HIPCHK(dev_memset(isseed, 0, n));
  HIPCHK(dev_memset(isowner, 0, n));
  HIPCHK(dev_memset(bad, 0, sizeof(int)));
  seed_mark_kernel<<<nblk(n_idofs), 256>>>(n_idofs, di, n, isseed, bad);
  best_seed_kernel<<<nblk(8 * n), 256>>>(n, A.ptr, A.col, A.val, isseed, best);
  best_key_kernel<<<nblk(n), 256>>>(n, best, key, idx);
  HIPCHK(hipGetLastError());
  int hb = 0;
  RCHK(read_int(bad, &hb, err));
  if (hb) { *err = "idofs out of range"; return MAMG_ERR_ARG; }
  RCHK(dsort_pairs_i32_i64(key, skey, idx, sidx, n, bits_for(n), nullptr, err));
  owner_kernel<<<nblk(n), 256>>>(n, skey, sidx, mmsize, owner, isowner);
  u8_to_i64_kernel<<<nblk(n), 256>>>(n, isowner, oscan);
  HIPCHK(hipGetLastError());
  RCHK(dscan_incl_i64(oscan, oscan, n, nullptr, err));
  RCHK(to_host(&B->nb, oscan + n - 1, 1, err));
  RCHK(S->alloc(&B->bid, n, err));
  RCHK(S->alloc(&B->bptr, B->nb + 1, err));
  RCHK(S->alloc(&B->mem, n, err));
  HIPCHK(dev_memset(B->bptr, 0, (B->nb + 1) * sizeof(int64_t)));
  bid_kernel<<<nblk(n), 256>>>(n, owner, oscan, B->bid, key, idx, (unsigned long long*)B->bptr);
  HIPCHK(hipGetLastError());
  RCHK(dscan_incl_i64(B->bptr, B->bptr, B->nb + 1, nullptr, err));
  return dsort_pairs_i32_i64(key, skey, idx, B->mem, n, bits_for(B->nb), nullptr, err);
}

// the node-aligned fast path of the seed blocks: *aligned and joined[] set
// when every joiner joins its own node's other dof (seed_align_kernel)
int seed_align_fast(const DevMat& A, int64_t nv, const int32_t* idofs, int64_t n_idofs, int mmsize, Scratch* S,
                    uint8_t* joined, bool* aligned, std::string* err) {
  const int64_t n = A.n;
  int32_t* di = nullptr;
  uint8_t* isseed = nullptr;
  int64_t* best = nullptr;
  int* bad = nullptr;
  RCHK(S->alloc(&di, n_idofs, err));
  RCHK(S->alloc(&isseed, n, err));
  RCHK(S->alloc(&best, n, err));
  RCHK(S->alloc(&bad, 2, err));
  HIPCHK(hipMemcpy(di, idofs, n_idofs * sizeof(int32_t), hipMemcpyHostToDevice));
  HIPCHK(dev_memset(isseed, 0, n));
  HIPCHK(dev_memset(bad, 0, 2 * sizeof(int)));
  seed_mark_kernel<<<nblk(n_idofs), 256>>>(n_idofs, di, n, isseed, bad);
  best_seed_kernel<<<nblk(8 * n), 256>>>(n, A.ptr, A.col, A.val, isseed, best);
  seed_align_kernel<<<nblk(nv), 256>>>(nv, isseed, best, mmsize, joined, bad + 1);
  HIPCHK(hipGetLastError());
  int hb[2] = {0, 0};
  RCHK(to_host(hb, bad, 2, err));
  if (hb[0]) { *err = "idofs out of range"; return MAMG_ERR_ARG; }
  *aligned = hb[1] == 0;
  for (void* q : {(void*)di, (void*)isseed, (void*)best, (void*)bad}) S->release(q);
  return MAMG_OK;
}

// D = D_B^-1 as a block CSR (setup.cpp block_inverse: row i holds its
// block's inverse row, columns = the block's members ascending)
int block_inverse_dev(GHier* G, const DevMat& A, const SeedBlocks& B, Scratch* S, DevMat* D, std::string* err) {
  const int64_t n = A.n, nb = B.nb;
  int64_t *pos = nullptr, *f = nullptr;
  int* bad = nullptr;
  RCHK(S->alloc(&pos, n, err));
  RCHK(S->alloc(&f, nb, err));
  RCHK(S->alloc(&bad, 1, err));
  HIPCHK(dev_memset(bad, 0, sizeof(int)));
  D->n = D->m = n;
  RCHK(galloc(G, &D->ptr, n + 1, err));
  HIPCHK(dev_memset(D->ptr, 0, sizeof(int64_t)));
  member_pos_kernel<<<nblk(n), 256>>>(n, B.mem, B.bid, B.bptr, pos, D->ptr);
  HIPCHK(hipGetLastError());
  RCHK(dscan_incl_i64(D->ptr, D->ptr, n + 1, nullptr, err));
  RCHK(to_host(&D->nnz, D->ptr + n, 1, err));
  RCHK(galloc(G, &D->col, D->nnz, err));
  RCHK(galloc(G, &D->val, D->nnz, err));
  blk_single_kernel<<<nblk(nb), 256>>>(nb, B.bptr, B.mem, A.ptr, A.col, A.val, D->ptr, D->col, D->val, bad);
  multi_flag_kernel<<<nblk(nb), 256>>>(nb, B.bptr, f);
  HIPCHK(hipGetLastError());
  RCHK(dscan_incl_i64(f, f, nb, nullptr, err));
  int64_t nm = 0;
  RCHK(to_host(&nm, f + nb - 1, 1, err));
  if (nm) {
    int64_t *list = nullptr, *gj = nullptr;
    RCHK(S->alloc(&list, nm, err));
    RCHK(S->alloc(&gj, nm, err));
    multi_list_kernel<<<nblk(nb), 256>>>(nb, B.bptr, f, list, gj);
    HIPCHK(hipGetLastError());
    RCHK(dscan_incl_i64(gj, gj, nm, nullptr, err));
    int64_t tot = 0;
    RCHK(to_host(&tot, gj + nm - 1, 1, err));
    double* scratch = nullptr;
    RCHK(S->alloc(&scratch, tot, err));
    blk_multi_kernel<<<(unsigned)nm, 64>>>(list, nm, gj, B.bptr, B.mem, B.bid, pos, A.ptr, A.col, A.val, scratch,
                                           D->ptr, D->col, D->val, bad);
    HIPCHK(hipGetLastError());
  }
  int hb = 0;
  RCHK(read_int(bad, &hb, err));
  if (hb) { *err = "smoother block not SPD (non-positive pivot)"; return MAMG_ERR_SETUP; }
  return MAMG_OK;
}

// rho_B = max_i sum_j |(D A)_ij| (setup.cpp block_rho: SMMP row of D A, sorted
// columns, zeros skipped) through the hash SpGEMM
int block_rho_dev(const DevMat& D, const DevMat& A, double* rho, std::string* err) {
  GHier tmp;
  DevMat C;
  RCHK(spgemm(&tmp, D, BCsr{A.ptr, A.col, A.val}, A.m, &C, err, A.n ? (double)A.nnz / (double)A.n : 1.0));
  Scratch S;
  unsigned long long* bits = nullptr;
  RCHK(shards_alloc(&S, &bits, err));
  rowabs_max_kernel<<<nblk(C.n), 256>>>(C.n, C.ptr, C.val, bits);
  HIPCHK(hipGetLastError());
  unsigned long long h = 0;
  RCHK(shards_read(bits, true, &h, err));
  std::memcpy(rho, &h, sizeof(double));
  return MAMG_OK;
}

// additive Schwarz on the seeds' overlapping rings (setup.cpp
// overlap_smoother): the blocks' inverses summed in seed order into the
// merged pattern (sorted (row, column) keys, stable, so each entry's run is in
// seed order), 1 / a_ii on uncovered dofs, then W = (relaxation / lambda) S
// with lambda from max(rho_iters, 30) power iterations of S A
int overlap_smoother_dev(GHier* G, const DevMat& A, const int32_t* seeds, int64_t ns, const mamg_params& p,
                         DevMat* W, std::string* err) {
  const int64_t n = A.n;
  const int maxlvl = p.Schwarz_maxlvl, mm = p.Schwarz_mmsize;
  if (ns > std::max<int64_t>(n / 8, 1) || (double)ns * mm * mm > 4e9) {
    *err = "SCHWARZ_ADDITIVE (dense overlapping seed blocks) is for sparse seed sets: " + std::to_string(ns) +
           " seeds of up to " + std::to_string(mm) + " dofs";
    return MAMG_ERR_UNSUPPORTED;
  }
  if (mm < 1 || mm > 8192) {
    *err = "GPU setup: SCHWARZ_ADDITIVE with Schwarz_mmsize " + std::to_string(mm) +
           " (1..8192 on the GPU); use the host setup (mamg_setup)";
    return MAMG_ERR_UNSUPPORTED;
  }
  for (int64_t k = 0; k < ns; ++k)
    if (seeds[k] < 0 || seeds[k] >= n) { *err = "idofs out of range"; return MAMG_ERR_ARG; }
  Scratch S;
  int32_t *ds = nullptr, *blk = nullptr;
  int64_t *blen = nullptr, *sq = nullptr, *gj = nullptr;
  uint8_t* cov = nullptr;
  int* bad = nullptr;
  RCHK(S.alloc(&ds, ns, err));
  RCHK(S.alloc(&blk, ns * mm, err));
  RCHK(S.alloc(&blen, ns, err));
  RCHK(S.alloc(&sq, ns, err));
  RCHK(S.alloc(&gj, ns, err));
  RCHK(S.alloc(&cov, n, err));
  RCHK(S.alloc(&bad, 1, err));
  HIPCHK(hipMemcpy(ds, seeds, ns * sizeof(int32_t), hipMemcpyHostToDevice));
  HIPCHK(dev_memset(cov, 0, n));
  HIPCHK(dev_memset(bad, 0, sizeof(int)));
  ring_bfs_kernel<<<(unsigned)ns, 64, 2 * (size_t)mm * sizeof(int32_t)>>>(ns, ds, A.ptr, A.col, maxlvl, mm, blk, blen);
  sq_len_kernel<<<nblk(ns), 256>>>(ns, blen, sq, gj);
  HIPCHK(hipGetLastError());
  RCHK(dscan_incl_i64(sq, sq, ns, nullptr, err));
  RCHK(dscan_incl_i64(gj, gj, ns, nullptr, err));
  int64_t nc = 0, ngj = 0;
  RCHK(to_host(&nc, sq + ns - 1, 1, err));
  RCHK(to_host(&ngj, gj + ns - 1, 1, err));
  double *inv = nullptr, *scratch = nullptr;
  RCHK(S.alloc(&inv, nc, err));
  RCHK(S.alloc(&scratch, ngj, err));
  ring_inv_kernel<<<(unsigned)ns, 256>>>(ns, mm, blk, blen, sq, gj, A.ptr, A.col, A.val, scratch, inv, cov, bad);
  HIPCHK(hipGetLastError());
  int hb = 0;
  RCHK(read_int(bad, &hb, err));
  if (hb) { *err = "Schwarz block not SPD"; return MAMG_ERR_SETUP; }
  S.release(scratch);
  // contributions: block keys, then the uncovered diagonal
  int64_t* uscan = nullptr;
  RCHK(S.alloc(&uscan, n, err));
  uncov_flag_kernel<<<nblk(n), 256>>>(n, cov, uscan);
  HIPCHK(hipGetLastError());
  RCHK(dscan_incl_i64(uscan, uscan, n, nullptr, err));
  int64_t nu = 0;
  RCHK(to_host(&nu, uscan + n - 1, 1, err));
  const int64_t e = nc + nu;
  uint64_t *key = nullptr, *skey = nullptr;
  int64_t *src = nullptr, *ssrc = nullptr;
  RCHK(S.alloc(&key, e, err));
  RCHK(S.alloc(&skey, e, err));
  RCHK(S.alloc(&src, e, err));
  RCHK(S.alloc(&ssrc, e, err));
  ring_keys_kernel<<<(unsigned)ns, 64>>>(ns, mm, n, blk, blen, sq, key, src);
  uncov_keys_kernel<<<nblk(n), 256>>>(n, cov, uscan, nc, key, src);
  HIPCHK(hipGetLastError());
  RCHK(dsort_pairs_u64_i64(key, skey, src, ssrc, e, bits_for(n * n - 1), nullptr, err));
  S.release(key);
  S.release(src);
  int64_t* fscan = nullptr;
  RCHK(S.alloc(&fscan, e, err));
  run_flag_kernel<<<nblk(e), 256>>>(e, skey, fscan);
  HIPCHK(hipGetLastError());
  RCHK(dscan_incl_i64(fscan, fscan, e, nullptr, err));
  int64_t nw = 0;
  RCHK(to_host(&nw, fscan + e - 1, 1, err));
  int64_t* ustart = nullptr;
  RCHK(S.alloc(&ustart, nw, err));
  W->n = W->m = n;
  W->nnz = nw;
  RCHK(galloc(G, &W->ptr, n + 1, err));
  RCHK(galloc(G, &W->col, nw, err));
  RCHK(galloc(G, &W->val, nw, err));
  HIPCHK(dev_memset(W->ptr, 0, (n + 1) * sizeof(int64_t)));
  run_start_kernel<<<nblk(e), 256>>>(e, n, skey, fscan, ustart, W->col, (unsigned long long*)W->ptr);
  HIPCHK(hipGetLastError());
  RCHK(dscan_incl_i64(W->ptr, W->ptr, n + 1, nullptr, err));
  run_sum_kernel<<<nblk(nw), 256>>>(nw, e, ustart, ssrc, inv, A.ptr, A.col, A.val, W->val);
  HIPCHK(hipGetLastError());
  // lambda_max(S A): inf-norm power iterations from the hash start vector
  double *v = nullptr, *t = nullptr, *w = nullptr;
  unsigned long long* bits = nullptr;
  RCHK(S.alloc(&v, n, err));
  RCHK(S.alloc(&t, n, err));
  RCHK(S.alloc(&w, n, err));
  RCHK(S.alloc(&bits, 2, err));
  hash_vec_kernel<<<nblk(n), 256>>>(n, v);
  const unsigned gm = (unsigned)std::min<int64_t>(nblk(n), 1024);
  for (int it = 0; it < std::max(p.rho_iters, 30); ++it) {
    row_spmv_kernel<<<nblk(n), 256>>>(n, A.ptr, A.col, A.val, nullptr, v, t);
    row_spmv_kernel<<<nblk(n), 256>>>(n, W->ptr, W->col, W->val, nullptr, t, w);
    HIPCHK(dev_memset(bits, 0, 2 * sizeof(unsigned long long), nullptr));
    maxabs2_kernel<<<gm, 256>>>(n, v, w, bits);
    vnorm_kernel<<<nblk(n), 256>>>(n, w, bits, v);
  }
  HIPCHK(hipGetLastError());
  unsigned long long hbits[2] = {0, 0};
  RCHK(to_host(hbits, bits, 2, err));
  double mv, mw;
  std::memcpy(&mv, &hbits[0], sizeof(double));
  std::memcpy(&mw, &hbits[1], sizeof(double));
  const double lam = mw / mv;
  scale_vals_kernel<<<nblk(nw), 256>>>(nw, p.relaxation / lam, W->val);
  HIPCHK(hipGetLastError());
  return MAMG_OK;
}

}  // namespace

void ring_blocks_free(RingBlocks* R) {
  for (void* q : {(void*)R->blk, (void*)R->blen, (void*)R->sq, (void*)R->inv}) tmp_free(q);
  *R = RingBlocks();
}

// the SCHWARZ_RINGS blocks: ring_bfs_kernel / ring_inv_kernel of the
// additive form (the same blocks and Gauss-Jordan inverses), kept per block
int ring_blocks_dev(const DevMat& A, const int32_t* seeds, int64_t ns, int maxlvl, int mm, RingBlocks* R,
                    std::string* err) {
  *R = RingBlocks();
  const int64_t n = A.n;
  if (ns <= 0) { *err = "seed rings: no seeds"; return MAMG_ERR_ARG; }
  if (mm < 1 || mm > 8192) { *err = "seed rings: Schwarz_mmsize must be in [1, 8192]"; return MAMG_ERR_UNSUPPORTED; }
  for (int64_t k = 0; k < ns; ++k)
    if (seeds[k] < 0 || seeds[k] >= n) { *err = "idofs out of range"; return MAMG_ERR_ARG; }
  Scratch S;
  RingBlocks B;
  B.ns = ns;
  B.mm = mm;
  int32_t* ds = nullptr;
  int64_t* gj = nullptr;
  uint8_t* cov = nullptr;
  int* bad = nullptr;
  auto fail = [&](int rc) { ring_blocks_free(&B); return rc; };
  if (tmp_malloc((void**)&B.blk, (size_t)ns * mm * sizeof(int32_t)) != hipSuccess ||
      tmp_malloc((void**)&B.blen, (size_t)ns * sizeof(int64_t)) != hipSuccess ||
      tmp_malloc((void**)&B.sq, (size_t)ns * sizeof(int64_t)) != hipSuccess) {
    (void)hipGetLastError();
    *err = "seed rings: device allocation failed";
    return fail(MAMG_ERR_HIP);
  }
  int rc;
  if ((rc = S.alloc(&ds, ns, err)) || (rc = S.alloc(&gj, ns, err)) || (rc = S.alloc(&cov, n, err)) ||
      (rc = S.alloc(&bad, 1, err)))
    return fail(rc);
  if (hipMemcpy(ds, seeds, ns * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess ||
      dev_memset(bad, 0, sizeof(int)) != hipSuccess) {
    *err = "seed rings: copy failed";
    return fail(MAMG_ERR_HIP);
  }
  ring_bfs_kernel<<<(unsigned)ns, 64, 2 * (size_t)mm * sizeof(int32_t)>>>(ns, ds, A.ptr, A.col, maxlvl, mm, B.blk,
                                                                         B.blen);
  sq_len_kernel<<<nblk(ns), 256>>>(ns, B.blen, B.sq, gj);
  if (hipGetLastError() != hipSuccess) { *err = "seed rings: launch failed"; return fail(MAMG_ERR_HIP); }
  if ((rc = dscan_incl_i64(B.sq, B.sq, ns, nullptr, err)) || (rc = dscan_incl_i64(gj, gj, ns, nullptr, err)))
    return fail(rc);
  int64_t ngj = 0;
  if ((rc = to_host(&B.ninv, B.sq + ns - 1, 1, err)) || (rc = to_host(&ngj, gj + ns - 1, 1, err))) return fail(rc);
  double* scratch = nullptr;
  if (tmp_malloc((void**)&B.inv, (size_t)std::max<int64_t>(B.ninv, 1) * sizeof(double)) != hipSuccess) {
    (void)hipGetLastError();
    *err = "seed rings: device allocation failed";
    return fail(MAMG_ERR_HIP);
  }
  if ((rc = S.alloc(&scratch, ngj, err))) return fail(rc);
  ring_inv_kernel<<<(unsigned)ns, 256>>>(ns, mm, B.blk, B.blen, B.sq, gj, A.ptr, A.col, A.val, scratch, B.inv, cov,
                                         bad);
  if (hipGetLastError() != hipSuccess) { *err = "seed rings: launch failed"; return fail(MAMG_ERR_HIP); }
  int hb = 0;
  if ((rc = read_int(bad, &hb, err))) return fail(rc);
  if (hb) { *err = "seed rings: a Schwarz block is not SPD (non-positive pivot)"; return fail(MAMG_ERR_SETUP); }
  *R = B;
  return MAMG_OK;
}

// The runtime loads a translation unit's code object at the first launch of
// one of its kernels (deferred loading).  dprims' (the hipCUB scans and
// sorts) took 46 ms inside the aggregation phase at nrefs=6, gsetup.hip's and
// device.hip's ~5-6 ms each (profiles/r05_setup_gaps.txt).  A helper
// thread launches one kernel of each while the host copies A_0 (or while the
// setup's first kernels run), once per device and process.
__global__ void gsetup_warm_kernel() {}

struct ModuleWarm {
  std::thread t;
  explicit ModuleWarm(int dev) {
    static std::atomic<uint64_t> done{0};
    const uint64_t bit = 1ull << (dev & 63);
    if (done.fetch_or(bit) & bit) return;
    t = std::thread([dev] {
      if (hipSetDevice(dev) != hipSuccess) { (void)hipGetLastError(); return; }
      hipStream_t s = nullptr;
      if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) { (void)hipGetLastError(); return; }
      gsetup_warm_kernel<<<1, 64, 0, s>>>();
      dprims_warm(s);
      device_warm(s);
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
      (void)hipGetLastError();
    });
  }
  ~ModuleWarm() {
    if (t.joinable()) t.join();
  }
};

int gpu_setup(const DevMat& A0, const int32_t* idofs, int64_t n_idofs, const mamg_params& p, GHier* G,
              std::string* err) {
  int rc = check_params(p, err);
  if (rc) return rc;
  if ((rc = check_patch_seeds(p, idofs, n_idofs, A0.n, err))) return rc;
  const int nf = p.num_functions;
  if (nf != 1 && nf != 2) {
    *err = "GPU setup covers num_functions 1 and 2; use the host setup (mamg_setup) for other profiles";
    return MAMG_ERR_UNSUPPORTED;
  }
  const bool nodal = nf == 2;
  if (A0.n != A0.m || A0.n <= 0 || A0.n % nf) {
    *err = "A must be square with a size divisible by num_functions";
    return MAMG_ERR_ARG;
  }
  G->params = p;
  G->device = p.device;
  ModuleWarm warm(p.device);   // no-op when the A_0 upload did it
  G->levels.clear();
  G->seeds.clear();
  G->generic = false;
  HIPCHK(hipSetDevice(p.device));
  Clock clk, tot;
  {
    Scratch S;
    int* bad = nullptr;
    RCHK(S.alloc(&bad, 1, err));
    HIPCHK(dev_memset(bad, 0, sizeof(int)));
    validate_kernel<<<nblk(8 * A0.n), 256>>>(A0.n, A0.m, A0.ptr, A0.col, bad);
    HIPCHK(hipGetLastError());
    int hb = 0;
    RCHK(read_int(bad, &hb, err));
    if (hb) {
      *err = "rowptr not monotone, or column index out of range or not strictly increasing within a row";
      return MAMG_ERR_ARG;
    }
  }
  // the host setup's per-level decisions (setup.cpp host_setup)
  const bool blockP = nodal && p.sa_block_diag;
  const bool rho_smoother = p.smoother == MAMG_SMOOTHER_JACOBI_RHO || p.smoother == MAMG_SMOOTHER_POLY;
  DevMat cur = A0;
  for (int l = 0; l < p.max_levels; ++l) {
    G->levels.emplace_back();
    GLevel& L = G->levels.back();
    if (l > 0) L.A = cur;
    const int64_t n = cur.n, nv = n / nf;
    L.n = n;
    bool last = (n <= p.coarse_dof) || (l == p.max_levels - 1);
    int64_t* agg = nullptr;
    int64_t nagg = 0;
    if (n % nf) { *err = "matrix size not divisible by num_functions"; return MAMG_ERR_ARG; }
    clk.lap();
    if (!last) {
      RCHK(aggregate(G, cur, nv, l, p.strong_coupled, !nodal, &agg, &nagg, err));
      if (nagg == 0 || nf * nagg >= n) last = true;
    }
    G->phase_ms[0] += clk.lap();
    if (last) {
      if (n > p.max_coarse_dense) {
        *err = "coarsest level " + std::to_string(n) + " too large for dense solve";
        return MAMG_ERR_SETUP;
      }
      RCHK(coarsest_inverse(G, cur, &L.Ainv, err));
      L.coarsest = true;
      G->phase_ms[4] += clk.lap();
      break;
    }
    L.agg = agg;
    L.nagg = nagg;
    Scratch S;
    // smoother: overlapping seed rings (ADDITIVE), seed blocks (node-aligned:
    // 2x2 node blocks with split nodes; else a general block CSR), 2x2 node
    // blocks, or point weights
    // seed rings (SCHWARZ_RINGS): the level-0 Schwarz data are built with the
    // apply layout (device.hip build_rings); the node-block smoother stands in
    const bool rings = seed_blocks_on(p, l, idofs, n_idofs) && p.Schwarz_type == MAMG_SCHWARZ_RINGS;
    const bool seeds = seed_blocks_on(p, l, idofs, n_idofs) && !rings;
    if (rings) {
      RCHK(check_ring_seeds(p, idofs, n_idofs, n, err));
      G->seeds.assign(idofs, idofs + n_idofs);
    }
    const bool pointSA = p.AMG_type == MAMG_SA_AMG && !blockP;
    bool node = false;              // smoother as 2x2 node blocks in Dsm / L.W
    bool full_nodes = false;        // ... and those are the full node blocks
    dv4_t* Dsm = nullptr;
    double rho_sm = 0.0;
    PointLevel PL;
    const bool point_smoother = !seeds && !(nodal && p.node_block_smoother);
    if (pointSA || point_smoother) RCHK(point_level(cur, p, pointSA || (point_smoother && rho_smoother), &S, &PL, err));
    if (seeds && p.Schwarz_type == MAMG_SCHWARZ_ADDITIVE) {
      RCHK(overlap_smoother_dev(G, cur, idofs, n_idofs, p, &L.WB, err));
    } else if (seeds) {
      bool aligned = false;
      SeedBlocks B;
      if (nodal) {                  // the bidomain's case: every joiner joins its node partner
        RCHK(galloc(G, &L.joined, nv, err));
        RCHK(seed_align_fast(cur, nv, idofs, n_idofs, p.Schwarz_mmsize, &S, L.joined, &aligned, err));
        if (!aligned) { G->release(L.joined); L.joined = nullptr; }
      }
      if (!aligned) RCHK(seed_blocks_dev(cur, idofs, n_idofs, p.Schwarz_mmsize, &S, &B, err));
      if (nodal && !aligned) {      // general blocks that may still be node-aligned
        int* bad = nullptr;
        RCHK(S.alloc(&bad, 1, err));
        HIPCHK(dev_memset(bad, 0, sizeof(int)));
        RCHK(galloc(G, &L.joined, nv, err));
        align_kernel<<<nblk(nv), 256>>>(nv, B.bid, B.bptr, L.joined, bad);
        HIPCHK(hipGetLastError());
        int hb = 0;
        RCHK(read_int(bad, &hb, err));
        aligned = hb == 0;
        if (!aligned) { G->release(L.joined); L.joined = nullptr; }
      }
      if (aligned) {
        RCHK(S.alloc(&Dsm, nv, err));
        RCHK(node_inverse(cur, nv, L.joined, Dsm, "smoother", err));
        node = true;
        // every node joined (the bidomain's seeds on every u2 dof): these are
        // the full node blocks, bit for bit, so SA reuses them and their rho
        // instead of a second inversion and rho pass (~19 ms at nrefs=6)
        int* split = nullptr;
        RCHK(S.alloc(&split, 1, err));
        HIPCHK(dev_memset(split, 0, sizeof(int)));
        any_split_kernel<<<nblk(nv), 256>>>(nv, L.joined, split);
        HIPCHK(hipGetLastError());
        int hs = 1;
        RCHK(read_int(split, &hs, err));
        full_nodes = hs == 0;
      } else {
        RCHK(block_inverse_dev(G, cur, B, &S, &L.WB, err));
        double rho = 0.0;
        RCHK(block_rho_dev(L.WB, cur, &rho, err));
        scale_vals_kernel<<<nblk(L.WB.nnz), 256>>>(L.WB.nnz, p.relaxation / rho, L.WB.val);
        HIPCHK(hipGetLastError());
      }
    } else if (nodal && p.node_block_smoother) {
      RCHK(S.alloc(&Dsm, nv, err));
      RCHK(node_inverse(cur, nv, nullptr, Dsm, "smoother", err));
      node = full_nodes = true;
    } else {
      RCHK(galloc(G, &L.winv, n, err));
      const int kind = p.smoother == MAMG_SMOOTHER_JACOBI ? 0 : p.smoother == MAMG_SMOOTHER_L1DIAG ? 1 : 2;
      winv_kernel<<<nblk(n), 256>>>(n, kind, p.relaxation, PL.rho, PL.dg, PL.rs, L.winv);
      HIPCHK(hipGetLastError());
    }
    if (node) {
      RCHK(block_rho(cur, nv, Dsm, &rho_sm, err));
      RCHK(galloc(G, (dv4_t**)&L.W, nv, err));
      scale_blocks_kernel<<<nblk(nv), 256>>>(nv, p.relaxation / rho_sm, Dsm, (dv4_t*)L.W);
      HIPCHK(hipGetLastError());
    } else {
      G->generic = true;
    }
    G->phase_ms[1] += clk.lap();
    // prolongator
    if (p.AMG_type == MAMG_SA_AMG && blockP) {
      dv4_t* Dsa = Dsm;
      double rho_sa = rho_sm;
      if (!full_nodes) {            // SA always smooths with the full node blocks
        RCHK(S.alloc(&Dsa, nv, err));
        RCHK(node_inverse(cur, nv, nullptr, Dsa, "SA node", err));
        RCHK(block_rho(cur, nv, Dsa, &rho_sa, err));
      }
      const double w = p.sa_omega / rho_sa;
      L.w_sa = w;
      GHier tmp;                    // A T lives only until P is built
      DevMat AT;
      RCHK(spgemm(&tmp, cur, BTent{agg, nv, nagg}, 2 * nagg, &AT, err, 1.0, true));
      L.P.n = n;
      L.P.m = 2 * nagg;
      RCHK(galloc(G, &L.P.ptr, n + 1, err));
      HIPCHK(dev_memset(L.P.ptr, 0, sizeof(int64_t)));
      smooth_p_kernel<false><<<nblk(n), 256>>>(nv, AT.ptr, AT.col, AT.val, Dsa, agg, nagg, w, L.P.ptr,
                                               nullptr, nullptr);
      HIPCHK(hipGetLastError());
      RCHK(dscan_incl_i64(L.P.ptr, L.P.ptr, n + 1, nullptr, err));
      RCHK(to_host(&L.P.nnz, L.P.ptr + n, 1, err));
      RCHK(galloc(G, &L.P.col, L.P.nnz, err));
      RCHK(galloc(G, &L.P.val, L.P.nnz, err));
      smooth_p_kernel<true><<<nblk(n), 256>>>(nv, AT.ptr, AT.col, AT.val, Dsa, agg, nagg, w, L.P.ptr,
                                              L.P.col, L.P.val);
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(nullptr));
    } else if (pointSA) {           // point SA: c_i = (sa_omega / rho) / a_ii
      const double w = p.sa_omega / PL.rho;
      L.w_sa = w;
      GHier tmp;
      DevMat AT;
      RCHK(spgemm(&tmp, cur, BTent{agg, nv, nagg}, nf * nagg, &AT, err, 1.0));
      L.P.n = n;
      L.P.m = nf * nagg;
      RCHK(galloc(G, &L.P.ptr, n + 1, err));
      HIPCHK(dev_memset(L.P.ptr, 0, sizeof(int64_t)));
      smooth_pt_kernel<false><<<nblk(n), 256>>>(n, nv, agg, nagg, w, PL.dinv, AT.ptr, AT.col, AT.val, L.P.ptr,
                                                nullptr, nullptr);
      HIPCHK(hipGetLastError());
      RCHK(dscan_incl_i64(L.P.ptr, L.P.ptr, n + 1, nullptr, err));
      RCHK(to_host(&L.P.nnz, L.P.ptr + n, 1, err));
      RCHK(galloc(G, &L.P.col, L.P.nnz, err));
      RCHK(galloc(G, &L.P.val, L.P.nnz, err));
      smooth_pt_kernel<true><<<nblk(n), 256>>>(n, nv, agg, nagg, w, PL.dinv, AT.ptr, AT.col, AT.val, L.P.ptr,
                                               L.P.col, L.P.val);
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(nullptr));
    } else {
      L.P.n = n;
      L.P.m = nf * nagg;
      RCHK(galloc(G, &L.P.ptr, n + 1, err));
      HIPCHK(dev_memset(L.P.ptr, 0, sizeof(int64_t)));
      tent_kernel<<<nblk(n), 256>>>(n, nv, agg, nagg, L.P.ptr, nullptr, nullptr, 0);
      RCHK(dscan_incl_i64(L.P.ptr, L.P.ptr, n + 1, nullptr, err));
      RCHK(to_host(&L.P.nnz, L.P.ptr + n, 1, err));
      RCHK(galloc(G, &L.P.col, L.P.nnz, err));
      RCHK(galloc(G, &L.P.val, L.P.nnz, err));
      tent_kernel<<<nblk(n), 256>>>(n, nv, agg, nagg, L.P.ptr, L.P.col, L.P.val, 1);
      HIPCHK(hipGetLastError());
    }
    G->phase_ms[2] += clk.lap();
    // Galerkin: R = P^T, A P, A_c = R (A P)
    RCHK(transpose(G, L.P, &L.R, err));
    RCHK(spgemm(G, cur, BCsr{L.P.ptr, L.P.col, L.P.val}, L.P.m, &L.AP, err, (double)L.P.nnz / std::max<int64_t>(1, L.P.n),
                nodal));
    DevMat next;
    RCHK(spgemm(G, L.R, BCsr{L.AP.ptr, L.AP.col, L.AP.val}, L.AP.m, &next, err, (double)L.AP.nnz / std::max<int64_t>(1, L.AP.n),
                nodal));
    if (!p.post_fusion || !nodal) {   // host: A P kept for the fused post-smoothing of nodal levels
      for (void* q : {(void*)L.AP.ptr, (void*)L.AP.col, (void*)L.AP.val}) G->release(q);
      L.AP = DevMat();
    }
    HIPCHK(hipStreamSynchronize(nullptr));
    G->phase_ms[3] += clk.lap();
    if (p.print_level > 0)
      std::fprintf(stderr, "[mamg gpu] level %d: n=%lld nnz=%lld nagg=%lld nnzP=%lld\n", l, (long long)n,
                   (long long)cur.nnz, (long long)nagg, (long long)L.P.nnz);
    cur = next;
  }
  if (G->generic)   // CSR apply layout: node-block levels as block CSRs too
    for (GLevel& L : G->levels) {
      if (L.coarsest || !L.W) continue;
      const int64_t nv = L.n / 2;
      L.WB.n = L.WB.m = L.n;
      RCHK(galloc(G, &L.WB.ptr, L.n + 1, err));
      HIPCHK(dev_memset(L.WB.ptr, 0, sizeof(int64_t)));
      node_wb_kernel<<<nblk(L.n), 256>>>(nv, (const dv4_t*)L.W, L.joined, L.WB.ptr, nullptr, nullptr, 0);
      HIPCHK(hipGetLastError());
      RCHK(dscan_incl_i64(L.WB.ptr, L.WB.ptr, L.n + 1, nullptr, err));
      RCHK(to_host(&L.WB.nnz, L.WB.ptr + L.n, 1, err));
      RCHK(galloc(G, &L.WB.col, L.WB.nnz, err));
      RCHK(galloc(G, &L.WB.val, L.WB.nnz, err));
      node_wb_kernel<<<nblk(L.n), 256>>>(nv, (const dv4_t*)L.W, L.joined, L.WB.ptr, L.WB.col, L.WB.val, 1);
      HIPCHK(hipGetLastError());
      G->release(L.W);
      L.W = nullptr;
    }
  HIPCHK(hipStreamSynchronize(nullptr));
  G->phase_ms[6] = tot.lap();
  return MAMG_OK;
}

// ---------------------------------------------------------------------------
// The bidomain generator (gen.cpp) on the device: one thread per vertex
// computes the vertex's integer P1 stencil on the Kuhn-split lattice and
// writes its two rows; same operations as the host generator (this file is
// compiled without FMA contraction), so the matrix is bitwise the host's.
// Multi-GPU ranks build A_0 in HBM this way instead of holding the global
// matrix in host memory (13 GB per rank at nrefs=6).
// ---------------------------------------------------------------------------
namespace {

__device__ __forceinline__ bool gen_bc(int dim, int64_t n, int64_t v) {
  const int64_t nn = n + 1;
  const int64_t a = dim == 2 ? v % nn : v / (nn * nn);
  return a == 0 || a == n;
}

__device__ __forceinline__ int gen_kpath(int dim, int a, int b) {
  if (a == b) return (a == 0 || a == dim) ? 1 : 2;
  return (a - b == 1 || b - a == 1) ? -1 : 0;
}

// the vertex's stencil in column order: cnt entries of (column, cK, cM)
__device__ int gen_stencil(int dim, int64_t n, int64_t v, int64_t* col, int* cK, int* cM) {
  const int64_t nn = n + 1;
  const int64_t c[3] = {v % nn, (v / nn) % nn, dim == 3 ? v / (nn * nn) : 0};
  const int64_t stride[3] = {1, nn, nn * nn};
  int accK[27], accM[27];
  bool used[27];
  for (int s = 0; s < 27; ++s) { accK[s] = 0; accM[s] = 0; used[s] = false; }
  const int perms3[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
  const int perms2[2][3] = {{0, 1, 0}, {1, 0, 0}};
  const int ncorner = dim == 3 ? 8 : 4, npath = dim == 3 ? 6 : 2;
  for (int q = 0; q < ncorner; ++q) {
    const int d[3] = {q & 1, (q >> 1) & 1, (q >> 2) & 1};
    bool ok = true;
    for (int k = 0; k < dim; ++k) {
      const int64_t lo = c[k] - d[k];
      if (lo < 0 || lo >= n) ok = false;
    }
    if (!ok) continue;
    for (int pth = 0; pth < npath; ++pth) {
      const int* perm = dim == 3 ? perms3[pth] : perms2[pth];
      int pv[4][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
      for (int t = 1; t <= dim; ++t) {
        for (int k = 0; k < 3; ++k) pv[t][k] = pv[t - 1][k];
        pv[t][perm[t - 1]] += 1;
      }
      int t_me = -1;
      for (int t = 0; t <= dim; ++t)
        if (pv[t][0] == d[0] && pv[t][1] == d[1] && pv[t][2] == d[2]) t_me = t;
      if (t_me < 0) continue;
      for (int s = 0; s <= dim; ++s) {
        const int slot = (pv[s][0] - d[0] + 1) + 3 * (pv[s][1] - d[1] + 1) + 9 * (pv[s][2] - d[2] + 1);
        used[slot] = true;
        accK[slot] += gen_kpath(dim, t_me, s);
        accM[slot] += (t_me == s) ? 2 : 1;
      }
    }
  }
  int cnt = 0;
  for (int dz = -1; dz <= 1; ++dz)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int slot = (dx + 1) + 3 * (dy + 1) + 9 * (dz + 1);
        if (!used[slot]) continue;
        col[cnt] = v + dx * stride[0] + dy * stride[1] + dz * stride[2];
        cK[cnt] = accK[slot];
        cM[cnt] = accM[slot];
        ++cnt;
      }
  return cnt;
}

// row length of vertex v's rows (2 k, or 1 on a Dirichlet vertex)
__global__ __launch_bounds__(256) void gen_len_kernel(int dim, int64_t n, int64_t nv, int64_t* __restrict__ len) {
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= nv) return;
  if (gen_bc(dim, n, v)) { len[v] = 1; return; }
  int64_t col[27];
  int cK[27], cM[27];
  const int cnt = gen_stencil(dim, n, v, col, cK, cM);
  int k = 0;
  for (int j = 0; j < cnt; ++j) k += !gen_bc(dim, n, col[j]);
  len[v] = 2 * k;
}

// rowptr of the u1 rows [0, nv] and the u2 rows [nv, 2 nv] from the
// inclusive scan of the lengths
__global__ __launch_bounds__(256) void gen_ptr_kernel(int64_t nv, const int64_t* __restrict__ scan,
                                                      int64_t* __restrict__ ptr) {
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (v > nv) return;
  const int64_t s = v ? scan[v - 1] : 0;
  ptr[v] = s;
  ptr[nv + v] = scan[nv - 1] + s;
}

__global__ __launch_bounds__(256) void gen_fill_kernel(int dim, int64_t n, int64_t nv, double kf1, double kf2,
                                                       double mf, const int64_t* __restrict__ ptr,
                                                       int32_t* __restrict__ colind, double* __restrict__ values) {
#pragma clang fp contract(off)
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= nv) return;
  const int64_t p1 = ptr[v], p2 = ptr[nv + v];
  if (gen_bc(dim, n, v)) {
    colind[p1] = (int32_t)v; values[p1] = 1.0;
    colind[p2] = (int32_t)(v + nv); values[p2] = 1.0;
    return;
  }
  int64_t col[27];
  int cK[27], cM[27];
  const int cnt = gen_stencil(dim, n, v, col, cK, cM);
  int k = 0;
  for (int j = 0; j < cnt; ++j)
    if (!gen_bc(dim, n, col[j])) { col[k] = col[j]; cK[k] = cK[j]; cM[k] = cM[j]; ++k; }
  for (int j = 0; j < k; ++j) {
    const double fK = (double)cK[j], fM = (double)cM[j];
    const double a11 = kf1 * fK + mf * fM, a22 = kf2 * fK + mf * fM, a12 = -(mf * fM);
    colind[p1 + j] = (int32_t)col[j];
    values[p1 + j] = a11;
    colind[p1 + k + j] = (int32_t)(col[j] + nv);
    values[p1 + k + j] = a12;
    colind[p2 + j] = (int32_t)col[j];
    values[p2 + j] = a12;
    colind[p2 + k + j] = (int32_t)(col[j] + nv);
    values[p2 + k + j] = a22;
  }
}

}  // namespace

int gen_bidomain_dev(int dim, int64_t n, double gamma, double k1, double k2, int64_t nnz, int64_t* ptr,
                     int32_t* colind, double* values, std::string* err) {
  if ((dim != 2 && dim != 3) || n < 1) { *err = "gen_bidomain_device: dim must be 2 or 3 and n >= 1"; return MAMG_ERR_ARG; }
  const int64_t nn = n + 1, nv = dim == 3 ? nn * nn * nn : nn * nn;
  if (2 * nv >= (int64_t)INT32_MAX) { *err = "gen_bidomain_device: too many rows for int32 columns"; return MAMG_ERR_ARG; }
  // the host generator's factors (gen.cpp gen_bidomain), computed on the host
  const double h = 1.0 / (double)n;
  double kf1, kf2, mf;
  if (dim == 3) {
    kf1 = k1 * h / 6.0;
    kf2 = k2 * h / 6.0;
    mf = gamma * h * h * h / 120.0;
  } else {
    kf1 = k1 / 2.0;
    kf2 = k2 / 2.0;
    mf = gamma * h * h / 24.0;
  }
  Scratch S;
  int64_t* len = nullptr;
  RCHK(S.alloc(&len, nv, err));
  gen_len_kernel<<<nblk(nv), 256>>>(dim, n, nv, len);
  HIPCHK(hipGetLastError());
  RCHK(dscan_incl_i64(len, len, nv, nullptr, err));
  int64_t half = 0;
  RCHK(to_host(&half, len + nv - 1, 1, err));
  if (2 * half != nnz) {
    *err = "gen_bidomain_device: nnz " + std::to_string(nnz) + " != the generator's " + std::to_string(2 * half);
    return MAMG_ERR_ARG;
  }
  gen_ptr_kernel<<<nblk(nv + 1), 256>>>(nv, len, ptr);
  gen_fill_kernel<<<nblk(nv), 256>>>(dim, n, nv, kf1, kf2, mf, ptr, colind, values);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(nullptr));
  return MAMG_OK;
}

int upload_a0(const CsrView& A, GHier* G, DevMat* D, std::string* err) {
  HIPCHK(hipSetDevice(G->device));
  ModuleWarm warm(G->device);
  Clock clk;
  D->n = A.n;
  D->m = A.m;
  D->nnz = A.nnz();
  RCHK(galloc(G, &D->ptr, A.n + 1, err));
  RCHK(galloc(G, &D->col, D->nnz, err));
  RCHK(galloc(G, &D->val, D->nnz, err));
  // the three arrays cut into k pieces each, copied by k host threads on
  // streams of their own: a pageable copy stages through the runtime's
  // pinned buffers on the calling thread, ~36 GB/s for one thread.  A/B at
  // nrefs=6 (MAMG_UPLOAD_THREADS, profiles/r05_upload_threads.txt): k = 1
  // 348-397 ms, 2 323 ms (default), 4 335 ms
  const char* e = opt("MAMG_UPLOAD_THREADS");
  const int k = e ? std::max(1, std::min(16, std::atoi(e))) : 2;
  if (k == 1) {
    HIPCHK(hipMemcpy(D->ptr, A.ptr, (A.n + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
    if (D->nnz) {
      HIPCHK(hipMemcpy(D->col, A.col, D->nnz * sizeof(int32_t), hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(D->val, A.val, D->nnz * sizeof(double), hipMemcpyHostToDevice));
    }
  } else {
    struct Piece { void* d; const void* h; size_t b; };
    std::vector<Piece> pieces;
    auto cut = [&](void* d, const void* h, size_t b) {
      const size_t q = (b + k - 1) / k;
      for (size_t o = 0; o < b; o += q) pieces.push_back({(char*)d + o, (const char*)h + o, std::min(q, b - o)});
    };
    cut(D->ptr, A.ptr, (A.n + 1) * sizeof(int64_t));
    if (D->nnz) {
      cut(D->col, A.col, D->nnz * sizeof(int32_t));
      cut(D->val, A.val, D->nnz * sizeof(double));
    }
    // the three arrays may be cached blocks whose earlier users (a handle
    // just closed, a previous setup) are still queued on the null stream;
    // the upload streams are non-blocking, so they wait for it here
    HIPCHK(hipStreamSynchronize(nullptr));
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    const int dev = G->device;
    for (int t = 0; t < k; ++t)
      th.emplace_back([&, t] {
        if (hipSetDevice(dev) != hipSuccess) { bad = 1; return; }
        hipStream_t st = nullptr;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) { bad = 1; return; }
        for (size_t i = t; i < pieces.size(); i += k)
          if (hipMemcpyAsync(pieces[i].d, pieces[i].h, pieces[i].b, hipMemcpyHostToDevice, st) != hipSuccess) bad = 1;
        if (hipStreamSynchronize(st) != hipSuccess) bad = 1;
        (void)hipStreamDestroy(st);
      });
    for (auto& x : th) x.join();
    if (bad) { *err = "A0 upload: " + std::string(hipGetErrorString(hipGetLastError())); return MAMG_ERR_HIP; }
  }
  G->phase_ms[GS_UPLOAD] = clk.lap();
  return MAMG_OK;
}

// ---------------------------------------------------------------------------
// Row-sharded Galerkin product on virtual ranks: the start of a
// partition-local setup.  Rank p owns the
// fine nodes [p nv / P, (p + 1) nv / P) (both fields' rows) and the coarse
// nodes [p nc / P, (p + 1) nc / P).  It computes
//   (A P) rows of its fine dofs  = A_p x P_ext,  P_ext = P's rows of the fine
//       dofs A_p's columns reach (its own and a halo); every other row empty;
//   A_c rows of its coarse dofs  = R_p x AP_ext, R_p = R = P^T's rows of its
//       coarse dofs, AP_ext = the (A P) rows of the fine dofs R_p reaches,
//       each taken from its OWNER's sharded result above (the exchange a
//       multi-GPU setup makes); every other row empty;
// with the setup's own SpGEMM (staged, node row pairs).  A row missing from a
// halo leaves a product incomplete, so the check is also that the halos are
// the right ones.  Each row is compared bit for bit: the (A P) rows with the
// unsharded product, the A_c rows with Ac (the hierarchy's next level).
// res[6]: (A P) rows that differ, A_c rows that differ, halo P rows read,
// halo (A P) rows read (summed over ranks), (A P) rows, A_c rows compared.
// Host-side row selection (a verification path, not a setup).
// ---------------------------------------------------------------------------
namespace {
int up_csr(GHier* G, const Csr& h, DevMat* d, std::string* err) {
  d->n = h.n; d->m = h.m; d->nnz = h.n ? h.ptr[h.n] : 0;
  RCHK(galloc(G, &d->ptr, d->n + 1, err));
  RCHK(galloc(G, &d->col, std::max<int64_t>(d->nnz, 1), err));
  RCHK(galloc(G, &d->val, std::max<int64_t>(d->nnz, 1), err));
  HIPCHK(hipMemcpy(d->ptr, h.ptr.data(), (d->n + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if (d->nnz) {
    HIPCHK(hipMemcpy(d->col, h.col.data(), d->nnz * sizeof(int32_t), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d->val, h.val.data(), d->nnz * sizeof(double), hipMemcpyHostToDevice));
  }
  return MAMG_OK;
}
int down_csr(const DevMat& d, Csr* h, std::string* err) {
  h->n = d.n; h->m = d.m;
  h->ptr.resize(d.n + 1);
  RCHK(to_host(h->ptr.data(), d.ptr, d.n + 1, err));
  const int64_t nnz = h->ptr[d.n];
  h->col.resize(nnz);
  h->val.resize(nnz);
  if (nnz) {
    RCHK(to_host(h->col.data(), d.col, nnz, err));
    RCHK(to_host(h->val.data(), d.val, nnz, err));
  }
  return MAMG_OK;
}
Csr view_csr(const CsrView& v) {
  Csr c;
  c.n = v.n; c.m = v.m;
  const int64_t nnz = v.nnz();
  c.ptr.assign(v.ptr, v.ptr + v.n + 1);
  c.col.assign(v.col, v.col + nnz);
  c.val.assign(v.val, v.val + nnz);
  return c;
}
// rows `rows` of M, in that order
Csr pick_rows(const Csr& M, const std::vector<int64_t>& rows) {
  Csr o;
  o.n = (int64_t)rows.size(); o.m = M.m;
  o.ptr.assign(1, 0);
  for (int64_t r : rows) {
    o.col.insert(o.col.end(), M.col.begin() + M.ptr[r], M.col.begin() + M.ptr[r + 1]);
    o.val.insert(o.val.end(), M.val.begin() + M.ptr[r], M.val.begin() + M.ptr[r + 1]);
    o.ptr.push_back((int64_t)o.col.size());
  }
  return o;
}
bool row_equal(const Csr& X, int64_t i, const Csr& Y, int64_t j) {
  const int64_t a = X.ptr[i], l = X.ptr[i + 1] - a, b = Y.ptr[j];
  if (Y.ptr[j + 1] - b != l) return false;
  return std::memcmp(&X.col[a], &Y.col[b], l * sizeof(int32_t)) == 0 &&
         std::memcmp(&X.val[a], &Y.val[b], l * sizeof(double)) == 0;
}
// the field-major rows of node range [lo, hi) of a 2-function matrix of h nodes per field
std::vector<int64_t> node_rows(int64_t lo, int64_t hi, int64_t h) {
  std::vector<int64_t> r;
  for (int f = 0; f < 2; ++f)
    for (int64_t I = lo; I < hi; ++I) r.push_back(f * h + I);
  return r;
}
}  // namespace

int sharded_galerkin_check(const CsrView& Av, const CsrView& Pv, const CsrView& Acv, int nranks, int device,
                           int64_t res[6], std::string* err) {
  for (int k = 0; k < 6; ++k) res[k] = 0;
  if (nranks < 1 || Av.n != Av.m || Av.n % 2 || Pv.n != Av.n || Pv.m % 2 || Acv.n != Pv.m || Acv.m != Pv.m) {
    *err = "sharded Galerkin check: A (2 nv x 2 nv), P (2 nv x 2 nc) and A_c (2 nc x 2 nc), field-major, nranks >= 1";
    return MAMG_ERR_ARG;
  }
  HIPCHK(hipSetDevice(device));
  GHier G;
  G.device = device;
  const int64_t n = Av.n, nv = n / 2, m = Pv.m, nc = m / 2;
  const Csr A = view_csr(Av), P = view_csr(Pv), Ac = view_csr(Acv);
  DevMat dA, dP, dR, dAP;
  RCHK(up_csr(&G, A, &dA, err));
  RCHK(up_csr(&G, P, &dP, err));
  RCHK(transpose(&G, dP, &dR, err));
  const double blenP = (double)dP.nnz / (double)std::max<int64_t>(1, dP.n);
  RCHK(spgemm(&G, dA, BCsr{dP.ptr, dP.col, dP.val}, m, &dAP, err, blenP, true));
  Csr R, AP;
  RCHK(down_csr(dR, &R, err));
  RCHK(down_csr(dAP, &AP, err));
  const double blenAP = (double)dAP.nnz / (double)std::max<int64_t>(1, dAP.n);
  auto fine0 = [&](int p) { return (int64_t)p * nv / nranks; };
  auto coarse0 = [&](int p) { return (int64_t)p * nc / nranks; };
  std::vector<Csr> APp(nranks);
  for (int p = 0; p < nranks; ++p) {   // (A P) rows of rank p's fine dofs
    const int64_t o0 = fine0(p), o1 = fine0(p + 1);
    const std::vector<int64_t> rows = node_rows(o0, o1, nv);
    const Csr Ap = pick_rows(A, rows);
    std::vector<char> need(n, 0);
    for (int32_t c : Ap.col) need[c] = 1;
    Csr Pext;
    Pext.n = n; Pext.m = m;
    Pext.ptr.assign(1, 0);
    for (int64_t i = 0; i < n; ++i) {
      if (need[i]) {
        Pext.col.insert(Pext.col.end(), P.col.begin() + P.ptr[i], P.col.begin() + P.ptr[i + 1]);
        Pext.val.insert(Pext.val.end(), P.val.begin() + P.ptr[i], P.val.begin() + P.ptr[i + 1]);
        const int64_t I = i % nv;
        res[2] += !(I >= o0 && I < o1);
      }
      Pext.ptr.push_back((int64_t)Pext.col.size());
    }
    GHier T;
    T.device = device;
    DevMat dAp, dPe, dC;
    RCHK(up_csr(&T, Ap, &dAp, err));
    RCHK(up_csr(&T, Pext, &dPe, err));
    RCHK(spgemm(&T, dAp, BCsr{dPe.ptr, dPe.col, dPe.val}, m, &dC, err, blenP, true));
    RCHK(down_csr(dC, &APp[p], err));
    for (int64_t r = 0; r < (int64_t)rows.size(); ++r) {
      res[0] += !row_equal(APp[p], r, AP, rows[r]);
      ++res[4];
    }
  }
  auto owner = [&](int64_t I) {   // rank of fine node I
    int p = (int)std::min<int64_t>(nranks - 1, I * nranks / std::max<int64_t>(nv, 1));
    while (p > 0 && I < fine0(p)) --p;
    while (p < nranks - 1 && I >= fine0(p + 1)) ++p;
    return p;
  };
  for (int p = 0; p < nranks; ++p) {   // A_c rows of rank p's coarse dofs
    const int64_t c0 = coarse0(p), c1 = coarse0(p + 1);
    const std::vector<int64_t> rows = node_rows(c0, c1, nc);
    const Csr Rp = pick_rows(R, rows);
    std::vector<char> need(n, 0);
    for (int32_t c : Rp.col) need[c] = 1;
    Csr APe;
    APe.n = n; APe.m = m;
    APe.ptr.assign(1, 0);
    const int64_t f0 = fine0(p), f1 = fine0(p + 1);
    for (int64_t i = 0; i < n; ++i) {
      if (need[i]) {           // the owner's row (fine dof i = f nv + I is row f (o1 - o0) + I - o0 there)
        const int64_t I = i % nv, f = i / nv;
        const int q = owner(I);
        const int64_t lq = f * (fine0(q + 1) - fine0(q)) + (I - fine0(q));
        const Csr& S = APp[q];
        APe.col.insert(APe.col.end(), S.col.begin() + S.ptr[lq], S.col.begin() + S.ptr[lq + 1]);
        APe.val.insert(APe.val.end(), S.val.begin() + S.ptr[lq], S.val.begin() + S.ptr[lq + 1]);
        res[3] += !(I >= f0 && I < f1);
      }
      APe.ptr.push_back((int64_t)APe.col.size());
    }
    GHier T;
    T.device = device;
    DevMat dRp, dAPe, dC;
    Csr Cp;
    RCHK(up_csr(&T, Rp, &dRp, err));
    RCHK(up_csr(&T, APe, &dAPe, err));
    RCHK(spgemm(&T, dRp, BCsr{dAPe.ptr, dAPe.col, dAPe.val}, m, &dC, err, blenAP, true));
    RCHK(down_csr(dC, &Cp, err));
    for (int64_t r = 0; r < (int64_t)rows.size(); ++r) {
      res[1] += !row_equal(Cp, r, Ac, rows[r]);
      ++res[5];
    }
  }
  return MAMG_OK;
}

int ghier_download(const GHier& G, const CsrView& A0, Hierarchy* H, std::string* err) {
  H->params = G.params;
  H->A0 = A0;
  H->levels.clear();
  H->seeds = G.seeds;
  auto dl = [&](const DevMat& M, Csr* C) -> int {
    C->n = M.n;
    C->m = M.m;
    C->ptr.resize(M.n + 1);
    C->col.resize(M.nnz);
    C->val.resize(M.nnz);
    RCHK(to_host(C->ptr.data(), M.ptr, M.n + 1, err));
    RCHK(to_host(C->col.data(), M.col, M.nnz, err));
    RCHK(to_host(C->val.data(), M.val, M.nnz, err));
    return MAMG_OK;
  };
  for (size_t l = 0; l < G.levels.size(); ++l) {
    const GLevel& g = G.levels[l];
    H->levels.emplace_back();
    HostLevel& h = H->levels.back();
    h.n = g.n;
    h.coarsest = g.coarsest;
    if (l > 0) RCHK(dl(g.A, &h.A));
    if (g.coarsest) {
      h.Ainv.resize(g.n * g.n);
      RCHK(to_host(h.Ainv.data(), g.Ainv, g.n * g.n, err));
      break;
    }
    const int64_t nv = g.n / G.params.num_functions;
    RCHK(dl(g.P, &h.P));
    RCHK(dl(g.R, &h.R));
    if (g.AP.n) RCHK(dl(g.AP, &h.AP));
    h.agg.resize(nv);
    RCHK(to_host(h.agg.data(), g.agg, nv, err));
    h.nagg = g.nagg;
    h.w_sa = g.w_sa;
    if (g.WB.n) {                   // general block smoother
      RCHK(dl(g.WB, &h.WB));
      continue;
    }
    if (g.winv) {                   // point smoother
      h.winv.resize(g.n);
      RCHK(to_host(h.winv.data(), g.winv, g.n, err));
      continue;
    }
    // smoother as the host's block CSR: node blocks {I, nv + I} (2 entries per
    // row), or singletons where level-0 seed blocks split a node
    std::vector<double> W(4 * nv);
    std::vector<uint8_t> jn(nv, 1);
    RCHK(to_host(W.data(), g.W, 4 * nv, err));
    if (g.joined) RCHK(to_host(jn.data(), g.joined, nv, err));
    Csr& B = h.WB;
    B.n = B.m = g.n;
    B.ptr.assign(g.n + 1, 0);
    for (int64_t i = 0; i < g.n; ++i) B.ptr[i + 1] = B.ptr[i] + (jn[i % nv] ? 2 : 1);
    B.col.resize(B.ptr[g.n]);
    B.val.resize(B.ptr[g.n]);
    for (int64_t i = 0; i < g.n; ++i) {
      const int64_t I = i % nv, f = i / nv;
      int64_t o = B.ptr[i];
      if (jn[I]) {
        B.col[o] = (int32_t)I; B.val[o] = W[4 * I + 2 * f];
        B.col[o + 1] = (int32_t)(nv + I); B.val[o + 1] = W[4 * I + 2 * f + 1];
      } else {
        B.col[o] = (int32_t)i; B.val[o] = W[4 * I + 3 * f];
      }
    }
  }
  return MAMG_OK;
}

namespace {

// ghost marks of one field-major matrix for every rank: row i (node I = i mod
// nr) belongs to the rank q whose range rown[q..q+1) holds I; a column node
// J = col mod nc outside coln[q..q+1) is a ghost of q: mark[q nc + J] = 1
// (dist.cpp external_node_cols, all ranks in one pass)
__global__ void ghost_mark_kernel(const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
                                  int64_t n, int64_t nr, int64_t nc, const int64_t* __restrict__ rown,
                                  const int64_t* __restrict__ coln, int nranks,
                                  uint8_t* __restrict__ mark) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t I = i % nr;
  int lo = 0, hi = nranks - 1;   // last q with rown[q] <= I (empty ranges skipped)
  while (lo < hi) {
    const int mid = (lo + hi + 1) / 2;
    if (rown[mid] <= I) lo = mid;
    else hi = mid - 1;
  }
  const int64_t c0 = coln[lo], c1 = coln[lo + 1];
  uint8_t* m = mark + (int64_t)lo * nc;
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) {
    const int64_t J = col[k] % nc;
    if (J < c0 || J >= c1) m[J] = 1;
  }
}

// one more hop of every rank's ghost region (node patches on N GPUs need the
// 3-hop ball): a ghost I of rank q (min[q nc + I] set) marks its row's
// columns outside q's range in mout (a copy of min beforehand)
__global__ void ghost_expand_kernel(const int64_t* __restrict__ ptr, const int32_t* __restrict__ col, int64_t n,
                                    int64_t nc, const int64_t* __restrict__ coln, int nranks,
                                    const uint8_t* __restrict__ min, uint8_t* __restrict__ mout) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t I = i % nc;
  for (int q = 0; q < nranks; ++q) {
    if (!min[(int64_t)q * nc + I]) continue;
    const int64_t c0 = coln[q], c1 = coln[q + 1];
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) {
      const int64_t J = col[k] % nc;
      if (J < c0 || J >= c1) mout[(int64_t)q * nc + J] = 1;
    }
  }
}

struct DevScratch {             // a null-stream ordered temporary (dmem.h), freed on scope exit
  void* p = nullptr;
  ~DevScratch() { tmp_free(p); }
};

}  // namespace

int ghier_download_rank(const GHier& G, const DevMat& A0d, const CsrView& A0, int rank, int nranks,
                        int64_t rep_nodes, bool post_fusion, Hierarchy* H, GhostLists* ghosts,
                        std::string* err, bool matrices, int hops0) {
  if (nranks < 1 || rank < 0 || rank >= nranks) { *err = "bad rank/nranks"; return MAMG_ERR_ARG; }
  if (G.generic) { *err = "rank download of a hierarchy without node-block smoothers"; return MAMG_ERR_UNSUPPORTED; }
  H->params = G.params;
  H->A0 = A0;
  H->levels.clear();
  int nl = 0;
  while (nl < (int)G.levels.size())
    if (G.levels[nl++].coarsest) break;
  // same ranges, replication and fusion decision as build_dist_plan
  std::vector<int64_t> nv(nl);
  std::vector<char> co(nl), rep;
  std::vector<std::vector<int64_t>> own;
  for (int l = 0; l < nl; ++l) { nv[l] = G.levels[l].n / 2; co[l] = G.levels[l].coarsest; }
  dist_ranges(nv, co, nranks, rep_nodes, &own, &rep);
  bool fuse = post_fusion;
  for (int l = 0; l + 1 < nl && fuse; ++l)
    if (G.levels[l].AP.n != G.levels[l].n) fuse = false;

  // full download of a matrix, or of the node rows [r0, r1) of both fields
  // (other rows empty: build_dist_plan reads no others)
  auto dl = [&](const DevMat& M, bool all, int64_t r0, int64_t r1, Csr* C) -> int {
    C->n = M.n;
    C->m = M.m;
    if (all) {
      C->ptr.resize(M.n + 1);
      C->col.resize(M.nnz);
      C->val.resize(M.nnz);
      RCHK(to_host(C->ptr.data(), M.ptr, M.n + 1, err));
      RCHK(to_host(C->col.data(), M.col, M.nnz, err));
      RCHK(to_host(C->val.data(), M.val, M.nnz, err));
      return MAMG_OK;
    }
    const int64_t nr = M.n / 2, w = r1 - r0;
    std::vector<int64_t> p0(w + 1), p1(w + 1);
    RCHK(to_host(p0.data(), M.ptr + r0, w + 1, err));
    RCHK(to_host(p1.data(), M.ptr + nr + r0, w + 1, err));
    const int64_t n0 = p0[w] - p0[0], n1 = p1[w] - p1[0];
    C->col.resize(n0 + n1);
    C->val.resize(n0 + n1);
    RCHK(to_host(C->col.data(), M.col + p0[0], n0, err));
    RCHK(to_host(C->val.data(), M.val + p0[0], n0, err));
    RCHK(to_host(C->col.data() + n0, M.col + p1[0], n1, err));
    RCHK(to_host(C->val.data() + n0, M.val + p1[0], n1, err));
    C->ptr.resize(M.n + 1);
    std::fill(C->ptr.begin(), C->ptr.begin() + r0, 0);
    for (int64_t t = 0; t <= w; ++t) C->ptr[r0 + t] = p0[t] - p0[0];
    std::fill(C->ptr.begin() + r1, C->ptr.begin() + nr + r0, n0);
    for (int64_t t = 0; t <= w; ++t) C->ptr[nr + r0 + t] = n0 + p1[t] - p1[0];
    std::fill(C->ptr.begin() + nr + r1, C->ptr.end(), n0 + n1);
    return MAMG_OK;
  };

  // ghost lists: the own rank's whole list, the others' inside the own range
  ghosts->assign(nl, std::vector<std::vector<int64_t>>(nranks));
  int64_t mark_bytes = 0;
  for (int l = 0; l < nl; ++l)
    if (!rep[l]) mark_bytes = std::max<int64_t>(mark_bytes, (int64_t)nranks * nv[l]);
  if (mark_bytes) {
    DevScratch rng, mk, mk2;
    HIPCHK(tmp_malloc(&rng.p, (size_t)nl * (nranks + 1) * sizeof(int64_t)));
    HIPCHK(tmp_malloc(&mk.p, (size_t)mark_bytes));
    if (hops0 > 1) HIPCHK(tmp_malloc(&mk2.p, (size_t)nranks * nv[0]));
    int64_t* drng = (int64_t*)rng.p;
    uint8_t* mark = (uint8_t*)mk.p;
    for (int l = 0; l < nl; ++l)
      HIPCHK(hipMemcpy(drng + (size_t)l * (nranks + 1), own[l].data(), (nranks + 1) * sizeof(int64_t),
                       hipMemcpyHostToDevice));
    std::vector<uint8_t> hm;
    for (int l = 0; l < nl; ++l) {
      if (rep[l]) continue;
      HIPCHK(dev_memset(mark, 0, (size_t)nranks * nv[l]));
      auto marks = [&](const DevMat& M, int rl) {
        if (M.n == 0) return;
        ghost_mark_kernel<<<nblk(M.n), 256>>>(M.ptr, M.col, M.n, nv[rl], nv[l], drng + (size_t)rl * (nranks + 1),
                                              drng + (size_t)l * (nranks + 1), nranks, mark);
      };
      marks(l == 0 ? A0d : G.levels[l].A, l);
      for (int hop = 1; l == 0 && hop < hops0; ++hop) {   // the ghost ball grown hop by hop
        uint8_t* m2 = (uint8_t*)mk2.p;
        HIPCHK(dev_copy(m2, mark, (size_t)nranks * nv[0]));
        ghost_expand_kernel<<<nblk(A0d.n), 256>>>(A0d.ptr, A0d.col, A0d.n, nv[0], drng, nranks, mark, m2);
        HIPCHK(dev_copy(mark, m2, (size_t)nranks * nv[0]));
      }
      if (l > 0) {
        marks(G.levels[l - 1].P, l - 1);
        if (fuse) marks(G.levels[l - 1].AP, l - 1);
      }
      HIPCHK(hipGetLastError());
      const int64_t o0 = own[l][rank], o1 = own[l][rank + 1];
      for (int q = 0; q < nranks; ++q) {
        const int64_t a = q == rank ? 0 : o0, b = q == rank ? nv[l] : o1;
        hm.resize(b - a);
        RCHK(to_host(hm.data(), mark + (size_t)q * nv[l] + a, b - a, err));
        std::vector<int64_t>& g = (*ghosts)[l][q];
        for (int64_t t = 0; t < b - a; ++t)
          if (hm[t]) g.push_back(a + t);
      }
    }
  }

  for (int l = 0; l < nl; ++l) {
    const GLevel& g = G.levels[l];
    H->levels.emplace_back();
    HostLevel& h = H->levels.back();
    h.n = g.n;
    h.coarsest = g.coarsest;
    const bool all = rep[l];
    const int64_t o0 = own[l][rank], o1 = own[l][rank + 1];
    if (l > 0 && matrices) RCHK(dl(g.A, all, o0, o1, &h.A));
    if (g.coarsest) {
      h.Ainv.resize(g.n * g.n);
      RCHK(to_host(h.Ainv.data(), g.Ainv, g.n * g.n, err));
      break;
    }
    if (!matrices) continue;
    RCHK(dl(g.P, all, o0, o1, &h.P));
    if (fuse) RCHK(dl(g.AP, all, o0, o1, &h.AP));
    h.nagg = g.nagg;
    h.w_sa = g.w_sa;
    // node blocks of the owned nodes (ghier_download's WB: a node split by
    // seed blocks keeps its two diagonal entries only)
    const int64_t w0 = all ? 0 : o0, w1 = all ? nv[l] : o1;
    h.wn0 = w0;
    h.Wn.resize(4 * (w1 - w0));
    RCHK(to_host(h.Wn.data(), g.W + 4 * w0, 4 * (w1 - w0), err));
    if (g.joined) {
      std::vector<uint8_t> jn(w1 - w0);
      RCHK(to_host(jn.data(), g.joined + w0, w1 - w0, err));
      for (int64_t t = 0; t < w1 - w0; ++t)
        if (!jn[t]) h.Wn[4 * t + 1] = h.Wn[4 * t + 2] = 0.0;
    }
  }
  return MAMG_OK;
}

}  // namespace mamg
