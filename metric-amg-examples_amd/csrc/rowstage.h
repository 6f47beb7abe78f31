// rowstage.h -- LDS staging of a wave's node rows for the setup/layout merges.
//
// The node-wise merges of the field-major CSR (node graph, block rho, CSR ->
// BSR2) give each lane one node I and walk rows I and nr + I sequentially, in
// column order (their sums must keep that order to stay bitwise equal to the
// host setup).  Read straight from HBM, the 64 lanes of a load instruction
// touch 64 different rows: every instruction splits into ~64 cache-line
// requests and the merges ran at ~0.1 TB/s.  Here the wave first copies the
// contiguous entry ranges of its 64 nodes' rows -- ptr[I0] .. ptr[I0 + 64] of
// field 0 and the same of field 1 -- into LDS with coalesced loads, then each
// lane merges from LDS in the same order as before.  Ranges longer than CAP
// are read from global memory exactly as before.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mamg {

constexpr int RS_NODES = 64;     // nodes per wave (= workgroup)
constexpr int RS_CAP = 2048;     // staged entries per field (A0: ~1900)
constexpr int RS_CAP_LONG = 8192; // level-1 rows: ~83 entries, ~5.3 K per field and wave
constexpr int RS_BATCH = 8;      // loads per lane in flight while staging

// VALS false (the count passes): columns only, 16 KB instead of 48 KB of LDS
// per workgroup, so 3 -> 10 waves per CU
// CAP: entries per field (RS_CAP; RS_CAP_LONG for the coarse Galerkin rows'
// column-only passes, 64 KB)
template <bool VALS, int CAP = RS_CAP>
struct RowStageT {
  int32_t c[2][CAP];
  double v[2][VALS ? CAP : 1];
};
using RowStage = RowStageT<true>;

// Row view of one field: entry k of the field's rows is LC[k - off],
// LV[k - off] in the staged LDS copy (lds), else C[k], V[k] in global memory.
// The two address spaces are explicit: the reads are ds_read / global_load,
// never FLAT loads (round 4: with one generic pointer for both, the FLAT
// loads of staged values intermittently returned zeros for a lane's whole
// row -- csr2bsr_kernel's 2x2 blocks of A P came out zero, and with them
// the level-0 K = P - W A P)
#define RS_AS1 __attribute__((address_space(1)))
#define RS_AS3 __attribute__((address_space(3)))
struct RowView {
  const int32_t* C;
  const double* V;
  const RS_AS3 int32_t* LC;
  const RS_AS3 double* LV;
  int64_t off;
  bool lds;
  __device__ __forceinline__ int32_t col(int64_t k) const {
    return lds ? LC[k - off] : *(const RS_AS1 int32_t*)(C + k);
  }
  __device__ __forceinline__ double val(int64_t k) const {
    return lds ? LV[k - off] : *(const RS_AS1 double*)(V + k);
  }
};

// Stage the rows of nodes [I0, I0 + RS_NODES) (clipped to nr) of both fields;
// fills view[2] (LDS when the ranges fit, else global).  Every lane of the
// wave must call it (the loads and the barrier are wave-wide).
template <bool VALS, int CAP>
__device__ __forceinline__ void stage_rows(RowStageT<VALS, CAP>& S, const int64_t* __restrict__ ptr,
                                           const int32_t* __restrict__ col, const double* __restrict__ val,
                                           int64_t nr, int64_t I0, RowView* view) {
  const int lane = threadIdx.x & 63;
  const int64_t I1 = I0 + RS_NODES < nr ? I0 + RS_NODES : nr;
  int64_t b[2], n[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    b[f] = ptr[f * nr + I0];
    n[f] = ptr[f * nr + I1] - b[f];
  }
  const bool fits = n[0] <= CAP && n[1] <= CAP;
  if (fits) {
    // RS_BATCH loads in flight per lane before their LDS writes: one load per
    // iteration waited out an HBM latency each time, and at 3 waves per CU
    // (48 KB each) the copy, not the merge, set the kernels' time
#pragma unroll
    for (int f = 0; f < 2; ++f)
      for (int64_t t0 = 0; t0 < n[f]; t0 += 64 * RS_BATCH) {
        int32_t cc[RS_BATCH];
        double vv[RS_BATCH];
#pragma unroll
        for (int u = 0; u < RS_BATCH; ++u) {
          const int64_t t = t0 + u * 64 + lane;
          if (t < n[f]) {
            cc[u] = col[b[f] + t];
            if (VALS) vv[u] = val[b[f] + t];
          }
        }
#pragma unroll
        for (int u = 0; u < RS_BATCH; ++u) {
          const int64_t t = t0 + u * 64 + lane;
          if (t < n[f]) {
            S.c[f][t] = cc[u];
            if (VALS) S.v[f][t] = vv[u];
          }
        }
      }
    __syncthreads();
#pragma unroll
    for (int f = 0; f < 2; ++f)
      view[f] = RowView{col, val, (const RS_AS3 int32_t*)S.c[f], (const RS_AS3 double*)S.v[f], b[f], true};
  } else {
#pragma unroll
    for (int f = 0; f < 2; ++f) view[f] = RowView{col, val, nullptr, nullptr, 0, false};
  }
}

// dst[slot[t]] = val[b + t] for t < n (the two-phase fills' value sweep, slot
// in LDS), RS_BATCH coalesced loads in flight per lane
__device__ __forceinline__ void scatter_staged(const int32_t* slot, const double* __restrict__ val, int64_t b,
                                               int64_t n, double* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  for (int64_t t0 = 0; t0 < n; t0 += 64 * RS_BATCH) {
    double vv[RS_BATCH];
#pragma unroll
    for (int u = 0; u < RS_BATCH; ++u) {
      const int64_t t = t0 + u * 64 + lane;
      if (t < n) vv[u] = val[b + t];
    }
#pragma unroll
    for (int u = 0; u < RS_BATCH; ++u) {
      const int64_t t = t0 + u * 64 + lane;
      if (t < n) dst[slot[t]] = vv[u];
    }
  }
}

// node I's four sorted column segments (q = 2 f + g: the entries of row
// f nr + I whose column lies in field g, node column = col - g nc)
__device__ __forceinline__ void stage_segs(const int64_t* __restrict__ ptr, const RowView* view, int64_t nr,
                                           int64_t nc, int64_t I, int64_t* k, int64_t* e) {
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int64_t a = ptr[f * nr + I], b = ptr[f * nr + I + 1];
    int64_t lo = a, hi = b;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (view[f].col(mid) < nc) lo = mid + 1; else hi = mid;
    }
    k[2 * f] = a; e[2 * f] = lo; k[2 * f + 1] = lo; e[2 * f + 1] = b;
  }
}

// Merge cursor over node I's four sorted segments (stage_segs): c[q] is the
// node column at segment q's head (INT64_MAX when exhausted).  Each column
// is read once, when its segment advances: the next node column is
// min(c), and the segments holding it are those with c[q] == J.
struct Seg4 {
  int64_t k[4], e[4], c[4];
  __device__ __forceinline__ void head(const RowView* vw, int64_t nc, int q) {
    c[q] = k[q] < e[q] ? (int64_t)vw[q >> 1].col(k[q]) - (q & 1) * nc : INT64_MAX;
  }
  __device__ __forceinline__ void init(const RowView* vw, int64_t nc) {
#pragma unroll
    for (int q = 0; q < 4; ++q) head(vw, nc, q);
  }
  __device__ __forceinline__ int64_t next() const {
    const int64_t a = c[0] < c[1] ? c[0] : c[1], b = c[2] < c[3] ? c[2] : c[3];
    return a < b ? a : b;
  }
};

}  // namespace mamg
