// setup.cpp -- host construction of the smoothed-aggregation hierarchy.
//
// Replaces the HAZmath metric-AMG setup behind
//   metricAMG(A, W, idofs=interface_dofs, parameters=...)  src/utils.py:86
// with the deterministic, GPU-parallel profile of DESIGN.md section 2:
//   strength of connection (theta = strong_coupled, src/amg_parameters.py:80)
//   -> round-synchronous MIS-2 aggregation with hash priorities
//   -> tentative P (unit entries) -> SA Jacobi smoothing (omega = 4/3 / rho)
//   -> Galerkin R A P with R = P^T
//   -> point smoother weights / seed-block (Schwarz) inverses on level 0
//      (seeds = idofs, src/utils.py:84-86, src/bidomain_3d.py:138)
//   -> dense inverse on the coarsest level (coarse_solver 32, :77).
//
// Every floating-point quantity is computed in exactly the operation order of
// oracle/mamg_oracle.py (sequential CSR-order sums from 0.0, SMMP SpGEMM order,
// exact-zero dropping, no FMA: this file is compiled with -ffp-contract=off),
// so the hierarchy is bitwise identical to the oracle's.  Loops over rows are
// OpenMP-parallel; each row is computed sequentially, so results do not
// depend on the thread count.
#include <omp.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>

#include "host.h"

namespace mamg {
namespace {

constexpr uint64_t ST_OUT = 0, ST_UND = 1, ST_IN = 2;

inline double diag_of(const CsrView& A, int64_t i) {
  const int32_t* b = A.col + A.ptr[i];
  const int32_t* e = A.col + A.ptr[i + 1];
  const int32_t* p = std::lower_bound(b, e, (int32_t)i);
  return (p != e && *p == i) ? A.val[p - A.col] : 0.0;
}

inline int64_t find_pos(const CsrView& A, int64_t i, int64_t j) {
  const int32_t* b = A.col + A.ptr[i];
  const int32_t* e = A.col + A.ptr[i + 1];
  const int32_t* p = std::lower_bound(b, e, (int32_t)j);
  return (p != e && *p == j) ? (int64_t)(p - A.col) : -1;
}

// sequential (CSR-order) sum of |a_ij| per row  (scipy csr_matvec of |A|@1)
std::vector<double> abs_rowsum(const CsrView& A) {
  std::vector<double> rs(A.n);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < A.n; ++i) {
    double s = 0.0;
    for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) s += std::fabs(A.val[k]) * 1.0;
    rs[i] = s;
  }
  return rs;
}

// ---------------------------------------------------------------------------
// SpGEMM in scipy SMMP order: for row i, for each A_ik (stored order), for each
// B_kj (stored order): sums[j] += A_ik * B_kj.  Exact zeros dropped, columns
// sorted.  Rows are independent -> parallel over row chunks.
// ---------------------------------------------------------------------------
struct Chunk {
  std::vector<int32_t> col;
  std::vector<double> val;
};

void spgemm(const CsrView& A, const CsrView& B, Csr* C) {
  const int64_t n = A.n;
  C->n = n;
  C->m = B.m;
  C->ptr.assign(n + 1, 0);
  const int64_t CH = 4096;
  const int64_t nch = (n + CH - 1) / CH;
  std::vector<Chunk> chunks(nch);
#pragma omp parallel
  {
    std::vector<double> sums(B.m, 0.0);
    std::vector<uint8_t> seen(B.m, 0);
    std::vector<int32_t> touched;
    std::vector<std::pair<int32_t, double>> row;
#pragma omp for schedule(dynamic, 1)
    for (int64_t c = 0; c < nch; ++c) {
      Chunk& out = chunks[c];
      const int64_t r0 = c * CH, r1 = std::min(n, r0 + CH);
      for (int64_t i = r0; i < r1; ++i) {
        touched.clear();
        for (int64_t kk = A.ptr[i]; kk < A.ptr[i + 1]; ++kk) {
          const int64_t k = A.col[kk];
          const double v = A.val[kk];
          for (int64_t jj = B.ptr[k]; jj < B.ptr[k + 1]; ++jj) {
            const int32_t j = B.col[jj];
            sums[j] += v * B.val[jj];
            if (!seen[j]) { seen[j] = 1; touched.push_back(j); }
          }
        }
        row.clear();
        for (int32_t j : touched) {
          if (sums[j] != 0.0) row.emplace_back(j, sums[j]);
          sums[j] = 0.0;
          seen[j] = 0;
        }
        std::sort(row.begin(), row.end(),
                  [](const std::pair<int32_t, double>& a, const std::pair<int32_t, double>& b) {
                    return a.first < b.first;
                  });
        C->ptr[i + 1] = (int64_t)row.size();
        for (auto& e : row) { out.col.push_back(e.first); out.val.push_back(e.second); }
      }
    }
  }
  for (int64_t i = 0; i < n; ++i) C->ptr[i + 1] += C->ptr[i];
  C->col.resize(C->ptr[n]);
  C->val.resize(C->ptr[n]);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t c = 0; c < nch; ++c) {
    const int64_t off = C->ptr[c * CH];
    std::copy(chunks[c].col.begin(), chunks[c].col.end(), C->col.begin() + off);
    std::copy(chunks[c].val.begin(), chunks[c].val.end(), C->val.begin() + off);
    Chunk().col.swap(chunks[c].col);
    Chunk().val.swap(chunks[c].val);
  }
}

// R = P^T with sorted rows (counting sort in row order == scipy P.T.tocsr()).
void transpose(const CsrView& P, Csr* R) {
  R->n = P.m;
  R->m = P.n;
  R->ptr.assign(P.m + 1, 0);
  const int64_t nnz = P.nnz();
  for (int64_t k = 0; k < nnz; ++k) R->ptr[P.col[k] + 1]++;
  for (int64_t i = 0; i < P.m; ++i) R->ptr[i + 1] += R->ptr[i];
  R->col.resize(nnz);
  R->val.resize(nnz);
  std::vector<int64_t> next(R->ptr.begin(), R->ptr.end() - 1);
  for (int64_t i = 0; i < P.n; ++i)
    for (int64_t k = P.ptr[i]; k < P.ptr[i + 1]; ++k) {
      const int64_t d = next[P.col[k]]++;
      R->col[d] = (int32_t)i;
      R->val[d] = P.val[k];
    }
}

// ---------------------------------------------------------------------------
// strength of connection, symmetrised: flags on A's pattern + extra (i,j)
// pairs whose mirror entry is absent from A (rare; not weighted in phase 3).
// ---------------------------------------------------------------------------
struct Strength {
  std::vector<uint8_t> flag;       // per A entry: (i,j) in S
  std::vector<int64_t> xptr;       // extras CSR (neighbours not in A's row)
  std::vector<int32_t> xcol;
};

// rowmax: theta relative to the row's largest off-diagonal coupling (the
// default), else to sqrt(|a_ii a_jj|) (classical, MAMG_STRENGTH_DIAG)
void strength(const CsrView& A, double theta, bool rowmax, Strength* S) {
  const int64_t n = A.n, nnz = A.nnz();
  std::vector<double> d(n);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) d[i] = std::fabs(diag_of(A, i));
  std::vector<uint8_t> f0(nnz, 0);
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t i = 0; i < n; ++i) {
    double m = 0.0;   // the row's largest coupling (oracle strength / node_strength)
    for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k)
      if (A.col[k] != i) m = std::max(m, std::fabs(A.val[k]));
    for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) {
      const int64_t j = A.col[k];
      if (j == i) continue;
      const double av = std::fabs(A.val[k]);
      const double s = std::sqrt(d[i] * d[j]);
      f0[k] = (av >= theta * (rowmax ? m : s)) && (av > 1e-12 * s);
    }
  }
  S->flag.assign(nnz, 0);
  std::vector<std::vector<std::pair<int32_t, int32_t>>> extra(omp_get_max_threads());
#pragma omp parallel
  {
    auto& ex = extra[omp_get_thread_num()];
#pragma omp for schedule(dynamic, 4096)
    for (int64_t i = 0; i < n; ++i)
      for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) {
        if (!f0[k]) continue;
        __atomic_store_n(&S->flag[k], (uint8_t)1, __ATOMIC_RELAXED);
        const int64_t j = A.col[k];
        const int64_t q = find_pos(A, j, i);
        if (q >= 0)
          __atomic_store_n(&S->flag[q], (uint8_t)1, __ATOMIC_RELAXED);
        else
          ex.emplace_back((int32_t)j, (int32_t)i);
      }
  }
  std::vector<std::pair<int32_t, int32_t>> all;
  for (auto& e : extra) all.insert(all.end(), e.begin(), e.end());
  std::sort(all.begin(), all.end());
  all.erase(std::unique(all.begin(), all.end()), all.end());
  S->xptr.assign(n + 1, 0);
  S->xcol.resize(all.size());
  for (size_t t = 0; t < all.size(); ++t) {
    S->xptr[all[t].first + 1]++;
    S->xcol[t] = all[t].second;
  }
  for (int64_t i = 0; i < n; ++i) S->xptr[i + 1] += S->xptr[i];
}

template <class F>
inline void for_strong(const CsrView& A, const Strength& S, int64_t i, F&& f) {
  for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k)
    if (S.flag[k]) f((int64_t)A.col[k]);
  for (int64_t k = S.xptr[i]; k < S.xptr[i + 1]; ++k) f((int64_t)S.xcol[k]);
}

// ---------------------------------------------------------------------------
// MIS-2 (oracle mis2) and aggregation (oracle aggregate_mis2)
// ---------------------------------------------------------------------------
int aggregate_mis2(const CsrView& A, const Strength& S, int level,
                   std::vector<int64_t>* agg_out, int64_t* nagg_out, std::string* err) {
  const int64_t n = A.n;
  std::vector<uint64_t> state(n), low(n), key(n), m1(n);
  std::vector<uint8_t> nonisol(n);
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t i = 0; i < n; ++i) {
    bool any = false;
    for_strong(A, S, i, [&](int64_t) { any = true; });
    nonisol[i] = any;
    state[i] = any ? ST_UND : ST_OUT;
    low[i] = ((uint64_t)(hash32((uint64_t)i, level) & 0x7FFFFFFFu) << 31) | (uint64_t)i;
  }
  for (int rounds = 0;; ++rounds) {
    if (rounds > 10000) { *err = "mis2 did not converge"; return MAMG_ERR_SETUP; }
    int64_t und = 0;
#pragma omp parallel for schedule(static) reduction(+ : und)
    for (int64_t i = 0; i < n; ++i) {
      key[i] = (state[i] << 62) | low[i];
      und += state[i] == ST_UND;
    }
    if (und == 0) break;
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t i = 0; i < n; ++i) {
      uint64_t m = key[i];
      for_strong(A, S, i, [&](int64_t j) { m = std::max(m, key[j]); });
      m1[i] = m;
    }
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t i = 0; i < n; ++i) {
      if (state[i] != ST_UND) continue;
      uint64_t m = m1[i];
      for_strong(A, S, i, [&](int64_t j) { m = std::max(m, m1[j]); });
      if (m == key[i]) state[i] = ST_IN;
      else if ((m >> 62) == ST_IN) state[i] = ST_OUT;
    }
  }
  // roots numbered in index order
  std::vector<int64_t>& agg = *agg_out;
  agg.assign(n, -1);
  int64_t nroots = 0;
  for (int64_t i = 0; i < n; ++i)
    if (state[i] == ST_IN) agg[i] = nroots++;
  // phase 2: neighbours of roots
  std::vector<int64_t> agg2(agg);
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t i = 0; i < n; ++i) {
    if (state[i] == ST_IN) continue;
    for_strong(A, S, i, [&](int64_t j) {
      if (state[j] == ST_IN) agg2[i] = agg[j];
    });
  }
  // phase 3: remaining non-isolated nodes -> strongest weighted neighbour
  std::vector<int64_t> agg3(agg2);
  int bad = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : bad)
  for (int64_t i = 0; i < n; ++i) {
    if (!nonisol[i] || agg2[i] >= 0) continue;
    double bw = -1.0;
    int64_t ba = -1;
    for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) {
      if (!S.flag[k]) continue;
      const double w = std::fabs(A.val[k]) * 1.0;
      if (w == 0.0) continue;
      const int64_t a = agg2[A.col[k]];
      if (a < 0) continue;
      if (w > bw || (w == bw && a < ba)) { bw = w; ba = a; }
    }
    if (ba < 0) bad++;
    agg3[i] = ba;
  }
  if (bad) { *err = "aggregation left a non-isolated node unassigned"; return MAMG_ERR_SETUP; }
  agg.swap(agg3);
  *nagg_out = nroots;
  return MAMG_OK;
}

// ---------------------------------------------------------------------------
// Vanek-Mandel-Brezina aggregation (oracle aggregate_vmb): sequential, index
// order.  Phase 1: a non-isolated node whose strong neighbourhood is all
// free starts an aggregate {i} + N(i).  Phase 2: every other non-isolated
// node joins the phase-1 aggregate of its strongest weighted neighbour
// (ties: smallest aggregate id).  The reference's parameters_standard and
// 3D-1D .dat select it (src/amg_parameters.py:16,36, src/input_metric.dat:89).
// ---------------------------------------------------------------------------
int aggregate_vmb(const CsrView& A, const Strength& S, int level,
                  std::vector<int64_t>* agg_out, int64_t* nagg_out, std::string* err) {
  (void)level;
  const int64_t n = A.n;
  std::vector<int64_t>& agg = *agg_out;
  agg.assign(n, -1);
  std::vector<uint8_t> nonisol(n, 0);
  int64_t nagg = 0;
  for (int64_t i = 0; i < n; ++i) {
    bool any = false, taken = false;
    for_strong(A, S, i, [&](int64_t j) {
      any = true;
      taken = taken || agg[j] >= 0;
    });
    nonisol[i] = any;
    if (!any || agg[i] >= 0 || taken) continue;
    agg[i] = nagg;
    for_strong(A, S, i, [&](int64_t j) { agg[j] = nagg; });
    ++nagg;
  }
  std::vector<int64_t> agg1(agg);
  int bad = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : bad)
  for (int64_t i = 0; i < n; ++i) {
    if (!nonisol[i] || agg1[i] >= 0) continue;
    double bw = -1.0;
    int64_t ba = -1;
    for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) {
      if (!S.flag[k]) continue;
      const double w = std::fabs(A.val[k]) * 1.0;
      if (w == 0.0) continue;
      const int64_t a = agg1[A.col[k]];
      if (a < 0) continue;
      if (w > bw || (w == bw && a < ba)) { bw = w; ba = a; }
    }
    if (ba < 0) bad++;
    agg[i] = ba;
  }
  if (bad) { *err = "VMB aggregation left a non-isolated node unassigned"; return MAMG_ERR_SETUP; }
  *nagg_out = nagg;
  return MAMG_OK;
}

// ---------------------------------------------------------------------------
// parallel heavy-edge matching aggregation (oracle aggregate_hem / hem_match)
// ---------------------------------------------------------------------------
constexpr int HEM_PASSES = 2, HEM_MAX_ROUNDS = 64;

inline uint32_t edge_hash(int64_t i, int64_t j, int lvl) {
  const int64_t a = std::min(i, j), b = std::max(i, j);
  return hash32((uint64_t)a, 0x5000 + lvl) ^ hash32((uint64_t)b, 0x6000 + lvl);
}

// handshake rounds: a free active node picks the free neighbour with the
// largest (weight, edge hash), smallest index on ties; mutual picks match
void hem_match(const CsrView& W, const std::vector<uint8_t>& act, int lvl, std::vector<int64_t>* mate_out) {
  const int64_t n = W.n;
  std::vector<int64_t>& mate = *mate_out;
  mate.assign(n, -1);
  std::vector<int64_t> choice(n);
  for (int round = 0; round < HEM_MAX_ROUNDS; ++round) {
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t i = 0; i < n; ++i) {
      int64_t best = -1;
      double bw = 0.0;
      uint32_t bh = 0;
      if (act[i] && mate[i] < 0)
        for (int64_t k = W.ptr[i]; k < W.ptr[i + 1]; ++k) {
          const int64_t j = W.col[k];
          if (j == i || !act[j] || mate[j] >= 0) continue;
          const double w = W.val[k];
          const uint32_t h = edge_hash(i, j, lvl);
          if (best < 0 || w > bw || (w == bw && (h > bh || (h == bh && j < best)))) {
            best = j; bw = w; bh = h;
          }
        }
      choice[i] = best;
    }
    int64_t got = 0;
#pragma omp parallel for schedule(static) reduction(+ : got)
    for (int64_t i = 0; i < n; ++i) {
      const int64_t c = choice[i];
      if (c >= 0 && choice[c] == i) { mate[i] = c; ++got; }
    }
    if (!got) break;
  }
}

int aggregate_hem(const CsrView& A, const Strength& S, int level, std::vector<int64_t>* agg_out,
                  int64_t* nagg_out, std::string* err) {
  const int64_t n = A.n;
  Csr W;   // strong graph weighted by |a_ij| (zeros dropped)
  W.n = W.m = n;
  W.ptr.assign(n + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k)
      if (S.flag[k] && A.col[k] != i && std::fabs(A.val[k]) * 1.0 != 0.0) {
        W.col.push_back(A.col[k]);
        W.val.push_back(std::fabs(A.val[k]) * 1.0);
      }
    W.ptr[i + 1] = (int64_t)W.col.size();
  }
  const Csr W1 = W;   // the pass-1 graph (absorption of the nodes left alone)
  std::vector<uint8_t> act(n);
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t i = 0; i < n; ++i) {
    bool any = false;
    for_strong(A, S, i, [&](int64_t) { any = true; });
    act[i] = any;
  }
  std::vector<int64_t>& agg = *agg_out;
  agg.assign(n, -1);
  for (int64_t i = 0; i < n; ++i)
    if (act[i]) agg[i] = i;
  int64_t nagg = n;
  for (int ps = 0; ps < HEM_PASSES; ++ps) {
    const int64_t m = W.n;
    std::vector<int64_t> mate;
    hem_match(W.view(), act, 16 * level + ps, &mate);
    std::vector<int64_t> a(m, -1);
    nagg = 0;
    for (int64_t i = 0; i < m; ++i) {   // roots (smallest member) numbered in index order
      if (!act[i]) continue;
      const int64_t r = mate[i] >= 0 ? std::min(i, mate[i]) : i;
      if (r == i) a[i] = nagg++;
    }
    for (int64_t i = 0; i < m; ++i)
      if (act[i] && mate[i] >= 0 && mate[i] < i) a[i] = a[mate[i]];
    for (int64_t i = 0; i < n; ++i)
      if (agg[i] >= 0) agg[i] = a[agg[i]];
    if (ps + 1 == HEM_PASSES) break;
    Csr T, Tt, WT, C;   // W_next = T^T W T, diagonal dropped
    T.n = m; T.m = nagg;
    T.ptr.assign(m + 1, 0);
    for (int64_t i = 0; i < m; ++i) {
      if (act[i]) { T.col.push_back((int32_t)a[i]); T.val.push_back(1.0); }
      T.ptr[i + 1] = (int64_t)T.col.size();
    }
    spgemm(W.view(), T.view(), &WT);
    transpose(T.view(), &Tt);
    spgemm(Tt.view(), WT.view(), &C);
    W = Csr();
    W.n = W.m = nagg;
    W.ptr.assign(nagg + 1, 0);
    for (int64_t i = 0; i < nagg; ++i) {
      for (int64_t k = C.ptr[i]; k < C.ptr[i + 1]; ++k)
        if (C.col[k] != i && C.val[k] != 0.0) { W.col.push_back(C.col[k]); W.val.push_back(C.val[k]); }
      W.ptr[i + 1] = (int64_t)W.col.size();
    }
    act.assign(nagg, 1);
  }
  // nodes left alone by every pass join the heaviest strong neighbour's
  // aggregate of >= 2 members (ties: smallest id); ids then compacted
  std::vector<int64_t> size(nagg, 0);
  for (int64_t i = 0; i < n; ++i)
    if (agg[i] >= 0) size[agg[i]]++;
  std::vector<int64_t> agg2(agg);
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t i = 0; i < n; ++i) {
    if (agg[i] < 0 || size[agg[i]] != 1) continue;
    double bw = 0.0;
    int64_t ba = -1;
    for (int64_t k = W1.ptr[i]; k < W1.ptr[i + 1]; ++k) {
      const int64_t a = agg[W1.col[k]];
      if (a < 0 || size[a] < 2) continue;
      const double w = W1.val[k];
      if (ba < 0 || w > bw || (w == bw && a < ba)) { bw = w; ba = a; }
    }
    if (ba >= 0) agg2[i] = ba;
  }
  std::vector<int64_t> newid(nagg, 0);
  for (int64_t i = 0; i < n; ++i)
    if (agg2[i] >= 0) newid[agg2[i]] = 1;
  int64_t used = 0;
  for (int64_t a = 0; a < nagg; ++a) newid[a] = newid[a] ? used++ : -1;
  for (int64_t i = 0; i < n; ++i) agg[i] = agg2[i] >= 0 ? newid[agg2[i]] : -1;
  *nagg_out = used;
  (void)err;
  return MAMG_OK;
}

void tentative(const std::vector<int64_t>& agg, int64_t nagg, Csr* T) {
  const int64_t n = (int64_t)agg.size();
  T->n = n;
  T->m = nagg;
  T->ptr.assign(n + 1, 0);
  for (int64_t i = 0; i < n; ++i) T->ptr[i + 1] = T->ptr[i] + (agg[i] >= 0);
  T->col.resize(T->ptr[n]);
  T->val.assign(T->ptr[n], 1.0);
  for (int64_t i = 0; i < n; ++i)
    if (agg[i] >= 0) T->col[T->ptr[i]] = (int32_t)agg[i];
}

// rho(D^-1 A) Gershgorin bound: max_i dinv_i * sum_j |a_ij|
double rho_gershgorin(const std::vector<double>& dinv, const std::vector<double>& rs) {
  double r = -INFINITY;
  for (size_t i = 0; i < rs.size(); ++i) r = std::max(r, dinv[i] * rs[i]);
  return r;
}

// rho estimate, oracle rho_estimate (iters > 0: inf-norm power iteration)
double rho_estimate(const CsrView& A, const std::vector<double>& dinv,
                    const std::vector<double>& rs, int iters) {
  if (iters == 0) return rho_gershgorin(dinv, rs);
  const int64_t n = A.n;
  std::vector<double> v(n), w(n);
  for (int64_t i = 0; i < n; ++i)
    v[i] = ((double)hash32((uint64_t)i, 977) / 4294967296.0) * 2.0 - 1.0;
  double rho = 0.0;
  for (int it = 0; it < iters; ++it) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      double s = 0.0;
      for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) s += A.val[k] * v[A.col[k]];
      w[i] = dinv[i] * s;
    }
    double mv = 0.0, mw = 0.0;
    for (int64_t i = 0; i < n; ++i) { mv = std::max(mv, std::fabs(v[i])); mw = std::max(mw, std::fabs(w[i])); }
    rho = mw / mv;
    for (int64_t i = 0; i < n; ++i) v[i] = w[i] / mw;
  }
  return rho;
}

// P = T - X, X_ij = c_i * AT_ij  (csr_binop_csr merge, zeros dropped)
void smooth_merge(const Csr& T, const Csr& AT, const std::vector<double>& c, Csr* P) {
  const int64_t n = T.n;
  P->n = n;
  P->m = T.m;
  P->ptr.assign(n + 1, 0);
  std::vector<Chunk> rows(n);  // simple two-pass: count then fill
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t i = 0; i < n; ++i) {
    int64_t cnt = 0;
    const bool ht = T.ptr[i + 1] > T.ptr[i];
    const int32_t tc = ht ? T.col[T.ptr[i]] : -1;
    bool tdone = !ht;
    for (int64_t k = AT.ptr[i]; k < AT.ptr[i + 1]; ++k) {
      const int32_t j = AT.col[k];
      const double x = c[i] * AT.val[k];
      if (!tdone && tc < j) { cnt++; tdone = true; }
      double r;
      if (x == 0.0) {            // X entry dropped by scipy (diags @ AT)
        if (!tdone && tc == j) { r = 1.0; tdone = true; } else continue;
      } else if (!tdone && tc == j) {
        r = 1.0 - x; tdone = true;
      } else {
        r = 0.0 - x;
      }
      if (r != 0.0) cnt++;
    }
    if (!tdone) cnt++;
    P->ptr[i + 1] = cnt;
  }
  for (int64_t i = 0; i < n; ++i) P->ptr[i + 1] += P->ptr[i];
  P->col.resize(P->ptr[n]);
  P->val.resize(P->ptr[n]);
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t i = 0; i < n; ++i) {
    int64_t o = P->ptr[i];
    const bool ht = T.ptr[i + 1] > T.ptr[i];
    const int32_t tc = ht ? T.col[T.ptr[i]] : -1;
    bool tdone = !ht;
    for (int64_t k = AT.ptr[i]; k < AT.ptr[i + 1]; ++k) {
      const int32_t j = AT.col[k];
      const double x = c[i] * AT.val[k];
      if (!tdone && tc < j) { P->col[o] = tc; P->val[o] = 1.0; ++o; tdone = true; }
      double r;
      if (x == 0.0) {
        if (!tdone && tc == j) { r = 1.0; tdone = true; } else continue;
      } else if (!tdone && tc == j) {
        r = 1.0 - x; tdone = true;
      } else {
        r = 0.0 - x;
      }
      if (r != 0.0) { P->col[o] = j; P->val[o] = r; ++o; }
    }
    if (!tdone) { P->col[o] = tc; P->val[o] = 1.0; ++o; }
  }
}

// point SA (oracle smooth_prolongator): P = T - (w dinv_i) (A T)_ij
void smooth_prolongator(const CsrView& A, const Csr& T, const std::vector<double>& c, Csr* P) {
  Csr AT;
  spgemm(A, T.view(), &AT);
  smooth_merge(T, AT, c, P);
}

// Gauss-Jordan without pivoting on a row-major n x n block (oracle
// batched_inverse): row_k /= p; row_i -= M_ik * row_k.
bool gauss_jordan(int64_t n, const double* a, double* inv) {
  const int64_t w = 2 * n;
  std::vector<double> M(n * w, 0.0);
  for (int64_t i = 0; i < n; ++i) {
    for (int64_t j = 0; j < n; ++j) M[i * w + j] = a[i * n + j];
    M[i * w + n + i] = 1.0;
  }
  std::vector<double> f(n);
  for (int64_t k = 0; k < n; ++k) {
    const double p = M[k * w + k];
    if (!(p > 0.0)) return false;
    for (int64_t j = 0; j < w; ++j) M[k * w + j] = M[k * w + j] / p;
    for (int64_t i = 0; i < n; ++i) f[i] = M[i * w + k];
    f[k] = 0.0;
    for (int64_t i = 0; i < n; ++i) {
      if (i == k) continue;
      const double fi = f[i];
      double* Mi = &M[i * w];
      const double* Mk = &M[k * w];
      for (int64_t j = 0; j < w; ++j) Mi[j] = Mi[j] - fi * Mk[j];
    }
  }
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j < n; ++j) inv[i * n + j] = M[i * w + n + j];
  return true;
}

// block inverse CSR (oracle block_inverse_csr): row i holds (D_B^-1)_{ij} for
// j in block(i), sorted; blocks numbered 0..nb-1, members ascending.
int block_inverse(const CsrView& A, const std::vector<int64_t>& bid, int64_t nb, Csr* D,
                  std::string* err) {
  const int64_t n = A.n;
  std::vector<int64_t> bptr(nb + 1, 0);
  for (int64_t j = 0; j < n; ++j) bptr[bid[j] + 1]++;
  for (int64_t b = 0; b < nb; ++b) bptr[b + 1] += bptr[b];
  std::vector<int64_t> mem(n), pos(n);
  {
    std::vector<int64_t> nx(bptr.begin(), bptr.end() - 1);
    for (int64_t j = 0; j < n; ++j) { const int64_t q = nx[bid[j]]++; mem[q] = j; pos[j] = q - bptr[bid[j]]; }
  }
  D->n = D->m = n;
  D->ptr.assign(n + 1, 0);
  for (int64_t i = 0; i < n; ++i) D->ptr[i + 1] = D->ptr[i] + (bptr[bid[i] + 1] - bptr[bid[i]]);
  D->col.resize(D->ptr[n]);
  D->val.resize(D->ptr[n]);
  int bad = 0;
#pragma omp parallel for schedule(dynamic, 1024) reduction(+ : bad)
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t s = bptr[b + 1] - bptr[b];
    std::vector<double> dense(s * s, 0.0), inv(s * s);
    for (int64_t a = 0; a < s; ++a) {
      const int64_t i = mem[bptr[b] + a];
      for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) {
        const int64_t j = A.col[k];
        if (bid[j] == b) dense[a * s + pos[j]] = A.val[k];
      }
    }
    if (!gauss_jordan(s, dense.data(), inv.data())) { bad++; continue; }
    for (int64_t a = 0; a < s; ++a) {
      const int64_t i = mem[bptr[b] + a];
      for (int64_t c = 0; c < s; ++c) {
        D->col[D->ptr[i] + c] = (int32_t)mem[bptr[b] + c];
        D->val[D->ptr[i] + c] = inv[a * s + c];
      }
    }
  }
  if (bad) { *err = "smoother block not SPD (non-positive pivot)"; return MAMG_ERR_SETUP; }
  return MAMG_OK;
}

// rho_B = max_i sum_j |(D A)_ij|  (SMMP row, sorted, sequential abs sum)
double block_rho(const CsrView& D, const CsrView& A) {
  const int64_t n = D.n, m = A.m;
  double rho = -INFINITY;
#pragma omp parallel
  {
    std::vector<double> sums(m, 0.0);
    std::vector<uint8_t> seen(m, 0);
    std::vector<int32_t> touched;
    double lrho = -INFINITY;
#pragma omp for schedule(dynamic, 4096)
    for (int64_t i = 0; i < n; ++i) {
      touched.clear();
      for (int64_t kk = D.ptr[i]; kk < D.ptr[i + 1]; ++kk) {
        const int64_t k = D.col[kk];
        const double v = D.val[kk];
        for (int64_t jj = A.ptr[k]; jj < A.ptr[k + 1]; ++jj) {
          const int32_t j = A.col[jj];
          sums[j] += v * A.val[jj];
          if (!seen[j]) { seen[j] = 1; touched.push_back(j); }
        }
      }
      std::sort(touched.begin(), touched.end());
      double s = 0.0;
      for (int32_t j : touched) {
        if (sums[j] != 0.0) s += std::fabs(sums[j]) * 1.0;
        sums[j] = 0.0;
        seen[j] = 0;
      }
      lrho = std::max(lrho, s);
    }
#pragma omp critical
    rho = std::max(rho, lrho);
  }
  return rho;
}

// W_B = (relaxation / rho_B) D_B^-1  (oracle block_smoother)
int block_smoother_from(const CsrView& A, const std::vector<int64_t>& bid, int64_t nb,
                        const mamg_params& p, Csr* W, std::string* err) {
  int rc = block_inverse(A, bid, nb, W, err);
  if (rc) return rc;
  const double rho = block_rho(W->view(), A);
  const double sc = p.relaxation / rho;
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < W->nnz(); ++k) W->val[k] = sc * W->val[k];
  return MAMG_OK;
}

// additive overlapping Schwarz on the seeds' rings (Schwarz_type ADDITIVE,
// oracle overlap_smoother): blocks = seed + breadth-first neighbours up to
// distance Schwarz_maxlvl (ascending columns, at most Schwarz_mmsize dofs),
// S = sum_k R_k^T A_k^-1 R_k (+ 1/a_ii on uncovered dofs) accumulated block by
// block in seed order, W = (relaxation / lambda) S with lambda from
// max(rho_iters, 30) power iterations of S A
int overlap_smoother(const CsrView& A, const int32_t* seeds, int64_t ns, const mamg_params& p, Csr* W,
                     std::string* err) {
  const int64_t n = A.n;
  const int maxlvl = p.Schwarz_maxlvl, mm = p.Schwarz_mmsize;
  if (ns > std::max<int64_t>(n / 8, 1) || (double)ns * mm * mm > 4e9) {
    *err = "SCHWARZ_ADDITIVE (dense overlapping seed blocks) is for sparse seed sets: " + std::to_string(ns) +
           " seeds of up to " + std::to_string(mm) + " dofs";
    return MAMG_ERR_UNSUPPORTED;
  }
  std::vector<std::vector<int64_t>> blocks(ns);
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t k = 0; k < ns; ++k) {
    const int64_t s0 = seeds[k];
    std::vector<int64_t> order{s0};
    std::vector<int> depth{0};
    auto seen = [&](int64_t j) { return std::find(order.begin(), order.end(), j) != order.end(); };
    size_t head = 0;
    while (head < order.size() && (int64_t)order.size() < mm) {
      const int64_t v = order[head];
      const int dv = depth[head];
      ++head;
      if (dv == maxlvl) continue;
      for (int64_t q = A.ptr[v]; q < A.ptr[v + 1]; ++q) {
        const int64_t j = A.col[q];
        if (!seen(j)) {
          order.push_back(j);
          depth.push_back(dv + 1);
          if ((int64_t)order.size() >= mm) break;
        }
      }
    }
    std::sort(order.begin(), order.end());
    blocks[k] = std::move(order);
  }
  // sorted pattern: every block's dense square, plus the uncovered diagonal
  std::vector<char> cov(n, 0);
  for (const auto& b : blocks)
    for (int64_t i : b) cov[i] = 1;
  std::vector<std::vector<int32_t>> rc(n);
  for (const auto& b : blocks)
    for (int64_t i : b)
      for (int64_t j : b) rc[i].push_back((int32_t)j);
  W->n = W->m = n;
  W->ptr.assign(n + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (!cov[i]) rc[i].push_back((int32_t)i);
    std::sort(rc[i].begin(), rc[i].end());
    rc[i].erase(std::unique(rc[i].begin(), rc[i].end()), rc[i].end());
    W->ptr[i + 1] = W->ptr[i] + (int64_t)rc[i].size();
  }
  W->col.resize(W->ptr[n]);
  W->val.assign(W->ptr[n], 0.0);
  for (int64_t i = 0; i < n; ++i) std::copy(rc[i].begin(), rc[i].end(), W->col.begin() + W->ptr[i]);
  std::vector<std::vector<int32_t>>().swap(rc);
  const CsrView Wv = W->view();
  for (const auto& b : blocks) {   // block order: the oracle's accumulation order
    const int64_t m = (int64_t)b.size();
    std::vector<double> dense(m * m, 0.0), inv(m * m);
    for (int64_t a = 0; a < m; ++a)
      for (int64_t c = 0; c < m; ++c) {
        const int64_t q = find_pos(A, b[a], b[c]);
        if (q >= 0) dense[a * m + c] = A.val[q];
      }
    if (!gauss_jordan(m, dense.data(), inv.data())) { *err = "Schwarz block not SPD"; return MAMG_ERR_SETUP; }
    for (int64_t a = 0; a < m; ++a)
      for (int64_t c = 0; c < m; ++c) W->val[find_pos(Wv, b[a], b[c])] += inv[a * m + c];
  }
  for (int64_t i = 0; i < n; ++i)
    if (!cov[i]) W->val[find_pos(Wv, i, i)] = 1.0 / diag_of(A, i);
  // lambda_max(S A): inf-norm power iterations (rho_estimate's start vector)
  std::vector<double> v(n), t(n), w(n);
  for (int64_t i = 0; i < n; ++i) v[i] = ((double)hash32((uint64_t)i, 977) / 4294967296.0) * 2.0 - 1.0;
  double lam = 0.0;
  for (int it = 0; it < std::max(p.rho_iters, 30); ++it) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      double s = 0.0;
      for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) s += A.val[k] * v[A.col[k]];
      t[i] = s;
    }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      double s = 0.0;
      for (int64_t k = W->ptr[i]; k < W->ptr[i + 1]; ++k) s += W->val[k] * t[W->col[k]];
      w[i] = s;
    }
    double mv = 0.0, mw = 0.0;
    for (int64_t i = 0; i < n; ++i) { mv = std::max(mv, std::fabs(v[i])); mw = std::max(mw, std::fabs(w[i])); }
    lam = mw / mv;
    for (int64_t i = 0; i < n; ++i) v[i] = w[i] / mw;
  }
  const double sc = p.relaxation / lam;
  for (double& x : W->val) x = sc * x;
  return MAMG_OK;
}

// node blocks: bid(f*nv + I) = I
void node_blocks(int64_t n, int nf, std::vector<int64_t>* bid, int64_t* nb) {
  const int64_t nv = n / nf;
  bid->resize(n);
  for (int64_t i = 0; i < n; ++i) (*bid)[i] = i % nv;
  *nb = nv;
}

// node graph (oracle node_strength): s_IJ = sqrt(sum of squares of the
// nf x nf block), accumulated over rows f*nv+I (f ascending), columns sorted.
void node_graph(const CsrView& A, int nf, Csr* G) {
  const int64_t nv = A.n / nf;
  G->n = G->m = nv;
  G->ptr.assign(nv + 1, 0);
  const int64_t CH = 4096;
  const int64_t nch = (nv + CH - 1) / CH;
  std::vector<Chunk> chunks(nch);
#pragma omp parallel
  {
    std::vector<double> acc(nv, 0.0);
    std::vector<uint8_t> seen(nv, 0);
    std::vector<int32_t> touched;
#pragma omp for schedule(dynamic, 1)
    for (int64_t c = 0; c < nch; ++c) {
      const int64_t r0 = c * CH, r1 = std::min(nv, r0 + CH);
      for (int64_t I = r0; I < r1; ++I) {
        touched.clear();
        for (int f = 0; f < nf; ++f) {
          const int64_t row = f * nv + I;
          for (int64_t k = A.ptr[row]; k < A.ptr[row + 1]; ++k) {
            const int32_t J = (int32_t)(A.col[k] % nv);
            acc[J] += A.val[k] * A.val[k];
            if (!seen[J]) { seen[J] = 1; touched.push_back(J); }
          }
        }
        std::sort(touched.begin(), touched.end());
        G->ptr[I + 1] = (int64_t)touched.size();
        for (int32_t J : touched) {
          chunks[c].col.push_back(J);
          chunks[c].val.push_back(std::sqrt(acc[J]));
          acc[J] = 0.0;
          seen[J] = 0;
        }
      }
    }
  }
  for (int64_t i = 0; i < nv; ++i) G->ptr[i + 1] += G->ptr[i];
  G->col.resize(G->ptr[nv]);
  G->val.resize(G->ptr[nv]);
  for (int64_t c = 0; c < nch; ++c) {
    std::copy(chunks[c].col.begin(), chunks[c].col.end(), G->col.begin() + G->ptr[c * CH]);
    std::copy(chunks[c].val.begin(), chunks[c].val.end(), G->val.begin() + G->ptr[c * CH]);
  }
}

// dof f*nv + I -> coarse dof f*nagg + agg[I]  (oracle tentative_nodal)
void tentative_nodal(const std::vector<int64_t>& agg, int64_t nagg, int nf, Csr* T) {
  const int64_t nv = (int64_t)agg.size(), n = nv * nf;
  T->n = n;
  T->m = nagg * nf;
  T->ptr.assign(n + 1, 0);
  for (int64_t i = 0; i < n; ++i) T->ptr[i + 1] = T->ptr[i] + (agg[i % nv] >= 0);
  T->col.resize(T->ptr[n]);
  T->val.assign(T->ptr[n], 1.0);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t I = i % nv, f = i / nv;
    if (agg[I] >= 0) T->col[T->ptr[i]] = (int32_t)(f * nagg + agg[I]);
  }
}

// seed blocks (oracle seed_blocks) -> W_B (block_smoother)
int block_smoother(const CsrView& A, const int32_t* idofs, int64_t n_idofs,
                   const mamg_params& p, Csr* W, std::string* err) {
  const int64_t n = A.n;
  std::vector<uint8_t> isseed(n, 0);
  for (int64_t t = 0; t < n_idofs; ++t) {
    if (idofs[t] < 0 || idofs[t] >= n) { *err = "idofs out of range"; return MAMG_ERR_ARG; }
    isseed[idofs[t]] = 1;
  }
  std::vector<int64_t> best(n, -1);
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t j = 0; j < n; ++j) {
    if (isseed[j]) continue;
    double bv = -1.0;
    int64_t bs = -1;
    for (int64_t k = A.ptr[j]; k < A.ptr[j + 1]; ++k) {
      const int64_t s = A.col[k];
      if (s == j || !isseed[s]) continue;
      const double v = std::fabs(A.val[k]);
      if (v > bv || (v == bv && s < bs)) { bv = v; bs = s; }
    }
    best[j] = bs;
  }
  // cap joiners per seed (lowest indices kept)
  std::vector<int64_t> owner(n);
  std::iota(owner.begin(), owner.end(), 0);
  {
    std::vector<int64_t> cnt(n, 0);
    for (int64_t j = 0; j < n; ++j) {           // ascending j == lowest first
      const int64_t s = best[j];
      if (s < 0) continue;
      if (cnt[s] < (int64_t)p.Schwarz_mmsize - 1) { owner[j] = s; cnt[s]++; }
    }
  }
  // block ids by owner index; members sorted
  std::vector<int64_t> bid(n, -1), bsize;
  std::vector<uint8_t> isowner(n, 0);
  for (int64_t j = 0; j < n; ++j) isowner[owner[j]] = 1;
  std::vector<int64_t> ownid(n, -1);
  int64_t nb = 0;
  for (int64_t j = 0; j < n; ++j)
    if (isowner[j]) ownid[j] = nb++;
  for (int64_t j = 0; j < n; ++j) bid[j] = ownid[owner[j]];
  return block_smoother_from(A, bid, nb, p, W, err);
}

// nodal SA (oracle smooth_prolongator_block):
// P = T - w (D_B^-1 (A T)), w = sa_omega / rho_B
int smooth_prolongator_block(const CsrView& A, const Csr& T, int nf, const mamg_params& p,
                             Csr* P, double* w_out, std::string* err) {
  std::vector<int64_t> bid;
  int64_t nb;
  node_blocks(A.n, nf, &bid, &nb);
  Csr D;
  int rc = block_inverse(A, bid, nb, &D, err);
  if (rc) return rc;
  const double rho = block_rho(D.view(), A);
  const double w = p.sa_omega / rho;
  *w_out = w;
  Csr AT, Y;
  spgemm(A, T.view(), &AT);
  spgemm(D.view(), AT.view(), &Y);
  const std::vector<double> one(A.n, 1.0);
  // X_ij = w * Y_ij; the merge below is shared with the point version with
  // c_i = 1 applied to the pre-scaled Y (1.0 * x == x exactly)
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < Y.nnz(); ++k) Y.val[k] = w * Y.val[k];
  smooth_merge(T, Y, one, P);
  return MAMG_OK;
}

}  // namespace

// greedy first-fit colour per seed block in block order (host.h): block k
// takes the smallest colour no earlier conflicting block holds; blocks
// conflict iff a member of one lies in the closed neighbourhood of a member of
// the other (so a colour's blocks write no x another of them reads)
void ring_colouring(const CsrView& A, const std::vector<int64_t>& bptr, const std::vector<int32_t>& mem,
                    std::vector<int32_t>* colour) {
  const int64_t nb = (int64_t)bptr.size() - 1, n = A.n;
  // blocks holding each dof (CSR, ascending block ids)
  std::vector<int64_t> dptr(n + 1, 0);
  for (int64_t k = 0; k < nb; ++k)
    for (int64_t t = bptr[k]; t < bptr[k + 1]; ++t) dptr[mem[t] + 1]++;
  for (int64_t i = 0; i < n; ++i) dptr[i + 1] += dptr[i];
  std::vector<int32_t> dblk(dptr[n]);
  {
    std::vector<int64_t> fill(dptr.begin(), dptr.end() - 1);
    for (int64_t k = 0; k < nb; ++k)
      for (int64_t t = bptr[k]; t < bptr[k + 1]; ++t) dblk[fill[mem[t]]++] = (int32_t)k;
  }
  colour->assign(nb, -1);
  std::vector<int64_t> mark;   // mark[c] == k: colour c taken by a conflicting block of k
  for (int64_t k = 0; k < nb; ++k) {
    auto touch = [&](int64_t j) {
      for (int64_t q = dptr[j]; q < dptr[j + 1]; ++q) {
        const int32_t l = dblk[q];
        if (l >= k) break;                 // ascending: only earlier (coloured) blocks
        const int32_t c = (*colour)[l];
        if ((int64_t)mark.size() <= c) mark.resize(c + 1, -1);
        mark[c] = k;
      }
    };
    for (int64_t t = bptr[k]; t < bptr[k + 1]; ++t) {
      const int64_t i = mem[t];
      touch(i);
      for (int64_t q = A.ptr[i]; q < A.ptr[i + 1]; ++q) touch(A.col[q]);
    }
    int32_t c = 0;
    while (c < (int32_t)mark.size() && mark[c] == k) ++c;
    (*colour)[k] = c;
  }
}

// exported for the GPU setup (host.h): VMB on a device-built strength graph
int aggregate_vmb_flags(const CsrView& G, const uint8_t* flag, std::vector<int64_t>* agg, int64_t* nagg,
                        std::string* err) {
  Strength S;
  S.flag.assign(flag, flag + G.nnz());
  S.xptr.assign(G.n + 1, 0);
  return aggregate_vmb(G, S, 0, agg, nagg, err);
}

// Chebyshev polynomial of degree m in W A on [hi / poly_ratio, hi], hi =
// relaxation (a bound of lambda_max(W A): W = (relaxation / rho_B) D^-1 with
// rho_B a Gershgorin bound), as m Richardson steps with w_k = 1 / tau_k, tau_k
// the polynomial's roots theta + delta cos((2k - 1) pi / (2m)), k = 1..m
int poly_weights(const mamg_params& p, double* w) {
  const int m = smoother_steps(p);
  if (p.smoother != MAMG_SMOOTHER_POLY) { w[0] = 1.0; return 1; }
  const double hi = p.relaxation, lo = hi / p.poly_ratio;
  const double theta = 0.5 * (hi + lo), delta = 0.5 * (hi - lo);
  const double pi = 3.14159265358979323846;
  for (int k = 1; k <= m; ++k) w[k - 1] = 1.0 / (theta + delta * std::cos((2 * k - 1) * pi / (2 * m)));
  return m;
}

// The reference's Schwarz_type names mean multiplicative Schwarz on the
// overlapping blocks seed + Schwarz_maxlvl ring (src/amg_parameters.py:83-87,
// src/utils.py:60-86).  SYMMETRIC with rings (Schwarz_maxlvl >= 1) on a nodal
// system runs as
//  * SCHWARZ_PATCHES when the rings are 1-rings and every node holds a seed
//    (the bidomain: one patch per node, both fields of its closed
//    neighbourhood -- the same blocks, a dedicated kernel);
//  * SCHWARZ_RINGS otherwise (sparse seed sets: EMI's interface dofs with the
//    default dict's 2-rings): one block per seed, greedy conflict colours, and
//    node-block GS on the dofs in no block ("the rest the GS smoother");
//  * without seeds no Schwarz level: the level smoother everywhere.
// With Schwarz_maxlvl 0 the blocks are the seeds' nodes, which do not
// overlap: the matching level smoother on the seed blocks.  Anything else
// keeps its name and check_params rejects it.  Mirrored by
// mamg_oracle.resolve_params.
mamg_params resolve_params(const mamg_params& in, const int32_t* idofs, int64_t n_idofs, int64_t n) {
  mamg_params p = in;
  if (p.Schwarz_levels < 1) return p;
  if (p.Schwarz_type == MAMG_SCHWARZ_SYMMETRIC && p.Schwarz_maxlvl >= 1 && p.num_functions == 2 &&
      p.node_block_smoother) {
    if (!idofs || n_idofs <= 0) {
      p.Schwarz_levels = 0;
      return p;
    }
    bool every = p.Schwarz_maxlvl == 1 && n >= 2 && n % 2 == 0;
    if (every) {
      const int64_t nv = n / 2;
      std::vector<char> has(nv, 0);
      for (int64_t t = 0; t < n_idofs; ++t)
        if (idofs[t] >= 0 && idofs[t] < n) has[idofs[t] % nv] = 1;
      for (int64_t I = 0; I < nv && every; ++I) every = has[I] != 0;
    }
    p.Schwarz_type = every ? MAMG_SCHWARZ_PATCHES : MAMG_SCHWARZ_RINGS;
  }
  return p;
}

// a caller's dict applied to a hierarchy built earlier (mamg_upload): the
// Schwarz name resolves as it did at setup
mamg_params resolve_like(const mamg_params& in, const mamg_params& built) {
  mamg_params p = in;
  if (p.Schwarz_levels >= 1 && p.Schwarz_type == MAMG_SCHWARZ_SYMMETRIC && p.Schwarz_maxlvl >= 1) {
    p.Schwarz_type = built.Schwarz_type;
    p.Schwarz_levels = built.Schwarz_levels;
  }
  return p;
}

int check_params(const mamg_params& p, std::string* err) {
  if (p.abi_version != MAMG_ABI_VERSION) { *err = "mamg_params.abi_version mismatch"; return MAMG_ERR_ARG; }
  if (p.AMG_type != MAMG_SA_AMG && p.AMG_type != MAMG_UA_AMG) { *err = "AMG_type must be SA_AMG or UA_AMG"; return MAMG_ERR_UNSUPPORTED; }
  if (p.cycle_type != MAMG_V_CYCLE && p.cycle_type != MAMG_W_CYCLE) { *err = "cycle_type must be V_CYCLE or W_CYCLE (AMLI/NL_AMLI/ADD not implemented)"; return MAMG_ERR_UNSUPPORTED; }
  if (p.smoother != MAMG_SMOOTHER_JACOBI && p.smoother != MAMG_SMOOTHER_L1DIAG && p.smoother != MAMG_SMOOTHER_JACOBI_RHO &&
      p.smoother != MAMG_SMOOTHER_GS && p.smoother != MAMG_SMOOTHER_SGS && p.smoother != MAMG_SMOOTHER_POLY) {
    *err = "smoother must be SMOOTHER_JACOBI, SMOOTHER_L1DIAG, SMOOTHER_JACOBI_RHO, SMOOTHER_GS, SMOOTHER_SGS or SMOOTHER_POLY";
    return MAMG_ERR_UNSUPPORTED;
  }
  if (p.smoother == MAMG_SMOOTHER_POLY &&
      (p.poly_degree < 1 || p.poly_degree > MAMG_POLY_MAX || !(p.poly_ratio > 1.0))) {
    *err = "SMOOTHER_POLY needs poly_degree in [1, 8] and poly_ratio > 1";
    return MAMG_ERR_ARG;
  }
  if ((p.smoother == MAMG_SMOOTHER_GS || p.smoother == MAMG_SMOOTHER_SGS) &&
      (p.num_functions != 2 || !p.node_block_smoother)) {
    *err = "multicolour GS/SGS smoothers are node-block smoothers: num_functions 2 and node_block_smoother 1";
    return MAMG_ERR_UNSUPPORTED;
  }
  if (p.aggregation_type != MAMG_MIS && p.aggregation_type != MAMG_HEM && p.aggregation_type != MAMG_VMB) {
    *err = "aggregation_type must be MIS (deterministic parallel MIS-2), HEM (parallel heavy-edge matching) or "
           "VMB (sequential Vanek-Mandel-Brezina, host setup): HEC/MWM are not implemented "
           "(parameters.to_gpu_profile maps a HAZmath dict explicitly)";
    return MAMG_ERR_UNSUPPORTED;
  }
  if (p.coarse_scaling != MAMG_OFF && p.coarse_scaling != MAMG_ON) { *err = "coarse_scaling must be OFF or ON"; return MAMG_ERR_ARG; }
  if (p.strength_measure != MAMG_STRENGTH_ROWMAX && p.strength_measure != MAMG_STRENGTH_DIAG) {
    *err = "strength_measure must be STRENGTH_ROWMAX (1) or STRENGTH_DIAG (0)";
    return MAMG_ERR_ARG;
  }
  if (p.coarse_solver != MAMG_COARSE_DENSE) { *err = "coarse_solver must be 32 (direct)"; return MAMG_ERR_UNSUPPORTED; }
  if (p.Schwarz_levels > 1) { *err = "Schwarz_levels > 1 not supported (seeds exist on level 0 only)"; return MAMG_ERR_UNSUPPORTED; }
  if (p.Schwarz_levels == 1) {
    // (after resolve_params) the level-0 blocks: the reference's overlapping
    // multiplicative form as node patches, additive overlapping rings, or the
    // level smoother on non-overlapping seed blocks
    const bool gsm = p.smoother == MAMG_SMOOTHER_GS || p.smoother == MAMG_SMOOTHER_SGS;
    const int t = p.Schwarz_type;
    if (t == MAMG_SCHWARZ_PATCHES) {
      if (p.num_functions != 2 || !p.node_block_smoother || p.Schwarz_maxlvl != 1) {
        *err = "SCHWARZ_PATCHES (multiplicative node-patch Schwarz) needs num_functions 2, node_block_smoother 1 "
               "and Schwarz_maxlvl 1";
        return MAMG_ERR_UNSUPPORTED;
      }
    } else if (t == MAMG_SCHWARZ_RINGS) {
      if (p.num_functions != 2 || !p.node_block_smoother || p.Schwarz_maxlvl < 1) {
        *err = "SCHWARZ_RINGS (multiplicative seed-ring Schwarz) needs num_functions 2, node_block_smoother 1 "
               "and Schwarz_maxlvl >= 1";
        return MAMG_ERR_UNSUPPORTED;
      }
      if (p.Schwarz_mmsize > RING_MAX_DOFS) {
        *err = "SCHWARZ_RINGS: Schwarz_mmsize " + std::to_string(p.Schwarz_mmsize) + " > " +
               std::to_string(RING_MAX_DOFS) + " dofs per block";
        return MAMG_ERR_UNSUPPORTED;
      }
    } else if (t == MAMG_SCHWARZ_SYMMETRIC || t == MAMG_SCHWARZ_FORWARD || t == MAMG_SCHWARZ_BACKWARD) {
      if (p.Schwarz_maxlvl >= 1) {
        *err = std::string("Schwarz_type ") + (t == MAMG_SCHWARZ_SYMMETRIC ? "SYMMETRIC" : t == MAMG_SCHWARZ_FORWARD ? "FORWARD" : "BACKWARD") +
               " with Schwarz_maxlvl " + std::to_string(p.Schwarz_maxlvl) +
               " is multiplicative Schwarz on overlapping seed + ring blocks; implemented as SYMMETRIC on nodal "
               "systems (num_functions 2, node_block_smoother 1: SCHWARZ_PATCHES / SCHWARZ_RINGS). "
               "Alternatives: SCHWARZ_ADDITIVE (the same overlapping blocks, additive) or SCHWARZ_SEED_BLOCKS "
               "(non-overlapping blocks, the level smoother)";
        return MAMG_ERR_UNSUPPORTED;
      }
      const int want = p.smoother == MAMG_SMOOTHER_SGS ? MAMG_SCHWARZ_SYMMETRIC
                       : p.smoother == MAMG_SMOOTHER_GS ? MAMG_SCHWARZ_FORWARD : -1;
      if (t != want) {
        *err = "Schwarz_type SYMMETRIC / FORWARD on the seeds' nodes (Schwarz_maxlvl 0) must match the smoother "
               "(SMOOTHER_SGS / SMOOTHER_GS); SCHWARZ_SEED_BLOCKS applies any level smoother to the seed blocks";
        return MAMG_ERR_UNSUPPORTED;
      }
    } else if (t == MAMG_SCHWARZ_ADDITIVE || t == MAMG_SCHWARZ_BLOCK_JACOBI) {
      if (gsm) {
        *err = "SCHWARZ_ADDITIVE / SCHWARZ_BLOCK_JACOBI are additive: use them with the Jacobi-family smoothers "
               "(SCHWARZ_SEED_BLOCKS or SCHWARZ_SYMMETRIC / FORWARD with Schwarz_maxlvl 0 for GS / SGS)";
        return MAMG_ERR_UNSUPPORTED;
      }
    } else if (t != MAMG_SCHWARZ_SEED_BLOCKS) {
      *err = "unknown Schwarz_type " + std::to_string(t);
      return MAMG_ERR_ARG;
    }
    if (p.Schwarz_maxlvl > 1 && t != MAMG_SCHWARZ_ADDITIVE && t != MAMG_SCHWARZ_RINGS) {
      *err = "Schwarz_maxlvl > 1 needs overlapping seed + ring blocks (SCHWARZ_SYMMETRIC on a nodal system, "
             "SCHWARZ_RINGS, or SCHWARZ_ADDITIVE); the non-overlapping seed blocks are the seeds' 1-rings";
      return MAMG_ERR_UNSUPPORTED;
    }
  }
  if (p.Schwarz_levels == 1 && p.Schwarz_mmsize < 1) { *err = "Schwarz_mmsize must be >= 1"; return MAMG_ERR_ARG; }
  if (p.Schwarz_maxlvl < 0) { *err = "Schwarz_maxlvl must be >= 0"; return MAMG_ERR_ARG; }
  if (p.Schwarz_maxlvl == 0 && (p.num_functions < 2 || !p.node_block_smoother)) {
    *err = "Schwarz_maxlvl 0 (seed blocks = the seeds' nodes) needs num_functions >= 2 and node_block_smoother 1";
    return MAMG_ERR_UNSUPPORTED;
  }
  if (p.max_levels < 1 || p.maxit < 1 || p.presmooth_iter < 1 || p.postsmooth_iter < 1 || p.coarse_dof < 1) {
    *err = "max_levels, maxit, presmooth_iter, postsmooth_iter, coarse_dof must be >= 1";
    return MAMG_ERR_ARG;
  }
  if (!(p.relaxation > 0.0) || !(p.sa_omega > 0.0) || !(p.strong_coupled >= 0.0)) { *err = "relaxation, sa_omega must be > 0, strong_coupled >= 0"; return MAMG_ERR_ARG; }
  if (p.num_functions < 1 || p.num_functions > 16) { *err = "num_functions must be in [1, 16]"; return MAMG_ERR_ARG; }
  if (p.spmv_lanes != 0 && (p.spmv_lanes < 2 || p.spmv_lanes > 64 || (p.spmv_lanes & (p.spmv_lanes - 1)))) {
    *err = "spmv_lanes must be 0 or a power of two in [2, 64]";
    return MAMG_ERR_ARG;
  }
  return MAMG_OK;
}

// SCHWARZ_PATCHES: one patch per node, so every node must hold a seed dof
// (the bidomain's idofs = every u2 dof, src/bidomain_3d.py:138)
int check_patch_seeds(const mamg_params& p, const int32_t* idofs, int64_t n_idofs, int64_t n, std::string* err) {
  if (p.Schwarz_levels < 1 || p.Schwarz_type != MAMG_SCHWARZ_PATCHES) return MAMG_OK;
  if (n < 2 || n % 2) { *err = "SCHWARZ_PATCHES needs a nodal system of even size (num_functions 2)"; return MAMG_ERR_ARG; }
  const int64_t nv = n / 2;
  std::vector<char> has(nv, 0);
  for (int64_t i = 0; i < n_idofs; ++i)
    if (idofs[i] >= 0 && idofs[i] < n) has[idofs[i] % nv] = 1;
  for (int64_t I = 0; I < nv; ++I)
    if (!has[I]) {
      *err = "SCHWARZ_PATCHES needs a seed dof (idofs) on every node; node " + std::to_string(I) + " has none";
      return MAMG_ERR_UNSUPPORTED;
    }
  return MAMG_OK;
}

// SCHWARZ_RINGS: seeds in range, and the dense blocks bounded
int check_ring_seeds(const mamg_params& p, const int32_t* idofs, int64_t n_idofs, int64_t n, std::string* err) {
  for (int64_t t = 0; t < n_idofs; ++t)
    if (idofs[t] < 0 || idofs[t] >= n) { *err = "idofs out of range"; return MAMG_ERR_ARG; }
  if ((double)n_idofs * p.Schwarz_mmsize * p.Schwarz_mmsize > 4e9) {
    *err = "SCHWARZ_RINGS (dense overlapping seed blocks) is for sparse seed sets: " + std::to_string(n_idofs) +
           " seeds of up to " + std::to_string(p.Schwarz_mmsize) + " dofs (limit: seeds x Schwarz_mmsize^2 <= 4e9, "
           "~400k seeds at mmsize 100); with a seed on every node use Schwarz_maxlvl 1 (the node patches, "
           "SCHWARZ_PATCHES) or the GPU profile (drivers -profile mi355x, parameters_metric_mi355x)";
    return MAMG_ERR_UNSUPPORTED;
  }
  return MAMG_OK;
}

int host_setup(const CsrView& A0, const int32_t* idofs, int64_t n_idofs,
               const mamg_params& p, Hierarchy* H, std::string* err) {
  int rc = check_params(p, err);
  if (rc) return rc;
  if ((rc = check_patch_seeds(p, idofs, n_idofs, A0.n, err))) return rc;
  if (A0.n != A0.m || A0.n <= 0) { *err = "A must be square and non-empty"; return MAMG_ERR_ARG; }
  for (int64_t i = 0; i < A0.n; ++i)
    if (A0.ptr[i + 1] < A0.ptr[i]) { *err = "rowptr not monotone"; return MAMG_ERR_ARG; }
  int64_t badcol = 0;
#pragma omp parallel for schedule(static) reduction(+ : badcol)
  for (int64_t i = 0; i < A0.n; ++i)
    for (int64_t k = A0.ptr[i]; k < A0.ptr[i + 1]; ++k) {
      const int32_t c = A0.col[k];
      badcol += (c < 0 || c >= A0.m || (k > A0.ptr[i] && c <= A0.col[k - 1]));
    }
  if (badcol) { *err = "column index out of range or not strictly increasing within a row"; return MAMG_ERR_ARG; }
  H->params = p;
  H->A0 = A0;
  H->levels.clear();
  H->seeds.clear();
  CsrView cur = A0;
  Csr next;
  for (int l = 0; l < p.max_levels; ++l) {
    H->levels.emplace_back();
    HostLevel& lev = H->levels.back();
    if (l > 0) { lev.A = std::move(next); next = Csr(); cur = lev.A.view(); }
    const int64_t n = cur.n;
    lev.n = n;
    bool last = (n <= p.coarse_dof) || (l == p.max_levels - 1);
    std::vector<int64_t> agg;
    int64_t nagg = 0;
    const int nf = p.num_functions;
    if (n % nf != 0) { *err = "matrix size not divisible by num_functions"; return MAMG_ERR_ARG; }
    if (!last) {
      if (nf > 1) {                 // nodal: aggregate the node graph
        Csr G;
        node_graph(cur, nf, &G);
        Strength S;
        strength(G.view(), p.strong_coupled, p.strength_measure == MAMG_STRENGTH_ROWMAX, &S);
        rc = p.aggregation_type == MAMG_HEM ? aggregate_hem(G.view(), S, l, &agg, &nagg, err)
             : p.aggregation_type == MAMG_VMB ? aggregate_vmb(G.view(), S, l, &agg, &nagg, err)
                                              : aggregate_mis2(G.view(), S, l, &agg, &nagg, err);
        if (rc) return rc;
        if (nagg == 0 || nf * nagg >= n) last = true;
      } else {
        Strength S;
        strength(cur, p.strong_coupled, p.strength_measure == MAMG_STRENGTH_ROWMAX, &S);
        rc = p.aggregation_type == MAMG_HEM ? aggregate_hem(cur, S, l, &agg, &nagg, err)
             : p.aggregation_type == MAMG_VMB ? aggregate_vmb(cur, S, l, &agg, &nagg, err)
                                              : aggregate_mis2(cur, S, l, &agg, &nagg, err);
        if (rc) return rc;
        if (nagg == 0 || nagg >= n) last = true;
      }
    }
    if (last) {
      if (n > p.max_coarse_dense) {
        *err = "coarsest level " + std::to_string(n) + " too large for dense solve";
        return MAMG_ERR_SETUP;
      }
      std::vector<double> dense(n * n, 0.0);
      for (int64_t i = 0; i < n; ++i)
        for (int64_t k = cur.ptr[i]; k < cur.ptr[i + 1]; ++k) dense[i * n + cur.col[k]] = cur.val[k];
      lev.Ainv.resize(n * n);
      if (!gauss_jordan(n, dense.data(), lev.Ainv.data())) { *err = "coarsest matrix not SPD"; return MAMG_ERR_SETUP; }
      lev.coarsest = true;
      break;
    }
    std::vector<double> dg(n), dinv(n);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) { dg[i] = diag_of(cur, i); dinv[i] = 1.0 / dg[i]; }
    const std::vector<double> rs = abs_rowsum(cur);
    const bool blockP = nf > 1 && p.sa_block_diag;
    const bool need_rho = (p.AMG_type == MAMG_SA_AMG && !blockP) || p.smoother == MAMG_SMOOTHER_JACOBI_RHO ||
                          p.smoother == MAMG_SMOOTHER_POLY;
    const double rho = need_rho ? rho_estimate(cur, dinv, rs, p.rho_iters) : 0.0;
    const bool rings = seed_blocks_on(p, l, idofs, n_idofs) && p.Schwarz_type == MAMG_SCHWARZ_RINGS;
    if (rings) {
      // seed rings: the level-0 Schwarz data are built with the apply layout
      // (device.hip build_rings); the node-block smoother stands in for W
      if ((rc = check_ring_seeds(p, idofs, n_idofs, n, err))) return rc;
      H->seeds.assign(idofs, idofs + n_idofs);
      std::vector<int64_t> bid;
      int64_t nb;
      node_blocks(n, nf, &bid, &nb);
      rc = block_smoother_from(cur, bid, nb, p, &lev.WB, err);
      if (rc) return rc;
    } else if (seed_blocks_on(p, l, idofs, n_idofs) && p.Schwarz_type == MAMG_SCHWARZ_ADDITIVE) {
      rc = overlap_smoother(cur, idofs, n_idofs, p, &lev.WB, err);
      if (rc) return rc;
    } else if (seed_blocks_on(p, l, idofs, n_idofs)) {
      rc = block_smoother(cur, idofs, n_idofs, p, &lev.WB, err);
      if (rc) return rc;
    } else if (nf > 1 && p.node_block_smoother) {
      std::vector<int64_t> bid;
      int64_t nb;
      node_blocks(n, nf, &bid, &nb);
      rc = block_smoother_from(cur, bid, nb, p, &lev.WB, err);
      if (rc) return rc;
    } else {
      lev.winv.resize(n);
#pragma omp parallel for schedule(static)
      for (int64_t i = 0; i < n; ++i) {
        double d;
        if (p.smoother == MAMG_SMOOTHER_JACOBI) d = dg[i];
        else if (p.smoother == MAMG_SMOOTHER_L1DIAG) d = rs[i];
        else d = dg[i] * rho;
        lev.winv[i] = p.relaxation / d;
      }
    }
    lev.agg = std::move(agg);
    lev.nagg = nagg;
    Csr T;
    if (nf > 1) tentative_nodal(lev.agg, nagg, nf, &T);
    else tentative(lev.agg, nagg, &T);
    if (p.AMG_type == MAMG_SA_AMG && blockP) {
      rc = smooth_prolongator_block(cur, T, nf, p, &lev.P, &lev.w_sa, err);
      if (rc) return rc;
    } else if (p.AMG_type == MAMG_SA_AMG) {
      const double w = p.sa_omega / rho;
      lev.w_sa = w;
      std::vector<double> c(n);
      for (int64_t i = 0; i < n; ++i) c[i] = w * dinv[i];
      smooth_prolongator(cur, T, c, &lev.P);
    } else {
      lev.P = std::move(T);
    }
    transpose(lev.P.view(), &lev.R);
    spgemm(cur, lev.P.view(), &lev.AP);
    spgemm(lev.R.view(), lev.AP.view(), &next);
    if (!p.post_fusion || nf != 2) lev.AP = Csr();
    if (p.print_level > 0)
      std::fprintf(stderr, "[mamg] level %d: n=%lld nnz=%lld nagg=%lld nnzP=%lld\n", l,
                   (long long)n, (long long)cur.nnz(), (long long)nagg, (long long)lev.P.nnz());
  }
  return MAMG_OK;
}

}  // namespace mamg
