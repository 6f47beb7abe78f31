// convert.cpp -- host-side layout conversion for the BSR2 device path
// (compiled by g++ with OpenMP, like the rest of the host code).
#include <omp.h>

#include <algorithm>

#include "host.h"

namespace mamg {

// ---- field-major CSR (rows f*nr+I, cols g*nc+J, 2 fields) -> 2x2 BSR -------
// node rows [r0, r1); block row I-r0 holds the distinct node columns J of the
// two rows f*nr+I (sorted), values (0,0) (0,1) (1,0) (1,1), absent = 0.
void to_bsr2_rows(const CsrView& M, int64_t nr, int64_t nc, int64_t r0, int64_t r1, HBsr* B) {
  const int64_t n = r1 - r0;
  B->nr = n;
  B->nc = nc;
  B->ptr.assign(n + 1, 0);
#pragma omp parallel
  {
    std::vector<int32_t> js;
#pragma omp for schedule(dynamic, 4096)
    for (int64_t I = r0; I < r1; ++I) {
      js.clear();
      for (int f = 0; f < 2; ++f) {
        const int64_t r = f * nr + I;
        for (int64_t k = M.ptr[r]; k < M.ptr[r + 1]; ++k) js.push_back((int32_t)(M.col[k] % nc));
      }
      std::sort(js.begin(), js.end());
      B->ptr[I - r0 + 1] = (int64_t)(std::unique(js.begin(), js.end()) - js.begin());
    }
  }
  for (int64_t i = 0; i < n; ++i) B->ptr[i + 1] += B->ptr[i];
  const int64_t nb = B->ptr[n];
  B->col.resize(nb);
  B->val.assign(4 * nb, 0.0);
#pragma omp parallel
  {
    std::vector<int32_t> js;
#pragma omp for schedule(dynamic, 4096)
    for (int64_t I = r0; I < r1; ++I) {
      js.clear();
      for (int f = 0; f < 2; ++f) {
        const int64_t r = f * nr + I;
        for (int64_t k = M.ptr[r]; k < M.ptr[r + 1]; ++k) js.push_back((int32_t)(M.col[k] % nc));
      }
      std::sort(js.begin(), js.end());
      js.erase(std::unique(js.begin(), js.end()), js.end());
      const int64_t o = B->ptr[I - r0];
      for (size_t t = 0; t < js.size(); ++t) B->col[o + t] = js[t];
      for (int f = 0; f < 2; ++f) {
        const int64_t r = f * nr + I;
        for (int64_t k = M.ptr[r]; k < M.ptr[r + 1]; ++k) {
          const int32_t J = (int32_t)(M.col[k] % nc);
          const int g = (int)(M.col[k] / nc);
          const int64_t t = std::lower_bound(js.begin(), js.end(), J) - js.begin();
          B->val[4 * (o + t) + 2 * f + g] = M.val[k];
        }
      }
    }
  }
}

void to_bsr2(const CsrView& M, int64_t nr, int64_t nc, HBsr* B) { to_bsr2_rows(M, nr, nc, 0, nr, B); }

void merge_bsr_rows(const HBsr& P, const HBsr& Q, HBsr* M) {
  const int64_t nr = P.nr;
  M->nr = nr;
  M->nc = P.nc;
  M->ptr.assign(2 * nr + 1, 0);
  for (int64_t I = 0; I < nr; ++I) {
    M->ptr[2 * I + 1] = M->ptr[2 * I] + (P.ptr[I + 1] - P.ptr[I]);
    M->ptr[2 * I + 2] = M->ptr[2 * I + 1] + (Q.ptr[I + 1] - Q.ptr[I]);
  }
  const int64_t nb = M->ptr[2 * nr];
  M->col.resize(nb);
  M->val.resize(4 * nb);
#pragma omp parallel for schedule(static)
  for (int64_t I = 0; I < nr; ++I) {
    int64_t d = M->ptr[2 * I];
    for (const HBsr* S : {&P, &Q})
      for (int64_t k = S->ptr[I]; k < S->ptr[I + 1]; ++k, ++d) {
        M->col[d] = S->col[k];
        for (int q = 0; q < 4; ++q) M->val[4 * d + q] = S->val[4 * k + q];
      }
  }
}

int to_sell(const HBsr& B, bool sym, int C, int sigma, HSell* S, std::string* err) {
  const int64_t nr = B.nr, ns = (nr + C - 1) / C;
  const bool merged = (int64_t)B.ptr.size() == 2 * nr + 1;
  auto row0 = [&](int64_t I, int64_t* a, int64_t* m, int64_t* e) {
    if (merged) { *a = B.ptr[2 * I]; *m = B.ptr[2 * I + 1]; *e = B.ptr[2 * I + 2]; }
    else { *a = B.ptr[I]; *m = *a; *e = B.ptr[I + 1]; }
  };
  S->perm.clear();
  if (sigma > 1) {   // sort rows by decreasing length inside windows of sigma rows
    S->perm.resize(nr);
#pragma omp parallel for schedule(static)
    for (int64_t w0 = 0; w0 < nr; w0 += sigma) {
      const int64_t w1 = std::min(nr, w0 + sigma);
      for (int64_t I = w0; I < w1; ++I) S->perm[I] = (int32_t)I;
      std::stable_sort(S->perm.begin() + w0, S->perm.begin() + w1, [&](int32_t x, int32_t y) {
        int64_t a, m, e, a2, m2, e2;
        row0(x, &a, &m, &e);
        row0(y, &a2, &m2, &e2);
        return e - a > e2 - a2;
      });
    }
  }
  auto row = [&](int64_t slot, int64_t* a, int64_t* m, int64_t* e) {
    row0(sigma > 1 ? S->perm[slot] : slot, a, m, e);
  };
  S->nr = nr;
  S->meta.assign(nr, 0);
  S->soff.assign(ns + 1, 0);
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
  for (int64_t s = 0; s < ns; ++s) {
    int64_t w = 0;
    for (int64_t I = s * C; I < std::min(nr, (s + 1) * C); ++I) {
      int64_t a, m, e;
      row(I, &a, &m, &e);
      if (e - a >= 0xffff) { bad = 1; continue; }
      S->meta[I] = (int32_t)((e - a) | ((m - a) << 16));
      w = std::max(w, e - a);
    }
    S->soff[s + 1] = C * w;
  }
  if (bad) { *err = "SELL: row longer than 65534 blocks"; return MAMG_ERR_UNSUPPORTED; }
  for (int64_t s = 0; s < ns; ++s) S->soff[s + 1] += S->soff[s];
  const int64_t nbs = S->soff[ns];
  S->nbs = nbs;
  const int per = sym ? 3 : 4;
  S->col.assign(nbs, 0);
  S->val.assign(per * nbs, 0.0);
#pragma omp parallel for schedule(static)
  for (int64_t I = 0; I < nr; ++I) {
    int64_t a, m, e;
    row(I, &a, &m, &e);
    int64_t kk = S->soff[I / C] + (I % C);
    for (int64_t k = a; k < e; ++k, kk += C) {
      S->col[kk] = B.col[k];
      const double* v = &B.val[4 * k];
      if (sym) {
        S->val[2 * kk] = v[0];
        S->val[2 * kk + 1] = v[3];
        S->val[2 * nbs + kk] = v[1];
      } else {
        for (int q = 0; q < 4; ++q) S->val[4 * kk + q] = v[q];
      }
    }
  }
  return MAMG_OK;
}

// W_B (or node-block smoother) -> one 2x2 block per node; false if some entry
// couples different nodes (then the BSR2 layout cannot fuse the smoother)
bool node_blocks_of(const CsrView& W, int64_t nv, std::vector<double>* blk) {
  blk->assign(4 * nv, 0.0);
  for (int64_t i = 0; i < W.n; ++i) {
    const int64_t I = i % nv, f = i / nv;
    for (int64_t k = W.ptr[i]; k < W.ptr[i + 1]; ++k) {
      const int64_t j = W.col[k];
      if (j % nv != I) return false;
      (*blk)[4 * I + 2 * f + j / nv] = W.val[k];
    }
  }
  return true;
}

}  // namespace mamg
