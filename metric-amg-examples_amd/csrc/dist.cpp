// dist.cpp -- row-partition plan for the multi-GPU V-cycle.
//
// Every rank runs the same deterministic host setup, so the plan of every rank
// is computable locally (no setup-time communication).  Per level l, nodes are
// split into nranks contiguous ranges of equal size (level 0 = z-slabs of the
// structured mesh; coarse aggregates are numbered by root index, so their
// ranges are slab-like too).  A level is *replicated* (computed redundantly on
// every rank, no exchange) once it has <= rep_nodes nodes, and so are all
// coarser levels; the coarsest (dense solve) always is.
//
// Rank-local data of a distributed level l (node-interleaved vectors
// [owned | ghost], ghosts sorted by global id, hence grouped by owner rank):
//   A_loc : owned rows, columns in local numbering
//   P_loc : owned fine rows, columns = level l+1 local (or global if l+1 is
//           replicated)
//   Rp_loc: transpose of P_loc -- rows = level l+1 [owned | ghost] (or all
//           nodes), columns = owned fine nodes.  R r is formed as partial
//           sums, then ghost partials are sent to their owners and added in
//           rank order (deterministic).
//   PA_loc: (post fusion) P_loc and AP_loc = (A P)_loc merged row by row, same
//           columns as P_loc: the fused post sweep x1 + P e + W (r1 - AP e)
//           needs only owned x1, r1 and e's ghosts (no fine-level halo)
//   ghosts(l) = external columns of A_loc  U  external columns of P_{l-1} loc
//               (U external columns of AP_{l-1} loc with post fusion)
//   send list to q = the owned nodes that are ghosts of q, in q's order.
// Only owned rows are converted to blocks (no global copy of A_0 per rank);
// ghost sets of all ranks come straight from the field-major CSR.
#include <omp.h>

#include <algorithm>
#include <numeric>

#include "dist.h"

namespace mamg {
namespace {

inline int owner_of(const std::vector<int64_t>& own, int64_t J) {
  return (int)(std::upper_bound(own.begin(), own.end(), J) - own.begin()) - 1;
}

// node columns (mod nc) of field-major CSR rows f*nr+I, I in [r0,r1), outside [o0,o1)
void external_node_cols(const CsrView& M, int64_t nr, int64_t nc, int64_t r0, int64_t r1,
                        int64_t o0, int64_t o1, std::vector<int64_t>* out) {
  std::vector<int64_t> v;
  for (int f = 0; f < 2; ++f)
    for (int64_t I = r0; I < r1; ++I) {
      const int64_t r = f * nr + I;
      for (int64_t k = M.ptr[r]; k < M.ptr[r + 1]; ++k) {
        const int64_t J = M.col[k] % nc;
        if (J < o0 || J >= o1) v.push_back(J);
      }
    }
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  out->insert(out->end(), v.begin(), v.end());
}

void sort_unique(std::vector<int64_t>* v) {
  std::sort(v->begin(), v->end());
  v->erase(std::unique(v->begin(), v->end()), v->end());
}

// remap the columns of a (row-local) block matrix in place, keeping each
// row's blocks sorted by local column
template <class F>
void remap_cols(HBsr* B, int64_t nc_local, F map) {
  B->nc = nc_local;
  std::vector<std::pair<int32_t, int64_t>> e;
  std::vector<double> v;
  for (int64_t I = 0; I < B->nr; ++I) {
    const int64_t p0 = B->ptr[I], p1 = B->ptr[I + 1];
    e.clear();
    for (int64_t k = p0; k < p1; ++k) e.emplace_back((int32_t)map(B->col[k]), k);
    std::sort(e.begin(), e.end());
    v.assign(B->val.begin() + 4 * p0, B->val.begin() + 4 * p1);
    for (int64_t t = 0; t < p1 - p0; ++t) {
      B->col[p0 + t] = e[t].first;
      for (int q = 0; q < 4; ++q) B->val[4 * (p0 + t) + q] = v[4 * (e[t].second - p0) + q];
    }
  }
}

// transpose a (nr x nc) 2x2-block matrix: blocks transposed too
void transpose_bsr(const HBsr& B, HBsr* T) {
  T->nr = B.nc;
  T->nc = B.nr;
  T->ptr.assign(T->nr + 1, 0);
  const int64_t nb = B.ptr[B.nr];
  for (int64_t k = 0; k < nb; ++k) T->ptr[B.col[k] + 1]++;
  for (int64_t i = 0; i < T->nr; ++i) T->ptr[i + 1] += T->ptr[i];
  T->col.resize(nb);
  T->val.resize(4 * nb);
  std::vector<int64_t> nx(T->ptr.begin(), T->ptr.end() - 1);
  for (int64_t I = 0; I < B.nr; ++I)
    for (int64_t k = B.ptr[I]; k < B.ptr[I + 1]; ++k) {
      const int64_t d = nx[B.col[k]]++;
      T->col[d] = (int32_t)I;
      const double* v = &B.val[4 * k];
      T->val[4 * d + 0] = v[0];
      T->val[4 * d + 1] = v[2];
      T->val[4 * d + 2] = v[1];
      T->val[4 * d + 3] = v[3];
    }
}

}  // namespace

void kmerge_rows(const HBsr& P, const HBsr& AP, const std::vector<double>& W, HBsr* K) {
  const int64_t nr = P.nr;
  K->nr = nr;
  K->nc = P.nc;
  K->ptr.assign(nr + 1, 0);
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1) {
      for (int64_t I = 0; I < nr; ++I) K->ptr[I + 1] += K->ptr[I];
      K->col.resize(K->ptr[nr]);
      K->val.resize(4 * K->ptr[nr]);
    }
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t I = 0; I < nr; ++I) {
      int64_t a = P.ptr[I], ae = P.ptr[I + 1], b = AP.ptr[I], be = AP.ptr[I + 1];
      int64_t o = pass ? K->ptr[I] : 0;
      const double* w = &W[4 * I];
      const double zero[4] = {0.0, 0.0, 0.0, 0.0};
      while (a < ae || b < be) {
        const int32_t ja = a < ae ? P.col[a] : INT32_MAX, jb = b < be ? AP.col[b] : INT32_MAX;
        const int32_t j = std::min(ja, jb);
        if (pass) {   // same operation order as device.hip kmerge_kernel
          const double* p = ja == j ? &P.val[4 * a] : zero;
          const double* q = jb == j ? &AP.val[4 * b] : zero;
          double* k = &K->val[4 * o];
          k[0] = p[0] - (w[0] * q[0] + w[1] * q[2]);
          k[1] = p[1] - (w[0] * q[1] + w[1] * q[3]);
          k[2] = p[2] - (w[2] * q[0] + w[3] * q[2]);
          k[3] = p[3] - (w[2] * q[1] + w[3] * q[3]);
          K->col[o] = j;
        }
        if (ja == j) ++a;
        if (jb == j) ++b;
        ++o;
      }
      if (!pass) K->ptr[I + 1] = o;
    }
  }
}

void dist_ranges(const std::vector<int64_t>& nv, const std::vector<char>& coarsest, int nranks,
                 int64_t rep_nodes, std::vector<std::vector<int64_t>>* own, std::vector<char>* rep) {
  const size_t nl = nv.size();
  own->assign(nl, std::vector<int64_t>(nranks + 1));
  rep->assign(nl, 0);
  bool r = false;
  for (size_t l = 0; l < nl; ++l) {
    if (l > 0 && (nv[l] <= rep_nodes || coarsest[l])) r = true;
    (*rep)[l] = r;
    for (int q = 0; q <= nranks; ++q) (*own)[l][q] = r ? (q == 0 ? 0 : nv[l]) : (nv[l] * q) / nranks;
  }
}

int build_dist_plan(const Hierarchy& H, const CsrView& A0, int rank, int nranks, int64_t rep_nodes,
                    bool fuse, DistPlan* plan, std::string* err, bool kpost, double kw,
                    const GhostLists* pre, bool meta_only) {
  // K = P - (kw W) AP: the first post-smoothing step's smoother (device.hip
  // poly_scaled: kw W elementwise, then the merge; bitwise the single-GPU K)
  auto kmerge_kw = [kw](const HBsr& P, const HBsr& AP, const std::vector<double>& W, HBsr* K) {
    if (kw == 1.0) { kmerge_rows(P, AP, W, K); return; }
    std::vector<double> Ws(W.size());
    for (size_t i = 0; i < W.size(); ++i) Ws[i] = kw * W[i];
    kmerge_rows(P, AP, Ws, K);
  };
  if (nranks < 1 || rank < 0 || rank >= nranks) { *err = "bad rank/nranks"; return MAMG_ERR_ARG; }
  if (H.params.num_functions != 2) { *err = "multi-GPU path needs num_functions == 2 (BSR2 layout)"; return MAMG_ERR_UNSUPPORTED; }
  const int nl = (int)H.levels.size();
  if (nl < 2) { *err = "multi-GPU path needs at least two levels"; return MAMG_ERR_UNSUPPORTED; }
  if (meta_only && !pre) { *err = "meta-only plan needs precomputed ghost lists"; return MAMG_ERR_ARG; }
  for (int l = 0; l + 1 < nl && fuse && !meta_only; ++l)
    if (H.levels[l].AP.n != H.levels[l].n) fuse = false;   // A P not kept by the setup
  plan->rank = rank;
  plan->nranks = nranks;
  plan->fuse = fuse;
  plan->kpost = kpost;
  plan->levels.assign(nl, DistLevel());
  auto Aview = [&](int l) { return l == 0 ? A0 : H.A(l); };
  {
    std::vector<int64_t> nv(nl);
    std::vector<char> co(nl), rep;
    std::vector<std::vector<int64_t>> own;
    for (int l = 0; l < nl; ++l) { nv[l] = H.levels[l].n / 2; co[l] = H.levels[l].coarsest; }
    dist_ranges(nv, co, nranks, rep_nodes, &own, &rep);
    for (int l = 0; l < nl; ++l) {
      const HostLevel& hl = H.levels[l];
      DistLevel& D = plan->levels[l];
      D.nv = nv[l];
      D.coarsest = hl.coarsest;
      D.replicated = rep[l];
      D.own = own[l];
      if (!meta_only && !hl.coarsest && hl.WB.n == 0 && hl.Wn.empty()) {
        *err = "multi-GPU path needs node-block smoothers on every level";
        return MAMG_ERR_UNSUPPORTED;
      }
    }
  }
  // ghost lists of every rank on distributed levels (send lists need them)
  GhostLists ghosts_here;
  if (!pre) ghosts_here.assign(nl, std::vector<std::vector<int64_t>>(nranks));
  const GhostLists& ghosts = pre ? *pre : ghosts_here;
  if (pre && ((int)pre->size() != nl || (*pre)[0].size() != (size_t)nranks)) {
    *err = "precomputed ghost lists do not match the hierarchy";
    return MAMG_ERR_ARG;
  }
#pragma omp parallel for collapse(2) schedule(dynamic, 1)
  for (int l = 0; l < nl; ++l)
    for (int q = 0; q < nranks; ++q) {
      const DistLevel& D = plan->levels[l];
      if (pre || D.replicated) continue;
      const int64_t o0 = D.own[q], o1 = D.own[q + 1];
      std::vector<int64_t> g;
      external_node_cols(Aview(l), D.nv, D.nv, o0, o1, o0, o1, &g);
      if (l > 0) {
        const DistLevel& F = plan->levels[l - 1];
        external_node_cols(H.levels[l - 1].P.view(), F.nv, D.nv, F.own[q], F.own[q + 1], o0, o1, &g);
        if (fuse)
          external_node_cols(H.levels[l - 1].AP.view(), F.nv, D.nv, F.own[q], F.own[q + 1], o0, o1, &g);
      }
      sort_unique(&g);
      ghosts_here[l][q] = std::move(g);
    }
  for (int l = 0; l < nl; ++l) {
    DistLevel& D = plan->levels[l];
    const HostLevel& hl = H.levels[l];
    if (meta_only && D.replicated) {   // ranges and lists only
      D.o0 = 0; D.o1 = D.nv; D.nloc = D.nv;
      D.ghost_off.assign(nranks + 1, 0);
      D.send_off.assign(nranks + 1, 0);
      continue;
    }
    // smoother blocks: Wfull holds nodes [w0, w0 + Wfull.size()/4)
    std::vector<double> Wfull;
    int64_t w0 = 0;
    if (!meta_only) {
      if (!hl.Wn.empty()) {
        Wfull = hl.Wn;
        w0 = hl.wn0;
      } else if (!hl.coarsest && !node_blocks_of(hl.WB.view(), D.nv, &Wfull)) {
        *err = "multi-GPU path needs node-block smoothers on every level";
        return MAMG_ERR_UNSUPPORTED;
      }
    }
    const int64_t w1 = w0 + (int64_t)Wfull.size() / 4;
    if (D.replicated) {
      D.o0 = 0; D.o1 = D.nv; D.nloc = D.nv;
      if (!hl.coarsest && (w0 != 0 || w1 != D.nv)) {
        *err = "smoother slice does not cover a replicated level";
        return MAMG_ERR_ARG;
      }
      to_bsr2(Aview(l), D.nv, D.nv, &D.A);
      D.W = std::move(Wfull);
      D.ghost_off.assign(nranks + 1, 0);
      D.send_off.assign(nranks + 1, 0);
      continue;
    }
    D.o0 = D.own[rank];
    D.o1 = D.own[rank + 1];
    D.nloc = D.o1 - D.o0;
    D.ghosts = ghosts[l][rank];
    D.ghost_off.assign(nranks + 1, 0);
    for (int64_t g : D.ghosts) D.ghost_off[owner_of(D.own, g) + 1]++;
    for (int q = 0; q < nranks; ++q) D.ghost_off[q + 1] += D.ghost_off[q];
    D.send_off.assign(nranks + 1, 0);
    D.send_idx.clear();
    for (int q = 0; q < nranks; ++q) {
      if (q != rank)
        for (int64_t g : ghosts[l][q])
          if (g >= D.o0 && g < D.o1) D.send_idx.push_back(g - D.o0);
      D.send_off[q + 1] = (int64_t)D.send_idx.size();
    }
    if (meta_only) continue;
    const int64_t o0 = D.o0, o1 = D.o1, nloc = D.nloc;
    const std::vector<int64_t>& gl = D.ghosts;
    to_bsr2_rows(Aview(l), D.nv, D.nv, o0, o1, &D.A);
    remap_cols(&D.A, nloc + (int64_t)gl.size(), [&](int64_t J) -> int64_t {
      if (J >= o0 && J < o1) return J - o0;
      return nloc + (std::lower_bound(gl.begin(), gl.end(), J) - gl.begin());
    });
    if (o0 < w0 || o1 > w1) {
      *err = "smoother slice does not cover the owned nodes";
      return MAMG_ERR_ARG;
    }
    D.W.assign(Wfull.begin() + 4 * (o0 - w0), Wfull.begin() + 4 * (o1 - w0));
  }
  // P_loc / Rp_loc (need the level l+1 numbering)
  for (int l = 0; l + 1 < nl && !meta_only; ++l) {
    DistLevel& D = plan->levels[l];
    const DistLevel& C = plan->levels[l + 1];
    const CsrView Pv = H.levels[l].P.view();
    if (D.replicated) {
      to_bsr2(Pv, D.nv, C.nv, &D.P);
      transpose_bsr(D.P, &D.Rp);
      if (fuse) {
        HBsr AP;
        to_bsr2(H.levels[l].AP.view(), D.nv, C.nv, &AP);
        if (kpost) kmerge_kw(D.P, AP, D.W, &D.K);
        else merge_bsr_rows(D.P, AP, &D.PA);
      }
      continue;
    }
    const int64_t c0 = C.o0, c1 = C.o1, cnloc = C.nloc;
    const std::vector<int64_t>& cg = C.ghosts;
    const bool crep = C.replicated;
    to_bsr2_rows(Pv, D.nv, C.nv, D.o0, D.o1, &D.P);
    const int64_t ncl = crep ? C.nv : cnloc + (int64_t)cg.size();
    auto cmap = [&](int64_t J) -> int64_t {
      if (crep) return J;
      if (J >= c0 && J < c1) return J - c0;
      return cnloc + (std::lower_bound(cg.begin(), cg.end(), J) - cg.begin());
    };
    remap_cols(&D.P, ncl, cmap);
    transpose_bsr(D.P, &D.Rp);
    if (fuse) {
      HBsr AP;
      to_bsr2_rows(H.levels[l].AP.view(), D.nv, C.nv, D.o0, D.o1, &AP);
      remap_cols(&AP, ncl, cmap);
      if (kpost) kmerge_kw(D.P, AP, D.W, &D.K);
      else merge_bsr_rows(D.P, AP, &D.PA);
    }
  }
  return MAMG_OK;
}

}  // namespace mamg
