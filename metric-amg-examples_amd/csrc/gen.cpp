// gen.cpp -- monolithic bidomain system on dolfin's structured P1 meshes.
//
// Restates the matrix the reference assembles with FEniCS/fenics_ii:
//   a00 = k1 (grad u1, grad v1) + g (u1, v1), a01 = a10 = -g (u, v),
//   a11 = k2 (grad u2, grad v2) + g (u2, v2)   (src/bidomain_2d.py:64-68)
// on UnitSquareMesh(n,n) 'right' / UnitCubeMesh(n,n,n) (src/utils.py:149-182),
// block order [u1; u2] (ii_convert, src/bidomain_3d.py:124,138), Dirichlet
// tags 1,2 = x=0,1 (2-D) / z=0,1 (3-D) (src/bidomain_2d.py:73,
// src/utils.py:159-160,177-178) eliminated symmetrically with unit diagonal.
// Dofs are numbered by vertex (dolfin's serial dof reordering is not
// reproducible without dolfin; documented in DESIGN.md).
//
// Every cell is a monotone lattice path (Kuhn split); its P1 stiffness is
// kfac * tridiag(1,2,..,2,1 / -1) and its mass mfac * (1 + delta_ij).  The
// assembled matrix is formed from exact integer counts, so the values are
// independent of assembly order and bitwise equal to
// oracle/mamg_oracle.py:bidomain_system.
#include <algorithm>
#include <array>
#include <cstring>

#include "host.h"

namespace mamg {
namespace {

struct Stencil {       // one vertex row of the single-field integer stencil
  int cnt = 0;
  std::array<int64_t, 27> col;
  std::array<int64_t, 27> cK;
  std::array<int64_t, 27> cM;
};

// local stiffness (integer) of a path simplex with dim+1 vertices
inline int kpath(int dim, int a, int b) {
  if (a == b) return (a == 0 || a == dim) ? 1 : 2;
  return (a - b == 1 || b - a == 1) ? -1 : 0;
}

void vertex_stencil(int dim, int64_t n, int64_t v, Stencil* st) {
  const int64_t nn = n + 1;
  int64_t c[3] = {v % nn, (v / nn) % nn, dim == 3 ? v / (nn * nn) : 0};
  const int64_t stride[3] = {1, nn, nn * nn};
  // accumulate on a {-1,0,1}^dim offset grid
  int64_t accK[27] = {0}, accM[27] = {0};
  bool used[27] = {false};
  int perms3[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
  int perms2[2][3] = {{0, 1, 0}, {1, 0, 0}};
  const int ncorner = dim == 3 ? 8 : 4;
  const int npath = dim == 3 ? 6 : 2;
  for (int q = 0; q < ncorner; ++q) {
    int d[3] = {q & 1, (q >> 1) & 1, (q >> 2) & 1};   // v's position in cell
    bool ok = true;
    for (int k = 0; k < dim; ++k) {
      int64_t lo = c[k] - d[k];
      if (lo < 0 || lo >= n) ok = false;
    }
    if (!ok) continue;
    for (int pth = 0; pth < npath; ++pth) {
      const int* perm = dim == 3 ? perms3[pth] : perms2[pth];
      int pv[4][3] = {{0, 0, 0}};
      for (int t = 1; t <= dim; ++t) {
        for (int k = 0; k < 3; ++k) pv[t][k] = pv[t - 1][k];
        pv[t][perm[t - 1]] += 1;
      }
      int t_me = -1;
      for (int t = 0; t <= dim; ++t)
        if (pv[t][0] == d[0] && pv[t][1] == d[1] && pv[t][2] == d[2]) t_me = t;
      if (t_me < 0) continue;
      for (int s = 0; s <= dim; ++s) {
        int off[3] = {pv[s][0] - d[0], pv[s][1] - d[1], pv[s][2] - d[2]};
        int slot = (off[0] + 1) + 3 * (off[1] + 1) + 9 * (off[2] + 1);
        used[slot] = true;
        accK[slot] += kpath(dim, t_me, s);
        accM[slot] += (t_me == s) ? 2 : 1;
      }
    }
  }
  // emit in increasing column order: slot order dz, dy, dx ascending
  st->cnt = 0;
  for (int dz = -1; dz <= 1; ++dz)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        int slot = (dx + 1) + 3 * (dy + 1) + 9 * (dz + 1);
        if (!used[slot]) continue;
        st->col[st->cnt] = v + dx * stride[0] + dy * stride[1] + dz * stride[2];
        st->cK[st->cnt] = accK[slot];
        st->cM[st->cnt] = accM[slot];
        st->cnt++;
      }
}

inline bool is_bc_vertex(int dim, int64_t n, int64_t v) {
  const int64_t nn = n + 1;
  int64_t a = dim == 2 ? v % nn : v / (nn * nn);
  return a == 0 || a == n;
}

}  // namespace

int gen_bidomain_size(int dim, int64_t n, int64_t* nrows, int64_t* nnz) {
  if ((dim != 2 && dim != 3) || n < 1) return MAMG_ERR_ARG;
  const int64_t nn = n + 1;
  const int64_t nv = dim == 3 ? nn * nn * nn : nn * nn;
  int64_t total = 0;
#pragma omp parallel for reduction(+ : total) schedule(static)
  for (int64_t v = 0; v < nv; ++v) {
    if (is_bc_vertex(dim, n, v)) { total += 2; continue; }
    Stencil st;
    vertex_stencil(dim, n, v, &st);
    int64_t k = 0;
    for (int j = 0; j < st.cnt; ++j)
      if (!is_bc_vertex(dim, n, st.col[j])) ++k;
    total += 4 * k;                       // two rows, two blocks each
  }
  *nrows = 2 * nv;
  *nnz = total;
  return MAMG_OK;
}

int gen_bidomain(int dim, int64_t n, double gamma, double k1, double k2,
                 int64_t* rowptr, int32_t* colind, double* values) {
  if ((dim != 2 && dim != 3) || n < 1) return MAMG_ERR_ARG;
  const int64_t nn = n + 1;
  const int64_t nv = dim == 3 ? nn * nn * nn : nn * nn;
  if (2 * nv >= (int64_t)INT32_MAX) return MAMG_ERR_ARG;
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
  // pass 1: row lengths
  std::vector<int32_t> len(nv);
#pragma omp parallel for schedule(static)
  for (int64_t v = 0; v < nv; ++v) {
    if (is_bc_vertex(dim, n, v)) { len[v] = 1; continue; }
    Stencil st;
    vertex_stencil(dim, n, v, &st);
    int k = 0;
    for (int j = 0; j < st.cnt; ++j)
      if (!is_bc_vertex(dim, n, st.col[j])) ++k;
    len[v] = 2 * k;
  }
  // rows 0..nv-1 (u1) then nv..2nv-1 (u2); row v and v+nv have equal length
  rowptr[0] = 0;
  for (int64_t v = 0; v < nv; ++v) rowptr[v + 1] = rowptr[v] + len[v];
  for (int64_t v = 0; v < nv; ++v) rowptr[nv + v + 1] = rowptr[nv + v] + len[v];
#pragma omp parallel for schedule(static)
  for (int64_t v = 0; v < nv; ++v) {
    int64_t p1 = rowptr[v], p2 = rowptr[nv + v];
    if (is_bc_vertex(dim, n, v)) {
      colind[p1] = (int32_t)v; values[p1] = 1.0;
      colind[p2] = (int32_t)(v + nv); values[p2] = 1.0;
      continue;
    }
    Stencil st;
    vertex_stencil(dim, n, v, &st);
    int k = 0;
    int64_t cols[27];
    double a11[27], a22[27], a12[27];
    for (int j = 0; j < st.cnt; ++j) {
      if (is_bc_vertex(dim, n, st.col[j])) continue;
      const double fK = (double)st.cK[j], fM = (double)st.cM[j];
      cols[k] = st.col[j];
      a11[k] = kf1 * fK + mf * fM;
      a22[k] = kf2 * fK + mf * fM;
      a12[k] = -(mf * fM);
      ++k;
    }
    for (int j = 0; j < k; ++j) {        // u1 row: [A11 | A12]
      colind[p1 + j] = (int32_t)cols[j];
      values[p1 + j] = a11[j];
      colind[p1 + k + j] = (int32_t)(cols[j] + nv);
      values[p1 + k + j] = a12[j];
    }
    for (int j = 0; j < k; ++j) {        // u2 row: [A21 | A22]
      colind[p2 + j] = (int32_t)cols[j];
      values[p2 + j] = a12[j];
      colind[p2 + k + j] = (int32_t)(cols[j] + nv);
      values[p2 + k + j] = a22[j];
    }
  }
  return MAMG_OK;
}

}  // namespace mamg
