// mms.cpp -- manufactured solution of the bidomain drivers: right-hand side
// (load + flux terms + Dirichlet lifting) and H1 errors on the generator's
// meshes (gen.cpp numbering: vertex v = x + (n+1) y + (n+1)^2 z, dofs [u1; u2]).
//
// Restates src/bidomain_2d.py:7-49 (setup_mms), :51-99 (get_system: loads,
// full-flux Neumann terms on tags 3, 4, Dirichlet u = exact on tags 1, 2),
// :239-256 (errornorm 'H1'), and src/bidomain_3d.py:7-49 (3-D solution):
//   2-D u1 = cos(pi (x + y)),      u2 = sin(pi (x - y))
//   3-D u1 = cos(pi (x + y + 2z)), u2 = sin(pi (x - y + z))
//   f1 = k1 pi^2 |a|^2 u1 + g (u1 - u2),  f2 = k2 pi^2 |c|^2 u2 + g (u2 - u1).
// Integrals: collapsed Gauss-Legendre (3 points per direction) on every Kuhn
// simplex -- the rule metric-amg-examples_amd/mms.py uses, which tests check
// this file against.  The Dirichlet rows are those gen.cpp eliminates:
// b = F - A[:, D] g off D, b = g on D.
#include <cmath>
#include <cstring>
#include <vector>

#include "host.h"

namespace mamg {
namespace {

struct Exact {
  int dim;
  double k1, k2, g, a[3], c[3], a2, c2;
  Exact(int d, double kappa1, double kappa2, double gamma) : dim(d), k1(kappa1), k2(kappa2), g(gamma) {
    const double A2[3] = {1, 1, 0}, C2[3] = {1, -1, 0}, A3[3] = {1, 1, 2}, C3[3] = {1, -1, 1};
    for (int k = 0; k < 3; ++k) { a[k] = d == 2 ? A2[k] : A3[k]; c[k] = d == 2 ? C2[k] : C3[k]; }
    a2 = c2 = 0.0;
    for (int k = 0; k < d; ++k) { a2 += a[k] * a[k]; c2 += c[k] * c[k]; }
  }
  // values, gradients (may be null) at x
  void eval(const double* x, double* u1, double* u2, double* g1, double* g2) const {
    double pa = 0.0, pc = 0.0;
    for (int k = 0; k < dim; ++k) { pa += x[k] * a[k]; pc += x[k] * c[k]; }
    pa *= M_PI;
    pc *= M_PI;
    *u1 = std::cos(pa);
    *u2 = std::sin(pc);
    if (g1) {
      const double sa = -M_PI * std::sin(pa), cc = M_PI * std::cos(pc);
      for (int k = 0; k < dim; ++k) { g1[k] = sa * a[k]; g2[k] = cc * c[k]; }
    }
  }
  void load(const double* x, double* f1, double* f2) const {
    double u1, u2;
    eval(x, &u1, &u2, nullptr, nullptr);
    *f1 = k1 * M_PI * M_PI * a2 * u1 + g * (u1 - u2);
    *f2 = k2 * M_PI * M_PI * c2 * u2 + g * (u2 - u1);
  }
};

// collapsed Gauss-Legendre rule on the reference d-simplex: barycentric
// coordinates and weights (sum 1/d!); x_k = u_k prod_{j<k} (1 - u_j)
struct Rule {
  int np = 0;
  double lam[27][4];
  double w[27];
};

Rule simplex_rule(int d) {
  const double t3[3] = {0.5 * (1.0 - std::sqrt(0.6)), 0.5, 0.5 * (1.0 + std::sqrt(0.6))};
  const double w3[3] = {5.0 / 18.0, 8.0 / 18.0, 5.0 / 18.0};
  Rule R;
  int idx[3] = {0, 0, 0};
  int total = 1;
  for (int k = 0; k < d; ++k) total *= 3;
  for (int p = 0; p < total; ++p) {
    int r = p;
    for (int k = d - 1; k >= 0; --k) { idx[k] = r % 3; r /= 3; }   // first axis slowest
    double wt = 1.0, scale = 1.0, sum = 0.0, x[3];
    for (int k = 0; k < d; ++k) wt *= w3[idx[k]];
    for (int k = 0; k < d; ++k) {
      const double u = t3[idx[k]];
      x[k] = u * scale;
      sum += x[k];
      if (k < d - 1) wt *= std::pow(1.0 - u, d - 1 - k);
      scale *= 1.0 - u;
    }
    R.lam[p][0] = 1.0 - sum;
    for (int k = 0; k < d; ++k) R.lam[p][k + 1] = x[k];
    R.w[p] = wt;
  }
  R.np = total;
  return R;
}

// Kuhn path simplices of a d-cube: vertex offsets pv[path][t][axis]
int kuhn_paths(int d, int pv[6][4][3]) {
  const int perms3[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
  const int perms2[2][3] = {{0, 1, 0}, {1, 0, 0}};
  const int np = d == 3 ? 6 : d == 2 ? 2 : 1;
  for (int p = 0; p < np; ++p) {
    const int* perm = d == 3 ? perms3[p] : perms2[p];
    for (int k = 0; k < 3; ++k) pv[p][0][k] = 0;
    for (int t = 1; t <= d; ++t) {
      for (int k = 0; k < 3; ++k) pv[p][t][k] = pv[p][t - 1][k];
      pv[p][t][d == 1 ? 0 : perm[t - 1]] += 1;
    }
  }
  return np;
}

struct Mesh {
  int dim;
  int64_t n, nn, nv;
  double h;
  int64_t stride[3];
  Mesh(int d, int64_t cells) : dim(d), n(cells), nn(cells + 1), h(1.0 / (double)cells) {
    stride[0] = 1; stride[1] = nn; stride[2] = nn * nn;
    nv = d == 3 ? nn * nn * nn : nn * nn;
  }
  int dax() const { return dim == 2 ? 0 : 2; }      // Dirichlet axis (tags 1, 2)
  int64_t vid(const int64_t* c) const {
    int64_t v = 0;
    for (int k = 0; k < dim; ++k) v += c[k] * stride[k];
    return v;
  }
  bool dirichlet(int64_t v) const {
    const int64_t a = dim == 2 ? v % nn : v / (nn * nn);
    return a == 0 || a == n;
  }
};

}  // namespace

int gen_bidomain_mms(int dim, int64_t n, double gamma, double k1, double k2, double* b) {
  if ((dim != 2 && dim != 3) || n < 1) return MAMG_ERR_ARG;
  const Mesh m(dim, n);
  const Exact ex(dim, k1, k2, gamma);
  const Rule R = simplex_rule(dim), FR = simplex_rule(dim - 1);
  int pv[6][4][3];
  const int npath = kuhn_paths(dim, pv);
  const int64_t nv = m.nv;
  double* b1 = b;
  double* b2 = b + nv;
  std::memset(b, 0, 2 * nv * sizeof(double));
  const double vol = std::pow(m.h, dim);
  // volume loads: planes of cells along the slowest axis, even planes then
  // odd ones (cells two planes apart share no vertex)
  const int slow = dim - 1;
  for (int parity = 0; parity < 2; ++parity) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t p = parity; p < n; p += 2) {
      int64_t c[3] = {0, 0, 0};
      c[slow] = p;
      const int64_t ninplane = dim == 3 ? n * n : n;
      for (int64_t q = 0; q < ninplane; ++q) {
        c[0] = q % n;
        if (dim == 3) c[1] = q / n;
        for (int pa = 0; pa < npath; ++pa) {
          int64_t vids[4];
          double X[4][3];
          for (int t = 0; t <= dim; ++t) {
            int64_t vc[3];
            for (int k = 0; k < dim; ++k) { vc[k] = c[k] + pv[pa][t][k]; X[t][k] = (double)vc[k] * m.h; }
            vids[t] = m.vid(vc);
          }
          for (int iq = 0; iq < R.np; ++iq) {
            double x[3] = {0, 0, 0};
            for (int t = 0; t <= dim; ++t)
              for (int k = 0; k < dim; ++k) x[k] += R.lam[iq][t] * X[t][k];
            double f1, f2;
            ex.load(x, &f1, &f2);
            const double wq = R.w[iq] * vol;
            for (int t = 0; t <= dim; ++t) {
              b1[vids[t]] += wq * R.lam[iq][t] * f1;
              b2[vids[t]] += wq * R.lam[iq][t] * f2;
            }
          }
        }
      }
    }
  }
  // full-flux terms on the faces x_ax = 0, 1 of the non-Dirichlet axes:
  // -(sigma . n, v) = (k grad u . n, v)
  {
    int fpv[6][4][3];
    const int nfp = kuhn_paths(dim - 1, fpv);
    const double fvol = std::pow(m.h, dim - 1);
    for (int ax = 0; ax < dim; ++ax) {
      if (ax == m.dax()) continue;
      int other[2], no = 0;
      for (int k = 0; k < dim; ++k)
        if (k != ax) other[no++] = k;
      const int64_t nface = dim == 3 ? n * n : n;
      for (int side = 0; side < 2; ++side) {
        const double nrm = side ? 1.0 : -1.0;
        for (int64_t q = 0; q < nface; ++q) {
          int64_t fc[2] = {q % n, q / n};
          for (int pa = 0; pa < nfp; ++pa) {
            int64_t vids[3];
            double X[3][3];
            for (int t = 0; t < dim; ++t) {
              int64_t vc[3] = {0, 0, 0};
              for (int k = 0; k < dim - 1; ++k) vc[other[k]] = fc[k] + fpv[pa][t][k];
              vc[ax] = side * n;
              for (int k = 0; k < dim; ++k) X[t][k] = (double)vc[k] * m.h;
              vids[t] = m.vid(vc);
            }
            for (int iq = 0; iq < FR.np; ++iq) {
              double x[3] = {0, 0, 0};
              for (int t = 0; t < dim; ++t)
                for (int k = 0; k < dim; ++k) x[k] += FR.lam[iq][t] * X[t][k];
              double u1, u2, g1[3], g2[3];
              ex.eval(x, &u1, &u2, g1, g2);
              const double t1 = ex.k1 * g1[ax] * nrm, t2 = ex.k2 * g2[ax] * nrm;
              const double wq = FR.w[iq] * fvol;
              for (int t = 0; t < dim; ++t) {
                b1[vids[t]] += wq * FR.lam[iq][t] * t1;
                b2[vids[t]] += wq * FR.lam[iq][t] * t2;
              }
            }
          }
        }
      }
    }
  }
  // lifting b -= A[:, D] g over the cells of the two Dirichlet layers, with
  // gen.cpp's element matrices (stiffness kpath, mass (1 + delta) / ((d+1)(d+2)))
  {
    const double kf = dim == 3 ? m.h / 6.0 : 0.5;
    const double mf = dim == 3 ? vol / 6.0 / 20.0 : vol / 2.0 / 12.0;
    auto kpath = [dim](int s, int t) -> double {
      if (s == t) return (s == 0 || s == dim) ? 1.0 : 2.0;
      return (s - t == 1 || t - s == 1) ? -1.0 : 0.0;
    };
    const int ax = m.dax();
    const int64_t nlayer = dim == 3 ? n * n : n;
    for (int layer = 0; layer < 2; ++layer) {
      for (int64_t q = 0; q < nlayer; ++q) {
        int64_t c[3] = {0, 0, 0};
        int o[2], no = 0;
        for (int k = 0; k < dim; ++k)
          if (k != ax) o[no++] = k;
        c[o[0]] = q % n;
        if (dim == 3) c[o[1]] = q / n;
        c[ax] = layer ? n - 1 : 0;
        for (int pa = 0; pa < npath; ++pa) {
          int64_t vids[4];
          double gd1[4], gd2[4];
          bool isd[4];
          for (int t = 0; t <= dim; ++t) {
            int64_t vc[3];
            double X[3];
            for (int k = 0; k < dim; ++k) { vc[k] = c[k] + pv[pa][t][k]; X[k] = (double)vc[k] * m.h; }
            vids[t] = m.vid(vc);
            isd[t] = m.dirichlet(vids[t]);
            ex.eval(X, &gd1[t], &gd2[t], nullptr, nullptr);
          }
          for (int s = 0; s <= dim; ++s) {
            if (isd[s]) continue;
            for (int t = 0; t <= dim; ++t) {
              if (!isd[t]) continue;
              const double K = kpath(s, t), M = mf * (s == t ? 2.0 : 1.0);
              b1[vids[s]] -= (ex.k1 * kf * K + gamma * M) * gd1[t] - gamma * M * gd2[t];
              b2[vids[s]] -= -gamma * M * gd1[t] + (ex.k2 * kf * K + gamma * M) * gd2[t];
            }
          }
        }
      }
    }
  }
  // Dirichlet rows: the exact values
#pragma omp parallel for schedule(static)
  for (int64_t v = 0; v < nv; ++v) {
    if (!m.dirichlet(v)) continue;
    double X[3];
    for (int k = 0; k < dim; ++k) X[k] = (double)((v / m.stride[k]) % m.nn) * m.h;
    ex.eval(X, &b1[v], &b2[v], nullptr, nullptr);
  }
  return MAMG_OK;
}

int bidomain_mms_error(int dim, int64_t n, double gamma, double k1, double k2, const double* x,
                       double* err) {
  if ((dim != 2 && dim != 3) || n < 1) return MAMG_ERR_ARG;
  const Mesh m(dim, n);
  const Exact ex(dim, k1, k2, gamma);
  const Rule R = simplex_rule(dim);
  int pv[6][4][3];
  const int npath = kuhn_paths(dim, pv);
  const int perms3[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
  const int perms2[2][3] = {{0, 1, 0}, {1, 0, 0}};
  const double vol = std::pow(m.h, dim);
  const int64_t ncell = dim == 3 ? n * n * n : n * n;
  double e1 = 0.0, e2 = 0.0;
#pragma omp parallel for reduction(+ : e1, e2) schedule(static)
  for (int64_t cid = 0; cid < ncell; ++cid) {
    int64_t c[3] = {cid % n, (cid / n) % n, dim == 3 ? cid / (n * n) : 0};
    for (int pa = 0; pa < npath; ++pa) {
      const int* perm = dim == 3 ? perms3[pa] : perms2[pa];
      double X[4][3], u1k[4], u2k[4];
      for (int t = 0; t <= dim; ++t) {
        int64_t vc[3];
        for (int k = 0; k < dim; ++k) { vc[k] = c[k] + pv[pa][t][k]; X[t][k] = (double)vc[k] * m.h; }
        const int64_t v = m.vid(vc);
        u1k[t] = x[v];
        u2k[t] = x[m.nv + v];
      }
      double gh1[3] = {0, 0, 0}, gh2[3] = {0, 0, 0};   // P1 gradient along the path's steps
      for (int j = 0; j < dim; ++j) {
        gh1[perm[j]] = (u1k[j + 1] - u1k[j]) / m.h;
        gh2[perm[j]] = (u2k[j + 1] - u2k[j]) / m.h;
      }
      double a1 = 0.0, a2 = 0.0;
      for (int iq = 0; iq < R.np; ++iq) {
        double xq[3] = {0, 0, 0}, uh1 = 0.0, uh2 = 0.0;
        for (int t = 0; t <= dim; ++t) {
          for (int k = 0; k < dim; ++k) xq[k] += R.lam[iq][t] * X[t][k];
          uh1 += R.lam[iq][t] * u1k[t];
          uh2 += R.lam[iq][t] * u2k[t];
        }
        double u1, u2, g1[3], g2[3];
        ex.eval(xq, &u1, &u2, g1, g2);
        double s1 = (u1 - uh1) * (u1 - uh1), s2 = (u2 - uh2) * (u2 - uh2);
        for (int k = 0; k < dim; ++k) {
          s1 += (g1[k] - gh1[k]) * (g1[k] - gh1[k]);
          s2 += (g2[k] - gh2[k]) * (g2[k] - gh2[k]);
        }
        a1 += R.w[iq] * s1;
        a2 += R.w[iq] * s2;
      }
      e1 += a1 * vol;
      e2 += a2 * vol;
    }
  }
  err[0] = std::sqrt(e1);
  err[1] = std::sqrt(e2);
  return MAMG_OK;
}

}  // namespace mamg
