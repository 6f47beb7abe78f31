// host_asan.cpp -- the host C++ of the library (setup.cpp, gen.cpp, mms.cpp,
// convert.cpp, dist.cpp) and the oracle's C cycle (oracle/vcycle_ref.c),
// compiled with -fsanitize=address,undefined and driven through their paths
// on small systems (sanitizer builds of the host code
// and the CPU oracle).  Built and run by
// tests/test_sanitize.py (CPU); exits non-zero on any failure, and the
// sanitizers abort on the first report (-fno-sanitize-recover=all).
//
// Covered: the P1 generator (2-D, 3-D), the manufactured right-hand side and
// H1 error; host_setup for the nodal SA profile (seed blocks), UA + HEM +
// W + SGS + scaling, VMB, POLY, scalar AMG with point smoothers, the
// additive overlapping rings (sparse seeds), the node patches and seed rings
// (their host-side checks and colourings), the classical strength measure;
// BSR2 / SELL conversions; the row-partition plan for P = 2, 3, 4; the
// oracle's C cycle and PCG on each hierarchy.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "dist.h"
#include "host.h"

extern "C" {
typedef struct {
  int64_t n, m;
  const int64_t* ptr;
  const int32_t* col;
  const double* val;
} ocsr;
typedef struct {
  int64_t n;
  int coarsest;
  ocsr A, P, R, W;
  const double* winv;
  const double* Ainv;
  double *t, *r, *b, *x, *c, *e, *u;
} olevel;
int oracle_apply(olevel* L, int nlev, int wcyc, int nu1, int nu2, int maxit, const double* r, double* z);
int oracle_pcg(olevel* L, int nlev, int wcyc, int nu1, int nu2, int maxit, const double* b, double* x,
               double tol, int maxiter, double* residuals, double* w);
int oracle_set_poly(int m, const double* w);
}

namespace mamg {
void set_error(const std::string& s) { std::fprintf(stderr, "set_error: %s\n", s.c_str()); }
}

using namespace mamg;

static int g_fail = 0;
#define CHECK(c, ...)                                     \
  do {                                                    \
    if (!(c)) {                                           \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                  \
      std::fprintf(stderr, "\n");                         \
      ++g_fail;                                           \
    }                                                     \
  } while (0)

static mamg_params defaults() {
  mamg_params p;
  std::memset(&p, 0, sizeof p);
  p.abi_version = MAMG_ABI_VERSION;
  p.AMG_type = MAMG_SA_AMG;
  p.cycle_type = MAMG_V_CYCLE;
  p.max_levels = 20;
  p.maxit = 1;
  p.smoother = MAMG_SMOOTHER_JACOBI_RHO;
  p.relaxation = 4.0 / 3.0;
  p.presmooth_iter = 1;
  p.postsmooth_iter = 1;
  p.coarse_dof = 100;
  p.coarse_solver = MAMG_COARSE_DENSE;
  p.aggregation_type = MAMG_MIS;
  p.max_aggregation = 100;
  p.amli_degree = 3;
  p.Schwarz_levels = 1;
  p.Schwarz_mmsize = 100;
  p.Schwarz_maxlvl = 1;
  p.Schwarz_type = MAMG_SCHWARZ_BLOCK_JACOBI;
  p.Schwarz_blksolver = MAMG_COARSE_DENSE;
  p.sa_omega = 4.0 / 3.0;
  p.max_coarse_dense = 8192;
  p.num_functions = 1;
  p.node_block_smoother = 1;
  p.sa_block_diag = 1;
  p.post_fusion = 1;
  p.poly_degree = 2;
  p.poly_ratio = 16.0;
  p.strength_measure = MAMG_STRENGTH_ROWMAX;
  return p;
}

struct System {
  int dim;
  int64_t n, N, nnz;
  std::vector<int64_t> ptr;
  std::vector<int32_t> col;
  std::vector<double> val;
  CsrView view() const {
    CsrView v;
    v.n = v.m = N;
    v.ptr = ptr.data();
    v.col = col.data();
    v.val = val.data();
    return v;
  }
};

static System bidomain(int dim, int64_t n, double gamma) {
  System s;
  s.dim = dim;
  s.n = n;
  CHECK(gen_bidomain_size(dim, n, &s.N, &s.nnz) == 0, "gen size");
  s.ptr.resize(s.N + 1);
  s.col.resize(s.nnz);
  s.val.resize(s.nnz);
  CHECK(gen_bidomain(dim, n, gamma, 2.0, 3.0, s.ptr.data(), s.col.data(), s.val.data()) == 0, "gen");
  s.nnz = s.ptr[s.N];
  return s;
}

static ocsr oc(const CsrView& v) { return ocsr{v.n, v.m, v.ptr, v.col, v.val}; }

// the oracle's C cycle + PCG on a host hierarchy; returns the iteration count
static int run_oracle(const Hierarchy& H, const System& s, int wcyc) {
  const int nl = (int)H.levels.size();
  std::vector<olevel> L(nl);
  std::vector<std::vector<double>> work(nl);
  for (int l = 0; l < nl; ++l) {
    const HostLevel& h = H.levels[l];
    olevel& o = L[l];
    std::memset(&o, 0, sizeof o);
    o.n = h.n;
    o.coarsest = h.coarsest;
    o.A = oc(H.A(l));
    if (!h.coarsest) {
      o.P = oc(h.P.view());
      o.R = oc(h.R.view());
      if (h.WB.n) o.W = oc(h.WB.view());
      o.winv = h.winv.empty() ? nullptr : h.winv.data();
    } else {
      o.Ainv = h.Ainv.data();
    }
    work[l].assign(7 * (size_t)h.n, 0.0);
    double* w = work[l].data();
    o.t = w; o.r = w + h.n; o.b = w + 2 * h.n; o.x = w + 3 * h.n; o.c = w + 4 * h.n; o.e = w + 5 * h.n;
    o.u = w + 6 * h.n;
  }
  std::vector<double> b(s.N), x(s.N), res(502), w(5 * (size_t)s.N);
  uint64_t st = 1234;
  for (auto& v : b) {   // xorshift uniform(-1, 1)
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    v = (double)(st >> 11) / 9007199254740992.0 * 2.0 - 1.0;
  }
  std::vector<double> z(s.N);
  CHECK(oracle_apply(L.data(), nl, wcyc, H.params.presmooth_iter, H.params.postsmooth_iter, 1, b.data(), z.data()) == 0,
        "oracle_apply");
  double zz = 0;
  for (double v : z) zz += v * v;
  CHECK(std::isfinite(zz) && zz > 0, "apply not finite");
  return oracle_pcg(L.data(), nl, wcyc, H.params.presmooth_iter, H.params.postsmooth_iter, 1, b.data(), x.data(),
                    1e-8, 500, res.data(), w.data());
}

static void case_setup(const char* name, const System& s, mamg_params p, const std::vector<int32_t>& idofs,
                       bool expect_ok = true, bool plan = false) {
  const mamg_params P = resolve_params(p, idofs.empty() ? nullptr : idofs.data(), (int64_t)idofs.size(), s.N);
  Hierarchy H;
  std::string err;
  const int rc = host_setup(s.view(), idofs.empty() ? nullptr : idofs.data(), (int64_t)idofs.size(), P, &H, &err);
  if (!expect_ok) {
    CHECK(rc != 0, "%s: expected a refusal", name);
    std::printf("%-44s refused as expected: %s\n", name, err.c_str());
    return;
  }
  CHECK(rc == 0, "%s: host_setup rc %d: %s", name, rc, err.c_str());
  if (rc) return;
  double w[MAMG_POLY_MAX];
  if (P.smoother == MAMG_SMOOTHER_POLY) {
    CHECK(poly_weights(P, w) == P.poly_degree, "poly weights");
    oracle_set_poly(P.poly_degree, w);
  } else {
    oracle_set_poly(0, nullptr);
  }
  int its = -2;
  const bool cyc = P.smoother != MAMG_SMOOTHER_GS && P.smoother != MAMG_SMOOTHER_SGS &&
                   P.Schwarz_type != MAMG_SCHWARZ_PATCHES && P.Schwarz_type != MAMG_SCHWARZ_RINGS &&
                   !P.coarse_scaling;   // what vcycle_ref.c restates
  if (cyc) {
    its = run_oracle(H, s, P.cycle_type == MAMG_W_CYCLE);
    CHECK(its > 0 && its < 500, "%s: oracle PCG iterations %d", name, its);
  }
  // node-block layouts of every level (BSR2, SELL-64) where the hierarchy is nodal
  if (P.num_functions == 2) {
    for (size_t l = 0; l + 1 < H.levels.size(); ++l) {
      const CsrView A = H.A((int)l);
      HBsr B;
      to_bsr2(A, A.n / 2, A.n / 2, &B);
      HSell S;
      CHECK(to_sell(B, false, 64, 1, &S, &err) == 0, "%s: to_sell level %zu: %s", name, l, err.c_str());
      std::vector<double> blk;
      if (H.levels[l].WB.n) (void)node_blocks_of(H.levels[l].WB.view(), A.n / 2, &blk);
    }
  }
  if (plan && P.num_functions == 2) {
    for (int nr : {2, 3, 4})
      for (int rank = 0; rank < nr; ++rank) {
        DistPlan dp;
        const int rc2 = build_dist_plan(H, s.view(), rank, nr, 100, true, &dp, &err);
        CHECK(rc2 == 0, "%s: build_dist_plan P=%d rank %d: %s", name, nr, rank, err.c_str());
      }
  }
  std::printf("%-44s levels %zu, oracle PCG its %d\n", name, H.levels.size(), its);
}

int main() {
  const System s2 = bidomain(2, 32, 1e6);
  const System s3 = bidomain(3, 8, 1e6);
  const System s3b = bidomain(3, 12, 1e2);
  std::vector<int32_t> seeds2, seeds3, seeds3b, sparse3;
  for (int64_t i = s2.N / 2; i < s2.N; ++i) seeds2.push_back((int32_t)i);
  for (int64_t i = s3.N / 2; i < s3.N; ++i) seeds3.push_back((int32_t)i);
  for (int64_t i = s3b.N / 2; i < s3b.N; ++i) seeds3b.push_back((int32_t)i);
  for (int64_t i = 0; i < s3.N; i += 37) sparse3.push_back((int32_t)i);

  mamg_params p = defaults();
  p.num_functions = 2;
  case_setup("nodal SA + seed blocks (2-D)", s2, p, seeds2, true, true);
  case_setup("nodal SA + seed blocks (3-D)", s3, p, seeds3, true, true);
  case_setup("nodal SA, no seeds (3-D, gamma 1e2)", s3b, p, {}, true, true);
  {
    mamg_params q = p;
    q.smoother = MAMG_SMOOTHER_POLY;
    q.poly_degree = 3;
    case_setup("POLY degree 3", s3b, q, seeds3b, true, true);
    q = p;
    q.strength_measure = MAMG_STRENGTH_DIAG;
    q.strong_coupled = 0.05;
    case_setup("classical strength measure", s3, q, seeds3);
    q = p;
    q.AMG_type = MAMG_UA_AMG;
    q.aggregation_type = MAMG_HEM;
    q.cycle_type = MAMG_W_CYCLE;
    q.smoother = MAMG_SMOOTHER_SGS;
    q.coarse_scaling = MAMG_ON;
    q.strong_coupled = 0.1;
    q.Schwarz_type = MAMG_SCHWARZ_SEED_BLOCKS;
    case_setup("reference family UA+HEM+W+SGS+scaling", s3, q, seeds3, true, true);
    q.Schwarz_type = MAMG_SCHWARZ_SYMMETRIC;
    case_setup("parameters_metric_schwarz (node patches)", s3, q, seeds3);
    q.Schwarz_maxlvl = 2;
    case_setup("SYMMETRIC 2-rings on every node (rings)", s3, q, seeds3);
    q.Schwarz_maxlvl = 1;
    case_setup("SYMMETRIC 1-rings, sparse seeds (rings)", s3, q, sparse3);
    q = p;
    q.AMG_type = MAMG_UA_AMG;
    q.aggregation_type = MAMG_VMB;
    q.cycle_type = MAMG_W_CYCLE;
    q.strong_coupled = 0.1;
    case_setup("parameters_standard-like VMB + W", s3, q, seeds3, true, true);
    q = p;
    q.Schwarz_type = MAMG_SCHWARZ_ADDITIVE;
    q.Schwarz_maxlvl = 2;
    case_setup("additive overlapping 2-rings, sparse seeds", s3, q, sparse3);
  }
  {
    mamg_params q = defaults();   // scalar AMG, point smoothers
    q.node_block_smoother = 0;
    case_setup("scalar SA, Jacobi-rho", s3b, q, {});
    q.smoother = MAMG_SMOOTHER_L1DIAG;
    q.AMG_type = MAMG_UA_AMG;
    q.cycle_type = MAMG_W_CYCLE;
    case_setup("scalar UA, L1 Jacobi, W", s2, q, {});
    q = defaults();
    q.Schwarz_maxlvl = 2;     // overlapping rings without SCHWARZ_ADDITIVE: refused
    case_setup("refusal path (rings on a scalar system)", s3, q, sparse3, false);
  }
  // manufactured solution: right-hand side and the H1 error of the zero vector
  for (const System* s : {&s2, &s3}) {
    std::vector<double> b(s->N), x(s->N, 0.0), e(4, 0.0);
    CHECK(gen_bidomain_mms(s->dim, s->n, 1e6, 2.0, 3.0, b.data()) == 0, "mms rhs");
    CHECK(bidomain_mms_error(s->dim, s->n, 1e6, 2.0, 3.0, x.data(), e.data()) == 0, "mms error");
    CHECK(std::isfinite(e[0]) && e[0] > 0, "mms error value");
  }
  std::printf("%s: %d failure(s)\n", g_fail ? "FAILED" : "host_asan ok", g_fail);
  return g_fail ? 1 : 0;
}
