/*
 * vcycle_ref.c -- plain-C restatement of Hierarchy.cycle / Hierarchy.apply
 * (oracle/mamg_oracle.py).  TEST INFRASTRUCTURE ONLY: called by tests/ and by
 * bench.py's cpu_baseline leg (OpenMP over rows, host cores).  Never linked
 * into the product.  Parity status: see mamg_oracle.py (parity unpinned
 * against HAZmath, which is absent from /root/reference).
 *
 * Cycle from x = 0 on level l (V, or W = second coarse visit on the updated
 * residual):  x = S b ; (nu1-1) x += S (b - A x) ; r = b - A x ; bc = R r ;
 * e = cycle(l+1, bc) [; e += cycle(l+1, bc - Ac e)] ; x += P e ;
 * nu2 times x += S (b - A x).   S = W_B (block) or diag(winv) (point).
 * POLY smoother (oracle_set_poly, mamg_oracle.poly_weights): every smoothing
 * is m steps x += w_k S (b - A x), k = 1..m before the coarse correction and
 * k = m..1 after it (the first pre step from x = 0 is x = w_1 S b).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int64_t n, m;
  const int64_t* ptr;
  const int32_t* col;
  const double* val;
} ocsr;

typedef struct {
  int64_t n;
  int coarsest;
  ocsr A, P, R, W;        /* W.n == 0 -> point smoother winv */
  const double* winv;
  const double* Ainv;     /* coarsest, row-major n x n */
  double *t, *r, *b, *x, *c, *e, *u; /* work vectors, length n */
} olevel;

static void spmv(const ocsr* M, const double* x, double* y) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < M->n; ++i) {
    double s = 0.0;
    for (int64_t k = M->ptr[i]; k < M->ptr[i + 1]; ++k) s += M->val[k] * x[M->col[k]];
    y[i] = s;
  }
}

/* r = b - A x */
static void resid(const ocsr* A, const double* x, const double* b, double* r) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < A->n; ++i) {
    double s = 0.0;
    for (int64_t k = A->ptr[i]; k < A->ptr[i + 1]; ++k) s += A->val[k] * x[A->col[k]];
    r[i] = b[i] - s;
  }
}

/* POLY step weights (0 steps: one unweighted step per sweep) */
static int g_poly_m = 0;
static double g_poly_w[16];

int oracle_set_poly(int m, const double* w) {
  if (m < 0 || m > 16) return -1;
  g_poly_m = m;
  for (int k = 0; k < m; ++k) g_poly_w[k] = w[k];
  return 0;
}

/* y = S v (smoother application) */
static void smooth_apply(const olevel* L, const double* v, double* y) {
  if (L->W.n > 0) {
    spmv(&L->W, v, y);
  } else {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < L->n; ++i) y[i] = L->winv[i] * v[i];
  }
}

/* y = w S v */
static void smooth_apply_w(const olevel* L, double w, const double* v, double* y) {
  smooth_apply(L, v, y);
  if (w != 1.0) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < L->n; ++i) y[i] = w * y[i];
  }
}

/* step weight of smoothing step s of a sweep sequence (pre: 1..m, post: m..1) */
static double step_w(int s, int pre) {
  if (g_poly_m == 0) return 1.0;
  const int k = s % g_poly_m;
  return g_poly_w[pre ? k : g_poly_m - 1 - k];
}

static void axpy1(int64_t n, const double* a, double* y) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) y[i] = y[i] + a[i];
}

static void cycle(olevel* L, int l, int wcyc, int nu1, int nu2, const double* b, double* x) {
  olevel* lv = &L[l];
  const int64_t n = lv->n;
  if (lv->coarsest) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      double s = 0.0;
      for (int64_t j = 0; j < n; ++j) s += lv->Ainv[i * n + j] * b[j];
      x[i] = s;
    }
    return;
  }
  olevel* C = &L[l + 1];
  const int steps = g_poly_m > 0 ? g_poly_m : 1;
  smooth_apply_w(lv, step_w(0, 1), b, x);
  for (int s = 1; s < nu1 * steps; ++s) {
    resid(&lv->A, x, b, lv->r);
    smooth_apply_w(lv, step_w(s, 1), lv->r, lv->u);
    axpy1(n, lv->u, x);
  }
  resid(&lv->A, x, b, lv->r);
  spmv(&lv->R, lv->r, C->b);
  cycle(L, l + 1, wcyc, nu1, nu2, C->b, C->x);
  if (wcyc && !C->coarsest) {
    resid(&C->A, C->x, C->b, C->c);
    cycle(L, l + 1, wcyc, nu1, nu2, C->c, C->e);
    axpy1(C->n, C->e, C->x);
  }
  spmv(&lv->P, C->x, lv->t);
  axpy1(n, lv->t, x);
  for (int s = 0; s < nu2 * steps; ++s) {
    resid(&lv->A, x, b, lv->r);
    smooth_apply_w(lv, step_w(s, 0), lv->r, lv->u);
    axpy1(n, lv->u, x);
  }
}

/* z = B r : maxit cycles from z = 0 (Hierarchy.apply) */
int oracle_apply(olevel* L, int nlev, int wcyc, int nu1, int nu2, int maxit, const double* r,
                 double* z) {
  if (nlev < 1) return -1;
  cycle(L, 0, wcyc, nu1, nu2, r, z);
  for (int it = 1; it < maxit; ++it) {
    resid(&L[0].A, z, r, L[0].c);
    cycle(L, 0, wcyc, nu1, nu2, L[0].c, L[0].e);
    axpy1(L[0].n, L[0].e, z);
  }
  return 0;
}

void oracle_set_threads(int n) {
#ifdef _OPENMP
  extern void omp_set_num_threads(int);
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

int oracle_num_threads(void) {
  int n = 1;
#pragma omp parallel
  {
#pragma omp single
    {
#ifdef _OPENMP
      extern int omp_get_num_threads(void);
      n = omp_get_num_threads();
#endif
    }
  }
  return n;
}

int oracle_spmv(const ocsr* A, const double* x, double* y) {
  spmv(A, x, y);
  return 0;
}

static double dotp(int64_t n, const double* a, const double* b) {
  double s = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : s)
  for (int64_t i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}

/*
 * cbc.block ConjGrad (mamg_oracle.pcg, krylov.ConjGrad) with B = oracle_apply
 * on L and the operator L[0].A: x from 0, residuals[k] = sqrt(<r_k, B r_k>),
 * absolute tolerance.  Work: 5 vectors of L[0].n (caller-owned in w).
 * Returns the iteration count (-1: <r,Br> < 0 at the start).
 */
int oracle_pcg(olevel* L, int nlev, int wcyc, int nu1, int nu2, int maxit, const double* b,
               double* x, double tol, int maxiter, double* residuals, double* w) {
  const int64_t n = L[0].n;
  double *r = w, *z = w + n, *d = w + 2 * n, *q = w + 3 * n;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) { x[i] = 0.0; r[i] = b[i]; }
  oracle_apply(L, nlev, wcyc, nu1, nu2, maxit, r, z);
  memcpy(d, z, n * sizeof(double));
  double rz = dotp(n, r, z);
  if (rz < 0) return -1;
  residuals[0] = __builtin_sqrt(rz);
  int it = 0;
  while (residuals[it] > tol && it < maxiter) {
    spmv(&L[0].A, d, q);
    const double dq = dotp(n, d, q);
    if (dq == 0.0) break;
    const double alpha = rz / dq;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) { x[i] = x[i] + alpha * d[i]; r[i] = r[i] - alpha * q[i]; }
    oracle_apply(L, nlev, wcyc, nu1, nu2, maxit, r, z);
    const double rz_prev = rz;
    rz = dotp(n, r, z);
    if (rz < 0) break;
    const double beta = rz / rz_prev;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) d[i] = z[i] + beta * d[i];
    residuals[it + 1] = __builtin_sqrt(rz);
    ++it;
  }
  return it;
}
