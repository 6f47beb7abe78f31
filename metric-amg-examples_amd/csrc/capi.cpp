// capi.cpp -- extern "C" boundary (include/mamg.h).  No exceptions cross it:
// every entry point catches, records a thread-local message and returns a
// negative status.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <new>
#include <string>

#include "device.h"
#include "dist.h"
#include "host.h"
#include "mamg_test.h"
#include "opts.h"

#if MAMG_DIAG
// Diagnosis build: a SIGSEGV tracer for host crashes inside the library or
// the HIP runtime.  On an alternate signal stack
// (a stack overflow leaves none), it prints the fault address, the faulting
// thread's stack bounds, the frame depth and the innermost / outermost native
// frames, then restores the previous handler (Python's faulthandler or the
// default) and returns, so the re-executed access reports as before.
#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>
namespace {
struct sigaction g_prev_segv;
constexpr int SEGV_FRAMES = 1 << 18;
void* g_frames[SEGV_FRAMES];
void segv_write(const char* s, int n) {
  while (n > 0) {
    const ssize_t w = write(2, s, n);
    if (w <= 0) return;
    s += w;
    n -= (int)w;
  }
}
void segv_trace(int sig, siginfo_t* si, void*) {
  char buf[512];
  void* sb = nullptr;
  size_t ss = 0;
  pthread_attr_t a;
  if (pthread_getattr_np(pthread_self(), &a) == 0) {
    pthread_attr_getstack(&a, &sb, &ss);
    pthread_attr_destroy(&a);
  }
  const int depth = backtrace(g_frames, SEGV_FRAMES);
  int n = std::snprintf(buf, sizeof buf,
                        "[mamg diag] signal %d at address %p; thread stack [%p, %p) = %.1f MiB; %d native frames%s\n",
                        sig, si ? si->si_addr : nullptr, sb, (char*)sb + ss, ss / 1048576.0, depth,
                        depth == SEGV_FRAMES ? " (buffer full)" : "");
  segv_write(buf, n);
  const int inner = depth < 48 ? depth : 48;
  segv_write("[mamg diag] innermost frames:\n", 30);
  backtrace_symbols_fd(g_frames, inner, 2);
  if (depth > inner) {
    const int outer = depth - inner < 32 ? depth - inner : 32;
    segv_write("[mamg diag] outermost frames:\n", 30);
    backtrace_symbols_fd(g_frames + depth - outer, outer, 2);
  }
  sigaction(SIGSEGV, &g_prev_segv, nullptr);
}
__attribute__((constructor)) void segv_install() {
  static char alt[1 << 20];
  stack_t st{};
  st.ss_sp = alt;
  st.ss_size = sizeof alt;
  sigaltstack(&st, nullptr);
  void* f[4];
  (void)backtrace(f, 4);                 // loads the unwinder before any fault
  struct sigaction sa{};
  sa.sa_sigaction = segv_trace;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_prev_segv);
}
}  // namespace
#endif

namespace mamg {
namespace {
thread_local std::string g_err;
}
void set_error(const std::string& s) { g_err = s; }
}  // namespace mamg

struct mamg_hier {
  mamg::Hierarchy H;   // level 0 is a view of the caller's CSR (must outlive this)
};

struct mamg_handle {
  mamg::DeviceHandle* d = nullptr;
};

struct mamg_plan {
  mamg::DistPlan P;
};

struct mamg_dhandle {
  mamg::DistHandle* d = nullptr;
};

using mamg::set_error;

#define GUARD_BEGIN try {
#define GUARD_END                                       \
  }                                                     \
  catch (const std::bad_alloc&) {                       \
    set_error("host allocation failed");                \
    return MAMG_ERR_NOMEM;                              \
  }                                                     \
  catch (const std::exception& e) {                     \
    set_error(std::string("internal error: ") + e.what()); \
    return MAMG_ERR_SETUP;                              \
  }

#define DEV_CALL(call)                    \
  GUARD_BEGIN                             \
  if (!h) { set_error("null handle"); return MAMG_ERR_ARG; } \
  std::string err;                        \
  int rc = (call);                        \
  if (rc) set_error(err);                 \
  return rc;                              \
  GUARD_END

namespace {
// The setup temporaries' cached blocks (dmem.h) stay cached for the
// process's next setup, up to the cache limit (mamg_set_setup_cache_limit;
// default an eighth of the device's HBM): with them released at the end of
// every setup, one phase of one or two later setups of a long-lived process
// took seconds (the bench's profile comparison: 5.5-5.9 s instead of 0.8 s in
// 2 of 2 runs, scripts/runs/gpu_r05z9.sh).  Above the
// limit the largest idle blocks are freed at the end of every setup;
// mamg_release_setup_cache() releases all of them.
// It also holds the capture lock for a single-GPU setup (device.hip
// capture_mutex): those setups run one at a time and never overlap another
// thread's stream capture.  A multi-GPU rank's setup does not take it: it
// waits in ncclCommInitRank for its peers, which may be threads of the same
// process (one process per GPU is the intended use).
struct TmpTrim {
  std::unique_lock<std::recursive_mutex> lock;
  explicit TmpTrim(bool serialize = true) {
    if (serialize) lock = std::unique_lock<std::recursive_mutex>(mamg::capture_mutex());
  }
  ~TmpTrim() { mamg::dev_tmp_trim_to_limit(); }
};

int to_view(const mamg_csr* A, mamg::CsrView* v) {
  if (!A || !A->rowptr || (A->nnz > 0 && (!A->colind || !A->values))) {
    set_error("null CSR pointer");
    return MAMG_ERR_ARG;
  }
  if (A->nrows <= 0 || A->ncols <= 0 || A->rowptr[0] != 0 || A->rowptr[A->nrows] != A->nnz) {
    set_error("inconsistent CSR sizes (rowptr[0] must be 0 and rowptr[n] == nnz)");
    return MAMG_ERR_ARG;
  }
  if (A->nrows > INT32_MAX || A->ncols > INT32_MAX) {
    set_error("matrix dimension exceeds int32 column index range");
    return MAMG_ERR_ARG;
  }
  v->n = A->nrows;
  v->m = A->ncols;
  v->ptr = A->rowptr;
  v->col = A->colind;
  v->val = A->values;
  return MAMG_OK;
}

// Seeds on both fields of one node (num_functions == 2: dof f nv + I) -- the
// EMI drivers pass the interface dofs of both sides (src/emi_3d.py:134-138)
// -- are reduced to the field-1 seed.  The field-0 dof then joins its
// strongest seed neighbour, the partner across the interface, and the
// coupled pair forms one block {u0_I, u1_I}.  Kept as two seeds, the pair
// would become two singleton blocks (non-overlapping Schwarz) and the
// smoother would lose the metric coupling: 500 vs 34 PCG iterations on EMI
// 3-D n = 16 at gamma = 1e6.
struct Seeds {
  std::vector<int32_t> v;
  const int32_t* ptr = nullptr;
  int64_t n = 0;
  Seeds(const int32_t* idofs, int64_t n_idofs, int64_t N, const mamg_params* p) : ptr(idofs), n(n_idofs) {
    // the seed-ring Schwarz keeps every seed: overlapping blocks, as the reference's
    if (!idofs || n_idofs <= 0 || !p || p->num_functions != 2 || N % 2 ||
        (p->Schwarz_type == MAMG_SCHWARZ_RINGS && p->Schwarz_levels >= 1))
      return;
    const int64_t nv = N / 2;
    std::vector<uint8_t> seed(N, 0);
    for (int64_t t = 0; t < n_idofs; ++t)
      if (idofs[t] >= 0 && idofs[t] < N) seed[idofs[t]] = 1;
    bool any = false;
    for (int64_t I = 0; I < nv && !any; ++I) any = seed[I] && seed[nv + I];
    if (!any) return;
    v.reserve(n_idofs);
    for (int64_t t = 0; t < n_idofs; ++t) {
      const int32_t s = idofs[t];
      if (s >= 0 && s < nv && seed[nv + s]) continue;
      v.push_back(s);
    }
    ptr = v.data();
    n = (int64_t)v.size();
  }
};
}  // namespace

extern "C" {

int mamg_abi_version(void) { return MAMG_ABI_VERSION; }

int mamg_release_setup_cache(void) {
  GUARD_BEGIN
  mamg::dev_tmp_trim();
  return MAMG_OK;
  GUARD_END
}
int mamg_set_setup_cache_limit(int64_t bytes) {
  GUARD_BEGIN
  mamg::dev_set_cache_limit(bytes < 0 ? -1 : bytes);
  return MAMG_OK;
  GUARD_END
}

int mamg_setup_cache_bytes(int device, int64_t* idle_bytes, int64_t* limit_bytes) {
  GUARD_BEGIN
  if (device < 0 || device > 63) { set_error("device out of range"); return MAMG_ERR_ARG; }
  if (idle_bytes) *idle_bytes = mamg::dev_cache_idle_bytes(device);
  if (limit_bytes) *limit_bytes = mamg::dev_cache_limit(device);
  return MAMG_OK;
  GUARD_END
}

int mamg_set_option(const char* name, const char* value) {
  GUARD_BEGIN
  if (!mamg::set_opt(name, value)) {
    set_error(std::string("unknown option ") + (name ? name : "(null)") + "; known: " + mamg::opt_names());
    return MAMG_ERR_ARG;
  }
  return MAMG_OK;
  GUARD_END
}

const char* mamg_option_names(void) { return mamg::opt_names(); }

const char* mamg_last_error(void) { return mamg::g_err.c_str(); }

void mamg_params_default(mamg_params* p) {
  std::memset(p, 0, sizeof(*p));
  p->abi_version = MAMG_ABI_VERSION;
  p->AMG_type = MAMG_SA_AMG;
  p->cycle_type = MAMG_V_CYCLE;
  p->max_levels = 20;
  p->maxit = 1;
  p->smoother = MAMG_SMOOTHER_JACOBI_RHO;
  p->relaxation = 4.0 / 3.0;
  p->presmooth_iter = 1;
  p->postsmooth_iter = 1;
  p->coarse_dof = 100;
  p->coarse_solver = MAMG_COARSE_DENSE;
  p->coarse_scaling = MAMG_OFF;
  p->aggregation_type = MAMG_MIS;
  p->strong_coupled = 0.0;
  p->max_aggregation = 100;
  p->amli_degree = 3;
  p->Schwarz_levels = 1;
  p->Schwarz_mmsize = 100;
  p->Schwarz_maxlvl = 1;
  p->Schwarz_type = MAMG_SCHWARZ_BLOCK_JACOBI;
  p->Schwarz_blksolver = MAMG_COARSE_DENSE;
  p->print_level = 0;
  p->sa_omega = 4.0 / 3.0;
  p->rho_iters = 0;
  p->max_coarse_dense = 8192;
  p->device = 0;
  p->spmv_lanes = 0;
  p->num_functions = 1;
  p->node_block_smoother = 1;
  p->sa_block_diag = 1;
  p->post_fusion = 1;
  p->poly_degree = 2;
  p->poly_ratio = 16.0;
  p->strength_measure = MAMG_STRENGTH_ROWMAX;
}

int mamg_gen_bidomain_size(int dim, int64_t n, int64_t* nrows, int64_t* nnz) {
  GUARD_BEGIN
  int rc = mamg::gen_bidomain_size(dim, n, nrows, nnz);
  if (rc) set_error("gen_bidomain_size: dim must be 2 or 3 and n >= 1");
  return rc;
  GUARD_END
}

int mamg_gen_bidomain(int dim, int64_t n, double gamma, double kappa1, double kappa2,
                      int64_t* rowptr, int32_t* colind, double* values) {
  GUARD_BEGIN
  if (!rowptr || !colind || !values) { set_error("null output buffer"); return MAMG_ERR_ARG; }
  int rc = mamg::gen_bidomain(dim, n, gamma, kappa1, kappa2, rowptr, colind, values);
  if (rc) set_error("gen_bidomain: bad dim/n");
  return rc;
  GUARD_END
}

int mamg_gen_bidomain_mms(int dim, int64_t n, double gamma, double kappa1, double kappa2, double* b) {
  GUARD_BEGIN
  if (!b) { set_error("null output buffer"); return MAMG_ERR_ARG; }
  int rc = mamg::gen_bidomain_mms(dim, n, gamma, kappa1, kappa2, b);
  if (rc) set_error("gen_bidomain_mms: dim must be 2 or 3 and n >= 1");
  return rc;
  GUARD_END
}

int mamg_bidomain_mms_error(int dim, int64_t n, double gamma, double kappa1, double kappa2,
                            const double* x, double* err) {
  GUARD_BEGIN
  if (!x || !err) { set_error("null argument"); return MAMG_ERR_ARG; }
  int rc = mamg::bidomain_mms_error(dim, n, gamma, kappa1, kappa2, x, err);
  if (rc) set_error("bidomain_mms_error: dim must be 2 or 3 and n >= 1");
  return rc;
  GUARD_END
}

int mamg_host_setup(const mamg_csr* A, const int32_t* idofs, int64_t n_idofs,
                    const mamg_params* params, mamg_hier** out) {
  GUARD_BEGIN
  if (!out || !params) { set_error("null argument"); return MAMG_ERR_ARG; }
  *out = nullptr;
  mamg::CsrView v;
  int rc = to_view(A, &v);
  if (rc) return rc;
  const mamg_params P = mamg::resolve_params(*params, idofs, n_idofs, v.n);   // the reference's Schwarz names
  mamg_hier* h = new mamg_hier();
  std::string err;
  Seeds S(idofs, n_idofs, v.n, &P);
  rc = mamg::host_setup(v, S.ptr, S.n, P, &h->H, &err);
  if (rc) { set_error(err); delete h; return rc; }
  *out = h;
  return MAMG_OK;
  GUARD_END
}

void mamg_hier_free(mamg_hier* h) { delete h; }

int mamg_hier_num_levels(const mamg_hier* h) { return h ? (int)h->H.levels.size() : MAMG_ERR_ARG; }

int mamg_hier_params(const mamg_hier* h, mamg_params* out) {
  if (!h || !out) { set_error("null argument"); return MAMG_ERR_ARG; }
  *out = h->H.params;
  return MAMG_OK;
}

int mamg_hier_level_sizes(const mamg_hier* h, int l, int64_t* s) {
  if (!h || l < 0 || l >= (int)h->H.levels.size() || !s) { set_error("bad level"); return MAMG_ERR_ARG; }
  const auto& L = h->H.levels[l];
  s[0] = L.n;
  s[1] = h->H.A(l).nnz();
  s[2] = L.P.nnz();
  s[3] = L.R.nnz();
  s[4] = L.WB.nnz();
  s[5] = L.coarsest ? 0 : h->H.levels[l + 1].n;
  return MAMG_OK;
}

int mamg_hier_level_export(const mamg_hier* h, int l, int64_t* Aptr, int32_t* Acol, double* Aval,
                           int64_t* Pptr, int32_t* Pcol, double* Pval, int64_t* Rptr,
                           int32_t* Rcol, double* Rval, int64_t* Wptr, int32_t* Wcol,
                           double* Wval, double* winv, int64_t* agg, double* Ainv) {
  if (!h || l < 0 || l >= (int)h->H.levels.size()) { set_error("bad level"); return MAMG_ERR_ARG; }
  const auto& L = h->H.levels[l];
  auto cp = [](const mamg::CsrView& M, int64_t* p, int32_t* c, double* v) {
    if (p && M.ptr) std::memcpy(p, M.ptr, (M.n + 1) * sizeof(int64_t));
    if (c && M.col) std::memcpy(c, M.col, M.nnz() * sizeof(int32_t));
    if (v && M.val) std::memcpy(v, M.val, M.nnz() * sizeof(double));
  };
  cp(h->H.A(l), Aptr, Acol, Aval);
  if (!L.P.ptr.empty()) cp(L.P.view(), Pptr, Pcol, Pval);
  if (!L.R.ptr.empty()) cp(L.R.view(), Rptr, Rcol, Rval);
  if (!L.WB.ptr.empty()) cp(L.WB.view(), Wptr, Wcol, Wval);
  if (winv && !L.winv.empty()) std::memcpy(winv, L.winv.data(), L.winv.size() * sizeof(double));
  if (agg && !L.agg.empty()) std::memcpy(agg, L.agg.data(), L.agg.size() * sizeof(int64_t));
  if (Ainv && !L.Ainv.empty()) std::memcpy(Ainv, L.Ainv.data(), L.Ainv.size() * sizeof(double));
  return MAMG_OK;
}

int mamg_hier_dist_plan(const mamg_hier* h, int rank, int nranks, int64_t rep_nodes,
                        mamg_plan** out) {
  GUARD_BEGIN
  if (!h || !out) { set_error("null argument"); return MAMG_ERR_ARG; }
  *out = nullptr;
  mamg_plan* p = new mamg_plan();
  std::string err;
  int rc = mamg::build_dist_plan(h->H, h->H.A0, rank, nranks, rep_nodes, h->H.params.post_fusion != 0,
                                 &p->P, &err);
  if (rc) { set_error(err); delete p; return rc; }
  *out = p;
  return MAMG_OK;
  GUARD_END
}

void mamg_plan_free(mamg_plan* p) { delete p; }
int mamg_plan_num_levels(const mamg_plan* p) { return p ? (int)p->P.levels.size() : MAMG_ERR_ARG; }

int mamg_plan_level_sizes(const mamg_plan* p, int l, int64_t* s) {
  if (!p || l < 0 || l >= (int)p->P.levels.size() || !s) { set_error("bad level"); return MAMG_ERR_ARG; }
  const mamg::DistLevel& D = p->P.levels[l];
  const int64_t v[16] = {D.nv, D.replicated, D.coarsest, D.o0, D.o1, (int64_t)D.ghosts.size(),
                         (int64_t)D.send_idx.size(),
                         D.A.ptr.empty() ? 0 : D.A.ptr[D.A.nr], D.A.nr, D.A.nc,
                         D.P.ptr.empty() ? 0 : D.P.ptr[D.P.nr], D.P.nr, D.P.nc,
                         D.Rp.ptr.empty() ? 0 : D.Rp.ptr[D.Rp.nr], D.Rp.nr, D.Rp.nc};
  std::memcpy(s, v, sizeof(v));
  return MAMG_OK;
}

int mamg_plan_level_export(const mamg_plan* p, int l, int64_t* ghosts, int64_t* ghost_off,
                           int64_t* send_idx, int64_t* send_off, int64_t* Aptr, int32_t* Acol,
                           double* Aval, int64_t* Pptr, int32_t* Pcol, double* Pval, int64_t* Rptr,
                           int32_t* Rcol, double* Rval, double* W) {
  if (!p || l < 0 || l >= (int)p->P.levels.size()) { set_error("bad level"); return MAMG_ERR_ARG; }
  const mamg::DistLevel& D = p->P.levels[l];
  auto cpv = [](auto* dst, const auto& src) {
    if (dst && !src.empty()) std::memcpy(dst, src.data(), src.size() * sizeof(src[0]));
  };
  cpv(ghosts, D.ghosts);
  cpv(ghost_off, D.ghost_off);
  cpv(send_idx, D.send_idx);
  cpv(send_off, D.send_off);
  cpv(Aptr, D.A.ptr); cpv(Acol, D.A.col); cpv(Aval, D.A.val);
  cpv(Pptr, D.P.ptr); cpv(Pcol, D.P.col); cpv(Pval, D.P.val);
  cpv(Rptr, D.Rp.ptr); cpv(Rcol, D.Rp.col); cpv(Rval, D.Rp.val);
  cpv(W, D.W);
  return MAMG_OK;
}

int mamg_comm_id_bytes(void) { return 128; }

int mamg_comm_unique_id(void* id) {
  GUARD_BEGIN
  if (!id) { set_error("null id buffer"); return MAMG_ERR_ARG; }
  std::string err;
  int rc = mamg::dist_get_unique_id(id, &err);
  if (rc) set_error(err);
  return rc;
  GUARD_END
}

namespace {
// v: the host A_0, or (devA != nullptr) only its sizes -- A_0 then lives in
// HBM (mamg_setup_dist_device) and every path that would read it on the host
// is refused
int setup_dist_impl(const mamg::CsrView& v, const mamg::DevMat* devA, const int32_t* idofs, int64_t n_idofs,
                    const mamg_params* params, int rank, int nranks, const void* comm_id, int64_t rep_nodes,
                    mamg_dhandle** out) {
  TmpTrim trim(false);
  int rc;
  const int64_t nnz0 = devA ? devA->nnz : v.nnz();
  const mamg_params P = mamg::resolve_params(*params, idofs, n_idofs, v.n);   // the reference's Schwarz names
  mamg::Hierarchy H;
  std::string err;
  // parameters first: an invalid or single-GPU-only profile is refused
  // before the rank touches its GPU
  if ((rc = mamg::check_params(P, &err)) || (rc = mamg::dist_check(P, &err))) {
    set_error(err);
    return rc;
  }
  Seeds S(idofs, n_idofs, v.n, &P);
  // setup phases to stderr with print_level >= 2 (HAZmath's setup printing)
  auto t_0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (P.print_level < 2) return;
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[mamg] rank %d/%d setup: %-24s %.3f s\n", rank, nranks, what,
                 std::chrono::duration<double>(t - t_0).count());
    t_0 = t;
  };
  mamg::GhostLists ghosts;
  bool pre = false;
  // every rank builds the same hierarchy: on its own GPU when the profile is
  // the GPU setup's (bitwise equal to the host setup), else on the host
  rc = MAMG_ERR_UNSUPPORTED;
  mamg::GHier G;
  mamg::DevMat dA;
  bool on_device = false;   // rank-local operators built from G in HBM
  if (P.num_functions == 2 && P.node_block_smoother &&
      (P.AMG_type == MAMG_UA_AMG || P.sa_block_diag)) {
    G.device = P.device;
    mamg::dev_prereserve(P.device, nnz0, nranks);   // rank-local layout memory first
    if (devA) { dA = *devA; rc = MAMG_OK; }
    else rc = mamg::upload_a0(v, &G, &dA, &err);
    lap("A0 upload");
    if (!rc) rc = mamg::gpu_setup(dA, S.ptr, S.n, P, &G, &err);
    lap("GPU setup");
    // default: ghost lists marked on the GPU, the rank's operators cut out of
    // G in HBM.  MAMG_DIST_TEST=full: the whole hierarchy downloaded and
    // planned on the host; =rows: the rank's rows downloaded, planned on the
    // host (both bitwise the default; tests)
    const char* e = mamg::opt("MAMG_DIST_TEST");
    const std::string et = e ? e : "";
    const int mode = et == "full" ? 1 : et == "rows" ? 2 : 0;
    if (rc) {
    } else if (devA && (mode != 0 || G.generic)) {
      err = "multi-GPU setup from a device A_0: this profile plans on the host from the host matrix "
            "(CSR-layout smoothers, MAMG_DIST_TEST); pass the host CSR (mamg_setup_dist)";
      rc = MAMG_ERR_UNSUPPORTED;
      devA = nullptr;   // not a fallback: reported below
      mamg::dev_prereserve_release();
      set_error(err);
      return rc;
    } else if (mode == 1 || G.generic) {   // generic smoothers: the host plan of the whole hierarchy
      rc = mamg::ghier_download(G, v, &H, &err);
    } else {
      // node patches on N GPUs read and write within 3 hops of a rank's
      // nodes, seed rings within 2 Schwarz_maxlvl + 1
      const bool patches = P.Schwarz_levels >= 1 && P.Schwarz_type == MAMG_SCHWARZ_PATCHES;
      const bool rings = P.Schwarz_levels >= 1 && P.Schwarz_type == MAMG_SCHWARZ_RINGS;
      rc = mamg::ghier_download_rank(G, dA, v, rank, nranks, rep_nodes, P.post_fusion != 0, &H,
                                     &ghosts, &err, mode == 2, patches ? 3 : rings ? 2 * P.Schwarz_maxlvl + 1 : 1);
      pre = !rc;
      on_device = !rc && mode != 2;
    }
    lap(on_device ? "ghost lists" : "hierarchy download");
    if (rc && rc != MAMG_ERR_UNSUPPORTED) { mamg::dev_prereserve_release(); set_error(err); return rc; }
  }
  if (rc == MAMG_ERR_UNSUPPORTED && devA) {
    mamg::dev_prereserve_release();
    set_error("multi-GPU setup from a device A_0 needs the GPU setup's profiles (num_functions 2, node-block "
              "smoothers, UA or block-diagonal SA): " + err);
    return MAMG_ERR_UNSUPPORTED;
  }
  if (rc == MAMG_ERR_UNSUPPORTED) rc = mamg::host_setup(v, S.ptr, S.n, P, &H, &err);
  if (rc) { mamg::dev_prereserve_release(); set_error(err); return rc; }
  mamg::DistHandle* d = nullptr;
  rc = mamg::dist_upload(H, v, P, rank, nranks, comm_id, rep_nodes, &d, &err, pre ? &ghosts : nullptr,
                         on_device ? &G : nullptr, on_device ? &dA : nullptr);
  lap("plan + rank-local upload");
  mamg::dev_prereserve_release();
  if (rc) { set_error(err); return rc; }
  *out = new mamg_dhandle{d};
  return MAMG_OK;
}
}  // namespace

int mamg_setup_dist(const mamg_csr* A, const int32_t* idofs, int64_t n_idofs,
                    const mamg_params* params, int rank, int nranks, const void* comm_id,
                    int64_t rep_nodes, mamg_dhandle** out) {
  GUARD_BEGIN
  if (!out || !params) { set_error("null argument"); return MAMG_ERR_ARG; }
  *out = nullptr;
  mamg::CsrView v;
  int rc = to_view(A, &v);
  if (rc) return rc;
  return setup_dist_impl(v, nullptr, idofs, n_idofs, params, rank, nranks, comm_id, rep_nodes, out);
  GUARD_END
}

int mamg_setup_dist_device(const mamg_csr* dA, const int32_t* idofs, int64_t n_idofs,
                           const mamg_params* params, int rank, int nranks, const void* comm_id,
                           int64_t rep_nodes, mamg_dhandle** out) {
  GUARD_BEGIN
  if (!out || !params || !dA || !dA->rowptr || (dA->nnz > 0 && (!dA->colind || !dA->values))) {
    set_error("null argument");
    return MAMG_ERR_ARG;
  }
  *out = nullptr;
  if (dA->nrows <= 0 || dA->ncols <= 0 || dA->nnz < 0 || dA->nrows > INT32_MAX || dA->ncols > INT32_MAX) {
    set_error("bad CSR sizes");
    return MAMG_ERR_ARG;
  }
  mamg::DevMat M;
  M.n = dA->nrows;
  M.m = dA->ncols;
  M.nnz = dA->nnz;
  M.ptr = const_cast<int64_t*>(dA->rowptr);
  M.col = const_cast<int32_t*>(dA->colind);
  M.val = const_cast<double*>(dA->values);
  mamg::CsrView v;          // sizes only: nothing on the host reads A_0
  v.n = M.n;
  v.m = M.m;
  return setup_dist_impl(v, &M, idofs, n_idofs, params, rank, nranks, comm_id, rep_nodes, out);
  GUARD_END
}

int mamg_gen_bidomain_device(int dim, int64_t n, double gamma, double kappa1, double kappa2, int64_t nnz,
                             int64_t* d_rowptr, int32_t* d_colind, double* d_values) {
  GUARD_BEGIN
  if (!d_rowptr || !d_colind || !d_values) { set_error("null output buffer"); return MAMG_ERR_ARG; }
  std::string err;
  int rc = mamg::gen_bidomain_dev(dim, n, gamma, kappa1, kappa2, nnz, d_rowptr, d_colind, d_values, &err);
  if (rc) set_error(err);
  return rc;
  GUARD_END
}

int mamg_dist_range(const mamg_dhandle* h, int64_t* o0, int64_t* o1, int64_t* nv) {
  if (!h || !o0 || !o1 || !nv) { set_error("null argument"); return MAMG_ERR_ARG; }
  mamg::dist_range(h->d, o0, o1, nv);
  return MAMG_OK;
}

int mamg_dist_apply_bytes(const mamg_dhandle* h, double* bytes) {
  if (!h || !bytes) { set_error("null argument"); return MAMG_ERR_ARG; }
  *bytes = mamg::dist_apply_bytes(h->d);
  return MAMG_OK;
}

int mamg_dist_apply_launches(const mamg_dhandle* h, int64_t counts[5]) {
  if (!h || !counts) { set_error("null argument"); return MAMG_ERR_ARG; }
  mamg::dist_apply_launches(h->d, counts);
  return MAMG_OK;
}

int mamg_dist_apply_device(mamg_dhandle* h, const double* d_r, double* d_z, void* stream) {
  DEV_CALL(mamg::dist_apply(h->d, d_r, d_z, stream, &err))
}

int mamg_dist_apply_graph(mamg_dhandle* h, const double* d_r, double* d_z, void* stream) {
  DEV_CALL(mamg::dist_apply_graph(h->d, d_r, d_z, stream, &err))
}

int mamg_dist_graph_prepare(mamg_dhandle* h, const double* d_r, double* d_z) {
  DEV_CALL(mamg::dist_graph_prepare(h->d, d_r, d_z, &err))
}

int mamg_dist_virtual_apply_graph(mamg_dhandle** hs, int n, const double** d_r, double** d_z, void* stream) {
  GUARD_BEGIN
  if (!hs || n < 1 || !d_r || !d_z) { set_error("null argument"); return MAMG_ERR_ARG; }
  std::vector<mamg::DistHandle*> H(n);
  std::vector<const double*> R(d_r, d_r + n);
  std::vector<double*> Z(d_z, d_z + n);
  for (int i = 0; i < n; ++i) H[i] = hs[i]->d;
  std::string err;
  int rc = mamg::dist_virtual_apply_graph(H, R, Z, stream, &err);
  if (rc) set_error(err);
  return rc;
  GUARD_END
}

int mamg_dist_spmv_device(mamg_dhandle* h, const double* d_x, double* d_y, void* stream) {
  DEV_CALL(mamg::dist_spmv(h->d, d_x, d_y, stream, &err))
}

int mamg_dist_virtual_spmv(mamg_dhandle** hs, int n, const double** d_x, double** d_y, void* stream) {
  GUARD_BEGIN
  if (!hs || n < 1 || !d_x || !d_y) { set_error("null argument"); return MAMG_ERR_ARG; }
  std::vector<mamg::DistHandle*> H(n);
  std::vector<const double*> X(d_x, d_x + n);
  std::vector<double*> Y(d_y, d_y + n);
  for (int i = 0; i < n; ++i) H[i] = hs[i]->d;
  std::string err;
  int rc = mamg::dist_virtual_spmv(H, X, Y, stream, &err);
  if (rc) set_error(err);
  return rc;
  GUARD_END
}

int mamg_dist_time_apply(mamg_dhandle* h, const double* d_r, double* d_z, int reps, int mode,
                         double* ms, double* kernel_ms, double* class_bytes, void* stream) {
  DEV_CALL(mamg::dist_time_apply(h->d, d_r, d_z, reps, mode, ms, kernel_ms, class_bytes, stream, &err))
}

int mamg_dist_virtual_apply(mamg_dhandle** hs, int n, const double** d_r, double** d_z,
                            void* stream) {
  GUARD_BEGIN
  if (!hs || n < 1 || !d_r || !d_z) { set_error("null argument"); return MAMG_ERR_ARG; }
  std::vector<mamg::DistHandle*> H(n);
  std::vector<const double*> R(d_r, d_r + n);
  std::vector<double*> Z(d_z, d_z + n);
  for (int i = 0; i < n; ++i) H[i] = hs[i]->d;
  std::string err;
  int rc = mamg::dist_virtual_apply(H, R, Z, stream, &err);
  if (rc) set_error(err);
  return rc;
  GUARD_END
}

int mamg_dist_set_exchange(mamg_dhandle* h, const mamg_exchange* ex) {
  GUARD_BEGIN
  if (!h || !ex || !ex->sendrecv || !ex->allreduce) { set_error("null argument"); return MAMG_ERR_ARG; }
  std::string err;
  int rc = mamg::dist_set_exchange(h->d, *ex, &err);
  if (rc) set_error(err);
  return rc;
  GUARD_END
}

void mamg_dist_destroy(mamg_dhandle* h) {
  if (!h) return;
  mamg::dist_destroy(h->d);
  delete h;
}

int mamg_setup(const mamg_csr* A, const int32_t* idofs, int64_t n_idofs,
               const mamg_params* params, mamg_handle** out) {
  GUARD_BEGIN
  TmpTrim trim;
  if (!out || !params) { set_error("null argument"); return MAMG_ERR_ARG; }
  *out = nullptr;
  mamg::CsrView v;
  int rc = to_view(A, &v);
  if (rc) return rc;
  const mamg_params P = mamg::resolve_params(*params, idofs, n_idofs, v.n);   // the reference's Schwarz names
  mamg::Hierarchy H;
  std::string err;
  Seeds S(idofs, n_idofs, v.n, &P);
  rc = mamg::host_setup(v, S.ptr, S.n, P, &H, &err);
  if (rc) { set_error(err); return rc; }
  mamg::DeviceHandle* d = nullptr;
  rc = mamg::dev_upload(H, v, P, &d, &err);
  if (rc) { set_error(err); return rc; }
  *out = new mamg_handle{d};
  return MAMG_OK;
  GUARD_END
}

int mamg_sharded_galerkin_check(const mamg_csr* A, const mamg_csr* P, const mamg_csr* Ac, int nranks, int device,
                                int64_t* res6) {
  GUARD_BEGIN
  TmpTrim trim;
  if (!res6) { set_error("null argument"); return MAMG_ERR_ARG; }
  mamg::CsrView a, p, c;
  int rc;
  if ((rc = to_view(A, &a)) || (rc = to_view(P, &p)) || (rc = to_view(Ac, &c))) return rc;
  std::string err;
  if ((rc = mamg::sharded_galerkin_check(a, p, c, nranks, device, res6, &err))) set_error(err);
  return rc;
  GUARD_END
}

int mamg_setup_gpu(const mamg_csr* A, const int32_t* idofs, int64_t n_idofs,
                   const mamg_params* params, mamg_handle** out) {
  GUARD_BEGIN
  TmpTrim trim;
  if (!out || !params) { set_error("null argument"); return MAMG_ERR_ARG; }
  *out = nullptr;
  mamg::CsrView v;
  int rc = to_view(A, &v);
  if (rc) return rc;
  const mamg_params P = mamg::resolve_params(*params, idofs, n_idofs, v.n);   // the reference's Schwarz names
  std::string err;
  mamg::GHier G;
  G.device = P.device;
  mamg::DevMat dA;
  Seeds S(idofs, n_idofs, v.n, &P);
  mamg::dev_prereserve(P.device, v.nnz(), 1);   // layout memory before the setup churn
  if ((rc = mamg::upload_a0(v, &G, &dA, &err)) || (rc = mamg::gpu_setup(dA, S.ptr, S.n, P, &G, &err))) {
    mamg::dev_prereserve_release();
    set_error(err);
    return rc;
  }
  mamg::DeviceHandle* d = nullptr;
  rc = mamg::dev_from_ghier(&G, dA, P, &d, &err);
  mamg::dev_prereserve_release();
  if (rc) { set_error(err); return rc; }
  *out = new mamg_handle{d};
  return MAMG_OK;
  GUARD_END
}

int mamg_setup_gpu_device(const mamg_csr* dA, const int32_t* idofs, int64_t n_idofs,
                          const mamg_params* params, mamg_handle** out) {
  GUARD_BEGIN
  TmpTrim trim;
  if (!out || !params || !dA || !dA->rowptr || (dA->nnz > 0 && (!dA->colind || !dA->values))) {
    set_error("null argument");
    return MAMG_ERR_ARG;
  }
  const mamg_params P = mamg::resolve_params(*params, idofs, n_idofs, dA->nrows);   // the reference's Schwarz names
  *out = nullptr;
  if (dA->nrows <= 0 || dA->ncols <= 0 || dA->nnz < 0 || dA->nrows > INT32_MAX || dA->ncols > INT32_MAX) {
    set_error("bad CSR sizes");
    return MAMG_ERR_ARG;
  }
  mamg::DevMat M;
  M.n = dA->nrows;
  M.m = dA->ncols;
  M.nnz = dA->nnz;
  M.ptr = const_cast<int64_t*>(dA->rowptr);
  M.col = const_cast<int32_t*>(dA->colind);
  M.val = const_cast<double*>(dA->values);
  std::string err;
  mamg::GHier G;
  G.device = P.device;
  Seeds S(idofs, n_idofs, M.n, &P);
  mamg::dev_prereserve(P.device, M.nnz, 1);   // layout memory before the setup churn
  int rc = mamg::gpu_setup(M, S.ptr, S.n, P, &G, &err);
  if (rc) { mamg::dev_prereserve_release(); set_error(err); return rc; }
  mamg::DeviceHandle* d = nullptr;
  rc = mamg::dev_from_ghier(&G, M, P, &d, &err);
  mamg::dev_prereserve_release();
  if (rc) { set_error(err); return rc; }
  *out = new mamg_handle{d};
  return MAMG_OK;
  GUARD_END
}

int mamg_gpu_host_setup(const mamg_csr* A, const int32_t* idofs, int64_t n_idofs,
                        const mamg_params* params, mamg_hier** out) {
  GUARD_BEGIN
  TmpTrim trim;
  if (!out || !params) { set_error("null argument"); return MAMG_ERR_ARG; }
  *out = nullptr;
  mamg::CsrView v;
  int rc = to_view(A, &v);
  if (rc) return rc;
  const mamg_params P = mamg::resolve_params(*params, idofs, n_idofs, v.n);   // the reference's Schwarz names
  std::string err;
  mamg::GHier G;
  G.device = P.device;
  mamg::DevMat dA;
  Seeds S(idofs, n_idofs, v.n, &P);
  if ((rc = mamg::upload_a0(v, &G, &dA, &err)) || (rc = mamg::gpu_setup(dA, S.ptr, S.n, P, &G, &err))) {
    set_error(err);
    return rc;
  }
  mamg_hier* h = new mamg_hier();
  rc = mamg::ghier_download(G, v, &h->H, &err);
  if (rc) { set_error(err); delete h; return rc; }
  *out = h;
  return MAMG_OK;
  GUARD_END
}

int mamg_setup_timings(const mamg_handle* h, double* ms8) {
  if (!h || !ms8) { set_error("null argument"); return MAMG_ERR_ARG; }
  mamg::dev_setup_ms(h->d, ms8);
  return MAMG_OK;
}

int mamg_layout_timings(const mamg_handle* h, double* ms4) {
  if (!h || !ms4) { set_error("null argument"); return MAMG_ERR_ARG; }
  mamg::dev_layout_ms(h->d, ms4);
  return MAMG_OK;
}

int mamg_upload(const mamg_hier* h, const mamg_csr* A, const mamg_params* params,
                mamg_handle** out) {
  GUARD_BEGIN
  TmpTrim trim;
  if (!h || !out || !params) { set_error("null argument"); return MAMG_ERR_ARG; }
  const mamg_params P = mamg::resolve_like(*params, h->H.params);   // as the setup resolved it
  *out = nullptr;
  mamg::CsrView v = h->H.A0;
  if (A) {
    int rc = to_view(A, &v);
    if (rc) return rc;
    if (v.n != h->H.A0.n || v.nnz() != h->H.A0.nnz()) {
      set_error("A does not match the hierarchy's level-0 matrix");
      return MAMG_ERR_ARG;
    }
  }
  std::string err;
  mamg::DeviceHandle* d = nullptr;
  int rc = mamg::dev_upload(h->H, v, P, &d, &err);
  if (rc) { set_error(err); return rc; }
  *out = new mamg_handle{d};
  return MAMG_OK;
  GUARD_END
}

void mamg_destroy(mamg_handle* h) {
  if (!h) return;
  mamg::dev_destroy(h->d);
  delete h;
}

int64_t mamg_nrows(const mamg_handle* h) { return h ? mamg::dev_nrows(h->d) : (int64_t)MAMG_ERR_ARG; }
int mamg_num_levels(const mamg_handle* h) { return h ? mamg::dev_num_levels(h->d) : MAMG_ERR_ARG; }
int mamg_device_layout(const mamg_handle* h) { return h ? mamg::dev_layout(h->d) : MAMG_ERR_ARG; }
int mamg_level_format(const mamg_handle* h, int level) {
  if (!h || level < 0 || level >= mamg::dev_num_levels(h->d)) {
    mamg::set_error("mamg_level_format: bad handle or level");
    return MAMG_ERR_ARG;
  }
  return mamg::dev_level_format(h->d, level);
}

int mamg_handle_params(const mamg_handle* h, mamg_params* out) {
  if (!h || !out) { set_error("null argument"); return MAMG_ERR_ARG; }
  *out = mamg::dev_params(h->d);
  return MAMG_OK;
}

int mamg_kregion_info(const mamg_handle* h, double* ms, int cap, int* n, int* kept) {
  if (!h || !n || !kept || (cap > 0 && !ms)) { set_error("null argument"); return MAMG_ERR_ARG; }
  std::vector<double> v;
  mamg::dev_kregion(h->d, &v, kept);
  *n = (int)v.size();
  for (int i = 0; i < cap && i < (int)v.size(); ++i) ms[i] = v[i];
  return MAMG_OK;
}

int mamg_apply_bytes(const mamg_handle* h, double* total) {
  if (!h || !total) { set_error("null argument"); return MAMG_ERR_ARG; }
  *total = mamg::dev_apply_bytes(h->d);
  return MAMG_OK;
}

int mamg_apply(mamg_handle* h, const double* r, double* z) {
  DEV_CALL(mamg::dev_apply_host(h->d, r, z, &err))
}

int mamg_apply_device(mamg_handle* h, const double* d_r, double* d_z, void* stream) {
  DEV_CALL(mamg::dev_apply(h->d, d_r, d_z, stream, &err))
}

int mamg_spmv_device(mamg_handle* h, const double* d_x, double* d_y, void* stream) {
  DEV_CALL(mamg::dev_spmv(h->d, d_x, d_y, stream, &err))
}

int mamg_pcg_device(mamg_handle* h, const double* d_b, double* d_x, double tol, int maxiter,
                    int relativeconv, double* residuals, double* alphas, double* betas,
                    int* niters, void* stream) {
  DEV_CALL(mamg::dev_pcg(h->d, d_b, d_x, tol, maxiter, relativeconv, residuals, alphas, betas,
                         niters, stream, &err))
}

int mamg_time_apply(mamg_handle* h, const double* d_r, double* d_z, int reps, int mode,
                    double* ms_per_apply, double* kernel_ms, double* class_bytes, void* stream) {
  DEV_CALL(mamg::dev_time_apply(h->d, d_r, d_z, reps, mode, ms_per_apply, kernel_ms, class_bytes,
                                stream, &err))
}

}  // extern "C"
