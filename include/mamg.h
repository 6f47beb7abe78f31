/*
 * mamg.h -- C-ABI of the MI355X-native metric-AMG preconditioner.
 *
 * This is the drop-in boundary for the reference's `metric_mono` hot path.
 * In the reference the boundary is Python -> SWIG (haznics) -> HAZmath C:
 *
 *   metricAMG(A, W, idofs=interface_dofs, parameters=parameters)
 *       /root/reference/src/utils.py:86  (without idofs: :88)
 *   BB * r   (cbc.block operator -> HAZmath precond fct, one cycle per call,
 *             `maxit: 1` /root/reference/src/amg_parameters.py:71)
 *       invoked by ConjGrad  /root/reference/src/bidomain_3d.py:149-150
 *   haznics.create_dvector / dvec_create_p / create_ivector  src/utils.py:104-111
 *   PETSc_to_dCSRmat(A)                                      src/utils.py:96,108
 *   haznics.fenics_metric_amg_solver_dcsr(A, b, x, idofs)    src/utils.py:119
 *
 * Conventions: plain pointers and sizes only; 0 = success, negative = error
 * (message via mamg_last_error(), thread-local); no exceptions cross the ABI;
 * the caller owns every input buffer (setup reads them, never keeps them);
 * the handle owns all device memory.  One handle per host thread / stream.
 * All arithmetic is IEEE binary64.  Matrices are CSR with int64 row pointers,
 * int32 column indices, column indices sorted within a row.
 */
#ifndef MAMG_H
#define MAMG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MAMG_ABI_VERSION 4

/* ---- status codes ---------------------------------------------------- */
enum {
  MAMG_OK = 0,
  MAMG_ERR_ARG = -1,          /* bad argument / shape                         */
  MAMG_ERR_HIP = -2,          /* HIP runtime error (no device, OOM, launch)   */
  MAMG_ERR_SETUP = -3,        /* hierarchy construction failed                */
  MAMG_ERR_UNSUPPORTED = -4,  /* parameter combination not implemented        */
  MAMG_ERR_NOMEM = -5,        /* host allocation failed                       */
  MAMG_ERR_BREAKDOWN = -6     /* PCG: <r,Br> < 0 (indefinite preconditioner)  */
};

/* ---- parameter enums (HAZmath names, build-defined values) ---------- */
enum { MAMG_UA_AMG = 1, MAMG_SA_AMG = 2 };                       /* AMG_type   */
enum { MAMG_V_CYCLE = 1, MAMG_W_CYCLE = 2 };                     /* cycle_type */
enum {                                                          /* smoother   */
  MAMG_SMOOTHER_JACOBI = 1,      /* x += w D^-1 r, w = relaxation             */
  MAMG_SMOOTHER_L1DIAG = 2,      /* x += w L1^-1 r, L1_ii = sum_j |a_ij|      */
  MAMG_SMOOTHER_JACOBI_RHO = 3,  /* x += (w/rho(D^-1A)) D^-1 r                */
  /* HAZmath's GS / SGS in a GPU-parallel order: multicolour node-block
   * Gauss-Seidel (forward / forward+backward), BSR2 layout only */
  MAMG_SMOOTHER_GS = 10,
  MAMG_SMOOTHER_SGS = 11,
  /* polynomial smoother (HAZmath/FASP SMOOTHER_POLY): Chebyshev of degree
   * poly_degree in W A on [relaxation/poly_ratio, relaxation], W the
   * JACOBI_RHO (block) smoother, applied as poly_degree weighted steps
   * x += w_k W (b - A x); pre steps k = 1..m, post m..1 (default profile) */
  MAMG_SMOOTHER_POLY = 12
};
enum {                                                   /* aggregation_type  */
  MAMG_VMB = 1, MAMG_MIS = 2, MAMG_MWM = 3, MAMG_HEC = 4, MAMG_HEM = 5
};  /* accepted: MIS (deterministic parallel MIS-2), HEM (parallel heavy-edge
       matching) and VMB (sequential Vanek-Mandel-
       Brezina; mamg_setup_gpu runs that one step on the host);
       MWM/HEC -> MAMG_ERR_UNSUPPORTED */
enum {                                                   /* Schwarz_type      */
  /* The reference's names (src/amg_parameters.py:83-87, src/utils.py:84):
   * multiplicative Schwarz on the OVERLAPPING blocks seed + Schwarz_maxlvl
   * ring.  SYMMETRIC with Schwarz_maxlvl >= 1 on a nodal system
   * (num_functions 2) runs as MAMG_SCHWARZ_PATCHES when the rings are 1-rings
   * and every node holds a seed (the bidomain), else as MAMG_SCHWARZ_RINGS
   * (sparse seed sets, e.g. EMI's interface); without seeds the level
   * smoother runs everywhere (Schwarz_levels resolved to 0).  With
   * Schwarz_maxlvl 0 the blocks are the seeds' nodes (no overlap) and the
   * type must match the smoother (SYMMETRIC: SGS, FORWARD: GS).  FORWARD /
   * BACKWARD on overlapping blocks and scalar systems return
   * MAMG_ERR_UNSUPPORTED. */
  MAMG_SCHWARZ_FORWARD = 1, MAMG_SCHWARZ_BACKWARD = 2, MAMG_SCHWARZ_SYMMETRIC = 3,
  MAMG_SCHWARZ_BLOCK_JACOBI = 4, /* additive non-overlapping seed blocks (GPU) */
  MAMG_SCHWARZ_ADDITIVE = 5,     /* additive overlapping seed + maxlvl-ring blocks
                                    (sparse seed sets, e.g. 3D-1D; CSR layout) */
  /* symmetric multiplicative Schwarz on the seeds' overlapping 1-ring blocks
     (the reference's SCHWARZ_SYMMETRIC with Schwarz_maxlvl 1): one patch per
     node = both fields of its closed neighbourhood, exact local solves, in a
     distance-3 multicolour order; level 0, BSR2 layout, 1 or N GPUs; needs a
     seed dof on every node (the bidomain's idofs) */
  MAMG_SCHWARZ_PATCHES = 6,
  /* the level smoother applied to NON-overlapping seed blocks (a seed plus
     the non-seed dofs that join it, <= Schwarz_mmsize): additive with the
     Jacobi family, multicolour forward with GS, symmetric with SGS (for the
     bidomain: node-block SGS on level 0) */
  MAMG_SCHWARZ_SEED_BLOCKS = 7,
  /* symmetric multiplicative Schwarz on one block per seed = the seed and its
     breadth-first Schwarz_maxlvl ring (<= Schwarz_mmsize dofs), exact local
     solves, blocks in a greedy conflict-colour order (a substitution for
     HAZmath's sequential seed order: the same blocks and local solves in
     another multiplicative order; the oracle's seed-order sweep gives the
     same EMI PCG counts, tests/test_rings_oracle.py), plus node-block GS on
     the dofs in no block (src/utils.py:84: "the interface_dofs has the
     Schwarz and the rest the GS smoother"): the reference's SCHWARZ_SYMMETRIC
     for any seed set that is not one seed per node with 1-rings (EMI's
     interface seeds, the default dict of src/utils.py:60-82); level 0, BSR2
     layout (num_functions 2), 1 or N GPUs */
  MAMG_SCHWARZ_RINGS = 8
};
enum { MAMG_OFF = 0, MAMG_ON = 1 };
enum {                                                   /* strength_measure  */
  /* J strong for I iff |a_IJ| >= strong_coupled * (the row's largest
   * off-diagonal |a_IK|): the default, because the classical measure below
   * collapses the bidomain hierarchy at strong_coupled 0.1 */
  MAMG_STRENGTH_ROWMAX = 1,
  /* classical: |a_IJ| >= strong_coupled * sqrt(|a_II a_JJ|) (Vanek, Mandel,
   * Brezina 1996; the measure HAZmath's aggregations are described with) */
  MAMG_STRENGTH_DIAG = 0
};
enum { MAMG_COARSE_DENSE = 32 };  /* coarse_solver: 32 (UMFPACK in HAZmath)  */

/* Parameter dictionary keys of /root/reference/src/amg_parameters.py:67-89
 * (and src/utils.py:60-82), same names, POD, versioned by abi_version. */
typedef struct mamg_params {
  int32_t abi_version;       /* = MAMG_ABI_VERSION                           */
  int32_t AMG_type;          /* MAMG_SA_AMG (default) | MAMG_UA_AMG          */
  int32_t cycle_type;        /* MAMG_V_CYCLE (default) | MAMG_W_CYCLE        */
  int32_t max_levels;        /* 20                                           */
  int32_t maxit;             /* cycles per apply, 1                          */
  int32_t smoother;          /* MAMG_SMOOTHER_JACOBI_RHO (mamg_params_default) */
  double relaxation;         /* 4/3                                          */
  int32_t presmooth_iter;    /* 1                                            */
  int32_t postsmooth_iter;   /* 1                                            */
  int32_t coarse_dof;        /* 100                                          */
  int32_t coarse_solver;     /* 32 -> dense direct                           */
  int32_t coarse_scaling;    /* MAMG_OFF | MAMG_ON: e <- <b_c,e>/<A_c e,e> e  */
  int32_t aggregation_type;  /* MAMG_MIS (parallel MIS-2) | MAMG_HEM | MAMG_VMB */
  double strong_coupled;     /* SoC threshold theta, 0.0                     */
  int32_t max_aggregation;   /* accepted, unused by MIS-2 (documented)       */
  int32_t amli_degree;       /* accepted, unused (no AMLI cycle)             */
  int32_t Schwarz_levels;    /* 1: seed-block Jacobi on level 0 if idofs     */
  int32_t Schwarz_mmsize;    /* max dofs per seed block, 100                 */
  int32_t Schwarz_maxlvl;    /* 1: seed + joined 1-ring; 0: seed node only   */
  int32_t Schwarz_type;      /* MAMG_SCHWARZ_BLOCK_JACOBI                    */
  int32_t Schwarz_blksolver; /* 32 -> dense block inverse                    */
  int32_t print_level;       /* 0 silent                                     */
  double sa_omega;           /* prolongator smoothing numerator, 4/3         */
  int32_t rho_iters;         /* 0: Gershgorin bound of rho(D^-1 A)           */
  int32_t max_coarse_dense;  /* largest coarsest level for dense solve, 8192 */
  int32_t device;            /* HIP device ordinal, 0                        */
  int32_t spmv_lanes;        /* 0 = auto; else lanes per row (2..64, pow2)   */
  /* nodal (systems) aggregation, build-defined extension: dofs field-major,
   * dof = f*nv + node for f < num_functions (the monolithic [u1; u2] order of
   * ii_convert, src/bidomain_3d.py:124,138).  >1 aggregates nodes with a
   * block-norm strength and keeps one coarse column per field/aggregate. */
  int32_t num_functions;     /* 1                                            */
  int32_t node_block_smoother; /* nodal: node-block Jacobi where no seed blocks (1) */
  int32_t sa_block_diag;     /* nodal: smooth P with node-block D^-1 (1)     */
  /* BSR2 device path: fold prolongation into the first post-smoothing sweep,
   * x = x1 + P e + W (r1 - (A P) e), with A P kept from the Galerkin product
   * (one pass over [P | AP] instead of P then A).  1 */
  int32_t post_fusion;
  /* MAMG_SMOOTHER_POLY: Chebyshev degree (1..8, 2) and interval ratio (16) */
  int32_t poly_degree;
  double poly_ratio;
  /* strength of connection: MAMG_STRENGTH_ROWMAX (default) | MAMG_STRENGTH_DIAG
   * (ABI 4) */
  int32_t strength_measure;
} mamg_params;

/* Host CSR view (caller-owned). */
typedef struct mamg_csr {
  int64_t nrows, ncols, nnz;
  const int64_t* rowptr;   /* nrows+1 */
  const int32_t* colind;   /* nnz, sorted per row */
  const double* values;    /* nnz */
} mamg_csr;

typedef struct mamg_handle mamg_handle;   /* device hierarchy + workspace   */
typedef struct mamg_hier mamg_hier;       /* host hierarchy (setup result)  */

/* ---- library ---------------------------------------------------------- */
int mamg_abi_version(void);
/* Release the device blocks the GPU setups keep cached for the process's next
 * setup (their temporaries: after a setup returns, none is in use).  Library
 * housekeeping with no reference counterpart: a caller sharing the GPU with
 * other allocators calls it after its setups; the library also releases them
 * by itself when one of its own allocations runs out of HBM. */
int mamg_release_setup_cache(void);
/* Bound of that cache, bytes per device: at the end of every setup the idle
 * blocks above it are freed (largest first).  bytes < 0: the default, an
 * eighth of the device's HBM; 0: everything released after every setup.
 * The SpGEMM staging block of the GPU setup counts against it. */
int mamg_set_setup_cache_limit(int64_t bytes);
/* Idle cached bytes of a device and its current limit (either may be NULL). */
int mamg_setup_cache_bytes(int device, int64_t* idle_bytes, int64_t* limit_bytes);
const char* mamg_last_error(void);
void mamg_params_default(mamg_params* p);

/* ---- problem generators (the reference's FEniCS assembly restated;
 *      src/bidomain_2d.py:51-99, meshes src/utils.py:149-182) ------------- */
/* Sizes of the monolithic bidomain system on UnitSquare/UnitCube(n). */
int mamg_gen_bidomain_size(int dim, int64_t n, int64_t* nrows, int64_t* nnz);
/* Fill caller buffers rowptr[nrows+1], colind[nnz], values[nnz]. */
int mamg_gen_bidomain(int dim, int64_t n, double gamma, double kappa1,
                      double kappa2, int64_t* rowptr, int32_t* colind,
                      double* values);

/* The same matrix built in device memory by gfx950 kernels (bitwise the host
 * generator's), into caller buffers d_rowptr[nrows+1], d_colind / d_values[nnz]
 * (sizes from mamg_gen_bidomain_size); synchronous.  Multi-GPU ranks generate
 * A_0 in HBM instead of holding it on the host. */
int mamg_gen_bidomain_device(int dim, int64_t n, double gamma, double kappa1, double kappa2, int64_t nnz,
                             int64_t* d_rowptr, int32_t* d_colind, double* d_values);

/* Manufactured solution of the bidomain drivers (src/bidomain_2d.py:7-99,
 * src/bidomain_3d.py:7-49): b[nrows] = the right-hand side of the system
 * mamg_gen_bidomain builds (loads, full-flux terms on tags 3/4, Dirichlet
 * lifting; exact values on the Dirichlet rows). */
int mamg_gen_bidomain_mms(int dim, int64_t n, double gamma, double kappa1,
                          double kappa2, double* b);
/* H1 errors err[2] = |u1 - u1h|_1, |u2 - u2h|_1 of a solution x[nrows]
 * (errornorm(u, uh, 'H1'), src/bidomain_2d.py:239-240). */
int mamg_bidomain_mms_error(int dim, int64_t n, double gamma, double kappa1,
                            double kappa2, const double* x, double* err);

/* ---- host setup (no GPU needed).  The hierarchy keeps a VIEW of A (level
 *      0): the caller keeps A alive until mamg_hier_free. ------------------ */
/* Replaces metricAMG.__init__'s HAZmath setup (src/utils.py:86).  idofs may
 * be NULL (n_idofs = 0): then no seed blocks (src/utils.py:88). */
int mamg_host_setup(const mamg_csr* A, const int32_t* idofs, int64_t n_idofs,
                    const mamg_params* params, mamg_hier** out);
void mamg_hier_free(mamg_hier* h);
int mamg_hier_num_levels(const mamg_hier* h);
/* The parameters the setup ran with, after the reference's Schwarz names are
 * resolved (SCHWARZ_SYMMETRIC on the 1-rings of a nodal system ->
 * SCHWARZ_PATCHES; see the Schwarz_type enum). */
int mamg_hier_params(const mamg_hier* h, mamg_params* out);
/* Sizes of level l: n, nnz(A), nnz(P), nnz(R), nnz(WB) (0 if point smoother),
 * ncoarse (n of level l+1, 0 on the coarsest). */
int mamg_hier_level_sizes(const mamg_hier* h, int l, int64_t* sizes6);
/* Export level l into caller buffers (any pointer may be NULL to skip):
 * A (ptr,col,val), P, R, WB (CSR), winv[n], agg[n] (int64), Ainv[n*n]. */
int mamg_hier_level_export(const mamg_hier* h, int l,
                           int64_t* Aptr, int32_t* Acol, double* Aval,
                           int64_t* Pptr, int32_t* Pcol, double* Pval,
                           int64_t* Rptr, int32_t* Rcol, double* Rval,
                           int64_t* Wptr, int32_t* Wcol, double* Wval,
                           double* winv, int64_t* agg, double* Ainv);

/* ---- multi-GPU partition plan (host only) --------- */
/* Rank `rank` of `nranks`: contiguous node ranges per level, ghost lists,
 * send lists, rank-local BSR2 matrices.  Levels with <= rep_nodes nodes (and
 * all coarser ones) are replicated. */
typedef struct mamg_plan mamg_plan;
int mamg_hier_dist_plan(const mamg_hier* h, int rank, int nranks, int64_t rep_nodes,
                        mamg_plan** out);
void mamg_plan_free(mamg_plan* p);
int mamg_plan_num_levels(const mamg_plan* p);
/* s[16]: nv, replicated, coarsest, o0, o1, nghost, nsend, nbA, nrA, ncA,
 *        nbP, nrP, ncP, nbR, nrR, ncR */
int mamg_plan_level_sizes(const mamg_plan* p, int l, int64_t* s);
/* Export (any pointer may be NULL): ghosts[nghost], ghost_off[nranks+1],
 * send_idx[nsend], send_off[nranks+1], A/P/Rp as BSR2 (ptr, col, val[4 nb]),
 * W[4 nloc]. */
int mamg_plan_level_export(const mamg_plan* p, int l, int64_t* ghosts, int64_t* ghost_off,
                           int64_t* send_idx, int64_t* send_off,
                           int64_t* Aptr, int32_t* Acol, double* Aval,
                           int64_t* Pptr, int32_t* Pcol, double* Pval,
                           int64_t* Rptr, int32_t* Rcol, double* Rval, double* W);

/* ---- multi-GPU apply (one process per GPU, RCCL over xGMI) ------------- */
typedef struct mamg_dhandle mamg_dhandle;
/* size of the RCCL unique id (128); rank 0 creates it, every rank passes it */
int mamg_comm_id_bytes(void);
int mamg_comm_unique_id(void* id);
/* Every rank passes the same global A / idofs / params (the setup -- on the
 * rank's GPU where the profile allows it, else on the host -- is replicated
 * and deterministic) and keeps only its node range of each level; levels
 * with <= rep_nodes nodes are replicated.  V and W cycles, coarse-grid
 * scaling, nu1 / nu2 >= 1; Jacobi-family, POLY and multicolour GS / SGS
 * smoothers on BSR2 (nodal) hierarchies.  SCHWARZ_PATCHES / SCHWARZ_RINGS,
 * CSR-layout hierarchies and maxit > 1 return MAMG_ERR_UNSUPPORTED. */
int mamg_setup_dist(const mamg_csr* A, const int32_t* idofs, int64_t n_idofs,
                    const mamg_params* params, int rank, int nranks, const void* comm_id,
                    int64_t rep_nodes, mamg_dhandle** out);
/* Same with A_0's rowptr / colind / values in device memory (read during
 * setup only), e.g. from mamg_gen_bidomain_device: no rank holds the global
 * matrix on the host.  Covers the GPU setup's node-block profiles (the rank's
 * operators are cut out of the hierarchy in HBM); profiles that plan on the
 * host return MAMG_ERR_UNSUPPORTED. */
int mamg_setup_dist_device(const mamg_csr* dA, const int32_t* idofs, int64_t n_idofs,
                           const mamg_params* params, int rank, int nranks, const void* comm_id,
                           int64_t rep_nodes, mamg_dhandle** out);
/* local node range [o0, o1) of level 0; local vectors are field-major
 * [u1(o0:o1); u2(o0:o1)] of length 2*(o1-o0) */
int mamg_dist_range(const mamg_dhandle* h, int64_t* o0, int64_t* o1, int64_t* nv);
int mamg_dist_apply_bytes(const mamg_dhandle* h, double* bytes);
/* what one mamg_dist_apply_device issues on this rank (counted from its op
 * list, nothing launched): counts[0] kernels, [1] RCCL send / receive groups,
 * [2] point-to-point messages, [3] all-reduces, [4] side-stream forks */
int mamg_dist_apply_launches(const mamg_dhandle* h, int64_t counts[5]);
int mamg_dist_apply_device(mamg_dhandle* h, const double* d_r_local, double* d_z_local,
                           void* stream);
/* The same apply replayed from a hipGraph: captured on the first call per
 * (d_r_local, d_z_local) pair, with the rank's kernels, the interior-row
 * side-stream fork and the RCCL send / receive groups and all-reduces inside
 * the capture, then one hipGraphLaunch per call on `stream`.  Bitwise the
 * eager apply's result (same kernels, same order).  MAMG_ERR_UNSUPPORTED for
 * a handle without an RCCL communicator and more than one rank (host-staged
 * or virtual exchanges) and after a failed capture on the handle (the message
 * names the capture error; mamg_dist_apply_device stays available).  No
 * reference counterpart (the reference is serial). */
int mamg_dist_apply_graph(mamg_dhandle* h, const double* d_r_local, double* d_z_local, void* stream);
/* Capture (or find) that graph without launching it: every rank can capture
 * and agree on the outcome before any rank launches a graph whose RCCL calls
 * wait for its peers. */
int mamg_dist_graph_prepare(mamg_dhandle* h, const double* d_r_local, double* d_z_local);
/* y = A x on the rank's rows (the PCG operator; x, y local field-major
 * slices): forward halo of x, then the rank-local A.  Replaces the A * d
 * product inside cbc.block ConjGrad (src/bidomain_3d.py:149) on N GPUs. */
int mamg_dist_spmv_device(mamg_dhandle* h, const double* d_x_local, double* d_y_local, void* stream);
/* mode 0: eager, events around the level-0 residual and K launches; 1:
 * eager, events around every op; 2: mamg_dist_apply_graph replays (events
 * around the whole run only, kernel_ms zero) */
int mamg_dist_time_apply(mamg_dhandle* h, const double* d_r, double* d_z, int reps, int mode,
                         double* ms_per_apply, double* kernel_ms, double* class_bytes,
                         void* stream);
/* Test mode: handles created with comm_id == NULL (no RCCL) on one device;
 * apply all n ranks in lockstep, exchanges as device copies. */
int mamg_dist_virtual_apply(mamg_dhandle** hs, int n, const double** d_r, double** d_z,
                            void* stream);
int mamg_dist_virtual_spmv(mamg_dhandle** hs, int n, const double** d_x, double** d_y, void* stream);
/* The virtual ranks' lockstep apply captured into one hipGraph and replayed
 * once (tests: the graph path against the eager lockstep run). */
int mamg_dist_virtual_apply_graph(mamg_dhandle** hs, int n, const double** d_r, double** d_z,
                                  void* stream);
void mamg_dist_destroy(mamg_dhandle* h);
/* Host-staged exchange backend: a pluggable transport for a handle made
 * with comm_id == NULL (one process per rank, e.g. torch.distributed gloo).
 * The pack / unpack kernels, the reverse-add in rank order and the op
 * schedule are the RCCL path's; only the transport differs: payloads are
 * staged through pinned host buffers and handed to the callbacks (0 = ok).
 * Arrays are indexed by rank; entries for this rank and zero counts are
 * unused.  Replaces RCCL where it cannot run (two ranks on one GPU). */
typedef struct mamg_exchange {
  void* ctx;
  /* send scount[q] doubles from send[q] to every rank q, receive rcount[q]
     doubles from q into recv[q] */
  int (*sendrecv)(void* ctx, int nranks, double* const* send, const int64_t* scount,
                  double* const* recv, const int64_t* rcount);
  /* in-place sum of buf[count] over all ranks (the same result on every rank) */
  int (*allreduce)(void* ctx, double* buf, int64_t count);
} mamg_exchange;
int mamg_dist_set_exchange(mamg_dhandle* h, const mamg_exchange* ex);

/* ---- device hierarchy ------------------------------------------------- */
/* Host setup + upload.  Level-0 matrix is uploaded from A directly. */
int mamg_setup(const mamg_csr* A, const int32_t* idofs, int64_t n_idofs,
               const mamg_params* params, mamg_handle** out);
/* GPU setup: the same hierarchy as mamg_setup, bit
 * for bit, built by gfx950 kernels -- strength, MIS-2 / HEM aggregation (VMB:
 * its one sequential step on the host), smoothers, SA prolongator, Galerkin
 * products, coarsest inverse -- and the apply layouts built in HBM (no host
 * round trip).  Covers num_functions 1 and 2 with every smoother the host
 * setup builds: node blocks, general (not node-aligned) seed blocks,
 * SCHWARZ_ADDITIVE rings, SCHWARZ_PATCHES / SCHWARZ_RINGS level-0 Schwarz,
 * point smoothers; nodal or point SA.  Other profiles (num_functions > 2, a
 * hash SpGEMM row of more than 2048 distinct columns) return
 * MAMG_ERR_UNSUPPORTED (use mamg_setup).  Replaces the setup half of
 * metricAMG.__init__ (src/utils.py:86).  A: host CSR, copied once. */
int mamg_setup_gpu(const mamg_csr* A, const int32_t* idofs, int64_t n_idofs,
                   const mamg_params* params, mamg_handle** out);
/* Same with A's rowptr/colind/values in device memory (read during setup
 * only; the caller may free them afterwards).  idofs: host array. */
int mamg_setup_gpu_device(const mamg_csr* dA, const int32_t* idofs, int64_t n_idofs,
                          const mamg_params* params, mamg_handle** out);
/* GPU setup, hierarchy copied back into a host mamg_hier (tests, multi-GPU
 * planning); the hierarchy keeps a view of A as mamg_host_setup does. */
int mamg_gpu_host_setup(const mamg_csr* A, const int32_t* idofs, int64_t n_idofs,
                        const mamg_params* params, mamg_hier** out);
/* Setup phase timings of a GPU-setup handle, ms[8]: aggregation, smoothers,
 * prolongator, Galerkin, coarsest, apply-layout build, setup total, A upload
 * (zeros for handles from mamg_setup / mamg_upload). */
int mamg_setup_timings(const mamg_handle* h, double* ms8);
/* The apply-layout phase of any handle split, ms[4]: layout build (device
 * formats of every level), level-0 K value region trials (bounded by time and
 * free HBM), operator re-homing, finish (tail plan,
 * final synchronisation). */
int mamg_layout_timings(const mamg_handle* h, double* ms4);

/* Upload an existing host hierarchy (level 0 matrix taken from A). */
int mamg_upload(const mamg_hier* h, const mamg_csr* A, const mamg_params* params,
                mamg_handle** out);
void mamg_destroy(mamg_handle* h);

int64_t mamg_nrows(const mamg_handle* h);
int mamg_num_levels(const mamg_handle* h);
/* Device layout chosen at upload: 0 = CSR (general), 1 = BSR2 (nodal
 * hierarchy with num_functions == 2 and node-block smoothers). */
int mamg_device_layout(const mamg_handle* h);
/* Storage of level l's operator on the device (BSR2 layout), bit flags:
 * MAMG_FMT_SELL (sliced-ELL, one lane per node row), MAMG_FMT_SYM (3 doubles
 * per symmetric 2x2 block), MAMG_FMT_POST_FUSED (prolongation fused with the
 * first post sweep), MAMG_FMT_POST_K (... through one stored operator
 * K = P - W (A P): z = x1 + W r1 + K e; else through [P | AP]),
 * MAMG_FMT_POST_SELL (K stored sliced-ELL), MAMG_FMT_HALF (A stored as its
 * upper half, ELL-64, lower blocks read through their mirrors), MAMG_FMT_BANDS
 * (the half-symmetric kernel walks the rows in plane bands per XCD; order
 * only, results are bitwise those of row order).
 * Returns flags >= 0, or < 0. */
enum { MAMG_FMT_SELL = 1, MAMG_FMT_SYM = 2, MAMG_FMT_POST_FUSED = 4, MAMG_FMT_POST_K = 8,
       MAMG_FMT_POST_SELL = 16, MAMG_FMT_HALF = 32, MAMG_FMT_BANDS = 64,
       MAMG_FMT_PATCHES = 128,  /* smoother: multiplicative node-patch Schwarz (SCHWARZ_PATCHES) */
       MAMG_FMT_GS = 256,       /* smoother: multicolour node-block GS / SGS sweeps */
       MAMG_FMT_RINGS = 512,    /* smoother: multiplicative seed-ring Schwarz + GS on the rest (SCHWARZ_RINGS) */
       MAMG_FMT_R_BANDS = 1024,    /* restriction rows walked plane band by plane band per XCD */
       MAMG_FMT_K_COL16 = 2048 };  /* K's columns as 16-bit offsets from a per-slice base */
int mamg_level_format(const mamg_handle* h, int level);
/* The parameters the handle runs (as mamg_hier_params). */
int mamg_handle_params(const mamg_handle* h, mamg_params* out);
/* Placement of the level-0 K values: the K kernel's
 * time per candidate memory region tried at upload, ms[0 .. *n) (at most cap),
 * and the index kept (*kept = -1: no selection ran). */
int mamg_kregion_info(const mamg_handle* h, double* ms, int cap, int* n, int* kept);
/* Algorithmic HBM bytes of one apply (SURVEY 8d formula) and of its dominant
 * kernel class; see DESIGN.md section 4. */
int mamg_apply_bytes(const mamg_handle* h, double* total_bytes);

/* z = B r : one preconditioner application (`maxit` cycles from x0 = 0).
 * Host pointers (copies in/out, synchronous). */
int mamg_apply(mamg_handle* h, const double* r, double* z);
/* Device pointers, enqueued on `stream` (hipStream_t, NULL = default).
 * r is not modified; r and z must not alias. */
int mamg_apply_device(mamg_handle* h, const double* d_r, double* d_z,
                      void* stream);
/* y = A x with the level-0 operator (device pointers). */
int mamg_spmv_device(mamg_handle* h, const double* d_x, double* d_y,
                     void* stream);

/* Device-resident preconditioned CG with cbc.block ConjGrad semantics
 * (src/bidomain_3d.py:149-160): x0 = d_x on entry, residuals = sqrt(<r,Br>),
 * stop when residual <= tol (times residual[0] if relativeconv) or after
 * maxiter iterations.  residuals[maxiter+1], alphas[maxiter], betas[maxiter]
 * are host buffers; *niters = len(residuals)-1.  Returns MAMG_ERR_BREAKDOWN
 * (x restored as cbc.block does) if <r,Br> < 0. */
int mamg_pcg_device(mamg_handle* h, const double* d_b, double* d_x, double tol,
                    int maxiter, int relativeconv, double* residuals,
                    double* alphas, double* betas, int* niters, void* stream);

/* Timing hook for bench/profiling: run `reps` applies eagerly (kernel by
 * kernel, no graph) on `stream`, timed with HIP events recorded on that
 * stream.  *ms_per_apply = mean wall time per apply.  kernel_ms[16] (if
 * non-NULL) = mean ms per apply per kernel class:
 * mode 0 instruments only classes 0 and 1 (the level-0 residual SpMV and the
 * level-0 post-smoothing / fused prolongation kernel, the two dominant
 * kernels), mode 1 instruments every launch.  class_bytes[16] (if non-NULL) =
 * algorithmic HBM bytes per apply of each class. */
int mamg_time_apply(mamg_handle* h, const double* d_r, double* d_z, int reps,
                    int mode, double* ms_per_apply, double* kernel_ms,
                    double* class_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MAMG_H */
