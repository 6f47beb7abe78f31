// gsetup.h -- device-resident hierarchy produced by the GPU setup
// (gsetup.hip) and consumed by the apply-layout builder (device.hip).
// Plain pointers only (no HIP types), so host translation units can include it.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "host.h"

namespace mamg {

// device CSR: int64 row pointers, int32 sorted columns, fp64 values
struct DevMat {
  int64_t n = 0, m = 0, nnz = 0;
  int64_t* ptr = nullptr;
  int32_t* col = nullptr;
  double* val = nullptr;
};

// one level of the SA hierarchy on the device (num_functions 1 or 2); every
// field-major CSR follows the host setup's definition bit for bit.  The
// smoother is exactly one of: W (2x2 node blocks), WB (general block CSR:
// seed blocks that are not node-aligned, or overlapping seed rings), winv
// (point smoother, one weight per dof)
struct GLevel {
  int64_t n = 0;              // dofs (nf nv)
  bool coarsest = false;
  DevMat A;                   // level 0: the caller's matrix (not owned)
  DevMat P, R, AP;            // prolongation, restriction = P^T, A P
  double* W = nullptr;        // 2x2 smoother block per node, node-major (4 nv)
  DevMat WB;                  // general block smoother (host HostLevel::WB)
  double* winv = nullptr;     // point smoother weights (host HostLevel::winv)
  uint8_t* joined = nullptr;  // level 0: 1 if node I's two dofs form one seed block
  double* Ainv = nullptr;     // coarsest: dense inverse, n x n row-major, dof order
  int64_t* agg = nullptr;     // aggregate of each node (-1 isolated)
  int64_t nagg = 0;
  double w_sa = 0.0;
};

struct GHier {
  mamg_params params;
  int device = 0;
  bool generic = false;       // some level's smoother is WB or winv: CSR apply layout
  std::vector<GLevel> levels;
  std::vector<int32_t> seeds; // SCHWARZ_RINGS: the level-0 seeds (blocks built with the apply layout)
  std::vector<void*> allocs;  // every device buffer above (owned)
  double phase_ms[8] = {};    // setup phase timings (see gsetup.hip)
  ~GHier();
  void release(void* p);      // free one owned buffer now
};

// GPU setup of the nodal smoothed-aggregation hierarchy
// from a device CSR A0 (kept as level 0, not copied); idofs are host ints.
int gpu_setup(const DevMat& A0, const int32_t* idofs, int64_t n_idofs, const mamg_params& p,
              GHier* G, std::string* err);
// copy a GPU hierarchy into a host Hierarchy (same fields the host setup
// fills; level-0 A is the given host view)
int ghier_download(const GHier& G, const CsrView& A0, Hierarchy* H, std::string* err);
// row-sharded Galerkin product on nranks virtual ranks, each row compared bit
// for bit with the unsharded (A P) and with Ac (gsetup.hip; res[6])
int sharded_galerkin_check(const CsrView& A, const CsrView& P, const CsrView& Ac, int nranks, int device,
                           int64_t res[6], std::string* err);
// multi-GPU: download only what rank `rank` of `nranks` reads (its node rows
// of every distributed level, replicated levels whole, no R / aggregates) and
// compute the ghost lists on the device (build_dist_plan's `pre`); A0d is the
// device copy of the host A0.  matrices = false: level sizes, the coarsest
// inverse and the ghost lists only (the operators are then built on the device)
int ghier_download_rank(const GHier& G, const DevMat& A0d, const CsrView& A0, int rank, int nranks,
                        int64_t rep_nodes, bool post_fusion, Hierarchy* H,
                        std::vector<std::vector<std::vector<int64_t>>>* ghosts, std::string* err,
                        bool matrices = true, int hops0 = 1);
// SCHWARZ_RINGS level-0 blocks (one per seed, setup.cpp overlap_smoother's
// breadth-first rings: members sorted, <= mm dofs) and their Gauss-Jordan
// inverses, from the device CSR A.  Device buffers (hipMalloc, the caller
// frees them): blk[ns * mm] members of block k at k * mm, blen[ns],
// sq[ns] inclusive scan of blen^2, inv[sq[ns - 1]] the row-major inverse of
// block k at sq[k - 1]; nothing in *R is allocated on error.
struct RingBlocks {
  int32_t* blk = nullptr;
  int64_t *blen = nullptr, *sq = nullptr;
  double* inv = nullptr;
  int64_t ns = 0, ninv = 0;
  int mm = 0;
};
int ring_blocks_dev(const DevMat& A, const int32_t* seeds, int64_t ns, int maxlvl, int mm, RingBlocks* R,
                    std::string* err);
void ring_blocks_free(RingBlocks* R);
// the bidomain generator (gen.cpp) on the current device into caller
// buffers (ptr[2 nv + 1], colind / values[nnz] with nnz from
// gen_bidomain_size); bitwise the host generator's matrix
int gen_bidomain_dev(int dim, int64_t n, double gamma, double k1, double k2, int64_t nnz, int64_t* ptr,
                     int32_t* colind, double* values, std::string* err);
// host CSR -> HBM, buffers owned by G (G->device selects the GPU)
int upload_a0(const CsrView& A, GHier* G, DevMat* D, std::string* err);

// phase_ms slots
enum { GS_AGGREGATE = 0, GS_SMOOTHER = 1, GS_PROLONG = 2, GS_GALERKIN = 3, GS_COARSEST = 4,
       GS_LAYOUT = 5, GS_TOTAL = 6, GS_UPLOAD = 7 };

// device primitives (dprims.hip)
int dscan_incl_i64(const int64_t* in, int64_t* out, int64_t n, void* stream, std::string* err);
// one tiny scan on `stream` (its own buffers, kept): loads dprims' code
// object, which the runtime defers to the first launch (gsetup.hip warm_modules)
void dprims_warm(void* stream);
// one empty kernel of device.hip on `stream` (the same, for its code object)
void device_warm(void* stream);
int dsort_pairs_i32_i64(const int32_t* kin, int32_t* kout, const int64_t* vin, int64_t* vout,
                        int64_t n, int key_bits, void* stream, std::string* err);
int dsort_pairs_u64_i64(const uint64_t* kin, uint64_t* kout, const int64_t* vin, int64_t* vout,
                        int64_t n, int key_bits, void* stream, std::string* err);

}  // namespace mamg
