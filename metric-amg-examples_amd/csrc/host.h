// host.h -- host-side data structures of the metric-AMG hierarchy.
//
// The host setup restates the oracle's algorithm (oracle/mamg_oracle.py) as a
// fixed sequence of IEEE binary64 operations; this translation unit family is
// compiled with -ffp-contract=off so that the hierarchy is bitwise identical
// to the oracle's (tests/test_host_setup.py checks this).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "mamg.h"

namespace mamg {

struct CsrView {            // non-owning (caller's level-0 matrix)
  int64_t n = 0, m = 0;
  const int64_t* ptr = nullptr;
  const int32_t* col = nullptr;
  const double* val = nullptr;
  int64_t nnz() const { return n ? ptr[n] : 0; }
};

struct Csr {                // owning
  int64_t n = 0, m = 0;
  std::vector<int64_t> ptr;
  std::vector<int32_t> col;
  std::vector<double> val;
  int64_t nnz() const { return ptr.empty() ? 0 : ptr[n]; }
  CsrView view() const {
    CsrView v;
    v.n = n; v.m = m; v.ptr = ptr.data(); v.col = col.data(); v.val = val.data();
    return v;
  }
};

struct HostLevel {
  Csr A;                    // level 0: empty (the caller's matrix is used)
  std::vector<double> winv; // point smoother weights (empty if WB used)
  Csr WB;                   // seed-block smoother (level 0 with idofs)
  std::vector<double> Wn;   // or: 2x2 node blocks of nodes [wn0, wn0 + Wn.size()/4)
  int64_t wn0 = 0;          //     (multi-GPU rank slice, gsetup.hip ghier_download_rank)
  Csr P, R;                 // prolongation / restriction (R = P^T)
  Csr AP;                   // A P (Galerkin intermediate; kept for post fusion)
  std::vector<int64_t> agg; // aggregate id per row (-1 isolated)
  int64_t nagg = 0;
  double w_sa = 0.0;
  std::vector<double> Ainv; // dense inverse on the coarsest level (row-major)
  bool coarsest = false;
  int64_t n = 0;
};

struct Hierarchy {
  mamg_params params;
  CsrView A0;               // level-0 matrix (caller-owned during setup)
  std::vector<HostLevel> levels;
  std::vector<int32_t> seeds;   // SCHWARZ_RINGS: the level-0 seeds (the blocks are built with the apply layout)
  CsrView A(int l) const { return l == 0 ? A0 : levels[l].A.view(); }
};

// setup.cpp
// Vanek-Mandel-Brezina aggregation on a strength graph given as the CSR G
// (node graph or scalar matrix; weights |val|) and one strong flag per entry
// (symmetric pattern: no extras).  Used by the GPU setup, which builds G and
// the flags on the device and runs this sequential step on the host.
int aggregate_vmb_flags(const CsrView& G, const uint8_t* flag, std::vector<int64_t>* agg, int64_t* nagg,
                        std::string* err);

int host_setup(const CsrView& A, const int32_t* idofs, int64_t n_idofs,
               const mamg_params& p, Hierarchy* out, std::string* err);
mamg_params resolve_params(const mamg_params& in, const int32_t* idofs, int64_t n_idofs, int64_t n);
mamg_params resolve_like(const mamg_params& in, const mamg_params& built);
int check_params(const mamg_params& p, std::string* err);
int check_patch_seeds(const mamg_params& p, const int32_t* idofs, int64_t n_idofs, int64_t n, std::string* err);
int check_ring_seeds(const mamg_params& p, const int32_t* idofs, int64_t n_idofs, int64_t n, std::string* err);
// SCHWARZ_RINGS: most dofs per seed block (one 128-thread workgroup per block
// holds its residual in LDS; device.hip ring_kernel)
constexpr int RING_MAX_DOFS = 256;
// greedy first-fit colouring of seed blocks (members sorted, any order) in
// block order on the conflict graph: a member of one in the closed
// neighbourhood (A's pattern) of a member of the other (mamg_oracle.ring_colouring)
void ring_colouring(const CsrView& A, const std::vector<int64_t>& bptr, const std::vector<int32_t>& mem,
                    std::vector<int32_t>* colour);
// SMOOTHER_POLY step weights w[0..poly_degree) (oracle mamg_oracle.poly_weights)
constexpr int MAMG_POLY_MAX = 8;
int poly_weights(const mamg_params& p, double* w);
// level-0 seed (Schwarz) blocks from idofs (src/utils.py:84-86).  Schwarz_maxlvl
// 0 = a seed's block is its own node without a ring, which with node-block
// smoothers is the node block: the seeds then change nothing and every level
// is node-aligned (BSR2 layout, GPU setup, multi-GPU; EMI's interface pairs)
inline bool seed_blocks_on(const mamg_params& p, int l, const int32_t* idofs, int64_t n_idofs) {
  return l == 0 && l < p.Schwarz_levels && idofs != nullptr && n_idofs > 0 && p.Schwarz_maxlvl >= 1;
}
// smoothing steps per sweep and their weights, pre order (1 step of weight 1
// for the Jacobi smoothers)
inline int smoother_steps(const mamg_params& p) {
  return p.smoother == MAMG_SMOOTHER_POLY ? p.poly_degree : 1;
}

// gen.cpp
int gen_bidomain_size(int dim, int64_t n, int64_t* nrows, int64_t* nnz);
int gen_bidomain(int dim, int64_t n, double gamma, double k1, double k2,
                 int64_t* rowptr, int32_t* colind, double* values);
// mms.cpp: manufactured-solution right-hand side and H1 errors
int gen_bidomain_mms(int dim, int64_t n, double gamma, double k1, double k2, double* b);
int bidomain_mms_error(int dim, int64_t n, double gamma, double k1, double k2, const double* x,
                       double* err);

// convert.cpp: field-major CSR (rows f*nr+I, cols g*nc+J, 2 fields) -> 2x2 BSR
struct HBsr {
  int64_t nr = 0, nc = 0;
  std::vector<int64_t> ptr;
  std::vector<int32_t> col;
  std::vector<double> val;   // 4 per block: (0,0) (0,1) (1,0) (1,1)
};
void to_bsr2(const CsrView& M, int64_t nr, int64_t nc, HBsr* B);
// node rows [r0, r1) only (B.nr = r1 - r0)
void to_bsr2_rows(const CsrView& M, int64_t nr, int64_t nc, int64_t r0, int64_t r1, HBsr* B);
// smoother matrix -> one 2x2 block per node; false if it couples two nodes
bool node_blocks_of(const CsrView& W, int64_t nv, std::vector<double>* blk);
// rows of P then rows of Q (same nr): M.ptr has 2 nr + 1 entries, row I of P in
// [ptr[2I], ptr[2I+1]), row I of Q in [ptr[2I+1], ptr[2I+2])
void merge_bsr_rows(const HBsr& P, const HBsr& Q, HBsr* M);
// sliced-ELL (slice height C) copy of a plain (ptr nr + 1) or merged (2 nr + 1)
// BSR2 matrix: block j of row I at soff[I / C] + C j + I % C; meta[I] = row
// length | (first-part length << 16); sym: diagonal pairs (2 per slot) then
// off-diagonals (1 per slot, at 2 nbs), else 4 doubles per slot; padding = 0
struct HSell {
  int64_t nr = 0, nbs = 0;
  std::vector<int64_t> soff;
  std::vector<int32_t> meta;
  std::vector<int32_t> col;
  std::vector<double> val;
  std::vector<int32_t> perm;   // sigma > 1: row of each slot (rows sorted by length per window)
};
int to_sell(const HBsr& B, bool sym, int C, int sigma, HSell* S, std::string* err);

// hash shared with the oracle (oracle/mamg_oracle.py:hash32)
inline uint32_t hash32(uint64_t i, int level) {
  uint32_t x = (uint32_t)(i & 0xFFFFFFFFu);
  uint32_t lv = (uint32_t)(((uint64_t)(int64_t)level * 0x85EBCA77ull) & 0xFFFFFFFFull);
  x = x * 0x9E3779B1u + lv;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

void set_error(const std::string& s);

}  // namespace mamg
