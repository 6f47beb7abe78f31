// dist.h -- rank-local plan of the row-partitioned V-cycle (see dist.cpp).
#pragma once
#include <string>
#include <vector>

#include "host.h"

namespace mamg {

struct DistLevel {
  int64_t nv = 0;                 // global nodes
  bool coarsest = false;
  bool replicated = false;        // computed redundantly on every rank
  std::vector<int64_t> own;       // [nranks+1] node ranges
  int64_t o0 = 0, o1 = 0, nloc = 0;
  std::vector<int64_t> ghosts;    // global ids, sorted (grouped by owner)
  std::vector<int64_t> ghost_off; // [nranks+1] ghost ranges per owner rank
  std::vector<int64_t> send_idx;  // owned local node indices, per dest rank
  std::vector<int64_t> send_off;  // [nranks+1]
  HBsr A;                         // owned rows x [owned | ghost] (replicated: global)
  HBsr P;                         // owned fine rows x level l+1 local (or global)
  HBsr Rp;                        // transpose of P (partial restriction)
  HBsr PA;                        // post fusion: merged [P_loc | AP_loc] (kpost == false)
  HBsr K;                         // post fusion: K_loc = P_loc - W (AP)_loc (kpost == true)
  std::vector<double> W;          // 4 per owned node
};

struct DistPlan {
  int rank = 0, nranks = 1;
  bool fuse = false, kpost = true;   // post fusion taken; through K (else [P | AP])
  std::vector<DistLevel> levels;
};

// ghost node lists [level][rank] (global ids, sorted).  build_dist_plan reads
// the own rank's list whole and the other ranks' lists only inside the own
// node range (the send lists), so a precomputed set may hold just that.
using GhostLists = std::vector<std::vector<std::vector<int64_t>>>;

// node ranges [level][nranks+1] and replication of every level, identical on
// all ranks: replicated from the first level with <= rep_nodes nodes (or the
// coarsest) down; level 0 never
void dist_ranges(const std::vector<int64_t>& nv, const std::vector<char>& coarsest, int nranks,
                 int64_t rep_nodes, std::vector<std::vector<int64_t>>* own, std::vector<char>* rep);

// fuse: prolongation fused into the post sweep (needs A P from the setup);
// kpost: through K = P - kw W (A P) (one operator), else through [P | AP].
// pre: ghost lists computed elsewhere (ghier_download_rank: then H holds only
// the rows this rank reads, and node-major smoother slices in HostLevel::Wn);
// nullptr = computed here from the full hierarchy.
// meta_only: ranges, ghosts and send lists only (the operators are built on
// the device from the GPU hierarchy, device.hip dev_rank_ops); H then needs
// only each level's n / coarsest (and the coarsest Ainv), `pre` is required.
int build_dist_plan(const Hierarchy& H, const CsrView& A0, int rank, int nranks, int64_t rep_nodes,
                    bool fuse, DistPlan* plan, std::string* err, bool kpost = true, double kw = 1.0,
                    const GhostLists* pre = nullptr, bool meta_only = false);
// K rows = P rows - W_I (AP rows), block-column union (both sorted, same columns)
void kmerge_rows(const HBsr& P, const HBsr& AP, const std::vector<double>& W, HBsr* K);

}  // namespace mamg
