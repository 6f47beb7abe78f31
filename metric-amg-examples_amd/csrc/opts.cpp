// opts.cpp -- process-wide switch table (opts.h).
#include "opts.h"

#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>

#ifndef MAMG_DIAG
#define MAMG_DIAG 0
#endif

namespace mamg {
namespace {

// every switch of the product library, with the default it stands for
// (DESIGN.md section 4 gives the measurements behind each default)
constexpr const char* kNames[] = {
    "MAMG_POST_K",                // 1: K = P - W A P after the coarse correction; 0: [P | AP]; 2: split K
    "MAMG_SELL_MIN_ROWS",         // rows from which level 0's operators take SELL-64 (1 << 20)
    "MAMG_MSELL_MIN_ROWS",        // rows from which coarse levels take multi-lane SELL-64 (never)
    "MAMG_TAIL_NODES",            // coarse tail: first level with at most this many nodes (auto)
    "MAMG_TAIL_VL",               // coarse tail: lanes per row cap (4)
    "MAMG_TAIL_LDS",              // coarse tail: LDS program size (auto)
    "MAMG_TAIL_PROG_LDS",         // 1: coarse tail's op descriptors copied into LDS; 0: scalar loads (default)
    "MAMG_TAIL_RES",              // 1: coarse tail's operators held in registers, one row per thread
    "MAMG_HALF",                  // 1: half-symmetric level-0 A; 0: SELL-64
    "MAMG_HALF_BANDS",            // 1: plane-band schedule of the half-symmetric kernel
    "MAMG_R_BANDS",               // 1: plane-band schedule of the level-0 restriction
    "MAMG_K_SORT",                // 1: K rows sorted by length inside SELL slices
    "MAMG_K_COL16",               // 1: level-0 K's columns as 16-bit offsets from a per-slice base
    "MAMG_FUSE_RBD",              // which restrictions write the next first sweep (2)
    "MAMG_CSR2BSR_FILL",          // 1: column-only LDS fill of CSR -> BSR2; 0: staged merge
    "MAMG_KREGION_TRIES",         // K value regions timed at upload
    "MAMG_KREGION_BUDGET_MS",     // time budget of that search
    "MAMG_REHOME",                // 1: operators re-homed after the setup
    "MAMG_PRERESERVE_B_PER_NNZ",  // layout reservation, bytes per A0 entry (20)
    "MAMG_POISON",                // 1: new double arrays start as NaN bytes (tests)
    "MAMG_OVERLAP",               // multi-GPU: interior rows during the halo (1)
    "MAMG_DIST_TEST",             // multi-GPU virtual ranks: "dry" skips exchanges (timing)
    "MAMG_SPGEMM_PAIR",           // 1: staged count pass over node row pairs
    "MAMG_SPGEMM_STAGE_GB",       // staging block cap (16; 0: unstaged products)
    "MAMG_SPGEMM_STAGE_STRIDE",   // staging stride cap (128)
    "MAMG_MIS_STAGED",            // 1: MIS-2 maxima over staged rows
    "MAMG_UPLOAD_THREADS",        // host threads copying A0 (2)
    "MAMG_PATCH_INV",             // node-patch inverses: 1 one patch per wave (round 5), 2 two per wave, 3 matrix cores (default)
};

struct Table {
  std::mutex m;
  std::map<std::string, size_t> set;   // name -> index into vals
  std::deque<std::string> vals;        // never shrinks: returned pointers stay valid
  std::string names;
};
Table& table() {
  static Table t;
  return t;
}
bool known(const char* name) {
  for (const char* k : kNames)
    if (std::strcmp(k, name) == 0) return true;
  return false;
}

}  // namespace

const char* opt(const char* name) {
  Table& t = table();
  {
    std::lock_guard<std::mutex> g(t.m);
    auto it = t.set.find(name);
    if (it != t.set.end()) return t.vals[it->second].c_str();
  }
#if MAMG_DIAG
  return std::getenv(name);
#else
  return nullptr;
#endif
}

bool set_opt(const char* name, const char* value) {
  if (!name || !known(name)) return false;
  Table& t = table();
  std::lock_guard<std::mutex> g(t.m);
  if (!value) {
    t.set.erase(name);
    return true;
  }
  t.vals.emplace_back(value);
  t.set[name] = t.vals.size() - 1;
  return true;
}

const char* opt_names() {
  Table& t = table();
  std::lock_guard<std::mutex> g(t.m);
  if (t.names.empty())
    for (const char* k : kNames) {
      if (!t.names.empty()) t.names += ',';
      t.names += k;
    }
  return t.names.c_str();
}

}  // namespace mamg
