// device.h -- device hierarchy interface (no HIP types; implemented in device.hip)
#pragma once
#include <mutex>
#include <string>

#include "gsetup.h"
#include "host.h"

namespace mamg {

struct DeviceHandle;

int dev_upload(const Hierarchy& H, const CsrView& A0, const mamg_params& p, DeviceHandle** out,
               std::string* err);
// apply handle from a GPU-setup hierarchy (everything stays in HBM); G's
// buffers are released level by level as the apply layouts are built
void dev_prereserve(int device, int64_t nnz, int nranks);
void dev_prereserve_release();
int dev_from_ghier(GHier* G, const DevMat& A0, const mamg_params& p, DeviceHandle** out,
                   std::string* err);
// setup phase timings of a handle built by the GPU setup (ms; zeros otherwise)
void dev_setup_ms(const DeviceHandle* h, double* ms8);
// apply-layout phases (ms): build, K value region trials, operator re-homing, finish
void dev_layout_ms(const DeviceHandle* h, double* ms4);
void dev_destroy(DeviceHandle* h);
// release the cached blocks of the setup temporaries (dmem.h tmp_trim_all)
void dev_tmp_trim();
// held across the library's stream captures and its setups (device.hip)
std::recursive_mutex& capture_mutex();
// the end of a setup: idle cached blocks above the cache limit freed
void dev_tmp_trim_to_limit();
// cache limit (bytes per device; < 0 default = HBM / 8, 0 = release every setup)
void dev_set_cache_limit(int64_t bytes);
int64_t dev_cache_limit(int device);
// idle cached bytes of a device (idle temporaries + the SpGEMM staging block)
int64_t dev_cache_idle_bytes(int device);
int64_t dev_nrows(const DeviceHandle* h);
int dev_num_levels(const DeviceHandle* h);
int dev_layout(const DeviceHandle* h);
int dev_level_format(const DeviceHandle* h, int level);
mamg_params dev_params(const DeviceHandle* h);
void dev_kregion(const DeviceHandle* h, std::vector<double>* ms, int* kept);
double dev_apply_bytes(const DeviceHandle* h);
int dev_apply(DeviceHandle* h, const double* d_r, double* d_z, void* stream, std::string* err);
int dev_apply_host(DeviceHandle* h, const double* r, double* z, std::string* err);
int dev_spmv(DeviceHandle* h, const double* d_x, double* d_y, void* stream, std::string* err);
int dev_pcg(DeviceHandle* h, const double* d_b, double* d_x, double tol, int maxiter,
            int relativeconv, double* residuals, double* alphas, double* betas,
            int* niters, void* stream, std::string* err);
int dev_time_apply(DeviceHandle* h, const double* d_r, double* d_z, int reps, int mode,
                   double* ms, double* kernel_ms, double* class_bytes, void* stream,
                   std::string* err);

// multi-GPU (device.hip, second half)
struct DistHandle;
int dist_get_unique_id(void* id, std::string* err);
// ghosts: precomputed ghost lists (ghier_download_rank), else nullptr; G / A0d:
// build the rank-local operators on the device from this GPU hierarchy (H then
// holds only level sizes and the coarsest inverse)
// the multi-GPU path's parameter limits (maxit 1, no SCHWARZ_PATCHES /
// SCHWARZ_RINGS), checked before a rank touches its GPU
int dist_check(const mamg_params& p, std::string* err);
int dist_upload(const Hierarchy& H, const CsrView& A0, const mamg_params& p, int rank, int nranks,
                const void* comm_id, int64_t rep_nodes, DistHandle** out, std::string* err,
                const std::vector<std::vector<std::vector<int64_t>>>* ghosts = nullptr,
                const GHier* G = nullptr, const DevMat* A0d = nullptr);
void dist_destroy(DistHandle* h);
void dist_range(const DistHandle* h, int64_t* o0, int64_t* o1, int64_t* nv);
double dist_apply_bytes(const DistHandle* h);
void dist_apply_launches(const DistHandle* h, int64_t c[5]);
int dist_apply(DistHandle* h, const double* d_r, double* d_z, void* stream, std::string* err);
int dist_spmv(DistHandle* h, const double* d_x, double* d_y, void* stream, std::string* err);
int dist_virtual_spmv(const std::vector<DistHandle*>& hs, const std::vector<const double*>& x,
                      const std::vector<double*>& y, void* stream, std::string* err);
int dist_time_apply(DistHandle* h, const double* d_r, double* d_z, int reps, int mode, double* ms,
                    double* kernel_ms, double* class_bytes, void* stream, std::string* err);
int dist_set_exchange(DistHandle* h, const mamg_exchange& ex, std::string* err);
int dist_virtual_apply(const std::vector<DistHandle*>& hs, const std::vector<const double*>& r,
                       const std::vector<double*>& z, void* stream, std::string* err);
// the apply replayed from a hipGraph captured on first use per (r, z) (RCCL
// calls inside the capture); MAMG_ERR_UNSUPPORTED for host-staged / virtual
// exchanges or after a failed capture (then the eager dist_apply)
int dist_apply_graph(DistHandle* h, const double* d_r, double* d_z, void* stream, std::string* err);
// capture (or find) the graph of (r, z) without launching it
int dist_graph_prepare(DistHandle* h, const double* d_r, double* d_z, std::string* err);
int dist_virtual_apply_graph(const std::vector<DistHandle*>& hs, const std::vector<const double*>& r,
                             const std::vector<double*>& z, void* stream, std::string* err);

}  // namespace mamg
