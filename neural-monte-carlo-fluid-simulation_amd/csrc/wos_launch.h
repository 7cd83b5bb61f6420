// wos_launch.h -- host entry points of the kernels in wos_kernel.hip.
#pragma once
#include <hip/hip_runtime.h>
#include "wos_scene.h"

namespace wos {
constexpr int kBlockThreads = 256;
constexpr int kWavesPerBlockHost = 4;
constexpr int kNumCounters = 9;
// queue slots (u64) after the counters: [kNumCounters] point queue, then the walk kernel's
// task queues from slot kNumCounters + 8 on, one per 64-byte line (wos_walk_kernel)
constexpr int kTaskQueueSlot0 = kNumCounters + 8;
constexpr int kNumCounterSlots = kTaskQueueSlot0 + kMaxTaskQueues * 8;
constexpr int kMainCounterSlots = kNumCounterSlots;  // the main solve's counter buffer

// the first balls of every estimated point (after launch_point_setup)
hipError_t launch_first_balls(int dim, const DevScene& sc, const DevParams& prm, const float* pts, int64_t n,
                              int64_t base, int64_t stride, const DevTasks& tk, unsigned long long* counters,
                              unsigned int* work, int grid, size_t shmem, int lhs_floats, hipStream_t s);
// per-point setup: pstate + first-ball radius + bucket histogram, before launch_lpt_order
hipError_t launch_point_setup(int dim, const DevScene& sc, const DevParams& prm, const float* pts, int64_t n,
                              const DevTasks& tk, hipStream_t s);
// zero n64 u64 words at a and n32 u32 words at b (one launch)
hipError_t launch_zero(unsigned long long* a, int n64, uint32_t* b, int n32, hipStream_t s);
// bucket offsets + point permutation for the walk queue
hipError_t launch_lpt_order(const DevTasks& tk, int64_t n, hipStream_t s);
hipError_t launch_walks(int dim, const DevScene& sc, const DevParams& prm, const DevTasks& tk, int64_t base,
                        int64_t stride, unsigned long long* counters, unsigned int* tqueue, int grid, size_t shmem,
                        int geom_floats, hipStream_t s);
hipError_t launch_fold(int dim, const DevParams& prm, const DevTasks& tk, int64_t n, float* p, float* g,
                       int32_t* nest, int32_t* steps, hipStream_t s);
// per-wave LDS scratch of the first-ball kernel
size_t first_ball_wave_lds_bytes(int lhs_floats, int n_pairs);
int first_ball_points_per_wave(int n_pairs);
// per-wave LDS scratch of the walk kernel (after the staged geometry, 16-B aligned)
size_t walk_wave_lds_bytes(int dim);
// which: 0 first-ball kernel, 1 walk kernel (the instantiation for LDS-staged or global geometry);
// robust: the robust-float instantiations (wos_robust.hip)
hipError_t occupancy_blocks_per_cu(int which, int dim, bool geom_global, size_t shmem, int* blocks,
                                   bool robust = false);
hipError_t occupancy_walk_blocks_per_cu(int dim, bool geom_global, const DevParams& prm, size_t shmem, int* blocks);
void diag_dump(const char* tag);  // WOS_DIAG builds: print + reset the walk-kernel diagnostics
void diag_dump_bstart(const char* tag);  // ... of the boundary-start walk kernels (wos_bvc.hip)
void diag_print(const char* tag, const void* sym);
hipError_t launch_math_selftest(int which, const double* x, double* out, int64_t n, hipStream_t s);

// boundary value caching (wos_bvc.hip), 2D
hipError_t launch_bvc_point_info(const DevScene& sc, const float* pts, int64_t n, float* dd, float* nd,
                                 int32_t* inside, float* src, hipStream_t s);
hipError_t launch_bvc_start(const DevScene& sc, const DevParams& prm, const float* bpt, const float* bnrm,
                            const uint8_t* aligned, const float* bdd, int64_t nb, const DevTasks& tk, int on_neumann,
                            uint32_t tag, hipStream_t s);
hipError_t launch_bvc_fd(const DevScene& sc, const float* pts, const float* sol, int64_t n, float* dn, hipStream_t s);
hipError_t launch_walks_bstart(const DevScene& sc, const DevParams& prm, const DevTasks& tk, int64_t base,
                               int64_t stride, unsigned long long* counters, unsigned int* tqueue, int grid,
                               size_t shmem, int geom_floats, hipStream_t s);
hipError_t occupancy_walk_bstart(bool geom_global, size_t shmem, int* blocks, bool robust = false);
hipError_t launch_bvc_fold(const DevTasks& tk, int64_t nb, float* sol, int32_t* nest, hipStream_t s);
hipError_t launch_bvc_splat_list(const float* edd, const float* end_, const int32_t* ein, int64_t ne, float cutoff,
                                 float mask, int double_sided, uint32_t* list, uint32_t* count, hipStream_t s);
hipError_t launch_bvc_splat(const float* recs, int r0, int r1, int first, int last, float* state,
                            const uint32_t* list, const uint32_t* count, const float* ept, int64_t ne,
                            float absorption, float radius_clamp, float reg, float* sol, float* grad, hipStream_t s);
hipError_t launch_bvc_fill(float* recs, int64_t b0, int64_t b1, const float* bsol, const float* bdn,
                           const DevScene& sc, int ignore_neumann, hipStream_t s);
// robust float semantics (wos_robust.hip): the same launches with Gfn<DIM, true>;
// the launchers above dispatch here when prm.robust is set
hipError_t launch_first_balls_rb(int dim, const DevScene& sc, const DevParams& prm, const float* pts, int64_t n,
                                 int64_t base, int64_t stride, const DevTasks& tk, unsigned long long* counters,
                                 unsigned int* work, int grid, size_t shmem, int lhs_floats, hipStream_t s);
hipError_t launch_walks_rb(int dim, bool bstart, const DevScene& sc, const DevParams& prm, const DevTasks& tk,
                           int64_t base, int64_t stride, unsigned long long* counters, unsigned int* tqueue, int grid,
                           size_t shmem, int geom_floats, hipStream_t s);
// which: 0 first-ball, 1 walk, 2 boundary-start walk
hipError_t occupancy_rb(int which, int dim, bool geom_global, size_t shmem, int* blocks);
}  // namespace wos
