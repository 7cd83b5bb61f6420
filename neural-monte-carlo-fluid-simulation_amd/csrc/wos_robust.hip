// wos_robust.hip -- the kernel instantiations of the robust float semantics
// (wos_solver_params.robust_float, DevParams::robust): Gfn<DIM, true>, whose Yukawa
// balls with mu R > kRobustMuR use exponentially scaled Bessels instead of the
// reference's float members (which overflow to NaN for 2D mu R > ~92,
// distributions.h:585-587,695; SURVEY.md section 7.2 hard part 4).  A translation unit
// of their own: the reference-semantics kernels (wos_kernel.hip, wos_bvc.hip) are
// compiled without any of this code, and the two sets build in parallel.
#include "wos_device.h"
#include "wos_launch.h"

namespace wos {

#define WOS_RB_FB(D, G)                                                                                            \
  template __global__ void wos_first_ball_kernel<D, G, true>(const DevScene, const DevParams, const float*, int64_t, \
                                                             int64_t, int64_t, const DevTasks, unsigned long long*,  \
                                                             unsigned int*, int, int)
#define WOS_RB_WALK(D, G, B)                                                                                       \
  template __global__ void wos_walk_kernel<D, G, B, true>(const DevScene, const DevParams, const DevTasks, int64_t, \
                                                          int64_t, unsigned long long*, unsigned int*, int)
WOS_RB_FB(2, false);
WOS_RB_FB(2, true);
WOS_RB_FB(3, false);
WOS_RB_FB(3, true);
template __global__ void wos_first_ball_kernel<2, false, true, true>(const DevScene, const DevParams, const float*,
                                                                     int64_t, int64_t, int64_t, const DevTasks,
                                                                     unsigned long long*, unsigned int*, int, int);
template __global__ void wos_first_ball_kernel<3, false, true, true>(const DevScene, const DevParams, const float*,
                                                                     int64_t, int64_t, int64_t, const DevTasks,
                                                                     unsigned long long*, unsigned int*, int, int);
WOS_RB_WALK(2, false, false);
WOS_RB_WALK(2, true, false);
WOS_RB_WALK(3, false, false);
WOS_RB_WALK(3, true, false);
WOS_RB_WALK(2, false, true);  // boundary value caching (boundary-start walks)
WOS_RB_WALK(2, true, true);
// two-phase walks
#define WOS_RB_TWO_PHASE(D, G)                                                                                    \
  template __global__ void wos_walk_first_kernel<D, G, true>(const DevScene, const DevParams, const DevTasks,      \
                                                             int64_t, int64_t, unsigned long long*, int);         \
  template __global__ void wos_walk_kernel<D, G, false, true, true>(const DevScene, const DevParams, const DevTasks, \
                                                                    int64_t, int64_t, unsigned long long*,        \
                                                                    unsigned int*, int)
WOS_RB_TWO_PHASE(2, false);
WOS_RB_TWO_PHASE(2, true);
WOS_RB_TWO_PHASE(3, false);
WOS_RB_TWO_PHASE(3, true);
#undef WOS_RB_TWO_PHASE
#undef WOS_RB_FB
#undef WOS_RB_WALK

hipError_t launch_first_balls_rb(int dim, const DevScene& sc, const DevParams& prm, const float* pts, int64_t n,
                                 int64_t base, int64_t stride, const DevTasks& tk, unsigned long long* counters,
                                 unsigned int* work, int grid, size_t shmem, int geom_floats, int lhs_floats,
                                 bool pre, hipStream_t s) {
  if (pre) {
    if (dim == 2)
      hipLaunchKernelGGL((wos_first_ball_kernel<2, false, true, true>), dim3(grid), dim3(kBlock), shmem, s, sc, prm,
                         pts, n, base, stride, tk, counters, work, 0, lhs_floats);
    else
      hipLaunchKernelGGL((wos_first_ball_kernel<3, false, true, true>), dim3(grid), dim3(kBlock), shmem, s, sc, prm,
                         pts, n, base, stride, tk, counters, work, 0, lhs_floats);
    return hipGetLastError();
  }
#define WOS_LAUNCH_FB(D, G)                                                                                       \
  hipLaunchKernelGGL((wos_first_ball_kernel<D, G, true>), dim3(grid), dim3(kBlock), shmem, s, sc, prm, pts, n, base, \
                     stride, tk, counters, work, geom_floats, lhs_floats)
  if (dim == 2) {
    if (sc.geom_global) WOS_LAUNCH_FB(2, true); else WOS_LAUNCH_FB(2, false);
  } else {
    if (sc.geom_global) WOS_LAUNCH_FB(3, true); else WOS_LAUNCH_FB(3, false);
  }
#undef WOS_LAUNCH_FB
  return hipGetLastError();
}

hipError_t launch_walks_rb(int dim, bool bstart, const DevScene& sc, const DevParams& prm, const DevTasks& tk,
                           int64_t base, int64_t stride, unsigned long long* counters, unsigned int* tqueue, int grid,
                           size_t shmem, int geom_floats, hipStream_t s) {
#define WOS_LAUNCH_WALK(D, G, B)                                                                                  \
  hipLaunchKernelGGL((wos_walk_kernel<D, G, B, true>), dim3(grid), dim3(kBlock), shmem, s, sc, prm, tk, base, stride, \
                     counters, tqueue, geom_floats)
  if (bstart) {
    if (dim != 2) return hipErrorInvalidValue;
    if (sc.geom_global) WOS_LAUNCH_WALK(2, true, true); else WOS_LAUNCH_WALK(2, false, true);
  } else if (dim == 2) {
    if (sc.geom_global) WOS_LAUNCH_WALK(2, true, false); else WOS_LAUNCH_WALK(2, false, false);
  } else {
    if (sc.geom_global) WOS_LAUNCH_WALK(3, true, false); else WOS_LAUNCH_WALK(3, false, false);
  }
#undef WOS_LAUNCH_WALK
  return hipGetLastError();
}

hipError_t launch_walks_two_phase_rb(int dim, const DevScene& sc, const DevParams& prm, const DevTasks& tk,
                                     int64_t base, int64_t stride, unsigned long long* counters, unsigned int* tqueue,
                                     int grid, size_t shmem, int geom_floats, hipStream_t s) {
  hipError_t e = hipMemsetAsync(tk.shist, 0, (2 * kCostBuckets + 1) * sizeof(uint32_t), s);
  if (e != hipSuccess) return e;
#define WOS_LAUNCH_FIRST(D, G)                                                                                 \
  hipLaunchKernelGGL((wos_walk_first_kernel<D, G, true>), dim3(grid), dim3(kBlock), shmem, s, sc, prm, tk, base, \
                     stride, counters, geom_floats)
#define WOS_LAUNCH_RESUME(D, G)                                                                                \
  hipLaunchKernelGGL((wos_walk_kernel<D, G, false, true, true>), dim3(grid), dim3(kBlock), shmem, s, sc, prm, tk, \
                     base, stride, counters, tqueue, geom_floats)
  if (dim == 2) {
    if (sc.geom_global) WOS_LAUNCH_FIRST(2, true); else WOS_LAUNCH_FIRST(2, false);
  } else {
    if (sc.geom_global) WOS_LAUNCH_FIRST(3, true); else WOS_LAUNCH_FIRST(3, false);
  }
  hipLaunchKernelGGL(wos_surv_offsets_kernel<0>, dim3(1), dim3(64), 0, s, tk.shist);
  const int sgrid = (int)((tk.T + 255) / 256);
  if (sgrid > 0) hipLaunchKernelGGL(wos_surv_scatter_kernel<0>, dim3(sgrid), dim3(256), 0, s, tk);
  if (dim == 2) {
    if (sc.geom_global) WOS_LAUNCH_RESUME(2, true); else WOS_LAUNCH_RESUME(2, false);
  } else {
    if (sc.geom_global) WOS_LAUNCH_RESUME(3, true); else WOS_LAUNCH_RESUME(3, false);
  }
#undef WOS_LAUNCH_FIRST
#undef WOS_LAUNCH_RESUME
  return hipGetLastError();
}

hipError_t occupancy_rb(int which, int dim, bool geom_global, size_t shmem, int* blocks) {
#define WOS_OCC(K) hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, K, kBlock, shmem)
  switch (which) {
    case 0:
      if (dim == 2) return geom_global ? WOS_OCC((wos_first_ball_kernel<2, true, true>)) : WOS_OCC((wos_first_ball_kernel<2, false, true>));
      return geom_global ? WOS_OCC((wos_first_ball_kernel<3, true, true>)) : WOS_OCC((wos_first_ball_kernel<3, false, true>));
    case 1:
      if (dim == 2) return geom_global ? WOS_OCC((wos_walk_kernel<2, true, false, true>)) : WOS_OCC((wos_walk_kernel<2, false, false, true>));
      return geom_global ? WOS_OCC((wos_walk_kernel<3, true, false, true>)) : WOS_OCC((wos_walk_kernel<3, false, false, true>));
    case 3:
      return dim == 2 ? WOS_OCC((wos_first_ball_kernel<2, false, true, true>)) : WOS_OCC((wos_first_ball_kernel<3, false, true, true>));
    default:
      return geom_global ? WOS_OCC((wos_walk_kernel<2, true, true, true>)) : WOS_OCC((wos_walk_kernel<2, false, true, true>));
  }
#undef WOS_OCC
}

}  // namespace wos
