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

template __global__ void wos_first_ball_kernel<2, true>(const DevScene, const DevParams, const float*, int64_t,
                                                         int64_t, int64_t, const DevTasks, unsigned long long*,
                                                         unsigned int*, int);
template __global__ void wos_first_ball_kernel<3, true>(const DevScene, const DevParams, const float*, int64_t,
                                                         int64_t, int64_t, const DevTasks, unsigned long long*,
                                                         unsigned int*, int);
#define WOS_RB_WALK(D, G, B)                                                                                       \
  template __global__ void wos_walk_kernel<D, G, B, true>(const DevScene, const DevParams, const DevTasks, int64_t, \
                                                          int64_t, unsigned long long*, unsigned int*, int)
WOS_RB_WALK(2, false, false);
WOS_RB_WALK(2, true, false);
WOS_RB_WALK(3, false, false);
WOS_RB_WALK(3, true, false);
WOS_RB_WALK(2, false, true);  // boundary value caching (boundary-start walks)
WOS_RB_WALK(2, true, true);
#undef WOS_RB_WALK

hipError_t launch_first_balls_rb(int dim, const DevScene& sc, const DevParams& prm, const float* pts, int64_t n,
                                 int64_t base, int64_t stride, const DevTasks& tk, unsigned long long* counters,
                                 unsigned int* work, int grid, size_t shmem, int lhs_floats, hipStream_t s) {
  if (dim == 2)
    hipLaunchKernelGGL((wos_first_ball_kernel<2, true>), dim3(grid), dim3(kBlock), shmem, s, sc, prm, pts, n, base,
                       stride, tk, counters, work, lhs_floats);
  else
    hipLaunchKernelGGL((wos_first_ball_kernel<3, true>), dim3(grid), dim3(kBlock), shmem, s, sc, prm, pts, n, base,
                       stride, tk, counters, work, lhs_floats);
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

hipError_t occupancy_rb(int which, int dim, bool geom_global, size_t shmem, int* blocks) {
#define WOS_OCC(K) hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, K, kBlock, shmem)
  switch (which) {
    case 0:
      return dim == 2 ? WOS_OCC((wos_first_ball_kernel<2, true>)) : WOS_OCC((wos_first_ball_kernel<3, true>));
    case 1:
      if (dim == 2) return geom_global ? WOS_OCC((wos_walk_kernel<2, true, false, true>)) : WOS_OCC((wos_walk_kernel<2, false, false, true>));
      return geom_global ? WOS_OCC((wos_walk_kernel<3, true, false, true>)) : WOS_OCC((wos_walk_kernel<3, false, false, true>));
    default:
      return geom_global ? WOS_OCC((wos_walk_kernel<2, true, true, true>)) : WOS_OCC((wos_walk_kernel<2, false, true, true>));
  }
#undef WOS_OCC
}

}  // namespace wos
