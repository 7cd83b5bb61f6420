// wos_kernel.hip -- gfx950 walk-on-stars solve: the kernel instantiations and their
// host launchers (device code in wos_device.h).
//
// One projection = wos_point_setup_kernel, the walk-queue order (wos_lpt_scatter_kernel),
// wos_first_ball_kernel, the persistent wos_walk_kernel and wos_fold_kernel (statistics
// + masked outputs), all on the caller's stream.
#include "wos_device.h"
#include <algorithm>
#include "wos_launch.h"

namespace wos {

// ---- walk-queue order: the permutation, buckets in descending cost order ----
// One launch: every block derives the bucket offsets from the final counts
// hist[0, kCostBuckets) itself (exclusive sums in descending bucket order), counts its
// points per bucket in LDS, reserves one range per bucket with an atomic on the fill
// cursors hist[kCostBuckets + b] (zeroed with the counts), then places its points.
// Order inside a bucket is immaterial: results do not depend on it.
__global__ __launch_bounds__(256) void wos_lpt_scatter_kernel(const DevTasks tk, int64_t n) {
  __shared__ uint32_t cnt[kCostBuckets], base[kCostBuckets], off[kCostBuckets];
  if (threadIdx.x < kCostBuckets) {
    cnt[threadIdx.x] = 0u;
    // offset of bucket b = points in buckets above b
    uint32_t acc = 0;
    for (int b = kCostBuckets - 1; b > (int)threadIdx.x; b--) acc += tk.hist[b];
    off[threadIdx.x] = acc;
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int b = 0;
  uint32_t local = 0;
  if (i < n) {
    b = (tk.pstate[i] >> 8) & (kCostBuckets - 1);
    local = atomicAdd(&cnt[b], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kCostBuckets && cnt[threadIdx.x])
    base[threadIdx.x] = off[threadIdx.x] + atomicAdd(&tk.hist[kCostBuckets + threadIdx.x], cnt[threadIdx.x]);
  __syncthreads();
  if (i < n) tk.perm[base[b] + local] = (uint32_t)i;
}

template __global__ void wos_first_ball_kernel<2>(const DevScene, const DevParams, const float*, int64_t, int64_t,
                                                   int64_t, const DevTasks, unsigned long long*, unsigned int*, int);
template __global__ void wos_first_ball_kernel<3>(const DevScene, const DevParams, const float*, int64_t, int64_t,
                                                   int64_t, const DevTasks, unsigned long long*, unsigned int*, int);
template __global__ void wos_point_setup_kernel<2>(const DevScene, const DevParams, const float*, int64_t,
                                                   const DevTasks);
template __global__ void wos_point_setup_kernel<3>(const DevScene, const DevParams, const float*, int64_t,
                                                   const DevTasks);
// walk kernels: <DIM, GG> with the Neumann term, and the Neumann-inert <DIM, GG, false, false, false>
#define WOS_WALK(D, G)                                                                                            \
  template __global__ void wos_walk_kernel<D, G>(const DevScene, const DevParams, const DevTasks, int64_t, int64_t, \
                                                 unsigned long long*, unsigned int*, int);                        \
  template __global__ void wos_walk_kernel<D, G, false, false, false>(const DevScene, const DevParams,            \
                                                                      const DevTasks, int64_t, int64_t,           \
                                                                      unsigned long long*, unsigned int*, int)
WOS_WALK(2, false);
WOS_WALK(2, true);
// 2D, LDS geometry, the tail-spreading instantiations (DevParams::tail_spread)
template __global__ void wos_walk_kernel<2, false, false, false, true, true>(const DevScene, const DevParams,
                                                                            const DevTasks, int64_t, int64_t,
                                                                            unsigned long long*, unsigned int*, int);
template __global__ void wos_walk_kernel<2, false, false, false, false, true>(const DevScene, const DevParams,
                                                                             const DevTasks, int64_t, int64_t,
                                                                             unsigned long long*, unsigned int*, int);
WOS_WALK(3, false);
WOS_WALK(3, true);
#undef WOS_WALK
template __global__ void wos_fold_kernel<2>(const DevParams, const DevTasks, int64_t, float*, float*, int32_t*,
                                            int32_t*);
template __global__ void wos_fold_kernel<3>(const DevParams, const DevTasks, int64_t, float*, float*, int32_t*,
                                            int32_t*);
template __global__ void wos_fold4_kernel<3>(const DevParams, const DevTasks, int64_t, float*, float*, int32_t*,
                                             int32_t*);
template __global__ void wos_fold4_kernel<2>(const DevParams, const DevTasks, int64_t, float*, float*, int32_t*,
                                             int32_t*);

// math self-test kernel (parity of the deterministic math with the CPU oracle)
__global__ void wos_math_selftest_kernel(int which, const double* x, double* out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double v = x[i], r = 0.0;
  switch (which) {
    case 0: r = dexp(v); break;
    case 1: r = dlog(v); break;
    case 2: { double s, c; dsincos(v, &s, &c); r = s; } break;
    case 3: { double s, c; dsincos(v, &s, &c); r = c; } break;
    case 4: r = datan(v); break;
    case 5: r = __builtin_sqrt(v); break;
    case 6: r = bessi0(v); break;
    case 7: r = bessi1(v); break;
    case 8: r = bessk0(v); break;
    case 9: r = bessk1(v); break;
    case 10: r = (double)fexp((float)v); break;
    case 11: r = (double)flog((float)v); break;
    case 12: r = (double)fsin((float)v); break;
    case 13: r = (double)fcos((float)v); break;
    case 14: r = (double)fcbrt((float)v); break;
    case 15: r = (double)__builtin_sqrtf((float)v); break;
    case 16: r = (double)i0_fast((float)v); break;
    case 17: r = (double)k0_fast((float)v); break;
    // the fused evaluator of the kernels (bessel_ik) must equal 6..9
    case 18: { double a, b; bessel_ik<true, false>(v, &r, &a, nullptr, nullptr); (void)b; } break;
    case 19: { double a; bessel_ik<false, true>(v, nullptr, nullptr, &r, &a); } break;
    case 20: { double a; bessel_ik<true, false>(v, &a, &r, nullptr, nullptr); } break;
    case 21: { double a; bessel_ik<false, true>(v, nullptr, nullptr, &a, &r); } break;
    case 22: { double a, b, c; bessel_ik<true, true>(v, &a, &r, &b, &c); } break;
    case 23: { double a, b, c; bessel_ik<true, true>(v, &a, &b, &c, &r); } break;
    // the fused float pair of the rejection fast path (k0i0_fast): 24 I0, 25 K0
    case 24: { float k, i; k0i0_fast((float)v, &k, &i); r = (double)i; } break;
    case 25: { float k, i; k0i0_fast((float)v, &k, &i); r = (double)k; } break;
    default: r = __builtin_nan("");
  }
  out[i] = r;
}


// ---------------------------------------------------------------------------
// host-side launchers (called from wos_capi.hip)
// ---------------------------------------------------------------------------
hipError_t launch_first_balls(int dim, const DevScene& sc, const DevParams& prm, const float* pts, int64_t n,
                              int64_t base, int64_t stride, const DevTasks& tk, unsigned long long* counters,
                              unsigned int* work, int grid, size_t shmem, int lhs_floats, hipStream_t s) {
  if (prm.robust)
    return launch_first_balls_rb(dim, sc, prm, pts, n, base, stride, tk, counters, work, grid, shmem, lhs_floats, s);
  if (dim == 2)
    hipLaunchKernelGGL(wos_first_ball_kernel<2>, dim3(grid), dim3(kBlock), shmem, s, sc, prm, pts, n, base, stride, tk,
                       counters, work, lhs_floats);
  else
    hipLaunchKernelGGL(wos_first_ball_kernel<3>, dim3(grid), dim3(kBlock), shmem, s, sc, prm, pts, n, base, stride, tk,
                       counters, work, lhs_floats);
  return hipGetLastError();
}

hipError_t launch_point_setup(int dim, const DevScene& sc, const DevParams& prm, const float* pts, int64_t n,
                              const DevTasks& tk, hipStream_t s) {
  const int grid = (int)((n * kSetupLanes + 255) / 256);
  if (grid < 1) return hipSuccess;
  if (dim == 2) hipLaunchKernelGGL(wos_point_setup_kernel<2>, dim3(grid), dim3(256), 0, s, sc, prm, pts, n, tk);
  else hipLaunchKernelGGL(wos_point_setup_kernel<3>, dim3(grid), dim3(256), 0, s, sc, prm, pts, n, tk);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void wos_zero_kernel(unsigned long long* a, int n64, uint32_t* b, int n32) {
  const int i0 = blockIdx.x * blockDim.x + threadIdx.x, di = gridDim.x * blockDim.x;
  for (int i = i0; i < n64; i += di) a[i] = 0ull;
  for (int i = i0; i < n32; i += di) b[i] = 0u;
}

hipError_t launch_zero(unsigned long long* a, int n64, uint32_t* b, int n32, hipStream_t s) {
  // one block per 1024 u64 (the grid-wide spreading control words can be ~10^4)
  const int grid = std::max(1, std::min(32, (std::max(n64, n32 / 2) + 1023) / 1024));
  hipLaunchKernelGGL(wos_zero_kernel, dim3(grid), dim3(256), 0, s, a, n64, b, n32);
  return hipGetLastError();
}

hipError_t launch_lpt_order(const DevTasks& tk, int64_t n, hipStream_t s) {
  const int grid = (int)((n + 255) / 256);
  if (grid > 0) hipLaunchKernelGGL(wos_lpt_scatter_kernel, dim3(grid), dim3(256), 0, s, tk, n);
  return hipGetLastError();
}

hipError_t launch_walks(int dim, const DevScene& sc, const DevParams& prm, const DevTasks& tk, int64_t base,
                        int64_t stride, unsigned long long* counters, unsigned int* tqueue, int grid, size_t shmem,
                        int geom_floats, hipStream_t s) {
  if (prm.robust)
    return launch_walks_rb(dim, false, sc, prm, tk, base, stride, counters, tqueue, grid, shmem, geom_floats, s);
#define WOS_LAUNCH_WALK(D, G)                                                                                    \
  do {                                                                                                           \
    if (prm.neumann_inert)                                                                                       \
      hipLaunchKernelGGL((wos_walk_kernel<D, G, false, false, false>), dim3(grid), dim3(kBlock), shmem, s, sc, \
                         prm, tk, base, stride, counters, tqueue, geom_floats);                                  \
    else                                                                                                         \
      hipLaunchKernelGGL((wos_walk_kernel<D, G>), dim3(grid), dim3(kBlock), shmem, s, sc, prm, tk, base, stride,  \
                         counters, tqueue, geom_floats);                                                         \
  } while (0)
  if (dim == 2) {
    if (sc.geom_global) {
      WOS_LAUNCH_WALK(2, true);
    } else if (prm.tail_spread) {
      if (prm.neumann_inert)
        hipLaunchKernelGGL((wos_walk_kernel<2, false, false, false, false, true>), dim3(grid), dim3(kBlock), shmem, s,
                           sc, prm, tk, base, stride, counters, tqueue, geom_floats);
      else
        hipLaunchKernelGGL((wos_walk_kernel<2, false, false, false, true, true>), dim3(grid), dim3(kBlock), shmem, s,
                           sc, prm, tk, base, stride, counters, tqueue, geom_floats);
    } else {
      WOS_LAUNCH_WALK(2, false);
    }
  } else {
    if (sc.geom_global) WOS_LAUNCH_WALK(3, true); else WOS_LAUNCH_WALK(3, false);
  }
#undef WOS_LAUNCH_WALK
  return hipGetLastError();
}

hipError_t launch_fold(int dim, const DevParams& prm, const DevTasks& tk, int64_t n, float* p, float* g,
                       int32_t* nest, int32_t* steps, hipStream_t s) {
  // the quad fold (pipelined staging), both dimensions: profiles/r5zm_ab_fold_pipe.log, r5zn_ab_fold4_2d.log
  if (tk.deriv == nullptr) {
    const int g4 = (int)((n + kFold4Points - 1) / kFold4Points);
    if (g4 < 1) return hipSuccess;
    if (dim == 3)
      hipLaunchKernelGGL(wos_fold4_kernel<3>, dim3(g4), dim3(4 * kFold4Points), 0, s, prm, tk, n, p, g, nest, steps);
    else
      hipLaunchKernelGGL(wos_fold4_kernel<2>, dim3(g4), dim3(4 * kFold4Points), 0, s, prm, tk, n, p, g, nest, steps);
    return hipGetLastError();
  }
  const int grid = (int)((n + kFoldPoints - 1) / kFoldPoints);
  if (grid < 1) return hipSuccess;
  if (dim == 2)
    hipLaunchKernelGGL(wos_fold_kernel<2>, dim3(grid), dim3(kFoldPoints), 0, s, prm, tk, n, p, g, nest, steps);
  else
    hipLaunchKernelGGL(wos_fold_kernel<3>, dim3(grid), dim3(kFoldPoints), 0, s, prm, tk, n, p, g, nest, steps);
  return hipGetLastError();
}

// P points' stratified samples and partners (fb_points_per_wave), then the sampler / shuffle scratch
size_t first_ball_wave_lds_bytes(int lhs_floats, int n_pairs) {
  const int P = fb_points_per_wave(n_pairs);
  return (size_t)2 * P * lhs_floats * sizeof(float) + fb_union_bytes(P * lhs_floats, 2 * n_pairs);
}

int first_ball_points_per_wave(int n_pairs) { return fb_points_per_wave(n_pairs); }

size_t walk_wave_lds_bytes(int dim) { return dim == 2 ? walk_scratch_bytes<2>() : walk_scratch_bytes<3>(); }

hipError_t occupancy_blocks_per_cu(int which, int dim, bool geom_global, size_t shmem, int* blocks, bool robust) {
  if (robust) return occupancy_rb(which, dim, geom_global, shmem, blocks);
  if (which == 0)
    return dim == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wos_first_ball_kernel<2>, kBlock, shmem)
                    : hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wos_first_ball_kernel<3>, kBlock, shmem);
  if (dim == 2)
    return geom_global ? hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wos_walk_kernel<2, true>, kBlock, shmem)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wos_walk_kernel<2, false>, kBlock, shmem);
  return geom_global ? hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wos_walk_kernel<3, true>, kBlock, shmem)
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wos_walk_kernel<3, false>, kBlock, shmem);
}

// residency of the walk instantiation launch_walks dispatches for these parameters (the
// tail-spreading and Neumann-inert kernels differ in static LDS and registers)
hipError_t occupancy_walk_blocks_per_cu(int dim, bool geom_global, const DevParams& prm, size_t shmem, int* blocks) {
  if (prm.robust) return occupancy_rb(1, dim, geom_global, shmem, blocks);
#define WOS_OCC(K) hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, K, kBlock, shmem)
  const bool inert = prm.neumann_inert != 0;
  if (dim == 2) {
    if (geom_global) return inert ? WOS_OCC((wos_walk_kernel<2, true, false, false, false>)) : WOS_OCC((wos_walk_kernel<2, true>));
    if (prm.tail_spread)
      return inert ? WOS_OCC((wos_walk_kernel<2, false, false, false, false, true>))
                   : WOS_OCC((wos_walk_kernel<2, false, false, false, true, true>));
    return inert ? WOS_OCC((wos_walk_kernel<2, false, false, false, false>)) : WOS_OCC((wos_walk_kernel<2, false>));
  }
  if (geom_global) return inert ? WOS_OCC((wos_walk_kernel<3, true, false, false, false>)) : WOS_OCC((wos_walk_kernel<3, true>));
  return inert ? WOS_OCC((wos_walk_kernel<3, false, false, false, false>)) : WOS_OCC((wos_walk_kernel<3, false>));
#undef WOS_OCC
}

void diag_dump(const char* tag) {
  diag_print(tag, HIP_SYMBOL(g_diag));
#if WOS_TIMELINE
  // the walk kernel's live lanes over time (bins of 2^kTlShift ticks of the 100 MHz clock)
  static unsigned long long tl[1 + TL_NUM * kTlBins];
  hipMemcpyFromSymbol(tl, HIP_SYMBOL(g_tl), sizeof(tl));
  const double bt = (double)(1u << kTlShift);
  int last = 0;
  for (int b = 0; b < kTlBins; b++)
    if (tl[1 + TL_WAVE * kTlBins + b]) last = b;
  fprintf(stderr, "[timeline %s] bin_us %.2f (bin: busy waves, live lanes, lanes/busy wave, tasks handed out, walks finished)\n",
          tag, bt / 100.0);
  for (int b = 0; b <= last; b++) {
    const double w = tl[1 + TL_WAVE * kTlBins + b] / bt, l = tl[1 + TL_LANE * kTlBins + b] / bt;
    fprintf(stderr, "[timeline %s] %3d %8.1f %9.1f %6.2f %9llu %9llu\n", tag, b, w, l, w > 0 ? l / w : 0.0,
            tl[1 + TL_START * kTlBins + b], tl[1 + TL_FIN * kTlBins + b]);
  }
  static unsigned long long z[1 + TL_NUM * kTlBins];
  hipMemcpyToSymbol(HIP_SYMBOL(g_tl), z, sizeof(z));
#endif
}

// g_diag is per translation unit: `sym` is the calling unit's copy
void diag_print(const char* tag, const void* sym) {
#if WOS_DIAG
  unsigned long long d[D_NUM];
  hipMemcpyFromSymbol(d, sym, sizeof(d));
  fprintf(stderr, "[diag %s] iters %llu lanes/iter %.2f  cycles/iter: step %.0f star %.0f ray %.0f sample %.0f loop %.0f  ray_overflow %llu\n",
          tag, d[D_ITERS], (double)d[D_LANES] / (double)(d[D_ITERS] ? d[D_ITERS] : 1),
          (double)d[D_STEP] / d[D_ITERS], (double)d[D_STAR] / d[D_ITERS], (double)d[D_RAY] / d[D_ITERS],
          (double)d[D_SAMPLE] / d[D_ITERS], (double)d[D_LOOP] / d[D_ITERS], d[D_RAYOVF]);
  const double fp = (double)(d[D_FB_PTS] ? d[D_FB_PTS] : 1);
  fprintf(stderr, "[diag %s] first-ball: points %llu cycles/point: setup %.0f lhs %.0f balls %.0f total %.0f\n", tag,
          d[D_FB_PTS], d[D_FB_SETUP] / fp, d[D_FB_LHS] / fp, d[D_FB_BALLS] / fp, d[D_FB_TOTAL] / fp);
  fprintf(stderr, "[diag %s] first-ball parts cycles/point: ball update %.0f  sample (member a) %.0f  member a %.0f  member b %.0f  stores %.0f\n",
          tag, d[D_FB_UPD] / fp, d[D_FB_SMP] / fp, d[D_FB_MA] / fp, d[D_FB_MB] / fp, d[D_FB_ST] / fp);
  fprintf(stderr, "[diag %s] first-ball source samples: rejection iterations per point: sum over lanes %.1f, max over lanes %.1f\n",
          tag, d[D_FB_ITSUM] / fp, d[D_FB_ITMAX] / fp);
  fprintf(stderr, "[diag %s] step parts cycles/iter: mid (ball update) %.0f  end %.0f  tail %.0f\n", tag,
          (double)d[D_MID] / (d[D_ITERS] ? d[D_ITERS] : 1), (double)d[D_END] / (d[D_ITERS] ? d[D_ITERS] : 1),
          (double)d[D_TAIL] / (d[D_ITERS] ? d[D_ITERS] : 1));
  fprintf(stderr, "[diag %s] rejection: calls %llu, lanes/call %.1f, generations/call %.2f, items/call %.1f, quick-rejected %.1f%%, undecided %.3f%%\n",
          tag, d[D_RCALLS], (double)d[D_RLANES] / (d[D_RCALLS] ? d[D_RCALLS] : 1), (double)d[D_RGENS] / (d[D_RCALLS] ? d[D_RCALLS] : 1),
          (double)d[D_RITEMS] / (d[D_RCALLS] ? d[D_RCALLS] : 1), 100.0 * d[D_RQUICK] / (d[D_RITEMS] ? d[D_RITEMS] : 1),
          100.0 * d[D_RUND] / (d[D_RITEMS] ? d[D_RITEMS] : 1));
  fprintf(stderr, "[diag %s] max cycles/point (first balls) %llu, longest walk %llu steps, longest walk-kernel wave %llu cycles\n",
          tag, d[D_FB_MAX], d[D_WMAXLEN], d[D_WAVEMAX]);
  fprintf(stderr, "[diag %s] star calls %llu: groups visited/call %.2f, candidates/call %.2f, exact/call %.2f\n", tag,
          d[D_SCALLS], (double)d[D_SGVISIT] / d[D_SCALLS], (double)d[D_SCAND] / d[D_SCALLS],
          (double)d[D_SEXACT] / d[D_SCALLS]);
  fprintf(stderr, "[diag %s] after the queue ran dry: %llu iterations (%.1f%%), lanes/iter %.2f, %.1f%% of loop cycles\n",
          tag, d[D_XITERS], 100.0 * d[D_XITERS] / (d[D_ITERS] ? d[D_ITERS] : 1),
          (double)d[D_XLANES] / (d[D_XITERS] ? d[D_XITERS] : 1), 100.0 * d[D_XLOOP] / (d[D_LOOP] ? d[D_LOOP] : 1));
  const double li = (double)(d[D_L_ITERS] ? d[D_L_ITERS] : 1);
  fprintf(stderr, "[diag %s] <=2 live lanes: %llu iterations, cycles/iter: loop %.0f step %.0f star %.0f (cell %.0f prefix %.0f "
                  "window %.0f final %.0f) mid %.0f ray %.0f end %.0f sample %.0f tail %.0f\n",
          tag, d[D_L_ITERS], d[D_L_LOOP] / li, d[D_L_STEP] / li, d[D_L_STAR] / li, d[D_L_S_CELL] / li, d[D_L_S_PFX] / li,
          d[D_L_S_WIN] / li, d[D_L_S_FIN] / li, d[D_L_MID] / li, d[D_L_RAY] / li, d[D_L_END] / li, d[D_L_SAMPLE] / li,
          d[D_L_TAIL] / li);
  fprintf(stderr, "[diag %s] <=2 live lanes star detail: prologue %.0f  list build+sync %.0f  star total (in-function) %.0f\n", tag,
          d[D_L_S_PRE] / li, d[D_L_S_BUILD] / li, d[D_L_S_POST] / li);
  unsigned long long z[D_NUM] = {};
  hipMemcpyToSymbol(sym, z, sizeof(z));
#else
  (void)tag;
  (void)sym;
#endif
}

hipError_t launch_math_selftest(int which, const double* x, double* out, int64_t n, hipStream_t s) {
  int grid = (int)((n + 255) / 256);
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(wos_math_selftest_kernel, dim3(grid), dim3(256), 0, s, which, x, out, n);
  return hipGetLastError();
}

}  // namespace wos

