// wos_launch.h -- host entry points of the kernels in wos_kernel.hip.
#pragma once
#include <hip/hip_runtime.h>
#include "wos_scene.h"

namespace wos {
constexpr int kBlockThreads = 256;
constexpr int kWavesPerBlockHost = 4;
constexpr int kNumCounters = 9;
int rec_floats(int dim);
hipError_t launch_solve(int dim, const DevScene& sc, const DevParams& prm, const float* pts, int64_t n,
                        int64_t base, int64_t stride, float* p, float* g, int32_t* nest, int32_t* steps,
                        unsigned long long* counters, unsigned int* work, int grid, size_t shmem,
                        int geom_floats, int lhs_floats, hipStream_t s);
hipError_t occupancy_blocks_per_cu(int dim, size_t shmem, int* blocks);
hipError_t launch_math_selftest(int which, const double* x, double* out, int64_t n, hipStream_t s);
}  // namespace wos
