// microbenchmarks of a lone wave's latencies (gfx950): s_memtime deltas
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k_lds_chain(unsigned long long* out, int n, int seed) {
  __shared__ int buf[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) buf[i] = (i * 7 + 1) & 1023;
  __syncthreads();
  int idx = (threadIdx.x + seed) & 1023;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) idx = buf[idx];
  __builtin_amdgcn_s_waitcnt(0);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = idx; }
}
__global__ void k_lds_chain_bcast(unsigned long long* out, int n, int seed) {
  __shared__ int buf[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) buf[i] = (i * 7 + 1) & 1023;
  __syncthreads();
  int idx = seed & 1023;  // all lanes same address
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) idx = buf[idx];
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = idx; }
}
__global__ void k_valu_chain(unsigned long long* out, int n, float seed) {
  float x = seed + threadIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) x = x * 1.0000001f + 0.5f;
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = (unsigned long long)x; }
}
__global__ void k_dvalu_chain(unsigned long long* out, int n, double seed) {
  double x = seed + threadIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) x = x * 1.0000001 + 0.5;
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = (unsigned long long)x; }
}
__global__ void k_gmem_chain(unsigned long long* out, const int* __restrict__ g, int n, int seed) {
  int idx = (seed + threadIdx.x) & ((1 << 20) - 1);
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) idx = g[idx];
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = idx; }
}
// dependent scalar loads (s_load_dword through the scalar cache; the table stays in it)
__global__ void k_smem_chain(unsigned long long* out, const int* __restrict__ g, int n, int seed) {
  int idx = __builtin_amdgcn_readfirstlane(seed & 1023);
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) idx = __builtin_amdgcn_readfirstlane(g[idx] & 1023);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = idx; }
}
__global__ void k_bperm_chain(unsigned long long* out, int n, int seed) {
  int v = threadIdx.x + seed;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) v = __shfl(v, (threadIdx.x + v) & 63);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = v; }
}
__global__ void k_ldsatomic(unsigned long long* out, int n, int seed) {
  __shared__ unsigned long long best[64];
  if (threadIdx.x < 64) best[threadIdx.x] = ~0ull;
  __syncthreads();
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) {
    atomicMin(&best[seed & 63], (unsigned long long)(threadIdx.x * 977 + i));
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  __builtin_amdgcn_s_waitcnt(0);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = best[seed & 63]; }
}
__global__ void k_clock(unsigned long long* out, int n) {
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  volatile float x = 1.0f;
  for (int i = 0; i < n; i++) x = x * 1.0000001f;
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }
}
int main1() {
  unsigned long long* d; hipMalloc(&d, 16);
  int* g; hipMalloc(&g, (1 << 20) * 4);
  int* h = (int*)malloc((1 << 20) * 4);
  for (int i = 0; i < (1 << 20); i++) h[i] = (int)(((long long)i * 2654435761LL + 12345) & ((1 << 20) - 1));
  hipMemcpy(g, h, (1 << 20) * 4, hipMemcpyHostToDevice);
  unsigned long long r[2];
  const int N = 1000;
  auto rep = [&](const char* name, double n) { hipDeviceSynchronize(); hipMemcpy(r, d, 16, hipMemcpyDeviceToHost); printf("%-22s %8.1f cycles/op\n", name, r[0] / n); };
  for (int rr = 0; rr < 2; rr++) {
    hipLaunchKernelGGL(k_clock, 1, 64, 0, 0, d, 100000); hipDeviceSynchronize(); hipMemcpy(r, d, 16, hipMemcpyDeviceToHost);
    printf("clock: memtime %llu realtime(100MHz) %llu -> %.0f MHz\n", r[0], r[1], r[0] / (r[1] / 100.0));
    hipLaunchKernelGGL(k_lds_chain, 1, 64, 0, 0, d, N, 3); rep("lds dep chain", N);
    hipLaunchKernelGGL(k_lds_chain_bcast, 1, 64, 0, 0, d, N, 3); rep("lds dep chain bcast", N);
    hipLaunchKernelGGL(k_valu_chain, 1, 64, 0, 0, d, N * 10, 1.0f); rep("valu f32 fma chain", N * 10);
    hipLaunchKernelGGL(k_dvalu_chain, 1, 64, 0, 0, d, N * 10, 1.0); rep("valu f64 fma chain", N * 10);
    hipLaunchKernelGGL(k_gmem_chain, 1, 64, 0, 0, d, g, 200, 5); rep("global dep chain 4MB", 200);
    hipLaunchKernelGGL(k_bperm_chain, 1, 64, 0, 0, d, N, 1); rep("shfl dep chain", N);
    hipLaunchKernelGGL(k_smem_chain, 1, 64, 0, 0, d, g, N, 7); rep("scalar-load dep chain", N);
    hipLaunchKernelGGL(k_ldsatomic, 1, 64, 0, 0, d, N, 1); rep("lds atomicMin64 same", N);
  }
  return 0;
}
// ---- conflicting LDS atomics: `lanes` lanes of a lone wave fold into one address
template <int W>
__global__ void k_atomic_k(unsigned long long* out, int n, int lanes, int op, int amask) {
  __shared__ unsigned long long b64[64];
  __shared__ unsigned int b32[64];
  if (threadIdx.x < 64) { b64[threadIdx.x] = ~0ull; b32[threadIdx.x] = op ? 0u : ~0u; }
  __syncthreads();
  const int lane = threadIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) {
    if (lane < lanes) {
      // address lane & amask (amask = 0 at run time: all lanes on one address, which the
      // compiler cannot see, so no wave-level atomic rewriting)
      if (W == 64) atomicMin(&b64[lane & amask], (unsigned long long)(lane * 977 + i));
      else if (op == 0) atomicMin(&b32[lane & amask], (unsigned)(lane * 977 + i));
      else atomicOr(&b32[lane & amask], 1u << (lane & 31));
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  __builtin_amdgcn_s_waitcnt(0);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = b64[0] + b32[0]; }
}
// distinct addresses (no conflict) for comparison
__global__ void k_atomic_distinct(unsigned long long* out, int n, int lanes) {
  __shared__ unsigned long long b64[64];
  if (threadIdx.x < 64) b64[threadIdx.x] = ~0ull;
  __syncthreads();
  const int lane = threadIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) {
    if (lane < lanes) atomicMin(&b64[lane], (unsigned long long)(lane * 977 + i));
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  __builtin_amdgcn_s_waitcnt(0);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = b64[0]; }
}
// wave min-reduction of a 64-bit key with DPP/permute (the alternative to the atomics)
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
  for (int d = 32; d >= 1; d >>= 1) {
    unsigned lo = __shfl_xor((unsigned)v, d), hi = __shfl_xor((unsigned)(v >> 32), d);
    unsigned long long o = ((unsigned long long)hi << 32) | lo;
    v = o < v ? o : v;
  }
  return v;
}
__global__ void k_wavemin(unsigned long long* out, int n) {
  unsigned long long v = threadIdx.x * 977ull + 5;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) v = wave_min_u64(v + i);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = v; }
}
int main2() {
  unsigned long long* d; hipMalloc(&d, 16);
  unsigned long long r[2];
  const int N = 200;
  auto rep = [&](const char* name, int k) { hipDeviceSynchronize(); hipMemcpy(r, d, 16, hipMemcpyDeviceToHost); printf("%-26s lanes %2d %8.1f cycles/round\n", name, k, r[0] / (double)N); };
  for (int k : {1, 2, 4, 8, 16, 32, 64}) {
    hipLaunchKernelGGL(k_atomic_k<64>, 1, 64, 0, 0, d, N, k, 0, 0); rep("atomicMin u64 same addr", k);
    hipLaunchKernelGGL(k_atomic_k<32>, 1, 64, 0, 0, d, N, k, 0, 0); rep("atomicMin u32 same addr", k);
    hipLaunchKernelGGL(k_atomic_k<32>, 1, 64, 0, 0, d, N, k, 1, 0); rep("atomicOr u32 same addr", k);
    hipLaunchKernelGGL(k_atomic_distinct, 1, 64, 0, 0, d, N, k); rep("atomicMin u64 distinct", k);
  }
  hipLaunchKernelGGL(k_wavemin, 1, 64, 0, 0, d, N); rep("wave_min_u64 (shfl_xor)", 64);
  return 0;
}
int main(int argc, char** argv) { if (argc > 1) return main2(); return main1(); }
