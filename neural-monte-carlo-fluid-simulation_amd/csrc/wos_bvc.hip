// wos_bvc.hip -- boundary value caching on the GPU (the reference's `bvc`,
// bindings/zombie/demo/demo.cpp:265-363, over boundary_value_caching/*.h).
//
//   wos_bvc_point_info_kernel  one lane per point: distances to the boundaries, the
//                              inside test and the source texel (grid.h:352-368,
//                              domain_sampler.h:50-58);
//   wos_bvc_start_kernel       one lane per boundary sample: the first sphere radius
//                              (walk_on_stars.h:400-419, the star radius from the
//                              sample itself, wave-cooperative) and its walk tasks;
//   wos_walk_kernel<2,GG,true> the walks of estimateSolution (walk_on_stars.h:422-463)
//                              on the solve's persistent walk kernel;
//   wos_bvc_fold_kernel        the Welford mean of each sample's recorded walks;
//   wos_bvc_splat_kernel       Splatter::splat (splatter.h:43-247): every evaluation
//                              point (one lane) folds the cached samples in order,
//                              staged through LDS in tiles (every lane reads the same
//                              record: a broadcast), with the free-space Green's
//                              functions (distributions.h:8-272) in the reference's
//                              float/double arithmetic.
#include "wos_bvc.h"
#include "wos_device.h"
#include "wos_launch.h"

namespace wos {

// closest point by one lane: the sequential `<=` scan keeps the highest index
// attaining the minimum d^2 -- the primitive closest_wave picks
template <int DIM>
__device__ Closest closest_lane(const float* prims, int np, const float* x) {
  constexpr int PS = Layout<DIM>::prim;
  float bk = kFltMax;
  int bi = -1;
  for (int p = 0; p < np; p++) {
    float pt[DIM], t0, t1;
    const float d = cp_prim<DIM>(prims + p * PS, x, pt, &t0, &t1);
    const float d2 = d * d;
    if (d2 <= bk) { bk = d2; bi = p; }
  }
  Closest c;
  c.prim = bi;
  c.d = kFltMax;
  c.t0 = c.t1 = 0.0f;
  c.p[0] = c.p[1] = c.p[2] = 0.0f;
  if (bi >= 0) c.d = cp_prim<DIM>(prims + bi * PS, x, c.p, &c.t0, &c.t1);
  return c;
}

template <int DIM>
__global__ __launch_bounds__(256) void wos_bvc_point_info_kernel(const DevScene sc, const float* __restrict__ pts,
                                                                 int64_t n, float* __restrict__ dd,
                                                                 float* __restrict__ nd, int32_t* __restrict__ inside,
                                                                 float* __restrict__ src) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x[DIM];
  for (int k = 0; k < DIM; k++) x[k] = pts[i * DIM + k];
  float nDist = kFltMax, nSigned = kFltMax;
  if (sc.n_prims > 0) {
    const Closest c = closest_lane<DIM>(sc.prim, sc.n_prims, x);
    nDist = c.d;
    nSigned = signed_dist<DIM>(sc.paux, c, x);
  }
  float dDist, dSigned;
  if (sc.n_dprims > 0) {
    const Closest c = closest_lane<DIM>(sc.dprim, sc.n_dprims, x);
    dDist = c.d;
    dSigned = signed_dist<DIM>(sc.dpaux, c, x);
  } else {
    dDist = dSigned = bbox_far_dist<DIM>(sc, x);
  }
  // insideDomain (fcpw_scene_loader.h:642-648)
  const bool in = !sc.watertight ? true
                  : (__builtin_fabsf(dSigned) < __builtin_fabsf(nSigned) ? dSigned < 0.0f : nSigned < 0.0f);
  if (dd) dd[i] = dDist;
  if (nd) nd[i] = nDist;
  if (inside) inside[i] = in ? 1 : 0;
  if (src) src[i] = source_value<DIM>(sc, x);
}

// The first sphere radius of estimateSolution (walk_on_stars.h:390-419) for every
// sample, then its walk tasks: WalkState(pt, n, prevDirection = n, FLT_MAX, 1, onNeumann)
// for each of the wpp walks.  on_neumann: a boundary sample (SampleType::OnNeumannBoundary);
// else a point in the domain (an evaluation point near the Dirichlet boundary,
// splatter.h:160-196, or a finite-difference Dirichlet sample).  Double-sided
// normal-aligned boundary samples walk with the flipped normal and query the star radius
// with flipNormalOrientation.  Walk w of sample i is seeded seed32(key, base + i, w, tag);
// from inside the epsilon shell only walk 0 runs (walk_on_stars.h:383-386).
template <int DIM>
__global__ __launch_bounds__(kBlock) void wos_bvc_start_kernel(const DevScene sc, const DevParams prm,
                                                               const float* __restrict__ bpt,
                                                               const float* __restrict__ bnrm,
                                                               const uint8_t* __restrict__ aligned,
                                                               const float* __restrict__ bdd, int64_t nb,
                                                               const DevTasks tk, int on_neumann, uint32_t tag) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave_u = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  StarLDS<DIM>* starL = reinterpret_cast<StarLDS<DIM>*>(reinterpret_cast<char*>(smem) +
                                                        wave_u * walk_scratch_bytes<DIM>());
  const LGeom G = geometry_view<DIM, true>(sc, smem, true, false);  // records read through L2
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = i < nb;
  float x[DIM], n[DIM], dd = 0.0f;
  bool flip = false;
  for (int k = 0; k < DIM; k++) { x[k] = 0.0f; n[k] = 0.0f; }
  if (valid) {
    for (int k = 0; k < DIM; k++) { x[k] = bpt[i * DIM + k]; n[k] = bnrm ? bnrm[i * DIM + k] : 0.0f; }
    dd = bdd[i];
    flip = on_neumann && sc.double_sided && aligned != nullptr && aligned[i] != 0;
    if (flip) for (int k = 0; k < DIM; k++) n[k] *= -1.0f;
  }
  const bool query = valid && dd > prm.epsilon_shell && prm.steps_before_maximal_spheres != 0;
  const float starQ = star_radius_wave<DIM, true>(G, sc, prm, query, x, dd, flip, starL, lane);
  if (!valid) return;
  float r0 = dd;
  if (query) r0 = prm.min_star_radius <= dd ? smax(0.99f * starQ, prm.min_star_radius) : starQ;
  const int64_t T = tk.T;
  for (int w = 0; w < tk.wpp; w++) {
    const int64_t t = i * tk.wpp + w;
    for (int k = 0; k < DIM; k++) {
      tk.pt[k * T + t] = x[k];
      tk.n0[k * T + t] = n[k];
    }
    tk.thr[t] = 1.0f;
    tk.tsrc[t] = 0.0f;
    tk.dd[t] = dd;
    tk.r0[t] = r0;
    const bool shell = !(dd > prm.epsilon_shell);
    tk.sflags[t] = (on_neumann ? 1u : 0u) | (shell && w > 0 ? 2u : 0u) | (tag << 8);
  }
  tk.pstate[i] = kPtEstimate;
  tk.perm[i] = (uint32_t)i;
}

// SampleStatistics::addSolutionEstimate over each sample's recorded walks, in walk
// order (walk_on_stars.h:450-462, 767-770)
__global__ __launch_bounds__(256) void wos_bvc_fold_kernel(const DevTasks tk, int64_t nb, float* __restrict__ sol,
                                                           int32_t* __restrict__ nest) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb) return;
  float mean = 0.0f;
  int N = 0;
  for (int w = 0; w < tk.wpp; w++) {
    const int64_t t = i * tk.wpp + w;
    if (!(tk.code[t] & 1u)) continue;
    N += 1;
    const float delta = tk.total[t] - mean;
    mean += delta / (float)N;
  }
  sol[i] = mean;
  if (nest) nest[i] = N;
}

// useFiniteDifferencesForBoundaryDerivatives (boundary_sampler.h:171-184): the normal derivative
// of a Dirichlet sample is (g(x') - u) / |d| with x' its projection onto the Dirichlet boundary
// (projectToDirichlet: the closest point, signed distance when double-sided) and u its estimate
__global__ __launch_bounds__(256) void wos_bvc_fd_kernel(const DevScene sc, const float* __restrict__ pts,
                                                         const float* __restrict__ sol, int64_t n,
                                                         float* __restrict__ dn) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x[2] = {pts[2 * i], pts[2 * i + 1]};
  float gv = sc.g_dirichlet, sd = 0.0f;
  if (sc.n_dprims > 0) {
    const Closest c = closest_lane<2>(sc.dprim, sc.n_dprims, x);
    sd = sc.double_sided ? signed_dist<2>(sc.dpaux, c, x) : c.d;
    gv = dirichlet_value<2>(sc, x);
  }
  dn[i] = (gv - sol[i]) / __builtin_fabsf(sd);
}

// ---- free-space Green's functions, 2D (distributions.h:85-119, 168-219) -------
struct FreeSpace2 {
  bool yukawa;
  float lambda, sqrtLambda;

  // K0, K1 at mu r (bessel::bessk0 / bessk1 in double, rounded to float) and
  // bessk(2, mu r) = K0 + (1 * 2 / (mu r)) K1 from the double values (bessel.hpp:584-608)
  __device__ __forceinline__ void bessel_k(float mur, float* K0, float* K1, float* K2) const {
    double i0, k0, i1, k1;
    bessel_ik<true, true>((double)mur, &i0, &k0, &i1, &k1);
    *K0 = (float)k0;
    *K1 = (float)k1;
    if (K2) {
      const double tox = 2.0 / (double)mur;
      *K2 = (float)(k0 + (1.0 * tox) * k1);
    }
  }
  __device__ __forceinline__ float evaluate(float r, float K0) const {
    if (!yukawa) return (float)((double)(-flog(r)) / kTwoPi);
    return (float)((double)K0 / kTwoPi);
  }
  __device__ __forceinline__ void gradient(float r, const float* xy, float K1, float* out) const {
    if (!yukawa) {
      const float s = (float)(kTwoPi * (double)(r * r));
      for (int k = 0; k < 2; k++) out[k] = (-xy[k]) / s;
      return;
    }
    const float Qr = sqrtLambda * K1;
    const float s = (float)(kTwoPi * (double)r);
    for (int k = 0; k < 2; k++) out[k] = ((-xy[k]) * Qr) / s;
  }
  __device__ __forceinline__ float poisson(float r, const float* xy, const float* n, float K1) const {
    const float nd = n[0] * xy[0] + n[1] * xy[1];
    if (!yukawa) return (float)((double)nd / (kTwoPi * (double)(r * r)));
    const float Qr = sqrtLambda * K1;
    return (float)((double)(nd * Qr) / (kTwoPi * (double)r));
  }
  __device__ __forceinline__ void poisson_gradient(float r, const float* xy, const float* n, float K0, float K1,
                                                   float K2, float* out) const {
    const float r2 = r * r;
    const float nd = n[0] * xy[0] + n[1] * xy[1];
    if (!yukawa) {
      const float c = 2.0f * (nd / r2);
      const float s = (float)(kTwoPi * (double)r2);
      for (int k = 0; k < 2; k++) out[k] = (n[k] - c * xy[k]) / s;
      return;
    }
    const float Qr1 = sqrtLambda * K1;
    const float Qr2 = lambda * (K0 + K2) / 2.0f;
    const float c = (nd / r2) * (Qr1 + r * Qr2);
    const float s = (float)(kTwoPi * (double)r);
    for (int k = 0; k < 2; k++) out[k] = (n[k] * Qr1 - c * xy[k]) / s;
  }
};

__device__ __forceinline__ bool finite_f(float v) { return __builtin_isfinite(v); }

// One (evaluation point, cached sample) term of Splatter::splat: the estimate and its
// gradient, and the statistics class it folds into (0 boundary, 1 normal-aligned,
// 2 domain; 3: skipped, a non-finite kernel value -- the reference's `continue`).
__device__ __forceinline__ int splat_term(const FreeSpace2& gf, const float* R, const float* x, float radius_clamp,
                                          float reg, float* est, float* ge) {
  const int kind = (int)R[7];
  const float pdf = R[4], value = R[5];
  const float yx[2] = {R[0] - x[0], R[1] - x[1]};
  const float xy[2] = {x[0] - R[0], x[1] - R[1]};
  float r = smax(radius_clamp, __builtin_sqrtf(yx[0] * yx[0] + yx[1] * yx[1]));
  float K0 = 0.0f, K1 = 0.0f, K2 = 0.0f;
  if (gf.yukawa) gf.bessel_k(r * gf.sqrtLambda, &K0, &K1, kind == kBvcDomain ? nullptr : &K2);
  float G = gf.evaluate(r, K0);
  float dG[2];
  gf.gradient(r, xy, K1, dG);
  // the kernel norms |dG|, |dP| only gate on finiteness (splatter.h:224-228, 273-275): the
  // square root of a sum of squares is finite exactly when the sum is
  const float dGNorm2 = dG[0] * dG[0] + dG[1] * dG[1];
  const bool al = kind == kBvcAligned || kind == kBvcDirichletAligned;
  if (kind != kBvcDomain) {  // splatBoundaryData (splatter.h:214-264)
    const float nd = R[6];
    const float s = al ? -1.0f : 1.0f;
    const float n[2] = {R[2] * s, R[3] * s};
    float P = gf.poisson(r, xy, n, K1);
    float dP[2];
    gf.poisson_gradient(r, xy, n, K0, K1, K2, dP);
    const float dPNorm2 = dP[0] * dP[0] + dP[1] * dP[1];
    if (!(finite_f(G) && finite_f(P) && finite_f(dGNorm2) && finite_f(dPNorm2))) return 3;
    if (reg > 0.0f) {
      r /= reg;
      P *= 1.0f - fexp(-r * r);  // computePoissonKernelRegularization<2> (splatter.h:28-32)
    }
    *est = (G * nd - P * value) / pdf;
    for (int k = 0; k < 2; k++) ge[k] = (dG[k] * nd - dP[k] * value) / pdf;
    return al ? 1 : 0;
  }
  // splatSourceData (splatter.h:267-301)
  if (!(finite_f(G) && finite_f(dGNorm2))) return 3;
  *est = (G * value) / pdf;
  for (int k = 0; k < 2; k++) ge[k] = (dG[k] * value) / pdf;
  return 2;
}

// The splat runs in two phases per tile of kSplatT cached samples, for kSplatPts
// evaluation points (one per lane) per workgroup of 4 waves:
//   terms  every wave evaluates a quarter of the tile's (point, sample) terms into LDS
//          -- the arithmetic, 4 waves per point set instead of one;
//   fold   waves 0, 1, 2 each run one component (solution, gradient x, gradient y) of
//          the point's three Welford statistics (SampleStatistics, splatter.h:315-334)
//          over the tile's terms in cache order -- the same division chain per
//          component as one lane running all three, so the result is unchanged; wave 3
//          stages the next tile's records.
// A launch folds the records [r0, r1) of the cache: the statistics start from zero
// (first) or from `state`, and end in the outputs (last) or in `state` -- so the splat
// of the Neumann samples can run while the Dirichlet samples are still being estimated,
// and the rest continues the same division chains exactly.  state: per point, per
// component, the three classes' means then their counts ([3][6][ne] words).
constexpr int kSplatPts = 64, kSplatT = 32, kSplatWaves = 4;

// The evaluation points the splat visits, packed (wave-ordered runs; the order only groups
// points into waves): not masked by saveEvaluationGrid (grid.h:393-409) -- their output is 0
// whatever their statistics -- and not within the cutoff of the Dirichlet boundary
// (splatter.h:94: a pointwise estimate, estimatePointwiseNearDirichletBoundary, replaces
// them).  Every other point's output is 0 (the outputs are cleared before the splat).
__global__ __launch_bounds__(256) void wos_bvc_splat_list_kernel(const float* __restrict__ edd,
                                                                 const float* __restrict__ end_,
                                                                 const int32_t* __restrict__ ein, int64_t ne,
                                                                 float cutoff, float mask, int double_sided,
                                                                 uint32_t* __restrict__ list,
                                                                 uint32_t* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool keep = false;
  if (i < ne) {
    const float dDist = edd[i];
    const bool in = ein[i] != 0;
    const float ad = __builtin_fabsf(dDist), an = __builtin_fabsf(end_[i]);
    const bool masked = (!in && !double_sided) || smin(ad, an) < mask;
    keep = !masked && !(dDist < cutoff);
  }
  const uint64_t b = __ballot(keep);
  if (b == 0) return;
  const int lane = threadIdx.x & 63;
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(count, (uint32_t)__popcll(b));
  base = (uint32_t)__shfl((int)base, 0);
  if (keep) list[base + rank] = (uint32_t)i;
}

// Splatter::splat over every listed evaluation point and every cached sample (boundary,
// normal-aligned, domain in cache order), then EvaluationPoint::getEstimatedSolution /
// getEstimatedGradient (splatter.h:315-334).
__global__ __launch_bounds__(kSplatPts * kSplatWaves) void wos_bvc_splat_kernel(
    const float* __restrict__ recs, int r0, int r1, int first, int last, float* __restrict__ state,
    const uint32_t* __restrict__ list, const uint32_t* __restrict__ count, const float* __restrict__ ept,
    int64_t ne, float absorption, float radius_clamp, float reg, float* __restrict__ sol_out,
    float* __restrict__ grad_out) {
  __shared__ float rtile[2][kSplatT * kBvcRec];
  __shared__ float term[3][kSplatT][kSplatPts];
  __shared__ uint8_t tcls[kSplatT][kSplatPts];
  const int64_t nl = (int64_t)*count;
  if ((int64_t)blockIdx.x * kSplatPts >= nl) return;  // block-uniform
  const int lane = threadIdx.x & (kSplatPts - 1);
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kSplatPts));
  const int64_t slot = (int64_t)blockIdx.x * kSplatPts + lane;  // list slot
  const bool valid = slot < nl;
  const int64_t i = valid ? (int64_t)list[slot] : 0;
  FreeSpace2 gf;
  gf.yukawa = absorption > 0.0f;
  gf.lambda = absorption;
  gf.sqrtLambda = __builtin_sqrtf(absorption);
  float x[2] = {0.0f, 0.0f};
  if (valid) { x[0] = ept[2 * i]; x[1] = ept[2 * i + 1]; }
  const bool splat = valid;
  // this wave's component of the three classes' statistics and their counts
  float m0 = 0.0f, m1 = 0.0f, m2 = 0.0f;
  int n0 = 0, n1 = 0, n2 = 0;
  float* sw = state + (size_t)(wave < 3 ? wave : 0) * 6 * ne + slot;  // this wave's component, by slot
  if (!first && valid && wave < 3) {
    m0 = sw[0]; m1 = sw[ne]; m2 = sw[2 * ne];
    n0 = __float_as_int(sw[3 * ne]); n1 = __float_as_int(sw[4 * ne]); n2 = __float_as_int(sw[5 * ne]);
  }
  const float* rr = recs + (size_t)r0 * kBvcRec;
  const int nrec = r1 - r0;
  for (int e = threadIdx.x; e < kSplatT * kBvcRec; e += kSplatPts * kSplatWaves)
    if (e < nrec * kBvcRec) rtile[0][e] = rr[e];
  __syncthreads();
  int buf = 0;
  for (int t0 = 0; t0 < nrec; t0 += kSplatT) {
    const int cnt = nrec - t0 < kSplatT ? nrec - t0 : kSplatT;
    // terms: samples wave, wave + 4, ... of the tile
    for (int j = wave; j < cnt; j += kSplatWaves) {
      float est = 0.0f, ge[2] = {0.0f, 0.0f};
      int c = 3;
      if (splat) c = splat_term(gf, &rtile[buf][j * kBvcRec], x, radius_clamp, reg, &est, ge);
      term[0][j][lane] = est;
      term[1][j][lane] = ge[0];
      term[2][j][lane] = ge[1];
      tcls[j][lane] = (uint8_t)c;
    }
    __syncthreads();
    if (wave < 3) {
      if (splat) {
        for (int j = 0; j < cnt; j++) {
          const int c = tcls[j][lane];
          if (c == 3) continue;
          const float v = term[wave][j][lane];
          int n = c == 0 ? n0 : c == 1 ? n1 : n2;
          float m = c == 0 ? m0 : c == 1 ? m1 : m2;
          n += 1;
          m += (v - m) / (float)n;
          if (c == 0) { m0 = m; n0 = n; } else if (c == 1) { m1 = m; n1 = n; } else { m2 = m; n2 = n; }
        }
      }
    } else {
      const int nx = t0 + kSplatT;
      for (int e = lane; e < kSplatT * kBvcRec; e += kSplatPts)
        if ((int64_t)nx * kBvcRec + e < (int64_t)nrec * kBvcRec) rtile[buf ^ 1][e] = rr[(size_t)nx * kBvcRec + e];
    }
    __syncthreads();
    buf ^= 1;
  }
  if (!valid || wave >= 3) return;
  if (!last) {
    sw[0] = m0; sw[ne] = m1; sw[2 * ne] = m2;
    sw[3 * ne] = __int_as_float(n0); sw[4 * ne] = __int_as_float(n1); sw[5 * ne] = __int_as_float(n2);
    return;
  }
  float v = m0;
  v += m1;
  v += m2;
  if (wave == 0) sol_out[i] = v;
  else grad_out[2 * i + (wave - 1)] = v;
}

template __global__ void wos_walk_kernel<2, false, true>(const DevScene, const DevParams, const DevTasks, int64_t,
                                                           int64_t, unsigned long long*, unsigned int*, int);
template __global__ void wos_walk_kernel<2, true, true>(const DevScene, const DevParams, const DevTasks, int64_t,
                                                          int64_t, unsigned long long*, unsigned int*, int);

// ---- host launchers ----------------------------------------------------------
void diag_dump_bstart(const char* tag) { diag_print(tag, HIP_SYMBOL(g_diag)); }

hipError_t launch_bvc_point_info(const DevScene& sc, const float* pts, int64_t n, float* dd, float* nd,
                                 int32_t* inside, float* src, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int grid = (int)((n + 255) / 256);
  hipLaunchKernelGGL(wos_bvc_point_info_kernel<2>, dim3(grid), dim3(256), 0, s, sc, pts, n, dd, nd, inside, src);
  return hipGetLastError();
}

size_t bvc_start_lds_bytes() { return (size_t)kWavesPerBlockHost * walk_scratch_bytes<2>(); }

hipError_t launch_bvc_start(const DevScene& sc, const DevParams& prm, const float* bpt, const float* bnrm,
                            const uint8_t* aligned, const float* bdd, int64_t nb, const DevTasks& tk, int on_neumann,
                            uint32_t tag, hipStream_t s) {
  if (nb <= 0) return hipSuccess;
  const int grid = (int)((nb + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(wos_bvc_start_kernel<2>, dim3(grid), dim3(kBlock), bvc_start_lds_bytes(), s, sc, prm, bpt, bnrm,
                     aligned, bdd, nb, tk, on_neumann, tag);
  return hipGetLastError();
}

hipError_t launch_bvc_fd(const DevScene& sc, const float* pts, const float* sol, int64_t n, float* dn, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(wos_bvc_fd_kernel, dim3((int)((n + 255) / 256)), dim3(256), 0, s, sc, pts, sol, n, dn);
  return hipGetLastError();
}

hipError_t launch_walks_bstart(const DevScene& sc, const DevParams& prm, const DevTasks& tk, int64_t base,
                               int64_t stride, unsigned long long* counters, unsigned int* tqueue, int grid,
                               size_t shmem, int geom_floats, hipStream_t s) {
  if (prm.robust)
    return launch_walks_rb(2, true, sc, prm, tk, base, stride, counters, tqueue, grid, shmem, geom_floats, s);
  if (sc.geom_global)
    hipLaunchKernelGGL((wos_walk_kernel<2, true, true>), dim3(grid), dim3(kBlock), shmem, s, sc, prm, tk, base, stride,
                       counters, tqueue, geom_floats);
  else
    hipLaunchKernelGGL((wos_walk_kernel<2, false, true>), dim3(grid), dim3(kBlock), shmem, s, sc, prm, tk, base,
                       stride, counters, tqueue, geom_floats);
  return hipGetLastError();
}

hipError_t occupancy_walk_bstart(bool geom_global, size_t shmem, int* blocks, bool robust) {
  if (robust) return occupancy_rb(2, 2, geom_global, shmem, blocks);
  return geom_global ? hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wos_walk_kernel<2, true, true>, kBlock, shmem)
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wos_walk_kernel<2, false, true>, kBlock, shmem);
}

hipError_t launch_bvc_fold(const DevTasks& tk, int64_t nb, float* sol, int32_t* nest, hipStream_t s) {
  if (nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(wos_bvc_fold_kernel, dim3((int)((nb + 255) / 256)), dim3(256), 0, s, tk, nb, sol, nest);
  return hipGetLastError();
}

hipError_t launch_bvc_splat_list(const float* edd, const float* end_, const int32_t* ein, int64_t ne, float cutoff,
                                 float mask, int double_sided, uint32_t* list, uint32_t* count, hipStream_t s) {
  if (ne <= 0) return hipSuccess;
  hipLaunchKernelGGL(wos_bvc_splat_list_kernel, dim3((int)((ne + 255) / 256)), dim3(256), 0, s, edd, end_, ein, ne,
                     cutoff, mask, double_sided, list, count);
  return hipGetLastError();
}

hipError_t launch_bvc_splat(const float* recs, int r0, int r1, int first, int last, float* state,
                            const uint32_t* list, const uint32_t* count, const float* ept, int64_t ne,
                            float absorption, float radius_clamp, float reg, float* sol, float* grad, hipStream_t s) {
  if (ne <= 0) return hipSuccess;
  hipLaunchKernelGGL(wos_bvc_splat_kernel, dim3((int)((ne + kSplatPts - 1) / kSplatPts)), dim3(kSplatPts * kSplatWaves),
                     0, s, recs, r0, r1, first, last, state, list, count, ept, ne, absorption, radius_clamp, reg, sol,
                     grad);
  return hipGetLastError();
}

// the estimated values of the boundary records [b0, b1): the solution, and the normal
// derivative -- a Dirichlet sample's estimate (kinds 3, 4), a Neumann sample's pde.neumann at its
// point (kinds 0, 1; boundary_sampler.h:126-133: 0 in the reference's scenes, the image-valued h
// when the scene has one) -- written once the walks that estimate them are done
__global__ __launch_bounds__(256) void wos_bvc_fill_kernel(float* __restrict__ recs, int64_t b0, int64_t b1,
                                                           const float* __restrict__ bsol,
                                                           const float* __restrict__ bdn, const DevScene sc,
                                                           int ignore_neumann) {
  const int64_t i = b0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= b1) return;
  float* R = recs + i * kBvcRec;
  const int kind = (int)R[7];
  R[5] = bsol[i];
  R[6] = (kind == kBvcDirichlet || kind == kBvcDirichletAligned) ? bdn[i]
         : ignore_neumann                                       ? 0.0f
                                                                : neumann_value(sc, R);
}

hipError_t launch_bvc_fill(float* recs, int64_t b0, int64_t b1, const float* bsol, const float* bdn,
                           const DevScene& sc, int ignore_neumann, hipStream_t s) {
  if (b1 <= b0) return hipSuccess;
  hipLaunchKernelGGL(wos_bvc_fill_kernel, dim3((int)((b1 - b0 + 255) / 256)), dim3(256), 0, s, recs, b0, b1, bsol, bdn,
                     sc, ignore_neumann);
  return hipGetLastError();
}

}  // namespace wos
