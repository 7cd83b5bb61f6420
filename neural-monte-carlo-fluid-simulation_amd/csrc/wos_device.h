// wos_device.h -- gfx950 walk-on-stars device code: the queries, the Green's
// functions, the samplers and the kernel templates (instantiated by wos_kernel.hip
// for the solve and by wos_bvc.hip for boundary value caching).
//
// One wavefront (64 lanes) owns one query point at a time; lane l runs
// antithetic pair l of that point (both members, sharing the pair's walk
// stream, walk_on_stars.h:494-616).  Neumann segments/triangles and the
// silhouette candidates are staged in LDS once per workgroup and scanned
// brute-force (every lane reads the same LDS word: broadcast, no conflicts).
// The per-point statistics (Welford means with sequential control variates,
// walk_on_stars.h:500-506,744-877) are folded in walk order by lanes 0..DIM
// in lockstep so the result is bit-identical to the sequential CPU oracle.
// Points are handed out by a device-scope atomic work counter (one returning
// atomicAdd per point), so uneven per-point cost (near-wall points run longer
// walks) does not leave waves idle at the tail.
//
// Numerics follow the reference operation by operation: float state, double
// Bessel evaluations rounded to float members (distributions.h:573-696), double
// 2*pi divisors, Eigen's float-scalar conversions -- see the oracle restatement
// (oracle/wos_oracle.c) which is the parity checker for this file.

#pragma once
#include <cstdio>

#include "wos_detmath.h"
#include "wos_scene.h"

namespace wos {

#ifndef WOS_DIAG
#define WOS_DIAG 0
#endif

constexpr int kWave = 64;
constexpr int kBlock = 256;

enum { WC_DIRICHLET = 0, WC_RR = 1, WC_MAXLEN = 2, WC_ESCAPED = 3 };

// counters[] slots
enum { C_STEPS = 0, C_WASTED, C_REC, C_ESC, C_MAXL, C_RR, C_DIR, C_PTS, C_ITERS, C_NUM };

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Diagnostic build only (-DWOS_DIAG=1, never shipped): per-section wave cycles
// (s_memtime) and lane-packing counters of the walk kernel.
enum { D_ITERS = 0, D_LANES, D_STAR, D_RAY, D_SAMPLE, D_STEP, D_LOOP, D_RAYOVF, D_SCALLS, D_SGVISIT, D_SCAND, D_SEXACT,
       D_FB_PTS, D_FB_SETUP, D_FB_LHS, D_FB_BALLS, D_FB_TOTAL, D_FB_MAX, D_WMAXLEN, D_WAVEMAX, D_RCALLS, D_RGENS, D_RITEMS, D_RQUICK, D_RUND, D_RLANES, D_MID, D_END, D_TAIL,
       D_XITERS, D_XLANES, D_XLOOP,
       // the same sections over iterations with <= 2 live lanes (a lone walk's critical path)
       D_L_ITERS, D_L_STEP, D_L_STAR, D_L_MID, D_L_RAY, D_L_END, D_L_SAMPLE, D_L_TAIL, D_L_LOOP,
       D_L_S_CELL, D_L_S_PFX, D_L_S_WIN, D_L_S_FIN, D_L_S_BUILD, D_L_S_PRE, D_L_S_POST,
       // first-ball parts: ball update, member a's source sample, the rest of member a, member b, task stores
       D_FB_UPD, D_FB_SMP, D_FB_MA, D_FB_MB, D_FB_ST, D_FB_ITSUM, D_FB_ITMAX, D_NUM };  // X: iterations after the wave's task queue ran dry
// slots holding maxima (folded with atomicMax)
__host__ __device__ constexpr bool diag_is_max(int k) { return k == D_FB_MAX || k == D_WMAXLEN || k == D_WAVEMAX; }
static __device__ unsigned long long g_diag[D_NUM];
#if WOS_DIAG
static __shared__ unsigned long long s_diag[D_NUM];
#endif
#if WOS_DIAG
#define DIAG_T0(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define DIAG_ADD(slot, v)                                                              \
  do {                                                                                 \
    const uint64_t dt_ = __builtin_amdgcn_s_memtime() - (v);                           \
    if ((int)(threadIdx.x & 63) == __builtin_amdgcn_readfirstlane((int)(threadIdx.x & 63))) \
      atomicAdd(&s_diag[slot], (unsigned long long)dt_);                               \
  } while (0)
#define DIAG_COUNT(slot, n)                                                            \
  do {                                                                                 \
    const unsigned long long n_ = (n);                                                 \
    if ((int)(threadIdx.x & 63) == __builtin_amdgcn_readfirstlane((int)(threadIdx.x & 63))) \
      atomicAdd(&s_diag[slot], n_);                                                    \
  } while (0)
#define DIAG_ADD_LONE(slot, lslot, v, lone)                                            \
  do {                                                                                 \
    const uint64_t dt_ = __builtin_amdgcn_s_memtime() - (v);                           \
    if ((int)(threadIdx.x & 63) == __builtin_amdgcn_readfirstlane((int)(threadIdx.x & 63))) { \
      atomicAdd(&s_diag[slot], (unsigned long long)dt_);                               \
      if (lone) atomicAdd(&s_diag[lslot], (unsigned long long)dt_);                    \
    }                                                                                  \
  } while (0)
#define DIAG_LONE(v, pred) const bool v = __popcll(__ballot(pred)) <= 2
#define DIAG_ADD_IF(slot, v, cond)                                                     \
  do {                                                                                 \
    const uint64_t dt_ = __builtin_amdgcn_s_memtime() - (v);                           \
    if ((cond) && (int)(threadIdx.x & 63) == __builtin_amdgcn_readfirstlane((int)(threadIdx.x & 63))) \
      atomicAdd(&s_diag[slot], (unsigned long long)dt_);                               \
  } while (0)
#define DIAG_LANE(slot) atomicAdd(&s_diag[slot], 1ull)
#define DIAG_MAX(slot, v) atomicMax(&s_diag[slot], (unsigned long long)(v))
#else
#define DIAG_T0(v)
#define DIAG_ADD(slot, v)
#define DIAG_COUNT(slot, n)
#define DIAG_ADD_LONE(slot, lslot, v, lone)
#define DIAG_LONE(v, pred)
#define DIAG_ADD_IF(slot, v, cond)
#define DIAG_LANE(slot)
#define DIAG_MAX(slot, v)
#endif

// Timeline build only (-DWOS_TIMELINE=1, never shipped): the walk kernel's live lanes over
// time.  Bins of 2^kTlShift ticks of the 100 MHz constant clock (s_memrealtime) from the
// launch's first wave (g_tl[0]); per bin the wave-ticks of iterations with a live lane
// (attributed to the bin the iteration starts in), the lane-ticks (live lanes x ticks), the
// tasks handed out and the walks finished.  Printed and reset by diag_print.
#ifndef WOS_TIMELINE
#define WOS_TIMELINE 0
#endif
constexpr int kTlBins = 384, kTlShift = 10;
enum { TL_WAVE = 0, TL_LANE, TL_START, TL_FIN, TL_NUM };
#if WOS_TIMELINE
static __device__ unsigned long long g_tl[1 + TL_NUM * kTlBins];
#endif

template <int DIM>
__device__ __forceinline__ float dotv(const float* a, const float* b) {
  float s = a[0] * b[0] + a[1] * b[1];
  if constexpr (DIM == 3) s = s + a[2] * b[2];
  return s;
}
template <int DIM>
__device__ __forceinline__ float normv(const float* a) { return __builtin_sqrtf(dotv<DIM>(a, a)); }

__device__ __forceinline__ void cross3(float* r, const float* a, const float* b) {
  float x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  r[0] = x; r[1] = y; r[2] = z;
}

// Eigen normalized(): v / sqrt(|v|^2) when |v|^2 > 0
template <int DIM>
__device__ __forceinline__ void normalize_div(float* v) {
  float z = dotv<DIM>(v, v);
  if (z > 0.0f) { float s = __builtin_sqrtf(z); for (int k = 0; k < DIM; k++) v[k] = v[k] / s; }
}
// enoki::normalize restated: v * (1/sqrt(|v|^2))
template <int DIM>
__device__ __forceinline__ void normalize_rcp(float* v) {
  float inv = 1.0f / __builtin_sqrtf(dotv<DIM>(v, v));
  for (int k = 0; k < DIM; k++) v[k] = v[k] * inv;
}

// ---------------------------------------------------------------------------
// geometry queries (brute force over LDS / global arrays)
// ---------------------------------------------------------------------------

// wide closest point on a segment (wide_query_operations.h:121-141)
template <int DIM>
__device__ __forceinline__ float cp_segment(const float* pa, const float* pb, const float* x, float* pt, float* t) {
  float u[DIM], v[DIM];
  for (int k = 0; k < DIM; k++) { u[k] = pb[k] - pa[k]; v[k] = x[k] - pa[k]; }
  float c1 = dotv<DIM>(u, v), c2 = dotv<DIM>(u, u);
  float tt = c1 * (1.0f / c2);
  if (c1 <= 0.0f) tt = 0.0f;
  if (c2 <= c1) tt = 1.0f;
  float d[DIM];
  for (int k = 0; k < DIM; k++) { pt[k] = pa[k] + u[k] * tt; d[k] = x[k] - pt[k]; }
  *t = tt;
  return normv<DIM>(d);
}

// wide closest point on a triangle (wide_query_operations.h:144-235)
__device__ __forceinline__ float cp_triangle(const float* pa, const float* pb, const float* pc, const float* x,
                                             float* pt, float* t0, float* t1) {
  float ab[3], ac[3], ax[3], d[3];
  for (int k = 0; k < 3; k++) { ab[k] = pb[k] - pa[k]; ac[k] = pc[k] - pa[k]; ax[k] = x[k] - pa[k]; }
  float d1 = dotv<3>(ab, ax), d2 = dotv<3>(ac, ax);
  if (d1 <= 0.0f && d2 <= 0.0f) {
    for (int k = 0; k < 3; k++) { pt[k] = pa[k]; d[k] = x[k] - pt[k]; }
    *t0 = 1.0f; *t1 = 0.0f; return normv<3>(d);
  }
  float bx[3]; for (int k = 0; k < 3; k++) bx[k] = x[k] - pb[k];
  float d3 = dotv<3>(ab, bx), d4 = dotv<3>(ac, bx);
  if (d3 >= 0.0f && d4 <= d3) {
    for (int k = 0; k < 3; k++) { pt[k] = pb[k]; d[k] = x[k] - pt[k]; }
    *t0 = 0.0f; *t1 = 1.0f; return normv<3>(d);
  }
  float cx[3]; for (int k = 0; k < 3; k++) cx[k] = x[k] - pc[k];
  float d5 = dotv<3>(ab, cx), d6 = dotv<3>(ac, cx);
  if (d6 >= 0.0f && d5 <= d6) {
    for (int k = 0; k < 3; k++) { pt[k] = pc[k]; d[k] = x[k] - pt[k]; }
    *t0 = 0.0f; *t1 = 0.0f; return normv<3>(d);
  }
  float vc = d1 * d4 - d3 * d2;
  if (vc <= 0.0f && d1 >= 0.0f && d3 <= 0.0f) {
    float v = d1 * (1.0f / (d1 - d3));
    for (int k = 0; k < 3; k++) { pt[k] = pa[k] + ab[k] * v; d[k] = x[k] - pt[k]; }
    *t0 = 1.0f - v; *t1 = v; return normv<3>(d);
  }
  float vb = d5 * d2 - d1 * d6;
  if (vb <= 0.0f && d2 >= 0.0f && d6 <= 0.0f) {
    float w = d2 * (1.0f / (d2 - d6));
    for (int k = 0; k < 3; k++) { pt[k] = pa[k] + ac[k] * w; d[k] = x[k] - pt[k]; }
    *t0 = 1.0f - w; *t1 = 0.0f; return normv<3>(d);
  }
  float va = d3 * d6 - d5 * d4;
  if (va <= 0.0f && (d4 - d3) >= 0.0f && (d5 - d6) >= 0.0f) {
    float w = (d4 - d3) * (1.0f / ((d4 - d3) + (d5 - d6)));
    for (int k = 0; k < 3; k++) { pt[k] = pb[k] + (pc[k] - pb[k]) * w; d[k] = x[k] - pt[k]; }
    *t0 = 0.0f; *t1 = 1.0f - w; return normv<3>(d);
  }
  float denom = 1.0f / (va + vb + vc);
  float v = vb * denom, w = vc * denom;
  for (int k = 0; k < 3; k++) { pt[k] = pa[k] + ab[k] * v + ac[k] * w; d[k] = x[k] - pt[k]; }
  *t0 = 1.0f - v - w; *t1 = v;
  return normv<3>(d);
}

// closest point on a 2D segment record [pa | u = pb - pa] (same arithmetic as cp_segment)
__device__ __forceinline__ float cp_segment_rec(const float* P, const float* x, float* pt, float* t) {
  float u0 = P[2], u1 = P[3];
  float v0 = x[0] - P[0], v1 = x[1] - P[1];
  float c1 = u0 * v0 + u1 * v1, c2 = u0 * u0 + u1 * u1;
  float tt = c1 * (1.0f / c2);
  if (c1 <= 0.0f) tt = 0.0f;
  if (c2 <= c1) tt = 1.0f;
  pt[0] = P[0] + u0 * tt; pt[1] = P[1] + u1 * tt;
  float d0 = x[0] - pt[0], d1 = x[1] - pt[1];
  *t = tt;
  return __builtin_sqrtf(d0 * d0 + d1 * d1);
}

template <int DIM>
__device__ __forceinline__ float cp_prim(const float* P, const float* x, float* pt, float* t0, float* t1) {
  if constexpr (DIM == 2) { *t1 = 0.0f; return cp_segment_rec(P, x, pt, t0); }
  else return cp_triangle(P, P + 3, P + 6, x, pt, t0, t1);
}

// Squared distance from x to a padded group box: below the computed distance of
// every member (the padding dwarfs the rounding of both), so skipping a group whose
// bound exceeds the running minimum never skips the scan's result.
template <int DIM>
__device__ __forceinline__ float box_dist2(const float* B, const float* x) {
  float d2 = 0.0f;
  for (int k = 0; k < DIM; k++) {
    const float e = smax(smax(B[k] - x[k], x[k] - B[4 + k]), 0.0f);
    d2 += e * e;
  }
  return d2;
}

struct Closest { float d; float p[3]; float t0, t1; int prim; };

// Closest point by ONE lane (the point-setup kernel: one point per lane), key fl(d*d),
// last index among equal keys (the reference's `<=` scan, baseline.inl:60-260).  The
// group of the smallest box bound is evaluated first for a running minimum when
// there are many groups, then every group whose bound does not exceed it; the
// update rule (smaller fl(d*d), or equal and a larger index) makes the result the
// brute-force one whatever the visiting order.
template <int DIM>
__device__ Closest closest_lane(const float* prims, const float* groups, int np, int ng, const float* x,
                                int sub = 0, int nsub = 1) {
  constexpr int PS = Layout<DIM>::prim;
  float bk = kFltMax;
  int bi = -1;
  const auto scan = [&](int g) {
    const int p1 = (g + 1) * kGroup < np ? (g + 1) * kGroup : np;
    for (int p = g * kGroup; p < p1; p++) {
      float pt[DIM], t0, t1;
      const float d = cp_prim<DIM>(prims + p * PS, x, pt, &t0, &t1);
      const float d2 = d * d;
      if (d2 < bk || (d2 == bk && p > bi)) { bk = d2; bi = p; }
    }
  };
  if (ng <= 16) {  // small meshes: every primitive (lane `sub` of nsub: every nsub-th one)
    for (int p = sub; p < np; p += nsub) {
      float pt[DIM], t0, t1;
      const float d = cp_prim<DIM>(prims + p * PS, x, pt, &t0, &t1);
      const float d2 = d * d;
      if (d2 <= bk) { bk = d2; bi = p; }
    }
    // the nsub lanes of a point are adjacent (nsub a power of two): min fl(d*d), larger index on ties
    for (int off = 1; off < nsub; off <<= 1) {
      const float ok = __shfl_xor(bk, off);
      const int oi = __shfl_xor(bi, off);
      if (ok < bk || (ok == bk && oi > bi)) { bk = ok; bi = oi; }
    }
    ng = 0;
  } else {
    float lbm = kFltMax;
    int gm = 0;
    for (int g = 0; g < ng; g++) {
      const float lb = box_dist2<DIM>(groups + g * kGroupStride, x);
      if (lb < lbm) { lbm = lb; gm = g; }
    }
    scan(gm);
  }
  for (int g = 0; g < ng; g++) {
    if (box_dist2<DIM>(groups + g * kGroupStride, x) > bk) continue;
    scan(g);
  }
  Closest c; c.prim = bi; c.d = kFltMax; c.t0 = c.t1 = 0.0f;
  c.p[0] = c.p[1] = c.p[2] = 0.0f;
  if (bi >= 0) c.d = cp_prim<DIM>(prims + bi * PS, x, c.p, &c.t0, &c.t1);
  return c;
}

// Interaction::computeNormal via normal(uv) (line_segments.inl:57-73, triangles.inl:61-89)
template <int DIM>
__device__ __forceinline__ void closest_normal(const float* aux, const Closest& c, float* n) {
  constexpr int AS = Layout<DIM>::aux;
  const float* A = aux + c.prim * AS;
  if constexpr (DIM == 2) {
    const float* src = (c.t0 <= kFltEps) ? A : (c.t0 >= 1.0f - kFltEps) ? A + 2 : A + 4;
    n[0] = src[0]; n[1] = src[1];
  } else {
    float u0 = c.t0, u1 = c.t1;
    int vI = -1, eI = -1;
    if (u0 >= 1.0f - kFltEps && u1 <= kFltEps) vI = 0;
    else if (u0 <= kFltEps && u1 >= 1.0f - kFltEps) vI = 1;
    else if (u0 <= kFltEps && u1 <= kFltEps) vI = 2;
    if (vI == -1) {
      if (u0 <= kFltEps) eI = 1;
      else if (u1 <= kFltEps) eI = 2;
      else if (u0 + u1 >= 1.0f - kFltEps) eI = 0;
    }
    const float* src = vI >= 0 ? A + 3 * vI : eI >= 0 ? A + 9 + 3 * eI : A + 18;
    n[0] = src[0]; n[1] = src[1]; n[2] = src[2];
  }
}

template <int DIM>
__device__ __forceinline__ float signed_dist(const float* aux, const Closest& c, const float* x) {
  float n[DIM], d[DIM];
  closest_normal<DIM>(aux, c, n);
  for (int k = 0; k < DIM; k++) d[k] = x[k] - c.p[k];
  return (dotv<DIM>(d, n) > 0.0f ? 1.0f : -1.0f) * c.d;
}

// computeDistToDirichlet without Dirichlet geometry: far bbox corner
// (fcpw_scene_loader.h:312-314, bounding_volumes.h:64-69)
template <int DIM>
__device__ __forceinline__ float bbox_far_dist(const DevScene& sc, const float* x) {
  float m[DIM];
  for (int k = 0; k < DIM; k++) m[k] = smin(sc.pmin[k] - x[k], x[k] - sc.pmax[k]);
  return __builtin_sqrtf(dotv<DIM>(m, m));
}

// ---------------------------------------------------------------------------
// Implicit 8-ary tree over a group array (DevTree, wos_scene.h).  A cursor (L, i)
// walks it depth-first in increasing group order without a stack: the siblings of
// node (L, i) are the aligned block 8 (i / 8) .. + 7 of level L, its parent is
// (L + 1, i / 8) and its children (L - 1, 8 i ..).  L = -1: done.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int tree_count(const DevTree& t, int L) {
  int v = t.n[0];
#pragma unroll
  for (int l = 1; l <= kTreeLevels; l++) v = L == l ? t.n[l] : v;
  return v;
}

__device__ __forceinline__ const float* tree_node(const DevTree& t, int L, int i) {
  int off = 0;
#pragma unroll
  for (int l = 1; l <= kTreeLevels; l++) off = L == l ? t.off[l] : off;
  return t.node + (size_t)(off + i) * kGroupStride;
}

// the first group of node (L, i)
__device__ __forceinline__ int tree_first(int L, int i) { return i << (3 * L); }

// Advances the cursor to the next group g < limit accepted by leaf_ok(g) inside
// subtrees whose boxes node_ok(box) accepts; returns g, or -1 with the cursor parked
// at the first node starting at or beyond `limit` (or done).
template <class NodeOk, class LeafOk>
__device__ __forceinline__ int tree_next(const DevTree& t, int& L, int& i, int limit, NodeOk node_ok,
                                         LeafOk leaf_ok) {
  const int top = t.levels;
  while (L >= 0) {
    if (tree_first(L, i) >= limit) return -1;
    const bool ok = L == 0 ? leaf_ok(i) : node_ok(tree_node(t, L, i));
    if (ok && L > 0) { L--; i <<= 3; continue; }
    const int found = ok ? i : -1;
    i++;
    while (L < top && ((i & 7) == 0 || i >= tree_count(t, L))) { i = ((i - 1) >> 3) + 1; L++; }
    if (L == top && i >= tree_count(t, L)) L = -1;
    if (found >= 0) return found;
  }
  return -1;
}

__device__ __forceinline__ int wave_min_int(int v) {
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const int o = __shfl_xor(v, off);
    v = o < v ? o : v;
  }
  return v;
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(v, off);
    v = o < v ? o : v;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)v, off);
    v = o < v ? o : v;
  }
  return v;
}

// Wave minima through DPP lane moves (VALU, a few cycles each) instead of six ds_bpermute
// round trips (~80 cycles each, tools/mb_latency.hip): within each row of 16 lanes by
// quad swaps and row mirrors, then across rows with row_bcast:15 / row_bcast:31, the
// result in lane 63.  A source lane outside the row mask keeps the destination's own
// value, which leaves a minimum unchanged.  Needs every lane active (the solo query
// forms are convergent); otherwise the ds_bpermute butterfly above.
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROWS, 0xF, false);
}
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ void dpp_min_step(uint32_t& hi, uint32_t& lo) {
  const uint32_t nh = dpp_u32<CTRL, ROWS>(hi), nl = dpp_u32<CTRL, ROWS>(lo);
  const bool take = (((unsigned long long)nh << 32) | nl) < (((unsigned long long)hi << 32) | lo);
  hi = take ? nh : hi;
  lo = take ? nl : lo;
}
__device__ __forceinline__ unsigned long long wave_min_u64_solo(unsigned long long v) {
  if (__builtin_amdgcn_read_exec() != ~0ull) return wave_min_u64(v);
  uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
  dpp_min_step<0xB1>(hi, lo);        // quad_perm [1, 0, 3, 2]
  dpp_min_step<0x4E>(hi, lo);        // quad_perm [2, 3, 0, 1]
  dpp_min_step<0x141>(hi, lo);       // row_half_mirror
  dpp_min_step<0x140>(hi, lo);       // row_mirror: every lane holds its row's minimum
  dpp_min_step<0x142, 0xA>(hi, lo);  // row_bcast:15 into rows 1 and 3
  dpp_min_step<0x143, 0xC>(hi, lo);  // row_bcast:31 into rows 2 and 3
  return ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)hi, 63) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
}
__device__ __forceinline__ uint32_t wave_min_u32_solo(uint32_t v) {
  if (__builtin_amdgcn_read_exec() != ~0ull) return wave_min_u32(v);
  v = min(v, dpp_u32<0xB1>(v));
  v = min(v, dpp_u32<0x4E>(v));
  v = min(v, dpp_u32<0x141>(v));
  v = min(v, dpp_u32<0x140>(v));
  v = min(v, dpp_u32<0x142, 0xA>(v));
  v = min(v, dpp_u32<0x143, 0xC>(v));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Inclusive prefix sum over the wave: in-row shifts by 1, 2, 4, 8 (DPP row_shr, zero from
// outside the row), then row 15's / row 31's sums broadcast into the following rows
// (row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3) -- six VALU adds instead
// of six ds_bpermute round trips (≈ 80 cycles each).  Needs the full exec mask (as the
// cooperative queries have); otherwise the shuffle form.
__device__ __forceinline__ uint32_t wave_incl_sum_u32(uint32_t v, int lane) {
  if (__builtin_amdgcn_read_exec() == ~0ull) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return v;
  }
  for (int dlt = 1; dlt < kWave; dlt <<= 1) {
    const uint32_t u = __shfl_up(v, dlt);
    if (lane >= dlt) v += u;
  }
  return v;
}
// lane 63's value (the total of an inclusive sum), wave-uniform
__device__ __forceinline__ uint32_t wave_last_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, kWave - 1);
}

// a lane's float value, wave-uniform
__device__ __forceinline__ float lane_bcast(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// computeDistToDirichlet (fcpw_scene_loader.h:299-315) over the Dirichlet
// primitives, groups of kGroup culled by their boxes.  The sequential `<=` scan
// returns d of the highest-index primitive attaining the minimum computed d^2;
// here the group with the smallest box bound is evaluated first (a tight running
// minimum), then every other group whose bound does not exceed it, keeping
// (min d^2, highest index) -- the same primitive, hence the same d.
//
// PROJ = true also returns that primitive's closest point in proj[DIM]: projectToDirichlet
// (fcpw_scene_loader.h:345-364) runs the same findClosestPoint scan.
template <int DIM, bool PROJ = false>
__device__ float dirichlet_dist_culled(const DevScene& sc, const float* dprim, const float* dgroup,
                                       const float* x, float* proj = nullptr) {
  if (sc.n_dprims <= 0) return bbox_far_dist<DIM>(sc, x);
  constexpr int PS = Layout<DIM>::prim;
  const int ng = sc.n_dgroups;
  if (sc.dtree.levels > 0) {
    // hierarchy: the greedy descent to the nearest-bound leaf gives a tight running
    // minimum, then the depth-first walk visits every group whose bound does not
    // exceed it (re-visiting that leaf changes nothing): the same primitive
    const DevTree& T = sc.dtree;
    float sr2 = kFltMax, best = kFltMax;
    int bestp = -1;
    auto eval_group = [&](int gi) {
      const int p1 = (gi + 1) * kGroup < sc.n_dprims ? (gi + 1) * kGroup : sc.n_dprims;
      for (int p = gi * kGroup; p < p1; p++) {
        float pt[DIM], t0, t1;
        const float d = cp_prim<DIM>(dprim + p * PS, x, pt, &t0, &t1);
        const float d2 = d * d;
        if (d2 < sr2 || (d2 == sr2 && p > bestp)) {
          sr2 = d2; best = d; bestp = p;
          if constexpr (PROJ) for (int k = 0; k < DIM; k++) proj[k] = pt[k];
        }
      }
    };
    {
      int L = T.levels, i0 = 0;
      while (true) {
        const int n = tree_count(T, L), i1 = (i0 + 8) < n ? i0 + 8 : n;
        int bi = i0;
        float bl = kFltMax;
        for (int i = i0; i < i1; i++) {
          const float lb = box_dist2<DIM>(L == 0 ? dgroup + i * kGroupStride : tree_node(T, L, i), x);
          if (lb < bl) { bl = lb; bi = i; }
        }
        if (L == 0) { eval_group(bi); break; }
        L--;
        i0 = bi << 3;
      }
    }
    int L = T.levels, i = 0;
    while (L >= 0) {
      const int g = tree_next(T, L, i, 0x7FFFFFFF,
                              [&](const float* B) { return !(box_dist2<DIM>(B, x) > sr2); },
                              [&](int gi) { return !(box_dist2<DIM>(dgroup + gi * kGroupStride, x) > sr2); });
      if (g >= 0) eval_group(g);
    }
    return best;
  }
  int g0 = 0;
  float lb0 = kFltMax;
  for (int gi = 0; gi < ng; gi++) {
    const float lb = box_dist2<DIM>(dgroup + gi * kGroupStride, x);
    if (lb < lb0) { lb0 = lb; g0 = gi; }
  }
  float sr2 = kFltMax, best = kFltMax;
  int bestp = -1;
  for (int k = 0; k < ng; k++) {
    const int gi = k == 0 ? g0 : (k <= g0 ? k - 1 : k);
    if (k > 0 && box_dist2<DIM>(dgroup + gi * kGroupStride, x) > sr2) continue;
    const int p1 = (gi + 1) * kGroup < sc.n_dprims ? (gi + 1) * kGroup : sc.n_dprims;
    for (int p = gi * kGroup; p < p1; p++) {
      float pt[DIM], t0, t1;
      const float d = cp_prim<DIM>(dprim + p * PS, x, pt, &t0, &t1);
      const float d2 = d * d;
      if (d2 < sr2 || (d2 == sr2 && p > bestp)) {
        sr2 = d2; best = d; bestp = p;
        if constexpr (PROJ) for (int k = 0; k < DIM; k++) proj[k] = pt[k];
      }
    }
  }
  return best;
}

template <int DIM>
__device__ float dirichlet_dist_lane(const DevScene& sc, const float* x) {
  if (sc.n_dprims <= 0) return bbox_far_dist<DIM>(sc, x);
  constexpr int PS = Layout<DIM>::prim;
  float sr2 = kFltMax, best = kFltMax;
  for (int p = 0; p < sc.n_dprims; p++) {
    float pt[DIM], t0, t1;
    float d = cp_prim<DIM>(sc.dprim + p * PS, x, pt, &t0, &t1);
    float d2 = d * d;
    if (d2 <= sr2) { sr2 = d2; best = d; }
  }
  return best;
}

// computeDistToDirichlet through the Dirichlet cell grid (2D, DevScene::dgrid): the
// segments of x's cell list in index order with the full scan's `<=` rule -- the full
// scan's distance (wos_host_scene.h DirGrid).  Returns a negative value when x lies
// outside the grid (the caller scans).
template <int DIM>
__device__ __forceinline__ float dirichlet_dist_grid(const DevScene& sc, const float* dprim, const float* x) {
  if constexpr (DIM != 2) {
    return -1.0f;
  } else {
    int c = 0;
    for (int k = 1; k >= 0; k--) {
      const int nk = sc.dgrid_n[k];
      const float v = (x[k] - sc.dgrid_min[k]) * sc.dgrid_inv[k];
      if (!(v >= 0.0f && v < (float)nk)) return -1.0f;
      int i = (int)v;
      if (i > nk - 1) i = nk - 1;
      c = c * nk + i;
    }
    const uint32_t b = sc.dgrid[c], e = sc.dgrid[c + 1];
    const uint16_t* lst = reinterpret_cast<const uint16_t*>(sc.dgrid + sc.dgrid_off_words);
    float sr2 = kFltMax, best = kFltMax;
    for (uint32_t i = b; i < e; i++) {
      const int p = (int)lst[i];
      float pt[2], t0, t1;
      const float d = cp_prim<2>(dprim + p * kPrimStride2, x, pt, &t0, &t1);
      const float d2 = d * d;
      if (d2 <= sr2) { sr2 = d2; best = d; }
    }
    return best;
  }
}

// computeDistToDirichlet for ONE querying lane of the wave (a lone walk), wave-cooperative:
// the group with the smallest box bound is evaluated first (kGroup lanes) for a running
// bound, then the primitives of every group whose bound does not exceed it, kGroup lanes
// per group; (fl(d*d), larger index on ties) minima by wave reductions, and the winner's
// distance from the same cp_prim -- dirichlet_dist_culled's value (a primitive with
// d^2 <= the bound lies in a group whose bound is <= d^2: never skipped).  Convergent.
template <int DIM>
__device__ __forceinline__ float dirichlet_dist_solo(const DevScene& sc, const float* dprim, const float* dgroup,
                                                     const float* xo, int lane) {
  constexpr int PS = Layout<DIM>::prim;
  const int ng = sc.n_dgroups, np = sc.n_dprims;
  unsigned long long gk = ~0ull;
  for (int g = lane; g < ng; g += kWave) {
    const unsigned long long k =
        ((unsigned long long)__float_as_uint(box_dist2<DIM>(dgroup + g * kGroupStride, xo)) << 32) | (uint32_t)g;
    gk = k < gk ? k : gk;
  }
  const int g0 = (int)(uint32_t)wave_min_u64_solo(gk);
  unsigned long long best = ~0ull;
  auto eval = [&](int p) {
    float pt[DIM], t0, t1;
    const float d = cp_prim<DIM>(dprim + p * PS, xo, pt, &t0, &t1);
    const unsigned long long k = ((unsigned long long)__float_as_uint(d * d) << 32) | (0xFFFFFFFFu - (uint32_t)p);
    best = k < best ? k : best;
  };
  if (lane < kGroup && g0 * kGroup + lane < np) eval(g0 * kGroup + lane);
  best = wave_min_u64_solo(best);
  const float sr2 = __uint_as_float((uint32_t)(best >> 32));
  for (int w0 = 0; w0 < ng; w0 += kWave) {
    const int g = w0 + lane;
    uint64_t pm = __ballot(g < ng && g != g0 && !(box_dist2<DIM>(dgroup + g * kGroupStride, xo) > sr2));
    while (pm != 0) {
      // lanes [kGroup q, kGroup (q + 1)) take the q-th group of the mask
      uint64_t mm = pm;
      for (int q = lane / kGroup; q > 0 && mm != 0; q--) mm &= mm - 1;
      for (int q = 0; q < kWave / kGroup && pm != 0; q++) pm &= pm - 1;
      if (mm != 0) {
        const int p = (w0 + __builtin_ctzll(mm)) * kGroup + (lane & (kGroup - 1));
        if (p < np) eval(p);
      }
    }
  }
  best = wave_min_u64_solo(best);
  const int pw = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull));
  float pt[DIM], t0, t1;
  return cp_prim<DIM>(dprim + pw * PS, xo, pt, &t0, &t1);
}

struct Hit { float p[3], n[3], d; };

// Exact ray-primitive test of the reference (mbvh.inl:521-609 + wide_query_operations.h
// 27-92, line_segments.inl / triangles.inl ray queries): accepts when the hit
// distance d satisfies 0 <= d <= rt and then shrinks rt to d.  Visiting primitives
// in index order this yields the minimum d, ties going to the larger index.
template <int DIM>
__device__ __forceinline__ bool ray_prim_exact(const float* P, const float* o, const float* dir, float& rt, Hit* h) {
  if constexpr (DIM == 2) {
    float u0 = P[0] - o[0], u1 = P[1] - o[1];
    float v0 = P[2], v1 = P[3];  // record holds v = pb - pa
    float dv = dir[0] * v1 - dir[1] * v0;
    if (!(__builtin_fabsf(dv) > kFltEps)) return false;
    float ud = u0 * dir[1] - u1 * dir[0];
    float uv = u0 * v1 - u1 * v0;
    float inv = 1.0f / dv;
    float t = ud * inv;
    if (!(t >= 0.0f && t <= 1.0f)) return false;
    float d = uv * inv;
    if (!(d >= 0.0f && d <= rt)) return false;
    rt = d;
    h->d = d;
    h->p[0] = P[0] + t * v0; h->p[1] = P[1] + t * v1;
    h->n[0] = v1; h->n[1] = -v0;
    return true;
  } else {
    float v1[3], v2[3], pp[3], s[3], q[3];
    for (int k = 0; k < 3; k++) { v1[k] = P[3 + k] - P[k]; v2[k] = P[6 + k] - P[k]; s[k] = o[k] - P[k]; }
    cross3(pp, dir, v2);
    float det = dotv<3>(v1, pp);
    if (!(__builtin_fabsf(det) > kFltEps)) return false;
    float inv = 1.0f / det;
    float v = dotv<3>(s, pp) * inv;
    if (!(v >= 0.0f && v <= 1.0f)) return false;
    cross3(q, s, v1);
    float w = dotv<3>(dir, q) * inv;
    if (!(w >= 0.0f && v + w <= 1.0f)) return false;
    float d = dotv<3>(v2, q) * inv;
    if (!(d >= 0.0f && d <= rt)) return false;
    rt = d;
    h->d = d;
    for (int k = 0; k < 3; k++) h->p[k] = P[k] + v1[k] * v + v2[k] * w;
    cross3(h->n, v1, v2);
    return true;
  }
}

template <int DIM>
__device__ __forceinline__ bool ray_hit_scan(const float* prims, int np, const float* o, const float* dir,
                                             float tmax, Hit* h) {
  constexpr int PS = Layout<DIM>::prim;
  bool found = false;
  float rt = tmax;
  for (int p = 0; p < np; p++) found |= ray_prim_exact<DIM>(prims + p * PS, o, dir, rt, h);
  if (found) normalize_rcp<DIM>(h->n);
  return found;
}

// Geometry as staged in LDS: primitives, silhouette candidates and the culling
// boxes of kGroup consecutive primitives / silhouettes.
struct LGeom {
  const float* prim;
  const float* sil;
  const float* pgroup;
  const float* sgroup;
  const uint32_t* sgrid;  // star-radius cell grid (u16 offsets | u8 lists), nullptr if none
  int sgrid_off_words;
  const float* dprim;     // Dirichlet primitives + their culling boxes (walk kernel)
  const float* dgroup;
};

// Certain rejection of a whole group for a ray segment [o, o + rt*dir]: slab
// test against the group's padded box.  The padding (1e-4 of the scene span)
// dwarfs the rounding of the slab arithmetic, so a group whose primitives the
// exact test could hit within rt is never skipped.  rcp(0) = inf and NaN slabs
// (origin exactly on a padded face) fall out of min/max, which only errs
// toward visiting.
template <int DIM>
__device__ __forceinline__ bool ray_box_maybe(const float* B, const float* o, const float* inv, float rt) {
  float tn = -kFltMax, tf = kFltMax;
  for (int k = 0; k < DIM; k++) {
    const float t1 = (B[k] - o[k]) * inv[k], t2 = (B[4 + k] - o[k]) * inv[k];
    tn = __builtin_fmaxf(tn, __builtin_fminf(t1, t2));
    tf = __builtin_fminf(tf, __builtin_fmaxf(t1, t2));
  }
  return tn <= tf && tf >= 0.0f && tn <= rt * 1.00001f + 1e-6f;
}

// First ray hit within tmax (mbvh.inl:521-609 + wide_query_operations.h:27-92)
// in index order: min d, ties to the larger index.  Groups of primitives the
// ray cannot reach are skipped (for the whole wave when no lane needs them);
// inside a group every primitive first goes through a division-free
// certain-rejection test using the hardware reciprocal (v_rcp_f32, |rel err| <=
// 2^-22; signs exact, magnitudes with a 1e-5 relative margin), so only
// primitives the exact test could accept reach the IEEE division.  Skipped
// groups and pre-filtered primitives are exactly those the plain loop rejects,
// so the result and every computed value equal the plain loop's (and the
// oracle's).
template <int DIM>
__device__ __forceinline__ bool ray_hit(const LGeom& G, int np, int ng, const float* o, const float* dir,
                                        float tmax, Hit* h) {
  constexpr int PS = Layout<DIM>::prim;
  float inv[DIM];
  for (int k = 0; k < DIM; k++) inv[k] = __builtin_amdgcn_rcpf(dir[k]);
  bool found = false;
  float rt = tmax;
  for (int gi = 0; gi < ng; gi++) {
    if (!ray_box_maybe<DIM>(G.pgroup + gi * kGroupStride, o, inv, rt)) continue;
    const int p1 = (gi + 1) * kGroup < np ? (gi + 1) * kGroup : np;
    for (int p = gi * kGroup; p < p1; p++) {
      const float* P = G.prim + p * PS;
      if constexpr (DIM == 2) {
        const float u0 = P[0] - o[0], u1 = P[1] - o[1];
        const float v0 = P[2], v1 = P[3];
        const float dv = dir[0] * v1 - dir[1] * v0;
        if (!(__builtin_fabsf(dv) > kFltEps)) continue;
        const float ud = u0 * dir[1] - u1 * dir[0];
        const float uv = u0 * v1 - u1 * v0;
        const float ra = __builtin_amdgcn_rcpf(dv);
        const float ta = ud * ra, da = uv * ra;
        if ((ta < 0.0f && __builtin_fabsf(ud) > 1e-30f) || ta > 1.00001f ||
            (da < 0.0f && __builtin_fabsf(uv) > 1e-30f) || da > rt * 1.00001f)
          continue;
      } else {
        float v1[3], v2[3], pp[3], sv[3], q[3];
        for (int k = 0; k < 3; k++) { v1[k] = P[3 + k] - P[k]; v2[k] = P[6 + k] - P[k]; sv[k] = o[k] - P[k]; }
        cross3(pp, dir, v2);
        const float det = dotv<3>(v1, pp);
        if (!(__builtin_fabsf(det) > kFltEps)) continue;
        const float ra = __builtin_amdgcn_rcpf(det);
        const float vn = dotv<3>(sv, pp), va = vn * ra;
        if ((va < 0.0f && __builtin_fabsf(vn) > 1e-30f) || va > 1.00001f) continue;
        cross3(q, sv, v1);
        const float wn = dotv<3>(dir, q), dn = dotv<3>(v2, q);
        const float wa = wn * ra, da = dn * ra;
        if ((wa < 0.0f && __builtin_fabsf(wn) > 1e-30f) || va + wa > 1.00002f ||
            (da < 0.0f && __builtin_fabsf(dn) > 1e-30f) || da > rt * 1.00001f)
          continue;
      }
      found |= ray_prim_exact<DIM>(P, o, dir, rt, h);
    }
  }
  if (found) normalize_rcp<DIM>(h->n);
  return found;
}

// occlusion-only ray test (hasLineOfSight, primitive.h:225-235)
template <int DIM>
__device__ bool ray_occluded(const float* prims, int np, const float* o, const float* dir, float tmax) {
  Hit h;
  return ray_hit_scan<DIM>(prims, np, o, dir, tmax, &h);
}

// isWideSilhouetteVertex / isWideSilhouetteEdge (wide_query_operations.h:328-395)
template <int DIM>
__device__ __forceinline__ bool is_silhouette(const float* S, const float* view, float d, bool flip, float prec) {
  float sign = flip ? 1.0f : -1.0f;
  const float* n0 = DIM == 2 ? S + 2 : S + 6;
  const float* n1 = DIM == 2 ? S + 4 : S + 9;
  if (!(d > prec)) {
    if constexpr (DIM == 2) {
      float det = n0[0] * n1[1] - n0[1] * n1[0];
      return sign * det > prec;
    } else {
      float ed[3], c[3];
      for (int k = 0; k < 3; k++) ed[k] = S[3 + k] - S[k];
      normalize_rcp<3>(ed);
      cross3(c, n0, n1);
      float ang = fatan2(dotv<3>(ed, c), dotv<3>(n0, n1));
      return sign * ang > prec;
    }
  }
  float inv = 1.0f / d;
  float u[DIM];
  for (int k = 0; k < DIM; k++) u[k] = view[k] * inv;
  float dot0 = dotv<DIM>(u, n0), dot1 = dotv<DIM>(u, n1);
  if (__builtin_fabsf(dot0) <= prec) return sign * dot1 > prec;
  if (__builtin_fabsf(dot1) <= prec) return sign * dot0 > prec;
  return dot0 * dot1 < 0.0f;
}

// isWideSilhouetteVertex without the division and square root: the view
// direction is normalised with the hardware rsq, whose error (with the dot-product
// rounding) stays below 1e-6 on the unit-scale dots, so outside a 1e-5 band
// around every threshold the decision equals the exact test's.  Returns 1/0 when
// certain, 2 when the exact test must decide.  (2D vertex candidates.)
__device__ __forceinline__ int silhouette_class2(const float* S, const float* view, float d2raw, bool flip,
                                                 float prec) {
  const float sign = flip ? 1.0f : -1.0f;
  const float* n0 = S + 2;
  const float* n1 = S + 4;
  const float p2 = prec * prec;
  if (d2raw < p2 * 0.9999f) {  // certainly d <= prec: the exact test's normal-only branch
    const float det = n0[0] * n1[1] - n0[1] * n1[0];
    return sign * det > prec ? 1 : 0;
  }
  if (d2raw <= p2 * 1.0001f) return 2;
  const float r = __builtin_amdgcn_rsqf(d2raw);
  const float dot0 = (view[0] * n0[0] + view[1] * n0[1]) * r;
  const float dot1 = (view[0] * n1[0] + view[1] * n1[1]) * r;
  const float tol = 1e-5f;
  const float a0 = __builtin_fabsf(dot0), a1 = __builtin_fabsf(dot1);
  float v;
  if (a0 < prec - tol) {
    v = sign * dot1;
  } else if (a0 > prec + tol) {
    if (a1 > prec + tol) return dot0 * dot1 < 0.0f ? 1 : 0;
    if (!(a1 < prec - tol)) return 2;
    v = sign * dot0;
  } else {
    return 2;
  }
  return v > prec + tol ? 1 : (v < prec - tol ? 0 : 2);
}

// Certain rejection of a whole silhouette group: the squared distance from x to
// the group's padded box exceeds r2 (with margin), so every candidate in it is
// rejected by the exact distance test too.
template <int DIM>
__device__ __forceinline__ bool ball_box_maybe(const float* B, const float* x, float r2) {
  float d2 = 0.0f;
  for (int k = 0; k < DIM; k++) {
    const float e = __builtin_fmaxf(__builtin_fmaxf(B[k] - x[k], x[k] - B[4 + k]), 0.0f);
    d2 += e * e;
  }
  return !(d2 > r2 * 1.00001f);
}

// Certain absence of silhouettes in a group, from the normal cone (axis a,
// half-angle alpha) and the view cone of x on the group's bounding sphere (axis
// w = x - c, half-angle beta = asin(rho/|w|)): every view direction u and every
// adjacent normal n then satisfy angle(u, n) in [theta - alpha - beta, theta +
// alpha + beta], theta = angle(w, a).  When that interval lies inside
// [0, acos(prec + m)) every dot is > prec + m (all faces front-facing), when it
// lies inside (pi - acos(prec + m), pi] every dot is < -(prec + m): either way the
// exact test (isWideSilhouetteVertex/Edge) rejects every candidate.  m = 1e-3
// dwarfs the error of the rsq/sqrt arithmetic used here.  Groups holding a
// candidate next to a missing primitive, or x within prec of the sphere, are
// never culled.
template <int DIM>
__device__ __forceinline__ bool cone_culled(const float* B, const float* x, float prec) {
  if (B[15] != 0.0f) return false;
  const float rho = B[11];
  float w[DIM];
  for (int k = 0; k < DIM; k++) w[k] = x[k] - B[8 + k];
  const float D2 = dotv<DIM>(w, w);
  const float lim = rho + 1.01f * prec + 1e-6f;
  if (!(D2 > lim * lim)) return false;
  const float invD = __builtin_amdgcn_rsqf(D2);
  const float sinb = rho * invD, cosb = __builtin_amdgcn_sqrtf(smax(0.0f, 1.0f - sinb * sinb));
  const float sina = B[3], cosa = B[7];
  const float cosg = cosa * cosb - sina * sinb, sing = sina * cosb + cosa * sinb;  // gamma = alpha + beta
  float wa = 0.0f;
  for (int k = 0; k < DIM; k++) wa += w[k] * B[12 + k];
  const float cost = smin(smax(wa * invD, -1.0f), 1.0f), sint = __builtin_amdgcn_sqrtf(smax(0.0f, 1.0f - cost * cost));
  const float thr = prec + 1e-3f;
  // front: theta + gamma in (0, pi) and cos(theta + gamma) > thr
  const float c_p = cost * cosg - sint * sing, s_p = sint * cosg + cost * sing;
  if (s_p > 1e-3f && c_p > thr) return true;
  // back: theta - gamma in (0, pi) and cos(theta - gamma) < -thr
  const float c_m = cost * cosg + sint * sing, s_m = sint * cosg - cost * sing;
  return s_m > 1e-3f && c_m < -thr;
}

// computeStarRadius (fcpw_scene_loader.h:621-641): the closest silhouette point
// within maxR, candidates in index order (brute force over the staged records,
// fcpw Baseline semantics); groups out of reach are skipped, 2D candidates are
// classified by silhouette_class2 before any exact square root or division.
template <int DIM>
__device__ __forceinline__ float star_radius(const LGeom& G, int ns, int nsg, int np, const float* x, float minR,
                                             float maxR, float prec, bool flipOrient) {
  constexpr int SS = Layout<DIM>::sil;
  if (minR > maxR) return maxR;
  if (np > 0) {
    bool flip = !flipOrient;
    float r2 = maxR < kFltMax ? maxR * maxR : kFltMax;
    float minR2 = minR * minR;
    bool found = false, done = false;
    float best = 0.0f;
    DIAG_LANE(D_SCALLS);
    if (!(minR2 >= r2)) {
      for (int gi = 0; gi < nsg && !done; gi++) {
        const float* B = G.sgroup + gi * kSGroupStride;
        if (!ball_box_maybe<DIM>(B, x, r2) || cone_culled<DIM>(B, x, prec)) continue;
        DIAG_LANE(D_SGVISIT);
        const int s1 = (gi + 1) * kGroup < ns ? (gi + 1) * kGroup : ns;
        for (int s = gi * kGroup; s < s1; s++) {
          const float* S = G.sil + s * SS;
          const float miss = DIM == 2 ? S[6] : S[12];
          float view[DIM], d;
          int cls = 2;
          if constexpr (DIM == 2) {
            view[0] = x[0] - S[0]; view[1] = x[1] - S[1];
            float d2raw = view[0] * view[0] + view[1] * view[1];
            // certain rejection: fl(fl(sqrt(q))^2) >= q(1 - 2^-22) > r2 (no sqrt needed)
            if (d2raw > r2 * 1.000001f) continue;
            DIAG_LANE(D_SCAND);
            cls = miss != 0.0f ? 1 : silhouette_class2(S, view, d2raw, flip, prec);
            if (cls == 0) continue;  // certainly not a silhouette: the exact loop skips it too
            DIAG_LANE(D_SEXACT);
            d = __builtin_sqrtf(d2raw);
          } else {
            // certain rejection against the edge's bounding sphere before the exact query
            float e[3], hl[3];
            for (int k = 0; k < 3; k++) { e[k] = x[k] - 0.5f * (S[k] + S[3 + k]); hl[k] = 0.5f * (S[3 + k] - S[k]); }
            float dm = __builtin_amdgcn_sqrtf(dotv<3>(e, e)), hr = __builtin_amdgcn_sqrtf(dotv<3>(hl, hl));
            float lo = dm - hr;
            if (lo > 0.0f && lo * lo > r2 * 1.0001f + 1e-6f * dm * dm) continue;
            float pt[3], t;
            d = cp_segment<3>(S, S + 3, x, pt, &t);
            for (int k = 0; k < 3; k++) view[k] = x[k] - pt[k];
            if (miss != 0.0f) cls = 1;
          }
          float d2 = d * d;
          if (d2 > r2) continue;
          bool sil_ok = cls == 1 ? true : is_silhouette<DIM>(S, view, d, flip, prec);
          if (sil_ok && d2 <= r2) {
            r2 = d2; best = d; found = true;
            if (minR2 >= r2) { done = true; break; }
          }
        }
      }
    }
    if (found) return smax(best, minR);
  }
  return smax(maxR, minR);
}

// offsetPointAlongDirection (fcpw_scene_loader.h:258-290)
template <int DIM>
__device__ __forceinline__ void offset_point(const float* p, const float* n, float* out) {
  const float origin = 1.0f / 32.0f, floatScale = 1.0f / 65536.0f, intScale = 256.0f;
  for (int k = 0; k < DIM; k++) {
    int no = cvt_trunc(n[k] * intScale);
    float po = bits_to_float((uint32_t)((int32_t)float_to_bits(p[k]) + (p[k] < 0 ? -no : no)));
    out[k] = __builtin_fabsf(p[k]) < origin ? p[k] + floatScale * n[k] : po;
  }
}

// Cost probes (never shipped; tools/build_variant.sh): WOS_PROBE bit k evaluates one piece of
// the walk step a second time on opaque copies of its inputs, results sunk -- the walks are
// unchanged, so the kernel's SQ_INSTS_VALU and time minus the base build's are that piece's
// dynamic instruction count and cost.  1: update_ball's Bessels (2D), 2: the direction-
// sampled Poisson kernel's Bessels (2D), 4: a cooperative rejection item (draws + fast test),
// 8: the star-radius query, 16: the ray query, 32: the whole source sample (sample_volume_wave).
#ifndef WOS_PROBE
#define WOS_PROBE 0
#endif
template <class T>
__device__ __forceinline__ T probe_opaque(T v) {
  asm volatile("" : "+v"(v));
  return v;
}
template <class T>
__device__ __forceinline__ void probe_sink(T v) {
  asm volatile("" ::"v"(v));
}

// HBM-accounting builds (never shipped, wrong results; tools/build_variant.sh): the walk kernel
// without its source-texel loads (WOS_ACCT_NOTEX) or its record stores (WOS_ACCT_NOREC) -- the
// walks themselves are unchanged -- so differences of the PMC traffic attribute its bytes
#ifndef WOS_ACCT_NOTEX
#define WOS_ACCT_NOTEX 0
#endif
#ifndef WOS_ACCT_NOREC
#define WOS_ACCT_NOREC 0
#endif

// PDE source lookup: scene.h:194-198 + image.h:53-58 (2D), scene_3d.h:120-126 (3D)
template <int DIM>
__device__ __forceinline__ float source_value(const DevScene& sc, const float* x) {
  if (sc.source == nullptr || WOS_ACCT_NOTEX) return 0.0f;
  if constexpr (DIM == 2) {
    float ux = (x[0] - sc.pmin[0]) / sc.ext[0];
    float uy = (x[1] - sc.pmin[1]) / sc.ext[1];
    int h = sc.sdims[0], w = sc.sdims[1];
    int i = sclamp(cvt_trunc(uy * (float)h), 0, h - 1);
    int j = sclamp(cvt_trunc(ux * (float)w), 0, w - 1);
    return sc.source[(size_t)i * w + j];
  } else {
    int X = sc.sdims[0], Y = sc.sdims[1], Z = sc.sdims[2];
    float ux = (x[0] - sc.pmin[0]) / sc.ext[0];
    float uy = (x[1] - sc.pmin[1]) / sc.ext[1];
    float uz = (x[2] - sc.pmin[2]) / sc.ext[2];
    int i = sclamp(cvt_trunc(ux * (float)X), 0, X - 1);
    int j = sclamp(cvt_trunc(uy * (float)Y), 0, Y - 1);
    int k = sclamp(cvt_trunc(uz * (float)Z), 0, Z - 1);
    return sc.source[((size_t)i * Y + j) * Z + k];
  }
}

// g at the position x where a walk reached the Dirichlet shell (setTerminalContribution,
// walk_on_stars.h:331-351): the constant, or -- image-valued data, 2D -- the image over
// sc.dbox at x's projection onto the Dirichlet boundary (projectToDirichlet,
// fcpw_scene_loader.h:345-364), looked up as Image::get (image.h:53-58) with the uv of the
// upstream demo's pde.dirichlet (scene.h:202-207).  Once per walk that reaches the shell.
template <int DIM>
__device__ float dirichlet_value(const DevScene& sc, const float* x) {
  if constexpr (DIM == 2) {
    if (sc.dimg != nullptr && sc.n_dprims > 0) {
      float proj[2] = {x[0], x[1]};
      dirichlet_dist_culled<DIM, true>(sc, sc.dprim, sc.dgroup, x, proj);
      const float ux = (proj[0] - sc.dbox[0]) / sc.dbox[2];
      const float uy = (proj[1] - sc.dbox[1]) / sc.dbox[3];
      const int h = sc.ddims[0], w = sc.ddims[1];
      const int i = sclamp(cvt_trunc(uy * (float)h), 0, h - 1);
      const int j2 = sclamp(cvt_trunc(ux * (float)w), 0, w - 1);
      return sc.dimg[(size_t)i * w + j2];
    }
  }
  return sc.g_dirichlet;
}

// h at a Neumann boundary sample y (walk_on_stars.h:253-256): the upstream demo's pde.neumann
// (scene.h:175-181, commented in the fork: uv = (y - bbox.pMin) / bbox.extent()) over sc.nbox,
// looked up as Image::get (image.h:53-58); 0 without an image (the reference's h, scene.h:176-181)
__device__ __forceinline__ float neumann_value(const DevScene& sc, const float* y) {
  if (sc.nimg == nullptr) return 0.0f;
  const float ux = (y[0] - sc.nbox[0]) / sc.nbox[2];
  const float uy = (y[1] - sc.nbox[1]) / sc.nbox[3];
  const int h = sc.ndims[0], w = sc.ndims[1];
  const int i = sclamp(cvt_trunc(uy * (float)h), 0, h - 1);
  const int j = sclamp(cvt_trunc(ux * (float)w), 0, w - 1);
  return sc.nimg[(size_t)i * w + j];
}

template <int DIM>
__device__ __forceinline__ bool outside_bbox(const DevScene& sc, const float* x) {
  for (int k = 0; k < DIM; k++)
    if (!(x[k] >= sc.pmin[k] && x[k] <= sc.pmax[k])) return true;
  return false;
}

// ---------------------------------------------------------------------------
// Green's functions on balls (distributions.h:273-832)
// ---------------------------------------------------------------------------
// A walk step's source texel is consumed at the next step (or when the walk ends), so its
// global load overlaps the next step's queries instead of stalling the tail (WalkState::pend)
// ---------------------------------------------------------------------------
// Robust float semantics (Gfn::yukawa == kYukScaled): the reference's Yukawa members
// rewritten with exponentially scaled Bessels (bessel_scaled) and e^{2(mu r - mu R)} <= 1,
// in double, rounded where the reference rounds its result -- operation for operation
// as oracle/wos_oracle.c (scaled_q0 and the g->scaled branches).  Out of line: the
// reference-semantics path keeps its registers.
// ---------------------------------------------------------------------------
#define WOS_COLD __device__ __attribute__((noinline))
// 2D K0(mur) - I0(mur) K0(muR)/I0(muR) (a0 = ke0(muR), a1 = ie0(muR));
// 3D e^-mur - e^-muR sinh(mur)/sinh(muR)
template <int DIM>
WOS_COLD double scaled_q0(float mur, float muR, float a0, float a1) {
  const double x = (double)mur, X = (double)muR;
  if constexpr (DIM == 2) {
    double ie0, ke0, ie1, ke1;
    bessel_scaled(x, &ie0, &ke0, &ie1, &ke1);
    return dexp(-x) * (ke0 - ie0 * ((double)a0 / (double)a1) * dexp(2.0 * (x - X)));
  } else {
    return dexp(-x) - dexp(x - 2.0 * X) * (1.0 - dexp(-2.0 * x)) / (1.0 - dexp(-2.0 * X));
  }
}

template <int DIM>
WOS_COLD void scaled_members(float muR, float* a0, float* a1, float* b0, float* b1) {
  double ie0, ke0, ie1, ke1;
  bessel_scaled((double)muR, &ie0, &ke0, &ie1, &ke1);
  *a0 = (float)ke0; *a1 = (float)ie0; *b0 = (float)ke1; *b1 = (float)ie1;
}

template <int DIM>
WOS_COLD float scaled_poisson_kernel(float muR, float a1) {
  const double X = (double)muR;
  if constexpr (DIM == 2) return (float)(dexp(-X) / (kTwoPi * (double)a1));
  else return (float)(X * 2.0 * dexp(-X) / (kFourPi * (1.0 - dexp(-2.0 * X))));
}

template <int DIM>
WOS_COLD float scaled_gradient_norm(float r, float sqrtL, float muR, float b0, float b1) {
  const float mur = r * sqrtL;
  const double x = (double)mur, X = (double)muR, t = dexp(2.0 * (x - X));
  if constexpr (DIM == 2) {
    double ie0, ke0, ie1, ke1;
    bessel_scaled(x, &ie0, &ke0, &ie1, &ke1);
    const double q = dexp(-x) * (ke1 - ie1 * ((double)b0 / (double)b1) * t);
    return (float)((double)sqrtL * q / (kTwoPi * (double)r));
  } else {
    const double q = dexp(-x) * ((1.0 + 1.0 / x) - i32_scaled(x) * ((1.0 + 1.0 / X) / i32_scaled(X)) * t);
    return (float)((double)sqrtL * q / (kFourPi * (double)(r * r)));
  }
}

// QR of the Poisson kernel gradient
template <int DIM>
WOS_COLD float scaled_pk_gradient(float muR, float sqrtL, float lambda, float R, float b1) {
  const double X = (double)muR;
  if constexpr (DIM == 2) return (float)((double)sqrtL * dexp(-X) / ((double)R * (double)b1));
  else return (float)((double)lambda * dexp(-X) / i32_scaled(X));
}

template <int DIM>
WOS_COLD float scaled_dir_poisson_kernel(float mur, float muR, float a0, float a1) {
  const double x = (double)mur, X = (double)muR, t = dexp(2.0 * (x - X));
  double q;
  if constexpr (DIM == 2) {
    double ie0, ke0, ie1, ke1;
    bessel_scaled(x, &ie0, &ke0, &ie1, &ke1);
    q = ke1 + ie1 * ((double)a0 / (double)a1) * t;
  } else {
    q = (1.0 + 1.0 / x) + i32_scaled(x) * (2.0 / (1.0 - dexp(-2.0 * X))) * t;
  }
  return (float)(x * dexp(-x) * q);
}

// Robust float semantics (DevParams::robust): Yukawa balls with mu R above this use
// exponentially scaled members (Gfn::yukawa == kYukScaled); below it the reference's
// float members are finite and are kept, so the two modes agree there bit for bit.
constexpr float kRobustMuR = 80.0f;
constexpr int kYukScaled = 2;

template <int DIM, bool RB = false>
struct Gfn {
  int yukawa;  // 0 harmonic, 1 Yukawa, kYukScaled Yukawa with scaled members (robust mode)
  float c[DIM], yVol[DIM], ySurf[DIM];
  float R, r;
  float lambda, sqrtLambda;
  float muR, A0, A1, B0, B1;   // 2D: K0muR I0muR K1muR I1muR ; 3D: expmuR sinhmuR K32muR I32muR
  static constexpr float rClamp = 1e-4f;

  __device__ __forceinline__ void init(bool yuk, float lam) {
    yukawa = yuk ? 1 : 0; lambda = lam; sqrtLambda = __builtin_sqrtf(lam);
  }

  // RB: the instantiation of the robust kernels; elsewhere the scaled branches are dead code
  __device__ __forceinline__ bool scaled() const { return RB && yukawa == kYukScaled; }

  // update_ball of a 2D Yukawa ball (reference members) with K0 I0 K1 I1 at mu R given
  // (the same update_ball evaluation, made by the point-setup kernel)
  __device__ __forceinline__ void set_ball(const float* cc, float RR, const float* m) {
    for (int k = 0; k < DIM; k++) { c[k] = cc[k]; yVol[k] = 0.0f; ySurf[k] = 0.0f; }
    R = RR; r = 0.0f;
    muR = R * sqrtLambda;
    A0 = m[0]; A1 = m[1]; B0 = m[2]; B1 = m[3];
  }

  __device__ __forceinline__ void update_ball(const float* cc, float RR, bool robust) {
    for (int k = 0; k < DIM; k++) { c[k] = cc[k]; yVol[k] = 0.0f; ySurf[k] = 0.0f; }
    R = RR; r = 0.0f;
    if (!yukawa) return;
    muR = R * sqrtLambda;
    if constexpr (RB) yukawa = (robust && muR > kRobustMuR) ? kYukScaled : 1;
    if (scaled()) {  // 3D scaled balls evaluate everything from mu R
      if constexpr (DIM == 2) scaled_members<DIM>(muR, &A0, &A1, &B0, &B1);
      return;
    }
    if constexpr (DIM == 2) {
      double i0, k0, i1, k1;
      bessel_ik<true, true>((double)muR, &i0, &k0, &i1, &k1);
      if (WOS_PROBE & 1) {
        double p0, p1, p2, p3;
        bessel_ik<true, true>(probe_opaque((double)muR), &p0, &p1, &p2, &p3);
        probe_sink(p0); probe_sink(p1); probe_sink(p2); probe_sink(p3);
      }
      A0 = (float)k0;
      A1 = (float)i0;
      B0 = (float)k1;
      B1 = (float)i1;
    } else {
      float expmuR = fexp(-muR);
      float exp2muR = expmuR * expmuR;
      float coshmuR = (1.0f + exp2muR) / (2.0f * expmuR);
      float sinhmuR = (1.0f - exp2muR) / (2.0f * expmuR);
      A0 = expmuR; A1 = sinhmuR;
      B0 = expmuR * (1.0f + 1.0f / muR);
      B1 = coshmuR - sinhmuR / muR;
      if (WOS_PROBE & 1) {
        const float m2 = probe_opaque(muR);
        const float e = fexp(-m2), e2 = e * e;
        const float ch = (1.0f + e2) / (2.0f * e), sh = (1.0f - e2) / (2.0f * e);
        probe_sink(e * (1.0f + 1.0f / m2)); probe_sink(ch - sh / m2); probe_sink(sh);
      }
    }
  }

  // G(r) for the current r (evaluate())
  __device__ __forceinline__ float evaluate() const {
    if (scaled()) {
      const double q = scaled_q0<DIM>(r * sqrtLambda, muR, A0, A1);
      if constexpr (DIM == 2) return (float)(q / kTwoPi);
      else return (float)(q / (kFourPi * (double)r));
    }
    if (!yukawa) {
      if constexpr (DIM == 2) return (float)((double)flog(R / r) / kTwoPi);
      else return (float)((double)(1.0f / r - 1.0f / R) / kFourPi);
    }
    float mur = r * sqrtLambda;
    if constexpr (DIM == 2) {
      double i0, k0;
      bessel_ik<true, false>((double)mur, &i0, &k0, nullptr, nullptr);
      float K0mur = (float)k0;
      float I0mur = (float)i0;
      return (float)((double)(K0mur - I0mur * A0 / A1) / kTwoPi);
    } else {
      float expmur = fexp(-mur);
      float sinhmur = (1.0f - expmur * expmur) / (2.0f * expmur);
      return (float)((double)(expmur - A0 * sinhmur / A1) / (kFourPi * (double)r));
    }
  }

  // 2D Yukawa (reference members): evaluate() and gradient_norm() from the Bessel values at
  // mu r, operation for operation -- for callers that evaluate all four orders at once
  __device__ __forceinline__ float evaluate_k0i0(double k0, double i0) const {
    const float K0mur = (float)k0, I0mur = (float)i0;
    return (float)((double)(K0mur - I0mur * A0 / A1) / kTwoPi);
  }
  __device__ __forceinline__ float gradient_norm_k1i1(double k1, double i1) const {
    const float K1mur = (float)k1, I1mur = (float)i1;
    const float Qr = sqrtLambda * (K1mur - I1mur * B0 / B1);
    return (float)((double)Qr / (kTwoPi * (double)r));
  }

  __device__ __forceinline__ float poisson_kernel() const {
    if (!yukawa) return DIM == 2 ? (float)(1.0 / kTwoPi) : (float)(1.0 / kFourPi);
    if (scaled()) return scaled_poisson_kernel<DIM>(muR, A1);
    if constexpr (DIM == 2) return (float)(1.0 / (kTwoPi * (double)A1));
    else return (float)((double)muR / (kFourPi * (double)A1));
  }

  __device__ __forceinline__ float norm() const {
    if (!yukawa) return DIM == 2 ? R * R / 4.0f : R * R / 6.0f;
    double pk = (double)poisson_kernel();
    return (float)((1.0 - (DIM == 2 ? kTwoPi : kFourPi) * pk) / (double)lambda);
  }

  __device__ __forceinline__ float gradient_norm() const {
    if (!yukawa) {
      if constexpr (DIM == 2) { float r2 = r * r; return (float)((double)(1.0f / r2 - 1.0f / (R * R)) / kTwoPi); }
      else { float r3 = r * r * r; return (float)((double)(1.0f / r3 - 1.0f / (R * R * R)) / kFourPi); }
    }
    float mur = r * sqrtLambda;
    if (scaled()) return scaled_gradient_norm<DIM>(r, sqrtLambda, muR, B0, B1);
    if constexpr (DIM == 2) {
      double i1, k1;
      bessel_ik<false, true>((double)mur, nullptr, nullptr, &i1, &k1);
      float K1mur = (float)k1;
      float I1mur = (float)i1;
      float Qr = sqrtLambda * (K1mur - I1mur * B0 / B1);
      return (float)((double)Qr / (kTwoPi * (double)r));
    } else {
      float r2 = r * r;
      float expmur = fexp(-mur);
      float exp2mur = expmur * expmur;
      float coshmur = (1.0f + exp2mur) / (2.0f * expmur);
      float sinhmur = (1.0f - exp2mur) / (2.0f * expmur);
      float K32mur = expmur * (1.0f + 1.0f / mur);
      float I32mur = coshmur - sinhmur / mur;
      float Qr = sqrtLambda * (K32mur - I32mur * B0 / B1);
      return (float)((double)Qr / (kFourPi * (double)r2));
    }
  }

  __device__ __forceinline__ void gradient(float* out) const {
    float gn = gradient_norm();
    for (int k = 0; k < DIM; k++) out[k] = (yVol[k] - c[k]) * gn;
  }

  __device__ __forceinline__ void poisson_kernel_gradient(float* out) const {
    float d[DIM];
    for (int k = 0; k < DIM; k++) d[k] = ySurf[k] - c[k];
    if (!yukawa) {
      if constexpr (DIM == 2) {
        float s = (float)((kTwoPi * (double)R) * (double)R);
        for (int k = 0; k < 2; k++) out[k] = (2.0f * d[k]) / s;
      } else {
        float s = (float)((kFourPi * (double)R) * (double)R);
        for (int k = 0; k < 3; k++) out[k] = (3.0f * d[k]) / s;
      }
      return;
    }
    if (scaled()) {
      const float QR = scaled_pk_gradient<DIM>(muR, sqrtLambda, lambda, R, B1);
      for (int k = 0; k < DIM; k++) out[k] = (d[k] * QR) / (float)(DIM == 2 ? kTwoPi : kFourPi);
      return;
    }
    if constexpr (DIM == 2) {
      float QR = sqrtLambda / (R * B1);
      for (int k = 0; k < 2; k++) out[k] = (d[k] * QR) / (float)kTwoPi;
    } else {
      float QR = lambda / B1;
      for (int k = 0; k < 3; k++) out[k] = (d[k] * QR) / (float)kFourPi;
    }
  }

  __device__ __forceinline__ float dir_sampled_poisson_kernel(const float* y) const {
    if (!yukawa) return 1.0f;
    float d[DIM];
    for (int k = 0; k < DIM; k++) d[k] = y[k] - c[k];
    float rr = smax(rClamp, normv<DIM>(d));
    float mur = rr * sqrtLambda;
    if (scaled()) return scaled_dir_poisson_kernel<DIM>(mur, muR, A0, A1);
    if constexpr (DIM == 2) {
      double i1, k1;
      bessel_ik<false, true>((double)mur, nullptr, nullptr, &i1, &k1);
      if (WOS_PROBE & 2) {
        double p1, p2;
        bessel_ik<false, true>(probe_opaque((double)mur), nullptr, nullptr, &p1, &p2);
        probe_sink(p1); probe_sink(p2);
      }
      const float K1mur = (float)k1;
      const float I1mur = (float)i1;
      float Q = K1mur + I1mur * A0 / A1;
      return mur * Q;
    } else {
      float expmur = fexp(-mur);
      float exp2mur = expmur * expmur;
      float coshmur = (1.0f + exp2mur) / (2.0f * expmur);
      float sinhmur = (1.0f - exp2mur) / (2.0f * expmur);
      float K32mur = expmur * (1.0f + 1.0f / mur);
      float I32mur = coshmur - sinhmur / mur;
      float Q = K32mur + I32mur * A0 / A1;
      if (WOS_PROBE & 2) {
        const float m2 = probe_opaque(mur);
        const float e = fexp(-m2), e2 = e * e;
        const float ch = (1.0f + e2) / (2.0f * e), sh = (1.0f - e2) / (2.0f * e);
        probe_sink(m2 * (e * (1.0f + 1.0f / m2) + (ch - sh / m2) * A0 / A1));
      }
      return mur * Q;
    }
  }

  // off-centred G(x,y): only reached in the non-finite (NaN-propagation) regime
  __device__ float evaluate_xy(const float* x, const float* y) const {
    float yx[DIM], xc[DIM], yc[DIM];
    for (int k = 0; k < DIM; k++) { yx[k] = y[k] - x[k]; xc[k] = x[k] - c[k]; yc[k] = y[k] - c[k]; }
    if (!yukawa) {
      float rr = smax(rClamp, normv<DIM>(yx));
      if constexpr (DIM == 2) return (float)((double)(flog(R * R - dotv<2>(xc, yc)) - flog(R * rr)) / kTwoPi);
      else return (float)((double)(1.0f / rr - R / (R * R - dotv<3>(xc, yc))) / kFourPi);
    }
    float r1 = smax(rClamp, normv<DIM>(yx));
    float r2 = (R * R - dotv<DIM>(xc, yc)) / R;
    float mur1 = r1 * sqrtLambda, mur2 = r2 * sqrtLambda;
    if (scaled()) {
      const double q1 = scaled_q0<DIM>(mur1, muR, A0, A1), q2 = scaled_q0<DIM>(mur2, muR, A0, A1);
      if constexpr (DIM == 2) return (float)((q1 - q2) / kTwoPi);
      else return (float)((q1 / (double)r1 - q2 / (double)r2) / kFourPi);
    }
    if constexpr (DIM == 2) {
      float K0mur1 = (float)bessk0((double)mur1), K0mur2 = (float)bessk0((double)mur2);
      float I0mur1 = (float)bessi0((double)mur1), I0mur2 = (float)bessi0((double)mur2);
      float Q1 = K0mur1 - I0mur1 * A0 / A1;
      float Q2 = K0mur2 - I0mur2 * A0 / A1;
      return (float)((double)(Q1 - Q2) / kTwoPi);
    } else {
      float e1 = fexp(-mur1), e2 = fexp(-mur2);
      float s1 = (1.0f - e1 * e1) / (2.0f * e1), s2 = (1.0f - e2 * e2) / (2.0f * e2);
      float Q1 = (e1 - A0 * s1 / A1) / r1;
      float Q2 = (e2 - A0 * s2 / A1) / r2;
      return (float)((double)(Q1 - Q2) / kFourPi);
    }
  }
};

template <int DIM>
__device__ __forceinline__ float pdf_sphere_uniform(float r) {
  if constexpr (DIM == 2) return (float)(1.0 / (kTwoPi * (double)r));
  else return (float)(1.0 / ((kFourPi * (double)r) * (double)r));
}

template <int DIM>
__device__ __forceinline__ void sample_unit_sphere(const float* u, float* out) {
  if constexpr (DIM == 2) {
    float phi = (float)(kTwoPi * (double)u[0]);
    fsincos(phi, &out[1], &out[0]);
  } else {
    float z = 1.0f - 2.0f * u[0];
    float r = __builtin_sqrtf(smax(0.0f, 1.0f - z * z));
    float phi = (float)(kTwoPi * (double)u[1]);
    float s, c;
    fsincos(phi, &s, &c);
    out[0] = r * c; out[1] = r * s; out[2] = z;
  }
}

// ---------------------------------------------------------------------------
// Certified float fast path for the rejection test.  The accept decision
// u < pdfRadius/bound is first evaluated with float Bessel approximations (same
// A&S polynomials, hardware exp2/log2/rsq); only when |u - T| falls inside a
// rigorous error band is the exact double-precision path (the reference's
// arithmetic) evaluated.  The decision -- hence every RNG draw and every later
// value -- is therefore identical to the exact loop.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float exp_fast(float x) {  // e^x to ~2 ulp for |x| < 87
  const float L = 1.44269502162933349609375f, Llo = 1.925963033500011e-08f;
  float hi = x * L;
  float lo = __builtin_fmaf(x, L, -hi) + x * Llo;
  return __builtin_amdgcn_exp2f(hi) * (1.0f + lo * 0.693147182f);
}

__device__ __forceinline__ float i0_fast(float x) {
  if (x < 3.75f) {
    float y = x / 3.75f;
    y = y * y;
    return 1.0f + y * (3.5156229f + y * (3.0899424f + y * (1.2067492f + y * (0.2659732f + y * (0.360768e-1f +
           y * 0.45813e-2f)))));
  }
  float y = 3.75f / x;
  float poly = 0.39894228f + y * (0.1328592e-1f + y * (0.225319e-2f + y * (-0.157565e-2f + y * (0.916281e-2f +
               y * (-0.2057706e-1f + y * (0.2635537e-1f + y * (-0.1647633e-1f + y * 0.392377e-2f)))))));
  return exp_fast(x) * __builtin_amdgcn_rsqf(x) * poly;
}

__device__ __forceinline__ float k0_fast(float x) {
  if (x <= 2.0f) {
    float y = x * x / 4.0f;
    return (-__builtin_amdgcn_logf(x * 0.5f) * 0.693147182f) * i0_fast(x) +
           (-0.57721566f + y * (0.42278420f + y * (0.23069756f + y * (0.3488590e-1f + y * (0.262698e-2f +
            y * (0.10750e-3f + y * 0.74e-5f))))));
  }
  float y = 2.0f / x;
  return exp_fast(-x) * __builtin_amdgcn_rsqf(x) * (1.25331414f + y * (-0.7832358e-1f + y * (0.2189568e-1f +
         y * (-0.1062446e-1f + y * (0.587872e-2f + y * (-0.251540e-2f + y * 0.53208e-3f))))));
}

__device__ __forceinline__ float i1_fast(float x) {
  if (x < 3.75f) {
    float y = x / 3.75f;
    y = y * y;
    return x * (0.5f + y * (0.87890594f + y * (0.51498869f + y * (0.15084934f + y * (0.2658733e-1f +
           y * (0.301532e-2f + y * 0.32411e-3f))))));
  }
  float y = 3.75f / x;
  float a = 0.2282967e-1f + y * (-0.2895312e-1f + y * (0.1787654e-1f - y * 0.420059e-2f));
  a = 0.39894228f + y * (-0.3988024e-1f + y * (-0.362018e-2f + y * (0.163801e-2f + y * (-0.1031555e-1f + y * a))));
  return exp_fast(x) * __builtin_amdgcn_rsqf(x) * a;
}

__device__ __forceinline__ float k1_fast(float x) {
  if (x <= 2.0f) {
    float y = x * x / 4.0f;
    return (__builtin_amdgcn_logf(x * 0.5f) * 0.693147182f) * i1_fast(x) +
           (1.0f / x) * (1.0f + y * (0.15443144f + y * (-0.67278579f + y * (-0.18156897f + y * (-0.1919402e-1f +
           y * (-0.110404e-2f + y * (-0.4686e-4f)))))));
  }
  float y = 2.0f / x;
  return exp_fast(-x) * __builtin_amdgcn_rsqf(x) * (1.25331414f + y * (0.23498619f + y * (-0.3655620e-1f +
         y * (0.1504268e-1f + y * (-0.780353e-2f + y * (0.325614e-2f + y * (-0.68245e-3f)))))));
}

// K0 and I0 of the rejection fast path at one argument: the polynomials of
// k0_fast / i0_fast, with I0 and x^-1/2 shared (k0_fast at x <= 2 re-evaluates I0) and
// the divisions by / of x as reciprocal products.  The reciprocals add ~1 ulp to y,
// far inside the 8e-6 band the decisions are certified with (the GPU self-test checks
// the <= 2e-6 error against the double-precision A&S functions).
__device__ __forceinline__ void k0i0_fast(float x, float* k0, float* i0) {
  const float rs = __builtin_amdgcn_rsqf(x);
  const float rx = __builtin_amdgcn_rcpf(x);
  float iv;
  if (x < 3.75f) {
    float y = x * 0.266666681f;
    y = y * y;
    iv = 1.0f + y * (3.5156229f + y * (3.0899424f + y * (1.2067492f + y * (0.2659732f + y * (0.360768e-1f +
         y * 0.45813e-2f)))));
  } else {
    const float y = 3.75f * rx;
    const float poly = 0.39894228f + y * (0.1328592e-1f + y * (0.225319e-2f + y * (-0.157565e-2f + y * (0.916281e-2f +
                       y * (-0.2057706e-1f + y * (0.2635537e-1f + y * (-0.1647633e-1f + y * 0.392377e-2f)))))));
    iv = exp_fast(x) * rs * poly;
  }
  float kv;
  if (x <= 2.0f) {
    const float y = x * x * 0.25f;
    kv = (-__builtin_amdgcn_logf(x * 0.5f) * 0.693147182f) * iv +
         (-0.57721566f + y * (0.42278420f + y * (0.23069756f + y * (0.3488590e-1f + y * (0.262698e-2f +
          y * (0.10750e-3f + y * 0.74e-5f))))));
  } else {
    const float y = 2.0f * rx;
    kv = exp_fast(-x) * rs * (1.25331414f + y * (-0.7832358e-1f + y * (0.2189568e-1f +
         y * (-0.1062446e-1f + y * (0.587872e-2f + y * (-0.251540e-2f + y * 0.53208e-3f))))));
  }
  *k0 = kv;
  *i0 = iv;
}

// Certain-reject bound of the Yukawa rejection test.  The test accepts iff
// u < T(r) = (K0(mu r) - rho I0(mu r)) r / (norm bound) (2D) or
// (e^{-mu r} - rho sinh(mu r)) r / (norm bound) (3D), with rho = A0/A1 > 0 and the
// subtracted term >= 0 for 0 <= r <= R, so T(r) <= r K0(mu r) / (norm bound)
// <= 0.46652 / (mu norm bound) (max_z z K0(z) at z = 0.595) and in 3D
// T(r) <= r e^{-mu r} / (norm bound) <= 1 / (e mu norm bound).  The constants carry
// a 1e-3 margin (far above the A&S polynomial error and the float rounding of the
// exact path), so u above the bound is the exact test's reject without evaluating
// r at all.  A non-positive or non-finite bound disables the shortcut.
// Tighter, per ball: T(r) <= R F(mu R) / (norm bound) with F(s) = max_x x Q_s(x)
// tabulated by bins of s with a 2 % margin (DevParams::rej_tab, wos_host_scene.h
// rejection_bound_table) -- the subtracted term is kept, so the bound follows the
// real peak of the threshold (tests/test_rejection_bounds.py checks both bounds).
// the rejection bound table (both dimensions) in LDS: read on every sampler call,
// one global round trip less on a walk step's critical path
static __shared__ float s_rej_tab[2 * kRejTabBins];
__device__ __forceinline__ float rej_tab_at(int i, const DevParams& prm) {
  return s_rej_tab[i];
}

template <int DIM>
__device__ __forceinline__ float rej_quick_bound(const DevParams& prm, float R, float muR, float sqrtL, float invNB) {
  const float C = DIM == 2 ? 0.4670f : 0.3683f;
  float q = C * invNB / sqrtL;
  if (prm.rej_tab != nullptr && muR >= 0.0f) {
    const int k = (int)(kRejTabScale * __builtin_sqrtf(muR));
    if (k < kRejTabBins) {
      // staged in LDS by stage_rej_jump (every kernel that samples)
      const float qt = R * rej_tab_at((DIM == 3 ? kRejTabBins : 0) + k, prm) * invNB;
      q = qt < q ? qt : q;
    }
  }
  return (q > 0.0f && q < 3.0e38f) ? q : 3.0e38f;
}

// sampleVolume + rejectionSampleGreensFn (distributions.h:362-383,404-410,486-500,591-599,710-720).
// need_pdf: the caller uses the returned pdf (first ball); walk steps ignore it.
// the float draw Pcg32::nextf makes from a stream state (before its step)
__device__ __forceinline__ float pcg_float_of(uint64_t state) {
  return bits_to_float((pcg_output(state) >> 9) | 0x3f800000u) - 1.0f;
}

template <int DIM, bool RB>
__device__ __forceinline__ void sample_volume(const DevParams& prm, Gfn<DIM, RB>& g, const float* dir, Pcg32& s,
                                              float* pdf, float* out, uint32_t* iters, bool need_pdf,
                                              float* r_pre = nullptr) {
  const float R = g.R;
  if (DIM == 3 && !g.yukawa) {
    float u1 = s.nextf(), u2 = s.nextf();
    float phi = (float)(kTwoPi * (double)u2);
    float r = (1.0f + __builtin_sqrtf(1.0f - fcbrt(u1 * u1)) * fcos(phi)) * R / 2.0f;
    r = smax(Gfn<DIM>::rClamp, r);
    if (r > R) r = R / 2.0f;
    g.r = r;
    for (int k = 0; k < DIM; k++) { g.yVol[k] = g.c[k] + r * dir[k]; out[k] = g.yVol[k]; }
    *pdf = g.evaluate() / g.norm();
    return;
  }
  float bound;
  if (!g.yukawa) {
    bound = 1.5f / R;
  } else {
    const float a = DIM == 2 ? 2.2f : 2.0f, b = DIM == 2 ? 0.6f : 0.5f;
    const float lam = g.lambda, sl = g.sqrtLambda;
    bound = R <= lam ? smax(smax(a / R, a / lam), smax(b * __builtin_sqrtf(R), b * sl))
                     : smax(smin(a / R, a / lam), smin(b * __builtin_sqrtf(R), b * sl));
  }
  // norm() depends only on the ball: hoisted out of the loop (same value every iteration)
  const float nrm = g.norm();
  // fast path: 2D Yukawa while I0 stays finite in float (float Bessels need mu*r < ~88)
  const bool fast = DIM == 2 && g.yukawa && g.muR < 80.0f;
  const float rho = g.A0 / g.A1;
  const float invNB = 1.0f / (nrm * bound);
  const float quick = g.yukawa ? rej_quick_bound<DIM>(prm, g.R, g.muR, g.sqrtLambda, invNB) : 3.0e38f;
  int iter = 0;
  // the stream walks two draws per iteration with one jump (state * A2 + C2); the radius
  // draw becomes a float only when the certain-reject test leaves u undecided (the
  // tiny-ball loops of near-wall points run to hundreds of iterations, nearly all of
  // them certain rejects: profiles/r3z_ab_seq_loop.log)
  uint64_t st = s.state, st1 = st;
  do {
    const float u = pcg_float_of(st);
    st1 = st * kPcgMult + kPcgInc;
    st = st * kPcgMult2 + kPcgInc2;
    iter++;
    int decided = -1;  // 1 accept, 0 reject, -1 undecided
    if (u > quick) continue;
    g.r = pcg_float_of(st1) * R;
    if (fast) {
      const float mur = g.r * g.sqrtLambda;
      float k0, i0v;
      k0i0_fast(mur, &k0, &i0v);
      const float ip = i0v * rho;
      const float c = g.r * invNB;
      const float Tf = (k0 - ip) * c;
      const float M = 8e-6f * (__builtin_fabsf(k0) + __builtin_fabsf(ip)) * c + 2e-6f * __builtin_fabsf(Tf) + 1e-30f;
      if (u < Tf - M) decided = 1;
      else if (u > Tf + M) decided = 0;
    }
    if (decided < 0) {
      float p = g.evaluate() / nrm;
      float pdfRadius = p / pdf_sphere_uniform<DIM>(g.r);
      decided = u < pdfRadius / bound ? 1 : 0;
    }
    if (decided == 1) break;
  } while (iter < 1000);
  s.state = st;
  g.r = pcg_float_of(st1) * R;  // the last iteration's radius (also when the limit ended the loop)
  if (need_pdf) *pdf = g.evaluate() / nrm;  // pdf of the last sampled radius (before the clamps)
  if (r_pre) *r_pre = g.r;
  *iters += (uint32_t)iter;
  g.r = smax(Gfn<DIM>::rClamp, g.r);
  if (g.r > R) g.r = R / 2.0f;
  for (int k = 0; k < DIM; k++) { g.yVol[k] = g.c[k] + g.r * dir[k]; out[k] = g.yVol[k]; }
}

// ---------------------------------------------------------------------------
// Wave-cooperative rejection sampling (rejectionSampleGreensFn, distributions.h:
// 362-383) for the 2D Yukawa fast path.  Iteration j of a lane's loop consumes
// draws 2j and 2j+1 of its PCG32 stream, and state_k = A_k * state_0 + C_k (the
// jump table), so the iterations of all lanes can be evaluated in any order by
// any lane.  Each generation gives every unfinished lane a block of B = 64 /
// (#unfinished) consecutive iterations spread over the wave; the owner then scans
// its block in order -- the first certain accept wins, an undecided iteration is
// decided by the owner with the exact double-precision test -- exactly the
// sequential loop's decisions, so the accepted radius, the iteration count and
// the stream position after the loop are the sequential ones.  This removes the
// geometric tail (the wave paid for the longest loop of its lanes).  Lanes off
// the fast path (3D, harmonic, mu*R >= 80) run the sequential loop.
// ---------------------------------------------------------------------------
constexpr int kRejMax = 1000;  // rejectionSampleGreensFn iteration limit
// minimum iterations per unfinished lane and generation of the cooperative sampler
// (2D acceptance ~21 %, 3D ~7 % on the shipped scenes)
// (A/B on MI355X, tools/ab.sh: 2D 3 beats 1 by 2-4 % on karman / C; 3D 8 in the first-ball
// kernel beats 16 by 8 %, while the walk kernel keeps 16)
#ifndef WOS_REJ_BMIN2
#define WOS_REJ_BMIN2 3
#endif
#ifndef WOS_REJ_BMIN3
#define WOS_REJ_BMIN3 16
#endif
#ifndef WOS_REJ_BMIN3_FB
#define WOS_REJ_BMIN3_FB 8
#endif
template <int DIM, bool FB>
constexpr int kRejBmin = DIM == 2 ? WOS_REJ_BMIN2 : (FB ? WOS_REJ_BMIN3_FB : WOS_REJ_BMIN3);
static_assert(WOS_REJ_BMIN2 <= 16 && WOS_REJ_BMIN3 <= 16 && WOS_REJ_BMIN3_FB <= 16, "RejLDS::surv holds 64 * 16 items");


// iterations each sampling lane evaluates on its own before the cooperative generations
// (0: none) in calls with at least WOS_REJ_OWN_MIN sampling lanes; 4 / 40 measured best
// (karman -3 %, config C -2 %, the cube -1.5 %, the stride-8 shard unchanged;
// profiles/r3y_ab_own_generation.log)
#ifndef WOS_REJ_OWN
#define WOS_REJ_OWN 4
#endif
constexpr int kRejOwn = WOS_REJ_OWN;
// 3D (acceptance ~7 %): iterations of the own generation -- the walk kernel's 32 (a lane accepts
// within them with P ~ 0.9; walk kernel on the cube at 128^3: 22.1 ms with 4, 20.8 with 16, 20.7
// with 24; with the radius-dependent screen (rej_xreject3) 19.4 ms with 24, 19.1 with 32), the
// first-ball kernel's 4 (16 made first balls +6 %; the screen there +1-4 %): profiles/r5k_ab_own3.log,
// r5l_ab_own3.log, r5zb_ab_xbound3.log, r5zc_ab_xbound3.log
#ifndef WOS_REJ_OWN3
#define WOS_REJ_OWN3 32
#endif
#ifndef WOS_REJ_OWN3_FB
#define WOS_REJ_OWN3_FB WOS_REJ_OWN
#endif
template <int DIM, bool FB>
constexpr int kRejOwnD = DIM == 2 ? WOS_REJ_OWN : (FB ? WOS_REJ_OWN3_FB : WOS_REJ_OWN3);
static_assert(WOS_REJ_OWN3 >= 0 && WOS_REJ_OWN3 <= 32 && WOS_REJ_OWN3_FB >= 0 && WOS_REJ_OWN3_FB <= 32, "own");
#ifndef WOS_REJ_OWN_MIN
#define WOS_REJ_OWN_MIN 40
#endif
constexpr int kRejOwnMin = WOS_REJ_OWN_MIN;  // sampling lanes for the own generation
static_assert(WOS_REJ_OWN >= 0 && WOS_REJ_OWN <= 16 && WOS_REJ_OWN < kRejMax, "WOS_REJ_OWN");

// PCG32 jump-ahead: state after k draws from s0 (DevParams::jump, built on the host)
__device__ __forceinline__ uint64_t jump_state(const DevParams& prm, uint64_t s0, int k) {
  const uint64_t A = prm.jump[2 * k], Cc = prm.jump[2 * k + 1];
  return A * s0 + Cc;
}

// The jump constants of the first kRejJumpLds rejection iterations (draw 2j) are
// staged in LDS by every kernel that samples (stage_rej_jump); later iterations
// (P ~ 1e-4 per sample) read the global table.
#ifndef WOS_REJ_JUMP_LDS
#define WOS_REJ_JUMP_LDS 128
#endif
constexpr int kRejJumpLds = WOS_REJ_JUMP_LDS > 0 ? WOS_REJ_JUMP_LDS : 1;
static __shared__ unsigned long long s_rej_jump[2 * kRejJumpLds];

__device__ __forceinline__ void stage_rej_jump(const DevParams& prm) {
  for (int i = threadIdx.x; i < 2 * kRejJumpLds; i += blockDim.x) s_rej_jump[i] = prm.jump[4 * (i >> 1) + (i & 1)];
  if (prm.rej_tab != nullptr)
    for (int i = threadIdx.x; i < 2 * kRejTabBins; i += blockDim.x) s_rej_tab[i] = prm.rej_tab[i];
}

// stream state before rejection iteration j (draw 2j) from stream start s0
__device__ __forceinline__ uint64_t rej_state(const DevParams& prm, uint64_t s0, int j) {
  if (WOS_REJ_JUMP_LDS > 0 && j < kRejJumpLds) return s_rej_jump[2 * j] * s0 + s_rej_jump[2 * j + 1];
  return jump_state(prm, s0, 2 * j);
}

// floor(item / B) for item < 2048, 1 <= B <= 32, with m = ceil(2^16 / B): writing
// item = qB + r, item*m/2^16 = q + (r + item*e/2^16)/B with e = mB - 2^16 < B, and
// item*e < 2^16, so the floor is q.  (A runtime u32 division is ~20 VALU ops per item.)
// The sampler's generation has items = nact * B with B = clamp(64 / nact, kRejBmin, kRejBcap):
// items <= 64 when B = floor(64 / nact) or B = kRejBcap (then nact < 2), else
// items = nact * kRejBmin <= 64 * kRejBmin.  rej_div needs items <= 2048 and B <= 32.
constexpr int kRejBcap = 32;
static_assert(kRejBcap <= 32, "rej_div: e = m B - 2^16 < B <= 32");
static_assert(kWave * (WOS_REJ_BMIN2 > WOS_REJ_BMIN3 ? WOS_REJ_BMIN2 : WOS_REJ_BMIN3) <= 2048 && kWave <= 2048,
              "rej_div: item * e < 2^16 needs items <= 2048");
__device__ __forceinline__ int rej_div(int item, int B, uint32_t mB) {
  return (int)(((uint32_t)item * mB) >> 16);
}

struct RejLDS {
  unsigned long long s0[kWave];
  float R[kWave], sqrtL[kWave];
  float c0[kWave], c1[kWave];  // 2D: rho = A0/A1, 1/(norm*bound)   3D: A0, A1 (ball members)
  float rho3[kWave], inv3[kWave];  // 3D: A0/A1, 1/(norm*bound) (fast path)
  float qb[kWave];                 // certain-reject bound (rej_quick_bound)
  float nrm[kWave], bound[kWave];
  uint32_t acc[kWave], und[kWave];
  uint32_t owner_of[kWave];
};

__device__ __forceinline__ float draw_float(uint64_t state) {
  return bits_to_float((pcg_output(state) >> 9) | 0x3f800000u) - 1.0f;
}

// the two draws of rejection iteration j from stream start s0
__device__ __forceinline__ void rej_draws(const DevParams& prm, uint64_t s0, int j, float* u, float* x) {
  const uint64_t st = rej_state(prm, s0, j);
  *u = draw_float(st);
  *x = draw_float(st * kPcgMult + kPcgInc);
}

// fast decision of one iteration: 1 accept, 0 reject, -1 undecided (see sample_volume)
__device__ __forceinline__ int rej_fast_decide(float u, float r, float sqrtL, float rho, float invNB) {
  const float mur = r * sqrtL;
  float k0, i0v;
  k0i0_fast(mur, &k0, &i0v);
  const float ip = i0v * rho;
  const float c = r * invNB;
  const float Tf = (k0 - ip) * c;
  const float M = 8e-6f * (__builtin_fabsf(k0) + __builtin_fabsf(ip)) * c + 2e-6f * __builtin_fabsf(Tf) + 1e-30f;
  return u < Tf - M ? 1 : (u > Tf + M ? 0 : -1);
}

// 3D analogue: e = exp(-mu r) from exp_fast (<= ~3 ulp) and an approximate
// reciprocal; the band M covers their error carried through the cancellation in
// sinh(mu r) = (1 - e^2) / 2e and Q = e - (A0/A1) sinh, plus the rounding of the
// exact path's float/double steps (~4 ulp of T), with a >= 4x margin.  Non-finite
// or underflowed e leaves M non-finite: undecided.
__device__ __forceinline__ int rej_fast_decide3(float u, float r, float sqrtL, float rho, float invNB) {
  const float mur = r * sqrtL;
  const float e = exp_fast(-mur);
  const float ie = __builtin_amdgcn_rcpf(e);
  const float sh = (1.0f - e * e) * 0.5f * ie;
  const float Q = e - rho * sh;
  const float c = r * invNB;
  const float Tf = Q * c;
  const float ar = __builtin_fabsf(rho);
  const float M = (2e-6f * e + ar * (3e-7f * ie + 2e-6f * e + 4e-6f * __builtin_fabsf(sh))) * c +
                  4e-6f * __builtin_fabsf(Tf) + 1e-30f;
  return u < Tf - M ? 1 : (u > Tf + M ? 0 : -1);
}

// Radius-dependent certain reject (3D Yukawa): the threshold
//   T(r) = r (e^{-mu r} - rho sinh(mu r)) invNB <= r e^{-mu r} invNB,
// rho = A0/A1 >= 0 and sinh >= 0 (the exact path's float subtraction of a non-negative term
// cannot exceed e^{-mu r} either).  The bound carries a 0.1 % relative margin (hardware exp2,
// the rounding of mu r and of the exact path's divisions: ~1e-5) plus 1e-6 R invNB absolute,
// so u above it is the exact test's reject.  r = 0 and mu r >= 80 are left to the tests.
// Round 2 measured the screen alone (every iteration still paid for the fast test whenever a
// lane of its wave needed it); the own generation now screens its whole block first and runs
// the fast test on the survivors only (tests/test_rejection_bounds.py checks the bound).
// The ball's constants come folded: kz = -sqrtL log2(e), kb = 1.001 invNB, so t = r kz and
// 2^t = e^{-mu r} up to the rounding of the folded product (a few ulp of t: <= 3e-5 relative
// in e below mu r = 80, far inside the margin).  t > -115 keeps mu r < 79.7.
__device__ __forceinline__ bool rej_xreject3(float u, float r, float kz, float kb, float xabs) {
  const float t = r * kz;
  if (!(r > 0.0f) || !(t > -115.0f)) return false;
  return u > __builtin_fmaf(r * kb, __builtin_amdgcn_exp2f(t), xabs);
}

// exact 3D Yukawa test of one iteration with an owner's ball constants: the same
// Gfn::evaluate / pdf arithmetic as sample_volume, hence the same decision
__device__ __forceinline__ int rej_exact_decide3(float u, float r, float R, float sqrtL, float A0, float A1, float nrm,
                                                 float bound) {
  Gfn<3> h;
  h.yukawa = 1;
  h.sqrtLambda = sqrtL;
  h.A0 = A0;
  h.A1 = A1;
  h.R = R;
  h.r = r;
  const float p = h.evaluate() / nrm;
  const float pdfRadius = p / pdf_sphere_uniform<3>(r);
  return u < pdfRadius / bound ? 1 : 0;
}

// Queries with exactly one querying lane (a lone walk in its wave) take the
// register-only solo forms (sampler, star radius, ray): every lane works on the one
// owner's items, owner data broadcast with readlane, results by ballot / wave reduction

// Convergent: every lane calls it.  Inactive lanes do nothing.  2D: certified float
// decisions by any lane, undecided ones by the owner (exact); 3D: certified float
// decisions by any lane, undecided ones by the same lane with the exact test (cheap
// single-precision arithmetic plus one exp).
template <int DIM, bool RB, bool FB = false>
__device__ __forceinline__ void sample_volume_wave(const DevParams& prm, bool active, Gfn<DIM, RB>& g, const float* dir,
                                                   Pcg32& s, float* pdf, float* out, uint32_t* iters,
                                                   bool need_pdf, RejLDS* L, int lane) {
  bool coop = false;
  float bound = 0.0f, nrm = 1.0f;
  if (active && g.yukawa && (DIM == 3 ? !g.scaled() : g.muR < 80.0f)) {
    const float R = g.R, lam = g.lambda, sl = g.sqrtLambda;
    const float a = DIM == 2 ? 2.2f : 2.0f, b = DIM == 2 ? 0.6f : 0.5f;
    bound = R <= lam ? smax(smax(a / R, a / lam), smax(b * __builtin_sqrtf(R), b * sl))
                     : smax(smin(a / R, a / lam), smin(b * __builtin_sqrtf(R), b * sl));
    nrm = g.norm();
    coop = true;
  }
  const uint64_t cmask = __ballot(coop);
  if (cmask != 0 && (cmask & (cmask - 1)) == 0) {
    // one sampling lane (a lone walk): lane l evaluates iteration j0 + l of the owner's
    // stream with the owner's constants broadcast from registers; the decisions come
    // back as ballots and are scanned in order -- no LDS, no wave syncs
    const int ol = __builtin_ctzll(cmask);
    const uint64_t s0 = s.state;
    const uint64_t s0o = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(s0 >> 32), ol) << 32) |
                         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)s0, ol);
    const float invNB = 1.0f / (nrm * bound);
    const float oR = lane_bcast(g.R, ol), oSL = lane_bcast(g.sqrtLambda, ol);
    const float oQB = lane_bcast(coop ? rej_quick_bound<DIM>(prm, g.R, g.muR, g.sqrtLambda, invNB) : 0.0f, ol);
    const float oRho = lane_bcast(coop ? g.A0 / g.A1 : 0.0f, ol), oInv = lane_bcast(invNB, ol);
    float oA0 = 0.0f, oA1 = 0.0f, oNrm = 0.0f, oBound = 0.0f;
    if constexpr (DIM == 3) {
      oA0 = lane_bcast(g.A0, ol); oA1 = lane_bcast(g.A1, ol); oNrm = lane_bcast(nrm, ol); oBound = lane_bcast(bound, ol);
    }
    DIAG_COUNT(D_RCALLS, 1);
    DIAG_COUNT(D_RLANES, 1);
    int jacc = -1;
    for (int j0 = 0; jacc < 0; j0 += kWave) {
      DIAG_COUNT(D_RGENS, 1);
      const int j = j0 + lane;
      int dcs = 0;
      if (j < kRejMax) {
        const uint64_t st = rej_state(prm, s0o, j);
        const float u = draw_float(st);
        DIAG_LANE(D_RITEMS);
        if (u > oQB) {
          DIAG_LANE(D_RQUICK);
        } else {
          const float x = draw_float(st * kPcgMult + kPcgInc);
          if constexpr (DIM == 2) {
            dcs = rej_fast_decide(u, x * oR, oSL, oRho, oInv);
          } else {
            const float rr = x * oR;
            dcs = rej_fast_decide3(u, rr, oSL, oRho, oInv);
            if (dcs < 0) dcs = rej_exact_decide3(u, rr, oR, oSL, oA0, oA1, oNrm, oBound);
          }
        }
      }
      const uint64_t acc = __ballot(dcs == 1), und = __ballot(dcs < 0);
      for (uint64_t m = acc | und; m != 0; m &= m - 1) {
        const int b = __builtin_ctzll(m);
        if ((acc >> b) & 1ull) { jacc = j0 + b; break; }
        // undecided: the exact test of sample_volume, by the owner
        int ok = 0;
        if (lane == ol) {
          float u, x;
          rej_draws(prm, s0, j0 + b, &u, &x);
          g.r = x * g.R;
          const float pr = g.evaluate() / nrm;
          const float pdfRadius = pr / pdf_sphere_uniform<DIM>(g.r);
          ok = u < pdfRadius / bound ? 1 : 0;
        }
        if (__builtin_amdgcn_readlane(ok, ol)) { jacc = j0 + b; break; }
      }
      if (jacc < 0 && j0 + kWave >= kRejMax) jacc = kRejMax - 1;  // limit: last radius kept
    }
    if (coop) {
      float u, x;
      rej_draws(prm, s0, jacc, &u, &x);
      g.r = x * g.R;
      s.state = rej_state(prm, s0, jacc + 1);
      *iters += (uint32_t)(jacc + 1);
      if (need_pdf) *pdf = g.evaluate() / nrm;
      g.r = smax(Gfn<DIM>::rClamp, g.r);
      if (g.r > g.R) g.r = g.R / 2.0f;
      for (int k = 0; k < DIM; k++) { g.yVol[k] = g.c[k] + g.r * dir[k]; out[k] = g.yVol[k]; }
    }
  } else if (cmask != 0) {
    const uint64_t s0 = s.state;
    // every unfinished lane is handed B iterations per generation and advances by B
    // when it does not accept among them, so all unfinished lanes stand at the same
    // iteration j0: wave-uniform (no per-owner base in LDS)
    int j0 = 0, jacc = -1;
    bool done = !coop;
    DIAG_COUNT(D_RCALLS, 1);
    DIAG_COUNT(D_RLANES, __popcll(__ballot(coop)));
#if WOS_REJ_OWN
    // generation 0 of a dense call (at least kRejOwnMin sampling lanes): every sampling lane
    // evaluates the first kRejOwn iterations of its own stream in registers (no LDS
    // broadcast, no atomics, no wave syncs); the lanes still without an accept continue
    // cooperatively from iteration kRejOwn.  Sparse calls keep the cooperative generations
    // from iteration 0 (shorter dependency chains for the few lanes of the tail).
    const bool own = __popcll(cmask) >= kRejOwnMin;
    if (own && !done) {
      const float invNB0 = 1.0f / (nrm * bound);
      const float qb0 = rej_quick_bound<DIM>(prm, g.R, g.muR, g.sqrtLambda, invNB0);
      uint32_t acc = 0u, und = 0u;
      if constexpr (DIM == 3 && !FB) {  // (the first-ball kernel's own generation of 4: no screen)
        // phase A: every iteration of the block through the two certain-reject screens (the
        // ball's bound on u, then the radius-dependent bound); phase B: the survivors in
        // order through the fast and the exact test, the first accept wins.  The wave pays
        // phase B's tests once per survivor round, not once per iteration.
        const float rho0 = g.A0 / g.A1, xabs = 1e-6f * g.R * invNB0;
        const float kz = g.sqrtLambda * -1.44269502f, kb = invNB0 * 1.001f;
        uint32_t surv = 0u;
        // the block's states in stream order, two draws per step (no jump-table reads)
        uint64_t st = s0;
#pragma unroll 4
        for (int b = 0; b < kRejOwnD<DIM, FB>; b++) {
          const float u = draw_float(st);
          DIAG_LANE(D_RITEMS);
          if (!(u > qb0) && !rej_xreject3(u, draw_float(st * kPcgMult + kPcgInc) * g.R, kz, kb, xabs))
            surv |= 1u << b;
          st = st * kPcgMult2 + kPcgInc2;
        }
        for (uint32_t m = surv; m != 0u; m &= m - 1u) {
          const int b = __builtin_ctz(m);
          float u, x;
          rej_draws(prm, s0, b, &u, &x);
          const float rr = x * g.R;
          int dcs = rej_fast_decide3(u, rr, g.sqrtLambda, rho0, invNB0);
          if (dcs < 0) dcs = rej_exact_decide3(u, rr, g.R, g.sqrtLambda, g.A0, g.A1, nrm, bound);
          if (dcs == 1) { jacc = b; done = true; break; }
        }
      } else {
      uint64_t st = s0;  // the block's states in stream order (no jump-table reads)
#pragma unroll 4
      for (int b = 0; b < kRejOwnD<DIM, FB>; b++) {
        const float u = draw_float(st);
        int dcs = 0;
        DIAG_LANE(D_RITEMS);
        if (!(u > qb0)) {
          const float x = draw_float(st * kPcgMult + kPcgInc);
          if constexpr (DIM == 2) {
            dcs = rej_fast_decide(u, x * g.R, g.sqrtLambda, g.A0 / g.A1, invNB0);
          } else {
            const float rr = x * g.R;
            dcs = rej_fast_decide3(u, rr, g.sqrtLambda, g.A0 / g.A1, invNB0);
            if (dcs < 0) dcs = rej_exact_decide3(u, rr, g.R, g.sqrtLambda, g.A0, g.A1, nrm, bound);
          }
        }
        if (dcs == 1) acc |= 1u << b;
        else if (dcs < 0) und |= 1u << b;
        st = st * kPcgMult2 + kPcgInc2;
      }
      for (uint32_t m = acc | und; m != 0u; m &= m - 1u) {
        const int b = __builtin_ctz(m);
        if ((acc >> b) & 1u) { jacc = b; done = true; break; }
        // undecided: the exact test of sample_volume
        float u, x;
        rej_draws(prm, s0, b, &u, &x);
        g.r = x * g.R;
        const float p = g.evaluate() / nrm;
        const float pdfRadius = p / pdf_sphere_uniform<DIM>(g.r);
        if (u < pdfRadius / bound) { jacc = b; done = true; break; }
      }
      }
    }
    j0 = own ? kRejOwnD<DIM, FB> : 0;
#endif
    if (!done) {
      L->s0[lane] = s0;
      L->R[lane] = g.R;
      L->sqrtL[lane] = g.sqrtLambda;
      const float invNB = 1.0f / (nrm * bound);
      L->qb[lane] = rej_quick_bound<DIM>(prm, g.R, g.muR, g.sqrtLambda, invNB);
      if constexpr (DIM == 2) {
        L->c0[lane] = g.A0 / g.A1;
        L->c1[lane] = 1.0f / (nrm * bound);
      } else {
        L->c0[lane] = g.A0;
        L->c1[lane] = g.A1;
        L->rho3[lane] = g.A0 / g.A1;
        L->inv3[lane] = 1.0f / (nrm * bound);
        L->nrm[lane] = nrm;
        L->bound[lane] = bound;
      }
    }
    for (;;) {
      const uint64_t pend = __ballot(!done);
      if (pend == 0) break;
      const int nact = __popcll(pend);
      DIAG_COUNT(D_RGENS, 1);
      // B consecutive iterations per unfinished lane, at least kRejBmin (fewer
      // generations -- each costs three wave syncs and the owners' scan -- for a
      // few iterations evaluated past an accept)
      int B = kWave / nact;
      B = B < kRejBmin<DIM, FB> ? kRejBmin<DIM, FB> : (B > kRejBcap ? kRejBcap : B);
      const int items = nact * B, per = (items + kWave - 1) / kWave;
      // item / B as a multiply-shift (exact: item < 2048, B <= 32, see rej_div)
      const uint32_t mB = (65536u + (uint32_t)B - 1u) / (uint32_t)B;
      if (!done) {
        const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(pend >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)pend, 0u));
        L->owner_of[rank] = (uint32_t)lane;
        L->acc[lane] = 0u;
        L->und[lane] = 0u;
      }
      wave_sync();
      for (int q = 0; q < per; q++) {
        const int item = lane * per + q;
        const int orank = rej_div(item, B, mB), b = item - orank * B;
        if (orank < nact) {
          const int owner = (int)L->owner_of[orank];
          const int j = j0 + b;
          if (j < kRejMax) {
            const uint64_t st = rej_state(prm, L->s0[owner], j);
            const float u = draw_float(st);
            if (WOS_PROBE & 4) {
              const uint64_t st2 = rej_state(prm, probe_opaque(L->s0[owner]), probe_opaque(j));
              const float u2 = draw_float(st2), x2 = draw_float(st2 * kPcgMult + kPcgInc);
              if constexpr (DIM == 2)
                probe_sink(rej_fast_decide(u2, x2 * L->R[owner], L->sqrtL[owner], L->c0[owner], L->c1[owner]));
            }
            int dcs = 0;
            DIAG_LANE(D_RITEMS);
            if (u > L->qb[owner]) {
              // certain reject: the radius draw is not needed
              DIAG_LANE(D_RQUICK);
            } else {
              const float x = draw_float(st * kPcgMult + kPcgInc);
              if constexpr (DIM == 2) {
                dcs = rej_fast_decide(u, x * L->R[owner], L->sqrtL[owner], L->c0[owner], L->c1[owner]);
              } else {
                const float rr = x * L->R[owner];
                dcs = rej_fast_decide3(u, rr, L->sqrtL[owner], L->rho3[owner], L->inv3[owner]);
                if (dcs < 0)
                  dcs = rej_exact_decide3(u, rr, L->R[owner], L->sqrtL[owner], L->c0[owner], L->c1[owner],
                                          L->nrm[owner], L->bound[owner]);
              }
            }
            if (dcs == 1) atomicOr(&L->acc[owner], 1u << b);
            else if (dcs < 0) { atomicOr(&L->und[owner], 1u << b); DIAG_LANE(D_RUND); }
          }
        }
      }
      wave_sync();
      if (!done) {
        const uint32_t acc = L->acc[lane], und = L->und[lane];
        int b = 0;
        while (!done && b < B) {
          if (j0 + b >= kRejMax) { jacc = kRejMax - 1; done = true; break; }  // limit: last radius kept
          const uint32_t m = (acc | und) >> b;
          if (m == 0u) { b = B; break; }
          b += __builtin_ctz(m);
          if (b >= B) break;
          if (j0 + b >= kRejMax) { jacc = kRejMax - 1; done = true; break; }
          if ((acc >> b) & 1u) { jacc = j0 + b; done = true; break; }
          // undecided: the exact test of sample_volume, by the owner
          float u, x;
          rej_draws(prm, s0, j0 + b, &u, &x);
          g.r = x * g.R;
          const float p = g.evaluate() / nrm;
          const float pdfRadius = p / pdf_sphere_uniform<DIM>(g.r);
          if (u < pdfRadius / bound) { jacc = j0 + b; done = true; break; }
          b++;
        }
        if (!done && j0 + B >= kRejMax) { jacc = kRejMax - 1; done = true; }
      }
      j0 += B;
      wave_sync();
    }
    if (coop) {
      float u, x;
      rej_draws(prm, s0, jacc, &u, &x);
      g.r = x * g.R;
      s.state = rej_state(prm, s0, jacc + 1);
      *iters += (uint32_t)(jacc + 1);
      if (need_pdf) *pdf = g.evaluate() / nrm;
      g.r = smax(Gfn<DIM>::rClamp, g.r);
      if (g.r > g.R) g.r = g.R / 2.0f;
      for (int k = 0; k < DIM; k++) { g.yVol[k] = g.c[k] + g.r * dir[k]; out[k] = g.yVol[k]; }
    }
  }
  if (active && !coop) sample_volume<DIM>(prm, g, dir, s, pdf, out, iters, need_pdf);
}

// ---------------------------------------------------------------------------
// walk (walk_on_stars.h:135-329)
// ---------------------------------------------------------------------------
template <int DIM>
struct WalkState {
  float pt[DIM], n[DIM], prevDir[DIM];
  float prevDist, throughput;
  bool onNeumann;
  int walkLength;
  float totalNeumann, totalSource;
  // the source contribution of the last step, added once its texel has arrived:
  // totalSource += pThr * (pNrm * pTex) in the reference's order (walk_on_stars.h:270-275)
  float pThr, pNrm, pTex;
  bool pend;
};

// Fold a deferred source contribution into totalSource (a no-op without one)
template <int DIM>
__device__ __forceinline__ void flush_source(WalkState<DIM>& st) {
  if (st.pend) {
    st.totalSource += st.pThr * (st.pNrm * st.pTex);
    st.pend = false;
  }
}

template <int DIM>
__device__ __forceinline__ float prim_area(const float* P) {
  if constexpr (DIM == 2) {
    float s[2] = {P[2], P[3]};  // record holds v = pb - pa
    return normv<2>(s);
  } else {
    float v1[3], v2[3], n[3];
    for (int k = 0; k < 3; k++) { v1[k] = P[3 + k] - P[k]; v2[k] = P[6 + k] - P[k]; }
    cross3(n, v1, v2);
    return 0.5f * normv<3>(n);
  }
}

// sampleNeumann's primitive choice (fcpw_scene_loader.h:599-620): fcpw's stochastic
// traversal, Mbvh::intersectStochasticFromNode (mbvh.inl:1099-1283), over its wide
// BVH (wos_fcpw_bvh.cpp, read from global memory): ONE root-to-leaf path, at each node
// a child among those whose box overlaps the ball, chosen with probability ~ the
// traversal weight |HarmonicGreensFnFreeSpace<3>::evaluate(max(|c - box centre|, 1e-2))|
// (scene.h:157-160) by rescaling one uniform (u -> u/p or (u-p)/(1-p)); in the leaf a
// primitive overlapping the ball ~ its area (intersectSpherePrimitives, :835-982; all
// of them when the leaf box lies inside the ball).  2D runs in fcpw's 3D frame (z = 0).
// Returns the primitive (-1: no sample) and its selection pdf (weight * traversalPdf) / total.
template <int DIM>
__device__ __forceinline__ int fcpw_stochastic_pick(const DevScene& sc, const float* prims, const float* x, float R,
                                                 float u, float* sel_pdf) {
  constexpr int PS = Layout<DIM>::prim;
  const int B = sc.nbvh_branch;
  const float r2 = R * R;
  const float c[3] = {x[0], x[1], DIM == 3 ? x[2] : 0.0f};
  float tpdf = 1.0f, d2NodeMax = kFltMax;
  int node = 0;
  for (;;) {
    const int32_t* C = sc.nbvh_child + node * B;
    if (C[0] < 0) {
      const bool inside = d2NodeMax <= r2;
      int sel = -1;
      float total = 0.0f, selw = 0.0f, uu = u;
#pragma clang loop unroll(disable)
      for (int p = 0; p < C[3]; p++) {
        const int q = sc.nbvh_ref[C[2] + p];
        const float* P = prims + q * PS;
        float d2 = 0.0f;
        if (!inside) {
          float pt[DIM], t0, t1;
          const float d = cp_prim<DIM>(P, x, pt, &t0, &t1);
          d2 = d * d;
        }
        if (d2 <= r2) {
          const float w = prim_area<DIM>(P);
          total += w;
          const float prob = w / total;
          if (uu < prob) { uu = uu / prob; sel = q; selw = w; }
          else uu = (uu - prob) / (1.0f - prob);
        }
      }
      if (sel < 0) return -1;
      float d = selw * tpdf;
      if (total > 0.0f) d /= total;
      *sel_pdf = d;
      return sel;
    }
    int sel = -1;
    float tot = 0.0f, selw = 0.0f, selmax = 0.0f;
#pragma clang loop unroll(disable)
    for (int w = 0; w < B; w++) {
      if (C[w] == 0x7FFFFFFF) continue;
      const float* bx = sc.nbvh_box + (node * B + w) * 6;
      // overlapWideBox (wide_query_operations.h:96-106)
      float mn[3], mx[3], ct[3];
      for (int k = 0; k < 3; k++) {
        const float a = bx[k] - c[k], b = c[k] - bx[3 + k];
        mn[k] = smax(smax(a, b), 0.0f);
        mx[k] = smin(a, b);
      }
      const float d2min = (mn[0] * mn[0] + mn[1] * mn[1]) + mn[2] * mn[2];
      const float d2max = (mx[0] * mx[0] + mx[1] * mx[1]) + mx[2] * mx[2];
      if (!(d2min <= r2)) continue;
      for (int k = 0; k < 3; k++) ct[k] = c[k] - (bx[k] + bx[3 + k]) * 0.5f;
      const float rr = smax(__builtin_sqrtf((ct[0] * ct[0] + ct[1] * ct[1]) + ct[2] * ct[2]), 1e-2f);
      const float weight = __builtin_fabsf((float)(1.0 / (kFourPi * (double)rr)));
      tot += weight;
      const float prob = weight / tot;
      if (u < prob) { sel = w; selw = weight; selmax = d2max; u = u / prob; }
      else u = (u - prob) / (1.0f - prob);
    }
    if (sel < 0) return -1;
    node = C[sel];
    tpdf *= selw / tot;
    d2NodeMax = selmax;
  }
}

// Neumann boundary sample (walk_on_stars.h:212-260).  With the reference's h == 0
// (scene.h:176-181) the term is exactly +0 unless G or the throughput is
// non-finite; only then the stochastic sample is evaluated -- at every step with
// image-valued h (DevScene::nimg).  flip: this step flipped the walk's normal
// (flipNormalOrientation, double-sided scenes); prec: silhouettePrecision.
template <int DIM, bool RB>
__device__ __forceinline__ void neumann_term(const DevScene& sc, const float* prims, const Gfn<DIM, RB>& g,
                                             WalkState<DIM>& st, float R, const float* rn, bool flip, float prec) {
  constexpr int PS = Layout<DIM>::prim;
  const int np = sc.n_prims;
  const float* x = st.pt;
  float sel_pdf = 0.0f;
  const int sel = fcpw_stochastic_pick<DIM>(sc, prims, x, R, rn[0], &sel_pdf);
  if (sel < 0) return;
  const float* P = prims + sel * PS;
  float sp[DIM], sn[DIM], pdf;
  if constexpr (DIM == 2) {
    float s0 = P[2], s1 = P[3];  // record holds v = pb - pa
    float sv[2] = {s0, s1};
    float area = normv<2>(sv), u = rn[1];
    sp[0] = P[0] + u * s0; sp[1] = P[1] + u * s1;
    sn[0] = s1 / area; sn[1] = -s0 / area;
    pdf = 1.0f / area;
  } else {
    float v1[3], v2[3];
    for (int k = 0; k < 3; k++) { v1[k] = P[3 + k] - P[k]; v2[k] = P[6 + k] - P[k]; }
    cross3(sn, v1, v2);
    float area = normv<3>(sn);
    float u1 = __builtin_sqrtf(rn[1]), u2 = rn[2], u = 1.0f - u1, v = u2 * u1, w = 1.0f - u - v;
    for (int k = 0; k < 3; k++) { sp[k] = P[k] * u + P[3 + k] * v + P[6 + k] * w; sn[k] /= area; }
    pdf = 2.0f / area;
  }
  // Interaction::d = (weight * traversalPdf) / total, then *= samplePoint's pdf (mbvh.inl:1265-1276)
  pdf = sel_pdf * pdf;
  float dts[DIM];
  for (int k = 0; k < DIM; k++) dts[k] = sp[k] - x[k];
  float distToSample = normv<DIM>(dts);
  float alpha = st.onNeumann ? 2.0f : 1.0f;
  if (sc.double_sided) {
    // the sample normal faces the walk (walk_on_stars.h:219-247): flipped with the walk's normal,
    // or when the sample lies behind it beyond the precision band -- on a concave boundary
    // (alpha 2) only when it also lies behind the walk's own normal
    float ds[DIM];
    for (int k = 0; k < DIM; k++) ds[k] = dts[k] / distToSample;
    if (flip) {
      for (int k = 0; k < DIM; k++) sn[k] *= -1.0f;
    } else if (dotv<DIM>(ds, sn) < -prec) {
      bool f = true;
      if (alpha > 1.0f) f = dotv<DIM>(ds, st.n) < -prec;
      if (f)
        for (int k = 0; k < DIM; k++) sn[k] *= -1.0f;
    }
  }
  if (pdf > 0.0f && distToSample < R) {
    float p1[DIM], p2[DIM], mn[DIM];
    for (int k = 0; k < DIM; k++) mn[k] = -st.n[k];
    if (st.onNeumann) offset_point<DIM>(x, mn, p1); else for (int k = 0; k < DIM; k++) p1[k] = x[k];
    for (int k = 0; k < DIM; k++) mn[k] = -sn[k];
    offset_point<DIM>(sp, mn, p2);
    float dd[DIM];
    for (int k = 0; k < DIM; k++) dd[k] = p2[k] - p1[k];
    float dn = normv<DIM>(dd);
    for (int k = 0; k < DIM; k++) dd[k] /= dn;
    if (!ray_occluded<DIM>(prims, np, p1, dd, dn)) {
      float G = g.evaluate_xy(x, sp);
      float hval = DIM == 2 ? neumann_value(sc, sp) : 0.0f;
      st.totalNeumann += st.throughput * alpha * G * hval / pdf;
    }
  }
}

// One iteration of the walk loop (walk_on_stars.h:135-329), split around the
// star-radius query so that the query can run wave-cooperatively:
//   walk_step_begin  -- loop test (Dirichlet distance above the epsilon shell),
//                       double-sided normal flip, whether a silhouette query is due;
//   star_radius_wave -- (convergent, all lanes) computeStarRadius;
//   walk_step_end    -- ball update, direction, ray, source sample, move, roulette.
// Returns -1 while the walk continues, else its termination code.
template <int DIM>
__device__ __forceinline__ int walk_step_begin(const DevScene& sc, const DevParams& prm, float dirichletDist,
                                               WalkState<DIM>& st, bool* flip, bool* query, float firstR = 0.0f) {
  if (!(dirichletDist > prm.epsilon_shell)) return WC_DIRICHLET;
  *flip = false;
  // first step of a boundary-start walk: the precomputed first sphere radius
  // (walk_on_stars.h:148-150), no normal flip, no star-radius query
  if (firstR > 0.0f) { *query = false; return -1; }
  if (sc.double_sided && st.onNeumann) {
    if (st.prevDist > 0.0f && dotv<DIM>(st.prevDir, st.n) < 0.0f) {
      for (int k = 0; k < DIM; k++) st.n[k] *= -1.0f;
      *flip = true;
    }
  }
  *query = !(prm.steps_before_maximal_spheres <= st.walkLength);
  return -1;
}

// ball + direction + ray origin; the ray query follows (walk_on_stars.h:169-210)
template <int DIM, bool RB>
__device__ __forceinline__ float walk_step_mid(const DevParams& prm, float dirichletDist, Pcg32& smp, Gfn<DIM, RB>& g,
                                               WalkState<DIM>& st, uint32_t* steps, bool query, float starQ,
                                               float* dir, float* org, float firstR = 0.0f) {
  float starRadius = dirichletDist;
  if (firstR > 0.0f) {
    starRadius = firstR;
  } else if (query) {
    starRadius = starQ;
    if (prm.min_star_radius <= dirichletDist) starRadius = smax(0.99f * starRadius, prm.min_star_radius);
  }
  g.update_ball(st.pt, starRadius, prm.robust != 0);
  (*steps)++;
  float u[2];
  u[0] = smp.nextf();
  if constexpr (DIM == 3) u[1] = smp.nextf();
  sample_unit_sphere<DIM>(u, dir);
  if (st.onNeumann && dotv<DIM>(st.n, dir) > 0.0f)
    for (int k = 0; k < DIM; k++) dir[k] *= -1.0f;
  if (st.onNeumann) {
    float mn[DIM];
    for (int k = 0; k < DIM; k++) mn[k] = -st.n[k];
    offset_point<DIM>(st.pt, mn, org);
  } else {
    for (int k = 0; k < DIM; k++) org[k] = st.pt[k];
  }
  return starRadius;
}

// after the ray query: the miss point and the Neumann term (walk_on_stars.h:200-260);
// the source sample (convergent, sample_volume_wave) and walk_step_tail follow
// NEU = false: the instantiation for scenes whose Neumann term is provably +0 at every
// step (DevParams::neumann_inert) -- the term's code is compiled out, the draws stay
template <int DIM, bool RB, bool NEU = true>
__device__ __forceinline__ void walk_step_end(const DevScene& sc, const DevParams& prm, const LGeom& G,
                                              Pcg32& smp, Gfn<DIM, RB>& g, WalkState<DIM>& st, float starRadius,
                                              const float* dir, const float* org, bool hit, Hit& ip, bool flip) {
  const int np = sc.n_prims;
  const float* prims = G.prim;
  if (!hit) {
    for (int k = 0; k < DIM; k++) { ip.p[k] = org[k] + starRadius * dir[k]; ip.n[k] = 0.0f; }
    ip.d = starRadius;
  }
  if (!prm.ignore_neumann) {
    float rn[3] = {0.0f, 0.0f, 0.0f};
    for (int k = 0; k < DIM; k++) rn[k] = smp.nextf();
    if constexpr (NEU) {
      bool nonfinite = !__builtin_isfinite(st.throughput) || (g.yukawa == 1 && g.muR > 85.0f);
      if ((nonfinite || sc.nimg != nullptr) && np > 0)
        neumann_term<DIM>(sc, prims, g, st, starRadius, rn, flip, prm.silhouette_precision);
    } else {
      (void)np; (void)prims;
    }
  }
}

// after the source sample (walk_on_stars.h:270-327)
template <int DIM, bool RB>
__device__ __forceinline__ int walk_step_tail(const DevScene& sc, const LGeom& G, const DevParams& prm,
                                              float& dirichletDist,
                                              Pcg32& smp, Gfn<DIM, RB>& g, WalkState<DIM>& st, const float* dir,
                                              bool hit, const Hit& ip, const float* sp) {
  if (!prm.ignore_source) {
    flush_source<DIM>(st);
    if (g.r <= ip.d) {
      st.pNrm = g.norm();
      st.pThr = st.throughput;
      st.pTex = source_value<DIM>(sc, sp);
      st.pend = true;
    }
  }
  if (!hit && outside_bbox<DIM>(sc, ip.p)) return WC_ESCAPED;
  st.prevDist = ip.d;
  for (int k = 0; k < DIM; k++) { st.prevDir[k] = dir[k]; st.pt[k] = ip.p[k]; st.n[k] = ip.n[k]; }
  st.onNeumann = hit;
  st.throughput *= g.dir_sampled_poisson_kernel(st.pt);
  if (st.throughput < prm.rr_threshold) {
    float survival = st.throughput / prm.rr_threshold;
    if (survival < smp.nextf()) { st.throughput = 0.0f; return WC_RR; }
    st.throughput = prm.rr_threshold;
  }
  st.walkLength++;
  if (st.walkLength > prm.max_walk_length) return WC_MAXLEN;
  if (sc.absorption > 0.0f && prm.steps_before_tikhonov == st.walkLength) g.init(true, sc.absorption);
  // the next Dirichlet distance: walk_iteration (dirichlet_dist_step), a lone walk's wave-cooperatively
  (void)dirichletDist;
  return -1;
}

// the Dirichlet distance at the new position of every continuing walk (walk_on_stars.h:324):
// per lane, or wave-cooperatively when only one walk of the wave continues.  Convergent.
template <int DIM>
__device__ __forceinline__ void dirichlet_dist_step(const DevScene& sc, const LGeom& G, bool want, const float* x,
                                                    float& dirichletDist, int lane) {
  if (DIM == 2 && sc.dgrid != nullptr) {
    // the cell grid: a short list per lane (outside the grid: the culled scan)
    if (want) {
      const float d = dirichlet_dist_grid<DIM>(sc, G.dprim, x);
      dirichletDist = d >= 0.0f ? d : dirichlet_dist_culled<DIM>(sc, G.dprim, G.dgroup, x);
    }
    return;
  }
  const uint64_t m = __ballot(want && sc.n_dprims > 0);
  if (m != 0 && (m & (m - 1)) == 0) {
    const int ol = __builtin_ctzll(m);
    float xo[DIM];
    for (int k = 0; k < DIM; k++) xo[k] = lane_bcast(x[k], ol);
    const float d = dirichlet_dist_solo<DIM>(sc, G.dprim, G.dgroup, xo, lane);
    if (want) dirichletDist = d;
    return;
  }
  if (want) dirichletDist = dirichlet_dist_culled<DIM>(sc, G.dprim, G.dgroup, x);
}

// ---------------------------------------------------------------------------
// First ray hit (intersectWithNeumann, fcpw_scene_loader.h:458-484), wave-cooperative.
// The sequential scan keeps the LAST primitive accepted with d <= rt (rt shrinking
// to each accepted d): that is the minimum d, ties to the larger index.  So the
// (lane, primitive) work spreads over the wave like the silhouette query: lanes
// mark the primitive groups their ray segment can reach (slab test with the
// initial tmax), the pairs are compacted, every lane evaluates items with the
// rcp pre-filter + exact test against tmax, and accepted hits fold into the
// owner's atomicMin on (d bits with -0 -> +0, ~index).  The owner then reruns
// the exact test on the winner for the hit record (identical arithmetic).
// ---------------------------------------------------------------------------
constexpr int kRayChunk = 16;
// Scenes with at most this many Neumann primitives (2D segments / 3D triangles) take the per-lane
// scan of ray_hit_wave when two or more lanes query: every lane tests every primitive
#ifndef WOS_RAY_SCAN_MAX2
#define WOS_RAY_SCAN_MAX2 24
#endif
#ifndef WOS_RAY_SCAN_MAX3
#define WOS_RAY_SCAN_MAX3 16
#endif
constexpr int kRayScanMax2 = WOS_RAY_SCAN_MAX2, kRayScanMax3 = WOS_RAY_SCAN_MAX3;

template <int DIM>
struct RayLDS {
  uint32_t list[kWave * kRayChunk];
  float qo[DIM][kWave], qd[DIM][kWave];
  float rt[kWave];
  unsigned long long best[kWave];
};

// rcp pre-filter of one primitive against rt: false only for certain rejections of the exact test
template <int DIM>
__device__ __forceinline__ bool ray_prim_prefilter(const float* P, const float* o, const float* dir, float rt) {
  if constexpr (DIM == 2) {
    const float u0 = P[0] - o[0], u1 = P[1] - o[1];
    const float v0 = P[2], v1 = P[3];
    const float dv = dir[0] * v1 - dir[1] * v0;
    if (!(__builtin_fabsf(dv) > kFltEps)) return false;
    const float ud = u0 * dir[1] - u1 * dir[0];
    const float uv = u0 * v1 - u1 * v0;
    const float ra = __builtin_amdgcn_rcpf(dv);
    const float ta = ud * ra, da = uv * ra;
    if ((ta < 0.0f && __builtin_fabsf(ud) > 1e-30f) || ta > 1.00001f ||
        (da < 0.0f && __builtin_fabsf(uv) > 1e-30f) || da > rt * 1.00001f)
      return false;
  } else {
    float v1[3], v2[3], pp[3], sv[3], q[3];
    for (int k = 0; k < 3; k++) { v1[k] = P[3 + k] - P[k]; v2[k] = P[6 + k] - P[k]; sv[k] = o[k] - P[k]; }
    cross3(pp, dir, v2);
    const float det = dotv<3>(v1, pp);
    if (!(__builtin_fabsf(det) > kFltEps)) return false;
    const float ra = __builtin_amdgcn_rcpf(det);
    const float vn = dotv<3>(sv, pp), va = vn * ra;
    if ((va < 0.0f && __builtin_fabsf(vn) > 1e-30f) || va > 1.00001f) return false;
    cross3(q, sv, v1);
    const float wn = dotv<3>(dir, q), dn = dotv<3>(v2, q);
    const float wa = wn * ra, da = dn * ra;
    if ((wa < 0.0f && __builtin_fabsf(wn) > 1e-30f) || va + wa > 1.00002f ||
        (da < 0.0f && __builtin_fabsf(dn) > 1e-30f) || da > rt * 1.00001f)
      return false;
  }
  return true;
}

// the pre-filter, then the exact test
template <int DIM>
__device__ __forceinline__ bool ray_prim_filtered(const float* P, const float* o, const float* dir, float& rt,
                                                  Hit* h) {
  return ray_prim_prefilter<DIM>(P, o, dir, rt) && ray_prim_exact<DIM>(P, o, dir, rt, h);
}


// Convergent: every lane of the wave calls it; lanes with active == false get false.
// TREE: the primitive-group hierarchy (sc.ptree) replaces the flat group scan when the
// scene has one (the global-memory geometry instantiation).
template <int DIM, bool TREE = false>
__device__ __forceinline__ bool ray_hit_wave(const LGeom& G, const DevScene& sc, bool active, const float* o,
                                             const float* dir, float tmax, Hit* h, RayLDS<DIM>* L, int lane) {
  constexpr int PS = Layout<DIM>::prim;
  const int np = sc.n_prims, ng = sc.n_pgroups;
  const bool need = active && np > 0;
  if (__ballot(need) == 0) return false;
  float inv[DIM];
  for (int k = 0; k < DIM; k++) inv[k] = __builtin_amdgcn_rcpf(dir[k]);
  const bool tree = TREE && sc.ptree.levels > 0;
  const uint64_t nmask = __ballot(need);
  if (!tree && np <= (DIM == 2 ? kRayScanMax2 : kRayScanMax3) && (nmask & (nmask - 1)) != 0) {
    // a handful of primitives (config C's box: 4 segments, the cube: 12 triangles): each querying
    // lane tests every primitive against its own ray with the same pre-filter + exact test as the
    // cooperative items (each against tmax) and keeps the minimum (d bits, ~index) -- no
    // compaction, no LDS, no wave syncs; the same winner, rerun exactly for the hit record.
    // Every primitive is pre-filtered first and the exact test runs on the candidates only: the
    // wave pays it once per candidate round instead of once per primitive (cube walk -3.5 %,
    // profiles/r5ze_ab_ray_scan_split.log)
    bool found = false;
    if (need) {
      unsigned long long best = ~0ull;
      static_assert(kRayScanMax2 <= 32 && kRayScanMax3 <= 32, "candidate mask");
      uint32_t cand = 0u;
      for (int p = 0; p < np; p++)
        if (ray_prim_prefilter<DIM>(G.prim + p * PS, o, dir, tmax)) cand |= 1u << p;
      for (uint32_t m = cand; m != 0u; m &= m - 1u) {
        const int p = __builtin_ctz(m);
        float rt = tmax;
        Hit hh;
        if (ray_prim_exact<DIM>(G.prim + p * PS, o, dir, rt, &hh)) {
          const unsigned long long key = ((unsigned long long)__float_as_uint(hh.d + 0.0f) << 32) |
                                         (0xFFFFFFFFu - (uint32_t)p);
          best = key < best ? key : best;
        }
      }
      if (best != ~0ull) {
        const int p = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull));
        float rt = tmax;
        found = ray_prim_exact<DIM>(G.prim + p * PS, o, dir, rt, h);
        if (found) normalize_rcp<DIM>(h->n);
      }
    }
    return found;
  }
  if (!tree && (nmask & (nmask - 1)) == 0) {
    // one querying lane: lane l tests group g0 + l against the owner's ray, then the
    // primitives of the accepted groups, kGroup lanes per group; the minimum key by a
    // wave reduction instead of LDS atomics
    const int ol = __builtin_ctzll(nmask);
    float oo[DIM], od[DIM], oi[DIM];
    for (int k = 0; k < DIM; k++) { oo[k] = lane_bcast(o[k], ol); od[k] = lane_bcast(dir[k], ol); oi[k] = lane_bcast(inv[k], ol); }
    const float ot = lane_bcast(tmax, ol);
    unsigned long long best = ~0ull;
    for (int g0 = 0; g0 < ng; g0 += kWave) {
      const int gi = g0 + lane;
      uint64_t gm = __ballot(gi < ng && ray_box_maybe<DIM>(G.pgroup + gi * kGroupStride, oo, oi, ot));
      while (gm != 0) {
        // lanes [kGroup q, kGroup (q + 1)) take the q-th accepted group of this round
        uint64_t mm = gm;
        for (int q = lane / kGroup; q > 0 && mm != 0; q--) mm &= mm - 1;
        for (int q = 0; q < kWave / kGroup && gm != 0; q++) gm &= gm - 1;
        if (mm != 0) {
          const int p = (g0 + __builtin_ctzll(mm)) * kGroup + (lane & (kGroup - 1));
          if (p < np) {
            float rt = ot;
            Hit hh;
            if (ray_prim_filtered<DIM>(G.prim + p * PS, oo, od, rt, &hh)) {
              const unsigned long long key =
                  ((unsigned long long)__float_as_uint(hh.d + 0.0f) << 32) | (0xFFFFFFFFu - (uint32_t)p);
              best = key < best ? key : best;
            }
          }
        }
      }
    }
    best = wave_min_u64_solo(best);
    bool found = false;
    if (need && best != ~0ull) {
      const int p = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull));
      float rt = tmax;
      found = ray_prim_exact<DIM>(G.prim + p * PS, o, dir, rt, h);
      if (found) normalize_rcp<DIM>(h->n);
    }
    return found;
  }
  if (need) {
    for (int k = 0; k < DIM; k++) { L->qo[k][lane] = o[k]; L->qd[k][lane] = dir[k]; }
    L->rt[lane] = tmax;
    L->best[lane] = ~0ull;
  }
  int cL = (tree && need) ? sc.ptree.levels : -1, ci = 0;
  for (int g0 = 0;; g0 += kRayChunk) {
    uint32_t mask = 0;
    if (tree) {
      // the window of kRayChunk groups starting at the lowest cursor of the wave; each
      // lane's cursor emits its accepted groups inside it (increasing order)
      g0 = wave_min_int(cL >= 0 ? tree_first(cL, ci) : 0x7FFFFFFF);
      if (g0 == 0x7FFFFFFF) break;
      if (cL >= 0) {
        int gi;
        while ((gi = tree_next(
                    sc.ptree, cL, ci, g0 + kRayChunk,
                    [&](const float* B) { return ray_box_maybe<DIM>(B, o, inv, tmax); },
                    [&](int q) { return ray_box_maybe<DIM>(G.pgroup + q * kGroupStride, o, inv, tmax); })) >= 0)
          mask |= 1u << (gi - g0);
      }
    } else {
      if (g0 >= ng) break;
      if (need) {
        const int gn = (ng - g0) < kRayChunk ? (ng - g0) : kRayChunk;
        for (int j = 0; j < gn; j++)
          if (ray_box_maybe<DIM>(G.pgroup + (g0 + j) * kGroupStride, o, inv, tmax)) mask |= 1u << j;
      }
    }
    const uint32_t cnt = (uint32_t)__popc(mask);
    const uint32_t incl = wave_incl_sum_u32(cnt, lane);
    const uint32_t total = wave_last_u32(incl);
    uint32_t pos = incl - cnt;
    for (uint32_t m = mask; m; m &= m - 1) L->list[pos++] = ((uint32_t)lane << 26) | (uint32_t)(g0 + __builtin_ctz(m));
    wave_sync();
    const uint32_t items = total * kGroup;
    for (uint32_t k = lane; k < items; k += kWave) {
      const uint32_t e = L->list[k / kGroup];
      const int owner = (int)(e >> 26);
      const int p = (int)(e & 0x3FFFFFFu) * kGroup + (int)(k % kGroup);
      if (p >= np) continue;
      float oo[DIM], dd[DIM];
      for (int q = 0; q < DIM; q++) { oo[q] = L->qo[q][owner]; dd[q] = L->qd[q][owner]; }
      float rt = L->rt[owner];
      Hit hh;
      if (ray_prim_filtered<DIM>(G.prim + p * PS, oo, dd, rt, &hh))
        atomicMin(&L->best[owner],
                  ((unsigned long long)__float_as_uint(hh.d + 0.0f) << 32) | (0xFFFFFFFFu - (uint32_t)p));
    }
    wave_sync();
  }
  bool found = false;
  if (need) {
    const unsigned long long key = L->best[lane];
    if (key != ~0ull) {
      const int p = (int)(0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull));
      float rt = tmax;
      found = ray_prim_exact<DIM>(G.prim + p * PS, o, dir, rt, h);
      if (found) normalize_rcp<DIM>(h->n);
    }
  }
  wave_sync();
  return found;
}

// ---------------------------------------------------------------------------
// computeStarRadius (fcpw_scene_loader.h:621-641), wave-cooperative.
//
// The sequential query visits the silhouette candidates in index order, accepts
// a candidate when it is a silhouette with d^2 <= r2 (r2 = the current best,
// initially maxR^2), and stops at the first accepted candidate with d^2 <= minR^2.
// Its result is therefore order-free: the d of the first (lowest-index) accepted
// candidate with d^2 <= minR^2 if there is one, else the d of the candidate with
// the minimum d^2, ties to the larger index -- each candidate judged against
// maxR^2 alone.  So the (lane, candidate) work can be spread over the wave:
//   1. each querying lane marks the silhouette groups it must visit (padded-box
//      distance within maxR, normal cone not certainly front/back facing);
//   2. the (lane, group) pairs are compacted into an LDS list (wave prefix sum);
//   3. all 64 lanes evaluate the candidate items of the list with the exact
//      per-candidate test and fold accepted ones into the owner's LDS slots with
//      atomicMin on (d^2 bits, ~index) and on the index (for the minR break);
//   4. the owner recomputes d of the winning candidate.
// The lane-divergent group loops of the sequential form (the wave paid for the
// union of every lane's groups) become ~(total work)/64 wave iterations.
// ---------------------------------------------------------------------------
constexpr int kStarChunk = 16;  // groups per compaction round: at most 64 * 16 list entries
// The star query's cell lists are copied to the wave list 16 entries per LDS round trip
// (dword reads + alignbyte) instead of one byte read per entry

template <int DIM>
struct StarLDS {
  uint32_t list[kWave * kStarChunk];
  float qx[DIM][kWave];
  float r2[kWave], minR2[kWave];
  uint32_t flip[kWave];
  uint32_t brk[kWave];
  unsigned long long best[kWave];
};

template <int DIM>
__host__ __device__ constexpr size_t walk_scratch_bytes() {
  constexpr size_t a = sizeof(StarLDS<DIM>), b = sizeof(RayLDS<DIM>), c = sizeof(RejLDS);
  return ((a > b ? (a > c ? a : c) : (b > c ? b : c)) + 15) & ~size_t(15);
}

// Exact per-candidate test of the sequential loop against r2 (see star_radius).
template <int DIM>
__device__ __forceinline__ bool star_candidate(const LGeom& G, int s, const float* x, float r2, bool flip,
                                               float prec, float* d2out, float* dout = nullptr) {
  constexpr int SS = Layout<DIM>::sil;
  const float* S = G.sil + s * SS;
  const float miss = DIM == 2 ? S[6] : S[12];
  float view[DIM], d;
  int cls = 2;
  if constexpr (DIM == 2) {
    view[0] = x[0] - S[0]; view[1] = x[1] - S[1];
    const float d2raw = view[0] * view[0] + view[1] * view[1];
    if (d2raw > r2 * 1.000001f) return false;  // certain: fl(fl(sqrt(q))^2) >= q(1 - 2^-22)
    cls = miss != 0.0f ? 1 : silhouette_class2(S, view, d2raw, flip, prec);
    if (cls == 0) return false;
    d = __builtin_sqrtf(d2raw);
  } else {
    float e[3], hl[3];
    for (int k = 0; k < 3; k++) { e[k] = x[k] - 0.5f * (S[k] + S[3 + k]); hl[k] = 0.5f * (S[3 + k] - S[k]); }
    const float dm = __builtin_amdgcn_sqrtf(dotv<3>(e, e)), hr = __builtin_amdgcn_sqrtf(dotv<3>(hl, hl));
    const float lo = dm - hr;
    if (lo > 0.0f && lo * lo > r2 * 1.0001f + 1e-6f * dm * dm) return false;
    float pt[3], t;
    d = cp_segment<3>(S, S + 3, x, pt, &t);
    for (int k = 0; k < 3; k++) view[k] = x[k] - pt[k];
    if (miss != 0.0f) cls = 1;
  }
  const float d2 = d * d;
  if (!(d2 <= r2)) return false;
  if (cls != 1 && !is_silhouette<DIM>(S, view, d, flip, prec)) return false;
  *d2out = d2;
  if (dout) *dout = d;
  return true;
}

// Cell of the star-radius grid holding x (cell = (iz * ny + iy) * nx + ix), or -1
// when there is no grid or x lies outside it.  The host built every cell's list for
// the cell enlarged well beyond the rounding of this index arithmetic.
template <int DIM>
__device__ __forceinline__ int star_cell(const DevScene& sc, const float* x) {
  int c = 0;
  for (int k = DIM - 1; k >= 0; k--) {
    const int nk = sc.sgrid_n[k];
    const float v = (x[k] - sc.sgrid_min[k]) * sc.sgrid_inv[k];
    if (!(v >= 0.0f && v < (float)nk)) return -1;
    int i = (int)v;
    if (i > nk - 1) i = nk - 1;
    c = c * nk + i;
  }
  return c;
}

template <int DIM>
__device__ __forceinline__ float star_candidate_dist(const LGeom& G, int s, const float* x) {
  constexpr int SS = Layout<DIM>::sil;
  const float* S = G.sil + s * SS;
  if constexpr (DIM == 2) {
    const float v0 = x[0] - S[0], v1 = x[1] - S[1];
    return __builtin_sqrtf(v0 * v0 + v1 * v1);
  } else {
    float pt[3], t;
    return cp_segment<3>(S, S + 3, x, pt, &t);
  }
}

// Convergent: every lane of the wave calls it.  Lanes with query == false get 0.
// TREE: the silhouette-group hierarchy (sc.stree) replaces the flat group scan.
template <int DIM, bool TREE = false>
__device__ __forceinline__ float star_radius_wave(const LGeom& G, const DevScene& sc, const DevParams& prm,
                                                  bool query, const float* x, float maxR, bool flipOrient,
                                                  StarLDS<DIM>* L, int lane) {
  DIAG_T0(t_sp);
  const float minR = prm.min_star_radius, prec = prm.silhouette_precision;
  float result = 0.0f, r2 = 0.0f, minR2 = 0.0f;
  bool need = false;
  if (query) {
    if (minR > maxR) {
      result = maxR;
    } else {
      result = smax(maxR, minR);
      if (sc.n_prims > 0) {
        r2 = maxR < kFltMax ? maxR * maxR : kFltMax;
        minR2 = minR * minR;
        need = !(minR2 >= r2);
      }
    }
  }
  // lanes inside the star grid take their cell's short candidate list; the rest
  // (no grid, outside it) share the wave-cooperative group scan below
  DIAG_LONE(lone, query);
  DIAG_ADD_IF(D_L_S_PRE, t_sp, lone);
  DIAG_T0(t_s0);
  int c_beg = 0, c_end = 0;
  bool use_cell = false;
  if (need && G.sgrid != nullptr) {
    const int cell = star_cell<DIM>(sc, x);
    if (cell >= 0) {
      const uint16_t* off = reinterpret_cast<const uint16_t*>(G.sgrid);
      c_beg = off[cell];
      c_end = off[cell + 1];
      use_cell = true;
    }
  }
  const uint64_t nmask = __ballot(need);
  if (nmask == 0) return result;
  if ((nmask & (nmask - 1)) == 0 &&
      __builtin_amdgcn_readlane((int)use_cell, __builtin_ctzll(nmask)) != 0) {
    // one querying lane inside the cell grid: lane l judges entry l of the owner's cell
    // list (64 at a time) against the owner's query; (d^2, ~index) minimum and the
    // lowest index within minR by wave reductions instead of the LDS list and atomics
    const int ol = __builtin_ctzll(nmask);
    float xo[DIM];
    for (int k = 0; k < DIM; k++) xo[k] = lane_bcast(x[k], ol);
    const float r2o = lane_bcast(r2, ol), minR2o = lane_bcast(minR2, ol);
    const bool flo = __builtin_amdgcn_readlane((int)flipOrient, ol) == 0;  // computeStarRadius passes !flip
    const int cb = __builtin_amdgcn_readlane(c_beg, ol), ce = __builtin_amdgcn_readlane(c_end, ol);
    const uint8_t* lst = reinterpret_cast<const uint8_t*>(G.sgrid + G.sgrid_off_words);
    unsigned long long best = ~0ull;
    uint32_t brk = 0xFFFFFFFFu;
    for (int k0 = cb; k0 < ce; k0 += kWave) {
      const int k = k0 + lane;
      if (k < ce) {
        const int sidx = (int)lst[k];
        float d2;
        if (star_candidate<DIM>(G, sidx, xo, r2o, flo, prec, &d2)) {
          const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | (0xFFFFFFFFu - (uint32_t)sidx);
          best = key < best ? key : best;
          if (d2 <= minR2o) brk = (uint32_t)sidx < brk ? (uint32_t)sidx : brk;
        }
      }
    }
    best = wave_min_u64_solo(best);
    brk = wave_min_u32_solo(brk);
    if (need) {
      int sw = -1;
      if (brk != 0xFFFFFFFFu) sw = (int)brk;
      else if (best != ~0ull) sw = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull));
      if (sw >= 0) result = smax(star_candidate_dist<DIM>(G, sw, x), minR);
    }
    return result;
  }
  if (need) {
    for (int k = 0; k < DIM; k++) L->qx[k][lane] = x[k];
    L->r2[lane] = r2;
    L->minR2[lane] = minR2;
    L->flip[lane] = flipOrient ? 0u : 1u;  // computeStarRadius passes !flipNormalOrientation
    L->brk[lane] = 0xFFFFFFFFu;
    L->best[lane] = ~0ull;
  }
  DIAG_ADD_IF(D_L_S_CELL, t_s0, lone);
  DIAG_T0(t_s1);
  if (__ballot(use_cell) != 0) {
    // the (lane, candidate) pairs of all cell lists, spread over the wave in windows
    // of the LDS list: the wave pays for the sum of the list lengths / 64 instead of
    // the longest list; accepted candidates fold into the owner like the group scan
    const uint32_t cnt = use_cell ? (uint32_t)(c_end - c_beg) : 0u;
    const uint32_t incl = wave_incl_sum_u32(cnt, lane);
    const uint32_t total = wave_last_u32(incl);
    const uint32_t first = incl - cnt;
    DIAG_ADD_IF(D_L_S_PFX, t_s1, lone);
    DIAG_T0(t_s2);
    constexpr uint32_t kWin = kWave * kStarChunk;
    for (uint32_t w0 = 0; w0 < total; w0 += kWin) {
      // this lane's entries inside the window, 16 at a time: the list bytes of a batch
      // come from five dword reads issued together (one LDS round trip per batch
      // instead of one per entry), realigned with alignbyte; reads are clamped to the
      // list's last dword
      {
        const uint32_t lo = first < w0 ? w0 - first : 0u;
        const uint32_t hi0 = first + cnt <= w0 + kWin ? cnt : (first < w0 + kWin ? w0 + kWin - first : 0u);
        const uint32_t* lw = G.sgrid + G.sgrid_off_words;
        const uint32_t last_w = cnt > 0u ? ((uint32_t)c_end - 1u) >> 2 : 0u;
        for (uint32_t i = lo; i < hi0; i += 16u) {
          const uint32_t b0 = (uint32_t)c_beg + i, wa = b0 >> 2;
          uint32_t wv[5];
#pragma unroll
          for (int j = 0; j < 5; j++) wv[j] = lw[(wa + (uint32_t)j) < last_w ? wa + (uint32_t)j : last_w];
          uint32_t al[4];
#pragma unroll
          for (int j = 0; j < 4; j++) al[j] = __builtin_amdgcn_alignbyte(wv[j + 1], wv[j], b0 & 3u);
          const uint32_t tag = (uint32_t)lane << 26;
#pragma unroll
          for (int j = 0; j < 16; j++)
            if (i + (uint32_t)j < hi0) L->list[first + i + (uint32_t)j - w0] = tag | ((al[j >> 2] >> (8 * (j & 3))) & 0xFFu);
        }
      }
      wave_sync();
      DIAG_ADD_IF(D_L_S_BUILD, t_s2, lone);
      const uint32_t items = (total - w0) < kWin ? (total - w0) : kWin;
      for (uint32_t k = lane; k < items; k += kWave) {
        const uint32_t e = L->list[k];
        const int owner = (int)(e >> 26);
        const int sidx = (int)(e & 0x3FFFFFFu);
        float xo[DIM];
        for (int q = 0; q < DIM; q++) xo[q] = L->qx[q][owner];
        float d2;
        if (star_candidate<DIM>(G, sidx, xo, L->r2[owner], L->flip[owner] != 0u, prec, &d2)) {
          atomicMin(&L->best[owner], ((unsigned long long)__float_as_uint(d2) << 32) | (0xFFFFFFFFu - (uint32_t)sidx));
          if (d2 <= L->minR2[owner]) atomicMin(&L->brk[owner], (uint32_t)sidx);
        }
      }
      wave_sync();
    }
    DIAG_ADD_IF(D_L_S_WIN, t_s2, lone);
  }
  const bool scan_groups = need && !use_cell;
  const int nsg = sc.n_sgroups, ns = sc.n_sil;
  const bool tree = TREE && sc.stree.levels > 0;
  int cL = (tree && scan_groups) ? sc.stree.levels : -1, ci = 0;
  for (int g0 = 0; __ballot(scan_groups) != 0; g0 += kStarChunk) {
    uint32_t mask = 0;
    if (tree) {
      g0 = wave_min_int(cL >= 0 ? tree_first(cL, ci) : 0x7FFFFFFF);
      if (g0 == 0x7FFFFFFF) break;
      if (cL >= 0) {
        int gi;
        while ((gi = tree_next(
                    sc.stree, cL, ci, g0 + kStarChunk, [&](const float* B) { return ball_box_maybe<DIM>(B, x, r2); },
                    [&](int q) {
                      const float* B = G.sgroup + q * kSGroupStride;
                      return ball_box_maybe<DIM>(B, x, r2) && !cone_culled<DIM>(B, x, prec);
                    })) >= 0)
          mask |= 1u << (gi - g0);
      }
    } else {
      if (g0 >= nsg) break;
      if (scan_groups) {
        const int gn = (nsg - g0) < kStarChunk ? (nsg - g0) : kStarChunk;
        for (int j = 0; j < gn; j++) {
          const float* B = G.sgroup + (g0 + j) * kSGroupStride;
          if (ball_box_maybe<DIM>(B, x, r2) && !cone_culled<DIM>(B, x, prec)) mask |= 1u << j;
        }
      }
    }
    const uint32_t cnt = (uint32_t)__popc(mask);
    const uint32_t incl = wave_incl_sum_u32(cnt, lane);
    const uint32_t total = wave_last_u32(incl);
    uint32_t pos = incl - cnt;
    for (uint32_t m = mask; m; m &= m - 1) L->list[pos++] = ((uint32_t)lane << 26) | (uint32_t)(g0 + __builtin_ctz(m));
    wave_sync();
    const uint32_t items = total * kGroup;
    for (uint32_t k = lane; k < items; k += kWave) {
      const uint32_t e = L->list[k / kGroup];
      const int owner = (int)(e >> 26);
      const int s = (int)(e & 0x3FFFFFFu) * kGroup + (int)(k % kGroup);
      if (s >= ns) continue;
      float xo[DIM];
      for (int q = 0; q < DIM; q++) xo[q] = L->qx[q][owner];
      float d2;
      if (star_candidate<DIM>(G, s, xo, L->r2[owner], L->flip[owner] != 0u, prec, &d2)) {
        atomicMin(&L->best[owner], ((unsigned long long)__float_as_uint(d2) << 32) | (0xFFFFFFFFu - (uint32_t)s));
        if (d2 <= L->minR2[owner]) atomicMin(&L->brk[owner], (uint32_t)s);
      }
    }
    wave_sync();
  }
  DIAG_T0(t_s3);
  if (need) {
    const uint32_t b = L->brk[lane];
    const unsigned long long key = L->best[lane];
    int s = -1;
    if (b != 0xFFFFFFFFu) s = (int)b;
    else if (key != ~0ull) s = (int)(0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull));
    if (s >= 0) result = smax(star_candidate_dist<DIM>(G, s, x), minR);
  }
  wave_sync();
  DIAG_ADD_IF(D_L_S_FIN, t_s3, lone);
  DIAG_ADD_IF(D_L_S_POST, t_sp, lone);
  return result;
}

// ---------------------------------------------------------------------------
// the solve: three kernels over one batch of points
// ---------------------------------------------------------------------------
//   1. wos_first_ball_kernel  -- one wave per query point (atomic point queue):
//      closest-point setup + inside test, the per-point stratified samples (all
//      lanes at once from a PCG32 jump-ahead table staged in LDS; the Fisher-Yates
//      shuffle resolved wave-parallel, exactly), then lane = antithetic pair: source sample + boundary
//      direction of the first ball for both members (walk_on_stars.h:494-575).
//      Each member becomes a walk task in HBM (start state + its record fields).
//   2. wos_walk_kernel        -- persistent: every lane runs one walk task at a
//      time, one step per loop iteration; a lane whose walk ends takes the next
//      task from its wave's window of the global task queue at the next
//      iteration, so lanes never idle behind the longest walk of a point.
//   3. wos_fold_kernel        -- one lane per point: the statistics in walk order
//      (Welford means with sequential control variates, walk_on_stars.h:500-506,
//      583-614, 744-877) and the masked outputs (grid.h:155-179, 207-237).
// The three stages touch HBM only for the task hand-off (~48 B per walk in 2D).  It is most of
// the walk kernel's traffic -- karman: 134 MB of start-state reads and 99 MB of record write-backs
// per launch, DESIGN.md "HBM bytes of the walk kernel" -- but 2 % of HBM bandwidth over the
// kernel's time: the walk arithmetic, not the hand-off, sets the time.

// stratifiedSample (sampling.h:435-457) on the per-point stream, drawn in parallel:
// draw k of the stream is pcg_output(A_k * s0 + C_k).  Diagonal draws k < n*sd;
// the shuffle's bounded draws follow in order (k = n*sd + i*n + j) unless one of
// them hits PCG's rejection threshold, in which case lane 0 replays the shuffle
// draws sequentially from the true stream.

// The shuffle `for j: swap(a[j], a[partner[j]])` (partner[j] >= j), wave-parallel
// and exact.  Position j is final after step j and receives the value position
// q = partner[j] holds just before step j.  Let V(k) be the original index held by
// position k just before step k: V(k) = V(link(k)) where link(k) = the last step
// m < k with partner[m] = k (it moved V(m) into k and nothing wrote k since), or k
// itself if no step wrote k.  Then the final a'[j] = a[P(j)] with P(j) = V(j) when
// q = j, else V(pred(j)) with pred(j) = the last step m < j with partner[m] = q,
// or q if none.  link is an atomicMax; V resolves by pointer jumping (chains are
// short for random partners); pred is the predecessor among equal targets, found
// chunk by chunk (64 steps) with a lane mask per target plus the running last
// writer of earlier chunks.  Scratch: 7 words per stratum (fb_union_bytes).
__device__ __forceinline__ void lhs_permute(float* strat, const int* partner, int nstrat, int sd, int dimi,
                                            char* scratch, int lane) {
  int* link = reinterpret_cast<int*>(scratch);
  int* val = link + nstrat;
  int* last = val + nstrat;
  int* perm = last + nstrat;
  float* tmp = reinterpret_cast<float*>(perm + nstrat);
  unsigned long long* cmask = reinterpret_cast<unsigned long long*>(tmp + nstrat + (nstrat & 1));
  const int* pd = partner + dimi * nstrat;
  for (int j = lane; j < nstrat; j += kWave) { link[j] = -1; last[j] = -1; cmask[j] = 0ull; }
  wave_sync();
  for (int j = lane; j < nstrat; j += kWave) {
    const int q = pd[j];
    if (q != j) atomicMax(&link[q], j);
  }
  wave_sync();
  for (int j = lane; j < nstrat; j += kWave) val[j] = j;
  wave_sync();
  // pointer jumping: link[j] >= 0 means "V(j) = V(link[j])", unresolved
  for (;;) {
    bool pending = false;
    int nl[4], nv[4];
    for (int c = 0, j = lane; j < nstrat; j += kWave, c++) {
      const int p = link[j];
      nl[c] = p;
      nv[c] = val[j];
      if (p >= 0) {
        const int pp = link[p];
        if (pp < 0) { nv[c] = val[p]; nl[c] = -1; } else { nl[c] = pp; pending = true; }
      }
    }
    wave_sync();
    for (int c = 0, j = lane; j < nstrat; j += kWave, c++) { link[j] = nl[c]; val[j] = nv[c]; }
    wave_sync();
    if (!__any(pending)) break;
  }
  // predecessor among steps with the same target, 64 steps at a time
  for (int c0 = 0; c0 < nstrat; c0 += kWave) {
    const int j = c0 + lane;
    const int q = j < nstrat ? pd[j] : j;
    const bool mover = j < nstrat && q != j;
    if (mover) atomicOr(&cmask[q], 1ull << lane);
    wave_sync();
    int P = 0;
    if (j < nstrat) {
      if (!mover) {
        P = val[j];
      } else {
        const unsigned long long below = cmask[q] & ((1ull << lane) - 1ull);
        const int pred = below ? c0 + 63 - __builtin_clzll(below) : last[q];
        P = pred >= 0 ? val[pred] : q;
      }
      perm[j] = P;
    }
    wave_sync();
    if (mover) { atomicMax(&last[q], j); cmask[q] = 0ull; }
    wave_sync();
  }
  for (int j = lane; j < nstrat; j += kWave) tmp[j] = strat[sd * perm[j] + dimi];
  wave_sync();
  for (int j = lane; j < nstrat; j += kWave) strat[sd * j + dimi] = tmp[j];
  wave_sync();
}

// per-wave first-ball scratch after the stratified samples and partners: the
// rejection sampler's LDS, or (before it) the shuffle scratch of lhs_permute -- only
// for 129..256 strata (fewer: lhs_permute_reg, in registers; more: the serial shuffle)
__host__ __device__ constexpr size_t fb_union_bytes(int lhs_floats, int nstrat) {
  const size_t a = sizeof(RejLDS),
               b = (nstrat > 2 * kWave && nstrat <= 4 * kWave) ? (size_t)28 * lhs_floats + 64 : 0;
  return ((a > b ? a : b) + 15) & ~size_t(15);
}

// Query points per first-ball wave.  One lane runs one antithetic pair, so a point
// with n_pairs <= 32 (64 walks or fewer: config D's 64 walks are 32 pairs) would leave
// lanes n_pairs..63 out of the per-pair arithmetic; the wave takes
// min(64 / n_pairs, kFbMaxPack) consecutive points of the queue instead, lane l
// running pair l % n_pairs of point slot l / n_pairs.  Each point's stratified
// samples are built in turn into its own LDS slot; seeds stay keyed by the global
// point index, so results do not depend on the packing.  The cap bounds the
// sequential stratified-sample builds per wave for tiny n_pairs.
constexpr int kFbMaxPack = 4;
__host__ __device__ constexpr int fb_points_per_wave(int n_pairs) {
  return (n_pairs > 0 && 2 * n_pairs <= kWave)
             ? (kWave / n_pairs < kFbMaxPack ? kWave / n_pairs : kFbMaxPack)
             : 1;
}

// The same permutation P(j) as lhs_permute, computed in registers: no LDS scratch, no
// atomics, no wave syncs.  Element e = 64 r + lane of a shuffle lives in chunk r (R chunks,
// nstrat <= 64 R).  For each chunk the wave ballots every bit of the partners; the lanes of
// chunk r whose partner equals t are then the AND over bits b of (ballot_b or its
// complement, as bit b of t), so link(k) and pred(j) are the highest such lane below the
// element (chunks below it entirely).  V resolves by pointer jumping and the final values by
// one lane permute (ds_bpermute) per chunk.  Up to MM shuffles (m0 .. m0 + M - 1; shuffle m
// is dimension m % SD of slot m / SD: samples at strat0 + slot * slot_floats, partners at
// part0 + slot * slot_floats + dim * nstrat) run side by side for instruction-level overlap.
template <int B0, int B1>
__device__ __forceinline__ uint64_t partner_bits_match(const uint64_t* bc, uint32_t t) {
  uint32_t lo = ~0u, hi = ~0u;
#pragma unroll
  for (int b = B0; b < B1; b++) {
    const uint32_t s = (uint32_t)((int32_t)(t << (31 - b)) >> 31);  // all ones when bit b of t is set
    lo &= ~((uint32_t)bc[b] ^ s);
    hi &= ~((uint32_t)(bc[b] >> 32) ^ s);
  }
  return ((uint64_t)hi << 32) | lo;
}

template <int R>
__device__ __forceinline__ int chunk_fetch(const int* v, int e) {  // element e of a shuffle's R chunks
  int r = __shfl(v[0], e & (kWave - 1));
#pragma unroll
  for (int c = 1; c < R; c++) {
    const int t = __shfl(v[c], e & (kWave - 1));
    r = (e >> 6) == c ? t : r;
  }
  return r;
}

template <int SD, int R, int MM>
__device__ __forceinline__ void lhs_permute_reg_body(float* strat0, const int* part0, int slot_floats, int m0, int M,
                                                     int nstrat, int lane) {
  constexpr int C = MM * R, NB = R == 1 ? 6 : (R == 2 ? 7 : 8);
  const uint64_t below = (1ull << lane) - 1ull;
  int q[C], L[C], V[C], a[C];
  uint64_t bc[C][NB], vc[C];
#pragma unroll
  for (int c = 0; c < C; c++) {
    const int m = m0 + c / R, e = (c % R) * kWave + lane;
    const bool ok = c / R < M && e < nstrat;
    const float* st = strat0 + (m / SD) * slot_floats;
    const int* pd = part0 + (m / SD) * slot_floats + (m % SD) * nstrat;
    q[c] = ok ? pd[e] : e;
    a[c] = ok ? __float_as_int(st[SD * e + m % SD]) : 0;
    vc[c] = __ballot(ok);
#pragma unroll
    for (int b = 0; b < NB; b++) bc[c][b] = __ballot(ok && ((q[c] >> b) & 1));
  }
  // link(k): the last step m < k with partner[m] = k (k's high bits are its chunk, a constant)
#pragma unroll
  for (int c = 0; c < C; c++) {
    const int r = c % R, c0 = c - r;
    int l = -1;
#pragma unroll
    for (int s = 0; s <= r; s++) {
      uint64_t mk = vc[c0 + s] & partner_bits_match<0, 6>(bc[c0 + s], (uint32_t)lane) &
                    partner_bits_match<6, NB>(bc[c0 + s], (uint32_t)(r * kWave));
      if (s == r) mk &= below;
      if (mk) l = s * kWave + 63 - __builtin_clzll(mk);
    }
    L[c] = l;
    V[c] = r * kWave + lane;
  }
  // V(k) = V(link(k)), by pointer jumping
  for (;;) {
    bool pending = false;
    int nl[C], nv[C];
#pragma unroll
    for (int c = 0; c < C; c++) {
      const int c0 = c - c % R, p = L[c] < 0 ? 0 : L[c];
      const int pl = chunk_fetch<R>(L + c0, p), pv = chunk_fetch<R>(V + c0, p);
      nl[c] = L[c];
      nv[c] = V[c];
      if (L[c] >= 0) {
        if (pl < 0) { nv[c] = pv; nl[c] = -1; } else { nl[c] = pl; pending = true; }
      }
    }
#pragma unroll
    for (int c = 0; c < C; c++) { L[c] = nl[c]; V[c] = nv[c]; }
    if (!__any(pending)) break;
  }
  // a'[j] = a[P(j)]: V(j) for a fixed point, else V(pred(j)), or q if no earlier step targets q
  int out[C];
#pragma unroll
  for (int c = 0; c < C; c++) {
    const int r = c % R, c0 = c - r, j = r * kWave + lane, qj = q[c];
    int pr = -1;
#pragma unroll
    for (int s = 0; s <= r; s++) {
      uint64_t mk = vc[c0 + s] & partner_bits_match<0, NB>(bc[c0 + s], (uint32_t)qj);
      if (s == r) mk &= below;
      if (mk) pr = s * kWave + 63 - __builtin_clzll(mk);
    }
    const int vp = chunk_fetch<R>(V + c0, pr < 0 ? 0 : pr);
    const int Pv = qj == j ? V[c] : (pr >= 0 ? vp : qj);
    out[c] = chunk_fetch<R>(a + c0, Pv);
  }
#pragma unroll
  for (int c = 0; c < C; c++) {
    const int m = m0 + c / R, e = (c % R) * kWave + lane;
    if (c / R < M && e < nstrat) strat0[(m / SD) * slot_floats + SD * e + m % SD] = __int_as_float(out[c]);
  }
  wave_sync();
}

// Out of line: inlined, the element arrays cost the first-ball kernels registers across the
// whole point loop (measured: within noise of inline for 2D, slower for 3D).
template <int SD, int R, int MM>
__device__ __attribute__((noinline)) void lhs_permute_reg(float* strat0, const int* part0, int slot_floats, int m0,
                                                          int M, int nstrat, int lane) {
  lhs_permute_reg_body<SD, R, MM>(strat0, part0, slot_floats, m0, M, nstrat, lane);
}

// A wave's stratified samples (every point slot, every dimension) are shuffled in one
// lhs_permute_reg pass when they fit its registers, instead of one pass per slot and dimension
__host__ __device__ constexpr bool lhs_all_fits(int n_pairs, int dim, int P) {
  // 3D only: a 2D wave with one point has one shuffle, and the out-of-line pass costs the 2D
  // first-ball kernel spills
  return dim == 3 &&
         P * (dim - 1) * ((2 * n_pairs + kWave - 1) / kWave == 3 ? 4 : (2 * n_pairs + kWave - 1) / kWave) <= 4;
}

// The jump constants of the stratified samples' first prm.lhs_jump_n draws, staged by the
// first-ball kernel in its dynamic LDS after the per-wave regions (the host sizes the table:
// at most kLhsJumpMax entries, none when it would cost the kernel a block per CU).  The draws
// then wait on no global load -- a global one also waited, in order, for the next point's
// coordinates and state the kernel prefetches just before (vmcnt counts loads in issue order).
__device__ __forceinline__ uint64_t lhs_jump_state(const DevParams& prm, const unsigned long long* ljump, uint64_t s0,
                                                   int k) {
  if (k < prm.lhs_jump_n) return ljump[2 * k] * s0 + ljump[2 * k + 1];
  return jump_state(prm, s0, k);
}

template <int DIM>
__device__ __forceinline__ void build_lhs(const DevParams& prm, const unsigned long long* ljump, int64_t gidx, float* strat,
                                          int* partner, char* scratch, int lane, bool permute = true) {
  constexpr int sd = DIM - 1;
  const int nstrat = 2 * prm.n_pairs;
  const int nd = nstrat * sd;
  Pcg32 ps;
  ps.seed(seed32(prm.seed, (uint64_t)gidx, 0, 0));
  const uint64_t s0 = ps.state;
  const float ome = 1.0f - kFltEps;
  const float inv = 1.0f / (float)nstrat;
  for (int idx = lane; idx < nd; idx += kWave) {
    const int i = sd == 1 ? idx : idx / sd;
    const uint32_t r = pcg_output(lhs_jump_state(prm, ljump, s0, idx));
    const float u = bits_to_float((r >> 9) | 0x3f800000u) - 1.0f;
    strat[idx] = smin(((float)i + u) * inv, ome);
  }
  bool rej = false;
  for (int idx = lane; idx < nd; idx += kWave) {
    const int j = sd == 1 ? idx : idx % nstrat;
    const uint32_t bound = (uint32_t)(nstrat - j);
    const uint32_t r = pcg_output(lhs_jump_state(prm, ljump, s0, nd + idx));
    // PCG's rejection threshold th = 2^32 mod bound < bound: only r < bound can fall below it
    if (r < bound) rej |= r < (~bound + 1u) % bound;
    partner[idx] = j + (int)(r % bound);
  }
  const bool any_rej = __any(rej);
  wave_sync();
  if (any_rej) {  // exact replay of the sequential stream (rare: P ~ n^2 / 2^32)
    if (lane == 0) {
      Pcg32 q;
      q.state = jump_state(prm, s0, nd);
      for (int i = 0; i < sd; ++i)
        for (int j = 0; j < nstrat; ++j) partner[i * nstrat + j] = j + (int)q.bounded((uint32_t)(nstrat - j));
    }
    wave_sync();
  }
  if (!permute) return;  // the caller shuffles (lhs_permute_reg over every slot)
  if (nstrat <= 2 * kWave) {
    for (int i = 0; i < sd; ++i) {
      if (nstrat <= kWave) lhs_permute_reg<sd, 1, 1>(strat, partner, 0, i, 1, nstrat, lane);
      else lhs_permute_reg<sd, 2, 1>(strat, partner, 0, i, 1, nstrat, lane);
    }
    return;
  }
  if (nstrat <= 4 * kWave) {
    for (int i = 0; i < sd; ++i) lhs_permute(strat, partner, nstrat, sd, i, scratch, lane);
    return;
  }
  if (lane == 0) {  // more strata than lhs_permute's per-lane registers: the serial shuffle
    for (int i = 0; i < sd; ++i)
      for (int j = 0; j < nstrat; ++j) {
        const int other = partner[i * nstrat + j];
        const float t = strat[sd * j + i];
        strat[sd * j + i] = strat[sd * other + i];
        strat[sd * other + i] = t;
      }
  }
  wave_sync();
}

// The first ball of pair w, both antithetic members (walk_on_stars.h:510-575);
// member a becomes task t0 + a.
// Called by every lane of the wave (the 3D source sample is wave-cooperative;
// 2D keeps the per-lane loop: measured faster for first balls, r1d);
// lanes with active == false run pair 0's arithmetic for nothing (helping the
// cooperative sampler) and write and count nothing.
// 2D first balls: K0, I0, K1, I1 at the sampled radius from one fused Bessel evaluation
// (pdf and gradient norm), and the second member reuses the first's gradient norm when its
// radius is the same float -- identical values, fewer double-precision exp / sqrt / divisions
template <int DIM, bool RB>
__device__ __forceinline__ void first_balls(const DevScene& sc, const DevParams& prm, const DevTasks& tk,
                                            const float* x, float firstR, const float* strat, int64_t gidx,
                                            bool active, int w, int64_t t0, bool yuk0, uint32_t* iters,
                                            RejLDS* rejL, int lane, const float* pb, const float* dn) {
  constexpr int sd = DIM - 1;
  if (DIM == 2 && !active) return;
  if (!active) w = 0;
  uint32_t dummy_iters = 0;
  if (!active) iters = &dummy_iters;
  const int64_t T = tk.T;
  float boundaryPdf = 0.0f, sourcePdf = 0.0f, boundaryPt[DIM], sourcePt[DIM];
  for (int k = 0; k < DIM; k++) { boundaryPt[k] = 0.0f; sourcePt[k] = 0.0f; }
  Pcg32 fs;
  fs.seed(seed32(prm.seed, (uint64_t)gidx, (uint64_t)w, 1));
  // the first ball (centre x, radius firstR) is the same for both members: its
  // Bessel constants are evaluated once (identical values either way)
  DIAG_T0(t_upd);
  Gfn<DIM, RB> g0;
  g0.init(yuk0, sc.absorption);
  if constexpr (!RB && DIM == 2) {
    // the Bessel members at mu R from the point-setup kernel (DevTasks::pball)
    if (g0.yukawa) g0.set_ball(x, firstR, pb);
    else g0.update_ball(x, firstR, false);
  } else {
    g0.update_ball(x, firstR, prm.robust != 0);
  }
  DIAG_ADD(D_FB_UPD, t_upd);
  // 2D: member a's sampled radius and its gradient norm (r_a < 0: none), reused by member b
  float r_a = -1.0f, gn_a = 0.0f;
  for (int a = 0; a < prm.n_anti; a++) {
    DIAG_T0(t_mem);
    const int64_t t = t0 + a;
    Gfn<DIM, RB> g = g0;
    float throughput = 1.0f, totalSource = 0.0f, firstSource = 0.0f;
    float sdir[DIM], bdir[DIM];
    for (int k = 0; k < DIM; k++) sdir[k] = 0.0f;
    if (!prm.ignore_source) {
      if (a == 0) {
        DIAG_T0(t_smp);
        float dir[DIM];
        sample_unit_sphere<DIM>(&strat[sd * (2 * w + 0)], dir);
        if constexpr (DIM == 3) {
          sample_volume_wave<DIM, RB, true>(prm, active, g, dir, fs, &sourcePdf, sourcePt, iters, true, rejL, lane);
        } else if (g.yukawa == 1) {
          // the pdf (K0, I0 at the sampled mu r, before the clamps) and the gradient norm
          // (K1, I1 at the clamped mu r) from one fused evaluation when the clamps kept r
          float rpre;
#if WOS_DIAG
          const uint32_t it0 = *iters;
#endif
          sample_volume<DIM>(prm, g, dir, fs, &sourcePdf, sourcePt, iters, false, &rpre);
#if WOS_DIAG
          {
            const uint32_t itn = *iters - it0;
            uint32_t mx = itn, sm = itn;
            for (int off = kWave / 2; off > 0; off >>= 1) {
              mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
              sm += (uint32_t)__shfl_xor((int)sm, off);
            }
            if (lane == 0) { atomicAdd(&s_diag[D_FB_ITSUM], (unsigned long long)sm); atomicAdd(&s_diag[D_FB_ITMAX], (unsigned long long)mx); }
          }
#endif
          const float nrm = g.norm();
          if (rpre == g.r) {
            double i0, k0, i1, k1;
            bessel_ik<true, true>((double)(g.r * g.sqrtLambda), &i0, &k0, &i1, &k1);
            sourcePdf = g.evaluate_k0i0(k0, i0) / nrm;
            gn_a = g.gradient_norm_k1i1(k1, i1);
          } else {
            const float rc = g.r;
            g.r = rpre;
            sourcePdf = g.evaluate() / nrm;
            g.r = rc;
            gn_a = g.gradient_norm();
          }
          r_a = g.r;
        } else {
          sample_volume<DIM>(prm, g, dir, fs, &sourcePdf, sourcePt, iters, true);
        }
        DIAG_ADD(D_FB_SMP, t_smp);
      } else {
        float sdv[DIM];
        for (int k = 0; k < DIM; k++) sdv[k] = sourcePt[k] - x[k];
        for (int k = 0; k < DIM; k++) g.yVol[k] = x[k] - sdv[k];
        g.r = normv<DIM>(sdv);
      }
      float gnorm = g.norm();
      float contrib = gnorm * source_value<DIM>(sc, g.yVol);
      totalSource += throughput * contrib;
      firstSource = contrib;
      float gr[DIM];
      if (DIM == 2 && g.yukawa == 1 && g.r == r_a) {
        // gradient() with the norm of member a's identical radius (same value)
        for (int k = 0; k < DIM; k++) gr[k] = (g.yVol[k] - g.c[k]) * gn_a;
      } else {
        g.gradient(gr);
      }
      float den = sourcePdf * gnorm;
      for (int k = 0; k < DIM; k++) sdir[k] = gr[k] / den;
    }
    if (a == 0) {
      const float* u = &strat[sd * (2 * w + 1)];
      float bd[DIM];
      if (prm.use_cosine) {
        if constexpr (DIM == 2) {
          float u1 = 2.0f * u[0] - 1.0f;
          bd[0] = u1; bd[1] = __builtin_sqrtf(smax(0.0f, 1.0f - u1 * u1));
        } else {
          float u1 = 2.0f * u[0] - 1.0f, u2 = 2.0f * u[1] - 1.0f, dx = 0.0f, dy = 0.0f;
          if (!(u1 == 0 && u2 == 0)) {
            float theta, rr;
            if (__builtin_fabsf(u1) > __builtin_fabsf(u2)) { rr = u1; theta = (float)(0.25 * kPi * (double)(u2 / u1)); }
            else { rr = u2; theta = (float)(0.5 * kPi * (double)(1.0f - 0.5f * (u1 / u2))); }
            float sn, cs;
            fsincos(theta, &sn, &cs);
            dx = rr * cs; dy = rr * sn;
          }
          bd[0] = dx; bd[1] = dy; bd[2] = __builtin_sqrtf(smax(0.0f, 1.0f - (dx * dx + dy * dy)));
        }
        if (fs.nextf() < 0.5f) bd[DIM - 1] *= -1.0f;
        float ct = __builtin_fabsf(bd[DIM - 1]);
        float pdfc = DIM == 2 ? ct / 2.0f : (float)((double)ct / kPi);
        boundaryPdf = 0.5f * pdfc;
        // transformCoordinates (sampling.h:176-203) with n = directionForDerivative
        // (dn: the point's own, e.g. a BVC Dirichlet sample's normal; else (1, 0[, 0]))
        if constexpr (DIM == 2) {
          const float n0 = dn ? dn[0] : 1.0f, n1 = dn ? dn[1] : 0.0f;
          float s0 = n1, s1 = -n0;
          float q0 = bd[0] * s0 + bd[1] * n0, q1 = bd[0] * s1 + bd[1] * n1;
          bd[0] = q0; bd[1] = q1;
        } else {
          const float n[3] = {dn ? dn[0] : 1.0f, dn ? dn[1] : 0.0f, dn ? dn[2] : 0.0f};
          float sign = __builtin_copysignf(1.0f, n[2]);
          const float aa = -1.0f / (sign + n[2]);
          const float b = n[0] * n[1] * aa;
          float b1[3] = {1.0f + sign * n[0] * n[0] * aa, sign * b, -sign * n[0]};
          float b2[3] = {b, sign + n[1] * n[1] * aa, -n[1]};
          float q[3];
          for (int k = 0; k < 3; k++) q[k] = bd[0] * b1[k] + bd[1] * b2[k] + bd[2] * n[k];
          for (int k = 0; k < 3; k++) bd[k] = q[k];
        }
      } else {
        sample_unit_sphere<DIM>(u, bd);
        boundaryPdf = pdf_sphere_uniform<DIM>(1.0f);
      }
      for (int k = 0; k < DIM; k++) { g.ySurf[k] = g.c[k] + g.R * bd[k]; boundaryPt[k] = g.ySurf[k]; }
    } else {
      float bd[DIM];
      for (int k = 0; k < DIM; k++) bd[k] = boundaryPt[k] - x[k];
      for (int k = 0; k < DIM; k++) g.ySurf[k] = x[k] - bd[k];
    }
    throughput *= g.poisson_kernel() / boundaryPdf;
    {
      float pg[DIM];
      g.poisson_kernel_gradient(pg);
      float den = boundaryPdf * throughput;
      for (int k = 0; k < DIM; k++) bdir[k] = pg[k] / den;
    }
    DIAG_ADD(a == 0 ? D_FB_MA : D_FB_MB, t_mem);
    if (!active) continue;
    DIAG_T0(t_st);
    tk.first[t] = firstSource;
    for (int k = 0; k < DIM; k++) {
      tk.bdir[k * T + t] = bdir[k];
      tk.sdir[k * T + t] = sdir[k];
      tk.pt[k * T + t] = g.ySurf[k];
    }
    tk.thr[t] = throughput;
    tk.tsrc[t] = totalSource;
    // without Dirichlet geometry the distance is the bbox far corner of the walk start,
    // recomputed by the walk kernel from the same floats instead of stored and reloaded
    if (sc.n_dprims > 0) {
      // the Dirichlet cell grid where it covers the point (2D), else the culled scan
      float d = -1.0f;
      if (DIM == 2 && sc.dgrid) d = dirichlet_dist_grid<DIM>(sc, sc.dprim, g.ySurf);
      tk.dd[t] = d >= 0.0f ? d : dirichlet_dist_culled<DIM>(sc, sc.dprim, sc.dgroup, g.ySurf);
    }
    DIAG_ADD(D_FB_ST, t_st);
  }
}

// LDS image: prims | silhouettes | prim groups | silhouette groups (each block 16-B aligned)
template <int DIM, bool GG>
__device__ __forceinline__ LGeom geometry_view(const DevScene& sc, float* smem, bool with_sil, bool copy) {
  constexpr int PS = Layout<DIM>::prim, SS = Layout<DIM>::sil;
  const int primN = sc.n_prims * PS, silN = sc.n_sil * SS;
  const int primAl = (primN + 3) & ~3, silAl = (silN + 3) & ~3;
  const int pgN = sc.n_pgroups * kGroupStride, sgN = sc.n_sgroups * kSGroupStride;
  LGeom G;
  if constexpr (GG) {  // too large for LDS: the same records, read through L2
    G.prim = sc.prim;
    G.sil = sc.sil;
    G.pgroup = sc.pgroup;
    G.sgroup = sc.sgroup;
    G.sgrid = with_sil ? sc.sgrid : nullptr;
    G.sgrid_off_words = sc.sgrid_off_words;
    G.dprim = sc.dprim;
    G.dgroup = sc.dgroup;
    return G;
  }
  G.prim = smem;
  G.sil = smem + primAl;
  G.pgroup = smem + primAl + silAl;
  G.sgroup = G.pgroup + pgN;
  uint32_t* gw = reinterpret_cast<uint32_t*>(smem + primAl + silAl + pgN + sgN);
  G.sgrid = (with_sil && sc.sgrid != nullptr) ? gw : nullptr;
  G.sgrid_off_words = sc.sgrid_off_words;
  const int sgridAl = sc.sgrid != nullptr ? ((sc.sgrid_words + 3) & ~3) : 0;
  const int dpN = sc.n_dprims * PS, dpAl = (dpN + 3) & ~3, dgN = sc.n_dgroups * kGroupStride;
  float* dbase = smem + primAl + silAl + pgN + sgN + sgridAl;
  G.dprim = with_sil ? dbase : sc.dprim;
  G.dgroup = with_sil ? dbase + dpAl : sc.dgroup;
  if (!copy) return G;
  for (int i = threadIdx.x; i < primN; i += kBlock) smem[i] = sc.prim[i];
  if (with_sil) {
    for (int i = threadIdx.x; i < silN; i += kBlock) smem[primAl + i] = sc.sil[i];
    for (int i = threadIdx.x; i < pgN; i += kBlock) smem[primAl + silAl + i] = sc.pgroup[i];
    for (int i = threadIdx.x; i < sgN; i += kBlock) smem[primAl + silAl + pgN + i] = sc.sgroup[i];
    if (sc.sgrid != nullptr)
      for (int i = threadIdx.x; i < sc.sgrid_words; i += kBlock) gw[i] = sc.sgrid[i];
    for (int i = threadIdx.x; i < dpN; i += kBlock) dbase[i] = sc.dprim[i];
    for (int i = threadIdx.x; i < dgN; i += kBlock) dbase[dpAl + i] = sc.dgroup[i];
  }
  return G;
}

template <int DIM, bool GG>
__device__ __forceinline__ LGeom stage_geometry(const DevScene& sc, float* smem, bool with_sil) {
  return geometry_view<DIM, GG>(sc, smem, with_sil, true);
}

// Kernel parameters re-read inside a loop: the view goes through an opaque copy of
// the pointer to the kernarg block, so every use in an iteration is a scalar load
// (scalar-cache hit) instead of a value held in SGPRs for the whole kernel.  The
// walk kernel's loop-invariant scene / parameter / task fields and the constants
// hoisted next to them otherwise overflow the SGPR file, whose spills into VGPR
// lanes then push the VGPRs into scratch.
// The walk kernel's parameters as they lie in the kernarg segment (the ABI lays the
// arguments out like the members of this struct: declaration order, natural alignment).
struct WalkKernArgs {
  DevScene sc;
  DevParams prm;
  DevTasks tk;
};
using KernArgsPtr = const __attribute__((address_space(4))) WalkKernArgs*;
__device__ __forceinline__ KernArgsPtr kernargs_opaque() {
  KernArgsPtr q = (KernArgsPtr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(q));
  return q;
}

__device__ __forceinline__ void flush_counter(unsigned long long* counters, int slot, uint32_t v, int lane) {
  unsigned long long s = v;
  for (int off = kWave / 2; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0 && s) atomicAdd(&counters[slot], s);
}

// per-point state bits written by the first-ball kernel
enum { kPtEstimate = 1, kPtMaskP = 2, kPtMaskG = 4 };

// ---- kernel 1: point setup + first balls ----------------------------------
constexpr unsigned int kPtGrab = 2;  // points per queue atomic of the first-ball kernel
// 3D: 3 waves/SIMD (168 VGPRs, 16-28 B/lane of spills) instead of the unconstrained 2:
// first balls -20 % on the cube configs (profiles/r2u_ab_fb3d_occupancy.log)
#ifndef WOS_FB_WAVES_PER_EU
#define WOS_FB_WAVES_PER_EU 3
#endif
// 2D: 4 waves/SIMD (128 VGPRs, 28 B/lane of spills) beats the unconstrained 155 VGPRs at
// 3 waves/SIMD: first balls -2 % on karman, -10 % on config C (A/B, profiles/r2t_ab_fb_occupancy.log)
#ifndef WOS_FB_WAVES_PER_EU2
#define WOS_FB_WAVES_PER_EU2 4
#endif

// Sample point setup: createSolutionGrid (grid.h:85-101) + insideDomain
// (fcpw_scene_loader.h:642-648) from the two closest-point queries, the masks of the
// outputs (grid.h:155-179, 207-237) and the cost bucket of the point.  Cost buckets
// order both queues: walks from points close to the boundary (small first ball) run
// longest, so the walk queue takes high buckets first; first balls cost ~ their
// radius (11.2 R rejection iterations per Yukawa sample at lambda = 350, the max over
// the 64 lanes of a wave), so the presorted first-ball queue runs the buckets in the
// opposite order.  Returns the pstate word; firstR = 0.99 min(dDist, nDist).
template <int DIM>
__device__ __forceinline__ int32_t point_state(const DevScene& sc, const DevParams& prm, float nDist, float nSigned,
                                               float dDist, float dSigned, int* bucket_out, float* firstR) {
  const bool inside = !sc.watertight ? true
                      : (__builtin_fabsf(dSigned) < __builtin_fabsf(nSigned) ? dSigned < 0.0f : nSigned < 0.0f);
  const bool estimate = inside || sc.double_sided || prm.force_estimate;
  const float mask = prm.boundary_distance_mask;
  const bool maskP = __builtin_fabsf(nDist) < mask;
  const bool maskG = (!inside && !sc.double_sided) || __builtin_fabsf(nDist) < mask;
  const float bd = smin(dDist, nDist);
  int bucket = 0;
  if (estimate) {
    const float l2 = __builtin_amdgcn_logf(smax(bd, 1e-9f));  // log2
    bucket = (int)sclamp((int)(-2.0f * l2) + 8, 1, kCostBuckets - 1);
  }
  *bucket_out = bucket;
  *firstR = 0.99f * bd;
  return (estimate ? kPtEstimate : 0) | (maskP ? kPtMaskP : 0) | (maskG ? kPtMaskG : 0) | (bucket << 8);
}

// lanes per point of the setup kernel's small-mesh scans: 4 measured -9 us on karman,
// +13 / +20 us on C / the cube (profiles/r2s_ab_setup_lanes.log): 1
#ifndef WOS_SETUP_LANES
#define WOS_SETUP_LANES 1
#endif
constexpr int kSetupLanes = WOS_SETUP_LANES;  // lanes per point of wos_point_setup_kernel (power of two)
#ifndef WOS_SETUP_LDS_FLOATS
#define WOS_SETUP_LDS_FLOATS 4096
#endif
constexpr int kSetupLdsFloats = WOS_SETUP_LDS_FLOATS;  // 16 KB: 1024 segments / 455 triangles
static_assert((kSetupLanes & (kSetupLanes - 1)) == 0 && kSetupLanes <= kWave, "kSetupLanes");
// Point setup: one point per kSetupLanes lanes (the exact scans of closest_lane), pstate +
// first-ball radius per point, the cost-bucket histogram of the walk queue and (2D Yukawa,
// reference float semantics) the first ball's Bessel members at mu R.  The first-ball kernel
// then takes the points in plain point order from an atomic queue.
template <int DIM>
__global__ __launch_bounds__(256) void wos_point_setup_kernel(const DevScene sc, const DevParams prm,
                                                             const float* __restrict__ pts, int64_t n,
                                                             const DevTasks tk) {
  __shared__ uint32_t s_hist[kCostBuckets];
  // small boundaries staged in LDS: every lane scans every record (broadcast reads)
  // instead of one global round trip per primitive
  __shared__ __attribute__((aligned(16))) float s_prim[kSetupLdsFloats];
  constexpr int PS = Layout<DIM>::prim;
  const int nfl = sc.n_prims * PS, dfl = sc.n_dprims * PS;
  const bool lds_n = nfl <= kSetupLdsFloats, lds_d = nfl + dfl <= kSetupLdsFloats;
  if (lds_n)
    for (int k = threadIdx.x; k < nfl; k += blockDim.x) s_prim[k] = sc.prim[k];
  if (lds_d)
    for (int k = threadIdx.x; k < dfl; k += blockDim.x) s_prim[nfl + k] = sc.dprim[k];
  if (threadIdx.x < kCostBuckets) s_hist[threadIdx.x] = 0u;
  __syncthreads();
  const float* nprim = lds_n ? s_prim : sc.prim;
  const float* dprim = lds_d ? s_prim + nfl : sc.dprim;
  // kSetupLanes adjacent lanes per point share the small-mesh scans (closest_lane);
  // the first of them writes the point's state
  const int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = gi / kSetupLanes;
  const int sub = (int)(gi % kSetupLanes);
  if (i < n) {
    float x[DIM];
    for (int k = 0; k < DIM; k++) x[k] = pts[i * DIM + k];
    float nDist = kFltMax, nSigned = kFltMax;
    if (sc.n_prims > 0) {
      const Closest c = closest_lane<DIM>(nprim, sc.pgroup, sc.n_prims, sc.n_pgroups, x, sub, kSetupLanes);
      nDist = c.d;
      nSigned = signed_dist<DIM>(sc.paux, c, x);
    }
    float dDist, dSigned;
    if (sc.n_dprims > 0) {
      const Closest c = closest_lane<DIM>(dprim, sc.dgroup, sc.n_dprims, sc.n_dgroups, x, sub, kSetupLanes);
      dDist = c.d;
      dSigned = signed_dist<DIM>(sc.dpaux, c, x);
    } else {
      dDist = dSigned = bbox_far_dist<DIM>(sc, x);
    }
    int bucket;
    float firstR;
    const int32_t ps = point_state<DIM>(sc, prm, nDist, nSigned, dDist, dSigned, &bucket, &firstR);
    if (sub == 0) {
      tk.pstate[i] = ps;
      tk.prad[i] = firstR;
      if constexpr (DIM == 2) {
        // robust solves (RB first-ball kernels) evaluate the scaled members themselves and never
        // read these (pre = !RB && ...): skip the double-precision work
        if (tk.pball != nullptr && !prm.robust && (ps & kPtEstimate) && sc.absorption > 0.0f &&
            prm.steps_before_tikhonov == 0) {
          Gfn<2> g;
          g.init(true, sc.absorption);
          g.update_ball(x, firstR, false);
          tk.pball[i] = g.A0;
          tk.pball[tk.pball_stride + i] = g.A1;
          tk.pball[2 * tk.pball_stride + i] = g.B0;
          tk.pball[3 * tk.pball_stride + i] = g.B1;
        }
      }
      atomicAdd(&s_hist[bucket], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x < kCostBuckets && s_hist[threadIdx.x]) atomicAdd(&tk.hist[threadIdx.x], s_hist[threadIdx.x]);
}

// RB: robust float semantics (DevParams::robust; Gfn::scaled) -- separate instantiations
// (wos_robust.hip), so the reference-semantics kernels carry none of its code.
// wos_point_setup_kernel ran first: point i's state and first-ball radius are read
// from pstate / prad (no geometry is staged: the first balls query none).
template <int DIM, bool RB = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(DIM == 2 ? WOS_FB_WAVES_PER_EU2 : WOS_FB_WAVES_PER_EU))) void wos_first_ball_kernel(
    const DevScene sc, const DevParams prm, const float* __restrict__ pts, int64_t n, int64_t base, int64_t stride,
    const DevTasks tk, unsigned long long* __restrict__ counters, unsigned int* __restrict__ work, int lhs_floats) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int npairs = prm.n_pairs;
  // P points per wave (fb_points_per_wave): slot s holds its stratified samples and
  // shuffle partners at wbase + 2 s lhs_floats; the rejection sampler's / shuffle's
  // scratch follows the P slots; the block's staged jump constants follow the waves
  const int P = fb_points_per_wave(npairs);
  const int wave_floats = 2 * P * lhs_floats + (int)(fb_union_bytes(P * lhs_floats, 2 * npairs) / sizeof(float));
  float* wbase = smem + wave * wave_floats;
  unsigned long long* ljump = reinterpret_cast<unsigned long long*>(smem + (int)(blockDim.x / kWave) * wave_floats);
  stage_rej_jump(prm);
  for (int i = threadIdx.x; i < 2 * prm.lhs_jump_n; i += blockDim.x) ljump[i] = prm.jump[i];
#if WOS_DIAG
  if (threadIdx.x < D_NUM) s_diag[threadIdx.x] = 0u;
#endif
  __syncthreads();
  RejLDS* rejL = reinterpret_cast<RejLDS*>(wbase + 2 * P * lhs_floats);
  // this lane's point slot and pair (P == 1: all lanes serve the one point, pairs w0 + lane);
  // span = lanes per slot, so lane s * span is slot s's first lane (wave-uniform)
  const int span = P > 1 ? npairs : kWave;
  const int slot = P > 1 ? lane / npairs : 0;
  const int wl = lane - slot * span;
  const bool used = slot < P;
  const int myslot = used ? slot : 0;

  uint32_t c_iters = 0, c_pts = 0;
  const bool yuk0 = sc.absorption > 0.0f && prm.steps_before_tikhonov == 0;

  // point queue, one chunk of P points ahead: the next index is taken (and each lane's
  // point coordinates, radius and state loaded) while the current chunk is processed, so
  // neither the queue atomic nor the point loads sit on a point's critical path.  Points
  // are taken kPtGrab chunks at a time (one queue atomic per grab: a single-address
  // atomic per point serialises at ~13 ns, which had bounded the whole kernel).
  const unsigned int take = kPtGrab * (unsigned int)P;
  unsigned int idx = 0;
  if (lane == 0) idx = atomicAdd(work, take);
  idx = __shfl(idx, 0);
  unsigned int cend = idx + take;
  float xn[DIM], rn = 0.0f;
  bool en = false;
  // 2D Yukawa, reference semantics: the first ball's Bessel members come from the setup kernel
  const bool pre = !RB && DIM == 2 && yuk0;
  float bn[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  {
    const unsigned int li = idx + (unsigned int)myslot;
    for (int k = 0; k < DIM; k++) xn[k] = (int64_t)li < n ? pts[(int64_t)li * DIM + k] : 0.0f;
    if ((int64_t)li < n) {
      rn = tk.prad[li];
      en = (tk.pstate[li] & kPtEstimate) != 0;
      if (pre)
        for (int k = 0; k < 4; k++) bn[k] = tk.pball[k * tk.pball_stride + li];
    }
  }
  for (;;) {
    if ((int64_t)idx >= n) break;
    float x[DIM];
    for (int k = 0; k < DIM; k++) x[k] = xn[k];
    float firstR = rn;
    const bool estimate = en && used;
    float pb[4];
    for (int k = 0; k < 4; k++) pb[k] = bn[k];
    const bool grab = idx + (unsigned int)P >= cend;  // wave-uniform
    unsigned int nidx_l0 = 0;
    if (grab && lane == 0) nidx_l0 = atomicAdd(work, take);
    DIAG_T0(t_fb0);
    // the next chunk: its index (the atomic has returned by now), coordinates, radius, state
    unsigned int nidx, ncend = cend;
    if (grab) {
      nidx = (unsigned int)__shfl((int)nidx_l0, 0);
      ncend = nidx + take;
    } else {
      nidx = idx + (unsigned int)P;
    }
    {
      const unsigned int li = nidx + (unsigned int)myslot;
      for (int k = 0; k < DIM; k++) xn[k] = (int64_t)li < n ? pts[(int64_t)li * DIM + k] : 0.0f;
      en = false;
      if ((int64_t)li < n) {
        rn = tk.prad[li];
        en = (tk.pstate[li] & kPtEstimate) != 0;
        if (pre)
          for (int k = 0; k < 4; k++) bn[k] = tk.pball[k * tk.pball_stride + li];
      }
    }
    // estimated slots: bit s * span set when point idx + s is estimated
    const uint64_t em = __ballot(estimate && wl == 0);
    if (em == 0) { idx = nidx; cend = ncend; continue; }
    c_pts += lane == 0 ? (uint32_t)__popcll(em) : 0u;
    DIAG_ADD(D_FB_SETUP, t_fb0);
    DIAG_COUNT(D_FB_PTS, __popcll(em));
    DIAG_T0(t_fb1);
    const bool all = lhs_all_fits(npairs, DIM, P);
    for (int s = 0; s < P; s++) {
      if (!all && !((em >> (s * span)) & 1ull)) continue;
      float* strat_s = wbase + 2 * s * lhs_floats;
      build_lhs<DIM>(prm, ljump, base + (int64_t)(idx + (unsigned int)s) * stride, strat_s,
                     reinterpret_cast<int*>(strat_s + lhs_floats), reinterpret_cast<char*>(rejL), lane, !all);
    }
    if constexpr (DIM == 3)
      if (all) {
        const int ns = 2 * npairs;
        const int* part0 = reinterpret_cast<const int*>(wbase + lhs_floats);
        if (ns <= kWave) lhs_permute_reg<DIM - 1, 1, 4>(wbase, part0, 2 * lhs_floats, 0, P * (DIM - 1), ns, lane);
        else lhs_permute_reg<DIM - 1, 2, 2>(wbase, part0, 2 * lhs_floats, 0, P * (DIM - 1), ns, lane);
      }
    DIAG_ADD(D_FB_LHS, t_fb1);
    DIAG_T0(t_fb2);
    // lanes without a point of their own (an unestimated slot, or beyond P slots) run the
    // first estimated slot's pair-0 arithmetic and write nothing (3D: they still serve the
    // cooperative sampler)
    const int fs = (int)(__builtin_ctzll(em) / (unsigned)span);
    const int es = estimate ? myslot : fs;
    if (!estimate) {
      for (int k = 0; k < DIM; k++) x[k] = lane_bcast(x[k], fs * span);
      firstR = lane_bcast(firstR, fs * span);
      for (int k = 0; k < 4; k++) pb[k] = lane_bcast(pb[k], fs * span);
    }
    const unsigned int pidx = idx + (unsigned int)es;
    const int64_t gidx = base + (int64_t)pidx * stride;
    const float* strat = wbase + 2 * es * lhs_floats;
    const int wend = P > 1 ? 1 : npairs;
    for (int w0 = 0; w0 < wend; w0 += kWave) {
      const int w = w0 + wl;
      first_balls<DIM, RB>(sc, prm, tk, x, firstR, strat, gidx, estimate && w < npairs, w,
                           (int64_t)pidx * tk.wpp + (int64_t)w * prm.n_anti, yuk0, &c_iters, rejL, lane,
                           pb, tk.ddir ? tk.ddir + (int64_t)pidx * DIM : nullptr);
    }
    DIAG_ADD(D_FB_BALLS, t_fb2);
    DIAG_ADD(D_FB_TOTAL, t_fb0);
    DIAG_MAX(D_FB_MAX, __builtin_amdgcn_s_memtime() - t_fb0);
    wave_sync();
    idx = nidx;
    cend = ncend;
  }
  flush_counter(counters, C_ITERS, c_iters, lane);
  flush_counter(counters, C_PTS, c_pts, lane);
#if WOS_DIAG
  __syncthreads();
  if (threadIdx.x < D_NUM) {
    if (diag_is_max(threadIdx.x)) atomicMax(&g_diag[threadIdx.x], s_diag[threadIdx.x]);
    else atomicAdd(&g_diag[threadIdx.x], s_diag[threadIdx.x]);
  }
#endif
}

// issue priority of the calling wave (s_setprio takes an immediate), uniform level 0..3
__device__ __forceinline__ void wave_priority(int level) {
  if (level == 1) __builtin_amdgcn_s_setprio(1);
  else if (level == 2) __builtin_amdgcn_s_setprio(2);
  else if (level >= 3) __builtin_amdgcn_s_setprio(3);
}

// ---- kernel 2: walks ---------------------------------------------------------
// The state a walk task starts from (the hand-out of walk_on_stars.h:494-579 after
// the first ball; BSTART: estimateSolution's boundary start, :437-439) ...
template <int DIM, bool BSTART, bool RB>
__device__ __forceinline__ void walk_start(const DevScene& sc, const DevParams& prm, const DevTasks& tk, int64_t t,
                                           uint32_t pidx, uint32_t w, const float* v_pt, float v_thr, float v_tsrc,
                                           float v_dd, int64_t base, int64_t stride, bool yuk0, WalkState<DIM>& st,
                                           Gfn<DIM, RB>& g, Pcg32& ws, float& ddist, uint32_t& wsteps, float& firstR) {
  for (int kk = 0; kk < DIM; kk++) { st.pt[kk] = v_pt[kk]; st.n[kk] = 0.0f; st.prevDir[kk] = 0.0f; }
  // prevDir/prevDist only matter once the walk stands on a Neumann boundary,
  // and every step rewrites them before that can happen
  st.prevDist = 0.0f;
  st.throughput = v_thr;
  st.onNeumann = false;
  st.walkLength = 0;
  st.totalNeumann = 0.0f;
  st.totalSource = v_tsrc;
  st.pend = false;
  ddist = v_dd;
  g.init(yuk0, sc.absorption);
  if constexpr (BSTART) {
    // WalkState(pt, currentNormal, prevDirection = normal, FLT_MAX, 1, onNeumann)
    // (walk_on_stars.h:437-439); walk w of sample pidx on its own stream
    for (int kk = 0; kk < DIM; kk++) { st.n[kk] = tk.n0[kk * tk.T + t]; st.prevDir[kk] = st.n[kk]; }
    st.prevDist = kFltMax;
    const uint32_t fl = tk.sflags[t];  // bit 0: starts on the Neumann boundary; bits 8..15: seed tag
    st.onNeumann = (fl & 1u) != 0u;
    firstR = tk.r0[t];
    ws.seed(seed32(prm.seed, (uint64_t)(base + (int64_t)pidx * stride), (uint64_t)w, (fl >> 8) & 0xFFu));
    wsteps = 0;
  } else {
    ws.seed(seed32(prm.seed, (uint64_t)(base + (int64_t)pidx * stride), (uint64_t)w, 2));
    wsteps = 1;  // the first ball
  }
}

// One iteration of the walk loop for every lane of the wave (convergent): the lanes
// with active == false take part in the cooperative queries only.  Returns the
// termination code (>= 0) or -1 while the walk continues.
template <int DIM, bool GG, bool BSTART, bool RB, bool NEU = true>
__device__ __forceinline__ int walk_iteration(const DevScene& sc, const DevParams& prm, const LGeom& G, bool active,
                                              WalkState<DIM>& st, Gfn<DIM, RB>& gc, Pcg32& ws, float& ddist,
                                              uint32_t& wsteps, float& firstR, StarLDS<DIM>* starL,
                                              RayLDS<DIM>* rayL, RejLDS* rejL, uint32_t* c_iters, int lane) {
  DIAG_T0(t_step);
  // This step's ball: only the Green's function's kind carries over from step to step (its
  // absorption is the scene's -- every Gfn::init takes sc.absorption -- and update_ball rebuilds
  // the ball before any use), so the ball's members are locals of the iteration instead of
  // loop-carried registers of the persistent loop (3D walk kernel scratch 108 -> 40 B/lane)
  Gfn<DIM, RB> g;
  g.yukawa = gc.yukawa; g.lambda = sc.absorption; g.sqrtLambda = __builtin_sqrtf(sc.absorption);
  int code = -1;
  DIAG_LONE(lone, active);
  bool flip = false, query = false;
  if (active) code = walk_step_begin<DIM>(sc, prm, ddist, st, &flip, &query, BSTART ? firstR : 0.0f);
  DIAG_T0(t_star);
  const float starQ = star_radius_wave<DIM, GG>(G, sc, prm, active && code < 0 && query, st.pt, ddist, flip, starL, lane);
  if (WOS_PROBE & 8) {
    float px[DIM];
    for (int k = 0; k < DIM; k++) px[k] = probe_opaque(st.pt[k]);
    probe_sink(star_radius_wave<DIM, GG>(G, sc, prm, active && code < 0 && query, px, probe_opaque(ddist), flip, starL,
                                         lane));
  }
  DIAG_ADD_LONE(D_STAR, D_L_STAR, t_star, lone);
  const bool live = active && code < 0;
  float dir[DIM], org[DIM], starR = 0.0f;
  for (int k = 0; k < DIM; k++) { dir[k] = 1.0f; org[k] = 0.0f; }
  DIAG_T0(t_mid);
  if (live) starR = walk_step_mid<DIM>(prm, ddist, ws, g, st, &wsteps, query, starQ, dir, org, BSTART ? firstR : 0.0f);
  DIAG_ADD_LONE(D_MID, D_L_MID, t_mid, lone);
  Hit ip;
  DIAG_T0(t_ray);
  const bool hit = ray_hit_wave<DIM, GG>(G, sc, live, org, dir, starR, &ip, rayL, lane);
  if (WOS_PROBE & 16) {
    Hit ip2;
    float po[DIM];
    for (int k = 0; k < DIM; k++) po[k] = probe_opaque(org[k]);
    probe_sink(ray_hit_wave<DIM, GG>(G, sc, live, po, dir, probe_opaque(starR), &ip2, rayL, lane) ? ip2.d : 0.0f);
  }
  DIAG_ADD_LONE(D_RAY, D_L_RAY, t_ray, lone);
  DIAG_T0(t_end);
  if (live) walk_step_end<DIM, RB, NEU>(sc, prm, G, ws, g, st, starR, dir, org, hit, ip, flip);
  DIAG_ADD_LONE(D_END, D_L_END, t_end, lone);
  float sp[DIM], pdf_unused;
  for (int k = 0; k < DIM; k++) sp[k] = 0.0f;
  DIAG_T0(t_smp);
  if ((WOS_PROBE & 32) && !prm.ignore_source) {
    Gfn<DIM, RB> g2 = g;
    Pcg32 ws2 = ws;
    ws2.state = probe_opaque(ws2.state);
    float sp2[DIM], pdf2;
    uint32_t it2 = 0;
    sample_volume_wave<DIM>(prm, live, g2, dir, ws2, &pdf2, sp2, &it2, false, rejL, lane);
    probe_sink(sp2[0]);
  }
  if (!prm.ignore_source) sample_volume_wave<DIM>(prm, live, g, dir, ws, &pdf_unused, sp, c_iters, false, rejL, lane);
  DIAG_ADD_LONE(D_SAMPLE, D_L_SAMPLE, t_smp, lone);
  DIAG_T0(t_tail);
  if (live) code = walk_step_tail<DIM>(sc, G, prm, ddist, ws, g, st, dir, hit, ip, sp);
  dirichlet_dist_step<DIM>(sc, G, live && code < 0, st.pt, ddist, lane);
  if (BSTART) firstR = 0.0f;  // firstStep = false (walk_on_stars.h:325)
  DIAG_ADD_LONE(D_TAIL, D_L_TAIL, t_tail, lone);
  DIAG_ADD_LONE(D_STEP, D_L_STEP, t_step, lone);
  if (live) gc.yukawa = g.yukawa;
  return code;
}

// the record of a finished walk (walk_on_stars.h:583-585: escaped and over-length walks are dropped)
template <int DIM>
__device__ __forceinline__ void walk_finish(const DevScene& sc, const DevParams& prm, const DevTasks& tk, int64_t t,
                                            int code, WalkState<DIM>& st, uint32_t wsteps, unsigned int* s_ctr) {
  flush_source<DIM>(st);
  const bool recorded = code == WC_DIRICHLET || code == WC_RR;
  if (recorded) {
    const float term = (code == WC_DIRICHLET && !prm.ignore_dirichlet) ? dirichlet_value<DIM>(sc, st.pt) : 0.0f;
    const float tot = st.throughput * term + st.totalNeumann + st.totalSource;
    if (!WOS_ACCT_NOREC) tk.total[t] = tot;
  }
  if (!WOS_ACCT_NOREC) tk.code[t] = (wsteps << 1) | (recorded ? 1u : 0u);
  DIAG_MAX(D_WMAXLEN, wsteps);
  atomicAdd(&s_ctr[recorded ? C_STEPS : C_WASTED], wsteps);
  atomicAdd(&s_ctr[code == WC_DIRICHLET ? C_DIR : code == WC_RR ? C_RR : code == WC_ESCAPED ? C_ESC : C_MAXL], 1u);
}

__device__ __forceinline__ void flush_walk_counters(unsigned long long* counters, const unsigned int* s_ctr) {
  if (threadIdx.x < C_NUM && threadIdx.x != C_ITERS && threadIdx.x != C_PTS) {
    unsigned int v = threadIdx.x == C_REC ? s_ctr[C_RR] + s_ctr[C_DIR] : s_ctr[threadIdx.x];
    if (v) atomicAdd(&counters[threadIdx.x], (unsigned long long)v);
  }
}

#ifndef WOS_TASK_GRAB
#define WOS_TASK_GRAB 64
#endif
constexpr unsigned int kTaskGrab = WOS_TASK_GRAB;  // tasks a wave takes from the global queue at once
#ifndef WOS_TASK_GRAB3
#define WOS_TASK_GRAB3 128u  // the same in 3D (wos_walk_kernel kGrabD)
#endif
// The walk queue is dealt round-robin over kTaskQueues counters in windows of kTaskGrab
// tasks (queue x serves windows x, x + Q, x + 2Q, ... of the cost order): a wave draws
// from the counter of its block's home queue and, once that one is exhausted, from the
// others in turn.  Each counter sits on its own 64-byte line (kTaskQueueStride u32), so
// the device-scope atomics of small windows do not serialize on one address.
#ifndef WOS_TASK_QUEUES
#define WOS_TASK_QUEUES 8
#endif
constexpr unsigned int kTaskQueues = WOS_TASK_QUEUES;
// head windows of 16 tasks (32 before round 5): karman -1 %, stride-8 shard -1.5 %, the hardest point alone -6 to -8 %,
// C and D unchanged (profiles/r5zi_ab_fb_order_head16.log, r5zj_ab_queue_knobs.log; 8 slowed the hardest point)
#ifndef WOS_TASK_GRAB_HEAD
#define WOS_TASK_GRAB_HEAD 16
#endif
#ifndef WOS_TASK_HEAD
#define WOS_TASK_HEAD 1
#endif
constexpr unsigned int kTaskGrabHead = WOS_TASK_GRAB_HEAD;  // window of the queue's head
constexpr unsigned int kTaskHead = WOS_TASK_HEAD;           // head windows per wave of the grid
static_assert((kTaskQueues & (kTaskQueues - 1)) == 0 && kTaskQueues <= (unsigned)kMaxTaskQueues, "power of two");


// ---- tail spreading inside a workgroup ------------------------------------------
// Once the walk queue is dry, a wave whose walks have all ended would leave its SIMD
// idle while a sibling wave of the same workgroup still carries many walks, each of
// its iterations paying for all of them.  Instead the idle wave announces itself
// (s_idle), and a sibling with >= 2 live walks hands it the upper half of them: the
// whole per-lane walk state, word for word, through the idle wave's LDS scratch (which
// it is not using) -- the walks continue bit for bit on another SIMD.  s_busy counts
// the waves holding walks (a donor counts its recipient before handing over), so an
// idle wave leaves once it reaches 0: no walk is left anywhere in the workgroup and
// none can appear (the queue is dry).
// The kernels with SPR = true hand over (2D, LDS geometry; chosen per solve,
// DevParams::tail_spread); 3D keeps SPR = false (its extra live state costs the throughput
// path scratch that its short tails do not return).  Only the loop-carried state moves.
constexpr int kSpreadMax = 32;  // walks per hand-over
// words of one walk's state between two steps: WalkState, the Green's function's kind (its
// absorption is the scene's, and its ball -- c, R, r, y*, muR and the Bessel members -- is rebuilt
// by update_ball before any use in the next step: walk_iteration), the PCG32 state, ddist,
// wsteps, task
template <int DIM>
constexpr int walk_pack_words() { return (3 * DIM + 6 + 4) + 1 + 2 + 3; }
// every member is moved (the struct sizes, bools padded to a word, match the counts)
static_assert(sizeof(WalkState<2>) == 4 * (3 * 2 + 6 + 4), "WalkState<2> members");
static_assert(sizeof(WalkState<3>) == 4 * (3 * 3 + 6 + 4), "WalkState<3> members");
static_assert(sizeof(Gfn<2, false>) == 4 * (1 + 3 * 2 + 9) && sizeof(Gfn<3, true>) == 4 * (1 + 3 * 3 + 9), "Gfn members");
static_assert(sizeof(Pcg32) == 8, "Pcg32 state");
// one walk's state into / out of mailbox slot `slot` (word-major, kSpreadMax slots per word)
template <int DIM, bool RB>
__device__ __forceinline__ void spread_put(uint32_t* mb, int slot, const WalkState<DIM>& st, const Gfn<DIM, RB>& g,
                                           const Pcg32& ws, float ddist, float firstR, uint32_t wsteps, uint32_t t) {
  int q = 0;
  auto put = [&](uint32_t v) {
    mb[(q++) * kSpreadMax + slot] = v;
  };
  auto putf = [&](float v) { put(__float_as_uint(v)); };
  for (int k = 0; k < DIM; k++) { putf(st.pt[k]); putf(st.n[k]); putf(st.prevDir[k]); }
  putf(st.prevDist); putf(st.throughput); put(st.onNeumann ? 1u : 0u); put((uint32_t)st.walkLength);
  putf(st.totalNeumann); putf(st.totalSource);
  putf(st.pThr); putf(st.pNrm); putf(st.pTex); put(st.pend ? 1u : 0u);
  put((uint32_t)g.yukawa);
  put((uint32_t)ws.state); put((uint32_t)(ws.state >> 32));
  (void)firstR;  // 0 after every step (a boundary-start walk's first-sphere radius is used once)
  putf(ddist); put(wsteps); put(t);
}
template <int DIM, bool RB>
__device__ __forceinline__ void spread_get(const uint32_t* mb, int slot, WalkState<DIM>& st, Gfn<DIM, RB>& g,
                                           Pcg32& ws, float& ddist, float& firstR, uint32_t& wsteps, int64_t& t) {
  int q = 0;
  auto get = [&]() { return mb[(q++) * kSpreadMax + slot]; };
  auto getf = [&]() { return __uint_as_float(get()); };
  for (int k = 0; k < DIM; k++) { st.pt[k] = getf(); st.n[k] = getf(); st.prevDir[k] = getf(); }
  st.prevDist = getf(); st.throughput = getf(); st.onNeumann = get() != 0u; st.walkLength = (int)get();
  st.totalNeumann = getf(); st.totalSource = getf();
  st.pThr = getf(); st.pNrm = getf(); st.pTex = getf(); st.pend = get() != 0u;
  g.yukawa = (int)get();
  const uint32_t lo = get(), hi = get();
  ws.state = ((uint64_t)hi << 32) | lo;
  ddist = getf(); firstR = 0.0f; wsteps = get(); t = (int64_t)get();
}
struct SpreadLDS {
  uint32_t busy, idle;
  uint32_t mbox[kBlock / kWave];
};

#ifndef WOS_WALK_WAVES_PER_EU
#define WOS_WALK_WAVES_PER_EU 4
#endif
#ifndef WOS_WALK_WAVES_PER_EU3
#define WOS_WALK_WAVES_PER_EU3 WOS_WALK_WAVES_PER_EU
#endif
// BSTART: the tasks are boundary-start walks (estimateSolution, walk_on_stars.h:353-464:
// start normal, first sphere radius, on-Neumann flag from DevTasks::n0/r0/sflags, no
// first ball, walk stream tag 6) -- boundary value caching (wos_bvc.hip).
template <int DIM, bool GG, bool BSTART = false, bool RB = false, bool NEU = true, bool SPR = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(DIM == 2 ? WOS_WALK_WAVES_PER_EU : WOS_WALK_WAVES_PER_EU3))) void wos_walk_kernel(
    const DevScene sc_arg, const DevParams prm_arg, const DevTasks tk_arg, int64_t base, int64_t stride,
    unsigned long long* __restrict__ counters, unsigned int* __restrict__ tqueue, int geom_floats) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ unsigned int s_ctr[C_NUM];
  __shared__ SpreadLDS s_spread;
  const DevScene& sc = sc_arg;
  const DevParams& prm = prm_arg;
  const DevTasks& tk = tk_arg;
  static_assert(walk_pack_words<DIM>() * kSpreadMax * 4 <= (int)walk_scratch_bytes<DIM>(), "mailbox fits the scratch");
  constexpr bool kSpread = SPR;
  const int lane = threadIdx.x & (kWave - 1);
  stage_geometry<DIM, GG>(sc, smem, true);
  stage_rej_jump(prm);
  // per-wave scratch shared by the star and ray queries (used one after the other)
  const int wave_u = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));  // wave-uniform: SGPR address
  char* wscratch = reinterpret_cast<char*>(smem + geom_floats) + wave_u * walk_scratch_bytes<DIM>();
  StarLDS<DIM>* starL = reinterpret_cast<StarLDS<DIM>*>(wscratch);
  RayLDS<DIM>* rayL = reinterpret_cast<RayLDS<DIM>*>(wscratch);
  RejLDS* rejL = reinterpret_cast<RejLDS*>(wscratch);
  if (threadIdx.x < C_NUM) s_ctr[threadIdx.x] = 0u;
  if (threadIdx.x == 0) { s_spread.busy = blockDim.x / kWave; s_spread.idle = 0u; }
  if (threadIdx.x < kBlock / kWave) s_spread.mbox[threadIdx.x] = 0u;
#if WOS_DIAG
  if (threadIdx.x < D_NUM) s_diag[threadIdx.x] = 0u;
#endif
  __syncthreads();

  const uint32_t T = (uint32_t)tk.T;
  const uint32_t wpp = (uint32_t)tk.wpp;
  // x / wpp as a shift when walks-per-point is a power of two (every shipped config)
  const int wsh = (wpp & (wpp - 1u)) == 0u ? __builtin_ctz(wpp) : -1;
  auto divw = [&](uint32_t x) -> uint32_t { return wsh >= 0 ? x >> wsh : x / wpp; };
  const bool yuk0 = sc.absorption > 0.0f && prm.steps_before_tikhonov == 0;
  uint32_t c_iters = 0;
  wave_priority(prm.wave_prio);
#if WOS_TIMELINE
  uint64_t tl_t0 = 0;
  if (lane == 0) {
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    const unsigned long long old = atomicCAS(&g_tl[0], 0ull, now);
    tl_t0 = old == 0ull ? now : old;
  }
  tl_t0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(tl_t0 >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)tl_t0);
  auto tl_bin = [&](uint64_t ts) -> int {
    const uint64_t b = ts > tl_t0 ? (ts - tl_t0) >> kTlShift : 0;
    return b < (uint64_t)kTlBins ? (int)b : kTlBins - 1;
  };
#endif

  DIAG_T0(t_wave);
  // ---- task supply: a window [wq, we) of the global queue (wave-uniform; lane i
  // holds perm[wp0 + i]) feeds a 64-slot ring of staged tasks, one per lane: ring
  // position (lane - head) & 63, positions [0, S) valid.  The ring is refilled at
  // the end of every iteration, so the loads of a staged task's point state are in
  // flight during a whole step and a lane that finishes a walk starts the next one
  // from registers (cross-lane shuffles) instead of a chain of dependent global loads.
  // <= 64 points per window
  // 3D: windows of 128 tasks (walk kernel -2 % on D and E, bit-exact: profiles/r5zo_ab_grab3.log; in 2D they
  // slowed the karman stride-8 shard, r5zl_ab_star_help2_queue.log)
  constexpr uint32_t kGrabD = DIM == 3 ? WOS_TASK_GRAB3 : kTaskGrab;
  const uint32_t G_win = kGrabD < 63u * wpp ? kGrabD : 63u * wpp;
  // the head of the cost order (the hardest points) is dealt in smaller windows, so the
  // long walks of one point spread over more waves: kTaskHead windows of kTaskGrabHead
  // tasks per wave of the grid, then windows of G_win
  const uint32_t G_head = kTaskGrabHead < G_win ? kTaskGrabHead : G_win;
  const uint32_t n_head = (uint32_t)__builtin_amdgcn_readfirstlane((int)(kTaskHead * gridDim.x * (blockDim.x / kWave)));
  const uint32_t NH = G_head > 0u ? ((T + G_head - 1u) / G_head < n_head ? (T + G_head - 1u) / G_head : n_head) : 0u;
  const uint64_t H = (uint64_t)NH * G_head < (uint64_t)T ? (uint64_t)NH * G_head : (uint64_t)T;
  uint32_t wq = 0, we = 0, wp0 = 0, wperm = 0;
  bool exhausted = false;
  const uint32_t qhome = blockIdx.x & (kTaskQueues - 1u);
  uint32_t qdone = 0u;  // queues found exhausted (wave-uniform)
  int head = 0, S = 0;
  uint32_t s_t = 0, s_ok = 0;  // staged task index, its point is estimated
  auto refill = [&](const DevTasks& tk) {
    while (S < kWave && !exhausted) {
      if (wq >= we) {
        unsigned int c = 0xFFFFFFFFu, len = 0u;
        if (lane == 0) {
          for (uint32_t k = 0; k < kTaskQueues; k++) {
            const uint32_t x = (qhome + k) & (kTaskQueues - 1u);
            if ((qdone >> x) & 1u) continue;
            // queue x's draws: its head windows x, x + Q, ... (< NH), then its tail windows
            const uint32_t d = atomicAdd(tqueue + x * kTaskQueueStride, 1u);
            const uint32_t nhx = NH > x ? (NH - x + kTaskQueues - 1u) / kTaskQueues : 0u;
            const uint64_t st = d < nhx ? (uint64_t)(d * kTaskQueues + x) * G_head
                                        : H + (uint64_t)((uint64_t)(d - nhx) * kTaskQueues + x) * G_win;
            if (st < (uint64_t)T) {
              c = (unsigned int)st;
              len = d < nhx ? G_head : G_win;
              break;
            }
            qdone |= 1u << x;  // exhausted: never drawn from again by this wave
          }
        }
        c = (unsigned int)__builtin_amdgcn_readlane((int)c, 0);
        len = (unsigned int)__builtin_amdgcn_readlane((int)len, 0);
        qdone = (uint32_t)__builtin_amdgcn_readlane((int)qdone, 0);
        if (c == 0xFFFFFFFFu) { exhausted = true; break; }
        wq = c;
        we = (T - c) < len ? T : c + len;
        wp0 = divw(c);
        const uint32_t np = divw(we - 1) - wp0 + 1;
        wperm = (uint32_t)lane < np ? tk.perm[wp0 + lane] : 0u;
      }
      const int avail = (int)(we - wq);
      const int take = (kWave - S) < avail ? (kWave - S) : avail;
      const int pos = ((lane - head) & (kWave - 1)) - S;
      const bool mine = pos >= 0 && pos < take;
      const uint32_t q = wq + (mine ? (uint32_t)pos : 0u), qp = divw(q);
      const uint32_t pidx = (uint32_t)__shfl((int)wperm, (int)(qp - wp0));  // queue position -> permuted point
      if (mine) {
        s_t = pidx * wpp + (q - qp * wpp);
        s_ok = tk.pstate[pidx] & kPtEstimate;
      }
      S += take;
      wq += (uint32_t)take;
    }
  };
  refill(tk);
  int64_t t = -1;           // this lane's task
  WalkState<DIM> st;
  Gfn<DIM, RB> g;
  Pcg32 ws;
  float ddist = 0.0f;
  uint32_t wsteps = 0;
  float firstR = 0.0f;  // BSTART: first sphere radius of the lane's walk, 0 after its first step

  for (;;) {
    DIAG_T0(t_loop);
#if WOS_TIMELINE
    const uint64_t tl_a = __builtin_amdgcn_s_memrealtime();
#endif
    // per-iteration views of the kernel parameters and of the staged geometry (see kview)
    KernArgsPtr ka = kernargs_opaque();
    const DevScene& sc = (const DevScene&)ka->sc;
    const DevParams& prm = (const DevParams&)ka->prm;
    const DevTasks& tk = (const DevTasks&)ka->tk;
    const LGeom G = geometry_view<DIM, GG>(sc, smem, true, false);
    // ---- hand staged tasks to idle lanes (uniform control flow)
    {
      const uint64_t need = __ballot(t < 0);
      if (need != 0 && S > 0) {
        const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
        const int k = __popcll(need);
        const int take = k < S ? k : S;
        const int src = (head + (rank < take ? rank : 0)) & (kWave - 1);
        // the staged task index with its point's estimate bit on top (tasks < 2^31): one shuffle
        const uint32_t v_pk = (uint32_t)__shfl((int)(s_t | (s_ok ? 0x80000000u : 0u)), src);
        const uint32_t v_t = v_pk & 0x7FFFFFFFu;
        const uint32_t v_ok = v_pk >> 31;
        float v_pt[DIM], v_thr = 0.0f, v_tsrc = 0.0f, v_dd = 0.0f;
        if (t < 0 && rank < take && v_ok) {  // the task record from memory, at hand-out
          for (int kk = 0; kk < DIM; kk++) v_pt[kk] = tk.pt[kk * tk.T + v_t];
          v_thr = tk.thr[v_t];
          v_tsrc = tk.tsrc[v_t];
          // boundary-start walks (BVC) always carry a stored distance
          v_dd = (BSTART || sc.n_dprims > 0) ? tk.dd[v_t] : bbox_far_dist<DIM>(sc, v_pt);
        }
        if (t < 0 && rank < take) {
          t = (int64_t)v_t;
          // BSTART: estimateSolution runs one walk only from inside the epsilon shell
          // (walk_on_stars.h:383-386): the start kernel marks the others (sflags bit 1)
          if (!v_ok || (BSTART && (tk.sflags[t] & 2u))) {  // point outside the domain: no walks
            tk.code[t] = 0u;
            t = -1;
          } else {
            const uint32_t pidx = divw(v_t);
            const uint32_t w = (v_t - pidx * wpp) >> (prm.n_anti - 1);  // n_anti is 1 or 2
            walk_start<DIM, BSTART, RB>(sc, prm, tk, t, pidx, w, v_pt, v_thr, v_tsrc, v_dd, base, stride, yuk0, st,
                                        g, ws, ddist, wsteps, firstR);
          }
        }
        head = (head + take) & (kWave - 1);
        S -= take;
#if WOS_TIMELINE
        if (lane == 0) atomicAdd(&g_tl[1 + TL_START * kTlBins + tl_bin(tl_a)], (unsigned long long)take);
#endif
      }
    }
    if (__ballot(t >= 0) == 0) {
      if (S == 0 && exhausted) {  // queue drained and every lane idle
        if (!kSpread) break;
        // idle: announce, then take a sibling's hand-over or leave once no wave holds walks
        if (lane == 0) {
          __hip_atomic_fetch_or(&s_spread.idle, 1u << wave_u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_sub(&s_spread.busy, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        uint32_t n = 0;
        for (;;) {
          n = __hip_atomic_load(&s_spread.mbox[wave_u], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
          n = (uint32_t)__builtin_amdgcn_readfirstlane((int)n);
          if (n != 0u) break;
          const uint32_t busy = (uint32_t)__builtin_amdgcn_readfirstlane(
              (int)__hip_atomic_load(&s_spread.busy, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
          if (busy == 0u) break;
          __builtin_amdgcn_s_sleep(4);
        }
        if (n == 0u) break;
        // the hand-over: slot i of the mailbox (word-major, kSpreadMax slots) -> lane i
        const uint32_t* mb = reinterpret_cast<const uint32_t*>(wscratch);
        if ((uint32_t)lane < n) spread_get<DIM, RB>(mb, lane, st, g, ws, ddist, firstR, wsteps, t);
        wave_sync();
        if (lane == 0) __hip_atomic_store(&s_spread.mbox[wave_u], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        continue;
      }
      refill(tk);
      continue;
    }
    DIAG_COUNT(D_ITERS, 1);
    DIAG_COUNT(D_LANES, __popcll(__ballot(t >= 0)));
#if WOS_DIAG
    const bool lone_it = __popcll(__ballot(t >= 0)) <= 2;
    if (lone_it) DIAG_COUNT(D_L_ITERS, 1);
#endif
    const int code = walk_iteration<DIM, GG, BSTART, RB, NEU>(sc, prm, G, t >= 0, st, g, ws, ddist, wsteps, firstR, starL,
                                                         rayL, rejL, &c_iters, lane);
#if WOS_TIMELINE
    {
      const unsigned long long nlive = (unsigned long long)__popcll(__ballot(t >= 0));
      const unsigned long long nfin = (unsigned long long)__popcll(__ballot(t >= 0 && code >= 0));
      const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - tl_a;
      if (lane == 0) {
        const int b = tl_bin(tl_a);
        atomicAdd(&g_tl[1 + TL_WAVE * kTlBins + b], dt);
        atomicAdd(&g_tl[1 + TL_LANE * kTlBins + b], dt * nlive);
        if (nfin) atomicAdd(&g_tl[1 + TL_FIN * kTlBins + b], nfin);
      }
    }
#endif
    if (t >= 0 && code >= 0) {
      walk_finish<DIM>(sc, prm, tk, t, code, st, wsteps, s_ctr);
      t = -1;
    }
    if (kSpread && exhausted && S == 0) {
      const uint64_t live = __ballot(t >= 0);
      const int k = __popcll(live);
      if (k >= 2 && __builtin_amdgcn_readfirstlane(
                        (int)__hip_atomic_load(&s_spread.idle, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0) {
        int to = -1;
        if (lane == 0) {
          uint32_t m = __hip_atomic_load(&s_spread.idle, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          while (m != 0u) {
            const uint32_t b = 1u << __builtin_ctz(m);
            const uint32_t old =
                __hip_atomic_fetch_and(&s_spread.idle, ~b, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old & b) {
              // the recipient holds walks from here on: counted before it can see them
              __hip_atomic_fetch_add(&s_spread.busy, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
              to = __builtin_ctz(b);
              break;
            }
            m = old & ~b;
          }
        }
        to = __builtin_amdgcn_readlane(to, 0);
        if (to >= 0) {
          // the upper half of the live walks (by lane rank), at most kSpreadMax
          const int kd = (k / 2) < kSpreadMax ? (k / 2) : kSpreadMax;
          const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(live >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)live, 0u));
          const bool give = t >= 0 && rank >= k - kd;
          uint32_t* mb = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(smem + geom_floats) +
                                                     to * walk_scratch_bytes<DIM>());
          if (give) {
            spread_put<DIM, RB>(mb, rank - (k - kd), st, g, ws, ddist, firstR, wsteps, (uint32_t)t);
            t = -1;
          }
          wave_sync();
          if (lane == 0)
            __hip_atomic_store(&s_spread.mbox[to], (uint32_t)kd, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
    refill(tk);
#if WOS_DIAG
    DIAG_ADD_LONE(D_LOOP, D_L_LOOP, t_loop, lone_it);
#endif
#if WOS_DIAG
    if (exhausted) {
      DIAG_COUNT(D_XITERS, 1);
      DIAG_COUNT(D_XLANES, __popcll(__ballot(t >= 0)));
      DIAG_ADD(D_XLOOP, t_loop);
    }
#endif
  }
  DIAG_MAX(D_WAVEMAX, __builtin_amdgcn_s_memtime() - t_wave);
  flush_counter(counters, C_ITERS, c_iters, lane);
  __syncthreads();
#if WOS_DIAG
  if (threadIdx.x < D_NUM) {
    if (diag_is_max(threadIdx.x)) atomicMax(&g_diag[threadIdx.x], s_diag[threadIdx.x]);
    else atomicAdd(&g_diag[threadIdx.x], s_diag[threadIdx.x]);
  }
#endif
  flush_walk_counters(counters, s_ctr);
}

// One thread per point, kFoldPoints points per block.  The records of the
// block's points are contiguous (point-major tasks), so they are staged through
// LDS in chunks of kFoldChunk records per point with coalesced 64-B loads, then
// every thread folds its own point's chunk in walk order.
#ifndef WOS_FOLD_POINTS
#define WOS_FOLD_POINTS 128
#endif
#ifndef WOS_FOLD_CHUNK
#define WOS_FOLD_CHUNK 16
#endif
// staging slots in flight per thread: 2D 8 (fold -10 % on karman, -13 % on config C),
// 3D 4 (8 measured +4 % on the cube), profiles/r3x_ab_solo_fold.log
#ifndef WOS_FOLD_UNROLL2
#define WOS_FOLD_UNROLL2 8
#endif
#ifndef WOS_FOLD_UNROLL3
#define WOS_FOLD_UNROLL3 4
#endif
// records staged per point and round: 2D 16; 3D (nine fields per record) WOS_FOLD_CHUNK3
#ifndef WOS_FOLD_CHUNK3
#define WOS_FOLD_CHUNK3 WOS_FOLD_CHUNK
#endif
constexpr int kFoldPoints = WOS_FOLD_POINTS, kFoldChunk = WOS_FOLD_CHUNK;
template <int DIM>
constexpr int kFoldChunkD = DIM == 2 ? WOS_FOLD_CHUNK : WOS_FOLD_CHUNK3;
template <int DIM>
constexpr int kFoldUnroll = DIM == 2 ? WOS_FOLD_UNROLL2 : WOS_FOLD_UNROLL3;

template <int DIM>
__global__ __launch_bounds__(kFoldPoints) void wos_fold_kernel(const DevParams prm, const DevTasks tk, int64_t n,
                                                               float* __restrict__ p_out,
                                                               float* __restrict__ g_out,
                                                               int32_t* __restrict__ nest_out,
                                                               int32_t* __restrict__ steps_out) {
  constexpr int NF = 3 + 2 * DIM;  // code | total | first | bdir[DIM] | sdir[DIM]
  constexpr int LD = kFoldChunkD<DIM> + 1;
  wave_priority(prm.wave_prio);
  __shared__ float lds[NF][kFoldPoints][LD];
  const int tid = threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.x * kFoldPoints;
  const int nb = (int)((n - p0) < kFoldPoints ? (n - p0) : kFoldPoints);
  const int64_t i = p0 + tid;
  const int64_t T = tk.T;
  const int wpp = tk.wpp;
  const int ps = tid < nb ? tk.pstate[i] : 0;
  const bool estimate = (ps & kPtEstimate) != 0;
  float mean[DIM + 1];
  for (int k = 0; k <= DIM; k++) mean[k] = 0.0f;
  float sFirst = 0.0f, cvb = 0.0f, cvs = 0.0f, sDeriv = 0.0f;
  int sN = 0;
  uint32_t steps = 0;
  // directionForDerivative (walk_on_stars.h:603-607): the point's own or (1, 0[, 0])
  float dn[DIM];
  for (int k = 0; k < DIM; k++) dn[k] = k == 0 ? 1.0f : 0.0f;
  if (tk.deriv && tk.ddir && tid < nb)
    for (int k = 0; k < DIM; k++) dn[k] = tk.ddir[i * DIM + k];
  for (int c0 = 0; c0 < wpp; c0 += kFoldChunkD<DIM>) {
    const int cnt = (wpp - c0) < kFoldChunkD<DIM> ? (wpp - c0) : kFoldChunkD<DIM>;
    // kFoldUnroll<DIM> staging slots in flight per thread: all their loads are issued
    // before the first LDS store (one HBM round trip per kFoldUnroll slots, not per slot)
    for (int e0 = tid; e0 < nb * kFoldChunkD<DIM>; e0 += kFoldPoints * kFoldUnroll<DIM>) {
      float v[kFoldUnroll<DIM>][NF];
#pragma unroll
      for (int u = 0; u < kFoldUnroll<DIM>; u++) {
        const int e = e0 + u * kFoldPoints;
        const int pp = e / kFoldChunkD<DIM>, j = e - pp * kFoldChunkD<DIM>;
        if (e >= nb * kFoldChunkD<DIM> || j >= cnt) continue;
        const int64_t t = (p0 + pp) * wpp + c0 + j;
        v[u][0] = __uint_as_float(tk.code[t]);
        v[u][1] = tk.total[t];
        v[u][2] = tk.first[t];
#pragma unroll
        for (int k = 0; k < DIM; k++) {
          v[u][3 + k] = tk.bdir[k * T + t];
          v[u][3 + DIM + k] = tk.sdir[k * T + t];
        }
      }
#pragma unroll
      for (int u = 0; u < kFoldUnroll<DIM>; u++) {
        const int e = e0 + u * kFoldPoints;
        const int pp = e / kFoldChunkD<DIM>, j = e - pp * kFoldChunkD<DIM>;
        if (e >= nb * kFoldChunkD<DIM> || j >= cnt) continue;
#pragma unroll
        for (int f = 0; f < NF; f++) lds[f][pp][j] = v[u][f];
      }
    }
    __syncthreads();
    if (estimate) {
      for (int j = 0; j < cnt; j++) {
        const int r = c0 + j;
        if (r % prm.n_anti == 0) {  // a new antithetic pair: control variates from the walks before it
          cvb = mean[0];
          cvs = sFirst / (float)(sN > 1 ? sN : 1);
          if (!prm.use_cv) { cvb = 0.0f; cvs = 0.0f; }
        }
        const uint32_t code = __float_as_uint(lds[0][tid][j]);
        steps += code >> 1;
        if (!(code & 1u)) continue;
        const float total = lds[1][tid][j];
        const float first = lds[2][tid][j];
        sN += 1;
        const float fN = (float)sN;
        {
          const float delta = total - mean[0];
          mean[0] += delta / fN;
        }
        float deriv = 0.0f;
        for (int k = 0; k < DIM; k++) {
          const float be = (total - first - cvb) * lds[3 + k][tid][j];
          const float se = (first - cvs) * lds[3 + DIM + k][tid][j];
          const float delta = (be + se) - mean[k + 1];
          mean[k + 1] += delta / fN;
          deriv += be * dn[k];
          deriv += se * dn[k];
        }
        sDeriv += deriv;  // addDerivativeContribution
        sFirst += first;
      }
    }
    __syncthreads();
  }
  if (tid >= nb) return;
  const bool maskP = ps & kPtMaskP, maskG = ps & kPtMaskG;
  p_out[i] = maskP ? 0.0f : mean[0];
  for (int k = 0; k < DIM; k++) g_out[i * DIM + k] = maskG ? 0.0f : mean[k + 1];
  if (nest_out) nest_out[i] = sN;
  if (steps_out) steps_out[i] = (int32_t)steps;
  if (tk.deriv) tk.deriv[i] = sDeriv / (float)(sN > 1 ? sN : 1);  // getEstimatedDerivative (unmasked)
}

// The same statistics with one lane QUAD per point: quad lane c runs component c's Welford chain
// (c = 0: the solution, c = 1..DIM: the gradient components; 2D leaves lane 3 idle), operation for
// operation as wos_fold_kernel's mean[c]; the control variate cvb -- the solution mean at a pair's
// start -- comes from quad lane 0 by a DPP quad broadcast, and the walk count and first-source sum
// (cvs) are kept by every lane.  Four chains in flight per point instead of one, and a quarter of
// the LDS per point, so four times the waves: the fold was latency-bound on one thread's chain of
// IEEE divisions per point (round 4, DESIGN).  Not for the derivative output (BVC's Dirichlet
// samples, DevTasks::deriv): wos_fold_kernel keeps that.  Both dimensions since its staging is
// software-pipelined (before that, 2D's five-float records folded faster one thread per point).
constexpr int kFold4Points = 64;  // points per 256-thread block
template <int DIM>
__global__ __launch_bounds__(4 * kFold4Points) void wos_fold4_kernel(const DevParams prm, const DevTasks tk, int64_t n,
                                                                     float* __restrict__ p_out,
                                                                     float* __restrict__ g_out,
                                                                     int32_t* __restrict__ nest_out,
                                                                     int32_t* __restrict__ steps_out) {
  constexpr int NF = 3 + 2 * DIM;  // code | total | first | bdir[DIM] | sdir[DIM]
  constexpr int CH = kFoldChunkD<DIM>;
  constexpr int LD = CH + 1;
  constexpr int NT = 4 * kFold4Points;
  wave_priority(prm.wave_prio);
  // one plane per field, planes FS words apart: FS = 1 (mod 64) puts the four lanes of a quad, which
  // read different planes at the same (point, walk), in different LDS banks
  constexpr int FS = kFold4Points * LD + 1;
  __shared__ float lds[NF * FS];
  const int tid = threadIdx.x;
  const int c = tid & 3, pp = tid >> 2;
  const int64_t p0 = (int64_t)blockIdx.x * kFold4Points;
  const int nb = (int)((n - p0) < kFold4Points ? (n - p0) : kFold4Points);
  const int64_t i = p0 + pp;
  const int64_t T = tk.T;
  const int wpp = tk.wpp;
  const int ps = pp < nb ? tk.pstate[i] : 0;
  const bool estimate = (ps & kPtEstimate) != 0;
  const bool comp = c <= DIM;
  const int fb = c >= 1 && comp ? 3 + (c - 1) : 3, fs = c >= 1 && comp ? 3 + DIM + (c - 1) : 3;
  float mean = 0.0f, sFirst = 0.0f, cvb = 0.0f, cvs = 0.0f;
  int sN = 0;
  uint32_t steps = 0;
  // software pipeline: the block's next chunk of records is loaded into registers (UE slots per
  // thread) while the current one is folded from LDS, so the HBM latency of the staging overlaps
  // the Welford chains (D fold 1.84 -> 1.44 ms, E at 96^3 1.53 -> 1.29 ms: profiles/r5zm_ab_fold_pipe.log;
  // with it the quad fold also beats the one-thread 2D fold: karman 0.109 -> 0.084 ms, C 0.81 -> 0.63 ms,
  // r5zn_ab_fold4_2d.log)
  constexpr int UE = (kFold4Points * CH + NT - 1) / NT;
  float w[UE][NF];
  auto load_next = [&](int c0n) {
    const int cntn = (wpp - c0n) < CH ? (wpp - c0n) : CH;
#pragma unroll
    for (int u = 0; u < UE; u++) {
      const int e = tid + u * NT;
      const int q = e / CH, j = e - q * CH;
      if (e >= nb * CH || j >= cntn) continue;
      const int64_t t = (p0 + q) * wpp + c0n + j;
      w[u][0] = __uint_as_float(tk.code[t]);
      w[u][1] = tk.total[t];
      w[u][2] = tk.first[t];
#pragma unroll
      for (int k = 0; k < DIM; k++) {
        w[u][3 + k] = tk.bdir[k * T + t];
        w[u][3 + DIM + k] = tk.sdir[k * T + t];
      }
    }
  };
  load_next(0);
  for (int c0 = 0; c0 < wpp; c0 += CH) {
    const int cnt = (wpp - c0) < CH ? (wpp - c0) : CH;
#pragma unroll
    for (int u = 0; u < UE; u++) {
      const int e = tid + u * NT;
      const int q = e / CH, j = e - q * CH;
      if (e >= nb * CH || j >= cnt) continue;
#pragma unroll
      for (int f = 0; f < NF; f++) lds[f * FS + q * LD + j] = w[u][f];
    }
    __syncthreads();
    if (c0 + CH < wpp) load_next(c0 + CH);  // in flight during the fold below
    if (estimate) {
      for (int j = 0; j < cnt; j++) {
        const int r = c0 + j;
        if (r % prm.n_anti == 0) {  // a new antithetic pair: control variates from the walks before it
          // quad lane 0's solution mean (DPP quad_perm [0,0,0,0])
          cvb = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(mean), 0x00, 0xF, 0xF, false));
          cvs = sFirst / (float)(sN > 1 ? sN : 1);
          if (!prm.use_cv) { cvb = 0.0f; cvs = 0.0f; }
        }
        const uint32_t code = __float_as_uint(lds[pp * LD + j]);
        steps += code >> 1;
        if (!(code & 1u)) continue;
        const float total = lds[FS + pp * LD + j];
        const float first = lds[2 * FS + pp * LD + j];
        sN += 1;
        const float fN = (float)sN;
        const float be = (total - first - cvb) * lds[fb * FS + pp * LD + j];
        const float se = (first - cvs) * lds[fs * FS + pp * LD + j];
        const float val = c == 0 ? total : be + se;
        const float delta = val - mean;
        mean += delta / fN;
        sFirst += first;
      }
    }
    __syncthreads();
  }
  if (pp >= nb || !comp) return;
  if (c == 0) {
    p_out[i] = (ps & kPtMaskP) ? 0.0f : mean;
    if (nest_out) nest_out[i] = sN;
    if (steps_out) steps_out[i] = (int32_t)steps;
  } else {
    g_out[i * DIM + (c - 1)] = (ps & kPtMaskG) ? 0.0f : mean;
  }
}

}  // namespace wos
