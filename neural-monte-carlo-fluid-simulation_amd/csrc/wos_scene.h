// wos_scene.h -- scene and solver-parameter layouts shared by the host-side scene
// preparation (wos_scene.cpp) and the gfx950 kernels (wos_kernel.hip).
//
// HBM layout (all float32, structure-of-records, 16-byte aligned):
//   prim  : Neumann primitives, packed per primitive
//           2D  [pa.x pa.y v.x v.y], v = pb - pa               (4 floats)
//           3D  [pa.xyz pb.xyz pc.xyz]                         (9 floats)
//   paux  : per-primitive normals used only by signed-distance queries
//           2D  [na.xy nb.xy nseg.xy]  (vertex normals at the ends + segment normal)
//           3D  [na nb nc | e0 e1 e2 | nface]  (vertex, edge, face normals; 21 floats)
//   sil   : silhouette candidates (vertices in 2D, edges in 3D)
//           2D  [p.xy n0.xy n1.xy miss pad]                    (8 floats)
//           3D  [pa.xyz pb.xyz n0.xyz n1.xyz miss pad pad pad] (16 floats)
//   dprim/dpaux : same as prim/paux for the (optional) Dirichlet boundary
//   source: the -div(u) grid, row-major; 2D (H rows ~ y, W cols ~ x), 3D (X,Y,Z)
//   pgroup/sgroup: padded boxes of kGroup consecutive prims / silhouettes
//           (8 / 16 floats, see kSGroupStride), used only to skip whole groups
//
// The Neumann prim + sil arrays are staged into LDS by every workgroup.
#pragma once
#include <stdint.h>

namespace wos {

constexpr int kPrimStride2 = 4, kPrimStride3 = 9;
constexpr int kAuxStride2 = 6, kAuxStride3 = 21;
constexpr int kSilStride2 = 8, kSilStride3 = 16;
// culling groups: kGroup consecutive primitives (or silhouette candidates) share
// one padded bounding box record [min.xyz pad max.xyz pad]; silhouette groups add
// a bounding sphere and the cone of their adjacent normals:
//   [min.xyz sin(alpha) | max.xyz cos(alpha) | c.xyz rho | axis.xyz nocull]
constexpr int kGroup = 8, kGroupStride = 8, kSGroupStride = 16;

// Bounding-volume hierarchy over a group array (the role of fcpw's 8-wide MBVH,
// mbvh.inl:702-818, for meshes far beyond the reference's): an implicit 8-ary tree
// whose level-0 nodes are the groups and whose node (L, i), L >= 1, bounds the
// groups [i 8^L, (i+1) 8^L) with the union of their padded boxes ([min pad | max pad],
// kGroupStride floats).  Levels are built until at most 8 nodes remain; scenes with
// at most kTreeMinGroups groups get none (levels = 0: the flat group scan).
constexpr int kTreeLevels = 8;
constexpr int kTreeMinGroups = 64;
struct DevTree {
  const float* node;           // level L's boxes at node + off[L] * kGroupStride (L >= 1)
  int32_t levels;              // 0: no tree
  int32_t n[kTreeLevels + 1];  // n[0] = groups, n[L] = nodes of level L
  int32_t off[kTreeLevels + 1];
};

template <int DIM> struct Layout;
template <> struct Layout<2> {
  static constexpr int prim = kPrimStride2, aux = kAuxStride2, sil = kSilStride2;
};
template <> struct Layout<3> {
  static constexpr int prim = kPrimStride3, aux = kAuxStride3, sil = kSilStride3;
};

struct DevScene {
  int32_t dim;
  int32_t n_prims, n_sil, n_dprims;
  const float* prim;
  const float* paux;
  const float* sil;
  const float* dprim;
  const float* dpaux;
  const float* source;
  const float* pgroup;   // n_pgroups boxes over consecutive Neumann primitives
  const float* sgroup;   // n_sgroups boxes over consecutive silhouette candidates
  const float* dgroup;   // n_dgroups boxes over consecutive Dirichlet primitives
  int32_t n_pgroups, n_sgroups, n_dgroups;
  DevTree ptree, stree, dtree;  // hierarchies over pgroup / sgroup / dgroup
  // fcpw's wide BVH over the Neumann primitives (wos_host_scene.h HostFcpwBvh), read
  // from global memory by the stochastic boundary sample; nullptr without Neumann prims
  const float* nbvh_box;
  const int32_t* nbvh_child;
  const int32_t* nbvh_ref;
  int32_t nbvh_branch;
  // 1: the kernels read the geometry records from global memory (L2) instead of
  // staging them in LDS -- scenes too large for the LDS budget (set per solve)
  int32_t geom_global;
  int32_t sdims[3];
  float pmin[3], pmax[3], ext[3];
  float absorption;
  float g_dirichlet;
  // image-valued Dirichlet data (wos_scene_desc.dirichlet_image; nullptr: g_dirichlet):
  // [ddims[0]][ddims[1]] over the rectangle dbox = (x0, y0, ex, ey)
  const float* dimg;
  int32_t ddims[2];
  float dbox[4];
  // image-valued Neumann data h (wos_scene_desc.neumann_image; nullptr: h = 0, the reference's):
  // [ndims[0]][ndims[1]] over the rectangle nbox = (x0, y0, ex, ey)
  const float* nimg;
  int32_t ndims[2];
  float nbox[4];
  int32_t watertight;
  int32_t double_sided;
  // star-radius cell grid (wos_host_scene.h StarGrid; nullptr: none): u16 cell
  // offsets then u8 candidate lists, staged into LDS by the walk kernel
  const uint32_t* sgrid;
  int32_t sgrid_words, sgrid_off_words;
  int32_t sgrid_n[3];
  float sgrid_min[3], sgrid_inv[3];
  // Dirichlet-distance cell grid (2D; wos_host_scene.h DirGrid; nullptr: none), global
  // memory: u32 cell offsets then u16 segment indices
  const uint32_t* dgrid;
  int32_t dgrid_off_words;
  int32_t dgrid_n[2];
  float dgrid_min[2], dgrid_inv[2];
};

struct DevParams {
  int32_t n_walks;          // as configured (nWalks)
  int32_t n_pairs;          // walks per antithetic iteration set (nWalks/2 or nWalks)
  int32_t n_anti;           // 2 with antithetic variates, else 1
  int32_t max_walk_length;
  int32_t steps_before_tikhonov;
  int32_t steps_before_maximal_spheres;
  float epsilon_shell;
  float min_star_radius;
  float silhouette_precision;
  float rr_threshold;
  float boundary_distance_mask;
  int32_t use_cv;
  int32_t use_cosine;
  int32_t ignore_dirichlet;
  int32_t ignore_neumann;
  int32_t ignore_source;
  int32_t robust;           // wos_solver_params.robust_float (Gfn::scaled)
  int32_t neumann_inert;    // 1: no ball can reach the float-overflow regime (walk kernel without the Neumann term)
  int32_t force_estimate;   // 1: estimate every point, inside the domain or not (BVC's Dirichlet samples:
                            // BoundarySampler::computeEstimates solves at every sample, boundary_sampler.h:125-166)
  int32_t tail_spread;      // 1: the walk kernel instantiation that hands walks to idle sibling waves
  int32_t wave_prio;        // 0..3: the walk / fold kernels' waves issue at this priority (s_setprio) --
                            // boundary value caching's concurrent walk sets, longest chain highest
  uint64_t seed;
  // PCG32 jump-ahead table: jump[2k], jump[2k+1] = (A_k, C_k) with
  // state_k = A_k * state_0 + C_k (mod 2^64); lets the lanes of a wave draw the
  // per-point stratified samples in parallel.  n_jump entries.
  const uint64_t* jump;
  int32_t n_jump;
  // entries of jump staged in the first-ball kernel's LDS (its stratified-sample draws; 0: none)
  int32_t lhs_jump_n;
  // certain-reject bounds of the Yukawa rejection threshold by bin of s = mu R
  // (wos_host_scene.h rejection_bound_table), kRejTabBins floats; nullptr: none
  const float* rej_tab;
};

// bins of the rejection bound table: bin = floor(kRejTabScale * sqrt(mu R))
// the walk kernel's task-queue counters (wos_launch.h kTaskQueueSlot0): at most
// kMaxTaskQueues, kTaskQueueStride u32 words (64 B) apart
constexpr int kMaxTaskQueues = 32;
constexpr unsigned int kTaskQueueStride = 16;
constexpr int kRejTabBins = 96;
// most jump constants the first-ball kernel stages in LDS (16 B each)
constexpr int kLhsJumpMax = 512;
constexpr float kRejTabScale = 8.0f;

// Walk-task workspace of one batch of points, SoA over T = n_points * wpp tasks
// (task t = point * wpp + pair * n_anti + member).  Written by the first-ball
// kernel, advanced by the walk kernel, folded by the statistics kernel.
struct DevTasks {
  float* pt;        // [DIM][T] walk start: the first ball's boundary sample
  float* thr;       // [T] throughput after the first ball
  float* tsrc;      // [T] source contribution of the first ball
  float* dd;        // [T] Dirichlet distance at pt
  float* first;     // [T] record: first-ball source value (control variate)
  float* bdir;      // [DIM][T] record: boundary gradient direction
  float* sdir;      // [DIM][T] record: source gradient direction
  float* total;     // [T] record: walk total
  uint32_t* code;   // [T] record: (steps << 1) | recorded
  int32_t* pstate;  // [n] bit0 estimated, bit1 mask p, bit2 mask grad p, bits 8..12 cost bucket
  uint32_t* perm;   // [n] walk-queue order of the points (longest expected walks first)
  uint32_t* hist;   // [2 * kCostBuckets] bucket counts, then running bucket offsets
  float* prad;      // [n] first-ball radius 0.99 min(dDist, nDist) (point-setup kernel -> presorted first balls)
  int64_t T;
  int32_t wpp;      // walks per point = n_pairs * n_anti
  // Boundary-start walks (estimateSolution, walk_on_stars.h:353-464; boundary value
  // caching): per task the start normal [DIM][T], the first sphere radius [T] and
  // bit 0 "starts on the Neumann boundary" [T].  They alias the first-ball record
  // arrays (bdir, first, sdir), which such walks do not use; nullptr otherwise.
  float* n0;
  float* r0;
  uint32_t* sflags;
  // [4][pball_stride] per point: the 2D Yukawa first ball's Bessel members K0 I0 K1 I1 at
  // mu R (Gfn::update_ball), written by the point-setup kernel (one lane per point) for the
  // reference-semantics first-ball kernel; nullptr: the first-ball kernel evaluates them
  float* pball;
  int64_t pball_stride;
  // per point [n][DIM] SampleEstimationData::directionForDerivative (nullptr: (1, 0[, 0]),
  // walk_on_stars.h:665-666) and the estimated directional derivative out [n]
  // (getEstimatedDerivative, :843-846; nullptr: not computed) -- BVC's Dirichlet samples
  const float* ddir;
  float* deriv;
};

// floats per task: start state pt[DIM] thr tsrc dd, record first bdir[DIM] sdir[DIM] total code
constexpr int task_floats(int dim) { return 3 * dim + 6; }
constexpr int kCostBuckets = 32;

}  // namespace wos
