// wos_host_scene.h -- host-side scene preparation (OBJ parsing, normals,
// silhouette candidates, padded bounding box) producing the packed records of
// wos_scene.h.  Pure CPU code; no HIP calls.
#pragma once
#include <array>
#include <stdint.h>
#include <string>
#include <vector>

#include "wos_scene.h"

namespace wos {

struct HostSceneInput {
  int dim = 2;
  const float* vertices = nullptr;
  const int32_t* prims = nullptr;
  int n_vertices = 0, n_prims = 0;
  const float* dvertices = nullptr;
  const int32_t* dprims = nullptr;
  int n_dvertices = 0, n_dprims = 0;
  int is_double_sided = 0;
};

struct HostTree {
  std::vector<float> node;  // levels 1.. of the implicit 8-ary tree (wos_scene.h DevTree)
  int levels = 0;
  int n[kTreeLevels + 1] = {};
  int off[kTreeLevels + 1] = {};
};
// the tree over `ngroups` group records of `stride` floats (box in the first 8)
void build_group_tree(const std::vector<float>& groups, int stride, int ngroups, HostTree& out);

// The Neumann boundary's wide BVH as fcpw builds it for the stochastic boundary sample
// (wos_fcpw_bvh.cpp): node i has `branch` children; child box w at
// box[(i * branch + w) * 6] = [min.xyz | max.xyz] (2D: z = 0 padded by FLT_EPSILON),
// child[i * branch + w] = child node index, INT_MAX when unused (box min = FLT_MAX,
// max = -FLT_MAX).  A leaf has child[0] < 0, child[2] = first reference,
// child[3] = reference count; ref[r] = primitive of reference r.
constexpr int kFcpwBranch = 4;  // FCPW_MBVH_BRANCHING_FACTOR (FCPW_USE_EIGHT_WIDE_BRANCHING off)
constexpr int kFcpwLeaf = 8;    // FCPW_SIMD_WIDTH of an AVX/AVX2 build (fcpw CMakeLists.txt:83-95)
struct HostFcpwBvh {
  int branch = kFcpwBranch, leaf = kFcpwLeaf;
  int n_nodes = 0, n_leaves = 0;
  std::vector<float> box;
  std::vector<int32_t> child;
  std::vector<int32_t> ref;
};
void build_fcpw_bvh(int dim, const float* verts, const int32_t* prims, int n_prims, int branch, int leaf,
                    HostFcpwBvh& out);

struct HostScene {
  int dim = 2;
  int n_prims = 0, n_sil = 0, n_dprims = 0;
  std::vector<float> prim, paux, sil, dprim, dpaux;
  std::vector<float> pgroup, sgroup, dgroup;  // culling boxes (kGroupStride floats each)
  int n_pgroups = 0, n_sgroups = 0, n_dgroups = 0;
  HostTree ptree, stree, dtree;
  HostFcpwBvh nbvh;  // Neumann boundary, for the stochastic boundary sample
  float pmin[3] = {0, 0, 0}, pmax[3] = {0, 0, 0}, ext[3] = {0, 0, 0};
};

// Star-radius cell grid: a uniform grid over the padded bounding box; cell c
// holds the ascending list of the silhouette candidates that can decide
// computeStarRadius (fcpw_scene_loader.h:621-641) for any point of the cell.
// A candidate is left out only when, for every point of the (slightly enlarged)
// cell, the exact test certainly rejects it (its two adjacent faces both face the
// point, or both face away, with margin) or it certainly lies farther than a
// candidate that is certainly a silhouette there (and farther than minR), so the
// sequential scan over the list returns the full scan's result bit for bit.
struct StarGrid {
  int n[3] = {1, 1, 1};
  float gmin[3] = {0.0f, 0.0f, 0.0f}, inv[3] = {0.0f, 0.0f, 0.0f};
  int ncell = 0;
  int off_words = 0;             // 32-bit words of the u16 offset table (ncell + 1 entries)
  std::vector<uint32_t> words;   // [u16 offsets | u8 candidate indices], little-endian packed
  size_t list_len = 0;
  float prec = -1.0f, min_r = -1.0f;  // the solver settings it was built for
};
// false when the scene has no / too many (> 255) silhouette candidates or the grid
// does not fit budget_bytes at a useful resolution (the kernel then scans groups)
bool build_star_grid(const HostScene& hs, float prec, float min_r, size_t budget_bytes, StarGrid& out);

// Dirichlet-distance cell grid (2D): a uniform grid over the padded bounding box; cell c
// holds the ascending list of the Dirichlet segments that can be the closest one
// (computeDistToDirichlet, fcpw_scene_loader.h:299-315) to a point of the (slightly
// enlarged) cell: segment s is left out only when its distance from every point of the
// cell is certainly above the distance from that point to another segment -- its
// box distance exceeds, with margin, the smallest corner-maximum distance U of the
// cell's segments.  A scan of the list in index order with the full scan's `<=` rule
// returns the full scan's distance bit for bit (the float argmin is within ~1e-6 of the
// true minimum, far inside the margin).
struct DirGrid {
  int n[2] = {1, 1};
  float gmin[2] = {0.0f, 0.0f}, inv[2] = {0.0f, 0.0f};
  int ncell = 0;
  int off_words = 0;             // u32 offsets (ncell + 1 entries)
  std::vector<uint32_t> words;   // [u32 offsets | u16 segment indices, packed]
  size_t list_len = 0;
  int max_list = 0;
};
// false for 3D scenes, no / too many Dirichlet segments, or lists too long to pay off
bool build_dirichlet_grid(const HostScene& hs, DirGrid& out);

// Upper bounds for the Yukawa rejection test (wos_kernel.hip rej_quick_bound): the
// accept threshold of rejectionSampleGreensFn at radius r = x R is
// T = R * x * Q_s(x) / (norm * bound) with s = mu R and
//   Q_s(x) = K0(s x) - K0(s) / I0(s) * I0(s x)                 (2D)
//   Q_s(x) = e^{-s x} - e^{-s} sinh(s x) / sinh(s)             (3D),
// so T <= R * F(s) / (norm * bound) with F(s) = max_x x Q_s(x).  tab[k] >= F(s) for
// every s of bin k (k = floor(kRejTabScale * sqrt(s))): the maximum over 16 values
// of s across the bin, each maximised over x on a grid refined around its peak,
// times 1.02 (the bins are narrow and F is smooth: the margin dwarfs both
// discretisations and the float rounding of the kernel's exact test).
void rejection_bound_table(int dim, float* tab);


bool prepare_scene(const HostSceneInput& in, HostScene& out, std::string& err);
bool load_obj(const std::string& path, int dim, bool flip, bool normalize_domain, std::vector<float>& verts,
              std::vector<int32_t>& prims, std::string& err);

}  // namespace wos
