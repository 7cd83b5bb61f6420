// wos_fcpw_bvh.cpp -- the Neumann boundary's wide BVH as fcpw builds it, for the
// stochastic boundary sample (sampleNeumann, fcpw_scene_loader.h:599-620 ->
// Mbvh::intersectStochasticFromNode, mbvh.inl:1099-1283).
//
// That query descends ONE root-to-leaf path, choosing among the children that
// overlap the ball with probability proportional to a weight of the distance to
// each child box's centre, so whether a sample exists at all -- and which
// primitive it lands on -- depends on the tree.  The tree is restated here from
// the scene loader's build call (fcpw_scene_loader.h:161-164:
// Bvh_OverlapSurfaceArea, vectorize = true -> makeAggregate, fcpw.inl:522-575):
//   * an Sbvh with CostHeuristic::OverlapSurfaceArea, 8 centroid buckets per axis,
//     packed leaves of leafSize = FCPW_SIMD_WIDTH references (sbvh.inl:3-235);
//   * collapsed into an Mbvh of FCPW_MBVH_BRANCHING_FACTOR children per node
//     (mbvh.inl:46-133).
// Geometry is handled in 3D exactly as fcpw's Scene<3> does for the 2D loader
// (z = 0, boxes padded by FLT_EPSILON in every axis).  Float arithmetic follows the
// reference's operation order; compiled with -ffp-contract=off like the kernels.
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>

#include "wos_host_scene.h"

namespace wos {
namespace {

struct Box3 {
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
  float mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  // BoundingBox::expandToInclude(point) pads by epsilon (bounding_volumes.h:41-45)
  void add_point(const float* p) {
    for (int k = 0; k < 3; k++) {
      mn[k] = std::min(mn[k], p[k] - FLT_EPSILON);
      mx[k] = std::max(mx[k], p[k] + FLT_EPSILON);
    }
  }
  void add_box(const Box3& b) {
    for (int k = 0; k < 3; k++) {
      mn[k] = std::min(mn[k], b.mn[k]);
      mx[k] = std::max(mx[k], b.mx[k]);
    }
  }
  // BoundingBox::surfaceArea (bounding_volumes.h:131-135): e = max(extent, 1e-5),
  // 2 * sum(prod(e) / e_k); Eigen reduces a fixed-size 3-vector as a tree,
  // x0 op (x1 op x2) (Redux.h redux_novec_unroller)
  float area() const {
    float e[3];
    for (int k = 0; k < 3; k++) e[k] = std::max(mx[k] - mn[k], 1e-5f);
    const float pr = e[0] * (e[1] * e[2]);
    return 2.0f * (pr / e[0] + (pr / e[1] + pr / e[2]));
  }
  bool valid() const { return mx[0] >= mn[0] && mx[1] >= mn[1] && mx[2] >= mn[2]; }
  Box3 intersect(const Box3& b) const {
    Box3 r;
    for (int k = 0; k < 3; k++) {
      r.mn[k] = std::max(mn[k], b.mn[k]);
      r.mx[k] = std::min(mx[k], b.mx[k]);
    }
    return r;
  }
  // Eigen maxCoeff(&index): the first maximal extent
  int max_dim() const {
    int d = 0;
    float m = mx[0] - mn[0];
    for (int k = 1; k < 3; k++)
      if (mx[k] - mn[k] > m) { m = mx[k] - mn[k]; d = k; }
    return d;
  }
};

struct SNode {
  Box3 box;
  int ref_offset = 0, n_refs = 0;
  int second = 0;  // offset of the second child (inner nodes)
};

constexpr int kBuckets = 8;  // Sbvh nBuckets default (sbvh.h:81)
constexpr int kSbvhMaxDepth = 64;

struct SbvhBuild {
  int leaf = 8;
  int depth_guess = 0;
  std::vector<int> prims;  // reference -> primitive
  std::vector<Box3> rbox;
  std::vector<std::array<float, 3>> rcen;
  std::vector<SNode> nodes;

  // computeSplitCost, OverlapSurfaceArea with packed leaves (sbvh.inl:3-37)
  float split_cost(const Box3& l, const Box3& r, int nl, int nr, int depth) const {
    if (depth > 0 && ((float)depth_guess / depth) < 1.5f && nl % leaf != 0 && nr % leaf != 0) return FLT_MAX;
    const Box3 bi = l.intersect(r);
    float cost = ((float)nl / r.area() + (float)nr / l.area()) * std::fabs(bi.area());
    if (!bi.valid()) cost *= -1.0f;
    return cost;
  }

  // computeObjectSplit (sbvh.inl:39-111)
  void object_split(const Box3& bb, const Box3& bc, int depth, int s, int e, int& dim, float& coord) const {
    float best = FLT_MAX;
    dim = -1;
    coord = 0.0f;
    for (int d = 0; d < 3; d++) {
      const float ext = bb.mx[d] - bb.mn[d];
      if (ext < 1e-6f) continue;
      const float width = ext / kBuckets;
      Box3 bbox[kBuckets];
      int bcnt[kBuckets] = {};
      for (int p = s; p < e; p++) {
        int b = (int)((rcen[p][d] - bb.mn[d]) / width);
        b = std::min(std::max(b, 0), kBuckets - 1);
        bbox[b].add_box(rbox[p]);
        bcnt[b] += 1;
      }
      Box3 rb[kBuckets];
      int rc[kBuckets] = {};
      Box3 acc;
      for (int b = kBuckets - 1; b > 0; b--) {
        acc.add_box(bbox[b]);
        rb[b] = acc;
        rc[b] = bcnt[b];
        if (b != kBuckets - 1) rc[b] += rc[b + 1];
      }
      Box3 lb;
      int nl = 0;
      for (int b = 1; b < kBuckets; b++) {
        lb.add_box(bbox[b - 1]);
        nl += bcnt[b - 1];
        if (nl > 0 && rc[b] > 0) {
          const float c = split_cost(lb, rb[b], nl, rc[b], depth);
          if (c < best) {
            best = c;
            dim = d;
            coord = bb.mn[d] + (float)b * width;
          }
        }
      }
    }
    if (dim == -1) {  // LongestAxisCenter fallback
      dim = bc.max_dim();
      coord = (bc.mn[dim] + bc.mx[dim]) * 0.5f;
    }
  }

  // performObjectSplit (sbvh.inl:113-140)
  int partition(int s, int e, int dim, float coord) {
    int mid = s;
    for (int i = s; i < e; i++) {
      if (rcen[i][dim] < coord) {
        std::swap(prims[i], prims[mid]);
        std::swap(rbox[i], rbox[mid]);
        std::swap(rcen[i], rcen[mid]);
        mid++;
      }
    }
    if (mid == s || mid == e) {
      mid = s + (e - s) / 2;
      while ((mid - s) % leaf != 0 && mid < e) mid++;
      if (mid == e) mid = s + (e - s) / 2;
    }
    return mid;
  }

  // buildRecursive (sbvh.inl:142-209): depth-first, left child at index + 1
  void build(int parent, int s, int e, int depth) {
    const int me = (int)nodes.size();
    Box3 bb, bc;
    for (int p = s; p < e; p++) {
      bb.add_box(rbox[p]);
      bc.add_point(rcen[p].data());
    }
    SNode node;
    node.box = bb;
    const int nr = e - s;
    const bool is_leaf = nr <= leaf || depth == kSbvhMaxDepth - 2;
    if (is_leaf) { node.ref_offset = s; node.n_refs = nr; }
    nodes.push_back(node);
    if (parent >= 0 && nodes[parent].second == 0 && me != parent + 1) nodes[parent].second = me - parent;
    if (is_leaf) return;
    int dim;
    float coord;
    object_split(bb, bc, depth, s, e, dim, coord);
    const int mid = partition(s, e, dim, coord);
    build(me, s, mid, depth + 1);
    build(me, mid, e, depth + 1);
  }
};

struct MbvhBuild {
  int branch = 4, leaf = 8;
  const SbvhBuild* sb = nullptr;
  HostFcpwBvh* out = nullptr;

  // collapseSbvh (mbvh.inl:46-133)
  int collapse(int si) {
    const SNode& sn = sb->nodes[si];
    const int mi = out->n_nodes++;
    out->box.resize((size_t)out->n_nodes * branch * 6);
    out->child.resize((size_t)out->n_nodes * branch);
    for (int w = 0; w < branch; w++) {
      float* B = &out->box[((size_t)mi * branch + w) * 6];
      for (int k = 0; k < 3; k++) { B[k] = FLT_MAX; B[3 + k] = -FLT_MAX; }
      out->child[(size_t)mi * branch + w] = INT_MAX;
    }
    if (sn.n_refs > 0) {
      int32_t* C = &out->child[(size_t)mi * branch];
      C[0] = -(out->n_leaves + 1);
      C[1] = sn.n_refs / leaf + (sn.n_refs % leaf != 0 ? 1 : 0);
      C[2] = sn.ref_offset;
      C[3] = sn.n_refs;
      out->n_leaves += C[1];
      return mi;
    }
    int cnt = 2;
    int nodes[8];
    nodes[0] = si + sn.second;
    nodes[1] = si + 1;
    for (;;) {
      if (cnt >= branch) break;
      float best = -FLT_MAX;
      int bi = -1;
      for (int i = 0; i < cnt; i++) {
        const SNode& c = sb->nodes[nodes[i]];
        if (c.n_refs == 0) {
          const float a = c.box.area();
          if (best < a) { best = a; bi = i; }
        }
      }
      if (bi == -1) break;
      const int x = nodes[bi];
      nodes[bi] = x + sb->nodes[x].second;
      nodes[cnt++] = x + 1;
    }
    std::sort(nodes, nodes + cnt);
    for (int i = 0; i < cnt; i++) {
      const SNode& c = sb->nodes[nodes[i]];
      const int ci = collapse(nodes[i]);
      float* B = &out->box[((size_t)mi * branch + i) * 6];
      for (int k = 0; k < 3; k++) { B[k] = c.box.mn[k]; B[3 + k] = c.box.mx[k]; }
      out->child[(size_t)mi * branch + i] = ci;
    }
    return mi;
  }
};

}  // namespace

void build_fcpw_bvh(int dim, const float* verts, const int32_t* prims, int n_prims, int branch, int leaf,
                    HostFcpwBvh& out) {
  out = HostFcpwBvh{};
  out.branch = branch;
  out.leaf = leaf;
  if (n_prims <= 0) return;
  const int nv = dim;  // vertices per primitive
  SbvhBuild sb;
  sb.leaf = leaf;
  sb.depth_guess = (int)std::log2((double)n_prims);
  sb.prims.resize(n_prims);
  sb.rbox.resize(n_prims);
  sb.rcen.resize(n_prims);
  for (int i = 0; i < n_prims; i++) {
    sb.prims[i] = i;
    float P[3][3] = {};
    for (int v = 0; v < nv; v++)
      for (int k = 0; k < dim; k++) P[v][k] = verts[(size_t)prims[(size_t)i * nv + v] * dim + k];
    // LineSegment / Triangle::boundingBox: box(pa) then expandToInclude(pb[, pc])
    Box3 b;
    for (int v = 0; v < nv; v++) b.add_point(P[v]);
    sb.rbox[i] = b;
    for (int k = 0; k < 3; k++)
      sb.rcen[i][k] = nv == 2 ? (P[0][k] + P[1][k]) * 0.5f : (P[0][k] + P[1][k] + P[2][k]) / 3.0f;
  }
  sb.nodes.reserve((size_t)2 * n_prims);
  sb.build(-1, 0, n_prims, 0);
  MbvhBuild mb;
  mb.branch = branch;
  mb.leaf = leaf;
  mb.sb = &sb;
  mb.out = &out;
  mb.collapse(0);
  out.ref.assign(sb.prims.begin(), sb.prims.end());
}

}  // namespace wos
