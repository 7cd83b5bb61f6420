// wos_host_scene.cpp -- host-side scene preparation (no GPU work here).
//
// Replaces what zombie/fcpw do at Scene construction time:
//   OBJ parsing        scene.h:104-145 (2D `v`/`l`), fcpw scene_loader.inl:29-150 (3D `f`)
//   bounding box       fcpw_scene_loader.h:75-93 + bounding_volumes.h:38-49 (FLT_EPSILON pad)
//   vertex/edge normals fcpw.inl:200-221,298-353
//   silhouettes        fcpw.inl:224-293, vertex_silhouettes.inl, edge_silhouettes.inl,
//                      ignore rule sbvh.inl:313-436 + scene.h:84-90
// and packs everything into the flat records described in wos_scene.h.
#include "wos_host_scene.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>

#include "wos_detmath.h"

namespace wos {

namespace {

struct V3 { float x[3] = {0.0f, 0.0f, 0.0f}; };

inline float dot3(const V3& a, const V3& b) { return a.x[0] * b.x[0] + a.x[1] * b.x[1] + a.x[2] * b.x[2]; }
inline V3 sub(const V3& a, const V3& b) { V3 r; for (int k = 0; k < 3; k++) r.x[k] = a.x[k] - b.x[k]; return r; }
inline V3 cross(const V3& a, const V3& b) {
  V3 r;
  r.x[0] = a.x[1] * b.x[2] - a.x[2] * b.x[1];
  r.x[1] = a.x[2] * b.x[0] - a.x[0] * b.x[2];
  r.x[2] = a.x[0] * b.x[1] - a.x[1] * b.x[0];
  return r;
}
inline void normalize(V3& v) {  // Eigen normalized()
  float z = dot3(v, v);
  if (z > 0.0f) { float s = std::sqrt(z); for (int k = 0; k < 3; k++) v.x[k] = v.x[k] / s; }
}
inline V3 seg_normal(const V3& pa, const V3& pb) {  // LineSegment::normal (line_segments.inl:46-55)
  V3 s = sub(pb, pa), n;
  n.x[0] = s.x[1]; n.x[1] = -s.x[0]; n.x[2] = 0.0f;
  return n;
}
inline V3 tri_normal(const V3& pa, const V3& pb, const V3& pc) {  // Triangle::normal
  return cross(sub(pb, pa), sub(pc, pa));
}

struct Geom {
  int dim = 0;
  std::vector<V3> v;
  std::vector<std::array<int, 3>> ix;
  std::vector<V3> vn, en;
  std::vector<std::array<int, 3>> pe;  // 3D edge ids per triangle
};

bool build_geom(Geom& g, int dim, int nv, int np, const float* v, const int32_t* ix, std::string& err) {
  g.dim = dim;
  g.v.resize(nv);
  g.ix.resize(np);
  for (int i = 0; i < nv; i++)
    for (int k = 0; k < dim; k++) g.v[i].x[k] = v[i * dim + k];
  for (int p = 0; p < np; p++) {
    g.ix[p] = {0, 0, 0};
    for (int k = 0; k < dim; k++) {
      int q = ix[p * dim + k];
      if (q < 0 || q >= nv) { err = "primitive " + std::to_string(p) + " references vertex out of range"; return false; }
      g.ix[p][k] = q;
    }
  }
  g.vn.assign(nv, V3());
  if (dim == 2) {
    for (int p = 0; p < np; p++) {
      V3 n = seg_normal(g.v[g.ix[p][0]], g.v[g.ix[p][1]]);
      normalize(n);
      for (int k = 0; k < 2; k++)
        for (int c = 0; c < 3; c++) g.vn[g.ix[p][k]].x[c] += 1.0f * n.x[c];
    }
    for (auto& n : g.vn) normalize(n);
  } else {
    std::map<std::pair<int, int>, int> emap;
    g.pe.resize(np);
    for (int p = 0; p < np; p++)
      for (int j = 0; j < 3; j++) {
        int I = g.ix[p][j], J = g.ix[p][(j + 1) % 3];
        if (I > J) std::swap(I, J);
        auto key = std::make_pair(I, J);
        auto it = emap.find(key);
        int e;
        if (it == emap.end()) { e = (int)emap.size(); emap[key] = e; } else e = it->second;
        g.pe[p][j] = e;
      }
    g.en.assign(emap.size(), V3());
    for (int p = 0; p < np; p++) {
      V3 n = tri_normal(g.v[g.ix[p][0]], g.v[g.ix[p][1]], g.v[g.ix[p][2]]);
      V3 nu = n;
      normalize(nu);
      V3 raw = n;
      float area = 0.5f * std::sqrt(dot3(raw, raw));
      for (int j = 0; j < 3; j++) {
        for (int c = 0; c < 3; c++) g.vn[g.ix[p][j]].x[c] += 1.0f * nu.x[c];
        for (int c = 0; c < 3; c++) g.en[g.pe[p][j]].x[c] += area * nu.x[c];
      }
    }
    for (auto& n : g.vn) normalize(n);
    for (auto& n : g.en) normalize(n);
  }
  return true;
}

void pack_prims(const Geom& g, std::vector<float>& prim, std::vector<float>& aux) {
  const int dim = g.dim, np = (int)g.ix.size();
  prim.clear(); aux.clear();
  for (int p = 0; p < np; p++) {
    if (dim == 2) {
      // 2D record [pa | v = pb - pa]: the edge vector every query (closest point,
      // ray, area, sampling) uses, precomputed with the same float rounding
      const V3 &pa = g.v[g.ix[p][0]], &pb = g.v[g.ix[p][1]];
      prim.push_back(pa.x[0]); prim.push_back(pa.x[1]);
      prim.push_back(pb.x[0] - pa.x[0]); prim.push_back(pb.x[1] - pa.x[1]);
    } else {
      for (int k = 0; k < dim; k++)
        for (int c = 0; c < dim; c++) prim.push_back(g.v[g.ix[p][k]].x[c]);
    }
    if (dim == 2) {
      V3 ns = seg_normal(g.v[g.ix[p][0]], g.v[g.ix[p][1]]);
      normalize(ns);
      const V3* src[3] = {&g.vn[g.ix[p][0]], &g.vn[g.ix[p][1]], &ns};
      for (auto* s : src) { aux.push_back(s->x[0]); aux.push_back(s->x[1]); }
    } else {
      V3 nf = tri_normal(g.v[g.ix[p][0]], g.v[g.ix[p][1]], g.v[g.ix[p][2]]);
      normalize(nf);
      for (int j = 0; j < 3; j++) for (int c = 0; c < 3; c++) aux.push_back(g.vn[g.ix[p][j]].x[c]);
      for (int j = 0; j < 3; j++) for (int c = 0; c < 3; c++) aux.push_back(g.en[g.pe[p][j]].x[c]);
      for (int c = 0; c < 3; c++) aux.push_back(nf.x[c]);
    }
  }
}

bool ignore_candidate(float angle, bool double_sided) { return double_sided ? false : angle < 1e-3f; }

// silhouette candidates, in order of first appearance over primitives
void build_silhouettes(const Geom& g, bool double_sided, std::vector<float>& sil, int& ns) {
  sil.clear(); ns = 0;
  const int nv = (int)g.v.size(), np = (int)g.ix.size();
  if (g.dim == 2) {
    std::vector<int> prev(nv, -1), next(nv, -1);
    for (int p = 0; p < np; p++) { next[g.ix[p][0]] = g.ix[p][1]; prev[g.ix[p][1]] = g.ix[p][0]; }
    std::vector<char> seen(nv, 0);
    for (int p = 0; p < np; p++)
      for (int k = 0; k < 2; k++) {
        int vi = g.ix[p][k];
        if (seen[vi]) continue;
        seen[vi] = 1;
        bool has0 = next[vi] != -1, has1 = prev[vi] != -1;
        V3 n0, n1;
        if (has0) { n0 = seg_normal(g.v[vi], g.v[next[vi]]); normalize(n0); }
        if (has1) { n1 = seg_normal(g.v[prev[vi]], g.v[vi]); normalize(n1); }
        if (has0 && has1) {
          float det = n0.x[0] * n1.x[1] - n1.x[0] * n0.x[1];
          if (ignore_candidate(det, double_sided)) continue;
        }
        const float rec[kSilStride2] = {g.v[vi].x[0], g.v[vi].x[1], n0.x[0], n0.x[1], n1.x[0], n1.x[1],
                                        (has0 && has1) ? 0.0f : 1.0f, 0.0f};
        sil.insert(sil.end(), rec, rec + kSilStride2);
        ns++;
      }
  } else {
    const int ne = (int)g.en.size();
    std::vector<std::array<int, 4>> sidx(ne, {-1, -1, -1, -1});
    for (int p = 0; p < np; p++)
      for (int j = 0; j < 3; j++) {
        int I = j - 1 < 0 ? 2 : j - 1, J = j, K = j + 1 > 2 ? 0 : j + 1;
        int e = g.pe[p][j];
        float orientation = 1.0f;
        if (g.ix[p][J] > g.ix[p][K]) { std::swap(J, K); orientation = -1.0f; }
        sidx[e][orientation == 1.0f ? 0 : 3] = g.ix[p][I];
        sidx[e][1] = g.ix[p][J];
        sidx[e][2] = g.ix[p][K];
      }
    std::vector<char> seen(ne, 0);
    for (int p = 0; p < np; p++)
      for (int k = 0; k < 3; k++) {
        int e = g.pe[p][k];
        if (seen[e]) continue;
        seen[e] = 1;
        bool has0 = sidx[e][3] != -1, has1 = sidx[e][0] != -1;
        V3 n0, n1;
        const V3 &pa = g.v[sidx[e][1]], &pb = g.v[sidx[e][2]];
        if (has0) { n0 = cross(sub(pb, pa), sub(g.v[sidx[e][3]], pa)); normalize(n0); }
        if (has1) { n1 = cross(sub(pa, pb), sub(g.v[sidx[e][0]], pb)); normalize(n1); }
        if (has0 && has1) {
          V3 ed = sub(pb, pa);
          normalize(ed);
          float ang = fatan2(dot3(ed, cross(n0, n1)), dot3(n0, n1));
          if (ignore_candidate(ang, double_sided)) continue;
        }
        float rec[kSilStride3] = {pa.x[0], pa.x[1], pa.x[2], pb.x[0], pb.x[1], pb.x[2], n0.x[0], n0.x[1],
                                  n0.x[2], n1.x[0], n1.x[1], n1.x[2], (has0 && has1) ? 0.0f : 1.0f, 0.0f,
                                  0.0f, 0.0f};
        sil.insert(sil.end(), rec, rec + kSilStride3);
        ns++;
      }
  }
}

}  // namespace

bool prepare_scene(const HostSceneInput& in, HostScene& out, std::string& err) {
  if (in.dim != 2 && in.dim != 3) { err = "dim must be 2 or 3"; return false; }
  if (in.n_vertices < 0 || in.n_prims < 0 || in.n_dvertices < 0 || in.n_dprims < 0) {
    err = "negative mesh size"; return false;
  }
  if ((in.n_prims > 0 && (!in.vertices || !in.prims)) || (in.n_dprims > 0 && (!in.dvertices || !in.dprims))) {
    err = "missing mesh arrays"; return false;
  }
  if (in.n_prims == 0 && in.n_dprims == 0) { err = "scene has no boundary primitives"; return false; }
  out = HostScene();
  out.dim = in.dim;
  Geom neu, dir;
  if (in.n_prims > 0 && !build_geom(neu, in.dim, in.n_vertices, in.n_prims, in.vertices, in.prims, err)) return false;
  if (in.n_dprims > 0 && !build_geom(dir, in.dim, in.n_dvertices, in.n_dprims, in.dvertices, in.dprims, err))
    return false;
  pack_prims(neu, out.prim, out.paux);
  pack_prims(dir, out.dprim, out.dpaux);
  out.n_prims = (int)neu.ix.size();
  out.n_dprims = (int)dir.ix.size();
  build_silhouettes(neu, in.is_double_sided != 0, out.sil, out.n_sil);
  if (in.n_prims > 0) build_fcpw_bvh(in.dim, in.vertices, in.prims, in.n_prims, kFcpwBranch, kFcpwLeaf, out.nbvh);
  // bounding box over all boundary vertices, padded by FLT_EPSILON per vertex
  for (int k = 0; k < 3; k++) { out.pmin[k] = kFltMax; out.pmax[k] = -kFltMax; }
  const Geom* gs[2] = {&neu, &dir};
  for (const Geom* g : gs)
    for (const V3& v : g->v)
      for (int k = 0; k < in.dim; k++) {
        out.pmin[k] = smin(out.pmin[k], v.x[k] - kFltEps);
        out.pmax[k] = smax(out.pmax[k], v.x[k] + kFltEps);
      }
  if (in.dim == 2) { out.pmin[2] = out.pmax[2] = 0.0f; }
  for (int k = 0; k < 3; k++) out.ext[k] = out.pmax[k] - out.pmin[k];
  // culling boxes, padded far beyond float rounding of the kernel's box tests
  float span = 0.0f;
  for (int k = 0; k < in.dim; k++) span = smax(span, out.ext[k]);
  const float pad = 1e-4f * span + 1e-6f;
  auto add_box = [&](std::vector<float>& boxes, const std::vector<const float*>& pts) {
    float lo[3] = {kFltMax, kFltMax, kFltMax}, hi[3] = {-kFltMax, -kFltMax, -kFltMax};
    for (const float* q : pts)
      for (int k = 0; k < in.dim; k++) { lo[k] = smin(lo[k], q[k]); hi[k] = smax(hi[k], q[k]); }
    for (int k = in.dim; k < 3; k++) lo[k] = hi[k] = 0.0f;
    const float rec[kGroupStride] = {lo[0] - pad, lo[1] - pad, lo[2] - pad, 0.0f,
                                     hi[0] + pad, hi[1] + pad, hi[2] + pad, 0.0f};
    boxes.insert(boxes.end(), rec, rec + kGroupStride);
  };
  for (int g0 = 0; g0 < out.n_prims; g0 += kGroup) {
    std::vector<const float*> pts;
    for (int p = g0; p < std::min(out.n_prims, g0 + kGroup); p++)
      for (int c = 0; c < in.dim; c++) pts.push_back(neu.v[neu.ix[p][c]].x);
    add_box(out.pgroup, pts);
    out.n_pgroups++;
  }
  for (int g0 = 0; g0 < out.n_dprims; g0 += kGroup) {
    std::vector<const float*> pts;
    for (int p = g0; p < std::min(out.n_dprims, g0 + kGroup); p++)
      for (int c = 0; c < in.dim; c++) pts.push_back(dir.v[dir.ix[p][c]].x);
    add_box(out.dgroup, pts);
    out.n_dgroups++;
  }
  const int SS = in.dim == 2 ? kSilStride2 : kSilStride3;
  for (int g0 = 0; g0 < out.n_sil; g0 += kGroup) {
    const int g1 = std::min(out.n_sil, g0 + kGroup);
    std::vector<const float*> pts;
    for (int q = g0; q < g1; q++) {
      pts.push_back(&out.sil[(size_t)q * SS]);
      if (in.dim == 3) pts.push_back(&out.sil[(size_t)q * SS + 3]);
    }
    std::vector<float> box;
    add_box(box, pts);
    // bounding sphere of the candidates (centre of the box; radius padded)
    double c[3], rho = 0.0;
    for (int k = 0; k < 3; k++) c[k] = 0.5 * ((double)box[k] + (double)box[4 + k]);
    for (const float* q : pts) {
      double r2 = 0.0;
      for (int k = 0; k < in.dim; k++) r2 += ((double)q[k] - c[k]) * ((double)q[k] - c[k]);
      rho = std::max(rho, std::sqrt(r2));
    }
    rho += pad;
    // cone of the adjacent normals n0, n1 of every candidate
    const int o0 = in.dim == 2 ? 2 : 6, o1 = in.dim == 2 ? 4 : 9, om = in.dim == 2 ? 6 : 12;
    double ax[3] = {0, 0, 0};
    bool nocull = false;
    for (int q = g0; q < g1; q++) {
      const float* S = &out.sil[(size_t)q * SS];
      if (S[om] != 0.0f) nocull = true;  // candidates next to a missing primitive are always silhouettes
      for (int k = 0; k < in.dim; k++) ax[k] += (double)S[o0 + k] + (double)S[o1 + k];
    }
    double an = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
    double alpha = 0.0;
    if (an < 1e-6) {
      nocull = true;
    } else {
      for (int k = 0; k < 3; k++) ax[k] /= an;
      for (int q = g0; q < g1; q++) {
        const float* S = &out.sil[(size_t)q * SS];
        for (int o : {o0, o1}) {
          double nn = 0.0, dt = 0.0;
          for (int k = 0; k < in.dim; k++) { nn += (double)S[o + k] * S[o + k]; dt += ax[k] * S[o + k]; }
          nn = std::sqrt(nn);
          double cosang = nn > 0.0 ? std::max(-1.0, std::min(1.0, dt / nn)) : -1.0;
          alpha = std::max(alpha, std::acos(cosang));
        }
      }
      alpha += 1e-3;
      if (alpha >= 1.5) nocull = true;  // a cone this wide never certifies a face direction
    }
    float rec[kSGroupStride] = {box[0], box[1], box[2], (float)std::sin(alpha),
                                box[4], box[5], box[6], (float)std::cos(alpha),
                                (float)c[0], (float)c[1], (float)c[2], (float)rho,
                                (float)ax[0], (float)ax[1], (float)ax[2], nocull ? 1.0f : 0.0f};
    out.sgroup.insert(out.sgroup.end(), rec, rec + kSGroupStride);
    out.n_sgroups++;
  }
  build_group_tree(out.pgroup, kGroupStride, out.n_pgroups, out.ptree);
  build_group_tree(out.sgroup, kSGroupStride, out.n_sgroups, out.stree);
  build_group_tree(out.dgroup, kGroupStride, out.n_dgroups, out.dtree);
  return true;
}

void build_group_tree(const std::vector<float>& groups, int stride, int ngroups, HostTree& t) {
  t = HostTree{};
  t.n[0] = ngroups;
  if (ngroups <= kTreeMinGroups) return;
  // level L's boxes: unions of the 8 consecutive boxes of level L-1 (the padded group
  // boxes at L = 1), so every node box contains its groups' padded boxes
  int prev_n = ngroups, L = 0;
  while (prev_n > 8 && L < kTreeLevels) {
    L++;
    const int n = (prev_n + 7) / 8;
    const size_t base = t.node.size() / kGroupStride;
    t.off[L] = (int)base;
    t.n[L] = n;
    for (int i = 0; i < n; i++) {
      float lo[3] = {kFltMax, kFltMax, kFltMax}, hi[3] = {-kFltMax, -kFltMax, -kFltMax};
      for (int c = 8 * i; c < std::min(prev_n, 8 * i + 8); c++) {
        const float* B = L == 1 ? &groups[(size_t)c * stride] : &t.node[((size_t)t.off[L - 1] + c) * kGroupStride];
        for (int k = 0; k < 3; k++) { lo[k] = smin(lo[k], B[k]); hi[k] = smax(hi[k], B[4 + k]); }
      }
      const float rec[kGroupStride] = {lo[0], lo[1], lo[2], 0.0f, hi[0], hi[1], hi[2], 0.0f};
      t.node.insert(t.node.end(), rec, rec + kGroupStride);
    }
    prev_n = n;
  }
  t.levels = L;
}

// ---------------------------------------------------------------------------
// star-radius cell grid (wos_host_scene.h StarGrid)
// ---------------------------------------------------------------------------
namespace {

struct SilGeo {
  double a[3] = {0, 0, 0}, b[3] = {0, 0, 0}, mid[3] = {0, 0, 0};
  double n0[3] = {0, 0, 0}, n1[3] = {0, 0, 0};
  double e0 = 0.0, e1 = 0.0;  // slack of the normal components along the edge (3D)
  double half = 0.0;
  bool miss = false;
};

double seg_point_dist(const SilGeo& s, const double* q, int dim) {
  double u[3] = {0, 0, 0}, uu = 0.0, uv = 0.0;
  for (int k = 0; k < dim; k++) {
    u[k] = s.b[k] - s.a[k];
    uu += u[k] * u[k];
    uv += u[k] * (q[k] - s.a[k]);
  }
  const double t = uu > 0.0 ? std::min(1.0, std::max(0.0, uv / uu)) : 0.0;
  double d2 = 0.0;
  for (int k = 0; k < dim; k++) {
    const double w = q[k] - (s.a[k] + t * u[k]);
    d2 += w * w;
  }
  return std::sqrt(d2);
}

double box_point_dist(const double* lo, const double* hi, const double* p, int dim) {
  double d2 = 0.0;
  for (int k = 0; k < dim; k++) {
    const double e = std::max(std::max(lo[k] - p[k], p[k] - hi[k]), 0.0);
    d2 += e * e;
  }
  return std::sqrt(d2);
}

}  // namespace

// Distance between an axis-aligned box [lo, hi] and the segment a-b (2D, double): 0 when
// they meet, else the smallest of the endpoints' box distances and the corners' segment
// distances (two disjoint convex polygons are closest at a vertex of one of them).
double box_seg_dist2d(const double* lo, const double* hi, const double* a, const double* b) {
  // Liang-Barsky clip of a + t (b - a), t in [0, 1], against the box
  double t0 = 0.0, t1 = 1.0;
  bool meets = true;
  for (int k = 0; k < 2 && meets; k++) {
    const double d = b[k] - a[k];
    if (d == 0.0) {
      if (a[k] < lo[k] || a[k] > hi[k]) meets = false;
    } else {
      double u = (lo[k] - a[k]) / d, v = (hi[k] - a[k]) / d;
      if (u > v) std::swap(u, v);
      t0 = std::max(t0, u);
      t1 = std::min(t1, v);
      if (t0 > t1) meets = false;
    }
  }
  if (meets) return 0.0;
  SilGeo g;
  for (int k = 0; k < 2; k++) { g.a[k] = a[k]; g.b[k] = b[k]; }
  double m = std::min(box_point_dist(lo, hi, a, 2), box_point_dist(lo, hi, b, 2));
  for (int q = 0; q < 4; q++) {
    const double c[3] = {(q & 1) ? hi[0] : lo[0], (q & 2) ? hi[1] : lo[1], 0.0};
    m = std::min(m, seg_point_dist(g, c, 2));
  }
  return m;
}

// For a cell box C (enlarged beyond the kernel's cell-index rounding) and a
// candidate s with adjacent normals n0, n1:
//   * f_i(x) = (x - a).n_i is linear in x, so its range over C is spanned by the
//     corners (3D edges: the closest point slides along the edge, which moves f_i
//     by at most |(b - a).n_i|, ~0 up to the records' rounding);
//   * the view length |x - closest(s)| is convex in x: at most its corner maximum
//     dmax, at least the box distance dmin (3D: box distance of the midpoint minus
//     the half length);
// so f_i > t*dmax over C proves the normalised dot u.n_i > t for every x in C.
// With t = prec + 1e-4 (the kernel's dots are accurate to ~1e-6) and dmin above
// prec (the exact test's direction branch): both dots of one sign -> the exact
// test rejects everywhere (culled); opposite signs -> it accepts everywhere
// (certain).  U = min over certain candidates of dmax bounds the result; a
// candidate with dmin > max(U, minR) (with margin) is strictly farther than a
// certain silhouette and cannot be the minR break either, so it never decides.
bool build_star_grid(const HostScene& hs, float prec, float min_r, size_t budget_bytes, StarGrid& out) {
  out = StarGrid();
  out.prec = prec;
  out.min_r = min_r;
  const int dim = hs.dim, ns = hs.n_sil;
  if (ns <= 0 || ns > 255) return false;
  const int SS = dim == 2 ? kSilStride2 : kSilStride3;
  const int o0 = dim == 2 ? 2 : 6, o1 = dim == 2 ? 4 : 9, om = dim == 2 ? 6 : 12;
  std::vector<SilGeo> sg(ns);
  for (int s = 0; s < ns; s++) {
    const float* S = &hs.sil[(size_t)s * SS];
    SilGeo& g = sg[s];
    double len2 = 0.0, d0 = 0.0, d1 = 0.0;
    for (int k = 0; k < dim; k++) {
      g.a[k] = S[k];
      g.b[k] = dim == 2 ? S[k] : S[3 + k];
      g.n0[k] = S[o0 + k];
      g.n1[k] = S[o1 + k];
      g.mid[k] = 0.5 * (g.a[k] + g.b[k]);
      const double e = g.b[k] - g.a[k];
      len2 += e * e;
      d0 += e * g.n0[k];
      d1 += e * g.n1[k];
    }
    g.miss = S[om] != 0.0f;
    g.half = 0.5 * std::sqrt(len2);
    g.e0 = std::fabs(d0) + 1e-6 * std::sqrt(len2);
    g.e1 = std::fabs(d1) + 1e-6 * std::sqrt(len2);
  }
  double span = 0.0;
  for (int k = 0; k < dim; k++) span = std::max(span, (double)hs.ext[k]);
  if (!(span > 0.0)) return false;
  const double gpad = 1e-3 * span + 1e-6;
  double glo[3] = {0, 0, 0}, gext[3] = {1, 1, 1}, vol = 1.0;
  for (int k = 0; k < dim; k++) {
    glo[k] = (double)hs.pmin[k] - gpad;
    gext[k] = ((double)hs.pmax[k] + gpad) - glo[k];
    vol *= gext[k];
  }
  const double t = (double)prec + 1e-4;
  const double near = 1.01 * (double)prec + 1e-6 * span + 1e-7;
  const double dslack = 1e-5 * span;
  const int ncorner = 1 << dim;
  std::vector<double> mind(ns), maxd(ns);
  std::vector<char> culled(ns);
  for (int target = 4096; target >= 64; target /= 2) {
    const double h = std::pow(vol / target, 1.0 / dim);
    int n[3] = {1, 1, 1};
    float gmin[3] = {0, 0, 0}, inv[3] = {0, 0, 0};
    for (int k = 0; k < dim; k++) {
      n[k] = std::max(1, (int)std::ceil(gext[k] / h));
      gmin[k] = (float)glo[k];
      inv[k] = (float)((double)n[k] / gext[k]);
    }
    const int ncell = n[0] * n[1] * n[2];
    std::vector<uint16_t> off((size_t)ncell + 1, 0);
    std::vector<uint8_t> lst;
    bool overflow = false;
    for (int c = 0; c < ncell && !overflow; c++) {
      const int ic[3] = {c % n[0], (c / n[0]) % n[1], c / (n[0] * n[1])};
      double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
      for (int k = 0; k < dim; k++) {
        const double w = 1.0 / (double)inv[k];
        const double delta = 1e-3 * w + 1e-5 * span;
        lo[k] = (double)gmin[k] + ic[k] * w - delta;
        hi[k] = (double)gmin[k] + (ic[k] + 1) * w + delta;
      }
      double U = HUGE_VAL;
      for (int s = 0; s < ns; s++) {
        const SilGeo& g = sg[s];
        double dmax = 0.0, f0lo = HUGE_VAL, f0hi = -HUGE_VAL, f1lo = HUGE_VAL, f1hi = -HUGE_VAL;
        for (int q = 0; q < ncorner; q++) {
          double cq[3] = {0, 0, 0};
          for (int k = 0; k < dim; k++) cq[k] = ((q >> k) & 1) ? hi[k] : lo[k];
          dmax = std::max(dmax, seg_point_dist(g, cq, dim));
          double f0 = 0.0, f1 = 0.0;
          for (int k = 0; k < dim; k++) {
            f0 += (cq[k] - g.a[k]) * g.n0[k];
            f1 += (cq[k] - g.a[k]) * g.n1[k];
          }
          f0lo = std::min(f0lo, f0); f0hi = std::max(f0hi, f0);
          f1lo = std::min(f1lo, f1); f1hi = std::max(f1hi, f1);
        }
        f0lo -= g.e0; f0hi += g.e0; f1lo -= g.e1; f1hi += g.e1;
        const double dmin = dim == 2 ? box_point_dist(lo, hi, g.a, dim)
                                     : std::max(0.0, box_point_dist(lo, hi, g.mid, dim) - g.half);
        mind[s] = dmin;
        maxd[s] = dmax * (1.0 + 1e-9);
        culled[s] = 0;
        bool certain = g.miss;
        if (!g.miss && dmin > near) {
          const double tm = t * dmax;
          const bool pos0 = f0lo > tm, neg0 = f0hi < -tm, pos1 = f1lo > tm, neg1 = f1hi < -tm;
          culled[s] = (pos0 && pos1) || (neg0 && neg1);
          certain = (pos0 && neg1) || (neg0 && pos1);
        }
        if (certain) U = std::min(U, maxd[s]);
      }
      const double thr = std::max(U, (double)min_r) * (1.0 + 1e-4) + dslack;
      for (int s = 0; s < ns; s++)
        if (!culled[s] && !(mind[s] > thr)) lst.push_back((uint8_t)s);
      if (lst.size() > 65535) overflow = true;
      off[(size_t)c + 1] = (uint16_t)lst.size();
    }
    if (overflow) continue;
    const int off_words = (ncell + 2) / 2;
    const int list_words = ((int)lst.size() + 3) / 4;
    if ((size_t)(off_words + list_words) * 4 > budget_bytes) continue;
    out.words.assign((size_t)off_words + list_words, 0u);
    std::memcpy(out.words.data(), off.data(), off.size() * sizeof(uint16_t));
    if (!lst.empty()) std::memcpy(out.words.data() + off_words, lst.data(), lst.size());
    for (int k = 0; k < 3; k++) {
      out.n[k] = n[k];
      out.gmin[k] = gmin[k];
      out.inv[k] = inv[k];
    }
    out.ncell = ncell;
    out.off_words = off_words;
    out.list_len = lst.size();
    return true;
  }
  return false;
}

// ---------------------------------------------------------------------------
// rejection bound table (wos_host_scene.h)
// ---------------------------------------------------------------------------
namespace {

double yukawa_q(int dim, double s, double x) {
  if (dim == 2) {
    const double k0s = bessk0(s), i0s = bessi0(s);
    return bessk0(s * x) - k0s / i0s * bessi0(s * x);
  }
  const double sx = s * x;
  const double sh = 0.5 * (std::exp(sx) - std::exp(-sx));
  const double shs = 0.5 * (std::exp(s) - std::exp(-s));
  return std::exp(-sx) - std::exp(-s) * sh / shs;
}

double yukawa_f(int dim, double s) {
  // max over x in (0, 1] of x * Q_s(x): coarse grid, then golden-section on the
  // bracket of the best sample (x Q_s(x) is unimodal)
  const int n = 256;
  double best = 0.0;
  int bi = 1;
  for (int i = 1; i <= n; i++) {
    const double x = (double)i / n;
    const double v = x * yukawa_q(dim, s, x);
    if (v > best) { best = v; bi = i; }
  }
  double a = (double)(bi - 1) / n, b = (double)std::min(bi + 1, n) / n;
  if (a <= 0.0) a = 1e-9;
  const double g = 0.5 * (std::sqrt(5.0) - 1.0);
  double c = b - g * (b - a), d = a + g * (b - a);
  double fc = c * yukawa_q(dim, s, c), fd = d * yukawa_q(dim, s, d);
  for (int it = 0; it < 60; it++) {
    if (fc > fd) { b = d; d = c; fd = fc; c = b - g * (b - a); fc = c * yukawa_q(dim, s, c); }
    else { a = c; c = d; fc = fd; d = a + g * (b - a); fd = d * yukawa_q(dim, s, d); }
  }
  return std::max(best, std::max(fc, fd));
}

}  // namespace

void rejection_bound_table(int dim, float* tab) {
  for (int k = 0; k < kRejTabBins; k++) {
    const double lo = std::max(1e-6, ((double)k / kRejTabScale) * ((double)k / kRejTabScale));
    const double hi = ((double)(k + 1) / kRejTabScale) * ((double)(k + 1) / kRejTabScale);
    double m = 0.0;
    for (int j = 0; j <= 15; j++) m = std::max(m, yukawa_f(dim, lo + (hi - lo) * j / 15.0));
    tab[k] = (float)(1.02 * m);
  }
}

// ---------------------------------------------------------------------------
// OBJ parsing
// ---------------------------------------------------------------------------
static int parse_face_index(const std::string& token) {  // scene_loader.inl:29-44
  std::stringstream in(token);
  std::string s;
  int idx[3] = {1, 1, 1};
  int i = 0;
  while (std::getline(in, s, '/')) {
    if (s != "\\") {
      std::stringstream ss(s);
      if (i < 3) ss >> idx[i++];
    }
  }
  return idx[0] - 1;
}

bool load_obj(const std::string& path, int dim, bool flip, bool normalize_domain, std::vector<float>& verts,
              std::vector<int32_t>& prims, std::string& err) {
  std::ifstream obj(path);
  if (!obj) { err = "Error opening file: " + path; return false; }
  verts.clear(); prims.clear();
  std::string line;
  if (dim == 2) {
    // scene.h:104-145
    while (std::getline(obj, line)) {
      std::istringstream ss(line);
      std::string token;
      ss >> token;
      if (token == "v") {
        float x = 0.0f, y = 0.0f;
        ss >> x >> y;
        verts.push_back(x); verts.push_back(y);
      } else if (token == "l") {
        size_t i = 0, j = 0;
        ss >> i >> j;
        if (flip) { prims.push_back((int32_t)(j - 1)); prims.push_back((int32_t)(i - 1)); }
        else { prims.push_back((int32_t)(i - 1)); prims.push_back((int32_t)(j - 1)); }
      }
    }
  } else {
    // fcpw loadTriangleSoupFromOBJFile (scene_loader.inl:100-150)
    while (std::getline(obj, line)) {
      std::stringstream ss(line);
      std::string token;
      ss >> token;
      if (token == "v") {
        float x = 0.0f, y = 0.0f, z = 0.0f;
        ss >> x >> y >> z;
        verts.push_back(x); verts.push_back(y); verts.push_back(z);
      } else if (token == "f") {
        while (ss >> token) {
          int pos = parse_face_index(token);
          if (pos < 0) {
            if (!std::getline(obj, line)) break;
            size_t i = line.find_first_not_of("\t\n\v\f\r ");
            if (i == std::string::npos) continue;
            pos = parse_face_index(line.substr(i));
          }
          prims.push_back(pos);
        }
      }
    }
    if (prims.size() % 3 != 0) { err = "OBJ face index count is not a multiple of 3 (triangles only)"; return false; }
    if (flip)
      for (size_t t = 0; t < prims.size(); t += 3) std::swap(prims[t + 1], prims[t + 2]);
  }
  const int nv = (int)(verts.size() / dim);
  for (int32_t q : prims)
    if (q < 0 || q >= nv) { err = "OBJ index out of range in " + path; return false; }
  if (normalize_domain && nv > 0) {
    // scene.h:132-142
    float cm[3] = {0.0f, 0.0f, 0.0f};
    for (int i = 0; i < nv; i++) for (int k = 0; k < dim; k++) cm[k] += verts[i * dim + k];
    for (int k = 0; k < dim; k++) cm[k] /= (float)nv;
    float radius = 0.0f;
    for (int i = 0; i < nv; i++) {
      float s = 0.0f;
      for (int k = 0; k < dim; k++) { verts[i * dim + k] -= cm[k]; s += verts[i * dim + k] * verts[i * dim + k]; }
      radius = smax(radius, std::sqrt(s));
    }
    for (int i = 0; i < nv; i++) for (int k = 0; k < dim; k++) verts[i * dim + k] /= radius;
  }
  return true;
}


bool build_dirichlet_grid(const HostScene& hs, DirGrid& out) {
  out = DirGrid();
  const int nd = hs.n_dprims;
  if (hs.dim != 2 || nd <= 0 || nd > 65535) return false;
  // segments a, b = a + v as the kernels' records hold them
  std::vector<double> sa(2 * (size_t)nd), sb(2 * (size_t)nd);
  for (int p = 0; p < nd; p++) {
    const float* P = &hs.dprim[(size_t)p * kPrimStride2];
    for (int k = 0; k < 2; k++) {
      sa[2 * p + k] = P[k];
      sb[2 * p + k] = (double)P[k] + (double)P[2 + k];
    }
  }
  double span = std::max((double)hs.ext[0], (double)hs.ext[1]);
  if (!(span > 0.0)) return false;
  const double gpad = 1e-3 * span + 1e-6;
  double glo[2], gext[2];
  for (int k = 0; k < 2; k++) {
    glo[k] = (double)hs.pmin[k] - gpad;
    gext[k] = ((double)hs.pmax[k] + gpad) - glo[k];
  }
  const double vol = gext[0] * gext[1];
  const double slack = 1e-5 * span;
  // the finest grid up to 128 x 128 cells whose lists stay short (the cost scales with ncell x nd)
  const int target = nd <= 512 ? 16384 : (nd <= 4096 ? 4096 : 1024);
  const double h = std::sqrt(vol / target);
  for (int k = 0; k < 2; k++) {
    out.n[k] = std::max(1, (int)std::ceil(gext[k] / h));
    out.gmin[k] = (float)glo[k];
    out.inv[k] = (float)((double)out.n[k] / gext[k]);
  }
  out.ncell = out.n[0] * out.n[1];
  std::vector<uint32_t> off((size_t)out.ncell + 1, 0u);
  std::vector<uint16_t> lst;
  std::vector<double> mind(nd);
  for (int c = 0; c < out.ncell; c++) {
    const int ic[2] = {c % out.n[0], c / out.n[0]};
    double lo[2], hi[2];
    for (int k = 0; k < 2; k++) {
      const double w = 1.0 / (double)out.inv[k];
      const double delta = 1e-3 * w + 1e-5 * span;
      lo[k] = (double)out.gmin[k] + ic[k] * w - delta;
      hi[k] = (double)out.gmin[k] + (ic[k] + 1) * w + delta;
    }
    double U = HUGE_VAL;
    for (int p = 0; p < nd; p++) {
      const double* a = &sa[2 * p];
      const double* b = &sb[2 * p];
      SilGeo g;
      for (int k = 0; k < 2; k++) { g.a[k] = a[k]; g.b[k] = b[k]; }
      double dmax = 0.0;
      for (int q = 0; q < 4; q++) {
        const double cq[3] = {(q & 1) ? hi[0] : lo[0], (q & 2) ? hi[1] : lo[1], 0.0};
        dmax = std::max(dmax, seg_point_dist(g, cq, 2));
      }
      U = std::min(U, dmax);
      mind[p] = box_seg_dist2d(lo, hi, a, b);
    }
    const double thr = U * (1.0 + 1e-4) + slack;
    for (int p = 0; p < nd; p++)
      if (!(mind[p] > thr)) lst.push_back((uint16_t)p);
    off[(size_t)c + 1] = (uint32_t)lst.size();
    out.max_list = std::max(out.max_list, (int)(off[(size_t)c + 1] - off[c]));
  }
  out.list_len = lst.size();
  // worth it only while the lists are short against the culled scan
  if (out.max_list > 256 || out.list_len > (size_t)out.ncell * 16) return false;
  out.off_words = out.ncell + 1;
  out.words.assign((size_t)out.off_words + (lst.size() + 1) / 2, 0u);
  std::memcpy(out.words.data(), off.data(), off.size() * sizeof(uint32_t));
  if (!lst.empty()) std::memcpy(out.words.data() + out.off_words, lst.data(), lst.size() * sizeof(uint16_t));
  return true;
}

}  // namespace wos
