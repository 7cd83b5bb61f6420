// Test-only C shim over the host scene preparation (csrc/wos_host_scene.cpp), built
// with plain g++ by tests/test_host_scene.py so the culling records (group boxes,
// silhouette cones) can be checked on the CPU.  Not part of the product library.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "wos_host_scene.h"

extern "C" int hs_prepare(int dim, const float* v, int nv, const int* ix, int np, int double_sided, float* prim,
                          int prim_cap, float* sil, int sil_cap, float* pg, int pg_cap, float* sg, int sg_cap,
                          int* counts) {
  wos::HostSceneInput in;
  in.dim = dim;
  in.vertices = v; in.n_vertices = nv;
  in.prims = ix; in.n_prims = np;
  in.is_double_sided = double_sided;
  wos::HostScene out;
  std::string err;
  if (!wos::prepare_scene(in, out, err)) return -1;
  if ((int)out.prim.size() > prim_cap || (int)out.sil.size() > sil_cap || (int)out.pgroup.size() > pg_cap ||
      (int)out.sgroup.size() > sg_cap)
    return -2;
  std::copy(out.prim.begin(), out.prim.end(), prim);
  std::copy(out.sil.begin(), out.sil.end(), sil);
  std::copy(out.pgroup.begin(), out.pgroup.end(), pg);
  std::copy(out.sgroup.begin(), out.sgroup.end(), sg);
  counts[0] = out.n_prims; counts[1] = out.n_sil; counts[2] = out.n_pgroups; counts[3] = out.n_sgroups;
  return 0;
}

// ---- star-radius grid soundness: full sequential scan vs the grid cell's list ----
namespace {

float dotf(const float* a, const float* b, int dim) {
  float s = a[0] * b[0] + a[1] * b[1];
  if (dim == 3) s = s + a[2] * b[2];
  return s;
}

// isWideSilhouetteVertex / Edge in float (the oracle's is_silhouette)
bool is_sil(int dim, const float* S, const float* view, float d, bool flip, float prec) {
  const float sign = flip ? 1.0f : -1.0f;
  const float* n0 = dim == 2 ? S + 2 : S + 6;
  const float* n1 = dim == 2 ? S + 4 : S + 9;
  if (!(d > prec)) {
    if (dim == 2) return sign * (n0[0] * n1[1] - n0[1] * n1[0]) > prec;
    float ed[3] = {S[3] - S[0], S[4] - S[1], S[5] - S[2]};
    float inv = 1.0f / std::sqrt(dotf(ed, ed, 3));
    for (float& e : ed) e *= inv;
    float c[3] = {n0[1] * n1[2] - n0[2] * n1[1], n0[2] * n1[0] - n0[0] * n1[2], n0[0] * n1[1] - n0[1] * n1[0]};
    return sign * std::atan2(dotf(ed, c, 3), dotf(n0, n1, 3)) > prec;
  }
  const float inv = 1.0f / d;
  float u[3] = {view[0] * inv, view[1] * inv, dim == 3 ? view[2] * inv : 0.0f};
  const float d0 = dotf(u, n0, dim), d1 = dotf(u, n1, dim);
  if (std::fabs(d0) <= prec) return sign * d1 > prec;
  if (std::fabs(d1) <= prec) return sign * d0 > prec;
  return d0 * d1 < 0.0f;
}

// one candidate: accepted with d^2 <= r2?  (view and d as the kernel computes them)
bool cand(int dim, const float* S, const float* x, float r2, bool flip, float prec, float* d2o, float* dout) {
  float view[3] = {0, 0, 0}, d;
  if (dim == 2) {
    view[0] = x[0] - S[0]; view[1] = x[1] - S[1];
    d = std::sqrt(view[0] * view[0] + view[1] * view[1]);
  } else {
    float u[3], v[3];
    for (int k = 0; k < 3; k++) { u[k] = S[3 + k] - S[k]; v[k] = x[k] - S[k]; }
    float c1 = dotf(u, v, 3), c2 = dotf(u, u, 3);
    float t = c1 * (1.0f / c2);
    if (c1 <= 0.0f) t = 0.0f;
    if (c2 <= c1) t = 1.0f;
    for (int k = 0; k < 3; k++) view[k] = x[k] - (S[k] + u[k] * t);
    d = std::sqrt(dotf(view, view, 3));
  }
  const float d2 = d * d;
  if (!(d2 <= r2)) return false;
  const bool miss = (dim == 2 ? S[6] : S[12]) != 0.0f;
  if (!miss && !is_sil(dim, S, view, d, flip, prec)) return false;
  *d2o = d2;
  *dout = d;
  return true;
}

float star_scan(int dim, const std::vector<float>& sil, const int* idx, int n, const float* x, float minR, float maxR,
                bool flip, float prec) {
  if (minR > maxR) return maxR;
  const int SS = dim == 2 ? wos::kSilStride2 : wos::kSilStride3;
  float r2 = maxR * maxR, minR2 = minR * minR, best = 0.0f;
  bool found = false;
  if (!(minR2 >= r2)) {
    for (int e = 0; e < n; e++) {
      float d2, d;
      if (cand(dim, &sil[(size_t)idx[e] * SS], x, r2, flip, prec, &d2, &d)) {
        r2 = d2; best = d; found = true;
        if (minR2 >= r2) break;
      }
    }
  }
  return found ? std::max(best, minR) : std::max(maxR, minR);
}

}  // namespace

// info[0..9]: ok, ncell, list_len, bytes, n0, n1, n2, points in the grid, max list length, 0
extern "C" int hs_star_grid_check(int dim, const float* v, int nv, const int* ix, int np, int double_sided,
                                  float prec, float min_r, const float* pts, int npts, int budget, int* info) {
  wos::HostSceneInput in;
  in.dim = dim;
  in.vertices = v; in.n_vertices = nv;
  in.prims = ix; in.n_prims = np;
  in.is_double_sided = double_sided;
  wos::HostScene hs;
  std::string err;
  if (!wos::prepare_scene(in, hs, err)) return -1;
  wos::StarGrid g;
  const bool ok = wos::build_star_grid(hs, prec, min_r, (size_t)budget, g);
  for (int k = 0; k < 10; k++) info[k] = 0;
  info[0] = ok;
  if (!ok) return 0;
  info[1] = g.ncell; info[2] = (int)g.list_len; info[3] = (int)(g.words.size() * 4);
  info[4] = g.n[0]; info[5] = g.n[1]; info[6] = g.n[2];
  const uint16_t* off = reinterpret_cast<const uint16_t*>(g.words.data());
  const uint8_t* lst = reinterpret_cast<const uint8_t*>(g.words.data() + g.off_words);
  for (int c = 0; c < g.ncell; c++) info[8] = std::max(info[8], (int)(off[c + 1] - off[c]));
  std::vector<int> all(hs.n_sil);
  for (int s = 0; s < hs.n_sil; s++) all[s] = s;
  int mismatches = 0;
  for (int i = 0; i < npts; i++) {
    const float* x = pts + (size_t)i * dim;
    // cell index exactly as the kernel computes it (star_cell)
    int c = 0;
    bool inside = true;
    for (int k = dim - 1; k >= 0 && inside; k--) {
      const float vv = (x[k] - g.gmin[k]) * g.inv[k];
      if (!(vv >= 0.0f && vv < (float)g.n[k])) { inside = false; break; }
      int ii = (int)vv;
      if (ii > g.n[k] - 1) ii = g.n[k] - 1;
      c = c * g.n[k] + ii;
    }
    if (!inside) continue;
    info[7]++;
    // maxR: far bbox corner distance (no Dirichlet geometry)
    float m2 = 0.0f;
    for (int k = 0; k < dim; k++) {
      const float m = std::min(hs.pmin[k] - x[k], x[k] - hs.pmax[k]);
      m2 += m * m;
    }
    const float maxR = std::sqrt(m2);
    std::vector<int> sub;
    for (int e = off[c]; e < off[c + 1]; e++) sub.push_back(lst[e]);
    for (int flip = 0; flip < 2; flip++) {
      const float a = star_scan(dim, hs.sil, all.data(), hs.n_sil, x, min_r, maxR, flip != 0, prec);
      const float b = star_scan(dim, hs.sil, sub.data(), (int)sub.size(), x, min_r, maxR, flip != 0, prec);
      if (std::memcmp(&a, &b, sizeof(float)) != 0) mismatches++;
    }
  }
  return mismatches;
}

// ---- Dirichlet-distance grid soundness: for every point inside the grid, every segment
// whose true (double) distance is within a relative 1e-6 (+ 1e-7 of the span) of the
// nearest one -- every segment the float scan could pick -- is on the point's cell list
// (cell index exactly as the kernel computes it, dirichlet_dist_grid).
extern "C" int hs_dir_grid_check(const float* v, int nv, const int* ix, int np, const float* dv, int ndv,
                                 const int* dix, int nd, const float* pts, int npts, int* info) {
  wos::HostSceneInput in;
  in.dim = 2;
  in.vertices = v; in.n_vertices = nv;
  in.prims = ix; in.n_prims = np;
  in.dvertices = dv; in.n_dvertices = ndv;
  in.dprims = dix; in.n_dprims = nd;
  wos::HostScene hs;
  std::string err;
  if (!wos::prepare_scene(in, hs, err)) return -1;
  wos::DirGrid g;
  const bool ok = wos::build_dirichlet_grid(hs, g);
  for (int k = 0; k < 8; k++) info[k] = 0;
  info[0] = ok;
  info[1] = g.ncell; info[2] = (int)g.list_len; info[3] = g.max_list; info[4] = g.n[0]; info[5] = g.n[1];
  if (!ok) return 0;
  const uint32_t* off = g.words.data();
  const uint16_t* lst = reinterpret_cast<const uint16_t*>(g.words.data() + g.off_words);
  const double span = std::max(hs.ext[0], hs.ext[1]);
  int bad = 0;
  for (int i = 0; i < npts; i++) {
    const float* x = pts + (size_t)i * 2;
    int c = 0;
    bool inside = true;
    for (int k = 1; k >= 0; k--) {
      const float vv = (x[k] - g.gmin[k]) * g.inv[k];
      if (!(vv >= 0.0f && vv < (float)g.n[k])) { inside = false; break; }
      int ii = (int)vv;
      if (ii > g.n[k] - 1) ii = g.n[k] - 1;
      c = c * g.n[k] + ii;
    }
    if (!inside) continue;
    info[6]++;
    std::vector<double> d(hs.n_dprims);
    double m = HUGE_VAL;
    for (int p = 0; p < hs.n_dprims; p++) {
      const float* P = &hs.dprim[(size_t)p * wos::kPrimStride2];
      const double a[2] = {P[0], P[1]}, u[2] = {P[2], P[3]};
      const double uu = u[0] * u[0] + u[1] * u[1];
      const double t = uu > 0.0 ? std::min(1.0, std::max(0.0, (u[0] * (x[0] - a[0]) + u[1] * (x[1] - a[1])) / uu)) : 0.0;
      const double w0 = x[0] - (a[0] + t * u[0]), w1 = x[1] - (a[1] + t * u[1]);
      d[p] = std::sqrt(w0 * w0 + w1 * w1);
      m = std::min(m, d[p]);
    }
    const double thr = m * (1.0 + 1e-6) + 1e-7 * span;
    for (int p = 0; p < hs.n_dprims; p++) {
      if (d[p] > thr) continue;
      if (!std::binary_search(lst + off[c], lst + off[c + 1], (uint16_t)p)) bad++;
    }
  }
  return bad;
}

// the rejection bound table of the kernels' certain-reject screen (wos_host_scene.h)

extern "C" int hs_rej_table(int dim, float* out) {
  wos::rejection_bound_table(dim, out);
  return wos::kRejTabBins;
}

// ---- group hierarchy (wos_host_scene.cpp build_group_tree) ----
// out_meta: [levels, n[0..kTreeLevels], off[0..kTreeLevels]]
extern "C" int hs_group_tree(const float* groups, int stride, int ngroups, float* nodes, int cap, int* out_meta) {
  std::vector<float> g(groups, groups + (size_t)stride * ngroups);
  wos::HostTree t;
  wos::build_group_tree(g, stride, ngroups, t);
  if ((int)t.node.size() > cap) return -2;
  std::copy(t.node.begin(), t.node.end(), nodes);
  out_meta[0] = t.levels;
  for (int l = 0; l <= wos::kTreeLevels; l++) {
    out_meta[1 + l] = t.n[l];
    out_meta[2 + wos::kTreeLevels + l] = t.off[l];
  }
  return (int)t.node.size();
}

// ---- fcpw's wide BVH over the Neumann boundary (csrc/wos_fcpw_bvh.cpp) ----
extern "C" int hs_fcpw_bvh(int dim, const float* v, int nv, const int* ix, int np, int branch, int leaf, float* box,
                           int* child, int* ref, int cap_nodes, int* n_nodes) {
  (void)nv;
  wos::HostFcpwBvh b;
  wos::build_fcpw_bvh(dim, v, ix, np, branch, leaf, b);
  *n_nodes = b.n_nodes;
  if (b.n_nodes > cap_nodes) return -2;
  std::copy(b.box.begin(), b.box.end(), box);
  std::copy(b.child.begin(), b.child.end(), child);
  std::copy(b.ref.begin(), b.ref.end(), ref);
  return 0;
}
