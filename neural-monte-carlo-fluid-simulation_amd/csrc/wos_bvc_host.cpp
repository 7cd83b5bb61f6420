// wos_bvc_host.cpp -- boundary value caching, host part: the boundary (Neumann and Dirichlet) and domain
// samplers (boundary_value_caching/boundary_sampler.h, domain_sampler.h) and the
// evaluation grid (demo/grid.h:352-368).  Float arithmetic in the reference's order
// (built with -ffp-contract=off, like the kernels), so the samples equal the CPU
// oracle's bit for bit.
//
// RNG: the reference seeds each sampler from std::chrono::system_clock
// (boundary_sampler.h:102-103, domain_sampler.h:26-27); here the counter-based
// streams seed32(key, 0, 0, 4) (boundary) and seed32(key, 0, 0, 5) (domain).  The
// reference visits the sampled segments in std::unordered_map order
// (boundary_sampler.h:335-389); here in ascending segment order -- the same
// distribution, deterministic.
#include "wos_bvc.h"

#include <cmath>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "wos_detmath.h"

namespace wos {
namespace {

// generateStratifiedSamples<DIM> (sampling.h:435-457)
void stratified(std::vector<float>& s, int n, int dims, Pcg32& g) {
  const float ome = 1.0f - kFltEps;
  const float inv = 1.0f / (float)n;
  s.assign((size_t)n * dims, 0.0f);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < dims; ++j) {
      const float sj = ((float)i + g.nextf()) * inv;
      s[(size_t)dims * i + j] = smin(sj, ome);
    }
  for (int i = 0; i < dims; ++i)
    for (int j = 0; j < n; ++j) {
      const int other = j + (int)g.bounded((uint32_t)(n - j));
      const float t = s[(size_t)dims * j + i];
      s[(size_t)dims * j + i] = s[(size_t)dims * other + i];
      s[(size_t)dims * other + i] = t;
    }
}

// CDFTable::build / sample (sampling.h:261-314)
struct Cdf {
  std::vector<float> table;
  float build(const std::vector<float>& w) {
    const int n = (int)w.size();
    if (n == 0) return 0.0f;
    table.assign(n + 1, 0.0f);
    for (int i = 1; i < n + 1; i++) table[i] = table[i - 1] + w[i - 1];
    const float total = table[n];
    if (total == 0.0f) {
      for (int i = 1; i < n + 1; i++) table[i] = (float)i / (float)n;
    } else {
      for (int i = 1; i < n + 1; i++) table[i] /= total;
    }
    return total;
  }
  int sample(float u) const {
    const int size = (int)table.size();
    int first = 0, len = size;
    while (len > 0) {
      const int half = len >> 1, middle = first + half;
      if (table[middle] <= u) {
        first = middle + 1;
        len -= half + 1;
      } else {
        len = half;
      }
    }
    return sclamp(first - 1, 0, size - 2);
  }
};

struct Seg {
  float pa[2], pb[2];
};

// The sampler's boundary (boundary_sampler.h:87-412): the Neumann segments, then the Dirichlet
// ones, whose vertices carry the sampler's own normals (computeNormals :193-236: unit segment
// normals summed per vertex, normalised).  The reference runs it over the scene's ONE mesh
// (demo.cpp:316 passes scene.vertices / scene.segments), so a vertex shared by a Neumann and a
// Dirichlet segment sums both segments' normals; here the two parts arrive as separate meshes,
// and a Dirichlet vertex is welded to every Neumann segment end at the same position.
struct Boundary {
  const float *v, *dv;
  const int32_t *ix, *dix;
  int np = 0, ndp = 0;
  std::vector<float> dn;  // [ndv][2]
  int size() const { return np + ndp; }
  bool dirichlet(int i) const { return i >= np; }
  Seg raw(int i) const {
    Seg s;
    const float* V = i < np ? v : dv;
    const int32_t* I = i < np ? ix : dix;
    const int p = i < np ? i : i - np;
    for (int k = 0; k < 2; k++) {
      s.pa[k] = V[2 * I[2 * p] + k];
      s.pb[k] = V[2 * I[2 * p + 1] + k];
    }
    return s;
  }
  // Dirichlet ends displaced along the vertex normals (`pa += normalOffset*normals[index[0]]`)
  Seg ends(int i, float offset) const {
    Seg s = raw(i);
    if (dirichlet(i)) {
      const int p = i - np;
      for (int k = 0; k < 2; k++) {
        s.pa[k] += offset * dn[2 * dix[2 * p] + k];
        s.pb[k] += offset * dn[2 * dix[2 * p + 1] + k];
      }
    }
    return s;
  }
};

// unit normal of segment (pa, pb) (lineSegmentNormal<2>(pa, pb, true): Eigen normalized())
void unit_normal(const Seg& g, float* n) {
  const float s0 = g.pb[0] - g.pa[0], s1 = g.pb[1] - g.pa[1];
  n[0] = s1;
  n[1] = -s0;
  const float z = n[0] * n[0] + n[1] * n[1];
  if (z > 0.0f) { const float r = std::sqrt(z); n[0] = n[0] / r; n[1] = n[1] / r; }
}

// position key of a vertex (+0 and -0 compare equal, as the float comparison does)
uint64_t pos_key(const float* p) {
  uint32_t a, b;
  const float x = p[0] + 0.0f, y = p[1] + 0.0f;
  std::memcpy(&a, &x, 4);
  std::memcpy(&b, &y, 4);
  return ((uint64_t)a << 32) | b;
}

void dirichlet_normals(Boundary& B, int ndv) {
  B.dn.assign((size_t)2 * ndv, 0.0f);
  // Dirichlet segments first, then the Neumann segment ends welded onto Dirichlet vertices: a
  // junction vertex has one segment of each kind, and a sum of two terms does not depend on
  // their order, so this equals the reference's one-mesh order (a vertex where three or more
  // segments meet could differ in the last bit)
  for (int p = 0; p < B.ndp; p++) {
    float n[2];
    unit_normal(B.raw(B.np + p), n);
    for (int q = 0; q < 2; q++)
      for (int k = 0; k < 2; k++) B.dn[2 * B.dix[2 * p + q] + k] += n[k];
  }
  if (B.np > 0 && B.ndp > 0) {
    std::unordered_map<uint64_t, std::vector<int>> at;
    for (int i = 0; i < ndv; i++) at[pos_key(B.dv + 2 * i)].push_back(i);
    for (int p = 0; p < B.np; p++) {
      const Seg g = B.raw(p);
      float n[2];
      unit_normal(g, n);
      for (const float* e : {g.pa, g.pb}) {
        const auto it = at.find(pos_key(e));
        if (it == at.end()) continue;
        for (const int i : it->second)
          for (int k = 0; k < 2; k++) B.dn[2 * i + k] += n[k];
      }
    }
  }
  for (int i = 0; i < ndv; i++) {
    const float z = B.dn[2 * i] * B.dn[2 * i] + B.dn[2 * i + 1] * B.dn[2 * i + 1];
    if (z > 0.0f) { const float r = std::sqrt(z); B.dn[2 * i] /= r; B.dn[2 * i + 1] /= r; }
  }
}

// buildCDFTable (boundary_sampler.h:291-331): weight = the (displaced) segment's length when
// pMid + normalOffset * n lies in the bounding box (the solve region of the boundary sampler,
// demo.cpp:299-301: !outsideBoundingDomain)
float build_table(const Boundary& B, const float* pmin, const float* pmax, float normal_offset, Cdf& cdf) {
  std::vector<float> w(B.size(), 0.0f);
  for (int i = 0; i < B.size(); i++) {
    const Seg g = B.raw(i);
    const float pMid[2] = {(g.pa[0] + g.pb[0]) / 2.0f, (g.pa[1] + g.pb[1]) / 2.0f};
    const float s0 = g.pb[0] - g.pa[0], s1 = g.pb[1] - g.pa[1];
    float n[2] = {s1, -s0};  // lineSegmentNormal(pa, pb, true): Eigen normalized()
    const float z = n[0] * n[0] + n[1] * n[1];
    if (z > 0.0f) { const float r = std::sqrt(z); n[0] = n[0] / r; n[1] = n[1] / r; }
    const float q[2] = {pMid[0] + normal_offset * n[0], pMid[1] + normal_offset * n[1]};
    const bool inside = q[0] >= pmin[0] && q[1] >= pmin[1] && q[0] <= pmax[0] && q[1] <= pmax[1];
    if (inside) {
      const Seg e = B.ends(i, normal_offset);
      const float t0 = e.pb[0] - e.pa[0], t1 = e.pb[1] - e.pa[1];
      w[i] = std::sqrt(t1 * t1 + (-t0) * (-t0));  // lineSegmentSurfaceArea
    }
  }
  return cdf.build(w);
}

// generateSamples (boundary_sampler.h:333-402): n stratified draws into the table,
// then per sampled segment one uniform draw (one sample) or a stratified set
void gen_boundary(const Boundary& B, const Cdf& cdf, int n, float total, float normal_offset, bool aligned, Pcg32& g,
                  BvcSampling& out) {
  if (!(total > 0.0f) || n <= 0) return;
  std::vector<float> strat;
  stratified(strat, n, 1, g);
  std::vector<int> count(cdf.table.size() - 1, 0);
  for (int i = 0; i < n; i++) count[cdf.sample(strat[i])]++;
  std::vector<float> u;
  for (int f = 0; f < (int)count.size(); f++) {
    const int c = count[f];
    if (c == 0) continue;
    if (c == 1) u.assign(1, g.nextf());
    else stratified(u, c, 1, g);
    const Seg sg = B.ends(f, normal_offset);
    const float s0 = sg.pb[0] - sg.pa[0], s1 = sg.pb[1] - sg.pa[1];
    for (int i = 0; i < c; i++) {
      // sampleLineSegmentUniformly<2> (sampling.h:213-224)
      const float pt[2] = {sg.pa[0] + u[i] * s0, sg.pa[1] + u[i] * s1};
      float nn[2] = {s1, -s0};
      const float norm = std::sqrt(nn[0] * nn[0] + nn[1] * nn[1]);
      nn[0] = nn[0] / norm;
      nn[1] = nn[1] / norm;
      out.bpt.push_back(pt[0]);
      out.bpt.push_back(pt[1]);
      out.bnrm.push_back(nn[0]);
      out.bnrm.push_back(nn[1]);
      out.aligned.push_back(aligned ? 1 : 0);
      out.dirichlet.push_back(B.dirichlet(f) ? 1 : 0);
    }
  }
}

}  // namespace

bool bvc_generate_samples(const float* v, int nv, const int32_t* ix, int np, const float* dv, int ndv,
                          const int32_t* dix, int ndp, const float pmin[2], const float pmax[2], bool double_sided,
                          int boundary_cache, int domain_cache, float normal_offset, bool ignore_source,
                          uint64_t seed, BvcSampling& out, std::string& err) {
  out = BvcSampling{};
  for (int i = 0; i < 2 * np; i++)
    if (ix[i] < 0 || ix[i] >= nv) { err = "bvc: segment index out of range"; return false; }
  for (int i = 0; i < 2 * ndp; i++)
    if (dix[i] < 0 || dix[i] >= ndv) { err = "bvc: Dirichlet segment index out of range"; return false; }
  Boundary B;
  B.v = v; B.ix = ix; B.np = np;
  B.dv = dv; B.dix = dix; B.ndp = ndp;
  dirichlet_normals(B, ndv);
  // ---- boundary samples (BoundarySampler::initialize + generateSamples)
  Pcg32 bs;
  bs.seed(seed32(seed, 0, 0, 4));
  Cdf t_main, t_aligned;
  const float a_main = build_table(B, pmin, pmax, -1.0f * normal_offset, t_main);
  if (double_sided) {
    const float a_al = build_table(B, pmin, pmax, normal_offset, t_aligned);
    const float total = a_main + a_al;
    const int n_main = (int)std::ceil((float)boundary_cache * a_main / total);
    const int n_al = (int)std::ceil((float)boundary_cache * a_al / total);
    out.pdf_main = 1.0f / a_main;
    out.pdf_aligned = 1.0f / a_al;
    gen_boundary(B, t_main, n_main, a_main, -1.0f * normal_offset, false, bs, out);
    out.nb_main = (int)out.aligned.size();
    gen_boundary(B, t_aligned, n_al, a_al, normal_offset, true, bs, out);
    out.nb_aligned = (int)out.aligned.size() - out.nb_main;
  } else {
    out.pdf_main = 1.0f / a_main;
    gen_boundary(B, t_main, boundary_cache, a_main, -1.0f * normal_offset, false, bs, out);
    out.nb_main = (int)out.aligned.size();
  }
  // ---- domain candidates (DomainSampler::generateSamples), inside test on the GPU
  const float ext[2] = {pmax[0] - pmin[0], pmax[1] - pmin[1]};
  float vol;
  if (double_sided) {
    vol = ext[0] * ext[1];
  } else {  // getSolveRegionVolume (scene.h:92-100): |Dirichlet part's + Neumann part's signedVolume|
    float sv = 0.0f;  // LineSegment::signedVolume, line_segments.inl:38-44
    for (int part = 0; part < 2; part++) {
      float sq = 0.0f;
      const int n0 = part == 0 ? np : 0, n1 = part == 0 ? np + ndp : np;  // the Dirichlet part first
      for (int i = n0; i < n1; i++) {
        const Seg g = B.raw(i);
        sq += 0.5f * (g.pa[0] * g.pb[1] - g.pa[1] * g.pb[0]);
      }
      sv += sq;
    }
    vol = std::fabs(sv);
  }
  out.volume = vol;
  out.pdf_domain = 1.0f / vol;
  if (!ignore_source && domain_cache > 0) {
    Pcg32 ds;
    ds.seed(seed32(seed, 0, 0, 5));
    int nstrat = domain_cache;
    if (vol > 0.0f) nstrat = (int)((float)nstrat * (ext[0] * ext[1] * out.pdf_domain));
    if (nstrat > 0) {
      std::vector<float> strat;
      stratified(strat, nstrat, 2, ds);
      out.dcand.resize((size_t)2 * nstrat);
      for (int i = 0; i < nstrat; i++)
        for (int j = 0; j < 2; j++) out.dcand[(size_t)2 * i + j] = pmin[j] + ext[j] * strat[(size_t)2 * i + j];
    }
  }
  return true;
}

void bvc_evaluation_grid(int res, const float pmin[2], const float ext[2], std::vector<float>& pts) {
  pts.resize((size_t)2 * res * res);
  for (int i = 0; i < res; i++)
    for (int j = 0; j < res; j++) {
      const size_t q = (size_t)i * res + j;
      pts[2 * q] = ((float)i / (float)res) * ext[0] + pmin[0];
      pts[2 * q + 1] = ((float)j / (float)res) * ext[1] + pmin[1];
    }
}

}  // namespace wos
