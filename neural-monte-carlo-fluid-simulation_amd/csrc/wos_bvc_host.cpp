// wos_bvc_host.cpp -- boundary value caching, host part: the boundary and domain
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

Seg segment(const float* v, const int32_t* ix, int p) {
  Seg s;
  for (int k = 0; k < 2; k++) {
    s.pa[k] = v[2 * ix[2 * p] + k];
    s.pb[k] = v[2 * ix[2 * p + 1] + k];
  }
  return s;
}

// buildCDFTable (boundary_sampler.h:291-331) on an all-Neumann boundary: weight =
// segment length when pMid + normalOffset * n lies in the bounding box (the solve
// region of the boundary sampler, demo.cpp:299-301: !outsideBoundingDomain)
float build_table(const float* v, const int32_t* ix, int np, const float* pmin, const float* pmax,
                  float normal_offset, Cdf& cdf) {
  std::vector<float> w(np, 0.0f);
  for (int i = 0; i < np; i++) {
    const Seg g = segment(v, ix, i);
    const float pMid[2] = {(g.pa[0] + g.pb[0]) / 2.0f, (g.pa[1] + g.pb[1]) / 2.0f};
    const float s0 = g.pb[0] - g.pa[0], s1 = g.pb[1] - g.pa[1];
    float n[2] = {s1, -s0};  // lineSegmentNormal(pa, pb, true): Eigen normalized()
    const float z = n[0] * n[0] + n[1] * n[1];
    if (z > 0.0f) { const float r = std::sqrt(z); n[0] = n[0] / r; n[1] = n[1] / r; }
    const float q[2] = {pMid[0] + normal_offset * n[0], pMid[1] + normal_offset * n[1]};
    const bool inside = q[0] >= pmin[0] && q[1] >= pmin[1] && q[0] <= pmax[0] && q[1] <= pmax[1];
    if (inside) w[i] = std::sqrt(s1 * s1 + (-s0) * (-s0));  // lineSegmentSurfaceArea
  }
  return cdf.build(w);
}

// generateSamples (boundary_sampler.h:333-402): n stratified draws into the table,
// then per sampled segment one uniform draw (one sample) or a stratified set
void gen_boundary(const float* v, const int32_t* ix, const Cdf& cdf, int n, float total, bool aligned, Pcg32& g,
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
    const Seg sg = segment(v, ix, f);
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
    }
  }
}

}  // namespace

bool bvc_generate_samples(const float* v, int nv, const int32_t* ix, int np, const float pmin[2],
                          const float pmax[2], bool double_sided, int boundary_cache, int domain_cache,
                          float normal_offset, bool ignore_source, uint64_t seed, BvcSampling& out,
                          std::string& err) {
  out = BvcSampling{};
  for (int i = 0; i < 2 * np; i++)
    if (ix[i] < 0 || ix[i] >= nv) { err = "bvc: segment index out of range"; return false; }
  // ---- boundary samples (BoundarySampler::initialize + generateSamples)
  Pcg32 bs;
  bs.seed(seed32(seed, 0, 0, 4));
  Cdf t_main, t_aligned;
  const float a_main = build_table(v, ix, np, pmin, pmax, -1.0f * normal_offset, t_main);
  if (double_sided) {
    const float a_al = build_table(v, ix, np, pmin, pmax, normal_offset, t_aligned);
    const float total = a_main + a_al;
    const int n_main = (int)std::ceil((float)boundary_cache * a_main / total);
    const int n_al = (int)std::ceil((float)boundary_cache * a_al / total);
    out.pdf_main = 1.0f / a_main;
    out.pdf_aligned = 1.0f / a_al;
    gen_boundary(v, ix, t_main, n_main, a_main, false, bs, out);
    out.nb_main = (int)out.aligned.size();
    gen_boundary(v, ix, t_aligned, n_al, a_al, true, bs, out);
    out.nb_aligned = (int)out.aligned.size() - out.nb_main;
  } else {
    out.pdf_main = 1.0f / a_main;
    gen_boundary(v, ix, t_main, boundary_cache, a_main, false, bs, out);
    out.nb_main = (int)out.aligned.size();
  }
  // ---- domain candidates (DomainSampler::generateSamples), inside test on the GPU
  const float ext[2] = {pmax[0] - pmin[0], pmax[1] - pmin[1]};
  float vol;
  if (double_sided) {
    vol = ext[0] * ext[1];
  } else {  // |signedVolume| of the boundary (LineSegment::signedVolume, line_segments.inl:38-44)
    float sv = 0.0f;
    for (int p = 0; p < np; p++) {
      const Seg g = segment(v, ix, p);
      sv += 0.5f * (g.pa[0] * g.pb[1] - g.pa[1] * g.pb[0]);
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

void bvc_evaluation_grid(int res, const float pmin[2], const float pmax[2], std::vector<float>& pts) {
  const float ext[2] = {pmax[0] - pmin[0], pmax[1] - pmin[1]};
  pts.resize((size_t)2 * res * res);
  for (int i = 0; i < res; i++)
    for (int j = 0; j < res; j++) {
      const size_t q = (size_t)i * res + j;
      pts[2 * q] = ((float)i / (float)res) * ext[0] + pmin[0];
      pts[2 * q + 1] = ((float)j / (float)res) * ext[1] + pmin[1];
    }
}

}  // namespace wos
