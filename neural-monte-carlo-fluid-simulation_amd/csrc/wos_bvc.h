// wos_bvc.h -- boundary value caching (the reference's `bvc`, demo.cpp:265-363):
// host-side sample generation and the device record layout shared with wos_bvc.hip.
//
//   BoundarySampler (boundary_value_caching/boundary_sampler.h:87-412): a CDF table
//     over the boundary segments weighted by length, stratified sampling of it, points
//     uniform on the chosen segments -- host C++ (O(cache size) work);
//   DomainSampler (domain_sampler.h:12-66): stratified points over the bounding box,
//     kept inside the solve region (the inside test runs on the GPU);
//   estimates at the boundary samples (walk_on_stars.h:353-464) and the Splatter
//     (splatter.h:43-247) -- wos_bvc.hip.
// The reference's bvc is 2D only (zombie3d exports no bvc).  Its boundary sampler takes
// every segment of the scene and types a segment by onNeumannBoundary at the midpoint
// (demo.cpp:300-313); here the Neumann mesh then the Dirichlet mesh.  Dirichlet samples
// sit normalOffset inside the boundary (the segment's ends displaced along the sampler's
// vertex normals) and carry solution + normal-derivative estimates.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace wos {

// one cached sample as the splat kernel reads it:
//   [x, y, nx, ny, pdf, value, normalDerivative, kind]
// value = the estimated solution (boundary samples) or the source (domain samples);
// kind = 0 Neumann boundary, 1 Neumann normal-aligned (double-sided), 2 domain,
// 3 Dirichlet boundary, 4 Dirichlet normal-aligned
constexpr int kBvcRec = 8;
enum { kBvcBoundary = 0, kBvcAligned = 1, kBvcDomain = 2, kBvcDirichlet = 3, kBvcDirichletAligned = 4 };

struct BvcSampling {
  // boundary samples: the main cache then the normal-aligned one (double-sided)
  std::vector<float> bpt, bnrm;  // [nb][2] point, unit segment normal (not flipped)
  std::vector<uint8_t> aligned;  // [nb]
  std::vector<uint8_t> dirichlet; // [nb] 1: on a Dirichlet segment (displaced inside)
  int nb_main = 0, nb_aligned = 0;
  float pdf_main = 0.0f, pdf_aligned = 0.0f;
  // domain candidates (before the inside test) and their pdf 1/volume
  std::vector<float> dcand;      // [nd][2]
  float pdf_domain = 0.0f;
  float volume = 0.0f;
};

// the Neumann boundary v[nv][2], ix[np][2], the Dirichlet boundary dv[ndv][2], dix[ndp][2],
// the padded bounding box.
bool bvc_generate_samples(const float* v, int nv, const int32_t* ix, int np, const float* dv, int ndv,
                          const int32_t* dix, int ndp, const float pmin[2], const float pmax[2], bool double_sided,
                          int boundary_cache, int domain_cache, float normal_offset, bool ignore_source,
                          uint64_t seed, BvcSampling& out, std::string& err);

// createEvaluationGrid (demo/grid.h:352-368): point (i, j) at index i * res + j over the box
// pmin + [0, ext]
void bvc_evaluation_grid(int res, const float pmin[2], const float ext[2], std::vector<float>& pts);

}  // namespace wos
