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

struct HostScene {
  int dim = 2;
  int n_prims = 0, n_sil = 0, n_dprims = 0;
  std::vector<float> prim, paux, sil, dprim, dpaux;
  std::vector<float> pgroup, sgroup;  // culling boxes (kGroupStride floats each)
  int n_pgroups = 0, n_sgroups = 0;
  float pmin[3] = {0, 0, 0}, pmax[3] = {0, 0, 0}, ext[3] = {0, 0, 0};
};

bool prepare_scene(const HostSceneInput& in, HostScene& out, std::string& err);
bool load_obj(const std::string& path, int dim, bool flip, bool normalize_domain, std::vector<float>& verts,
              std::vector<int32_t>& prims, std::string& err);

}  // namespace wos
