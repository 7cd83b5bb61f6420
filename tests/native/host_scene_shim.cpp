// Test-only C shim over the host scene preparation (csrc/wos_host_scene.cpp), built
// with plain g++ by tests/test_host_scene.py so the culling records (group boxes,
// silhouette cones) can be checked on the CPU.  Not part of the product library.
#include <algorithm>
#include <cstring>
#include <string>

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
