// wos_capi.hip -- the extern "C" boundary declared in include/wos.h.
//
// Owns device memory for the scene (geometry records + source grid) and a
// grow-only per-scene workspace (staging buffers for host pointers, counters,
// work queue).  Errors are reported as status codes + wos_last_error(), never by
// aborting the process (the reference aborts: config.h:8-11, scene.h:106-109).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/wos.h"
#include "wos_detmath.h"
#include "wos_host_scene.h"
#include "wos_launch.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                         \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) return fail(WOS_E_DEVICE, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

template <typename T>
hipError_t upload(T** dst, const std::vector<T>& src) {
  *dst = nullptr;
  if (src.empty()) return hipSuccess;
  hipError_t e = hipMalloc((void**)dst, src.size() * sizeof(T));
  if (e != hipSuccess) return e;
  return hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice);
}

}  // namespace

struct wos_scene {
  int device = 0;
  wos::HostScene host;
  wos::DevScene dev{};
  float *d_prim = nullptr, *d_paux = nullptr, *d_sil = nullptr, *d_dprim = nullptr, *d_dpaux = nullptr;
  float* d_source = nullptr;
  float *d_pgroup = nullptr, *d_sgroup = nullptr;
  // workspace
  std::mutex mu;
  float* d_pts = nullptr;
  float* d_p = nullptr;
  float* d_g = nullptr;
  int32_t* d_nest = nullptr;
  int32_t* d_steps = nullptr;
  size_t ws_points = 0;
  uint64_t* d_jump = nullptr;  // PCG32 jump-ahead table (A_k, C_k), grow-only
  int n_jump = 0;
  float* d_tasks = nullptr;      // walk-task workspace (DevTasks arrays), grow-only
  int64_t task_cap = 0;          // tasks
  int32_t* d_pstate = nullptr;   // per-point state + queue permutation of one batch, then bucket counters
  int64_t pstate_cap = 0;
  unsigned long long* d_counters = nullptr;  // kNumCounters u64 + work counter
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::vector<hipEvent_t> bev;  // per-batch kernel boundary events (4 per batch), grow-only
  int num_cus = 0;
  // star-radius cell grid, built on first use for the solver's (precision, minR)
  wos::StarGrid sgrid;
  bool sgrid_built = false, sgrid_ok = false;
  uint32_t* d_sgrid = nullptr;
};

extern "C" {

const char* wos_last_error(void) { return g_err.c_str(); }
int32_t wos_abi_version(void) { return WOS_ABI_VERSION; }

int32_t wos_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int wos_load_obj(const char* path, int32_t dim, int32_t flip_orientation, int32_t normalize, wos_mesh* out) {
  if (!path || !out) return fail(WOS_E_INVALID, "wos_load_obj: null argument");
  if (dim != 2 && dim != 3) return fail(WOS_E_INVALID, "wos_load_obj: dim must be 2 or 3");
  std::vector<float> v;
  std::vector<int32_t> ix;
  std::string err;
  if (!wos::load_obj(path, dim, flip_orientation != 0, normalize != 0, v, ix, err))
    return fail(err.rfind("Error opening", 0) == 0 ? WOS_E_IO : WOS_E_INVALID, err);
  out->dim = dim;
  out->n_vertices = (int32_t)(v.size() / dim);
  out->n_prims = (int32_t)(ix.size() / dim);
  out->vertices = (float*)std::malloc(std::max<size_t>(1, v.size()) * sizeof(float));
  out->prims = (int32_t*)std::malloc(std::max<size_t>(1, ix.size()) * sizeof(int32_t));
  if (!out->vertices || !out->prims) return fail(WOS_E_NOMEM, "wos_load_obj: out of memory");
  if (!v.empty()) std::memcpy(out->vertices, v.data(), v.size() * sizeof(float));
  if (!ix.empty()) std::memcpy(out->prims, ix.data(), ix.size() * sizeof(int32_t));
  return WOS_OK;
}

void wos_mesh_free(wos_mesh* mesh) {
  if (!mesh) return;
  std::free(mesh->vertices);
  std::free(mesh->prims);
  mesh->vertices = nullptr;
  mesh->prims = nullptr;
  mesh->n_vertices = mesh->n_prims = 0;
}

void wos_default_params(wos_solver_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  // defaults of runWalkOnStars_sampled (demo.cpp:121-137) and grid.h:159
  p->n_walks = 128;
  p->max_walk_length = 1024;
  p->steps_before_tikhonov = 1024;
  p->steps_before_maximal_spheres = 1024;
  p->epsilon_shell = 1e-3f;
  p->min_star_radius = 1e-3f;
  p->silhouette_precision = 1e-3f;
  p->russian_roulette_threshold = 0.0f;
  p->boundary_distance_mask = 0.0f;
  p->seed = 0x5EED0001ULL;
}

static void scene_release(wos_scene* s) {
  if (!s) return;
  hipSetDevice(s->device);
  hipFree(s->d_prim); hipFree(s->d_paux); hipFree(s->d_sil); hipFree(s->d_dprim); hipFree(s->d_dpaux);
  hipFree(s->d_source);
  hipFree(s->d_pgroup); hipFree(s->d_sgroup);
  hipFree(s->d_pts); hipFree(s->d_p); hipFree(s->d_g); hipFree(s->d_nest); hipFree(s->d_steps);
  hipFree(s->d_counters);
  hipFree(s->d_jump);
  hipFree(s->d_tasks);
  hipFree(s->d_pstate);
  hipFree(s->d_sgrid);
  if (s->ev0) hipEventDestroy(s->ev0);
  if (s->ev1) hipEventDestroy(s->ev1);
  for (hipEvent_t e : s->bev) hipEventDestroy(e);
}

int wos_scene_create(const wos_scene_desc* d, int32_t device, wos_scene** out) {
  if (!d || !out) return fail(WOS_E_INVALID, "wos_scene_create: null argument");
  *out = nullptr;
  if (d->dim != 2 && d->dim != 3) return fail(WOS_E_INVALID, "wos_scene_create: dim must be 2 or 3");
  const int nsd = d->dim == 2 ? 2 : 3;
  for (int k = 0; k < nsd; k++)
    if (d->source && d->source_dims[k] <= 0) return fail(WOS_E_INVALID, "wos_scene_create: bad source dims");
  if (!(d->absorption >= 0.0f)) return fail(WOS_E_INVALID, "wos_scene_create: absorption must be >= 0");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(WOS_E_DEVICE, "wos_scene_create: no HIP device available");
  if (device < 0 || device >= ndev) return fail(WOS_E_INVALID, "wos_scene_create: device index out of range");

  wos::HostSceneInput in;
  in.dim = d->dim;
  in.vertices = d->vertices; in.prims = d->prims; in.n_vertices = d->n_vertices; in.n_prims = d->n_prims;
  in.dvertices = d->dvertices; in.dprims = d->dprims; in.n_dvertices = d->n_dvertices; in.n_dprims = d->n_dprims;
  in.is_double_sided = d->is_double_sided;
  auto* s = new wos_scene();
  std::string err;
  if (!wos::prepare_scene(in, s->host, err)) { delete s; return fail(WOS_E_INVALID, "wos_scene_create: " + err); }
  s->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = upload(&s->d_prim, s->host.prim);
  if (e == hipSuccess) e = upload(&s->d_paux, s->host.paux);
  if (e == hipSuccess) e = upload(&s->d_sil, s->host.sil);
  if (e == hipSuccess) e = upload(&s->d_dprim, s->host.dprim);
  if (e == hipSuccess) e = upload(&s->d_dpaux, s->host.dpaux);
  if (e == hipSuccess) e = upload(&s->d_pgroup, s->host.pgroup);
  if (e == hipSuccess) e = upload(&s->d_sgroup, s->host.sgroup);
  size_t nsrc = 0;
  if (d->source) {
    nsrc = (size_t)d->source_dims[0] * d->source_dims[1] * (d->dim == 3 ? d->source_dims[2] : 1);
    if (e == hipSuccess) e = hipMalloc((void**)&s->d_source, nsrc * sizeof(float));
    if (e == hipSuccess)
      e = hipMemcpy(s->d_source, d->source, nsrc * sizeof(float),
                    d->source_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMalloc((void**)&s->d_counters, wos::kNumCounterSlots * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipEventCreate(&s->ev0);
  if (e == hipSuccess) e = hipEventCreate(&s->ev1);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&s->num_cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess) {
    std::string msg = std::string("wos_scene_create: ") + hipGetErrorString(e);
    scene_release(s);
    delete s;
    return fail(WOS_E_DEVICE, msg);
  }
  wos::DevScene& ds = s->dev;
  ds.dim = d->dim;
  ds.n_prims = s->host.n_prims;
  ds.n_sil = s->host.n_sil;
  ds.n_dprims = s->host.n_dprims;
  ds.prim = s->d_prim; ds.paux = s->d_paux; ds.sil = s->d_sil; ds.dprim = s->d_dprim; ds.dpaux = s->d_dpaux;
  ds.source = s->d_source;
  ds.pgroup = s->d_pgroup; ds.sgroup = s->d_sgroup;
  ds.n_pgroups = s->host.n_pgroups; ds.n_sgroups = s->host.n_sgroups;
  for (int k = 0; k < 3; k++) {
    ds.sdims[k] = d->source ? (k < nsd ? d->source_dims[k] : 1) : 0;
    ds.pmin[k] = s->host.pmin[k]; ds.pmax[k] = s->host.pmax[k]; ds.ext[k] = s->host.ext[k];
  }
  ds.absorption = d->absorption;
  ds.g_dirichlet = d->dirichlet_value;
  ds.watertight = d->is_watertight;
  ds.double_sided = d->is_double_sided;
  *out = s;
  return WOS_OK;
}

int wos_scene_destroy(wos_scene* s) {
  if (!s) return WOS_OK;
  scene_release(s);
  delete s;
  return WOS_OK;
}

int wos_scene_get_info(const wos_scene* s, wos_scene_info* info) {
  if (!s || !info) return fail(WOS_E_INVALID, "wos_scene_get_info: null argument");
  info->dim = s->host.dim;
  info->n_prims = s->host.n_prims;
  info->n_silhouettes = s->host.n_sil;
  info->n_dprims = s->host.n_dprims;
  info->device = s->device;
  for (int k = 0; k < 3; k++) { info->bbox_min[k] = s->host.pmin[k]; info->bbox_max[k] = s->host.pmax[k]; }
  return WOS_OK;
}

static int ensure_workspace(wos_scene* s, size_t npts) {
  if (npts <= s->ws_points) return WOS_OK;
  const int dim = s->host.dim;
  hipFree(s->d_pts); hipFree(s->d_p); hipFree(s->d_g); hipFree(s->d_nest); hipFree(s->d_steps);
  s->d_pts = s->d_p = s->d_g = nullptr; s->d_nest = s->d_steps = nullptr; s->ws_points = 0;
  size_t cap = npts + npts / 4 + 1024;
  HIP_TRY(hipMalloc((void**)&s->d_pts, cap * dim * sizeof(float)));
  HIP_TRY(hipMalloc((void**)&s->d_p, cap * sizeof(float)));
  HIP_TRY(hipMalloc((void**)&s->d_g, cap * dim * sizeof(float)));
  HIP_TRY(hipMalloc((void**)&s->d_nest, cap * sizeof(int32_t)));
  HIP_TRY(hipMalloc((void**)&s->d_steps, cap * sizeof(int32_t)));
  s->ws_points = cap;
  return WOS_OK;
}

// walk tasks per batch: 2^24 tasks = 0.8 GB (2D) / 1.0 GB (3D) of workspace
static constexpr int64_t kMaxBatchTasks = (int64_t)1 << 24;

static int ensure_tasks(wos_scene* s, int64_t tasks, int64_t points) {
  const int tf = wos::task_floats(s->host.dim);
  if (tasks > s->task_cap) {
    hipFree(s->d_tasks);
    s->d_tasks = nullptr; s->task_cap = 0;
    HIP_TRY(hipMalloc((void**)&s->d_tasks, (size_t)tasks * tf * sizeof(float)));
    s->task_cap = tasks;
  }
  if (points > s->pstate_cap) {
    hipFree(s->d_pstate);
    s->d_pstate = nullptr; s->pstate_cap = 0;
    HIP_TRY(hipMalloc((void**)&s->d_pstate, ((size_t)2 * points + 2 * wos::kCostBuckets) * sizeof(int32_t)));
    s->pstate_cap = points;
  }
  return WOS_OK;
}

// SoA views into the task workspace for a batch of T tasks
static wos::DevTasks task_view(wos_scene* s, int dim, int64_t T, int32_t wpp) {
  wos::DevTasks tk{};
  float* f = s->d_tasks;
  tk.pt = f; f += dim * T;
  tk.thr = f; f += T;
  tk.tsrc = f; f += T;
  tk.dd = f; f += T;
  tk.first = f; f += T;
  tk.bdir = f; f += dim * T;
  tk.sdir = f; f += dim * T;
  tk.total = f; f += T;
  tk.code = (uint32_t*)f;
  tk.pstate = s->d_pstate;
  tk.perm = (uint32_t*)(s->d_pstate + s->pstate_cap);
  tk.hist = (uint32_t*)(s->d_pstate + 2 * s->pstate_cap);
  tk.T = T;
  tk.wpp = wpp;
  return tk;
}

// state_k = A_k * state_0 + C_k for the PCG32 LCG (multiplier kPcgMult, increment kPcgInc)
static int ensure_jump(wos_scene* s, int k_needed) {
  if (k_needed <= s->n_jump) return WOS_OK;
  // >= 2 * 1000 + 2: the wave-cooperative rejection sampler jumps up to 1000 iterations ahead
  const int cap = std::max(k_needed, 4096);
  std::vector<uint64_t> t(2 * (size_t)cap);
  uint64_t A = 1u, Cc = 0u;
  for (int k = 0; k < cap; k++) {
    t[2 * k] = A; t[2 * k + 1] = Cc;
    A = A * wos::kPcgMult;
    Cc = Cc * wos::kPcgMult + wos::kPcgInc;
  }
  hipFree(s->d_jump);
  s->d_jump = nullptr; s->n_jump = 0;
  HIP_TRY(hipMalloc((void**)&s->d_jump, t.size() * sizeof(uint64_t)));
  HIP_TRY(hipMemcpy(s->d_jump, t.data(), t.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
  s->n_jump = cap;
  return WOS_OK;
}

// dynamic LDS a workgroup may use: 160 KB per CU minus the kernels' static LDS
// (rejection jump table 2 KB, counters, histogram)
static constexpr size_t kLdsDynamicMax = 160 * 1024 - 4096;

// LDS budget of the star-radius grid (staged by every walk-kernel workgroup)
static constexpr size_t kStarGridBudget = 16 * 1024;

static bool star_grid_enabled() {
  const char* e = std::getenv("WOS_STAR_GRID");  // "0": always the cooperative group scan (A/B runs, tests)
  return !(e && e[0] == '0');
}

// (re)build the star grid for the solver's silhouette precision and minR
static int ensure_star_grid(wos_scene* s, float prec, float min_r) {
  if (s->sgrid_built && s->sgrid.prec == prec && s->sgrid.min_r == min_r) return WOS_OK;
  hipFree(s->d_sgrid);
  s->d_sgrid = nullptr;
  s->sgrid_ok = wos::build_star_grid(s->host, prec, min_r, kStarGridBudget, s->sgrid);
  s->sgrid_built = true;
  if (s->sgrid_ok) {
    HIP_TRY(hipMalloc((void**)&s->d_sgrid, s->sgrid.words.size() * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(s->d_sgrid, s->sgrid.words.data(), s->sgrid.words.size() * sizeof(uint32_t),
                      hipMemcpyHostToDevice));
  }
  return WOS_OK;
}

int wos_solve(wos_scene* s, const wos_solver_params* prm, const float* pts, int64_t n, int64_t index_base,
              int64_t index_stride, float* p, float* grad, int32_t* n_est, int32_t* steps, wos_stats* stats,
              void* stream, uint32_t flags) {
  if (!s || !prm) return fail(WOS_E_INVALID, "wos_solve: null scene/params");
  if (n < 0) return fail(WOS_E_INVALID, "wos_solve: negative point count");
  if (n > 0 && (!pts || !p || !grad)) return fail(WOS_E_INVALID, "wos_solve: null point/output buffer");
  if (n >= (int64_t)0xFFFFFFF0LL) return fail(WOS_E_INVALID, "wos_solve: too many points for one call");
  if (prm->n_walks < 1) return fail(WOS_E_INVALID, "wos_solve: nWalks must be >= 1");
  if (prm->max_walk_length < 0) return fail(WOS_E_INVALID, "wos_solve: maxWalkLength must be >= 0");
  if (!(prm->epsilon_shell >= 0.0f) || !(prm->min_star_radius >= 0.0f) || !(prm->silhouette_precision >= 0.0f))
    return fail(WOS_E_INVALID, "wos_solve: negative tolerance");
  std::lock_guard<std::mutex> lock(s->mu);
  const int dim = s->host.dim;
  HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = (hipStream_t)stream;

  wos::DevParams dp{};
  const bool anti = !prm->disable_gradient_antithetic_variates;
  dp.n_walks = prm->n_walks;
  dp.n_anti = anti ? 2 : 1;
  dp.n_pairs = anti ? std::max(1, prm->n_walks / 2) : prm->n_walks;
  dp.max_walk_length = prm->max_walk_length;
  dp.steps_before_tikhonov = prm->steps_before_tikhonov;
  dp.steps_before_maximal_spheres = prm->steps_before_maximal_spheres;
  dp.epsilon_shell = prm->epsilon_shell;
  dp.min_star_radius = prm->min_star_radius;
  dp.silhouette_precision = prm->silhouette_precision;
  dp.rr_threshold = prm->russian_roulette_threshold;
  dp.boundary_distance_mask = prm->boundary_distance_mask;
  dp.use_cv = !prm->disable_gradient_control_variates;
  dp.use_cosine = prm->use_cosine_sampling;
  dp.ignore_dirichlet = prm->ignore_dirichlet;
  dp.ignore_neumann = prm->ignore_neumann;
  dp.ignore_source = prm->ignore_source;
  dp.seed = prm->seed;
  {
    // diagonal draws + shuffle draws of the stratified samples
    const int k_needed = 2 * (2 * dp.n_pairs) * (dim - 1);
    int rc = ensure_jump(s, k_needed);
    if (rc != WOS_OK) return rc;
    dp.jump = s->d_jump;
    dp.n_jump = s->n_jump;
  }

  // LDS: staged geometry (+ per wave: stratified samples and their shuffle partners
  // in the first-ball kernel)
  const int PS = dim == 2 ? wos::kPrimStride2 : wos::kPrimStride3;
  const int SS = dim == 2 ? wos::kSilStride2 : wos::kSilStride3;
  const int primAl = (s->host.n_prims * PS + 3) & ~3;
  const int silAl = (s->host.n_sil * SS + 3) & ~3;
  const int geom_floats =
      primAl + silAl + wos::kGroupStride * s->host.n_pgroups + wos::kSGroupStride * s->host.n_sgroups;
  // the walk kernel also stages the star-radius grid (after the silhouette groups)
  wos::DevScene dsc = s->dev;
  dsc.sgrid = nullptr;
  dsc.sgrid_words = dsc.sgrid_off_words = 0;
  if (star_grid_enabled() && s->host.n_sil > 0) {
    int rc = ensure_star_grid(s, prm->silhouette_precision, prm->min_star_radius);
    if (rc != WOS_OK) return rc;
    if (s->sgrid_ok) {
      dsc.sgrid = s->d_sgrid;
      dsc.sgrid_words = (int32_t)s->sgrid.words.size();
      dsc.sgrid_off_words = s->sgrid.off_words;
      for (int k = 0; k < 3; k++) {
        dsc.sgrid_n[k] = s->sgrid.n[k];
        dsc.sgrid_min[k] = s->sgrid.gmin[k];
        dsc.sgrid_inv[k] = s->sgrid.inv[k];
      }
    }
  }
  int geom_floats_walk = geom_floats + ((dsc.sgrid_words + 3) & ~3);
  const int lhs_floats = ((2 * dp.n_pairs * (dim - 1)) + 3) & ~3;
  const size_t shmem_fb =
      (size_t)geom_floats * sizeof(float) + wos::kWavesPerBlockHost * wos::first_ball_wave_lds_bytes(lhs_floats);
  size_t shmem_walk =
      (size_t)geom_floats_walk * sizeof(float) + wos::kWavesPerBlockHost * wos::walk_wave_lds_bytes(dim);
  if (dsc.sgrid != nullptr && shmem_walk > kLdsDynamicMax) {  // no room: the group scan alone
    dsc.sgrid = nullptr;
    dsc.sgrid_words = dsc.sgrid_off_words = 0;
    geom_floats_walk = geom_floats;
    shmem_walk = (size_t)geom_floats * sizeof(float) + wos::kWavesPerBlockHost * wos::walk_wave_lds_bytes(dim);
  }
  if (std::max(shmem_fb, shmem_walk) > kLdsDynamicMax)
    return fail(WOS_E_CAPACITY, "wos_solve: scene + nWalks exceed the LDS budget of the staged kernels (" +
                                    std::to_string(std::max(shmem_fb, shmem_walk)) + " bytes)");

  const float* d_pts = pts;
  float* d_p = p;
  float* d_g = grad;
  int32_t* d_nest = n_est;
  int32_t* d_steps = steps;
  const bool dev_ptrs = (flags & WOS_PTRS_DEVICE) != 0;
  if (!dev_ptrs && n > 0) {
    int rc = ensure_workspace(s, (size_t)n);
    if (rc != WOS_OK) return rc;
    HIP_TRY(hipMemcpyAsync(s->d_pts, pts, (size_t)n * dim * sizeof(float), hipMemcpyHostToDevice, st));
    d_pts = s->d_pts; d_p = s->d_p; d_g = s->d_g;
    d_nest = n_est ? s->d_nest : nullptr;
    d_steps = steps ? s->d_steps : nullptr;
  }
  HIP_TRY(hipMemsetAsync(s->d_counters, 0, wos::kNumCounterSlots * sizeof(unsigned long long), st));

  // points are solved in batches whose walk tasks fit the task workspace
  const int64_t wpp = (int64_t)dp.n_pairs * dp.n_anti;
  const int64_t batch = std::max<int64_t>(1, std::min<int64_t>(n, kMaxBatchTasks / wpp));
  int grid_fb = 0, grid_walk = 0;
  if (n > 0) {
    int rc = ensure_tasks(s, batch * wpp, batch);
    if (rc != WOS_OK) return rc;
    int bpc = 0;
    HIP_TRY(wos::occupancy_blocks_per_cu(0, dim, shmem_fb, &bpc));
    grid_fb = (int)std::min<int64_t>((batch + wos::kWavesPerBlockHost - 1) / wos::kWavesPerBlockHost,
                                     (int64_t)std::max(1, bpc) * std::max(1, s->num_cus));
    HIP_TRY(wos::occupancy_blocks_per_cu(1, dim, shmem_walk, &bpc));
    grid_walk = std::max(1, bpc) * std::max(1, s->num_cus);
  }
  unsigned int* q_points = (unsigned int*)(s->d_counters + wos::kNumCounters);
  unsigned int* q_tasks = (unsigned int*)(s->d_counters + wos::kNumCounters + 1);
  const int64_t n_batches = n > 0 ? (n + batch - 1) / batch : 0;
  while ((int64_t)s->bev.size() < 4 * n_batches) {
    hipEvent_t e = nullptr;
    HIP_TRY(hipEventCreate(&e));
    s->bev.push_back(e);
  }
  HIP_TRY(hipEventRecord(s->ev0, st));
  for (int64_t b0 = 0; b0 < n; b0 += batch) {
    hipEvent_t* ev = &s->bev[4 * (b0 / batch)];
    const int64_t nb = std::min(batch, n - b0);
    wos::DevTasks tk = task_view(s, dim, nb * wpp, (int32_t)wpp);
    const int64_t bbase = index_base + b0 * index_stride;
    if (b0 > 0)
      HIP_TRY(hipMemsetAsync(s->d_counters + wos::kNumCounters, 0, 2 * sizeof(unsigned long long), st));
    HIP_TRY(hipMemsetAsync(tk.hist, 0, 2 * wos::kCostBuckets * sizeof(uint32_t), st));
    HIP_TRY(hipEventRecord(ev[0], st));
    HIP_TRY(wos::launch_first_balls(dim, s->dev, dp, d_pts + b0 * dim, nb, bbase, index_stride, tk, s->d_counters,
                                    q_points, grid_fb, shmem_fb, geom_floats, lhs_floats, st));
    HIP_TRY(wos::launch_lpt_order(tk, nb, st));
    HIP_TRY(hipEventRecord(ev[1], st));
    const int walk_grid = (int)std::min<int64_t>(grid_walk, (tk.T + 63) / 64);
    HIP_TRY(wos::launch_walks(dim, dsc, dp, tk, bbase, index_stride, s->d_counters, q_tasks, walk_grid,
                              shmem_walk, geom_floats_walk, st));
    HIP_TRY(hipEventRecord(ev[2], st));
    HIP_TRY(wos::launch_fold(dim, dp, tk, nb, d_p + b0, d_g + b0 * dim, d_nest ? d_nest + b0 : nullptr,
                             d_steps ? d_steps + b0 : nullptr, st));
    HIP_TRY(hipEventRecord(ev[3], st));
  }
  HIP_TRY(hipEventRecord(s->ev1, st));
  if (!dev_ptrs && n > 0) {
    HIP_TRY(hipMemcpyAsync(p, d_p, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(grad, d_g, (size_t)n * dim * sizeof(float), hipMemcpyDeviceToHost, st));
    if (n_est) HIP_TRY(hipMemcpyAsync(n_est, d_nest, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    if (steps) HIP_TRY(hipMemcpyAsync(steps, d_steps, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  }
  if ((flags & WOS_ASYNC) && dev_ptrs) return WOS_OK;
  HIP_TRY(hipStreamSynchronize(st));
  wos::diag_dump(dim == 2 ? "2d" : "3d");
  if (stats) {
    unsigned long long c[wos::kNumCounters];
    HIP_TRY(hipMemcpy(c, s->d_counters, sizeof(c), hipMemcpyDeviceToHost));
    stats->walk_steps = c[0];
    stats->wasted_steps = c[1];
    stats->walks_recorded = c[2];
    stats->walks_escaped = c[3];
    stats->walks_max_length = c[4];
    stats->walks_rr = c[5];
    stats->walks_dirichlet = c[6];
    stats->points_estimated = c[7];
    stats->rejection_iters = c[8];
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, s->ev0, s->ev1));
    stats->kernel_ms = ms;
    stats->first_ball_ms = stats->walk_ms = stats->fold_ms = 0.0;
    stats->walk_launches = (uint64_t)n_batches;
    for (int64_t b = 0; b < n_batches; b++) {
      hipEvent_t* ev = &s->bev[4 * b];
      float a = 0.0f, w = 0.0f, f = 0.0f;
      HIP_TRY(hipEventElapsedTime(&a, ev[0], ev[1]));
      HIP_TRY(hipEventElapsedTime(&w, ev[1], ev[2]));
      HIP_TRY(hipEventElapsedTime(&f, ev[2], ev[3]));
      stats->first_ball_ms += a; stats->walk_ms += w; stats->fold_ms += f;
    }
  }
  return WOS_OK;
}

int wos_selftest_math(int32_t which, const double* x, double* out, int64_t n, int32_t device) {
  if (!x || !out || n < 0) return fail(WOS_E_INVALID, "wos_selftest_math: bad argument");
  if (n == 0) return WOS_OK;
  HIP_TRY(hipSetDevice(device));
  double *dx = nullptr, *dy = nullptr;
  HIP_TRY(hipMalloc((void**)&dx, n * sizeof(double)));
  hipError_t e = hipMalloc((void**)&dy, n * sizeof(double));
  if (e == hipSuccess) e = hipMemcpy(dx, x, n * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = wos::launch_math_selftest(which, dx, dy, n, nullptr);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(out, dy, n * sizeof(double), hipMemcpyDeviceToHost);
  hipFree(dx);
  hipFree(dy);
  if (e != hipSuccess) return fail(WOS_E_DEVICE, std::string("wos_selftest_math: ") + hipGetErrorString(e));
  return WOS_OK;
}

}  // extern "C"
