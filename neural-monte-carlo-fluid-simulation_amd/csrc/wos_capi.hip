// wos_capi.hip -- the extern "C" boundary declared in include/wos.h.
//
// Device memory lives at three levels, sized for a time-stepper that builds a
// new Scene(sceneConfig, div) for every projection (model_split.py:191):
//   * per device (DevCtx, kept for the process): the solve workspace -- walk
//     tasks, per-point state, PCG32 jump table, counters, staging buffers for
//     host pointers, timing events.  Shared by every scene on the device, so a
//     fresh scene costs no workspace allocation;
//   * per geometry (Geom, shared by content, the 8 most recent kept after their
//     last scene is gone): the prepared boundary records and the star-radius
//     grids built for it, so re-creating a scene on the same boundary skips the
//     preparation and the upload;
//   * per scene: the source grid (replaceable in place, wos_scene_set_source).
// Errors are reported as status codes + wos_last_error(), never by aborting the
// process (the reference aborts: config.h:8-11, scene.h:106-109).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <list>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <condition_variable>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/wos.h"
#include "wos_bvc.h"
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
  if (e != hipSuccess) { *dst = nullptr; return e; }
  e = hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice);
  if (e != hipSuccess) {  // no half-initialised buffer is ever handed out
    hipFree(*dst);
    *dst = nullptr;
  }
  return e;
}

// ---- per-device solve workspace ---------------------------------------------
// Timing events + a pinned copy of the counters of one enqueued solve, so a solve
// enqueued with WOS_ASYNC can report its statistics later (wos_solve_stats) while
// the next solves are already queued behind it.
struct StatSlot {
  uint64_t ticket = 0;                  // 0: empty
  unsigned long long* h_cnt = nullptr;  // pinned host copy of the kNumCounters counters
  hipEvent_t ev0 = nullptr, ev1 = nullptr, done = nullptr;
  std::vector<hipEvent_t> bev;          // per-chunk kernel boundary events (4 per chunk), grow-only
  int64_t n_batches = 0;
  int32_t bpc_fb = 0, bpc_walk = 0, walk_lds = 0, star_grid = 0, geom_global = 0, dir_grid = 0;
};
constexpr int kStatSlots = 16;

// A walk-task workspace with its own counters and non-blocking stream: boundary value
// caching runs its independent walk sets (the boundary samples' walks, the walks of the
// evaluation points near the Dirichlet boundary) beside the Dirichlet samples' solve on
// the call's stream, so one set's long tail overlaps the others' bulk.
struct TaskWs {
  float* tasks = nullptr;
  int64_t task_cap = 0;
  int32_t* pstate = nullptr;
  int64_t pstate_cap = 0;
  unsigned long long* counters = nullptr;  // kNumCounterSlots
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
};
constexpr int kSideWs = 2;

struct DevCtx {
  std::mutex mu;  // one solve at a time per device (the workspace is shared)
  bool ready = false;
  int num_cus = 0;
  float* d_pts = nullptr;
  float* d_p = nullptr;
  float* d_g = nullptr;
  int32_t* d_nest = nullptr;
  int32_t* d_steps = nullptr;
  size_t ws_points = 0;
  uint64_t* d_jump = nullptr;  // PCG32 jump-ahead table (A_k, C_k), grow-only
  int n_jump = 0;
  float* d_tasks = nullptr;    // walk-task workspace (DevTasks arrays), grow-only
  int64_t task_cap = 0;
  int32_t* d_pstate = nullptr; // per-point state + queue permutation of one batch, then bucket counters
  int64_t pstate_cap = 0;
  unsigned long long* d_counters = nullptr;  // kNumCounters u64 + work counters (kMainCounterSlots)
  StatSlot slot[kStatSlots];   // ring indexed by ticket % kStatSlots
  uint64_t next_ticket = 1;
  hipEvent_t done = nullptr;   // end of the last enqueued solve
  hipStream_t last_stream = nullptr;
  bool inflight = false;       // a solve may still run on last_stream
  float* d_rejtab = nullptr;   // rejection bound table, 2D then 3D (DevParams::rej_tab)
  int stat_waiters = 0;        // wos_solve_stats calls waiting on a slot's event without the lock
  std::condition_variable no_waiters;
  TaskWs side[kSideWs];        // boundary value caching's side-stream workspaces (lazy)
  hipStream_t bvc_dir = nullptr;  // boundary value caching: the Dirichlet samples' solve (lazy)
  hipEvent_t bvc_dir_done = nullptr;
};

constexpr int kMaxDevices = 64;
DevCtx g_ctx[kMaxDevices];  // never destroyed: the HIP runtime may be gone at process exit

void ctx_free(DevCtx& c) {
  hipFree(c.d_pts); hipFree(c.d_p); hipFree(c.d_g); hipFree(c.d_nest); hipFree(c.d_steps);
  hipFree(c.d_jump); hipFree(c.d_tasks); hipFree(c.d_pstate); hipFree(c.d_counters); hipFree(c.d_rejtab);
  c.d_rejtab = nullptr;
  for (StatSlot& q : c.slot) {
    if (q.ev0) hipEventDestroy(q.ev0);
    if (q.ev1) hipEventDestroy(q.ev1);
    if (q.done) hipEventDestroy(q.done);
    for (hipEvent_t e : q.bev) hipEventDestroy(e);
    if (q.h_cnt) hipHostFree(q.h_cnt);
    q = StatSlot{};
  }
  if (c.done) hipEventDestroy(c.done);
  if (c.bvc_dir_done) hipEventDestroy(c.bvc_dir_done);
  if (c.bvc_dir) hipStreamDestroy(c.bvc_dir);
  c.bvc_dir_done = nullptr;
  c.bvc_dir = nullptr;
  for (TaskWs& w : c.side) {
    hipFree(w.tasks); hipFree(w.pstate); hipFree(w.counters);
    if (w.done) hipEventDestroy(w.done);
    if (w.stream) hipStreamDestroy(w.stream);
    w = TaskWs{};
  }
  c.d_pts = c.d_p = c.d_g = nullptr;
  c.d_nest = c.d_steps = nullptr;
  c.ws_points = 0;
  c.d_jump = nullptr; c.n_jump = 0;
  c.d_tasks = nullptr; c.task_cap = 0;
  c.d_pstate = nullptr; c.pstate_cap = 0;
  c.d_counters = nullptr;
  c.done = nullptr;
  c.last_stream = nullptr;
  c.inflight = false;
  c.ready = false;
}

// the rejection bound tables (host, computed once per process)
const std::vector<float>& rejection_tables() {
  static std::once_flag once;
  // [2D bound | 3D bound] (DevParams::rej_tab)
  static std::vector<float> t(2 * wos::kRejTabBins);
  std::call_once(once, [] {
    wos::rejection_bound_table(2, t.data());
    wos::rejection_bound_table(3, t.data() + wos::kRejTabBins);
  });
  return t;
}

// caller holds c.mu and has selected the device
int ctx_ready(DevCtx& c, int device) {
  if (c.ready) return WOS_OK;
  {
    const std::vector<float>& t = rejection_tables();
    HIP_TRY(hipMalloc((void**)&c.d_rejtab, t.size() * sizeof(float)));
    HIP_TRY(hipMemcpy(c.d_rejtab, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  HIP_TRY(hipDeviceGetAttribute(&c.num_cus, hipDeviceAttributeMultiprocessorCount, device));
  HIP_TRY(hipMalloc((void**)&c.d_counters, wos::kMainCounterSlots * sizeof(unsigned long long)));
  for (StatSlot& q : c.slot) {
    HIP_TRY(hipHostMalloc((void**)&q.h_cnt, wos::kNumCounters * sizeof(unsigned long long)));
    HIP_TRY(hipEventCreate(&q.ev0));
    HIP_TRY(hipEventCreate(&q.ev1));
    HIP_TRY(hipEventCreateWithFlags(&q.done, hipEventDisableTiming));
  }
  HIP_TRY(hipEventCreateWithFlags(&c.done, hipEventDisableTiming));
  c.ready = true;
  return WOS_OK;
}

// order `st` after the last solve enqueued on another stream (the workspace and,
// for set_source, the source grid may still be in use there)
hipError_t ctx_order(DevCtx& c, hipStream_t st) {
  if (c.inflight && c.last_stream != st && c.done) return hipStreamWaitEvent(st, c.done, 0);
  return hipSuccess;
}

// ---- prepared geometry, shared by content -----------------------------------
struct Geom {
  int device = 0;
  int dim = 2, double_sided = 0;
  std::vector<float> v, dv;  // the key: exactly the inputs of prepare_scene
  std::vector<int32_t> ix, dix;
  wos::HostScene host;
  float *d_prim = nullptr, *d_paux = nullptr, *d_sil = nullptr, *d_dprim = nullptr, *d_dpaux = nullptr;
  float *d_pgroup = nullptr, *d_sgroup = nullptr, *d_dgroup = nullptr;
  float *d_ptree = nullptr, *d_stree = nullptr, *d_dtree = nullptr;
  float* d_nbox = nullptr;  // fcpw's Neumann BVH (stochastic boundary sample)
  int32_t *d_nchild = nullptr, *d_nref = nullptr;
  std::mutex mu;  // star grids
  struct Grid {
    float prec, min_r;
    bool ok;
    wos::StarGrid grid;
    uint32_t* d = nullptr;
  };
  std::list<Grid> grids;  // stable addresses (a solve keeps a pointer)
  // the Dirichlet-distance cell grid (geometry only: built once, on first use)
  bool dgrid_built = false, dgrid_ok = false;
  wos::DirGrid dgrid;
  uint32_t* d_dgrid = nullptr;
  ~Geom() {
    hipSetDevice(device);
    hipFree(d_prim); hipFree(d_paux); hipFree(d_sil); hipFree(d_dprim); hipFree(d_dpaux);
    hipFree(d_pgroup); hipFree(d_sgroup); hipFree(d_dgroup);
    hipFree(d_ptree); hipFree(d_stree); hipFree(d_dtree);
    hipFree(d_nbox); hipFree(d_nchild); hipFree(d_nref);
    for (Grid& g : grids) hipFree(g.d);
    hipFree(d_dgrid);
  }
};

std::mutex g_geom_mu;
// most recent first; heap-held and never destroyed (no hipFree during static teardown)
std::vector<std::shared_ptr<Geom>>& g_geom_lru = *new std::vector<std::shared_ptr<Geom>>();
constexpr size_t kGeomCacheSize = 8;

template <typename T>
bool same(const std::vector<T>& a, const T* b, int n) {
  return a.size() == (size_t)n && (n == 0 || std::memcmp(a.data(), b, (size_t)n * sizeof(T)) == 0);
}

bool geom_matches(const Geom& g, const wos_scene_desc* d, int device) {
  const int dim = d->dim;
  return g.device == device && g.dim == dim && g.double_sided == d->is_double_sided &&
         same(g.v, d->vertices, d->n_vertices * dim) && same(g.ix, d->prims, d->n_prims * dim) &&
         same(g.dv, d->dvertices, d->n_dvertices * dim) && same(g.dix, d->dprims, d->n_dprims * dim);
}

// the prepared geometry of `d` on `device`: from the cache, else prepared + uploaded
int geom_get(const wos_scene_desc* d, int device, std::shared_ptr<Geom>& out) {
  {
    std::lock_guard<std::mutex> lk(g_geom_mu);
    for (size_t i = 0; i < g_geom_lru.size(); i++)
      if (geom_matches(*g_geom_lru[i], d, device)) {
        out = g_geom_lru[i];
        std::rotate(g_geom_lru.begin(), g_geom_lru.begin() + i, g_geom_lru.begin() + i + 1);
        return WOS_OK;
      }
  }
  auto g = std::make_shared<Geom>();
  const int dim = d->dim;
  g->device = device;
  g->dim = dim;
  g->double_sided = d->is_double_sided;
  if (d->n_vertices > 0) g->v.assign(d->vertices, d->vertices + (size_t)d->n_vertices * dim);
  if (d->n_prims > 0) g->ix.assign(d->prims, d->prims + (size_t)d->n_prims * dim);
  if (d->n_dvertices > 0) g->dv.assign(d->dvertices, d->dvertices + (size_t)d->n_dvertices * dim);
  if (d->n_dprims > 0) g->dix.assign(d->dprims, d->dprims + (size_t)d->n_dprims * dim);
  wos::HostSceneInput in;
  in.dim = dim;
  in.vertices = d->vertices; in.prims = d->prims; in.n_vertices = d->n_vertices; in.n_prims = d->n_prims;
  in.dvertices = d->dvertices; in.dprims = d->dprims; in.n_dvertices = d->n_dvertices; in.n_dprims = d->n_dprims;
  in.is_double_sided = d->is_double_sided;
  std::string err;
  if (!wos::prepare_scene(in, g->host, err)) return fail(WOS_E_INVALID, "wos_scene_create: " + err);
  HIP_TRY(upload(&g->d_prim, g->host.prim));
  HIP_TRY(upload(&g->d_paux, g->host.paux));
  HIP_TRY(upload(&g->d_sil, g->host.sil));
  HIP_TRY(upload(&g->d_dprim, g->host.dprim));
  HIP_TRY(upload(&g->d_dpaux, g->host.dpaux));
  HIP_TRY(upload(&g->d_pgroup, g->host.pgroup));
  HIP_TRY(upload(&g->d_dgroup, g->host.dgroup));
  HIP_TRY(upload(&g->d_sgroup, g->host.sgroup));
  HIP_TRY(upload(&g->d_ptree, g->host.ptree.node));
  HIP_TRY(upload(&g->d_stree, g->host.stree.node));
  HIP_TRY(upload(&g->d_dtree, g->host.dtree.node));
  HIP_TRY(upload(&g->d_nbox, g->host.nbvh.box));
  HIP_TRY(upload(&g->d_nchild, g->host.nbvh.child));
  HIP_TRY(upload(&g->d_nref, g->host.nbvh.ref));
  {
    std::lock_guard<std::mutex> lk(g_geom_mu);
    g_geom_lru.insert(g_geom_lru.begin(), g);
    if (g_geom_lru.size() > kGeomCacheSize) g_geom_lru.pop_back();
  }
  out = g;
  return WOS_OK;
}

// LDS budget of the star-radius grid (staged by every walk-kernel workgroup)
constexpr size_t kStarGridBudget = 16 * 1024;

// dynamic LDS a workgroup may use: 160 KB per CU minus the kernels' static LDS
// (rejection jump table 2 KB, counters, histogram)
constexpr size_t kLdsDynamicMax = 160 * 1024 - 4096;

// the star grid of `g` for the solver's silhouette precision and minR (built once)
int star_grid(Geom& g, float prec, float min_r, const Geom::Grid** out) {
  std::lock_guard<std::mutex> lk(g.mu);
  for (const Geom::Grid& x : g.grids)
    if (x.prec == prec && x.min_r == min_r) { *out = &x; return WOS_OK; }
  Geom::Grid x{prec, min_r, false, {}, nullptr};
  // cached (ok or not) only once its upload has succeeded: a failed upload is reported and
  // the next solve builds the grid again
  if (wos::build_star_grid(g.host, prec, min_r, kStarGridBudget, x.grid)) {
    HIP_TRY(upload(&x.d, x.grid.words));
    x.ok = true;
  }
  g.grids.push_back(std::move(x));
  *out = &g.grids.back();
  return WOS_OK;
}

int dir_grid(Geom& g, bool* ok) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (!g.dgrid_built) {
    // built / ok only once the upload has succeeded (upload leaves d_dgrid null on failure),
    // so no later solve reads a half-initialised grid
    const bool have = wos::build_dirichlet_grid(g.host, g.dgrid);
    if (have) HIP_TRY(upload(&g.d_dgrid, g.dgrid.words));
    g.dgrid_ok = have;
    g.dgrid_built = true;
  }
  *ok = g.dgrid_ok;
  return WOS_OK;
}

// walk tasks per batch: 2^28 tasks = 16 GB of workspace at most (60 B per task, sized for 3D), 5.6 % of a
// MI355X's 288 GB -- config E (2^31 walks) runs in 8 batches, D (2^27) and each rank's share of an 8-GPU
// E in one.  Fewer batches, fewer ramp-downs of the persistent kernels: against 2^24 (round 5) C 12.8 ->
// 11.6 ms, D 26.0 -> 24.0 ms, E 420 -> 376 ms, first balls of E 127 -> 102 ms, bit-exact
// (profiles/r6c_ab_batch.log; 2^26 / 2^27 in between).  A smaller solve allocates only what it uses.
#ifndef WOS_BATCH_LOG2
#define WOS_BATCH_LOG2 28
#endif
static_assert(WOS_BATCH_LOG2 <= 30, "task indices carry a flag in bit 31 (wos_walk_kernel hand-out)");
constexpr int64_t kDefaultBatchTasks = (int64_t)1 << WOS_BATCH_LOG2;
std::atomic<int64_t> g_max_batch_tasks{kDefaultBatchTasks};  // wos_set_max_batch_tasks

}  // namespace

struct wos_scene {
  int device = 0;
  std::shared_ptr<Geom> geom;
  wos::DevScene dev{};
  float* d_source = nullptr;
  size_t source_cap = 0;  // floats
  float* d_dimg = nullptr;  // image-valued Dirichlet data (wos_scene_desc.dirichlet_image)
  float* d_nimg = nullptr;  // image-valued Neumann data (wos_scene_desc.neumann_image)
  std::mutex mu;          // solve vs set_source on the same scene
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

static int check_source_dims(int dim, const int32_t* dims, size_t* nsrc) {
  const int nsd = dim == 2 ? 2 : 3;
  size_t n = 1;
  for (int k = 0; k < nsd; k++) {
    if (dims[k] <= 0) return fail(WOS_E_INVALID, "bad source dims");
    n *= (size_t)dims[k];
  }
  *nsrc = n;
  return WOS_OK;
}

int wos_scene_create(const wos_scene_desc* d, int32_t device, wos_scene** out) {
  if (!d || !out) return fail(WOS_E_INVALID, "wos_scene_create: null argument");
  *out = nullptr;
  if (d->dim != 2 && d->dim != 3) return fail(WOS_E_INVALID, "wos_scene_create: dim must be 2 or 3");
  size_t nsrc = 0;
  if (d->source && check_source_dims(d->dim, d->source_dims, &nsrc) != WOS_OK)
    return fail(WOS_E_INVALID, "wos_scene_create: bad source dims");
  if (!(d->absorption >= 0.0f)) return fail(WOS_E_INVALID, "wos_scene_create: absorption must be >= 0");
  size_t ndimg = 0;
  if (d->dirichlet_image) {
    if (d->dim != 2) return fail(WOS_E_INVALID, "wos_scene_create: dirichlet_image is 2D only");
    if (d->dirichlet_image_dims[0] < 1 || d->dirichlet_image_dims[1] < 1 ||
        (int64_t)d->dirichlet_image_dims[0] * d->dirichlet_image_dims[1] > (int64_t)1 << 28)
      return fail(WOS_E_INVALID, "wos_scene_create: bad dirichlet_image dims");
    if (!(d->dirichlet_image_box[2] > 0.0f) || !(d->dirichlet_image_box[3] > 0.0f))
      return fail(WOS_E_INVALID, "wos_scene_create: dirichlet_image_box extent must be > 0");
    ndimg = (size_t)d->dirichlet_image_dims[0] * d->dirichlet_image_dims[1];
  }
  size_t nnimg = 0;
  if (d->neumann_image) {
    if (d->dim != 2) return fail(WOS_E_INVALID, "wos_scene_create: neumann_image is 2D only");
    if (d->neumann_image_dims[0] < 1 || d->neumann_image_dims[1] < 1 ||
        (int64_t)d->neumann_image_dims[0] * d->neumann_image_dims[1] > (int64_t)1 << 28)
      return fail(WOS_E_INVALID, "wos_scene_create: bad neumann_image dims");
    const float* nb = d->neumann_image_box;
    if (!std::isfinite(nb[0]) || !std::isfinite(nb[1]) || !(nb[2] > 0.0f) || !(nb[3] > 0.0f) ||
        !std::isfinite(nb[2]) || !std::isfinite(nb[3]))
      return fail(WOS_E_INVALID, "wos_scene_create: neumann_image_box needs a finite corner and extents > 0");
    nnimg = (size_t)d->neumann_image_dims[0] * d->neumann_image_dims[1];
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(WOS_E_DEVICE, "wos_scene_create: no HIP device available");
  if (device < 0 || device >= ndev || device >= kMaxDevices)
    return fail(WOS_E_INVALID, "wos_scene_create: device index out of range");
  HIP_TRY(hipSetDevice(device));
  std::shared_ptr<Geom> geom;
  int rc = geom_get(d, device, geom);
  if (rc != WOS_OK) return rc;
  auto* s = new wos_scene();
  s->device = device;
  s->geom = geom;
  if (d->source) {
    hipError_t e = hipMalloc((void**)&s->d_source, nsrc * sizeof(float));
    if (e == hipSuccess)
      e = hipMemcpy(s->d_source, d->source, nsrc * sizeof(float),
                    d->source_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      hipFree(s->d_source);
      delete s;
      return fail(WOS_E_DEVICE, std::string("wos_scene_create: ") + hipGetErrorString(e));
    }
    s->source_cap = nsrc;
  }
  if (ndimg) {
    hipError_t e = hipMalloc((void**)&s->d_dimg, ndimg * sizeof(float));
    if (e == hipSuccess)
      e = hipMemcpy(s->d_dimg, d->dirichlet_image, ndimg * sizeof(float),
                    d->dirichlet_image_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      hipFree(s->d_dimg);
      hipFree(s->d_source);
      delete s;
      return fail(WOS_E_DEVICE, std::string("wos_scene_create: ") + hipGetErrorString(e));
    }
  }
  if (nnimg) {
    hipError_t e = hipMalloc((void**)&s->d_nimg, nnimg * sizeof(float));
    if (e == hipSuccess)
      e = hipMemcpy(s->d_nimg, d->neumann_image, nnimg * sizeof(float),
                    d->neumann_image_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      hipFree(s->d_nimg);
      hipFree(s->d_dimg);
      hipFree(s->d_source);
      delete s;
      return fail(WOS_E_DEVICE, std::string("wos_scene_create: ") + hipGetErrorString(e));
    }
  }
  const wos::HostScene& h = geom->host;
  wos::DevScene& ds = s->dev;
  ds.dim = d->dim;
  ds.n_prims = h.n_prims;
  ds.n_sil = h.n_sil;
  ds.n_dprims = h.n_dprims;
  ds.prim = geom->d_prim; ds.paux = geom->d_paux; ds.sil = geom->d_sil;
  ds.dprim = geom->d_dprim; ds.dpaux = geom->d_dpaux;
  ds.source = s->d_source;
  ds.pgroup = geom->d_pgroup; ds.sgroup = geom->d_sgroup; ds.dgroup = geom->d_dgroup;
  ds.n_pgroups = h.n_pgroups; ds.n_sgroups = h.n_sgroups; ds.n_dgroups = h.n_dgroups;
  auto tree = [](const wos::HostTree& ht, const float* dnode) {
    wos::DevTree t{};
    t.node = dnode;
    t.levels = ht.levels;
    for (int l = 0; l <= wos::kTreeLevels; l++) { t.n[l] = ht.n[l]; t.off[l] = ht.off[l]; }
    return t;
  };
  ds.ptree = tree(h.ptree, geom->d_ptree);
  ds.stree = tree(h.stree, geom->d_stree);
  ds.dtree = tree(h.dtree, geom->d_dtree);
  ds.nbvh_box = geom->d_nbox;
  ds.nbvh_child = geom->d_nchild;
  ds.nbvh_ref = geom->d_nref;
  ds.nbvh_branch = h.nbvh.branch;
  const int nsd = d->dim == 2 ? 2 : 3;
  for (int k = 0; k < 3; k++) {
    ds.sdims[k] = d->source ? (k < nsd ? d->source_dims[k] : 1) : 0;
    ds.pmin[k] = h.pmin[k]; ds.pmax[k] = h.pmax[k]; ds.ext[k] = h.ext[k];
  }
  ds.absorption = d->absorption;
  ds.g_dirichlet = d->dirichlet_value;
  ds.dimg = s->d_dimg;
  for (int k = 0; k < 2; k++) ds.ddims[k] = ndimg ? d->dirichlet_image_dims[k] : 0;
  for (int k = 0; k < 4; k++) ds.dbox[k] = ndimg ? d->dirichlet_image_box[k] : 0.0f;
  ds.nimg = s->d_nimg;
  for (int k = 0; k < 2; k++) ds.ndims[k] = nnimg ? d->neumann_image_dims[k] : 0;
  for (int k = 0; k < 4; k++) ds.nbox[k] = nnimg ? d->neumann_image_box[k] : 0.0f;
  ds.watertight = d->is_watertight;
  ds.double_sided = d->is_double_sided;
  *out = s;
  return WOS_OK;
}

int wos_scene_set_source(wos_scene* s, const float* source, const int32_t* dims, int32_t on_device, void* stream) {
  if (!s || !source || !dims) return fail(WOS_E_INVALID, "wos_scene_set_source: null argument");
  size_t nsrc = 0;
  if (check_source_dims(s->dev.dim, dims, &nsrc) != WOS_OK) return fail(WOS_E_INVALID, "wos_scene_set_source: bad source dims");
  std::lock_guard<std::mutex> lock(s->mu);
  HIP_TRY(hipSetDevice(s->device));
  hipStream_t st = (hipStream_t)stream;
  DevCtx& c = g_ctx[s->device];
  {
    std::lock_guard<std::mutex> lk(c.mu);
    HIP_TRY(ctx_order(c, st));  // a solve on another stream may still read the old grid
  }
  if (nsrc > s->source_cap) {
    HIP_TRY(hipStreamSynchronize(st));
    hipFree(s->d_source);
    s->d_source = nullptr;
    s->source_cap = 0;
    HIP_TRY(hipMalloc((void**)&s->d_source, nsrc * sizeof(float)));
    s->source_cap = nsrc;
  }
  HIP_TRY(hipMemcpyAsync(s->d_source, source, nsrc * sizeof(float),
                         on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
  const int nsd = s->dev.dim == 2 ? 2 : 3;
  s->dev.source = s->d_source;
  for (int k = 0; k < 3; k++) s->dev.sdims[k] = k < nsd ? dims[k] : 1;
  return WOS_OK;
}

int wos_scene_destroy(wos_scene* s) {
  if (!s) return WOS_OK;
  {
    std::lock_guard<std::mutex> lock(s->mu);
    hipSetDevice(s->device);
    DevCtx& c = g_ctx[s->device];
    std::lock_guard<std::mutex> lk(c.mu);
    if (c.inflight) hipEventSynchronize(c.done);  // an async solve may still read the source
    hipFree(s->d_source);
    hipFree(s->d_dimg);
    hipFree(s->d_nimg);
  }
  delete s;
  return WOS_OK;
}

int64_t wos_set_max_batch_tasks(int64_t max_tasks) {
  const int64_t v = max_tasks <= 0 ? kDefaultBatchTasks
                                   : std::min<int64_t>(std::max<int64_t>(max_tasks, (int64_t)1 << 16), (int64_t)1 << 30);
  return g_max_batch_tasks.exchange(v);
}

int wos_release_caches(int32_t device) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  for (int dv = 0; dv < std::min(ndev, kMaxDevices); dv++) {
    if (device >= 0 && dv != device) continue;
    DevCtx& c = g_ctx[dv];
    std::unique_lock<std::mutex> lk(c.mu);
    // the slot events may be awaited by wos_solve_stats outside the lock
    c.no_waiters.wait(lk, [&] { return c.stat_waiters == 0; });
    if (!c.ready) continue;
    HIP_TRY(hipSetDevice(dv));
    HIP_TRY(hipDeviceSynchronize());
    ctx_free(c);
  }
  std::lock_guard<std::mutex> lk(g_geom_mu);
  if (device < 0) {
    g_geom_lru.clear();
  } else {
    g_geom_lru.erase(std::remove_if(g_geom_lru.begin(), g_geom_lru.end(),
                                    [&](const std::shared_ptr<Geom>& g) { return g->device == device; }),
                     g_geom_lru.end());
  }
  return WOS_OK;
}

int wos_scene_get_info(const wos_scene* s, wos_scene_info* info) {
  if (!s || !info) return fail(WOS_E_INVALID, "wos_scene_get_info: null argument");
  const wos::HostScene& h = s->geom->host;
  info->dim = h.dim;
  info->n_prims = h.n_prims;
  info->n_silhouettes = h.n_sil;
  info->n_dprims = h.n_dprims;
  info->device = s->device;
  for (int k = 0; k < 3; k++) { info->bbox_min[k] = h.pmin[k]; info->bbox_max[k] = h.pmax[k]; }
  return WOS_OK;
}

}  // extern "C"

namespace {

int ensure_workspace(DevCtx& c, int dim, size_t npts) {
  if (npts <= c.ws_points) return WOS_OK;
  hipFree(c.d_pts); hipFree(c.d_p); hipFree(c.d_g); hipFree(c.d_nest); hipFree(c.d_steps);
  c.d_pts = c.d_p = c.d_g = nullptr; c.d_nest = c.d_steps = nullptr; c.ws_points = 0;
  const size_t cap = npts + npts / 4 + 1024;
  HIP_TRY(hipMalloc((void**)&c.d_pts, cap * 3 * sizeof(float)));  // either dimension
  HIP_TRY(hipMalloc((void**)&c.d_p, cap * sizeof(float)));
  HIP_TRY(hipMalloc((void**)&c.d_g, cap * 3 * sizeof(float)));
  HIP_TRY(hipMalloc((void**)&c.d_nest, cap * sizeof(int32_t)));
  HIP_TRY(hipMalloc((void**)&c.d_steps, cap * sizeof(int32_t)));
  (void)dim;
  c.ws_points = cap;
  return WOS_OK;
}


int ensure_tasks_in(float*& d_tasks, int64_t& task_cap, int32_t*& d_pstate, int64_t& pstate_cap, int dim,
                    int64_t tasks, int64_t points) {
  // sized for 3D records so either dimension fits
  const int tf = std::max(wos::task_floats(dim), wos::task_floats(3));
  if (tasks > task_cap) {
    hipFree(d_tasks);
    d_tasks = nullptr; task_cap = 0;
    HIP_TRY(hipMalloc((void**)&d_tasks, (size_t)tasks * tf * sizeof(float)));
    task_cap = tasks;
  }
  if (points > pstate_cap) {
    hipFree(d_pstate);
    d_pstate = nullptr; pstate_cap = 0;
    HIP_TRY(hipMalloc((void**)&d_pstate, ((size_t)7 * points + 2 * wos::kCostBuckets) * sizeof(int32_t)));
    pstate_cap = points;
  }
  return WOS_OK;
}

int ensure_tasks(DevCtx& c, int dim, int64_t tasks, int64_t points) {
  return ensure_tasks_in(c.d_tasks, c.task_cap, c.d_pstate, c.pstate_cap, dim, tasks, points);
}

// SoA views into a task workspace for a chunk of T tasks
wos::DevTasks task_view_in(float* d_tasks, int32_t* d_pstate, int64_t pstate_cap, int dim, int64_t T, int32_t wpp) {
  wos::DevTasks tk{};
  float* f = d_tasks;
  tk.pt = f; f += dim * T;
  tk.thr = f; f += T;
  tk.tsrc = f; f += T;
  tk.dd = f; f += T;
  tk.first = f; f += T;
  tk.bdir = f; f += dim * T;
  tk.sdir = f; f += dim * T;
  tk.total = f; f += T;
  tk.code = (uint32_t*)f;
  tk.pstate = d_pstate;
  tk.perm = (uint32_t*)(d_pstate + pstate_cap);
  tk.prad = (float*)(d_pstate + 2 * pstate_cap);
  tk.hist = (uint32_t*)(d_pstate + 3 * pstate_cap);
  tk.pball = (float*)(d_pstate + 3 * pstate_cap + 2 * wos::kCostBuckets);
  tk.pball_stride = pstate_cap;
  tk.T = T;
  tk.wpp = wpp;
  return tk;
}

wos::DevTasks task_view(DevCtx& c, int dim, int64_t T, int32_t wpp) {
  return task_view_in(c.d_tasks, c.d_pstate, c.pstate_cap, dim, T, wpp);
}

// Stream priorities of boundary value caching's walk sets: the Dirichlet samples' solve and
// the Neumann samples' walks feed the splat (high), the near-boundary walks do not (low).

int bvc_priority(bool high) {
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return 0;
  return high ? greatest : least;
}

// a side workspace's stream, event and counters (created on first use)
int side_ready(TaskWs& w, int priority) {
  if (!w.stream) HIP_TRY(hipStreamCreateWithPriority(&w.stream, hipStreamNonBlocking, priority));
  if (!w.done) HIP_TRY(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
  if (!w.counters) HIP_TRY(hipMalloc((void**)&w.counters, wos::kNumCounterSlots * sizeof(unsigned long long)));
  return WOS_OK;
}

// state_k = A_k * state_0 + C_k for the PCG32 LCG (multiplier kPcgMult, increment kPcgInc)
int ensure_jump(DevCtx& c, int k_needed) {
  if (k_needed <= c.n_jump) return WOS_OK;
  // >= 2 * 1000 + 2: the wave-cooperative rejection sampler jumps up to 1000 iterations ahead
  const int cap = std::max(k_needed, 4096);
  std::vector<uint64_t> t(2 * (size_t)cap);
  uint64_t A = 1u, Cc = 0u;
  for (int k = 0; k < cap; k++) {
    t[2 * k] = A; t[2 * k + 1] = Cc;
    A = A * wos::kPcgMult;
    Cc = Cc * wos::kPcgMult + wos::kPcgInc;
  }
  hipFree(c.d_jump);
  c.d_jump = nullptr; c.n_jump = 0;
  HIP_TRY(hipMalloc((void**)&c.d_jump, t.size() * sizeof(uint64_t)));
  HIP_TRY(hipMemcpy(c.d_jump, t.data(), t.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
  c.n_jump = cap;
  return WOS_OK;
}

// statistics of the solve held by slot q (its done event has completed)
int fill_stats(const StatSlot& q, wos_stats* stats) {
  *stats = wos_stats{};
  const unsigned long long* cnt = q.h_cnt;
  stats->walk_steps = cnt[0];
  stats->wasted_steps = cnt[1];
  stats->walks_recorded = cnt[2];
  stats->walks_escaped = cnt[3];
  stats->walks_max_length = cnt[4];
  stats->walks_rr = cnt[5];
  stats->walks_dirichlet = cnt[6];
  stats->points_estimated = cnt[7];
  stats->rejection_iters = cnt[8];
  float ms = 0.0f;
  HIP_TRY(hipEventElapsedTime(&ms, q.ev0, q.ev1));
  stats->kernel_ms = ms;
  stats->walk_launches = (uint64_t)q.n_batches;
  for (int64_t b = 0; b < q.n_batches; b++) {
    const hipEvent_t* ev = &q.bev[4 * b];
    float a = 0.0f, w = 0.0f, f = 0.0f;
    HIP_TRY(hipEventElapsedTime(&a, ev[0], ev[1]));
    HIP_TRY(hipEventElapsedTime(&w, ev[1], ev[2]));
    HIP_TRY(hipEventElapsedTime(&f, ev[2], ev[3]));
    stats->first_ball_ms += a; stats->walk_ms += w; stats->fold_ms += f;
  }
  stats->first_ball_blocks_per_cu = q.bpc_fb;
  stats->walk_blocks_per_cu = q.bpc_walk;
  stats->walk_lds_bytes = q.walk_lds;
  stats->star_grid = q.star_grid;
  stats->geom_global = q.geom_global;
  stats->dir_grid = q.dir_grid;
  stats->ticket = q.ticket;
  return WOS_OK;
}

// The walk kernel's LDS image for a solve on `s`: staged geometry, the star-radius
// grid of the solver's precision / minR (if it fits), the Dirichlet primitives.
struct WalkLayout {
  wos::DevScene dsc;          // the scene with its star grid (or none)
  int geom_floats = 0;        // Neumann records + culling boxes
  int geom_floats_walk = 0;   // + the star grid + the Dirichlet records (the walk kernel)
  size_t shmem_walk = 0;      // dynamic LDS of a walk-kernel workgroup
};

int walk_layout(wos_scene* s, const wos_solver_params* prm, WalkLayout& L) {
  Geom& geom = *s->geom;
  const wos::HostScene& host = geom.host;
  const int dim = host.dim;
  const int PS = dim == 2 ? wos::kPrimStride2 : wos::kPrimStride3;
  const int SS = dim == 2 ? wos::kSilStride2 : wos::kSilStride3;
  const int primAl = (host.n_prims * PS + 3) & ~3;
  const int silAl = (host.n_sil * SS + 3) & ~3;
  L.geom_floats = primAl + silAl + wos::kGroupStride * host.n_pgroups + wos::kSGroupStride * host.n_sgroups;
  // the walk kernel also stages the star-radius grid (after the silhouette groups)
  wos::DevScene& dsc = L.dsc;
  dsc = s->dev;
  dsc.sgrid = nullptr;
  dsc.sgrid_words = dsc.sgrid_off_words = 0;
  if (!(prm->schedule & WOS_SCHED_NO_STAR_GRID) && host.n_sil > 0) {
    const Geom::Grid* gr = nullptr;
    int rc = star_grid(geom, prm->silhouette_precision, prm->min_star_radius, &gr);
    if (rc != WOS_OK) return rc;
    if (gr->ok) {
      dsc.sgrid = gr->d;
      dsc.sgrid_words = (int32_t)gr->grid.words.size();
      dsc.sgrid_off_words = gr->grid.off_words;
      for (int k = 0; k < 3; k++) {
        dsc.sgrid_n[k] = gr->grid.n[k];
        dsc.sgrid_min[k] = gr->grid.gmin[k];
        dsc.sgrid_inv[k] = gr->grid.inv[k];
      }
    }
  }
  // the Dirichlet-distance cell grid (global memory)
  dsc.dgrid = nullptr;
  if (!(prm->schedule & WOS_SCHED_NO_DIR_GRID) && host.dim == 2 && host.n_dprims > 0) {
    bool ok = false;
    int rc = dir_grid(geom, &ok);
    if (rc != WOS_OK) return rc;
    if (ok) {
      dsc.dgrid = geom.d_dgrid;
      dsc.dgrid_off_words = geom.dgrid.off_words;
      for (int k = 0; k < 2; k++) {
        dsc.dgrid_n[k] = geom.dgrid.n[k];
        dsc.dgrid_min[k] = geom.dgrid.gmin[k];
        dsc.dgrid_inv[k] = geom.dgrid.inv[k];
      }
    }
  }
  // ... and the Dirichlet primitives with their culling boxes (after the grid)
  const int dir_floats = ((host.n_dprims * PS + 3) & ~3) + wos::kGroupStride * host.n_dgroups;
  L.geom_floats_walk = L.geom_floats + ((dsc.sgrid_words + 3) & ~3) + dir_floats;
  L.shmem_walk = (size_t)L.geom_floats_walk * sizeof(float) + wos::kWavesPerBlockHost * wos::walk_wave_lds_bytes(dim);
  if (dsc.sgrid != nullptr && L.shmem_walk > kLdsDynamicMax) {  // no room: the group scan alone
    dsc.sgrid = nullptr;
    dsc.sgrid_words = dsc.sgrid_off_words = 0;
    L.geom_floats_walk = L.geom_floats + dir_floats;
    L.shmem_walk =
        (size_t)L.geom_floats_walk * sizeof(float) + wos::kWavesPerBlockHost * wos::walk_wave_lds_bytes(dim);
  }
  return WOS_OK;
}

// device allocations of one call, freed on every exit path
struct DevBufs {
  std::vector<void*> p;
  ~DevBufs() { for (void* q : p) hipFree(q); }
  template <typename T>
  hipError_t get(T** out, size_t n) {
    *out = nullptr;
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, std::max<size_t>(1, n) * sizeof(T));
    if (e == hipSuccess) { p.push_back(q); *out = (T*)q; }
    return e;
  }
};

// DevParams of a solve (walk_on_stars.h WalkSettings from the solver keys)
wos::DevParams dev_params(const wos_solver_params* prm) {
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
  dp.robust = prm->robust_float != 0;
  dp.seed = prm->seed;
  return dp;
}

// what a solve needs beyond wos_solve's arguments (BVC's Dirichlet samples): per point the
// direction of the derivative [n][dim] and the derivative out [n] (device pointers), and
// estimation at every point regardless of the inside test
struct SolveExtra {
  const float* ddir = nullptr;
  float* deriv = nullptr;
  bool force_estimate = false;
  int wave_prio = 0;  // the walk / fold kernels' waves at this issue priority (0..3)
};

int solve_locked(wos_scene* s, const wos_solver_params* prm, const float* pts, int64_t n, int64_t index_base,
                 int64_t index_stride, float* p, float* grad, int32_t* n_est, int32_t* steps, wos_stats* stats,
                 void* stream, uint32_t flags, const SolveExtra& ex);

}  // namespace

extern "C" {

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
  HIP_TRY(hipSetDevice(s->device));
  DevCtx& c = g_ctx[s->device];
  std::lock_guard<std::mutex> lk(c.mu);
  return solve_locked(s, prm, pts, n, index_base, index_stride, p, grad, n_est, steps, stats, stream, flags,
                      SolveExtra{});
}

}  // extern "C"

namespace {

// wos_solve with the scene's and the device context's locks held
int solve_locked(wos_scene* s, const wos_solver_params* prm, const float* pts, int64_t n, int64_t index_base,
                 int64_t index_stride, float* p, float* grad, int32_t* n_est, int32_t* steps, wos_stats* stats,
                 void* stream, uint32_t flags, const SolveExtra& ex) {
  Geom& geom = *s->geom;
  const wos::HostScene& host = geom.host;
  const int dim = host.dim;
  hipStream_t st = (hipStream_t)stream;
  DevCtx& c = g_ctx[s->device];
  {
    int rc = ctx_ready(c, s->device);
    if (rc != WOS_OK) return rc;
  }

  wos::DevParams dp = dev_params(prm);
  dp.force_estimate = ex.force_estimate ? 1 : 0;
  dp.wave_prio = ex.wave_prio;
  {
    // diagonal draws + shuffle draws of the stratified samples
    const int k_needed = 2 * (2 * dp.n_pairs) * (dim - 1);
    int rc = ensure_jump(c, k_needed);
    if (rc != WOS_OK) return rc;
    dp.jump = c.d_jump;
    dp.n_jump = c.n_jump;
    dp.rej_tab = c.d_rejtab;
  }

  // LDS: the walk kernel's staged geometry; per wave, the first-ball kernel's stratified
  // samples and their shuffle partners
  WalkLayout wl;
  {
    int rc = walk_layout(s, prm, wl);
    if (rc != WOS_OK) return rc;
  }
  wos::DevScene dsc = wl.dsc;
  int geom_floats_walk = wl.geom_floats_walk;
  size_t shmem_walk = wl.shmem_walk;
  const int lhs_floats = ((2 * dp.n_pairs * (dim - 1)) + 3) & ~3;
  // the first-ball kernel stages no geometry (the point-setup kernel did the queries)
  const size_t shmem_fb = wos::kWavesPerBlockHost * wos::first_ball_wave_lds_bytes(lhs_floats, dp.n_pairs);
  size_t shmem_fb_run = shmem_fb;  // + the staged jump constants (dp.lhs_jump_n), decided below
#ifndef WOS_LHS_JUMP_STAGE
#define WOS_LHS_JUMP_STAGE 1
#endif
  // scenes beyond the LDS budget (or WOS_SCHED_GEOM_GLOBAL): geometry read from global
  // memory through L2, LDS for the per-wave scratch only
  wos::DevScene dfb = s->dev;
  // the first-ball kernel's walk-start Dirichlet distances read the cell grid too (global memory)
  dfb.dgrid = dsc.dgrid;
  dfb.dgrid_off_words = dsc.dgrid_off_words;
  for (int k = 0; k < 2; k++) {
    dfb.dgrid_n[k] = dsc.dgrid_n[k];
    dfb.dgrid_min[k] = dsc.dgrid_min[k];
    dfb.dgrid_inv[k] = dsc.dgrid_inv[k];
  }
  // (only the walk kernel stages geometry, so only its LDS decides)
  if ((prm->schedule & WOS_SCHED_GEOM_GLOBAL) || shmem_walk > kLdsDynamicMax) {
    dfb.geom_global = 1;
    dsc.geom_global = 1;
    geom_floats_walk = 0;
    shmem_walk = wos::kWavesPerBlockHost * wos::walk_wave_lds_bytes(dim);
  }
  if (shmem_fb > kLdsDynamicMax)
    return fail(WOS_E_CAPACITY, "wos_solve: nWalks exceed the LDS budget of the first-ball kernel (" +
                                    std::to_string(shmem_fb) + " bytes of stratified samples per block)");
  if (shmem_walk > kLdsDynamicMax)
    return fail(WOS_E_CAPACITY, "wos_solve: the walk kernel's per-wave scratch exceeds the LDS budget (" +
                                    std::to_string(shmem_walk) + " bytes)");

  // the shared workspace may still be in use by a solve enqueued on another stream
  HIP_TRY(ctx_order(c, st));

  const float* d_pts = pts;
  float* d_p = p;
  float* d_g = grad;
  int32_t* d_nest = n_est;
  int32_t* d_steps = steps;
  const bool dev_ptrs = (flags & WOS_PTRS_DEVICE) != 0;
  if (!dev_ptrs && n > 0) {
    int rc = ensure_workspace(c, dim, (size_t)n);
    if (rc != WOS_OK) return rc;
    HIP_TRY(hipMemcpyAsync(c.d_pts, pts, (size_t)n * dim * sizeof(float), hipMemcpyHostToDevice, st));
    d_pts = c.d_pts; d_p = c.d_p; d_g = c.d_g;
    d_nest = n_est ? c.d_nest : nullptr;
    d_steps = steps ? c.d_steps : nullptr;
  }

  // Points are solved in chunks whose walk tasks fit the task workspace.
  const int64_t wpp = (int64_t)dp.n_pairs * dp.n_anti;
  // The Neumann term (h == 0) is +0 at every step unless a ball's float members overflow
  // (mu R > 85 is the kernels' gate).  In a watertight single-sided scene every estimated
  // point and walk lies inside the boundary's bounding box, so R < its diagonal: below
  // the gate the walk kernel runs without the term's code (bit-identical results;
  // WOS_SCHED_FULL_NEUMANN keeps the full kernel).
  {
    double diag2 = 0.0;
    for (int k = 0; k < 3; k++) diag2 += (double)host.ext[k] * host.ext[k];
    const double mu_r = std::sqrt(std::max(0.0, (double)s->dev.absorption)) * std::sqrt(diag2) * 1.01;
    // (image-valued h makes the term non-zero at every step: never inert)
    dp.neumann_inert = (!dp.robust && s->dev.watertight && !s->dev.double_sided && mu_r < 80.0 && !s->dev.nimg &&
                        !(prm->schedule & WOS_SCHED_FULL_NEUMANN)) ? 1 : 0;
  }
  // Walks handed to idle sibling waves once the queue is dry (the walk kernel's SPR
  // instantiation): 2D scenes with LDS geometry (karman -4 %, its stride-8 shard -13 %,
  // config C neutral); 3D pays more for the extra live state than its short tails return
  // (profiles/r4zc_*, r4ze_*)
  dp.tail_spread = (dim == 2 && !dp.robust && !dsc.geom_global && !(prm->schedule & WOS_SCHED_NO_TAIL_SPREAD)) ? 1 : 0;
#ifdef WOS_ACCT_NOSPREAD
  dp.tail_spread = 0;  // HBM-accounting build: the walk kernel without tail spreading (no scratch)
#endif
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(n, g_max_batch_tasks.load() / wpp));
  const int64_t n_chunks = n > 0 ? (n + chunk - 1) / chunk : 0;
  int grid_fb = 0, grid_walk = 0, bpc_fb = 0, bpc_walk = 0;
  if (n > 0) {
    int rc = ensure_tasks(c, dim, chunk * wpp, chunk);
    if (rc != WOS_OK) return rc;
    HIP_TRY(wos::occupancy_blocks_per_cu(0, dim, false, shmem_fb, &bpc_fb, dp.robust != 0));
    // the stratified samples' jump constants in LDS, unless they cost the first-ball kernel a block per CU
    const int jn = std::min(2 * (2 * dp.n_pairs) * (dim - 1), wos::kLhsJumpMax);
    const size_t shmem_j = shmem_fb + (size_t)jn * 2 * sizeof(uint64_t);
    int bpc_j = 0;
    if (jn > 0 && shmem_j <= kLdsDynamicMax)
      HIP_TRY(wos::occupancy_blocks_per_cu(0, dim, false, shmem_j, &bpc_j, dp.robust != 0));
    if (WOS_LHS_JUMP_STAGE && jn > 0 && bpc_j >= bpc_fb) {
      dp.lhs_jump_n = jn;
      shmem_fb_run = shmem_j;
    }
    const int64_t fb_waves = (chunk + wos::first_ball_points_per_wave(dp.n_pairs) - 1) / wos::first_ball_points_per_wave(dp.n_pairs);
    grid_fb = (int)std::min<int64_t>((fb_waves + wos::kWavesPerBlockHost - 1) / wos::kWavesPerBlockHost,
                                     (int64_t)std::max(1, bpc_fb) * std::max(1, c.num_cus));
    // the walk instantiation launch_walks will dispatch (tail spreading has its own LDS and state)
    HIP_TRY(wos::occupancy_walk_blocks_per_cu(dim, dsc.geom_global != 0, dp, shmem_walk, &bpc_walk));
    grid_walk = std::max(1, bpc_walk) * std::max(1, c.num_cus);
  }
  const uint64_t ticket = c.next_ticket++;
  StatSlot& q = c.slot[ticket % kStatSlots];
  while ((int64_t)q.bev.size() < 4 * n_chunks) {
    hipEvent_t e = nullptr;
    HIP_TRY(hipEventCreate(&e));
    q.bev.push_back(e);
  }
  q.ticket = ticket;
  q.n_batches = n_chunks;
  q.bpc_fb = bpc_fb;
  q.bpc_walk = bpc_walk;
  q.walk_lds = (int32_t)shmem_walk;
  q.star_grid = dsc.sgrid != nullptr;
  q.geom_global = dsc.geom_global;
  q.dir_grid = dsc.dgrid != nullptr;
  HIP_TRY(hipEventRecord(q.ev0, st));
  if (n_chunks == 0) HIP_TRY(wos::launch_zero(c.d_counters, wos::kMainCounterSlots, nullptr, 0, st));
  for (int64_t k = 0; k < n_chunks; k++) {
    const int64_t b0 = k * chunk;
    hipEvent_t* ev = &q.bev[4 * k];
    const int64_t nb = std::min(chunk, n - b0);
    wos::DevTasks tk = task_view(c, dim, nb * wpp, (int32_t)wpp);
    tk.ddir = ex.ddir ? ex.ddir + b0 * dim : nullptr;
    tk.deriv = ex.deriv ? ex.deriv + b0 : nullptr;
    const int64_t bbase = index_base + b0 * index_stride;
    unsigned long long* qslot = c.d_counters + wos::kNumCounters;
    unsigned int* q_points = (unsigned int*)qslot;
    unsigned int* q_tasks = (unsigned int*)(c.d_counters + wos::kTaskQueueSlot0);
    const int walk_grid = (int)std::min<int64_t>(grid_walk, (tk.T + 63) / 64);
    // one launch zeroes the counters (first chunk: all of them; later chunks: the queues) and
    // the bucket histogram -- instead of two or three memset dispatches
    HIP_TRY(wos::launch_zero(k == 0 ? c.d_counters : qslot,
                             k == 0 ? wos::kNumCounterSlots : wos::kNumCounterSlots - wos::kNumCounters,
                             tk.hist, 2 * wos::kCostBuckets, st));
    HIP_TRY(hipEventRecord(ev[0], st));
    HIP_TRY(wos::launch_point_setup(dim, dfb, dp, d_pts + b0 * dim, nb, tk, st));
    HIP_TRY(wos::launch_lpt_order(tk, nb, st));
    HIP_TRY(wos::launch_first_balls(dim, dfb, dp, d_pts + b0 * dim, nb, bbase, index_stride, tk, c.d_counters,
                                    q_points, grid_fb, shmem_fb_run, lhs_floats, st));
    HIP_TRY(hipEventRecord(ev[1], st));
    HIP_TRY(wos::launch_walks(dim, dsc, dp, tk, bbase, index_stride, c.d_counters, q_tasks, walk_grid,
                              shmem_walk, geom_floats_walk, st));
    HIP_TRY(hipEventRecord(ev[2], st));
    HIP_TRY(wos::launch_fold(dim, dp, tk, nb, d_p + b0, d_g + b0 * dim, d_nest ? d_nest + b0 : nullptr,
                             d_steps ? d_steps + b0 : nullptr, st));
    HIP_TRY(hipEventRecord(ev[3], st));
  }
  HIP_TRY(hipEventRecord(q.ev1, st));
  HIP_TRY(hipMemcpyAsync(q.h_cnt, c.d_counters, wos::kNumCounters * sizeof(unsigned long long),
                         hipMemcpyDeviceToHost, st));
  if (!dev_ptrs && n > 0) {
    HIP_TRY(hipMemcpyAsync(p, d_p, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(grad, d_g, (size_t)n * dim * sizeof(float), hipMemcpyDeviceToHost, st));
    if (n_est) HIP_TRY(hipMemcpyAsync(n_est, d_nest, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    if (steps) HIP_TRY(hipMemcpyAsync(steps, d_steps, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipEventRecord(q.done, st));
  HIP_TRY(hipEventRecord(c.done, st));
  c.last_stream = st;
  c.inflight = true;
  if ((flags & WOS_ASYNC) && dev_ptrs) {
    if (stats) {
      *stats = wos_stats{};
      stats->ticket = ticket;
    }
    return WOS_OK;
  }
  HIP_TRY(hipStreamSynchronize(st));
  c.inflight = false;
  wos::diag_dump(dim == 2 ? "2d" : "3d");
  if (stats) {
    int rc = fill_stats(q, stats);
    if (rc != WOS_OK) return rc;
  }
  return WOS_OK;
}

}  // namespace

extern "C" {

int wos_solve_stats(wos_scene* s, uint64_t ticket, wos_stats* stats) {
  if (!s || !stats) return fail(WOS_E_INVALID, "wos_solve_stats: null scene/stats");
  const auto unknown = [&] {
    return fail(WOS_E_INVALID, "wos_solve_stats: unknown ticket (more than " + std::to_string(kStatSlots) +
                                   " solves were enqueued on this device after it)");
  };
  HIP_TRY(hipSetDevice(s->device));
  DevCtx& c = g_ctx[s->device];
  hipEvent_t done = nullptr;
  {
    // only the ticket check and the event handle under the locks: waiting here would
    // stall every other enqueuer on the device behind this solve
    std::lock_guard<std::mutex> lock(s->mu);
    std::lock_guard<std::mutex> lk(c.mu);
    StatSlot& q = c.slot[ticket % kStatSlots];
    if (ticket == 0 || q.ticket != ticket) return unknown();
    done = q.done;
    c.stat_waiters++;
  }
  const hipError_t e = hipEventSynchronize(done);
  std::lock_guard<std::mutex> lock(s->mu);
  std::lock_guard<std::mutex> lk(c.mu);
  if (--c.stat_waiters == 0) c.no_waiters.notify_all();
  if (e != hipSuccess) return fail(WOS_E_DEVICE, std::string("wos_solve_stats: ") + hipGetErrorString(e));
  StatSlot& q = c.slot[ticket % kStatSlots];
  // the slot was recycled by a later solve while we waited (its event re-recorded)
  if (q.ticket != ticket) return unknown();
  HIP_TRY(hipEventSynchronize(q.done));
  return fill_stats(q, stats);
}

void wos_default_bvc_params(wos_bvc_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  // defaults of runBoundaryValueCaching (demo.cpp:274-290)
  p->n_walks_solution = 128;
  p->n_walks_gradient = 640;
  p->boundary_cache_size = 1024;
  p->domain_cache_size = 1024;
  p->grid_res = 0;
  p->normal_offset = 5.0f * 1e-3f;
  p->radius_clamp = 1e-3f;
  p->kernel_regularization = 0.0f;
}

int wos_bvc(wos_scene* s, const wos_solver_params* prm, const wos_bvc_params* bp, float* solution, float* grad,
            float* samples, int64_t samples_capacity, int64_t* counts, wos_stats* stats) {
  if (!s || !prm || !bp || !solution || !grad) return fail(WOS_E_INVALID, "wos_bvc: null argument");
  if (bp->grid_res < 1) return fail(WOS_E_INVALID, "wos_bvc: gridRes must be >= 1");
  if (bp->n_walks_solution < 1) return fail(WOS_E_INVALID, "wos_bvc: nWalksForCachedSolutionEstimates must be >= 1");
  if (bp->boundary_cache_size < 0 || bp->domain_cache_size < 0) return fail(WOS_E_INVALID, "wos_bvc: negative cache size");
  if (prm->max_walk_length < 0) return fail(WOS_E_INVALID, "wos_bvc: maxWalkLength must be >= 0");
  {
    // both extents 0: the scene's bounding box; else both finite and > 0 (and a finite corner)
    const float* gb = bp->grid_box;
    const bool unset = gb[2] == 0.0f && gb[3] == 0.0f;
    const bool valid = std::isfinite(gb[0]) && std::isfinite(gb[1]) && std::isfinite(gb[2]) && std::isfinite(gb[3]) &&
                       gb[2] > 0.0f && gb[3] > 0.0f;
    if (!unset && !valid)
      return fail(WOS_E_INVALID, "wos_bvc: grid_box needs both extents 0 (the scene's box) or both finite and > 0");
  }
  std::lock_guard<std::mutex> lock(s->mu);
  Geom& geom = *s->geom;
  const wos::HostScene& host = geom.host;
  if (host.dim != 2) return fail(WOS_E_INVALID, "wos_bvc: boundary value caching is 2D (the reference exports it from the 2D module only)");
  if (host.n_prims + host.n_dprims <= 0) return fail(WOS_E_INVALID, "wos_bvc: scene has no boundary");
  const bool has_dir = host.n_dprims > 0;
  if (has_dir && bp->n_walks_gradient < 1)
    return fail(WOS_E_INVALID, "wos_bvc: nWalksForCachedGradientEstimates must be >= 1");
  HIP_TRY(hipSetDevice(s->device));
  DevCtx& c = g_ctx[s->device];
  std::lock_guard<std::mutex> lk(c.mu);
  {
    int rc = ctx_ready(c, s->device);
    if (rc != WOS_OK) return rc;
  }
  hipStream_t st = nullptr;
  HIP_TRY(ctx_order(c, st));
  HIP_TRY(hipStreamSynchronize(st));

  // ---- host: boundary samples (Neumann then Dirichlet segments), domain candidates,
  // evaluation grid (over grid_box, else the scene's bounding box)
  wos::BvcSampling smp;
  std::string err;
  const float pmin[2] = {host.pmin[0], host.pmin[1]}, pmax[2] = {host.pmax[0], host.pmax[1]};
  if (!wos::bvc_generate_samples(geom.v.data(), (int)(geom.v.size() / 2), geom.ix.data(), (int)(geom.ix.size() / 2),
                                 geom.dv.data(), (int)(geom.dv.size() / 2), geom.dix.data(),
                                 (int)(geom.dix.size() / 2), pmin, pmax, geom.double_sided != 0,
                                 bp->boundary_cache_size, bp->domain_cache_size, bp->normal_offset,
                                 prm->ignore_source != 0, prm->seed, smp, err))
    return fail(WOS_E_INVALID, "wos_bvc: " + err);
  float gmin[2] = {pmin[0], pmin[1]}, gext[2] = {pmax[0] - pmin[0], pmax[1] - pmin[1]};
  if (bp->grid_box[2] > 0.0f && bp->grid_box[3] > 0.0f) {
    gmin[0] = bp->grid_box[0]; gmin[1] = bp->grid_box[1];
    gext[0] = bp->grid_box[2]; gext[1] = bp->grid_box[3];
  }
  std::vector<float> ept;
  wos::bvc_evaluation_grid(bp->grid_res, gmin, gext, ept);
  const int64_t nb = (int64_t)smp.aligned.size();
  const int64_t nd = (int64_t)(smp.dcand.size() / 2);
  const int64_t ne = (int64_t)bp->grid_res * bp->grid_res;
  // runs of consecutive boundary samples of one type (the sampler emits a cache's Neumann
  // samples before its Dirichlet ones): [begin, end), Dirichlet?
  struct Run { int64_t b0, b1; bool dir; };
  std::vector<Run> runs;
  for (int64_t i = 0; i < nb; i++) {
    const bool d = smp.dirichlet[i] != 0;
    if (runs.empty() || runs.back().dir != d || runs.back().b1 != i) runs.push_back({i, i + 1, d});
    else runs.back().b1 = i + 1;
  }
  // BoundarySampler::computeEstimates (boundary_sampler.h:154-166): a Dirichlet sample's
  // derivative is along its normal, reversed for normal-aligned samples of double-sided scenes
  std::vector<float> ddir_h(2 * nb, 0.0f);
  for (int64_t i = 0; i < nb; i++) {
    const float sg = (geom.double_sided && smp.aligned[i]) ? -1.0f : 1.0f;
    ddir_h[2 * i] = smp.bnrm[2 * i] * sg;
    ddir_h[2 * i + 1] = smp.bnrm[2 * i + 1] * sg;
  }

  // ---- device buffers (freed on every exit)
  DevBufs B;
  float *d_bpt, *d_bnrm, *d_bdd, *d_bsol, *d_bdn, *d_ddir, *d_dc, *d_dsrc, *d_ept, *d_edd, *d_end, *d_sol, *d_grad;
  int32_t *d_bnest, *d_din, *d_ein;
  uint8_t* d_al;
  HIP_TRY(B.get(&d_bpt, 2 * nb)); HIP_TRY(B.get(&d_bnrm, 2 * nb)); HIP_TRY(B.get(&d_bdd, nb));
  HIP_TRY(B.get(&d_bsol, nb)); HIP_TRY(B.get(&d_bdn, nb)); HIP_TRY(B.get(&d_ddir, 2 * nb));
  float* d_dgrad;  // the Dirichlet samples' gradient (unused output of the solve)
  HIP_TRY(B.get(&d_bnest, nb)); HIP_TRY(B.get(&d_al, nb)); HIP_TRY(B.get(&d_dgrad, 2 * nb));
  HIP_TRY(B.get(&d_dc, 2 * nd)); HIP_TRY(B.get(&d_din, nd)); HIP_TRY(B.get(&d_dsrc, nd));
  HIP_TRY(B.get(&d_ept, 2 * ne)); HIP_TRY(B.get(&d_edd, ne)); HIP_TRY(B.get(&d_end, ne)); HIP_TRY(B.get(&d_ein, ne));
  HIP_TRY(B.get(&d_sol, ne)); HIP_TRY(B.get(&d_grad, 2 * ne));
  if (nb > 0) {
    HIP_TRY(hipMemcpy(d_bpt, smp.bpt.data(), 2 * nb * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_bnrm, smp.bnrm.data(), 2 * nb * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_al, smp.aligned.data(), nb, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_ddir, ddir_h.data(), 2 * nb * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(hipMemsetAsync(d_bdn, 0, nb * sizeof(float), st));
  }
  if (nd > 0) HIP_TRY(hipMemcpy(d_dc, smp.dcand.data(), 2 * nd * sizeof(float), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(d_ept, ept.data(), 2 * ne * sizeof(float), hipMemcpyHostToDevice));

  const uint64_t ticket = c.next_ticket++;
  StatSlot& q = c.slot[ticket % kStatSlots];
  while (q.bev.size() < 4) {
    hipEvent_t e = nullptr;
    HIP_TRY(hipEventCreate(&e));
    q.bev.push_back(e);
  }
  q.ticket = ticket;
  q.n_batches = 1;
  q.bpc_fb = 0;
  q.bpc_walk = 0;
  HIP_TRY(hipEventRecord(q.ev0, st));
  HIP_TRY(hipEventRecord(q.bev[0], st));
  const wos::DevScene& sc0 = s->dev;
  HIP_TRY(wos::launch_bvc_point_info(sc0, d_bpt, nb, d_bdd, nullptr, nullptr, nullptr, st));
  HIP_TRY(wos::launch_bvc_point_info(sc0, d_dc, nd, nullptr, nullptr, d_din, d_dsrc, st));
  HIP_TRY(wos::launch_bvc_point_info(sc0, d_ept, ne, d_edd, d_end, d_ein, nullptr, st));
  // the splat's packed point list; the outputs of every other point are 0
  uint32_t *d_slist = nullptr, *d_scount = nullptr;
  HIP_TRY(B.get(&d_slist, ne)); HIP_TRY(B.get(&d_scount, 1));
  HIP_TRY(hipMemsetAsync(d_scount, 0, sizeof(uint32_t), st));
  HIP_TRY(hipMemsetAsync(d_sol, 0, ne * sizeof(float), st));
  HIP_TRY(hipMemsetAsync(d_grad, 0, 2 * ne * sizeof(float), st));
  HIP_TRY(wos::launch_bvc_splat_list(d_edd, d_end, d_ein, ne, bp->normal_offset, prm->boundary_distance_mask,
                                     geom.double_sided, d_slist, d_scount, st));
  // the cache size is known once the domain candidates' inside test is: a samples buffer
  // too small for it fails here, before the walks, with counts[] filled for a retry
  // (one host round trip: the inside test and source of the domain candidates, the
  // evaluation points' Dirichlet distances)
  std::vector<float> dsrc(nd), edd_h(has_dir ? ne : 0);
  std::vector<int32_t> din(nd);
  if (nd > 0) {
    HIP_TRY(hipMemcpyAsync(din.data(), d_din, nd * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(dsrc.data(), d_dsrc, nd * sizeof(float), hipMemcpyDeviceToHost, st));
  }
  if (has_dir) HIP_TRY(hipMemcpyAsync(edd_h.data(), d_edd, ne * sizeof(float), hipMemcpyDeviceToHost, st));
  if (nd > 0 || has_dir) HIP_TRY(hipStreamSynchronize(st));
  std::vector<uint8_t> dkeep(nd);
  int64_t nd_keep = 0;
  for (int64_t i = 0; i < nd; i++) {
    const float x = smp.dcand[2 * i], y = smp.dcand[2 * i + 1];
    // insideSolveRegion (demo.cpp:302-304): the inside test, or the bounding box if double-sided
    dkeep[i] = geom.double_sided ? (x >= pmin[0] && y >= pmin[1] && x <= pmax[0] && y <= pmax[1]) : din[i] != 0;
    nd_keep += dkeep[i];
  }
  if (samples && samples_capacity < nb + nd_keep) {
    if (counts) { counts[0] = smp.nb_main; counts[1] = smp.nb_aligned; counts[2] = nd_keep; counts[3] = nb + nd_keep; }
    HIP_TRY(hipStreamSynchronize(st));
    c.inflight = false;
    q.ticket = 0;  // the slot holds no finished solve: wos_solve_stats on it reports an unknown ticket
    return fail(WOS_E_CAPACITY, "wos_bvc: samples buffer holds " + std::to_string(samples_capacity) + " of " +
                                    std::to_string(nb + nd_keep) + " samples (counts[3])");
  }
  // evaluation points within normalOffset of the Dirichlet boundary (splatter.h:160-196)
  std::vector<int64_t> near_idx;
  std::vector<float> near_pt;
  if (has_dir) {
    for (int64_t i = 0; i < ne; i++)
      if (edd_h[i] < bp->normal_offset) {
        near_idx.push_back(i);
        near_pt.push_back(ept[2 * i]);
        near_pt.push_back(ept[2 * i + 1]);
      }
  }
  const int64_t nn = (int64_t)near_idx.size();
  float *d_npt = nullptr, *d_ndd = nullptr, *d_nsol = nullptr;
  int32_t* d_nnest = nullptr;
  HIP_TRY(B.get(&d_npt, 2 * nn)); HIP_TRY(B.get(&d_ndd, nn)); HIP_TRY(B.get(&d_nsol, nn)); HIP_TRY(B.get(&d_nnest, nn));
  if (nn > 0) {
    std::vector<float> ndd(nn);
    for (int64_t k = 0; k < nn; k++) ndd[k] = edd_h[near_idx[k]];
    HIP_TRY(hipMemcpy(d_npt, near_pt.data(), 2 * nn * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_ndd, ndd.data(), nn * sizeof(float), hipMemcpyHostToDevice));
  }

  // ---- the cache (splatter order): boundary samples (value = the solution, filled in on the
  // device once their walks are done; the Neumann value 0: pde.neumann, scene.h:176-181;
  // Dirichlet samples also their normal derivative), then the domain samples inside the
  // solve region (value = the source)
  std::vector<float> recs;
  recs.reserve((size_t)(nb + nd_keep) * wos::kBvcRec);
  for (int64_t i = 0; i < nb; i++) {
    const bool al = smp.aligned[i] != 0, dir = smp.dirichlet[i] != 0;
    const int kind = dir ? (al ? wos::kBvcDirichletAligned : wos::kBvcDirichlet) : (al ? wos::kBvcAligned : wos::kBvcBoundary);
    const float r[wos::kBvcRec] = {smp.bpt[2 * i], smp.bpt[2 * i + 1], smp.bnrm[2 * i], smp.bnrm[2 * i + 1],
                                   al ? smp.pdf_aligned : smp.pdf_main, 0.0f, 0.0f, (float)kind};
    recs.insert(recs.end(), r, r + wos::kBvcRec);
  }
  for (int64_t i = 0; i < nd; i++) {
    if (!dkeep[i]) continue;
    const float r[wos::kBvcRec] = {smp.dcand[2 * i], smp.dcand[2 * i + 1], 0.0f, 0.0f, smp.pdf_domain, dsrc[i], 0.0f,
                                   (float)wos::kBvcDomain};
    recs.insert(recs.end(), r, r + wos::kBvcRec);
  }
  const int64_t nd_kept = nd_keep;
  const int64_t nrec = nb + nd_kept;
  float *d_recs = nullptr, *d_state = nullptr;
  HIP_TRY(B.get(&d_recs, (size_t)nrec * wos::kBvcRec));
  HIP_TRY(B.get(&d_state, (size_t)18 * ne));
  if (nrec > 0) HIP_TRY(hipMemcpy(d_recs, recs.data(), recs.size() * sizeof(float), hipMemcpyHostToDevice));

  // ---- Three independent walk sets, on three streams (their tails overlap the others' bulk):
  //   bvc_dir            the Dirichlet samples' estimateSolutionAndGradient along the normal
  //                      (nWalksForCachedGradientEstimates, keyed by the sample index) on the
  //                      solve pipeline, solution and derivative unmasked;
  //   side[0]            estimateSolution walks (walk_on_stars.h:353-464) of the Neumann
  //                      boundary samples (nWalksForCachedSolutionEstimates, seed tag 6) and
  //                      the finite-difference Dirichlet samples (nWalksForCachedGradient-
  //                      Estimates, tag 8);
  //   side[1]            estimateSolution walks of the evaluation points near the Dirichlet
  //                      boundary (nWalksForCachedSolutionEstimates, tag 7, keyed by rank).
  // Every allocation (layout grids, jump table, workspaces) happens before the first launch:
  // hipFree / hipMalloc would serialise the streams.
  WalkLayout wl;
  wos_solver_params wp0 = *prm;
  {
    int rc = walk_layout(s, &wp0, wl);
    if (rc != WOS_OK) return rc;
  }
  wos::DevScene dsc = wl.dsc;
  if ((prm->schedule & WOS_SCHED_GEOM_GLOBAL) || wl.shmem_walk > kLdsDynamicMax) {
    dsc.geom_global = 1;
    wl.geom_floats_walk = 0;
    wl.shmem_walk = wos::kWavesPerBlockHost * wos::walk_wave_lds_bytes(2);
  }
  const bool dir_solve = has_dir && !bp->use_finite_differences;
  wos_solver_params gp = *prm;
  gp.n_walks = bp->n_walks_gradient;
  gp.boundary_distance_mask = 0.0f;
  {
    // the Dirichlet solves' stratified-sample draws (solve_locked) bound the table from above
    int rc = ensure_jump(c, std::max(4096, 4 * std::max(1, bp->n_walks_gradient)));
    if (rc != WOS_OK) return rc;
  }
  int64_t side_tasks[kSideWs] = {0, 0}, side_points[kSideWs] = {0, 0};
  const int64_t max_batch = g_max_batch_tasks.load();
  for (const Run& r : runs) {
    const int64_t m = r.b1 - r.b0;
    if (!r.dir || bp->use_finite_differences) {
      const int64_t w = r.dir ? bp->n_walks_gradient : bp->n_walks_solution;
      if (m * w > max_batch) return fail(WOS_E_CAPACITY, "wos_bvc: samples x nWalks exceed one task batch");
      side_tasks[0] = std::max(side_tasks[0], m * w);
      side_points[0] = std::max(side_points[0], m);
    } else if (dir_solve) {
      const int64_t wpp = gp.disable_gradient_antithetic_variates ? gp.n_walks : 2 * std::max(1, gp.n_walks / 2);
      const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(m, max_batch / wpp));
      int rc = ensure_tasks(c, 2, chunk * wpp, chunk);
      if (rc != WOS_OK) return rc;
    }
  }
  if (nn * bp->n_walks_solution > max_batch)
    return fail(WOS_E_CAPACITY, "wos_bvc: samples x nWalks exceed one task batch");
  side_tasks[1] = nn * bp->n_walks_solution;
  side_points[1] = nn;
  for (int k = 0; k < kSideWs; k++) {
    TaskWs& w = c.side[k];
    int rc = side_ready(w, bvc_priority(k == 0));
    if (rc == WOS_OK) rc = ensure_tasks_in(w.tasks, w.task_cap, w.pstate, w.pstate_cap, 2, side_tasks[k], side_points[k]);
    if (rc != WOS_OK) return rc;
  }
  if (!c.bvc_dir) HIP_TRY(hipStreamCreateWithPriority(&c.bvc_dir, hipStreamNonBlocking, bvc_priority(true)));
  if (!c.bvc_dir_done) HIP_TRY(hipEventCreateWithFlags(&c.bvc_dir_done, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(q.bev[1], st));
  HIP_TRY(hipStreamWaitEvent(c.bvc_dir, q.bev[1], 0));
  for (TaskWs& w : c.side) {
    HIP_TRY(hipStreamWaitEvent(w.stream, q.bev[1], 0));
    HIP_TRY(wos::launch_zero(w.counters, wos::kNumCounterSlots, nullptr, 0, w.stream));
  }

  std::vector<uint64_t> dtickets;
  if (dir_solve) {
    SolveExtra ex;
    ex.force_estimate = true;
    ex.wave_prio = 2;
    for (const Run& r : runs) {
      if (!r.dir) continue;
      ex.ddir = d_ddir + 2 * r.b0;
      ex.deriv = d_bdn + r.b0;
      wos_stats rs{};
      int rc = solve_locked(s, &gp, d_bpt + 2 * r.b0, r.b1 - r.b0, r.b0, 1, d_bsol + r.b0, d_dgrad, d_bnest + r.b0,
                            nullptr, &rs, c.bvc_dir, WOS_PTRS_DEVICE | WOS_ASYNC, ex);
      if (rc != WOS_OK) return rc;
      dtickets.push_back(rs.ticket);
    }
  }
  HIP_TRY(hipEventRecord(c.bvc_dir_done, c.bvc_dir));

  bool first_walk[kSideWs] = {true, true};
  auto walks = [&](int k, const float* pts_d, const float* nrm_d, const uint8_t* al_d, const float* dd_d, int64_t np_,
                   int64_t base, int n_walks, int on_neumann, uint32_t tag, float* sol_d, int32_t* nest_d) -> int {
    if (np_ <= 0) return WOS_OK;
    TaskWs& w = c.side[k];
    wos_solver_params wp = *prm;
    wp.n_walks = n_walks;
    wp.disable_gradient_antithetic_variates = 1;  // one walk per task, no pairs
    wos::DevParams dp = dev_params(&wp);
    dp.jump = c.d_jump;
    dp.n_jump = c.n_jump;
    dp.rej_tab = c.d_rejtab;
    // the Neumann samples' harmonic walks run longest (reflecting, up to maxWalkLength): top
    // issue priority; the near-boundary walks feed nothing downstream: none
    dp.wave_prio = k == 0 ? 3 : 0;
    const int64_t wpp = n_walks;
    wos::DevTasks tk = task_view_in(w.tasks, w.pstate, w.pstate_cap, 2, np_ * wpp, (int32_t)wpp);
    tk.n0 = tk.bdir;
    tk.r0 = tk.first;
    tk.sflags = reinterpret_cast<uint32_t*>(tk.sdir);
    // the walk queue's counters start at 0 for every launch
    if (!first_walk[k])
      HIP_TRY(wos::launch_zero(w.counters + wos::kNumCounters, wos::kNumCounterSlots - wos::kNumCounters, nullptr, 0,
                               w.stream));
    first_walk[k] = false;
    HIP_TRY(wos::launch_bvc_start(dsc, dp, pts_d, nrm_d, al_d, dd_d, np_, tk, on_neumann, tag, w.stream));
    int bpc = 0;
    HIP_TRY(wos::occupancy_walk_bstart(dsc.geom_global != 0, wl.shmem_walk, &bpc, dp.robust != 0));
    const int grid = (int)std::min<int64_t>((int64_t)std::max(1, bpc) * std::max(1, c.num_cus), (tk.T + 63) / 64);
    unsigned int* q_tasks = (unsigned int*)(w.counters + wos::kTaskQueueSlot0);
    HIP_TRY(wos::launch_walks_bstart(dsc, dp, tk, base, 1, w.counters, q_tasks, grid, wl.shmem_walk,
                                     wl.geom_floats_walk, w.stream));
    HIP_TRY(wos::launch_bvc_fold(tk, np_, sol_d, nest_d, w.stream));
    q.bpc_walk = bpc;
    return WOS_OK;
  };
  for (const Run& r : runs) {
    const int64_t m = r.b1 - r.b0;
    int rc = WOS_OK;
    if (!r.dir)
      rc = walks(0, d_bpt + 2 * r.b0, d_bnrm + 2 * r.b0, d_al + r.b0, d_bdd + r.b0, m, r.b0, bp->n_walks_solution, 1,
                 6u, d_bsol + r.b0, d_bnest + r.b0);
    else if (bp->use_finite_differences)
      rc = walks(0, d_bpt + 2 * r.b0, d_bnrm + 2 * r.b0, d_al + r.b0, d_bdd + r.b0, m, r.b0, bp->n_walks_gradient, 0,
                 8u, d_bsol + r.b0, d_bnest + r.b0);
    if (rc != WOS_OK) return rc;
    if (r.dir && bp->use_finite_differences)
      HIP_TRY(wos::launch_bvc_fd(s->dev, d_bpt + 2 * r.b0, d_bsol + r.b0, m, d_bdn + r.b0, c.side[0].stream));
  }
  {
    int rc = walks(1, d_npt, nullptr, nullptr, d_ndd, nn, 0, bp->n_walks_solution, 0, 7u, d_nsol, d_nnest);
    if (rc != WOS_OK) return rc;
  }
  q.walk_lds = (int32_t)wl.shmem_walk;
  q.star_grid = dsc.sgrid != nullptr;
  q.geom_global = dsc.geom_global;
  q.dir_grid = dsc.dgrid != nullptr;

  // ---- the splat in two launches over the cache order: the records whose values side[0]
  // estimates (the Neumann samples before the first Dirichlet sample of the solve; all the
  // boundary samples without one) as soon as side[0]'s walks are done, beside the
  // Dirichlet solve; then the rest on the call's stream, continuing the same statistics
  int64_t p1 = nb;
  if (dir_solve)
    for (int64_t i = 0; i < nb; i++)
      if (smp.dirichlet[i]) { p1 = i; break; }
  const float ab = s->dev.absorption;
  const bool part1 = p1 > 0, part1_last = p1 == nrec;
  if (part1) {
    HIP_TRY(wos::launch_bvc_fill(d_recs, 0, p1, d_bsol, d_bdn, s->dev, prm->ignore_neumann, c.side[0].stream));
    HIP_TRY(wos::launch_bvc_splat(d_recs, 0, (int)p1, 1, part1_last ? 1 : 0, d_state, d_slist, d_scount, d_ept, ne,
                                  ab, bp->radius_clamp, bp->kernel_regularization, d_sol, d_grad, c.side[0].stream));
  }
  for (TaskWs& w : c.side) HIP_TRY(hipEventRecord(w.done, w.stream));
  HIP_TRY(hipStreamWaitEvent(st, c.bvc_dir_done, 0));
  HIP_TRY(hipStreamWaitEvent(st, c.side[0].done, 0));
  HIP_TRY(hipEventRecord(q.bev[2], st));
  if (!(part1 && part1_last)) {
    HIP_TRY(wos::launch_bvc_fill(d_recs, p1, nb, d_bsol, d_bdn, s->dev, prm->ignore_neumann, st));
    HIP_TRY(wos::launch_bvc_splat(d_recs, part1 ? (int)p1 : 0, (int)nrec, part1 ? 0 : 1, 1, d_state, d_slist,
                                  d_scount, d_ept, ne, ab, bp->radius_clamp, bp->kernel_regularization, d_sol,
                                  d_grad, st));
  }
  std::vector<float> nsol(nn);
  HIP_TRY(hipStreamWaitEvent(st, c.side[1].done, 0));
  HIP_TRY(hipEventRecord(q.bev[3], st));
  HIP_TRY(hipEventRecord(q.ev1, st));
  // the walk counters of both side workspaces (summed below); the Dirichlet solves' own
  // counters are in their stat slots
  std::vector<unsigned long long> cnt1(wos::kNumCounters);
  HIP_TRY(hipMemcpyAsync(q.h_cnt, c.side[0].counters, wos::kNumCounters * sizeof(unsigned long long),
                         hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(cnt1.data(), c.side[1].counters, wos::kNumCounters * sizeof(unsigned long long),
                         hipMemcpyDeviceToHost, st));
  if (nn > 0) HIP_TRY(hipMemcpyAsync(nsol.data(), d_nsol, nn * sizeof(float), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(solution, d_sol, ne * sizeof(float), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(grad, d_grad, 2 * ne * sizeof(float), hipMemcpyDeviceToHost, st));
  if (samples && nrec > 0)  // the cache with its estimated values
    HIP_TRY(hipMemcpyAsync(recs.data(), d_recs, recs.size() * sizeof(float), hipMemcpyDeviceToHost, st));
  std::vector<float> end_h(nn > 0 ? ne : 0);
  std::vector<int32_t> ein_h(nn > 0 ? ne : 0);
  if (nn > 0) {
    HIP_TRY(hipMemcpyAsync(end_h.data(), d_end, ne * sizeof(float), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(ein_h.data(), d_ein, ne * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipEventRecord(q.done, st));
  HIP_TRY(hipStreamSynchronize(st));
  c.inflight = false;
  for (int k = 0; k < wos::kNumCounters; k++) q.h_cnt[k] += cnt1[k];
  wos::diag_dump("bvc");  // DIAG builds only
  wos::diag_dump_bstart("bvc-bstart");
  // the pointwise estimates near the Dirichlet boundary replace the (unsplatted) points'
  // statistics: solution = the estimate, gradient 0 (evalPt.reset, splatter.h:186-192),
  // then saveEvaluationGrid's mask (grid.h:404-408)
  for (int64_t k = 0; k < nn; k++) {
    const int64_t i = near_idx[k];
    const bool masked = (ein_h[i] == 0 && !geom.double_sided) ||
                        std::min(std::fabs(edd_h[i]), std::fabs(end_h[i])) < prm->boundary_distance_mask;
    solution[i] = masked ? 0.0f : nsol[k];
  }
  if (counts) { counts[0] = smp.nb_main; counts[1] = smp.nb_aligned; counts[2] = nd_kept; counts[3] = nrec; }
  if (stats) {
    int rc = fill_stats(q, stats);
    if (rc != WOS_OK) return rc;
    stats->points_estimated = (uint64_t)nb;
    // the Dirichlet solves ran inside this call's span: their counters, not their times
    for (uint64_t t : dtickets) {
      const StatSlot& dq = c.slot[t % kStatSlots];
      if (dq.ticket != t) continue;
      wos_stats rs{};
      rc = fill_stats(dq, &rs);
      if (rc != WOS_OK) return rc;
      stats->walk_steps += rs.walk_steps; stats->wasted_steps += rs.wasted_steps;
      stats->walks_recorded += rs.walks_recorded; stats->walks_escaped += rs.walks_escaped;
      stats->walks_max_length += rs.walks_max_length; stats->walks_rr += rs.walks_rr;
      stats->walks_dirichlet += rs.walks_dirichlet; stats->rejection_iters += rs.rejection_iters;
    }
  }
  if (samples && nrec > 0) {
    if (samples_capacity < nrec)
      return fail(WOS_E_CAPACITY, "wos_bvc: samples buffer holds " + std::to_string(samples_capacity) + " of " +
                                      std::to_string(nrec) + " samples (counts[3])");
    std::memcpy(samples, recs.data(), recs.size() * sizeof(float));
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
