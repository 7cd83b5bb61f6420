/*
 * wos.h -- C ABI of the MI355X walk-on-stars pressure-projection engine.
 *
 * This is the drop-in boundary for the one hot path of
 * Pranav-Jain/Neural-Monte-Carlo-Fluid-Simulation: the zombie / zombie3d WoSt
 * estimator behind the pybind11 module `zombie_bindings`
 * (bindings/zombie/demo/demo.cpp:393-401, bindings/zombie3d/demo/demo.cpp:119-125).
 * Plain pointers and sizes only; no torch / STL types cross this boundary.
 *
 * Every function returns WOS_OK (0) or a negative WOS_E* status; the message of
 * the last failure on the calling thread is available from wos_last_error()
 * (the reference aborts the interpreter instead: config.h:8-11, scene.h:106-109).
 */
#ifndef WOS_H
#define WOS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WOS_ABI_VERSION 10

enum {
    WOS_OK = 0,
    WOS_E_INVALID = -1,     /* bad argument / config value            */
    WOS_E_IO = -2,          /* file missing / unreadable               */
    WOS_E_DEVICE = -3,      /* HIP runtime error                       */
    WOS_E_CAPACITY = -4,    /* scene too large for the LDS-staged path */
    WOS_E_NOMEM = -5
};

/* flags for wos_solve */
#define WOS_PTRS_DEVICE 0x1u   /* pts/p/grad/n_est/steps are device pointers on the scene's device */
#define WOS_ASYNC       0x2u   /* with WOS_PTRS_DEVICE: enqueue on `stream` and return; only
                                  stats->ticket is filled (read the rest with wos_solve_stats) */

/* A boundary mesh: 2D line segments (dim=2) or 3D triangles (dim=3). */
typedef struct wos_mesh {
    int32_t dim;
    int32_t n_vertices;
    int32_t n_prims;
    float *vertices;          /* n_vertices * dim */
    int32_t *prims;           /* n_prims * dim (0-based vertex indices) */
} wos_mesh;

/* Replaces Scene::loadOBJ (bindings/zombie/demo/scene.h:104-145, 2D `v`/`l`
 * lines, flipOrientation swaps segment ends, normalizeDomain recentres) and
 * zombie::loadSurfaceMesh<3> (include/zombie/utils/fcpw_scene_loader.h:47-73).
 * Arrays are malloc'd; release with wos_mesh_free. */
int wos_load_obj(const char *path, int32_t dim, int32_t flip_orientation,
                 int32_t normalize, wos_mesh *out);
void wos_mesh_free(wos_mesh *mesh);

typedef struct wos_scene_desc {
    int32_t dim;                     /* 2 or 3 */
    const float *vertices;           /* Neumann boundary (the reference's OBJ "boundary") */
    const int32_t *prims;
    int32_t n_vertices, n_prims;
    const float *dvertices;          /* optional Dirichlet boundary (empty in the reference) */
    const int32_t *dprims;
    int32_t n_dvertices, n_dprims;
    float dirichlet_value;           /* constant g on the Dirichlet boundary */
    float absorption;                /* scene.absorptionCoeff (lambda) */
    int32_t is_watertight;           /* scene.isWatertight */
    int32_t is_double_sided;         /* scene.isDoubleSided */
    const float *source;             /* -div(u) grid: 2D [H][W] (rows ~ y); 3D [X][Y][Z] */
    int32_t source_dims[3];
    int32_t source_on_device;        /* source is a device pointer (copied d2d) */
    /* optional image-valued Dirichlet data (2D, ABI 8), replacing dirichlet_value: g at a walk's
       projection x onto the Dirichlet boundary is Image::get((x - x0) / ex, (y - y0) / ey)
       (setTerminalContribution walk_on_stars.h:331-351 -> projectToDirichlet
       fcpw_scene_loader.h:345-364 -> the upstream demo's pde.dirichlet, scene.h:202-207 commented
       in the fork: x0, y0 = bbox.pMin, ex = ey = bbox.extent().maxCoeff(); image.h:53-58) */
    const float *dirichlet_image;    /* [H][W] row-major, row ~ y; NULL: constant dirichlet_value */
    int32_t dirichlet_image_dims[2]; /* H, W */
    float dirichlet_image_box[4];    /* x0, y0, ex, ey: the rectangle the image covers */
    int32_t dirichlet_image_on_device;
    /* optional image-valued Neumann data h (2D, ABI 9): pde.neumann at a boundary sample y is
       Image::get((y - x0) / ex, (y - y0) / ey) (the upstream demo's pde.neumann, scene.h:175-181
       commented in the fork: uv = (x - bbox.pMin) / bbox.extent(); image.h:53-58).  It enters the
       walk's Neumann term throughput * alpha * G * h / pdf at every step (walk_on_stars.h:212-260)
       and a BVC Neumann sample's normal derivative (boundary_sampler.h:126-133).  NULL: h = 0,
       the reference's pde.neumann (scene.h:176-181, scene_3d.h:108-111) */
    const float *neumann_image;      /* [H][W] row-major, row ~ y */
    int32_t neumann_image_dims[2];   /* H, W */
    float neumann_image_box[4];      /* x0, y0, ex, ey */
    int32_t neumann_image_on_device;
} wos_scene_desc;

typedef struct wos_scene wos_scene;

/* Replaces Scene::Scene(json, mat) (scene.h:54-77) / Scene(json, mat3d)
 * (scene_3d.h:22-40): normals, silhouettes (fcpw.inl:224-353, sbvh.inl:313-436),
 * padded bbox, then uploads geometry + source to `device`. */
int wos_scene_create(const wos_scene_desc *desc, int32_t device, wos_scene **out);
int wos_scene_destroy(wos_scene *scene);

/* Replaces the source grid (-div u) of an existing scene.  The reference rebuilds
 * the whole scene every projection to change only this (model_split.py:185-191,
 * Scene(sceneConfig, div) -> scene.h:54-77 / scene_3d.h:22-40); here geometry
 * stays resident.  dims as wos_scene_desc.source_dims; `on_device`: `source` is
 * a device pointer on the scene's device.  The copy is ordered on `stream`
 * (hipStream_t, NULL = null stream) after any solve still running on another
 * stream. */
int wos_scene_set_source(wos_scene *scene, const float *source, const int32_t *dims,
                         int32_t on_device, void *stream);

/* Scenes share a per-device solve workspace and a cache of prepared geometries
 * (keyed by content), so the reference's per-step Scene(...) costs neither a
 * workspace allocation nor a re-preparation.  This releases both for `device`
 * (-1: every device); live scenes stay valid and the next solve reallocates. */
int wos_release_caches(int32_t device);

/* Walk tasks per batch (ABI 10).  A solve runs its points in batches of at most this many walk
 * tasks (the per-device workspace holds one batch: 60 B per task); default 2^28 = 16 GB at most,
 * sized for a 288 GB MI355X (fewer batches, fewer ramp-downs of the persistent kernels).  A
 * caller that shares the GPU with other work can cap it.  max_tasks <= 0: the default; else
 * clamped to [2^16, 2^30].  Returns the previous value.  Results do not depend on it. */
int64_t wos_set_max_batch_tasks(int64_t max_tasks);

typedef struct wos_scene_info {
    int32_t dim, n_prims, n_silhouettes, n_dprims, device;
    float bbox_min[3], bbox_max[3];
} wos_scene_info;
int wos_scene_get_info(const wos_scene *scene, wos_scene_info *info);

/* Solver / output settings: the keys runWalkOnStars_sampled reads
 * (demo.cpp:121-137) plus output.boundaryDistanceMask (grid.h:159) and the
 * counter-based RNG key that replaces the clock seeds. */
typedef struct wos_solver_params {
    int32_t n_walks;                        /* nWalks (128) */
    int32_t max_walk_length;                /* maxWalkLength (1024) */
    int32_t steps_before_tikhonov;          /* setpsBeforeApplyingTikhonov (maxWalkLength) */
    int32_t steps_before_maximal_spheres;   /* setpsBeforeUsingMaximalSpheres (maxWalkLength) */
    float epsilon_shell;                    /* epsilonShell (1e-3) */
    float min_star_radius;                  /* minStarRadius (1e-3) */
    float silhouette_precision;             /* silhouettePrecision (1e-3) */
    float russian_roulette_threshold;       /* russianRouletteThreshold (0) */
    float boundary_distance_mask;           /* output.boundaryDistanceMask (0) */
    int32_t disable_gradient_control_variates;
    int32_t disable_gradient_antithetic_variates;
    int32_t use_cosine_sampling;            /* useCosineSamplingForDirectionalDerivatives */
    int32_t ignore_dirichlet;
    int32_t ignore_neumann;
    int32_t ignore_source;
    uint64_t seed;                          /* RNG key */
    int32_t robust_float;                   /* 0 (default): the reference's float Bessel members, which
                                               overflow to NaN for 2D Yukawa balls with mu R > ~92
                                               (distributions.h:585-587,695); 1: balls with mu R > 80 use
                                               exponentially scaled Bessels and ratios (finite, correct) --
                                               identical to mode 0 on every ball with mu R <= 80 */
    uint32_t schedule;                      /* WOS_SCHED_* bits: how the solve is scheduled on the GPU,
                                               never what it computes (results are bit-identical) */
} wos_solver_params;

/* wos_solver_params.schedule (no reference analogue; 0 = the engine's choice) */
#define WOS_SCHED_GEOM_GLOBAL   0x1u  /* read the geometry records through L2 even when they fit LDS */
#define WOS_SCHED_FULL_NEUMANN  0x2u  /* keep the walk kernel's Neumann term even when it is provably +0 */
#define WOS_SCHED_NO_STAR_GRID  0x4u  /* no star-radius cell grid: the cooperative group scan alone */
#define WOS_SCHED_NO_DIR_GRID   0x8u  /* no Dirichlet-distance cell grid (2D): the culled scans alone */
#define WOS_SCHED_NO_TAIL_SPREAD 0x10u /* no hand-over of walks to idle sibling waves once the queue is dry */
#define WOS_SCHED_NO_GRID_SPREAD 0x20u /* reserved, no effect: grid-wide hand-over was measured slower than the
                                          in-workgroup one and removed (ABI 9 keeps the bit so callers still build) */

void wos_default_params(wos_solver_params *p);

typedef struct wos_stats {
    uint64_t walk_steps;        /* ball steps of recorded walks (first ball + walk() iterations) */
    uint64_t wasted_steps;      /* ball steps of dropped walks (escaped / over max length) */
    uint64_t walks_recorded;
    uint64_t walks_escaped;
    uint64_t walks_max_length;
    uint64_t walks_rr;
    uint64_t walks_dirichlet;
    uint64_t points_estimated;
    uint64_t rejection_iters;
    double kernel_ms;           /* device time of the whole solve: all batches, all kernels (HIP events) */
    double first_ball_ms;       /* of which: point setup + first balls (wos_first_ball_kernel) */
    double walk_ms;             /* of which: the walks (wos_walk_kernel) -- the dominant kernel */
    double fold_ms;             /* of which: statistics + masked outputs (wos_fold_kernel) */
    uint64_t walk_launches;     /* walk-kernel launches (one per batch of points) */
    int32_t first_ball_blocks_per_cu;  /* occupancy of the launches (256-thread workgroups per CU) */
    int32_t walk_blocks_per_cu;
    int32_t walk_lds_bytes;     /* dynamic LDS per walk-kernel workgroup */
    int32_t star_grid;          /* 1: the star-radius cell grid was used */
    int32_t geom_global;        /* 1: geometry read from global memory (too large for LDS) */
    int32_t dir_grid;                       /* the walk kernel used the Dirichlet-distance cell grid (2D) */
    uint64_t ticket;            /* id of this solve on its device (for wos_solve_stats) */
} wos_stats;

/* Replaces runWalkOnStars_sampled (demo.cpp:119-205) / runWalkOnStars_3d
 * (zombie3d/demo/demo.cpp:15-116) for n query points pts[n*dim]:
 *   p[n]          masked pressure    (grid.h:155-179)
 *   grad[n*dim]   masked gradient    (grid.h:207-237)
 *   n_est[n]      recorded walks per point (optional, may be NULL)
 *   steps[n]      ball steps per point incl. wasted (optional, may be NULL)
 * The RNG of point i is keyed by the global index index_base + i*index_stride,
 * so sharding the points across GPUs does not change any result.
 * `stream` is a hipStream_t (NULL = the device's null stream). */
int wos_solve(wos_scene *scene, const wos_solver_params *params,
              const float *pts, int64_t n, int64_t index_base, int64_t index_stride,
              float *p, float *grad, int32_t *n_est, int32_t *steps,
              wos_stats *stats, void *stream, uint32_t flags);

/* Boundary value caching: the reference's `bvc(scene, solver, output)`
 * (bindings/zombie/demo/demo.cpp:265-363, exported at :396), replaced here.
 * Solver keys as for wos_solve plus the BVC keys demo.cpp:269-290 reads. */
typedef struct wos_bvc_params {
    int32_t n_walks_solution;       /* nWalksForCachedSolutionEstimates (128) */
    int32_t n_walks_gradient;       /* nWalksForCachedGradientEstimates (640): Dirichlet samples only */
    int32_t boundary_cache_size;    /* boundaryCacheSize (1024) */
    int32_t domain_cache_size;      /* domainCacheSize (1024) */
    int32_t grid_res;               /* output.gridRes (required) */
    int32_t use_finite_differences; /* useFiniteDifferencesForBoundaryDerivatives (Dirichlet samples only) */
    float normal_offset;            /* normalOffsetForCachedDirichletSamples (5 epsilonShell) */
    float radius_clamp;             /* radiusClampForKernels (1e-3) */
    float kernel_regularization;    /* regularizationForKernels (0) */
    float grid_box[4];              /* evaluation grid x0, y0, ex, ey (ABI 8; extent 0: the scene's
                                       bounding box -- createEvaluationGrid(bbox.pMin, bbox.pMax),
                                       demo.cpp:311, grid.h:352-368) */
} wos_bvc_params;

void wos_default_bvc_params(wos_bvc_params *p);

/* runBoundaryValueCaching (demo.cpp:265-363) on a 2D scene, blocking, host buffers:
 *   solution[g*g], grad[g*g*2]  the evaluation grid (point (i, j) at index i*g + j,
 *                               x = i/g * extent + box min over grid_box, grid.h:352-368),
 *                               masked as saveEvaluationGrid does (grid.h:393-409);
 *   samples[k*8] (optional)     the cached samples [x y nx ny pdf value dn/dn kind], kind 0
 *                               Neumann boundary, 1 Neumann normal-aligned, 2 domain (value =
 *                               the source), 3 Dirichlet boundary, 4 Dirichlet normal-aligned
 *                               (the sample normalOffset inside the boundary, value = the
 *                               estimated solution, dn/dn its estimated normal derivative),
 *                               if samples_capacity holds them (else WOS_E_CAPACITY);
 *   counts[4] (optional)        boundary, normal-aligned, domain samples, total.
 * Boundary samples cover the Neumann and the Dirichlet segments (boundary_sampler.h:87-412);
 * evaluation points within normalOffset of the Dirichlet boundary take a pointwise
 * estimateSolution (splatter.h:160-196).  3D scenes return WOS_E_INVALID (zombie3d exports no
 * bvc).  The three walk sets (Dirichlet samples, Neumann samples, near-boundary points) run
 * on three streams at once; stats: kernel_ms the whole call, first_ball_ms the point
 * queries, walk_ms until the cache is complete, fold_ms the splat and the near-boundary
 * walks still running beside it. */
int wos_bvc(wos_scene *scene, const wos_solver_params *params, const wos_bvc_params *bvc,
            float *solution, float *grad, float *samples, int64_t samples_capacity, int64_t *counts,
            wos_stats *stats);

/* Statistics of an earlier solve on the scene's device, by stats->ticket: waits for
 * that solve to finish, then fills *stats.  A time-stepper can enqueue the projection
 * (WOS_ASYNC) and keep queueing device work behind it, as the reference's caller does
 * with its training loop after wost() (model_split.py:272-283).  The last 16 solves
 * per device are held; older tickets return WOS_E_INVALID.  No reference analogue. */
int wos_solve_stats(wos_scene *scene, uint64_t ticket, wos_stats *stats);

/* Device self-test of the deterministic math used by the kernel (for the
 * GPU-vs-oracle parity tests): which = 0 exp, 1 log, 2 sin, 3 cos, 4 atan,
 * 5 sqrt, 6 bessi0, 7 bessi1, 8 bessk0, 9 bessk1 (double); 10 expf, 11 logf,
 * 12 sinf, 13 cosf, 14 cbrtf (float in, float out widened to double); 15 sqrtf,
 * 16 i0_fast, 17 k0_fast, 18-23 the fused double evaluator, 24/25 I0/K0 of the fused
 * float pair of the rejection fast path. */
int wos_selftest_math(int32_t which, const double *x, double *out, int64_t n, int32_t device);

const char *wos_last_error(void);
int32_t wos_abi_version(void);
int32_t wos_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* WOS_H */
