/*
 * oracle/wos_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the zombie walk-on-stars (WoSt) pressure solve that
 * Pranav-Jain/Neural-Monte-Carlo-Fluid-Simulation calls through
 * zombie_bindings.wost(...) (bindings/zombie/demo/demo.cpp:119-205,
 * bindings/zombie3d/demo/demo.cpp:15-116).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as the
 * checker / CPU baseline -- never as the product path.
 *
 * Parity status: the reference path cannot be compiled or run here (denied,
 * SURVEY.md §8c) and ships no golden vectors for this path, so this oracle is
 * pinned by analytic known-answer tests (screened-Poisson box problems) and by
 * internal consistency (det vs libm math modes); see DESIGN.md "Oracle".
 */
#ifndef WOS_ORACLE_H
#define WOS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_scene_desc {
    int32_t dim;              /* 2 (line segments) or 3 (triangles) */
    int32_t n_vertices;
    int32_t n_prims;
    const float *vertices;    /* n_vertices * dim */
    const int32_t *prims;     /* n_prims * dim vertex indices */
    /* optional Dirichlet boundary (absent in every shipped scene) */
    int32_t n_dvertices;
    int32_t n_dprims;
    const float *dvertices;
    const int32_t *dprims;
    float dirichlet_value;    /* constant g on the Dirichlet boundary */
    float absorption;         /* lambda (scene.absorptionCoeff) */
    int32_t is_watertight;
    int32_t is_double_sided;
    /* source grid: 2D (h=dims[0] rows ~ y, w=dims[1] cols ~ x); 3D (X,Y,Z) */
    const float *source;
    int32_t source_dims[3];
    /* optional image-valued Dirichlet data g (2D): [h][w] row-major, row ~ y, covering the
       rectangle dirichlet_image_box = {x0, y0, ex, ey}: g(x) = Image::get((x - x0) / ex,
       (y - y0) / ey) (image.h:53-58) at the walk's projection onto the Dirichlet boundary, as
       the upstream demo's setPDE did (scene.h:202-207, commented in the fork: x0, y0 = bbox.pMin,
       ex = ey = bbox.extent().maxCoeff()); NULL: the constant dirichlet_value */
    const float *dirichlet_image;
    int32_t dirichlet_image_dims[2];
    float dirichlet_image_box[4];
    /* optional image-valued Neumann data h (2D): [h][w] row-major, row ~ y, over the rectangle
       neumann_image_box = {x0, y0, ex, ey}: h(y) = Image::get((y - x0) / ex, (y - y0) / ey) at a
       stochastic boundary sample y (the upstream demo's pde.neumann, scene.h:175-181 commented in
       the fork, which has h = 0); NULL: h = 0 */
    const float *neumann_image;
    int32_t neumann_image_dims[2];
    float neumann_image_box[4];
} oracle_scene_desc;

typedef struct oracle_params {
    int32_t n_walks;
    int32_t max_walk_length;
    int32_t steps_before_tikhonov;
    int32_t steps_before_maximal_spheres;
    float epsilon_shell;
    float min_star_radius;
    float silhouette_precision;
    float russian_roulette_threshold;
    float boundary_distance_mask;
    int32_t disable_gradient_control_variates;
    int32_t disable_gradient_antithetic_variates;
    int32_t use_cosine_sampling;
    int32_t ignore_dirichlet;
    int32_t ignore_neumann;
    int32_t ignore_source;
    uint64_t seed;            /* counter-based RNG key (replaces system_clock seeds) */
    int32_t math_mode;        /* 0 = det (matches GPU), 1 = glibc libm */
    int32_t n_threads;        /* std thread count for the CPU baseline */
    int32_t robust_float;     /* 0 = the reference's float members (NaN for mu R > ~92), 1 = robust */
} oracle_params;

typedef struct oracle_stats {
    uint64_t walk_steps;        /* updateBall calls of recorded walks */
    uint64_t wasted_steps;      /* updateBall calls of dropped walks */
    uint64_t walks_recorded;
    uint64_t walks_escaped;
    uint64_t walks_max_length;
    uint64_t walks_rr;
    uint64_t walks_dirichlet;
    uint64_t points_estimated;
    uint64_t rejection_iters;
} oracle_stats;

/* Solve at n points (pts: n*dim).  index_base/index_stride give the global
 * point index used for RNG keying: gidx = index_base + i*index_stride.
 * Outputs: p[n], grad[n*dim]; optional per-point arrays (may be NULL):
 * n_est[n] (recorded walks), steps[n] (walk steps incl. wasted). */
int oracle_solve(const oracle_scene_desc *scene, const oracle_params *prm,
                 const float *pts, int64_t n, int64_t index_base, int64_t index_stride,
                 float *p, float *grad, int32_t *n_est, int32_t *steps,
                 oracle_stats *stats);

/* oracle_solve plus the per-point Welford M2 of the solution estimates (sol_m2[n], may be
 * NULL; the sample variance is sol_m2 / (n_est - 1), SampleStatistics walk_on_stars.h:744-877)
 * -- for the statistical pin against the reference's own engine solution. */
int oracle_solve_m2(const oracle_scene_desc *scene, const oracle_params *prm,
                    const float *pts, int64_t n, int64_t index_base, int64_t index_stride,
                    float *p, float *grad, int32_t *n_est, int32_t *steps, float *sol_m2,
                    oracle_stats *stats);

/* Boundary value caching: runBoundaryValueCaching (bindings/zombie/demo/demo.cpp:
 * 265-363), 2D scenes with Neumann and Dirichlet boundaries.  Outputs as wos_bvc
 * (include/wos.h). */
typedef struct oracle_bvc_params {
    int32_t n_walks_solution, n_walks_gradient, boundary_cache_size, domain_cache_size, grid_res;
    int32_t use_finite_differences;
    float normal_offset, radius_clamp, kernel_regularization;
    float grid_box[4];        /* evaluation grid x0, y0, ex, ey (extent 0: the scene's bounding box) */
} oracle_bvc_params;

int oracle_bvc(const oracle_scene_desc *scene, const oracle_params *prm, const oracle_bvc_params *bvc,
               float *solution, float *grad, float *samples, int64_t samples_capacity, int64_t *counts,
               oracle_stats *stats);

/* Geometry helpers exposed for unit tests. */
int oracle_point_info(const oracle_scene_desc *scene, const float *pt,
                      float *dirichlet_dist, float *neumann_dist,
                      float *signed_neumann_dist, int32_t *inside,
                      float *star_radius, int32_t *n_silhouettes);

double oracle_bessel(int which, double x, int math_mode); /* 0:i0 1:i1 2:k0 3:k1 */
double oracle_math(int which, double x, int math_mode);   /* 0 exp 1 log 2 sin 3 cos 4 atan, f32: 10 expf 11 logf 12 sinf 13 cosf 14 cbrtf */
uint32_t oracle_seed32(uint64_t key, uint64_t idx, uint64_t pair, uint32_t tag);
int oracle_lhs(uint32_t seed, int n, int dims, float *out); /* stratified samples */
/* fcpw's wide BVH over a boundary mesh as the oracle builds it (cap_nodes nodes of
 * `branch` children: box [6 * branch], child [branch]; ref [np]) */
/* fcpw's stochastic traversal (sampleNeumann's primitive choice) at ball (x, R) for
 * n uniforms: chosen primitive (-1: none) and its selection pdf */
int oracle_fcpw_pick(const oracle_scene_desc *scene, const float *x, float R, int n, const float *us, int32_t *sel,
                     float *pdf);
int oracle_fcpw_bvh(int dim, const float *v, int nv, const int32_t *ix, int np, int branch, int leaf,
                    float *box, int32_t *child, int32_t *ref, int cap_nodes, int *n_nodes);

#ifdef __cplusplus
}
#endif
#endif
