/*
 * oracle/wos_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, brute-force geometry) of the zombie walk-on-stars
 * estimator exactly as the reference's zombie_bindings.wost() runs it:
 *
 *   boundary      bindings/zombie/demo/demo.cpp:119-205 (runWalkOnStars_sampled)
 *   sample pts    bindings/zombie/demo/grid.h:69-102, masks grid.h:155-237
 *   estimator     include/zombie/point_estimation/walk_on_stars.h:466-617
 *   walk loop     walk_on_stars.h:135-329, terminal 331-351, stats 744-877
 *   Green's fns   include/zombie/core/distributions.h:273-832
 *   sampling      include/zombie/core/sampling.h:23-64,107-203,435-478
 *   Bessel        deps/bessel/bessel.hpp:373-555 (double precision)
 *   RNG           deps/pcg32/pcg32.h:53-112
 *   geometry      include/zombie/utils/fcpw_scene_loader.h:252-651 over fcpw's
 *                 semantics: line_segments.inl:46-254, triangles.inl:48-131,
 *                 wide_query_operations.h:27-235,328-395,
 *                 vertex_silhouettes.inl:29-118, edge_silhouettes.inl:40-140,
 *                 bounding_volumes.h:38-75, interaction.h:32-34,
 *                 fcpw.inl:200-353, sbvh.inl:313-436 (silhouette ignore rule)
 *   scene / PDE   bindings/zombie/demo/scene.h:54-200, image.h:42-58,
 *                 bindings/zombie3d/demo/scene_3d.h:22-128
 *
 * For the deterministic queries fcpw's wide BVH is replaced by fcpw's own
 * brute-force "Baseline" semantics (aggregates/baseline.inl); they are
 * order-independent except for exact ties (resolved "last wins", as the
 * reference's `<=` scans do).  The stochastic Neumann sample, whose result
 * depends on the tree, walks fcpw's tree itself, restated here
 * (geom_build_fcpw_bvh: sbvh.inl:3-235 + mbvh.inl:46-133; fcpw_stochastic_pick:
 * mbvh.inl:835-982,1099-1283).
 *
 * Deliberate, documented deviations from the reference:
 *  - RNG seeds: the reference seeds every point and every antithetic pair from
 *    std::chrono::system_clock (walk_on_stars.h:498,639).  Here seeds are a
 *    counter-based hash of (key, global point index, pair, stream tag).  The
 *    first-ball source draws of pair w use their own stream instead of the tail
 *    of pair w-1's walk stream.
 *  - Enoki's approximate rcp/rsqrt (+Newton step) are replaced by exact IEEE
 *    1/x and x/sqrt(.) -- same operation structure, deterministic.
 *  - math_mode 0 ("det") uses oracle/detmath.h instead of glibc so the GPU can
 *    reproduce results bit-for-bit; math_mode 1 uses glibc like the reference.
 */
#define _GNU_SOURCE
#include "wos_oracle.h"
#include "detmath.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#define PI_D 3.141592653589793
#define TWO_PI_D 6.283185307179586     /* 2.0f*M_PI evaluated in double */
#define FOUR_PI_D 12.566370614359172   /* 4.0f*M_PI evaluated in double */
#define FEPS FLT_EPSILON
/* FCPW_MBVH_BRANCHING_FACTOR (FCPW_USE_EIGHT_WIDE_BRANCHING off) and FCPW_SIMD_WIDTH of an
 * AVX/AVX2 build (fcpw CMakeLists.txt:83-99): the shape of the tree sampleNeumann walks */
#define ORACLE_FCPW_BRANCH 4
#define ORACLE_FCPW_LEAF 8

/* ------------------------------------------------------------------------- */
/* math mode                                                                 */
/* ------------------------------------------------------------------------- */
static __thread int g_libm = 0;
/* robust float semantics (oracle_params.robust_float): Yukawa balls with mu R > ROBUST_MUR
 * use exponentially scaled Bessels and ratios (SURVEY.md section 7.2 hard part 4) */
static __thread int g_robust = 0;
#define ROBUST_MUR 80.0f

static inline double m_exp(double x) { return g_libm ? exp(x) : dm_exp(x); }
static inline double m_log(double x) { return g_libm ? log(x) : dm_log(x); }
static inline float m_expf(float x) { return g_libm ? expf(x) : dm_expf(x); }
static inline float m_logf(float x) { return g_libm ? logf(x) : dm_logf(x); }
static inline float m_cosf(float x) { return g_libm ? cosf(x) : dm_cosf(x); }
static inline float m_sinf(float x) { return g_libm ? sinf(x) : dm_sinf(x); }
static inline float m_cbrtf(float x) { return g_libm ? cbrtf(x) : dm_cbrtf(x); }
static inline float m_atan2f(float y, float x) { return g_libm ? atan2f(y, x) : dm_atan2f(y, x); }

/* std::max / std::min / std::clamp semantics (NaN-order matters) */
static inline float smaxf(float a, float b) { return (a < b) ? b : a; }
static inline float sminf(float a, float b) { return (b < a) ? b : a; }
static inline int sclampi(int v, int lo, int hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }

/* int(float) with x86 cvttss2si semantics: NaN / out of range -> INT_MIN */
static inline int cvt_trunc(float x)
{
    if (!(x > -2147483904.0f && x < 2147483648.0f)) return (int)0x80000000u;
    return (int)x;
}

static inline float float_bits_add(float f, int d)
{
    int32_t i; memcpy(&i, &f, 4); i += d; float r; memcpy(&r, &i, 4); return r;
}

/* ------------------------------------------------------------------------- */
/* Bessel functions (double), bessel.hpp:373-555                             */
/* ------------------------------------------------------------------------- */
static double bessi0(double x)
{
    double ax, ans, y;
    if ((ax = fabs(x)) < 3.75) {
        y = x / 3.75; y = y * y;
        ans = 1.0 + y * (3.5156229 + y * (3.0899424 + y * (1.2067492
              + y * (0.2659732 + y * (0.360768e-1 + y * 0.45813e-2)))));
    } else {
        y = 3.75 / ax;
        ans = (m_exp(ax) / sqrt(ax)) * (0.39894228 + y * (0.1328592e-1
              + y * (0.225319e-2 + y * (-0.157565e-2 + y * (0.916281e-2
              + y * (-0.2057706e-1 + y * (0.2635537e-1 + y * (-0.1647633e-1
              + y * 0.392377e-2))))))));
    }
    return ans;
}

static double bessi1(double x)
{
    double ax, ans, y;
    if ((ax = fabs(x)) < 3.75) {
        y = x / 3.75; y = y * y;
        ans = ax * (0.5 + y * (0.87890594 + y * (0.51498869 + y * (0.15084934
              + y * (0.2658733e-1 + y * (0.301532e-2 + y * 0.32411e-3))))));
    } else {
        y = 3.75 / ax;
        ans = 0.2282967e-1 + y * (-0.2895312e-1 + y * (0.1787654e-1 - y * 0.420059e-2));
        ans = 0.39894228 + y * (-0.3988024e-1 + y * (-0.362018e-2
              + y * (0.163801e-2 + y * (-0.1031555e-1 + y * ans))));
        ans *= (m_exp(ax) / sqrt(ax));
    }
    return x < 0.0 ? -ans : ans;
}

static double bessk0(double x)
{
    double y, ans;
    if (x <= 2.0) {
        y = x * x / 4.0;
        ans = (-m_log(x / 2.0) * bessi0(x)) + (-0.57721566 + y * (0.42278420
              + y * (0.23069756 + y * (0.3488590e-1 + y * (0.262698e-2
              + y * (0.10750e-3 + y * 0.74e-5))))));
    } else {
        y = 2.0 / x;
        ans = (m_exp(-x) / sqrt(x)) * (1.25331414 + y * (-0.7832358e-1
              + y * (0.2189568e-1 + y * (-0.1062446e-1 + y * (0.587872e-2
              + y * (-0.251540e-2 + y * 0.53208e-3))))));
    }
    return ans;
}

static double bessk1(double x)
{
    double y, ans;
    if (x <= 2.0) {
        y = x * x / 4.0;
        ans = (m_log(x / 2.0) * bessi1(x)) + (1.0 / x) * (1.0 + y * (0.15443144
              + y * (-0.67278579 + y * (-0.18156897 + y * (-0.1919402e-1
              + y * (-0.110404e-2 + y * (-0.4686e-4)))))));
    } else {
        y = 2.0 / x;
        ans = (m_exp(-x) / sqrt(x)) * (1.25331414 + y * (0.23498619
              + y * (-0.3655620e-1 + y * (0.1504268e-1 + y * (-0.780353e-2
              + y * (0.325614e-2 + y * (-0.68245e-3)))))));
    }
    return ans;
}

/* Robust mode: exponentially scaled A&S functions ie_v(x) = e^-x I_v(x), ke_v(x) =
 * e^x K_v(x), x > 0 -- the polynomials above without the exponential (large x) or
 * times the compensating exponential (small x), so nothing overflows for any x. */
static void bess_scaled(double x, double *ie0, double *ke0, double *ie1, double *ke1)
{
    if (x < 3.75) {
        double e = m_exp(-x);
        *ie0 = bessi0(x) * e;
        *ie1 = bessi1(x) * e;
    } else {
        double y = 3.75 / x, sx = sqrt(x);
        *ie0 = (0.39894228 + y * (0.1328592e-1 + y * (0.225319e-2 + y * (-0.157565e-2 + y * (0.916281e-2
               + y * (-0.2057706e-1 + y * (0.2635537e-1 + y * (-0.1647633e-1 + y * 0.392377e-2)))))))) / sx;
        double a = 0.2282967e-1 + y * (-0.2895312e-1 + y * (0.1787654e-1 - y * 0.420059e-2));
        a = 0.39894228 + y * (-0.3988024e-1 + y * (-0.362018e-2 + y * (0.163801e-2 + y * (-0.1031555e-1 + y * a))));
        *ie1 = a / sx;
    }
    if (x <= 2.0) {
        double e = m_exp(x);
        *ke0 = bessk0(x) * e;
        *ke1 = bessk1(x) * e;
    } else {
        double y = 2.0 / x, sx = sqrt(x);
        *ke0 = (1.25331414 + y * (-0.7832358e-1 + y * (0.2189568e-1 + y * (-0.1062446e-1 + y * (0.587872e-2
               + y * (-0.251540e-2 + y * 0.53208e-3)))))) / sx;
        *ke1 = (1.25331414 + y * (0.23498619 + y * (-0.3655620e-1 + y * (0.1504268e-1 + y * (-0.780353e-2
               + y * (0.325614e-2 + y * (-0.68245e-3))))))) / sx;
    }
}

/* 3D: e^-x I_{3/2}-like member scaled: (cosh x - sinh x / x) e^-x */
static inline double i32s(double x)
{
    double e2 = m_exp(-2.0 * x);
    return 0.5 * ((1.0 + e2) - (1.0 - e2) / x);
}

/* ------------------------------------------------------------------------- */
/* PCG32, pcg32.h:53-112                                                      */
/* ------------------------------------------------------------------------- */
typedef struct { uint64_t state, inc; } pcg_t;

static inline uint32_t pcg_next(pcg_t *g)
{
    uint64_t old = g->state;
    g->state = old * 0x5851f42d4c957f2dULL + g->inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((~rot + 1u) & 31));
}
static inline void pcg_seed(pcg_t *g, uint64_t initstate, uint64_t initseq)
{
    g->state = 0u; g->inc = (initseq << 1u) | 1u;
    pcg_next(g); g->state += initstate; pcg_next(g);
}
static inline float pcg_float(pcg_t *g)
{
    uint32_t u = (pcg_next(g) >> 9) | 0x3f800000u; float f; memcpy(&f, &u, 4); return f - 1.0f;
}
static inline uint32_t pcg_bounded(pcg_t *g, uint32_t bound)
{
    uint32_t th = (~bound + 1u) % bound;
    for (;;) { uint32_t r = pcg_next(g); if (r >= th) return r % bound; }
}

static inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
uint32_t oracle_seed32(uint64_t key, uint64_t idx, uint64_t pair, uint32_t tag)
{
    uint64_t h = mix64(key ^ mix64(idx * 0x9E3779B97F4A7C15ULL + pair * 0xD1B54A32D192ED03ULL
                                   + (uint64_t)tag * 0x8CB92BA72F3D8DD7ULL + 0x632BE59BD9B4E019ULL));
    return (uint32_t)(h >> 32);
}

/* generateStratifiedSamples<DIM>, sampling.h:435-457 */
static void gen_stratified(float *s, int n, int dims, pcg_t *g)
{
    const float ome = 1.0f - FEPS;
    float inv = 1.0f / (float)n;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < dims; ++j) {
            float sj = ((float)i + pcg_float(g)) * inv;
            s[dims * i + j] = sminf(sj, ome);
        }
    for (int i = 0; i < dims; ++i)
        for (int j = 0; j < n; ++j) {
            int other = j + (int)pcg_bounded(g, (uint32_t)(n - j));
            float t = s[dims * j + i]; s[dims * j + i] = s[dims * other + i]; s[dims * other + i] = t;
        }
}

int oracle_lhs(uint32_t seed, int n, int dims, float *out)
{
    pcg_t g; pcg_seed(&g, seed, 1u);
    gen_stratified(out, n, dims, &g);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* small vector helpers (3 components; 2D data has z = 0)                    */
/* ------------------------------------------------------------------------- */
static inline float dot3(const float *a, const float *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline float norm3(const float *a) { return sqrtf(dot3(a, a)); }
static inline void sub3(float *r, const float *a, const float *b) { r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2]; }
static inline void cross3(float *r, const float *a, const float *b)
{
    float x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
    r[0] = x; r[1] = y; r[2] = z;
}
/* Eigen normalized(): v / sqrt(squaredNorm) if > 0 */
static inline void normalize3(float *v)
{
    float z = dot3(v, v);
    if (z > 0.0f) { float s = sqrtf(z); v[0] /= s; v[1] /= s; v[2] /= s; }
}
/* enoki::normalize as restated: v * (1/sqrt(squaredNorm)) */
static inline void normalize_rcp3(float *v)
{
    float inv = 1.0f / sqrtf(dot3(v, v));
    v[0] *= inv; v[1] *= inv; v[2] *= inv;
}

/* ------------------------------------------------------------------------- */
/* geometry (one boundary: Neumann or Dirichlet)                             */
/* ------------------------------------------------------------------------- */
typedef struct {
    int dim, nv, np;
    float (*v)[3];
    int32_t (*ix)[3];
    float (*vn)[3];       /* vertex normals (fcpw.inl:306-353) */
    int ne;               /* 3D edges */
    int32_t *pe;          /* 3 edge indices per triangle (assignEdgeIndices) */
    float (*en)[3];       /* edge normals */
    /* silhouette candidates (vertices in 2D, edges in 3D) */
    int ns;
    float (*sa)[3], (*sb)[3], (*sn0)[3], (*sn1)[3];
    int32_t *smiss;
    /* fcpw's wide BVH (Neumann boundary; geom_build_fcpw_bvh) */
    int nb_branch, nb_nodes, nb_leaves;
    float *nb_box;        /* [node][branch][min.xyz max.xyz] */
    int32_t *nb_child;    /* [node][branch]; leaf: [-(leaf+1), leaf count, first ref, ref count] */
    int32_t *nb_ref;      /* reference -> primitive */
} geom_t;

static void geom_free(geom_t *g)
{
    free(g->v); free(g->ix); free(g->vn); free(g->pe); free(g->en);
    free(g->sa); free(g->sb); free(g->sn0); free(g->sn1); free(g->smiss);
    free(g->nb_box); free(g->nb_child); free(g->nb_ref);
    memset(g, 0, sizeof(*g));
}

static void prim_normal(const geom_t *g, int p, float *n, int normalize)
{
    if (g->dim == 2) {
        const float *pa = g->v[g->ix[p][0]], *pb = g->v[g->ix[p][1]];
        float s[3]; sub3(s, pb, pa);
        n[0] = s[1]; n[1] = -s[0]; n[2] = 0.0f;
    } else {
        const float *pa = g->v[g->ix[p][0]], *pb = g->v[g->ix[p][1]], *pc = g->v[g->ix[p][2]];
        float v1[3], v2[3]; sub3(v1, pb, pa); sub3(v2, pc, pa);
        cross3(n, v1, v2);
    }
    if (normalize) normalize3(n);
}

static float prim_area(const geom_t *g, int p)
{
    if (g->dim == 2) {
        float s[3]; sub3(s, g->v[g->ix[p][1]], g->v[g->ix[p][0]]); return norm3(s);
    }
    float n[3]; prim_normal(g, p, n, 0); return 0.5f * norm3(n);
}

/* ignore rule scene.h:84-90 / sbvh.inl:340-355,405-421 */
static int ignore_candidate(float angle, int double_sided) { return double_sided ? 0 : (angle < 1e-3f); }

static int geom_build(geom_t *g, int dim, int nv, int np, const float *v, const int32_t *ix,
                      int build_silhouettes, int double_sided)
{
    memset(g, 0, sizeof(*g));
    g->dim = dim; g->nv = nv; g->np = np;
    if (nv <= 0 || np <= 0) return 0;
    g->v = calloc((size_t)nv, sizeof(*g->v));
    g->ix = calloc((size_t)np, sizeof(*g->ix));
    g->vn = calloc((size_t)nv, sizeof(*g->vn));
    for (int i = 0; i < nv; i++) for (int k = 0; k < dim; k++) g->v[i][k] = v[i * dim + k];
    for (int p = 0; p < np; p++) for (int k = 0; k < dim; k++) {
        int32_t q = ix[p * dim + k];
        if (q < 0 || q >= nv) return -1;
        g->ix[p][k] = q;
    }
    if (dim == 2) {
        /* computeNormals<3, LineSegment> (fcpw.inl:305-325), unweighted */
        for (int p = 0; p < np; p++) {
            float n[3]; prim_normal(g, p, n, 1);
            for (int k = 0; k < 2; k++) {
                float *d = g->vn[g->ix[p][k]];
                d[0] += 1.0f * n[0]; d[1] += 1.0f * n[1]; d[2] += 1.0f * n[2];
            }
        }
        for (int i = 0; i < nv; i++) normalize3(g->vn[i]);
        if (build_silhouettes) {
            /* computeSilhouettes (fcpw.inl:237-260): prev/next per vertex */
            int32_t *prev = malloc(sizeof(int32_t) * nv), *next = malloc(sizeof(int32_t) * nv);
            char *ref = calloc((size_t)nv, 1);
            for (int i = 0; i < nv; i++) prev[i] = next[i] = -1;
            for (int p = 0; p < np; p++) {
                int a = g->ix[p][0], b = g->ix[p][1];
                next[a] = b; prev[b] = a; ref[a] = ref[b] = 1;
            }
            g->sa = calloc((size_t)nv, sizeof(*g->sa)); g->sb = calloc((size_t)nv, sizeof(*g->sb));
            g->sn0 = calloc((size_t)nv, sizeof(*g->sn0)); g->sn1 = calloc((size_t)nv, sizeof(*g->sn1));
            g->smiss = calloc((size_t)nv, sizeof(int32_t));
            /* candidates in order of first appearance over segments (sbvh.inl:330-369) */
            char *seen = calloc((size_t)nv, 1);
            for (int p = 0; p < np; p++) for (int k = 0; k < 2; k++) {
                int vi = g->ix[p][k];
                if (seen[vi]) continue;
                seen[vi] = 1;
                int has0 = next[vi] != -1, has1 = prev[vi] != -1;
                float n0[3] = {0, 0, 0}, n1[3] = {0, 0, 0};
                if (has0) { float s[3]; sub3(s, g->v[next[vi]], g->v[vi]); n0[0] = s[1]; n0[1] = -s[0]; normalize3(n0); }
                if (has1) { float s[3]; sub3(s, g->v[vi], g->v[prev[vi]]); n1[0] = s[1]; n1[1] = -s[0]; normalize3(n1); }
                int ignore = 0;
                if (has0 && has1) {
                    float det = n0[0] * n1[1] - n1[0] * n0[1];
                    ignore = ignore_candidate(det, double_sided);
                }
                if (ignore) continue;
                int s = g->ns++;
                memcpy(g->sa[s], g->v[vi], sizeof(float) * 3);
                memcpy(g->sn0[s], n0, sizeof(float) * 3);
                memcpy(g->sn1[s], n1, sizeof(float) * 3);
                g->smiss[s] = !(has0 && has1);
            }
            free(prev); free(next); free(ref); free(seen);
        }
    } else {
        /* assignEdgeIndices (fcpw.inl:200-221): edge id by first appearance of sorted pair */
        g->pe = malloc(sizeof(int32_t) * 3 * np);
        int32_t (*ekey)[2] = malloc(sizeof(*ekey) * 3 * np);
        int ne = 0;
        for (int p = 0; p < np; p++) for (int j = 0; j < 3; j++) {
            int I = g->ix[p][j], J = g->ix[p][(j + 1) % 3];
            if (I > J) { int t = I; I = J; J = t; }
            int e = -1;
            for (int q = 0; q < ne; q++) if (ekey[q][0] == I && ekey[q][1] == J) { e = q; break; }
            if (e < 0) { e = ne++; ekey[e][0] = I; ekey[e][1] = J; }
            g->pe[3 * p + j] = e;
        }
        g->ne = ne;
        g->en = calloc((size_t)ne, sizeof(*g->en));
        /* computeNormals<3, Triangle> (fcpw.inl:327-353): vertex normals unweighted,
         * edge normals area-weighted */
        for (int p = 0; p < np; p++) {
            float n[3]; prim_normal(g, p, n, 1);
            float area = prim_area(g, p);
            for (int j = 0; j < 3; j++) {
                float *d = g->vn[g->ix[p][j]];
                d[0] += 1.0f * n[0]; d[1] += 1.0f * n[1]; d[2] += 1.0f * n[2];
                float *e = g->en[g->pe[3 * p + j]];
                e[0] += area * n[0]; e[1] += area * n[1]; e[2] += area * n[2];
            }
        }
        for (int i = 0; i < nv; i++) normalize3(g->vn[i]);
        for (int e = 0; e < ne; e++) normalize3(g->en[e]);
        if (build_silhouettes) {
            /* SilhouetteEdge indices (fcpw.inl:262-293): [0]/[3] opposite vertices, [1],[2] endpoints */
            int32_t (*sidx)[4] = malloc(sizeof(*sidx) * ne);
            for (int e = 0; e < ne; e++) sidx[e][0] = sidx[e][1] = sidx[e][2] = sidx[e][3] = -1;
            for (int p = 0; p < np; p++) for (int j = 0; j < 3; j++) {
                int I = j - 1 < 0 ? 2 : j - 1, J = j, K = j + 1 > 2 ? 0 : j + 1;
                int e = g->pe[3 * p + j];
                float orientation = 1.0f;
                if (g->ix[p][J] > g->ix[p][K]) { int t = J; J = K; K = t; orientation = -1.0f; }
                sidx[e][orientation == 1.0f ? 0 : 3] = g->ix[p][I];
                sidx[e][1] = g->ix[p][J];
                sidx[e][2] = g->ix[p][K];
            }
            g->sa = calloc((size_t)ne, sizeof(*g->sa)); g->sb = calloc((size_t)ne, sizeof(*g->sb));
            g->sn0 = calloc((size_t)ne, sizeof(*g->sn0)); g->sn1 = calloc((size_t)ne, sizeof(*g->sn1));
            g->smiss = calloc((size_t)ne, sizeof(int32_t));
            char *seen = calloc((size_t)ne, 1);
            for (int p = 0; p < np; p++) for (int k = 0; k < 3; k++) {
                int e = g->pe[3 * p + k];
                if (seen[e]) continue;
                seen[e] = 1;
                int has0 = sidx[e][3] != -1, has1 = sidx[e][0] != -1;
                float n0[3] = {0, 0, 0}, n1[3] = {0, 0, 0};
                /* SilhouetteEdge::normal(fIndex) edge_silhouettes.inl:45-68 */
                if (has0) {
                    float v1[3], v2[3]; sub3(v1, g->v[sidx[e][2]], g->v[sidx[e][1]]); sub3(v2, g->v[sidx[e][3]], g->v[sidx[e][1]]);
                    cross3(n0, v1, v2); normalize3(n0);
                }
                if (has1) {
                    float v1[3], v2[3]; sub3(v1, g->v[sidx[e][1]], g->v[sidx[e][2]]); sub3(v2, g->v[sidx[e][0]], g->v[sidx[e][2]]);
                    cross3(n1, v1, v2); normalize3(n1);
                }
                int ignore = 0;
                if (has0 && has1) {
                    float ed[3]; sub3(ed, g->v[sidx[e][2]], g->v[sidx[e][1]]); normalize3(ed);
                    float c[3]; cross3(c, n0, n1);
                    float ang = m_atan2f(dot3(ed, c), dot3(n0, n1));
                    ignore = ignore_candidate(ang, double_sided);
                }
                if (ignore) continue;
                int s = g->ns++;
                memcpy(g->sa[s], g->v[sidx[e][1]], sizeof(float) * 3);
                memcpy(g->sb[s], g->v[sidx[e][2]], sizeof(float) * 3);
                memcpy(g->sn0[s], n0, sizeof(float) * 3);
                memcpy(g->sn1[s], n1, sizeof(float) * 3);
                g->smiss[s] = !(has0 && has1);
            }
            free(sidx); free(seen);
        }
        free(ekey);
    }
    return 0;
}

/* wide closest point on a segment (wide_query_operations.h:121-141) */
static float closest_point_segment(const float *pa, const float *pb, const float *x, float *pt, float *t)
{
    float u[3], v[3]; sub3(u, pb, pa); sub3(v, x, pa);
    float c1 = dot3(u, v), c2 = dot3(u, u);
    float tt = c1 * (1.0f / c2);
    if (c1 <= 0.0f) tt = 0.0f;
    if (c2 <= c1) tt = 1.0f;
    pt[0] = pa[0] + u[0] * tt; pt[1] = pa[1] + u[1] * tt; pt[2] = pa[2] + u[2] * tt;
    *t = tt;
    float d[3]; sub3(d, x, pt);
    return norm3(d);
}

/* wide closest point on a triangle (wide_query_operations.h:144-235) */
static float closest_point_triangle(const float *pa, const float *pb, const float *pc, const float *x,
                                    float *pt, float *t0, float *t1)
{
    float ab[3], ac[3], ax[3]; sub3(ab, pb, pa); sub3(ac, pc, pa); sub3(ax, x, pa);
    float d1 = dot3(ab, ax), d2 = dot3(ac, ax);
    float d[3];
    if (d1 <= 0.0f && d2 <= 0.0f) { memcpy(pt, pa, 12); *t0 = 1.0f; *t1 = 0.0f; sub3(d, x, pt); return norm3(d); }
    float bx[3]; sub3(bx, x, pb);
    float d3 = dot3(ab, bx), d4 = dot3(ac, bx);
    if (d3 >= 0.0f && d4 <= d3) { memcpy(pt, pb, 12); *t0 = 0.0f; *t1 = 1.0f; sub3(d, x, pt); return norm3(d); }
    float cx[3]; sub3(cx, x, pc);
    float d5 = dot3(ab, cx), d6 = dot3(ac, cx);
    if (d6 >= 0.0f && d5 <= d6) { memcpy(pt, pc, 12); *t0 = 0.0f; *t1 = 0.0f; sub3(d, x, pt); return norm3(d); }
    float vc = d1 * d4 - d3 * d2;
    if (vc <= 0.0f && d1 >= 0.0f && d3 <= 0.0f) {
        float v = d1 * (1.0f / (d1 - d3));
        for (int k = 0; k < 3; k++) pt[k] = pa[k] + ab[k] * v;
        *t0 = 1.0f - v; *t1 = v; sub3(d, x, pt); return norm3(d);
    }
    float vb = d5 * d2 - d1 * d6;
    if (vb <= 0.0f && d2 >= 0.0f && d6 <= 0.0f) {
        float w = d2 * (1.0f / (d2 - d6));
        for (int k = 0; k < 3; k++) pt[k] = pa[k] + ac[k] * w;
        *t0 = 1.0f - w; *t1 = 0.0f; sub3(d, x, pt); return norm3(d);
    }
    float va = d3 * d6 - d5 * d4;
    if (va <= 0.0f && (d4 - d3) >= 0.0f && (d5 - d6) >= 0.0f) {
        float w = (d4 - d3) * (1.0f / ((d4 - d3) + (d5 - d6)));
        for (int k = 0; k < 3; k++) pt[k] = pb[k] + (pc[k] - pb[k]) * w;
        *t0 = 0.0f; *t1 = 1.0f - w; sub3(d, x, pt); return norm3(d);
    }
    float denom = 1.0f / (va + vb + vc);
    float v = vb * denom, w = vc * denom;
    for (int k = 0; k < 3; k++) pt[k] = pa[k] + ab[k] * v + ac[k] * w;
    *t0 = 1.0f - v - w; *t1 = v;
    sub3(d, x, pt); return norm3(d);
}

typedef struct { float d; float p[3]; float n[3]; float t0, t1; int prim; } cp_t;

/* findClosestPoint over all primitives; returns prim index or -1.  Selection key is
 * fl(d*d) with `<=` (last wins), mbvh.inl:1297-1351. */
static int closest_point(const geom_t *g, const float *x, cp_t *out, int record_normal)
{
    if (g->np <= 0) return -1;
    float sr2 = FLT_MAX; int best = -1;
    for (int p = 0; p < g->np; p++) {
        float pt[3], t0 = 0.0f, t1 = 0.0f, d;
        if (g->dim == 2) d = closest_point_segment(g->v[g->ix[p][0]], g->v[g->ix[p][1]], x, pt, &t0);
        else d = closest_point_triangle(g->v[g->ix[p][0]], g->v[g->ix[p][1]], g->v[g->ix[p][2]], x, pt, &t0, &t1);
        float d2 = d * d;
        if (d2 <= sr2) { sr2 = d2; best = p; out->d = d; memcpy(out->p, pt, 12); out->t0 = t0; out->t1 = t1; }
    }
    out->prim = best;
    if (best >= 0 && record_normal) {
        /* Interaction::computeNormal -> primitive normal(uv) */
        if (g->dim == 2) {
            float t = out->t0;
            if (t <= FEPS) memcpy(out->n, g->vn[g->ix[best][0]], 12);
            else if (t >= 1.0f - FEPS) memcpy(out->n, g->vn[g->ix[best][1]], 12);
            else prim_normal(g, best, out->n, 1);
        } else {
            float u0 = out->t0, u1 = out->t1;
            int vI = -1, eI = -1;
            if (u0 >= 1.0f - FEPS && u1 <= FEPS) vI = 0;
            else if (u0 <= FEPS && u1 >= 1.0f - FEPS) vI = 1;
            else if (u0 <= FEPS && u1 <= FEPS) vI = 2;
            if (vI == -1) {
                if (u0 <= FEPS) eI = 1;
                else if (u1 <= FEPS) eI = 2;
                else if (u0 + u1 >= 1.0f - FEPS) eI = 0;
            }
            if (vI >= 0) memcpy(out->n, g->vn[g->ix[best][vI]], 12);
            else if (eI >= 0) memcpy(out->n, g->en[g->pe[3 * best + eI]], 12);
            else prim_normal(g, best, out->n, 1);
        }
    }
    return best;
}

/* Interaction::signedDistance (interaction.h:32-34) with sign == 0 */
static float signed_distance(const cp_t *c, const float *x)
{
    float d[3]; sub3(d, x, c->p);
    return (dot3(d, c->n) > 0.0f ? 1.0f : -1.0f) * c->d;
}

/* ray first hit (mbvh.inl:521-609 + wide_query_operations.h:27-92) */
typedef struct { float p[3], n[3], d; } hit_t;
static int ray_first_hit(const geom_t *g, const float *o, const float *dir, float tmax, hit_t *h, int occlusion)
{
    int found = 0;
    float rt = tmax;
    for (int p = 0; p < g->np; p++) {
        if (g->dim == 2) {
            const float *pa = g->v[g->ix[p][0]], *pb = g->v[g->ix[p][1]];
            float u[3], v[3]; sub3(u, pa, o); sub3(v, pb, pa);
            float dv = dir[0] * v[1] - dir[1] * v[0];
            if (!(fabsf(dv) > FEPS)) continue;
            float inv = 1.0f / dv;
            float ud = u[0] * dir[1] - u[1] * dir[0];
            float t = ud * inv;
            if (!(t >= 0.0f && t <= 1.0f)) continue;
            float uv = u[0] * v[1] - u[1] * v[0];
            float d = uv * inv;
            if (!(d >= 0.0f && d <= rt)) continue;
            if (occlusion) return 1;
            rt = d; found = 1;
            h->d = d;
            h->p[0] = pa[0] + t * v[0]; h->p[1] = pa[1] + t * v[1]; h->p[2] = pa[2] + t * v[2];
            h->n[0] = v[1]; h->n[1] = -v[0]; h->n[2] = 0.0f; normalize_rcp3(h->n);
        } else {
            const float *pa = g->v[g->ix[p][0]], *pb = g->v[g->ix[p][1]], *pc = g->v[g->ix[p][2]];
            float v1[3], v2[3], pp[3]; sub3(v1, pb, pa); sub3(v2, pc, pa);
            cross3(pp, dir, v2);
            float det = dot3(v1, pp);
            if (!(fabsf(det) > FEPS)) continue;
            float inv = 1.0f / det;
            float s[3]; sub3(s, o, pa);
            float v = dot3(s, pp) * inv;
            if (!(v >= 0.0f && v <= 1.0f)) continue;
            float q[3]; cross3(q, s, v1);
            float w = dot3(dir, q) * inv;
            if (!(w >= 0.0f && v + w <= 1.0f)) continue;
            float d = dot3(v2, q) * inv;
            if (!(d >= 0.0f && d <= rt)) continue;
            if (occlusion) return 1;
            rt = d; found = 1;
            h->d = d;
            for (int k = 0; k < 3; k++) h->p[k] = pa[k] + v1[k] * v + v2[k] * w;
            cross3(h->n, v1, v2); normalize_rcp3(h->n);
        }
    }
    return found;
}

/* isWideSilhouetteVertex / isWideSilhouetteEdge (wide_query_operations.h:328-395) */
static int is_silhouette(int dim, const float *pa, const float *pb, const float *n0, const float *n1,
                         const float *view, float d, int flip, float prec)
{
    float sign = flip ? 1.0f : -1.0f;
    if (!(d > prec)) {
        if (dim == 2) {
            float det = n0[0] * n1[1] - n0[1] * n1[0];
            return sign * det > prec;
        } else {
            float ed[3]; sub3(ed, pb, pa); normalize_rcp3(ed);
            float c[3]; cross3(c, n0, n1);
            float ang = m_atan2f(dot3(ed, c), dot3(n0, n1));
            return sign * ang > prec;
        }
    }
    float inv = 1.0f / d;
    float u[3] = {view[0] * inv, view[1] * inv, view[2] * inv};
    float dot0 = dot3(u, n0), dot1 = dot3(u, n1);
    if (fabsf(dot0) <= prec) return sign * dot1 > prec;
    if (fabsf(dot1) <= prec) return sign * dot0 > prec;
    return dot0 * dot1 < 0.0f;
}

/* computeStarRadius (fcpw_scene_loader.h:621-641) via brute-force closest silhouette */
static float star_radius(const geom_t *g, const float *x, float minR, float maxR, float prec, int flipOrient)
{
    if (minR > maxR) return maxR;
    if (g->np > 0) {
        int flip = flipOrient ? 0 : 1;  /* FCPW's convention flips normals */
        float r2 = maxR < FLT_MAX ? maxR * maxR : FLT_MAX;
        float minR2 = minR * minR;
        int found = 0; float best = 0.0f;
        if (!(minR2 >= r2)) {
            for (int s = 0; s < g->ns; s++) {
                float view[3], d;
                if (g->dim == 2) {
                    sub3(view, x, g->sa[s]); d = norm3(view);
                } else {
                    float pt[3], t; d = closest_point_segment(g->sa[s], g->sb[s], x, pt, &t);
                    sub3(view, x, pt);
                }
                float d2 = d * d;
                if (d2 > r2) continue;
                int sil = g->smiss[s] ? 1 : is_silhouette(g->dim, g->sa[s], g->sb[s], g->sn0[s], g->sn1[s], view, d, flip, prec);
                if (sil && d2 <= r2) {
                    r2 = d2; best = d; found = 1;
                    if (minR2 >= r2) break;
                }
            }
        }
        if (found) return smaxf(best, minR);
    }
    return smaxf(maxR, minR);
}

/* offsetPointAlongDirection (fcpw_scene_loader.h:258-290) */
static void offset_point(int dim, const float *p, const float *n, float *out)
{
    const float origin = 1.0f / 32.0f, floatScale = 1.0f / 65536.0f, intScale = 256.0f;
    for (int k = 0; k < dim; k++) {
        int no = cvt_trunc(n[k] * intScale);
        float po = float_bits_add(p[k], p[k] < 0 ? -no : no);
        out[k] = fabsf(p[k]) < origin ? p[k] + floatScale * n[k] : po;
    }
    if (dim == 2) out[2] = 0.0f;
}

/* ------------------------------------------------------------------------- */
/* fcpw's wide BVH over the Neumann boundary, for the stochastic boundary    */
/* sample (sampleNeumann, fcpw_scene_loader.h:599-620).  The scene loader     */
/* builds Bvh_OverlapSurfaceArea with vectorize = true (:161-164), i.e. an    */
/* Sbvh (OverlapSurfaceArea cost, 8 buckets, packed leaves of FCPW_SIMD_WIDTH */
/* references; sbvh.inl:3-235) collapsed into an Mbvh with                    */
/* FCPW_MBVH_BRANCHING_FACTOR children (mbvh.inl:46-133).  fcpw's Scene<3>    */
/* holds 2D segments with z = 0; boxes carry the FLT_EPSILON padding of       */
/* BoundingBox::expandToInclude(point) in every axis.                          */
/* ------------------------------------------------------------------------- */
#define OR_BVH_BUCKETS 8
#define OR_SBVH_MAX_DEPTH 64

typedef struct { float mn[3], mx[3]; } obox_t;

static void obox_empty(obox_t *b) { for (int k = 0; k < 3; k++) { b->mn[k] = FLT_MAX; b->mx[k] = -FLT_MAX; } }
static void obox_point(obox_t *b, const float *p)
{
    for (int k = 0; k < 3; k++) { b->mn[k] = sminf(b->mn[k], p[k] - FEPS); b->mx[k] = smaxf(b->mx[k], p[k] + FEPS); }
}
static void obox_box(obox_t *b, const obox_t *o)
{
    for (int k = 0; k < 3; k++) { b->mn[k] = sminf(b->mn[k], o->mn[k]); b->mx[k] = smaxf(b->mx[k], o->mx[k]); }
}
/* BoundingBox::surfaceArea (bounding_volumes.h:131-135); Eigen's fixed-size-3 reductions
 * pair as x0 op (x1 op x2) (Redux.h redux_novec_unroller) */
static float obox_area(const obox_t *b)
{
    float e[3];
    for (int k = 0; k < 3; k++) e[k] = smaxf(b->mx[k] - b->mn[k], 1e-5f);
    float pr = e[0] * (e[1] * e[2]);
    return 2.0f * (pr / e[0] + (pr / e[1] + pr / e[2]));
}

typedef struct { obox_t box; int off, n, second; } osnode_t;

typedef struct {
    int leaf, depth_guess, nn;
    int *prim; obox_t *rb; float (*rc)[3];
    osnode_t *nodes;
} osbvh_t;

/* computeSplitCost (sbvh.inl:3-37), OverlapSurfaceArea, packLeaves */
static float osbvh_cost(const osbvh_t *s, const obox_t *l, const obox_t *r, int nl, int nr, int depth)
{
    if (depth > 0 && ((float)s->depth_guess / depth) < 1.5f && nl % s->leaf != 0 && nr % s->leaf != 0) return FLT_MAX;
    obox_t bi;
    for (int k = 0; k < 3; k++) { bi.mn[k] = smaxf(l->mn[k], r->mn[k]); bi.mx[k] = sminf(l->mx[k], r->mx[k]); }
    float cost = ((float)nl / obox_area(r) + (float)nr / obox_area(l)) * fabsf(obox_area(&bi));
    int valid = bi.mx[0] >= bi.mn[0] && bi.mx[1] >= bi.mn[1] && bi.mx[2] >= bi.mn[2];
    if (!valid) cost *= -1.0f;
    return cost;
}

static void osbvh_build(osbvh_t *s, int parent, int st, int en, int depth)
{
    int me = s->nn++;
    obox_t bb, bc; obox_empty(&bb); obox_empty(&bc);
    for (int p = st; p < en; p++) { obox_box(&bb, &s->rb[p]); obox_point(&bc, s->rc[p]); }
    osnode_t *nd = &s->nodes[me];
    nd->box = bb; nd->off = 0; nd->n = 0; nd->second = 0;
    int nr = en - st;
    int leaf = nr <= s->leaf || depth == OR_SBVH_MAX_DEPTH - 2;
    if (leaf) { nd->off = st; nd->n = nr; }
    /* the second child to touch its parent records its offset (sbvh.inl:182-192) */
    if (parent >= 0 && me != parent + 1) s->nodes[parent].second = me - parent;
    if (leaf) return;
    /* computeObjectSplit (sbvh.inl:39-111) */
    float best = FLT_MAX, coord = 0.0f;
    int dim = -1;
    for (int d = 0; d < 3; d++) {
        float ext = bb.mx[d] - bb.mn[d];
        if (ext < 1e-6f) continue;
        float width = ext / OR_BVH_BUCKETS;
        obox_t bk[OR_BVH_BUCKETS], rk[OR_BVH_BUCKETS], acc, lb;
        int cnt[OR_BVH_BUCKETS], rcnt[OR_BVH_BUCKETS];
        for (int b = 0; b < OR_BVH_BUCKETS; b++) { obox_empty(&bk[b]); cnt[b] = 0; rcnt[b] = 0; }
        for (int p = st; p < en; p++) {
            int b = (int)((s->rc[p][d] - bb.mn[d]) / width);
            if (b < 0) b = 0;
            if (b > OR_BVH_BUCKETS - 1) b = OR_BVH_BUCKETS - 1;
            obox_box(&bk[b], &s->rb[p]); cnt[b]++;
        }
        obox_empty(&acc);
        for (int b = OR_BVH_BUCKETS - 1; b > 0; b--) {
            obox_box(&acc, &bk[b]); rk[b] = acc;
            rcnt[b] = cnt[b] + (b != OR_BVH_BUCKETS - 1 ? rcnt[b + 1] : 0);
        }
        obox_empty(&lb);
        int nl = 0;
        for (int b = 1; b < OR_BVH_BUCKETS; b++) {
            obox_box(&lb, &bk[b - 1]); nl += cnt[b - 1];
            if (nl > 0 && rcnt[b] > 0) {
                float c = osbvh_cost(s, &lb, &rk[b], nl, rcnt[b], depth);
                if (c < best) { best = c; dim = d; coord = bb.mn[d] + (float)b * width; }
            }
        }
    }
    if (dim == -1) {  /* LongestAxisCenter fallback: the first longest centroid-box axis */
        dim = 0;
        float m = bc.mx[0] - bc.mn[0];
        for (int k = 1; k < 3; k++) if (bc.mx[k] - bc.mn[k] > m) { m = bc.mx[k] - bc.mn[k]; dim = k; }
        coord = (bc.mn[dim] + bc.mx[dim]) * 0.5f;
    }
    /* performObjectSplit (sbvh.inl:113-140) */
    int mid = st;
    for (int i = st; i < en; i++) {
        if (s->rc[i][dim] < coord) {
            int tp = s->prim[i]; s->prim[i] = s->prim[mid]; s->prim[mid] = tp;
            obox_t tb = s->rb[i]; s->rb[i] = s->rb[mid]; s->rb[mid] = tb;
            float tc[3]; memcpy(tc, s->rc[i], 12); memcpy(s->rc[i], s->rc[mid], 12); memcpy(s->rc[mid], tc, 12);
            mid++;
        }
    }
    if (mid == st || mid == en) {
        mid = st + (en - st) / 2;
        while ((mid - st) % s->leaf != 0 && mid < en) mid++;
        if (mid == en) mid = st + (en - st) / 2;
    }
    osbvh_build(s, me, st, mid, depth + 1);
    osbvh_build(s, me, mid, en, depth + 1);
}

/* collapseSbvh (mbvh.inl:46-133) */
static int ombvh_collapse(geom_t *g, const osbvh_t *s, int si)
{
    const int B = g->nb_branch;
    const osnode_t *sn = &s->nodes[si];
    int mi = g->nb_nodes++;
    for (int w = 0; w < B; w++) {
        float *bx = g->nb_box + ((size_t)mi * B + w) * 6;
        for (int k = 0; k < 3; k++) { bx[k] = FLT_MAX; bx[3 + k] = -FLT_MAX; }
        g->nb_child[(size_t)mi * B + w] = INT32_MAX;
    }
    if (sn->n > 0) {
        int32_t *c = g->nb_child + (size_t)mi * B;
        c[0] = -(g->nb_leaves + 1);
        c[1] = sn->n / s->leaf + (sn->n % s->leaf != 0);
        c[2] = sn->off; c[3] = sn->n;
        g->nb_leaves += c[1];
        return mi;
    }
    int list[8], cnt = 2;
    list[0] = si + sn->second; list[1] = si + 1;
    while (cnt < B) {
        float best = -FLT_MAX; int bi = -1;
        for (int i = 0; i < cnt; i++) {
            const osnode_t *c = &s->nodes[list[i]];
            if (c->n == 0) { float a = obox_area(&c->box); if (best < a) { best = a; bi = i; } }
        }
        if (bi < 0) break;
        int x = list[bi];
        list[bi] = x + s->nodes[x].second;
        list[cnt++] = x + 1;
    }
    for (int i = 1; i < cnt; i++)  /* std::sort, ascending */
        for (int j = i; j > 0 && list[j - 1] > list[j]; j--) { int t = list[j]; list[j] = list[j - 1]; list[j - 1] = t; }
    for (int i = 0; i < cnt; i++) {
        const osnode_t *c = &s->nodes[list[i]];
        float *bx = g->nb_box + ((size_t)mi * B + i) * 6;
        for (int k = 0; k < 3; k++) { bx[k] = c->box.mn[k]; bx[3 + k] = c->box.mx[k]; }
        g->nb_child[(size_t)mi * B + i] = ombvh_collapse(g, s, list[i]);
    }
    return mi;
}

static int geom_build_fcpw_bvh(geom_t *g, int branch, int leaf)
{
    int np = g->np, nvp = g->dim;
    if (np <= 0) return 0;
    osbvh_t s;
    memset(&s, 0, sizeof(s));
    s.leaf = leaf;
    s.depth_guess = (int)log2((double)np);
    s.prim = (int *)malloc(sizeof(int) * np);
    s.rb = (obox_t *)malloc(sizeof(obox_t) * np);
    s.rc = (float (*)[3])malloc(sizeof(float) * 3 * np);
    s.nodes = (osnode_t *)malloc(sizeof(osnode_t) * 2 * (size_t)np);
    g->nb_branch = branch;
    g->nb_box = (float *)malloc(sizeof(float) * 6 * branch * 2 * (size_t)np);
    g->nb_child = (int32_t *)malloc(sizeof(int32_t) * branch * 2 * (size_t)np);
    if (!s.prim || !s.rb || !s.rc || !s.nodes || !g->nb_box || !g->nb_child) return -1;
    for (int i = 0; i < np; i++) {
        s.prim[i] = i;
        obox_empty(&s.rb[i]);
        for (int v = 0; v < nvp; v++) obox_point(&s.rb[i], g->v[g->ix[i][v]]);
        const float *pa = g->v[g->ix[i][0]], *pb = g->v[g->ix[i][1]];
        for (int k = 0; k < 3; k++)
            s.rc[i][k] = nvp == 2 ? (pa[k] + pb[k]) * 0.5f : (pa[k] + pb[k] + g->v[g->ix[i][2]][k]) / 3.0f;
    }
    osbvh_build(&s, -1, 0, np, 0);
    g->nb_nodes = 0; g->nb_leaves = 0;
    ombvh_collapse(g, &s, 0);
    g->nb_ref = (int32_t *)malloc(sizeof(int32_t) * np);
    for (int i = 0; i < np; i++) g->nb_ref[i] = s.prim[i];
    free(s.prim); free(s.rb); free(s.rc); free(s.nodes);
    return 0;
}

/* Mbvh::intersectStochasticFromNode (mbvh.inl:1099-1283) with LineSegment /
 * Triangle leaves (intersectSpherePrimitives, :835-982), the traversal weight of the
 * demo scene (|HarmonicGreensFnFreeSpace<3>::evaluate(max(r, 1e-2))|, scene.h:157-160)
 * and no primitive weight.  One root-to-leaf path; returns the chosen primitive (or
 * -1: no sample) and its selection pdf ((weight * traversalPdf) / leaf total). */
static int fcpw_stochastic_pick(const geom_t *g, const float *x, float R, float u, float *sel_pdf)
{
    const int B = g->nb_branch;
    const float r2 = R * R;
    float c[3] = {x[0], x[1], g->dim == 3 ? x[2] : 0.0f};
    float tpdf = 1.0f, d2NodeMax = FLT_MAX;
    int node = 0;
    for (;;) {
        const int32_t *C = g->nb_child + (size_t)node * B;
        if (C[0] < 0) {
            int inside = d2NodeMax <= r2, sel = -1;
            float total = 0.0f, selw = 0.0f, uu = u;
            for (int p = 0; p < C[3]; p++) {
                int q = g->nb_ref[C[2] + p];
                float d2 = 0.0f;
                if (!inside) {
                    float pt[3], t0 = 0, t1 = 0, d;
                    if (g->dim == 2) d = closest_point_segment(g->v[g->ix[q][0]], g->v[g->ix[q][1]], c, pt, &t0);
                    else d = closest_point_triangle(g->v[g->ix[q][0]], g->v[g->ix[q][1]], g->v[g->ix[q][2]], c, pt, &t0, &t1);
                    d2 = d * d;
                }
                if (d2 <= r2) {
                    float w = prim_area(g, q);
                    total += w;
                    float prob = w / total;
                    if (uu < prob) { uu = uu / prob; sel = q; selw = w; }
                    else uu = (uu - prob) / (1.0f - prob);
                }
            }
            if (sel < 0) return -1;
            float d = selw * tpdf;
            if (total > 0.0f) d /= total;
            *sel_pdf = d;
            return sel;
        }
        int sel = -1;
        float tot = 0.0f, selw = 0.0f, selmax = 0.0f;
        for (int w = 0; w < B; w++) {
            if (C[w] == INT32_MAX) continue;
            const float *bx = g->nb_box + ((size_t)node * B + w) * 6;
            /* overlapWideBox (wide_query_operations.h:96-106) */
            float mn[3], mx[3], ctr[3];
            for (int k = 0; k < 3; k++) {
                float a = bx[k] - c[k], b = c[k] - bx[3 + k];
                mn[k] = smaxf(smaxf(a, b), 0.0f);
                mx[k] = sminf(a, b);
            }
            float d2min = dot3(mn, mn), d2max = dot3(mx, mx);
            if (!(d2min <= r2)) continue;
            for (int k = 0; k < 3; k++) ctr[k] = c[k] - (bx[k] + bx[3 + k]) * 0.5f;
            float rr = smaxf(sqrtf(dot3(ctr, ctr)), 1e-2f);
            float weight = fabsf((float)(1.0 / (FOUR_PI_D * (double)rr)));
            tot += weight;
            float prob = weight / tot;
            if (u < prob) { sel = w; selw = weight; selmax = d2max; u = u / prob; }
            else u = (u - prob) / (1.0f - prob);
        }
        if (sel < 0) return -1;
        node = C[sel];
        tpdf *= selw / tot;
        d2NodeMax = selmax;
    }
}

/* the stochastic pick for a batch of uniforms at one ball (CPU property tests) */
int oracle_fcpw_pick(const oracle_scene_desc *scene, const float *x, float R, int n, const float *us, int32_t *sel,
                     float *pdf);

/* the tree as built (CPU test against the product's host build) */
int oracle_fcpw_bvh(int dim, const float *v, int nv, const int32_t *ix, int np, int branch, int leaf,
                    float *box, int32_t *child, int32_t *ref, int cap_nodes, int *n_nodes)
{
    geom_t g;
    memset(&g, 0, sizeof(g));
    g.dim = dim; g.nv = nv; g.np = np;
    g.v = (float (*)[3])calloc((size_t)nv, sizeof(float) * 3);
    g.ix = (int32_t (*)[3])calloc((size_t)np, sizeof(int32_t) * 3);
    for (int i = 0; i < nv; i++) for (int k = 0; k < dim; k++) g.v[i][k] = v[i * dim + k];
    for (int p = 0; p < np; p++) for (int k = 0; k < dim; k++) g.ix[p][k] = ix[p * dim + k];
    int rc = geom_build_fcpw_bvh(&g, branch, leaf);
    if (rc == 0) {
        *n_nodes = g.nb_nodes;
        if (g.nb_nodes > cap_nodes) rc = -2;
        else {
            memcpy(box, g.nb_box, sizeof(float) * 6 * branch * (size_t)g.nb_nodes);
            memcpy(child, g.nb_child, sizeof(int32_t) * branch * (size_t)g.nb_nodes);
            memcpy(ref, g.nb_ref, sizeof(int32_t) * (size_t)np);
        }
    }
    free(g.v); free(g.ix); free(g.nb_box); free(g.nb_child); free(g.nb_ref);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* scene                                                                      */
/* ------------------------------------------------------------------------- */
typedef struct {
    int dim;
    geom_t neu, dir;
    float pmin[3], pmax[3], ext[3];
    float g_dirichlet, absorption;
    int watertight, double_sided;
    const float *src; int sdims[3];
    const float *dimg; int ddims[2]; float dbox[4];
    const float *nimg; int ndims[2]; float nbox[4];   /* image-valued Neumann data (NULL: h = 0) */
} scene_t;

static int scene_build(scene_t *sc, const oracle_scene_desc *d)
{
    memset(sc, 0, sizeof(*sc));
    if (d->dim != 2 && d->dim != 3) return -1;
    sc->dim = d->dim;
    if (geom_build(&sc->neu, d->dim, d->n_vertices, d->n_prims, d->vertices, d->prims, 1, d->is_double_sided)) return -1;
    if (geom_build(&sc->dir, d->dim, d->n_dvertices, d->n_dprims, d->dvertices, d->dprims, 0, d->is_double_sided)) return -1;
    if (geom_build_fcpw_bvh(&sc->neu, ORACLE_FCPW_BRANCH, ORACLE_FCPW_LEAF)) return -1;
    /* computeBoundingBox (fcpw_scene_loader.h:75-93), BoundingBox::expandToInclude pads by FLT_EPSILON */
    for (int k = 0; k < 3; k++) { sc->pmin[k] = FLT_MAX; sc->pmax[k] = -FLT_MAX; }
    const geom_t *gs[2] = {&sc->neu, &sc->dir};
    for (int q = 0; q < 2; q++) for (int i = 0; i < gs[q]->nv; i++) for (int k = 0; k < d->dim; k++) {
        float lo = gs[q]->v[i][k] - FEPS, hi = gs[q]->v[i][k] + FEPS;
        sc->pmin[k] = sminf(sc->pmin[k], lo);   /* cwiseMin */
        sc->pmax[k] = smaxf(sc->pmax[k], hi);
    }
    if (d->dim == 2) { sc->pmin[2] = sc->pmax[2] = 0.0f; }
    for (int k = 0; k < 3; k++) sc->ext[k] = sc->pmax[k] - sc->pmin[k];
    sc->g_dirichlet = d->dirichlet_value;
    sc->absorption = d->absorption;
    sc->watertight = d->is_watertight; sc->double_sided = d->is_double_sided;
    sc->src = d->source;
    for (int k = 0; k < 3; k++) sc->sdims[k] = d->source_dims[k];
    if (d->dirichlet_image) {
        if (d->dim != 2 || d->dirichlet_image_dims[0] < 1 || d->dirichlet_image_dims[1] < 1) return -1;
        sc->dimg = d->dirichlet_image;
        sc->ddims[0] = d->dirichlet_image_dims[0]; sc->ddims[1] = d->dirichlet_image_dims[1];
        for (int k = 0; k < 4; k++) sc->dbox[k] = d->dirichlet_image_box[k];
        if (!(sc->dbox[2] > 0.0f) || !(sc->dbox[3] > 0.0f)) return -1;
    }
    if (d->neumann_image) {
        if (d->dim != 2 || d->neumann_image_dims[0] < 1 || d->neumann_image_dims[1] < 1) return -1;
        sc->nimg = d->neumann_image;
        sc->ndims[0] = d->neumann_image_dims[0]; sc->ndims[1] = d->neumann_image_dims[1];
        for (int k = 0; k < 4; k++) sc->nbox[k] = d->neumann_image_box[k];
        if (!(sc->nbox[2] > 0.0f) || !(sc->nbox[3] > 0.0f)) return -1;
    }
    return 0;
}

static void scene_free(scene_t *sc) { geom_free(&sc->neu); geom_free(&sc->dir); }

int oracle_fcpw_pick(const oracle_scene_desc *scene, const float *x, float R, int n, const float *us, int32_t *sel,
                     float *pdf)
{
    scene_t sc;
    if (scene_build(&sc, scene)) { scene_free(&sc); return -3; }
    if (sc.neu.np <= 0) { scene_free(&sc); return -1; }
    for (int i = 0; i < n; i++) { pdf[i] = 0.0f; sel[i] = fcpw_stochastic_pick(&sc.neu, x, R, us[i], &pdf[i]); }
    scene_free(&sc);
    return 0;
}

/* computeDistToDirichlet (fcpw_scene_loader.h:299-315) */
static float dist_dirichlet(const scene_t *sc, const float *x, int signed_)
{
    if (sc->dir.np > 0) {
        cp_t c; closest_point(&sc->dir, x, &c, signed_);
        return signed_ ? signed_distance(&c, x) : c.d;
    }
    float u[3], v[3], m[3];
    sub3(u, sc->pmin, x); sub3(v, x, sc->pmax);
    for (int k = 0; k < 3; k++) m[k] = sminf(u[k], v[k]);
    if (sc->dim == 2) m[2] = 0.0f;
    return sqrtf(dot3(m, m));
}

/* computeDistToNeumann (fcpw_scene_loader.h:316-330) */
static float dist_neumann(const scene_t *sc, const float *x, int signed_)
{
    if (sc->neu.np > 0) {
        cp_t c; closest_point(&sc->neu, x, &c, signed_);
        return signed_ ? signed_distance(&c, x) : c.d;
    }
    return FLT_MAX;
}

/* insideDomain (fcpw_scene_loader.h:642-648) */
static int inside_domain(const scene_t *sc, const float *x)
{
    if (!sc->watertight) return 1;
    float d1 = dist_dirichlet(sc, x, 1), d2 = dist_neumann(sc, x, 1);
    return fabsf(d1) < fabsf(d2) ? d1 < 0.0f : d2 < 0.0f;
}

static int outside_bbox(const scene_t *sc, const float *x)
{
    for (int k = 0; k < sc->dim; k++) if (!(x[k] >= sc->pmin[k] && x[k] <= sc->pmax[k])) return 1;
    return 0;
}

/* PDE source: scene.h:194-198 + image.h:53-58 (2D), scene_3d.h:120-126 (3D) */
static float source_value(const scene_t *sc, const float *x)
{
    if (!sc->src) return 0.0f;
    if (sc->dim == 2) {
        float ux = (x[0] - sc->pmin[0]) / sc->ext[0];
        float uy = (x[1] - sc->pmin[1]) / sc->ext[1];
        int h = sc->sdims[0], w = sc->sdims[1];
        int i = sclampi(cvt_trunc(uy * (float)h), 0, h - 1);
        int j = sclampi(cvt_trunc(ux * (float)w), 0, w - 1);
        return sc->src[(size_t)i * w + j];
    }
    int X = sc->sdims[0], Y = sc->sdims[1], Z = sc->sdims[2];
    float ux = (x[0] - sc->pmin[0]) / sc->ext[0];
    float uy = (x[1] - sc->pmin[1]) / sc->ext[1];
    float uz = (x[2] - sc->pmin[2]) / sc->ext[2];
    int i = sclampi(cvt_trunc(ux * (float)X), 0, X - 1);
    int j = sclampi(cvt_trunc(uy * (float)Y), 0, Y - 1);
    int k = sclampi(cvt_trunc(uz * (float)Z), 0, Z - 1);
    return sc->src[((size_t)i * Y + j) * Z + k];
}

/* ------------------------------------------------------------------------- */
/* g at a walk's last position: setTerminalContribution (walk_on_stars.h:331-351) projects it
 * onto the Dirichlet boundary (projectToDirichlet, fcpw_scene_loader.h:345-364: findClosestPoint,
 * the same `<=` scan as computeDistToDirichlet) and evaluates pde.dirichlet there: the upstream
 * setPDE the fork keeps commented (scene.h:202-207), uv = (x - pMin) / maxLength -- here
 * (x - box origin) / box extent per axis, which is that with extent = (maxLength, maxLength) --
 * then Image::get (image.h:53-58: i = clamp(int(uv.y * h)), j = clamp(int(uv.x * w))). */
static float dirichlet_value(const scene_t *sc, const float *x)
{
    if (!sc->dimg) return sc->g_dirichlet;
    cp_t c;
    if (closest_point(&sc->dir, x, &c, 0) < 0) return sc->g_dirichlet;
    float ux = (c.p[0] - sc->dbox[0]) / sc->dbox[2];
    float uy = (c.p[1] - sc->dbox[1]) / sc->dbox[3];
    int h = sc->ddims[0], w = sc->ddims[1];
    int i = sclampi(cvt_trunc(uy * (float)h), 0, h - 1);
    int j = sclampi(cvt_trunc(ux * (float)w), 0, w - 1);
    return sc->dimg[(size_t)i * w + j];
}

/* h at a Neumann boundary sample y: the upstream demo's pde.neumann (scene.h:175-181, commented
 * in the fork: uv = (y - bbox.pMin) / bbox.extent()) over the image's box, then Image::get
 * (image.h:53-58); pde.neumannDoubleSided reads the same image for either side. */
static float neumann_value(const scene_t *sc, const float *y)
{
    if (!sc->nimg) return 0.0f;
    float ux = (y[0] - sc->nbox[0]) / sc->nbox[2];
    float uy = (y[1] - sc->nbox[1]) / sc->nbox[3];
    int h = sc->ndims[0], w = sc->ndims[1];
    int i = sclampi(cvt_trunc(uy * (float)h), 0, h - 1);
    int j = sclampi(cvt_trunc(ux * (float)w), 0, w - 1);
    return sc->nimg[(size_t)i * w + j];
}

/* ------------------------------------------------------------------------- */
/* Green's functions on balls (distributions.h:273-832)                       */
/* ------------------------------------------------------------------------- */
typedef struct {
    int dim, yukawa;
    float c[3], yVol[3], ySurf[3];
    float R, r, rClamp;
    float lambda, sqrtLambda;
    float muR, K0muR, I0muR, K1muR, I1muR;       /* 2D */
    float expmuR, sinhmuR, K32muR, I32muR;       /* 3D */
    int scaled;  /* robust mode, mu R > ROBUST_MUR: 2D members hold ke0 ie0 ke1 ie1 of mu R */
} gfn_t;

static void gfn_init(gfn_t *g, int dim, int yukawa, float lambda)
{
    memset(g, 0, sizeof(*g));
    g->dim = dim; g->yukawa = yukawa; g->lambda = lambda; g->sqrtLambda = sqrtf(lambda);
    g->rClamp = 1e-4f;
}

static void gfn_update_ball(gfn_t *g, const float *c, float R)
{
    memcpy(g->c, c, 12);
    memset(g->yVol, 0, 12); memset(g->ySurf, 0, 12);
    g->R = R; g->r = 0.0f; g->rClamp = 1e-4f;
    if (!g->yukawa) return;
    g->muR = R * g->sqrtLambda;
    g->scaled = g_robust && g->muR > ROBUST_MUR;
    if (g->scaled) {  /* 3D scaled balls evaluate everything from mu R */
        if (g->dim == 2) {
            double ie0, ke0, ie1, ke1;
            bess_scaled((double)g->muR, &ie0, &ke0, &ie1, &ke1);
            g->K0muR = (float)ke0; g->I0muR = (float)ie0; g->K1muR = (float)ke1; g->I1muR = (float)ie1;
        }
        return;
    }
    if (g->dim == 2) {
        g->K0muR = (float)bessk0((double)g->muR);
        g->I0muR = (float)bessi0((double)g->muR);
        g->K1muR = (float)bessk1((double)g->muR);
        g->I1muR = (float)bessi1((double)g->muR);
    } else {
        g->expmuR = m_expf(-g->muR);
        float exp2muR = g->expmuR * g->expmuR;
        float coshmuR = (1.0f + exp2muR) / (2.0f * g->expmuR);
        g->sinhmuR = (1.0f - exp2muR) / (2.0f * g->expmuR);
        g->K32muR = g->expmuR * (1.0f + 1.0f / g->muR);
        g->I32muR = coshmuR - g->sinhmuR / g->muR;
    }
}

/* robust-mode forms of the members below (g->scaled): the reference's expressions
 * rewritten with ie/ke and e^{2(mu r - mu R)} <= 1, in double, rounded where the
 * reference rounds its result */
static double scaled_q0(const gfn_t *g, float mur)  /* 2D K0(mur) - I0(mur) K0(muR)/I0(muR); 3D e^-mur - e^-muR sinh(mur)/sinh(muR) */
{
    double x = (double)mur, X = (double)g->muR;
    if (g->dim == 2) {
        double ie0, ke0, ie1, ke1;
        bess_scaled(x, &ie0, &ke0, &ie1, &ke1);
        return m_exp(-x) * (ke0 - ie0 * ((double)g->K0muR / (double)g->I0muR) * m_exp(2.0 * (x - X)));
    }
    return m_exp(-x) - m_exp(x - 2.0 * X) * (1.0 - m_exp(-2.0 * x)) / (1.0 - m_exp(-2.0 * X));
}

static float gfn_evaluate(const gfn_t *g)
{
    if (g->yukawa && g->scaled) {
        float mur = g->r * g->sqrtLambda;
        double q = scaled_q0(g, mur);
        if (g->dim == 2) return (float)(q / TWO_PI_D);
        return (float)(q / (FOUR_PI_D * (double)g->r));
    }
    float r = g->r, R = g->R;
    if (!g->yukawa) {
        if (g->dim == 2) return (float)((double)m_logf(R / r) / TWO_PI_D);
        return (float)((double)(1.0f / r - 1.0f / R) / FOUR_PI_D);
    }
    float mur = r * g->sqrtLambda;
    if (g->dim == 2) {
        float K0mur = (float)bessk0((double)mur);
        float I0mur = (float)bessi0((double)mur);
        return (float)((double)(K0mur - I0mur * g->K0muR / g->I0muR) / TWO_PI_D);
    }
    float expmur = m_expf(-mur);
    float sinhmur = (1.0f - expmur * expmur) / (2.0f * expmur);
    return (float)((double)(expmur - g->expmuR * sinhmur / g->sinhmuR) / (FOUR_PI_D * (double)r));
}

static float gfn_poisson_kernel(const gfn_t *g)
{
    if (!g->yukawa) return g->dim == 2 ? (float)(1.0 / TWO_PI_D) : (float)(1.0 / FOUR_PI_D);
    if (g->scaled) {
        double X = (double)g->muR;
        if (g->dim == 2) return (float)(m_exp(-X) / (TWO_PI_D * (double)g->I0muR));
        return (float)(X * 2.0 * m_exp(-X) / (FOUR_PI_D * (1.0 - m_exp(-2.0 * X))));
    }
    if (g->dim == 2) return (float)(1.0 / (TWO_PI_D * (double)g->I0muR));
    return (float)((double)g->muR / (FOUR_PI_D * (double)g->sinhmuR));
}

static float gfn_norm(const gfn_t *g)
{
    if (!g->yukawa) return g->dim == 2 ? g->R * g->R / 4.0f : g->R * g->R / 6.0f;
    double pk = (double)gfn_poisson_kernel(g);
    if (g->dim == 2) return (float)((1.0 - TWO_PI_D * pk) / (double)g->lambda);
    return (float)((1.0 - FOUR_PI_D * pk) / (double)g->lambda);
}

static float gfn_gradient_norm(const gfn_t *g)
{
    float r = g->r, R = g->R;
    if (!g->yukawa) {
        if (g->dim == 2) { float r2 = r * r; return (float)((double)(1.0f / r2 - 1.0f / (R * R)) / TWO_PI_D); }
        float r3 = r * r * r; return (float)((double)(1.0f / r3 - 1.0f / (R * R * R)) / FOUR_PI_D);
    }
    float mur = r * g->sqrtLambda;
    if (g->scaled) {
        double x = (double)mur, X = (double)g->muR, t = m_exp(2.0 * (x - X)), q;
        if (g->dim == 2) {
            double ie0, ke0, ie1, ke1;
            bess_scaled(x, &ie0, &ke0, &ie1, &ke1);
            q = m_exp(-x) * (ke1 - ie1 * ((double)g->K1muR / (double)g->I1muR) * t);
            return (float)((double)g->sqrtLambda * q / (TWO_PI_D * (double)r));
        }
        q = m_exp(-x) * ((1.0 + 1.0 / x) - i32s(x) * ((1.0 + 1.0 / X) / i32s(X)) * t);
        return (float)((double)g->sqrtLambda * q / (FOUR_PI_D * (double)(r * r)));
    }
    if (g->dim == 2) {
        float K1mur = (float)bessk1((double)mur);
        float I1mur = (float)bessi1((double)mur);
        float Qr = g->sqrtLambda * (K1mur - I1mur * g->K1muR / g->I1muR);
        return (float)((double)Qr / (TWO_PI_D * (double)r));
    }
    float r2 = r * r;
    float expmur = m_expf(-mur);
    float exp2mur = expmur * expmur;
    float coshmur = (1.0f + exp2mur) / (2.0f * expmur);
    float sinhmur = (1.0f - exp2mur) / (2.0f * expmur);
    float K32mur = expmur * (1.0f + 1.0f / mur);
    float I32mur = coshmur - sinhmur / mur;
    float Qr = g->sqrtLambda * (K32mur - I32mur * g->K32muR / g->I32muR);
    return (float)((double)Qr / (FOUR_PI_D * (double)r2));
}

static void gfn_gradient(const gfn_t *g, float *out)
{
    float gn = gfn_gradient_norm(g);
    for (int k = 0; k < g->dim; k++) out[k] = (g->yVol[k] - g->c[k]) * gn;
}

static void gfn_poisson_kernel_gradient(const gfn_t *g, float *out)
{
    float d[3]; for (int k = 0; k < 3; k++) d[k] = g->ySurf[k] - g->c[k];
    if (!g->yukawa) {
        if (g->dim == 2) {
            float s = (float)((TWO_PI_D * (double)g->R) * (double)g->R);
            for (int k = 0; k < 2; k++) out[k] = (2.0f * d[k]) / s;
        } else {
            float s = (float)((FOUR_PI_D * (double)g->R) * (double)g->R);
            for (int k = 0; k < 3; k++) out[k] = (3.0f * d[k]) / s;
        }
        return;
    }
    if (g->scaled) {
        double X = (double)g->muR;
        float QR = g->dim == 2 ? (float)((double)g->sqrtLambda * m_exp(-X) / ((double)g->R * (double)g->I1muR))
                               : (float)((double)g->lambda * m_exp(-X) / i32s(X));
        for (int k = 0; k < g->dim; k++) out[k] = (d[k] * QR) / (float)(g->dim == 2 ? TWO_PI_D : FOUR_PI_D);
        return;
    }
    if (g->dim == 2) {
        float QR = g->sqrtLambda / (g->R * g->I1muR);
        for (int k = 0; k < 2; k++) out[k] = (d[k] * QR) / (float)TWO_PI_D;
    } else {
        float QR = g->lambda / g->I32muR;
        for (int k = 0; k < 3; k++) out[k] = (d[k] * QR) / (float)FOUR_PI_D;
    }
}

static float gfn_dir_sampled_poisson_kernel(const gfn_t *g, const float *y)
{
    if (!g->yukawa) return 1.0f;
    float d[3] = {0, 0, 0}; for (int k = 0; k < g->dim; k++) d[k] = y[k] - g->c[k];
    float r = smaxf(g->rClamp, norm3(d));
    float mur = r * g->sqrtLambda;
    if (g->scaled) {
        double x = (double)mur, X = (double)g->muR, t = m_exp(2.0 * (x - X)), q;
        if (g->dim == 2) {
            double ie0, ke0, ie1, ke1;
            bess_scaled(x, &ie0, &ke0, &ie1, &ke1);
            q = ke1 + ie1 * ((double)g->K0muR / (double)g->I0muR) * t;
        } else {
            q = (1.0 + 1.0 / x) + i32s(x) * (2.0 / (1.0 - m_exp(-2.0 * X))) * t;
        }
        return (float)(x * m_exp(-x) * q);
    }
    if (g->dim == 2) {
        float K1mur = (float)bessk1((double)mur);
        float I1mur = (float)bessi1((double)mur);
        float Q = K1mur + I1mur * g->K0muR / g->I0muR;
        return mur * Q;
    }
    float expmur = m_expf(-mur);
    float exp2mur = expmur * expmur;
    float coshmur = (1.0f + exp2mur) / (2.0f * expmur);
    float sinhmur = (1.0f - exp2mur) / (2.0f * expmur);
    float K32mur = expmur * (1.0f + 1.0f / mur);
    float I32mur = coshmur - sinhmur / mur;
    float Q = K32mur + I32mur * g->expmuR / g->sinhmuR;
    return mur * Q;
}

/* off-centred G(x,y), distributions.h:458-464,532-537,612-632,760-776 */
static float gfn_evaluate_xy(const gfn_t *g, const float *x, const float *y)
{
    float yx[3] = {0, 0, 0}, xc[3] = {0, 0, 0}, yc[3] = {0, 0, 0};
    for (int k = 0; k < g->dim; k++) { yx[k] = y[k] - x[k]; xc[k] = x[k] - g->c[k]; yc[k] = y[k] - g->c[k]; }
    float R = g->R;
    if (!g->yukawa) {
        float r = smaxf(g->rClamp, norm3(yx));
        if (g->dim == 2) return (float)((double)(m_logf(R * R - dot3(xc, yc)) - m_logf(R * r)) / TWO_PI_D);
        return (float)((double)(1.0f / r - R / (R * R - dot3(xc, yc))) / FOUR_PI_D);
    }
    float r1 = smaxf(g->rClamp, norm3(yx));
    float r2 = (R * R - dot3(xc, yc)) / R;
    float mur1 = r1 * g->sqrtLambda, mur2 = r2 * g->sqrtLambda;
    if (g->scaled) {
        double q1 = scaled_q0(g, mur1), q2 = scaled_q0(g, mur2);
        if (g->dim == 2) return (float)((q1 - q2) / TWO_PI_D);
        return (float)((q1 / (double)r1 - q2 / (double)r2) / FOUR_PI_D);
    }
    if (g->dim == 2) {
        float K0mur1 = (float)bessk0((double)mur1), K0mur2 = (float)bessk0((double)mur2);
        float I0mur1 = (float)bessi0((double)mur1), I0mur2 = (float)bessi0((double)mur2);
        float Q1 = K0mur1 - I0mur1 * g->K0muR / g->I0muR;
        float Q2 = K0mur2 - I0mur2 * g->K0muR / g->I0muR;
        return (float)((double)(Q1 - Q2) / TWO_PI_D);
    }
    float e1 = m_expf(-mur1), e2 = m_expf(-mur2);
    float s1 = (1.0f - e1 * e1) / (2.0f * e1), s2 = (1.0f - e2 * e2) / (2.0f * e2);
    float Q1 = (e1 - g->expmuR * s1 / g->sinhmuR) / r1;
    float Q2 = (e2 - g->expmuR * s2 / g->sinhmuR) / r2;
    return (float)((double)(Q1 - Q2) / FOUR_PI_D);
}

static inline float pdf_sphere_uniform(int dim, float r)
{
    if (dim == 2) return (float)(1.0 / (TWO_PI_D * (double)r));
    return (float)(1.0 / ((FOUR_PI_D * (double)r) * (double)r));
}

static void sample_unit_sphere(int dim, const float *u, float *out)
{
    if (dim == 2) {
        float phi = (float)(TWO_PI_D * (double)u[0]);
        out[0] = m_cosf(phi); out[1] = m_sinf(phi); out[2] = 0.0f;
    } else {
        float z = 1.0f - 2.0f * u[0];
        float r = sqrtf(smaxf(0.0f, 1.0f - z * z));
        float phi = (float)(TWO_PI_D * (double)u[1]);
        out[0] = r * m_cosf(phi); out[1] = r * m_sinf(phi); out[2] = z;
    }
}

/* sampleVolume (distributions.h:404-410,486-500,591-599,710-720) + rejectionSampleGreensFn (362-383) */
static void gfn_sample_volume(gfn_t *g, const float *dir, pcg_t *s, float *pdf, float *out, uint64_t *iters)
{
    float R = g->R;
    if (!g->yukawa && g->dim == 3) {
        float u1 = pcg_float(s), u2 = pcg_float(s);
        float phi = (float)(TWO_PI_D * (double)u2);
        float r = (1.0f + sqrtf(1.0f - m_cbrtf(u1 * u1)) * m_cosf(phi)) * R / 2.0f;
        r = smaxf(g->rClamp, r);
        if (r > R) r = R / 2.0f;
        g->r = r;
        for (int k = 0; k < 3; k++) g->yVol[k] = g->c[k] + r * dir[k];
        *pdf = gfn_evaluate(g) / gfn_norm(g);
        memcpy(out, g->yVol, 12);
        return;
    }
    float bound;
    if (!g->yukawa) bound = 1.5f / R;
    else {
        float a = g->dim == 2 ? 2.2f : 2.0f, b = g->dim == 2 ? 0.6f : 0.5f;
        float lam = g->lambda, sl = g->sqrtLambda;
        bound = R <= lam ? smaxf(smaxf(a / R, a / lam), smaxf(b * sqrtf(R), b * sl))
                         : smaxf(sminf(a / R, a / lam), sminf(b * sqrtf(R), b * sl));
    }
    int iter = 0;
    do {
        float u = pcg_float(s);
        g->r = pcg_float(s) * R;
        *pdf = gfn_evaluate(g) / gfn_norm(g);
        float pdfRadius = *pdf / pdf_sphere_uniform(g->dim, g->r);
        iter++;
        if (u < pdfRadius / bound) break;
    } while (iter < 1000);
    *iters += (uint64_t)iter;
    g->r = smaxf(g->rClamp, g->r);
    if (g->r > R) g->r = R / 2.0f;
    for (int k = 0; k < 3; k++) g->yVol[k] = g->c[k] + g->r * dir[k];
    if (g->dim == 2) g->yVol[2] = 0.0f;
    memcpy(out, g->yVol, 12);
}

/* ------------------------------------------------------------------------- */
/* walk                                                                      */
/* ------------------------------------------------------------------------- */
enum { WC_DIRICHLET = 0, WC_RR = 1, WC_MAXLEN = 2, WC_ESCAPED = 3 };

typedef struct {
    float pt[3], n[3], prevDir[3];
    float prevDist, throughput;
    int onNeumann, walkLength;
    float terminal, totalNeumann, totalSource, firstSource;
    float sdir[3], bdir[3];
} wstate_t;

typedef struct {
    uint64_t steps, iters;
} wcount_t;

/* Neumann boundary sample + contribution (walk_on_stars.h:212-260).  With the
 * reference's h == 0 (scene.h:176-181) the term is exactly +0 unless G or the
 * throughput is non-finite; only then is the stochastic sample run.  Image-valued
 * h (sc->nimg) runs it at every step.  `flip`: the step flipped the walk's normal
 * (flipNormalOrientation, double-sided scenes); `prec`: silhouettePrecision. */
static void neumann_term(const scene_t *sc, const gfn_t *g, wstate_t *st, float R, const float *rn, int flip,
                         float prec)
{
    const geom_t *ng = &sc->neu;
    int nonfinite = !isfinite(st->throughput) || (g->yukawa && !g->scaled && g->muR > 85.0f);
    if ((!nonfinite && !sc->nimg) || ng->np <= 0) return;
    const float *x = st->pt;
    /* sampleNeumann: fcpw's stochastic traversal picks the primitive (randNums[0]) */
    float sel_pdf = 0.0f;
    int sel = fcpw_stochastic_pick(ng, x, R, rn[0], &sel_pdf);
    if (sel < 0) return;
    float sp[3], sn[3], pdf;
    if (ng->dim == 2) {
        const float *pa = ng->v[ng->ix[sel][0]], *pb = ng->v[ng->ix[sel][1]];
        float s[3]; sub3(s, pb, pa);
        float area = norm3(s), u = rn[1];
        for (int k = 0; k < 3; k++) sp[k] = pa[k] + u * s[k];
        sn[0] = s[1] / area; sn[1] = -s[0] / area; sn[2] = 0.0f;
        pdf = 1.0f / area;
    } else {
        const float *pa = ng->v[ng->ix[sel][0]], *pb = ng->v[ng->ix[sel][1]], *pc = ng->v[ng->ix[sel][2]];
        float v1[3], v2[3]; sub3(v1, pb, pa); sub3(v2, pc, pa); cross3(sn, v1, v2);
        float area = norm3(sn);
        float u1 = sqrtf(rn[1]), u2 = rn[2], u = 1.0f - u1, v = u2 * u1, w = 1.0f - u - v;
        for (int k = 0; k < 3; k++) { sp[k] = pa[k] * u + pb[k] * v + pc[k] * w; sn[k] /= area; }
        pdf = 2.0f / area;
    }
    /* Interaction::d: (weight * traversalPdf) / total, then *= samplePoint's pdf */
    pdf = sel_pdf * pdf;
    float dts[3]; sub3(dts, sp, x);
    if (sc->dim == 2) dts[2] = 0.0f;
    float distToSample = norm3(dts);
    float alpha = st->onNeumann ? 2.0f : 1.0f;
    if (sc->double_sided) {
        /* the sample normal faces the walk (walk_on_stars.h:219-247): flipped with the walk's
         * normal, or when the sample lies behind it beyond the precision band -- on a concave
         * boundary (alpha 2) only when it also lies behind the walk's own normal */
        float ds[3];
        for (int k = 0; k < 3; k++) ds[k] = dts[k] / distToSample;
        if (sc->dim == 2) ds[2] = 0.0f;
        if (flip) {
            for (int k = 0; k < 3; k++) sn[k] *= -1.0f;
        } else if (dot3(ds, sn) < -prec) {
            int f = 1;
            if (alpha > 1.0f) f = dot3(ds, st->n) < -prec;
            if (f) for (int k = 0; k < 3; k++) sn[k] *= -1.0f;
        }
    }
    if (pdf > 0.0f && distToSample < R) {
        /* intersectsWithNeumann (fcpw_scene_loader.h:485-499) -> hasLineOfSight (primitive.h:225-235) */
        float p1[3], p2[3], mn[3];
        for (int k = 0; k < 3; k++) mn[k] = -st->n[k];
        if (st->onNeumann) offset_point(sc->dim, x, mn, p1); else memcpy(p1, x, 12);
        for (int k = 0; k < 3; k++) mn[k] = -sn[k];
        offset_point(sc->dim, sp, mn, p2);
        float dd[3]; sub3(dd, p2, p1);
        float dn = norm3(dd);
        for (int k = 0; k < 3; k++) dd[k] /= dn;
        hit_t h;
        int occluded = ray_first_hit(ng, p1, dd, dn, &h, 1);
        if (!occluded) {
            float G = gfn_evaluate_xy(g, x, sp);
            float hval = neumann_value(sc, sp);
            st->totalNeumann += st->throughput * alpha * G * hval / pdf;
        }
    }
}

/* walk() (walk_on_stars.h:135-329); first_r > 0: the first step's sphere radius is
 * given (firstSphereRadius of estimateSolution, :148-150) -- no flip, no query */
static int walk(const scene_t *sc, const oracle_params *prm, float dirichletDist, float first_r,
                pcg_t *smp, gfn_t *g, wstate_t *st, wcount_t *cnt)
{
    const int dim = sc->dim;
    int firstStep = 1;
    while (dirichletDist > prm->epsilon_shell) {
        float starRadius;
        int flip = 0;
        if (firstStep && first_r > 0.0f) {
            starRadius = first_r;
        } else {
        if (sc->double_sided && st->onNeumann) {
            float dp = 0.0f; for (int k = 0; k < dim; k++) dp += st->prevDir[k] * st->n[k];
            if (st->prevDist > 0.0f && dp < 0.0f) { for (int k = 0; k < dim; k++) st->n[k] *= -1.0f; flip = 1; }
        }
        if (prm->steps_before_maximal_spheres <= st->walkLength) {
            starRadius = dirichletDist;
        } else {
            starRadius = star_radius(&sc->neu, st->pt, prm->min_star_radius, dirichletDist,
                                     prm->silhouette_precision, flip);
            if (prm->min_star_radius <= dirichletDist)
                starRadius = smaxf(0.99f * starRadius, prm->min_star_radius);
        }
        }
        gfn_update_ball(g, st->pt, starRadius);
        cnt->steps++;
        float u[2] = {pcg_float(smp), 0.0f};
        if (dim == 3) u[1] = pcg_float(smp);
        float dir[3]; sample_unit_sphere(dim, u, dir);
        float nd = 0.0f; for (int k = 0; k < dim; k++) nd += st->n[k] * dir[k];
        if (st->onNeumann && nd > 0.0f) for (int k = 0; k < dim; k++) dir[k] *= -1.0f;

        hit_t ip; memset(&ip, 0, sizeof(ip)); ip.d = FLT_MAX;
        int hit = 0;
        if (sc->neu.np > 0) {
            float o[3];
            if (st->onNeumann) { float mn[3] = {-st->n[0], -st->n[1], -st->n[2]}; offset_point(dim, st->pt, mn, o); }
            else memcpy(o, st->pt, 12);
            hit = ray_first_hit(&sc->neu, o, dir, starRadius, &ip, 0);
        }
        if (!hit) {
            float cp[3];
            if (st->onNeumann) { float mn[3] = {-st->n[0], -st->n[1], -st->n[2]}; offset_point(dim, st->pt, mn, cp); }
            else memcpy(cp, st->pt, 12);
            for (int k = 0; k < 3; k++) ip.p[k] = cp[k] + starRadius * dir[k];
            if (dim == 2) ip.p[2] = 0.0f;
            ip.d = starRadius;
            ip.n[0] = ip.n[1] = ip.n[2] = 0.0f;
        }
        if (!prm->ignore_neumann) {
            float rn[3] = {0, 0, 0};
            for (int k = 0; k < dim; k++) rn[k] = pcg_float(smp);
            neumann_term(sc, g, st, starRadius, rn, flip, prm->silhouette_precision);
        }
        if (!prm->ignore_source) {
            float pdf, sp[3];
            gfn_sample_volume(g, dir, smp, &pdf, sp, &cnt->iters);
            if (g->r <= ip.d) {
                float contrib = gfn_norm(g) * source_value(sc, sp);
                st->totalSource += st->throughput * contrib;
            }
        }
        if (!hit && outside_bbox(sc, ip.p)) return WC_ESCAPED;
        st->prevDist = ip.d;
        memcpy(st->prevDir, dir, 12);
        memcpy(st->pt, ip.p, 12);
        memcpy(st->n, ip.n, 12);
        st->onNeumann = hit;
        st->throughput *= gfn_dir_sampled_poisson_kernel(g, st->pt);
        if (st->throughput < prm->russian_roulette_threshold) {
            float survival = st->throughput / prm->russian_roulette_threshold;
            if (survival < pcg_float(smp)) { st->throughput = 0.0f; return WC_RR; }
            st->throughput = prm->russian_roulette_threshold;
        }
        st->walkLength++;
        if (st->walkLength > prm->max_walk_length) return WC_MAXLEN;
        if (sc->absorption > 0.0f && prm->steps_before_tikhonov == st->walkLength) {
            gfn_init(g, dim, 1, sc->absorption);
        }
        dirichletDist = dist_dirichlet(sc, st->pt, 0);
        firstStep = 0;
    }
    return WC_DIRICHLET;
}

/* ------------------------------------------------------------------------- */
/* statistics (walk_on_stars.h:744-877)                                       */
/* ------------------------------------------------------------------------- */
typedef struct {
    float solMean, solM2, gMean[3], gM2[3], totalFirst, totalDeriv;
    int nSol, nGrad, totalLen;
} stats_t;

static inline void welford(float est, float *mean, float *M2, int N)
{
    float delta = est - *mean;
    *mean += delta / (float)N;
    float delta2 = est - *mean;
    *M2 += delta * delta2;
}

/* ------------------------------------------------------------------------- */
/* estimateSolutionAndGradient (walk_on_stars.h:466-617)                      */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint64_t steps, wasted, rec, esc, maxl, rr, dir, iters;
} pcount_t;

static void estimate_point(const scene_t *sc, const oracle_params *prm, const float *x, uint64_t gidx,
                           float dDist, float nDist, stats_t *S, pcount_t *pc, const float *ddir)
{
    const int dim = sc->dim;
    int nWalks = prm->n_walks, nAnti = 1;
    int useAnti = !prm->disable_gradient_antithetic_variates;
    int useCV = !prm->disable_gradient_control_variates;
    memset(S, 0, sizeof(*S));
    if (useAnti) { nWalks = nWalks / 2; if (nWalks < 1) nWalks = 1; nAnti = 2; }
    float boundaryDist = sminf(dDist, nDist);
    float firstR = 0.99f * boundaryDist;
    int sd = dim - 1;
    float *strat = malloc(sizeof(float) * (size_t)sd * 2 * nWalks);
    {
        pcg_t ps; pcg_seed(&ps, oracle_seed32(prm->seed, gidx, 0, 0), 1u);
        gen_stratified(strat, 2 * nWalks, sd, &ps);
    }
    /* SampleEstimationData::directionForDerivative: (1, 0[, 0]) by default (walk_on_stars.h:
     * 665-666); BVC's Dirichlet samples pass their normal (boundary_sampler.h:154-166) */
    const float dirForDeriv[3] = {ddir ? ddir[0] : 1.0f, ddir ? ddir[1] : 0.0f, ddir && dim == 3 ? ddir[2] : 0.0f};
    int yuk0 = sc->absorption > 0.0f && prm->steps_before_tikhonov == 0;
    for (int w = 0; w < nWalks; w++) {
        float boundaryPdf = 0.0f, sourcePdf = 0.0f, boundaryPt[3] = {0, 0, 0}, sourcePt[3] = {0, 0, 0};
        pcg_t fs; pcg_seed(&fs, oracle_seed32(prm->seed, gidx, (uint64_t)w, 1), 1u);
        uint32_t wseed = oracle_seed32(prm->seed, gidx, (uint64_t)w, 2);
        float cvb = 0.0f, cvs = 0.0f;
        if (useCV) { cvb = S->solMean; int N = S->nSol > 1 ? S->nSol : 1; cvs = S->totalFirst / (float)N; }
        for (int a = 0; a < nAnti; a++) {
            gfn_t g; gfn_init(&g, dim, yuk0, sc->absorption);
            wstate_t st; memset(&st, 0, sizeof(st));
            memcpy(st.pt, x, 12); st.throughput = 1.0f;
            gfn_update_ball(&g, st.pt, firstR);
            uint64_t stepsBefore = 1;
            if (!prm->ignore_source) {
                if (a == 0) {
                    float dir[3]; sample_unit_sphere(dim, &strat[sd * (2 * w + 0)], dir);
                    gfn_sample_volume(&g, dir, &fs, &sourcePdf, sourcePt, &pc->iters);
                } else {
                    float sdv[3] = {0, 0, 0};
                    for (int k = 0; k < dim; k++) sdv[k] = sourcePt[k] - st.pt[k];
                    for (int k = 0; k < dim; k++) g.yVol[k] = st.pt[k] - sdv[k];
                    g.r = norm3(sdv);
                }
                float gnorm = gfn_norm(&g);
                float contrib = gnorm * source_value(sc, g.yVol);
                st.totalSource += st.throughput * contrib;
                st.firstSource = contrib;
                float gr[3] = {0, 0, 0}; gfn_gradient(&g, gr);
                float den = sourcePdf * gnorm;
                for (int k = 0; k < dim; k++) st.sdir[k] = gr[k] / den;
            }
            if (a == 0) {
                const float *u = &strat[sd * (2 * w + 1)];
                float bd[3] = {0, 0, 0};
                if (prm->use_cosine_sampling) {
                    if (dim == 2) {
                        float u1 = 2.0f * u[0] - 1.0f;
                        bd[0] = u1; bd[1] = sqrtf(smaxf(0.0f, 1.0f - u1 * u1));
                    } else {
                        float u1 = 2.0f * u[0] - 1.0f, u2 = 2.0f * u[1] - 1.0f, dx = 0.0f, dy = 0.0f;
                        if (!(u1 == 0 && u2 == 0)) {
                            /* sampleUnitDiskConcentric (sampling.h:122-146) */
                            float theta, r;
                            if (fabsf(u1) > fabsf(u2)) { r = u1; theta = (float)(0.25 * PI_D * (double)(u2 / u1)); }
                            else { r = u2; theta = (float)(0.5 * PI_D * (double)(1.0f - 0.5f * (u1 / u2))); }
                            dx = r * m_cosf(theta); dy = r * m_sinf(theta);
                        }
                        bd[0] = dx; bd[1] = dy; bd[2] = sqrtf(smaxf(0.0f, 1.0f - (dx * dx + dy * dy)));
                    }
                    if (pcg_float(&fs) < 0.5f) bd[dim - 1] *= -1.0f;
                    float ct = fabsf(bd[dim - 1]);
                    float pdfc = dim == 2 ? ct / 2.0f : (float)((double)ct / PI_D);
                    boundaryPdf = 0.5f * pdfc;
                    /* transformCoordinates (sampling.h:176-203) with n = directionForDerivative */
                    const float *n = dirForDeriv;
                    if (dim == 2) {
                        float s0 = n[1], s1 = -n[0];
                        float t0 = bd[0] * s0 + bd[1] * n[0], t1 = bd[0] * s1 + bd[1] * n[1];
                        bd[0] = t0; bd[1] = t1;
                    } else {
                        float sign = copysignf(1.0f, n[2]);
                        const float aa = -1.0f / (sign + n[2]);
                        const float b = n[0] * n[1] * aa;
                        float b1[3] = {1.0f + sign * n[0] * n[0] * aa, sign * b, -sign * n[0]};
                        float b2[3] = {b, sign + n[1] * n[1] * aa, -n[1]};
                        float t[3];
                        for (int k = 0; k < 3; k++) t[k] = bd[0] * b1[k] + bd[1] * b2[k] + bd[2] * n[k];
                        memcpy(bd, t, 12);
                    }
                } else {
                    sample_unit_sphere(dim, u, bd);
                    boundaryPdf = pdf_sphere_uniform(dim, 1.0f);
                }
                for (int k = 0; k < dim; k++) g.ySurf[k] = g.c[k] + g.R * bd[k];
                memcpy(boundaryPt, g.ySurf, 12);
            } else {
                float bd[3] = {0, 0, 0};
                for (int k = 0; k < dim; k++) bd[k] = boundaryPt[k] - st.pt[k];
                for (int k = 0; k < dim; k++) g.ySurf[k] = st.pt[k] - bd[k];
            }
            st.prevDist = g.R;
            for (int k = 0; k < dim; k++) st.prevDir[k] = (g.ySurf[k] - st.pt[k]) / g.R;
            memcpy(st.pt, g.ySurf, 12);
            st.throughput *= gfn_poisson_kernel(&g) / boundaryPdf;
            {
                float pg[3] = {0, 0, 0}; gfn_poisson_kernel_gradient(&g, pg);
                float den = boundaryPdf * st.throughput;
                for (int k = 0; k < dim; k++) st.bdir[k] = pg[k] / den;
            }
            float dd = dist_dirichlet(sc, st.pt, 0);
            pcg_t ws; pcg_seed(&ws, wseed, 1u);
            wcount_t wc = {0, 0};
            int code = walk(sc, prm, dd, 0.0f, &ws, &g, &st, &wc);
            pc->iters += wc.iters;
            uint64_t total_steps = stepsBefore + wc.steps;
            if (code == WC_DIRICHLET || code == WC_RR) {
                st.terminal = (code == WC_DIRICHLET && !prm->ignore_dirichlet) ? dirichlet_value(sc, st.pt) : 0.0f;
                float total = st.throughput * st.terminal + st.totalNeumann + st.totalSource;
                float bc = total - st.firstSource;
                float ge[3];
                float deriv = 0.0f;
                for (int k = 0; k < dim; k++) {
                    float be = (bc - cvb) * st.bdir[k];
                    float se = (st.firstSource - cvs) * st.sdir[k];
                    ge[k] = be + se;
                    deriv += be * dirForDeriv[k];
                    deriv += se * dirForDeriv[k];
                }
                S->nSol += 1; welford(total, &S->solMean, &S->solM2, S->nSol);
                S->totalFirst += st.firstSource;
                S->nGrad += 1;
                for (int k = 0; k < dim; k++) welford(ge[k], &S->gMean[k], &S->gM2[k], S->nGrad);
                S->totalDeriv += deriv;
                S->totalLen += st.walkLength;
                pc->steps += total_steps; pc->rec++;
                if (code == WC_RR) pc->rr++; else pc->dir++;
            } else {
                pc->wasted += total_steps;
                if (code == WC_ESCAPED) pc->esc++; else pc->maxl++;
            }
        }
    }
    free(strat);
}

/* ------------------------------------------------------------------------- */
/* batch driver                                                              */
/* ------------------------------------------------------------------------- */
typedef struct {
    const scene_t *sc; const oracle_params *prm;
    const float *pts; int64_t n, base, stride;
    float *p, *grad; int32_t *n_est, *steps; float *sol_m2;
    atomic_llong next;
    pthread_mutex_t mu;
    oracle_stats tot;
} job_t;

static void solve_one(job_t *J, int64_t i, pcount_t *pc, uint64_t *nest)
{
    const scene_t *sc = J->sc; const int dim = sc->dim;
    float x[3] = {0, 0, 0};
    for (int k = 0; k < dim; k++) x[k] = J->pts[i * dim + k];
    float dDist = dist_dirichlet(sc, x, 0);
    float nDist = dist_neumann(sc, x, 0);
    int inside = inside_domain(sc, x);
    stats_t S; memset(&S, 0, sizeof(S));
    int estimated = 0;
    pcount_t before = *pc;
    if (inside || sc->double_sided) {
        estimate_point(sc, J->prm, x, (uint64_t)(J->base + i * J->stride), dDist, nDist, &S, pc, NULL);
        estimated = 1; (*nest)++;
    }
    float mask = J->prm->boundary_distance_mask;
    int maskP = fabsf(nDist) < mask;
    int maskG = (!inside && !sc->double_sided) || fabsf(nDist) < mask;
    J->p[i] = maskP ? 0.0f : (estimated ? S.solMean : 0.0f);
    for (int k = 0; k < dim; k++) J->grad[i * dim + k] = maskG ? 0.0f : (estimated ? S.gMean[k] : 0.0f);
    if (J->n_est) J->n_est[i] = S.nSol;
    if (J->sol_m2) J->sol_m2[i] = S.solM2;
    if (J->steps) J->steps[i] = (int32_t)((pc->steps - before.steps) + (pc->wasted - before.wasted));
}

static void *worker(void *arg)
{
    job_t *J = (job_t *)arg;
    pcount_t pc; memset(&pc, 0, sizeof(pc));
    uint64_t nest = 0;
    g_libm = J->prm->math_mode == 1;
    g_robust = J->prm->robust_float != 0;
    for (;;) {
        int64_t i = atomic_fetch_add(&J->next, 16);
        if (i >= J->n) break;
        int64_t e = i + 16 < J->n ? i + 16 : J->n;
        for (int64_t k = i; k < e; k++) solve_one(J, k, &pc, &nest);
    }
    pthread_mutex_lock(&J->mu);
    J->tot.walk_steps += pc.steps; J->tot.wasted_steps += pc.wasted;
    J->tot.walks_recorded += pc.rec; J->tot.walks_escaped += pc.esc;
    J->tot.walks_max_length += pc.maxl; J->tot.walks_rr += pc.rr;
    J->tot.walks_dirichlet += pc.dir; J->tot.points_estimated += nest;
    J->tot.rejection_iters += pc.iters;
    pthread_mutex_unlock(&J->mu);
    return NULL;
}

int oracle_solve(const oracle_scene_desc *scene, const oracle_params *prm,
                 const float *pts, int64_t n, int64_t index_base, int64_t index_stride,
                 float *p, float *grad, int32_t *n_est, int32_t *steps, oracle_stats *stats)
{
    return oracle_solve_m2(scene, prm, pts, n, index_base, index_stride, p, grad, n_est, steps, NULL, stats);
}

int oracle_solve_m2(const oracle_scene_desc *scene, const oracle_params *prm,
                    const float *pts, int64_t n, int64_t index_base, int64_t index_stride,
                    float *p, float *grad, int32_t *n_est, int32_t *steps, float *sol_m2,
                    oracle_stats *stats)
{
    if (!scene || !prm || (n > 0 && (!pts || !p || !grad))) return -1;
    if (prm->n_walks < 1) return -2;
    scene_t sc;
    g_libm = prm->math_mode == 1;
    g_robust = prm->robust_float != 0;
    if (scene_build(&sc, scene)) { scene_free(&sc); return -3; }
    job_t J; memset(&J, 0, sizeof(J));
    J.sc = &sc; J.prm = prm; J.pts = pts; J.n = n; J.base = index_base; J.stride = index_stride;
    J.p = p; J.grad = grad; J.n_est = n_est; J.steps = steps; J.sol_m2 = sol_m2;
    atomic_init(&J.next, 0);
    pthread_mutex_init(&J.mu, NULL);
    int nt = prm->n_threads > 0 ? prm->n_threads : 1;
    if (nt > 256) nt = 256;
    pthread_t th[256];
    for (int t = 1; t < nt; t++) pthread_create(&th[t], NULL, worker, &J);
    worker(&J);
    for (int t = 1; t < nt; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&J.mu);
    if (stats) *stats = J.tot;
    scene_free(&sc);
    return 0;
}

int oracle_point_info(const oracle_scene_desc *scene, const float *pt,
                      float *dirichlet_dist, float *neumann_dist,
                      float *signed_neumann_dist, int32_t *inside,
                      float *star_radius_out, int32_t *n_silhouettes)
{
    scene_t sc;
    g_libm = 0;
    if (scene_build(&sc, scene)) { scene_free(&sc); return -3; }
    float x[3] = {0, 0, 0};
    for (int k = 0; k < sc.dim; k++) x[k] = pt[k];
    float dd = dist_dirichlet(&sc, x, 0);
    if (dirichlet_dist) *dirichlet_dist = dd;
    if (neumann_dist) *neumann_dist = dist_neumann(&sc, x, 0);
    if (signed_neumann_dist) *signed_neumann_dist = dist_neumann(&sc, x, 1);
    if (inside) *inside = inside_domain(&sc, x);
    if (star_radius_out) *star_radius_out = star_radius(&sc.neu, x, 1e-3f, dd, 1e-3f, 0);
    if (n_silhouettes) *n_silhouettes = sc.neu.ns;
    scene_free(&sc);
    return 0;
}

double oracle_bessel(int which, double x, int math_mode)
{
    g_libm = math_mode == 1;
    switch (which) {
    case 0: return bessi0(x);
    case 1: return bessi1(x);
    case 2: return bessk0(x);
    case 3: return bessk1(x);
    default: return NAN;
    }
}

double oracle_math(int which, double x, int math_mode)
{
    g_libm = math_mode == 1;
    switch (which) {
    case 0: return m_exp(x);
    case 1: return m_log(x);
    case 2: return g_libm ? sin(x) : ({ double s, c; dm_sincos(x, &s, &c); s; });
    case 3: return g_libm ? cos(x) : ({ double s, c; dm_sincos(x, &s, &c); c; });
    case 4: return g_libm ? atan(x) : dm_atan(x);
    case 10: return m_expf((float)x);
    case 11: return m_logf((float)x);
    case 12: return m_sinf((float)x);
    case 13: return m_cosf((float)x);
    case 14: return m_cbrtf((float)x);
    default: return NAN;
    }
}

/* ========================================================================= */
/* Boundary value caching: runBoundaryValueCaching (demo.cpp:265-363) over    */
/* boundary_value_caching/{boundary_sampler,domain_sampler,splatter}.h, 2D,   */
/* Neumann and Dirichlet boundaries.                                          */
/* RNG (documented deviation): boundary sampler stream seed32(key,0,0,4),     */
/* domain sampler seed32(key,0,0,5), walk w of boundary sample i             */
/* seed32(key,i,w,6); sampled segments visited in ascending order (the        */
/* reference: clock seeds, std::unordered_map order, boundary_sampler.h:335). */
/* ========================================================================= */

/* CDFTable (sampling.h:261-314) */
static float cdf_build(float *table, const float *w, int n)
{
    if (n <= 0) return 0.0f;
    table[0] = 0.0f;
    for (int i = 1; i < n + 1; i++) table[i] = table[i - 1] + w[i - 1];
    float total = table[n];
    if (total == 0.0f) { for (int i = 1; i < n + 1; i++) table[i] = (float)i / (float)n; }
    else { for (int i = 1; i < n + 1; i++) table[i] /= total; }
    return total;
}

static int cdf_sample(const float *table, int size, float u)
{
    int first = 0, len = size;
    while (len > 0) {
        int half = len >> 1, middle = first + half;
        if (table[middle] <= u) { first = middle + 1; len -= half + 1; }
        else len = half;
    }
    return sclampi(first - 1, 0, size - 2);
}

/* The BoundarySampler's boundary (boundary_sampler.h:87-412): every segment of the scene, here the
 * Neumann segments then the Dirichlet ones (the reference: the OBJ's order, typed by
 * onNeumannBoundary at the midpoint, demo.cpp:300-313); Dirichlet vertices carry the sampler's
 * own vertex normals (computeNormals :193-236: unit segment normals summed, normalised) over the
 * scene's one mesh (demo.cpp:316): a Dirichlet vertex also sums the normals of the Neumann
 * segments ending at its position (the two parts arrive as separate meshes; welded by position). */
typedef struct {
    int ns, nn;                 /* segments, of which the first nn are Neumann */
    const float *(*a), *(*b);   /* endpoints */
    const float *(*na), *(*nb); /* Dirichlet vertex normals (NULL for Neumann segments) */
    float (*dn)[3];             /* storage of the Dirichlet vertex normals */
} bseg_t;

static void bseg_build(const scene_t *sc, bseg_t *B)
{
    const geom_t *N = &sc->neu, *D = &sc->dir;
    B->nn = N->np; B->ns = N->np + D->np;
    B->a = calloc((size_t)B->ns + 1, sizeof(float *)); B->b = calloc((size_t)B->ns + 1, sizeof(float *));
    B->na = calloc((size_t)B->ns + 1, sizeof(float *)); B->nb = calloc((size_t)B->ns + 1, sizeof(float *));
    B->dn = calloc((size_t)D->nv + 1, sizeof(float[3]));
    for (int p = 0; p < D->np; p++) {
        const float *pa = D->v[D->ix[p][0]], *pb = D->v[D->ix[p][1]];
        float s0 = pb[0] - pa[0], s1 = pb[1] - pa[1];
        float n[2] = {s1, -s0};
        float z = n[0] * n[0] + n[1] * n[1];
        if (z > 0.0f) { float r = sqrtf(z); n[0] = n[0] / r; n[1] = n[1] / r; }
        for (int q = 0; q < 2; q++) { float *v = B->dn[D->ix[p][q]]; v[0] += n[0]; v[1] += n[1]; }
    }
    /* junctions: Neumann segment ends at a Dirichlet vertex's position (brute force) */
    for (int p = 0; p < N->np && D->np > 0; p++) {
        const float *pa = N->v[N->ix[p][0]], *pb = N->v[N->ix[p][1]];
        float s0 = pb[0] - pa[0], s1 = pb[1] - pa[1];
        float n[2] = {s1, -s0};
        float z = n[0] * n[0] + n[1] * n[1];
        if (z > 0.0f) { float r = sqrtf(z); n[0] = n[0] / r; n[1] = n[1] / r; }
        for (int q = 0; q < 2; q++) {
            const float *e = q ? pb : pa;
            for (int i = 0; i < D->nv; i++)
                if (D->v[i][0] == e[0] && D->v[i][1] == e[1]) { B->dn[i][0] += n[0]; B->dn[i][1] += n[1]; }
        }
    }
    for (int i = 0; i < D->nv; i++) {
        float z = B->dn[i][0] * B->dn[i][0] + B->dn[i][1] * B->dn[i][1];
        if (z > 0.0f) { float r = sqrtf(z); B->dn[i][0] /= r; B->dn[i][1] /= r; }
    }
    for (int i = 0; i < N->np; i++) { B->a[i] = N->v[N->ix[i][0]]; B->b[i] = N->v[N->ix[i][1]]; }
    for (int p = 0; p < D->np; p++) {
        int i = N->np + p;
        B->a[i] = D->v[D->ix[p][0]]; B->b[i] = D->v[D->ix[p][1]];
        B->na[i] = B->dn[D->ix[p][0]]; B->nb[i] = B->dn[D->ix[p][1]];
    }
}

static void bseg_free(bseg_t *B) { free(B->a); free(B->b); free(B->na); free(B->nb); free(B->dn); }

/* segment i's endpoints, a Dirichlet segment's displaced along its vertex normals by `offset`
 * (`pa += normalOffset*normals[index[0]]`, boundary_sampler.h:307-310,367-370) */
static void bseg_ends(const bseg_t *B, int i, float offset, float *pa, float *pb)
{
    pa[0] = B->a[i][0]; pa[1] = B->a[i][1]; pb[0] = B->b[i][0]; pb[1] = B->b[i][1];
    if (i >= B->nn) {
        pa[0] += offset * B->na[i][0]; pa[1] += offset * B->na[i][1];
        pb[0] += offset * B->nb[i][0]; pb[1] += offset * B->nb[i][1];
    }
}

/* buildCDFTable (boundary_sampler.h:291-331) */
static float bvc_table(const bseg_t *B, const scene_t *sc, float offset, float *table)
{
    float *w = calloc((size_t)B->ns + 1, sizeof(float));
    for (int i = 0; i < B->ns; i++) {
        const float *pa0 = B->a[i], *pb0 = B->b[i];
        float pm[2] = {(pa0[0] + pb0[0]) / 2.0f, (pa0[1] + pb0[1]) / 2.0f};
        float s0 = pb0[0] - pa0[0], s1 = pb0[1] - pa0[1];
        float n[2] = {s1, -s0};
        float z = n[0] * n[0] + n[1] * n[1];
        if (z > 0.0f) { float r = sqrtf(z); n[0] = n[0] / r; n[1] = n[1] / r; }
        float q[2] = {pm[0] + offset * n[0], pm[1] + offset * n[1]};
        int in = q[0] >= sc->pmin[0] && q[1] >= sc->pmin[1] && q[0] <= sc->pmax[0] && q[1] <= sc->pmax[1];
        if (in) {
            float pa[2], pb[2];
            bseg_ends(B, i, offset, pa, pb);
            float t0 = pb[0] - pa[0], t1 = pb[1] - pa[1];
            w[i] = sqrtf(t1 * t1 + (-t0) * (-t0));
        }
    }
    float total = cdf_build(table, w, B->ns);
    free(w);
    return total;
}

typedef struct { float *rec; int n, cap; } recbuf_t;
static void rec_push(recbuf_t *b, const float *r)
{
    if (b->n == b->cap) { b->cap = b->cap ? 2 * b->cap : 256; b->rec = realloc(b->rec, sizeof(float) * 8 * (size_t)b->cap); }
    memcpy(b->rec + 8 * (size_t)b->n, r, sizeof(float) * 8); b->n++;
}

/* sample kinds of the cache records [x y nx ny pdf value dn/dn kind] */
enum { KB_NEUMANN = 0, KB_NEUMANN_ALIGNED = 1, KB_DOMAIN = 2, KB_DIRICHLET = 3, KB_DIRICHLET_ALIGNED = 4 };

/* generateSamples (boundary_sampler.h:333-402) */
static void bvc_gen_boundary(const bseg_t *B, const float *table, int n, float total, float offset, int aligned,
                             pcg_t *rng, recbuf_t *out, float pdf)
{
    if (!(total > 0.0f) || n <= 0) return;
    float *strat = malloc(sizeof(float) * (size_t)n);
    gen_stratified(strat, n, 1, rng);
    int *count = calloc((size_t)B->ns, sizeof(int));
    for (int i = 0; i < n; i++) count[cdf_sample(table, B->ns + 1, strat[i])]++;
    for (int f = 0; f < B->ns; f++) {
        int c = count[f];
        if (!c) continue;
        float *u = malloc(sizeof(float) * (size_t)c);
        if (c == 1) u[0] = pcg_float(rng); else gen_stratified(u, c, 1, rng);
        float pa[2], pb[2];
        bseg_ends(B, f, offset, pa, pb);
        float s0 = pb[0] - pa[0], s1 = pb[1] - pa[1];
        float kind = f >= B->nn ? (aligned ? KB_DIRICHLET_ALIGNED : KB_DIRICHLET) : (aligned ? KB_NEUMANN_ALIGNED : KB_NEUMANN);
        for (int i = 0; i < c; i++) {
            float nn[2] = {s1, -s0};
            float norm = sqrtf(nn[0] * nn[0] + nn[1] * nn[1]);
            float r[8] = {pa[0] + u[i] * s0, pa[1] + u[i] * s1, nn[0] / norm, nn[1] / norm, pdf, 0.0f, 0.0f, kind};
            rec_push(out, r);
        }
        free(u);
    }
    free(count); free(strat);
}

/* estimateSolution (walk_on_stars.h:353-464) at a sample point: on the Neumann boundary (a
 * boundary sample) or in the domain (an evaluation point near the Dirichlet boundary,
 * splatter.h:160-196, or a finite-difference Dirichlet sample); walk w seeded
 * seed32(key, sidx, w, tag) */
static float bvc_estimate(const scene_t *sc, const oracle_params *prm, const float *pt, const float *nrm, int aligned,
                          int on_neumann, int nWalks, uint64_t sidx, uint32_t tag, pcount_t *pc)
{
    float x[3] = {pt[0], pt[1], 0.0f};
    float dDist = dist_dirichlet(sc, x, 0);
    if (dDist <= prm->epsilon_shell) nWalks = 1;
    float cn[3] = {nrm[0], nrm[1], 0.0f};
    int flip = 0;
    if (sc->double_sided && on_neumann && aligned) { cn[0] *= -1.0f; cn[1] *= -1.0f; flip = 1; }
    float firstR;
    if (dDist > prm->epsilon_shell && prm->steps_before_maximal_spheres != 0) {
        firstR = star_radius(&sc->neu, x, prm->min_star_radius, dDist, prm->silhouette_precision, flip);
        if (prm->min_star_radius <= dDist) firstR = smaxf(0.99f * firstR, prm->min_star_radius);
    } else {
        firstR = dDist;
    }
    int yuk0 = sc->absorption > 0.0f && prm->steps_before_tikhonov == 0;
    float mean = 0.0f; int N = 0;
    for (int w = 0; w < nWalks; w++) {
        gfn_t g; gfn_init(&g, 2, yuk0, sc->absorption);
        wstate_t st; memset(&st, 0, sizeof(st));
        memcpy(st.pt, x, 12); memcpy(st.n, cn, 12); memcpy(st.prevDir, cn, 12);
        st.prevDist = FLT_MAX; st.throughput = 1.0f; st.onNeumann = on_neumann;
        pcg_t ws; pcg_seed(&ws, oracle_seed32(prm->seed, sidx, (uint64_t)w, tag), 1u);
        wcount_t wc = {0, 0};
        int code = walk(sc, prm, dDist, firstR, &ws, &g, &st, &wc);
        pc->iters += wc.iters;
        if (code == WC_DIRICHLET || code == WC_RR) {
            float term = (code == WC_DIRICHLET && !prm->ignore_dirichlet) ? dirichlet_value(sc, st.pt) : 0.0f;
            float total = st.throughput * term + st.totalNeumann + st.totalSource;
            N += 1;
            float delta = total - mean;
            mean += delta / (float)N;
            pc->steps += wc.steps; pc->rec++;
            if (code == WC_RR) pc->rr++; else pc->dir++;
        } else {
            pc->wasted += wc.steps;
            if (code == WC_ESCAPED) pc->esc++; else pc->maxl++;
        }
    }
    return mean;
}

/* free-space Green's functions, 2D (distributions.h:85-119, 168-219) */
typedef struct { int yukawa; float lambda, sqrtLambda; } fs2_t;

static void fs2_k(float mur, float *K0, float *K1, float *K2)
{
    double k0 = bessk0((double)mur), k1 = bessk1((double)mur);
    *K0 = (float)k0; *K1 = (float)k1;
    double tox = 2.0 / (double)mur;                /* bessel::bessk(2, x), bessel.hpp:584-608 */
    *K2 = (float)(k0 + (1.0 * tox) * k1);
}

typedef struct { float mean, g[2]; int n; } sstat_t;
static void sstat_add(sstat_t *s, float est, const float *ge)
{
    s->n += 1;
    float fN = (float)s->n;
    s->mean += (est - s->mean) / fN;
    for (int k = 0; k < 2; k++) s->g[k] += (ge[k] - s->g[k]) / fN;
}

/* Splatter::splat of every cached sample onto one evaluation point (splatter.h:43-301) */
static void bvc_splat_point(const fs2_t *gf, const float *x, const recbuf_t *rb, float radius_clamp, float reg,
                            float *sol, float *grad)
{
    sstat_t st[3]; memset(st, 0, sizeof(st));
    for (int j = 0; j < rb->n; j++) {
        const float *R = rb->rec + 8 * (size_t)j;
        int kind = (int)R[7];
        int slot = kind == KB_DOMAIN ? 2 : (kind == KB_NEUMANN_ALIGNED || kind == KB_DIRICHLET_ALIGNED) ? 1 : 0;
        float pdf = R[4], value = R[5];
        float yx[2] = {R[0] - x[0], R[1] - x[1]}, xy[2] = {x[0] - R[0], x[1] - R[1]};
        float r = smaxf(radius_clamp, sqrtf(yx[0] * yx[0] + yx[1] * yx[1]));
        float K0 = 0, K1 = 0, K2 = 0;
        if (gf->yukawa) fs2_k(r * gf->sqrtLambda, &K0, &K1, &K2);
        float G, dG[2];
        if (!gf->yukawa) {
            G = (float)((double)(-m_logf(r)) / TWO_PI_D);
            float s = (float)(TWO_PI_D * (double)(r * r));
            for (int k = 0; k < 2; k++) dG[k] = (-xy[k]) / s;
        } else {
            G = (float)((double)K0 / TWO_PI_D);
            float Qr = gf->sqrtLambda * K1;
            float s = (float)(TWO_PI_D * (double)r);
            for (int k = 0; k < 2; k++) dG[k] = ((-xy[k]) * Qr) / s;
        }
        float dGNorm = sqrtf(dG[0] * dG[0] + dG[1] * dG[1]);
        float est, ge[2];
        if (kind != KB_DOMAIN) {
            float sg = slot == 1 ? -1.0f : 1.0f;
            float n[2] = {R[2] * sg, R[3] * sg};
            float nd = n[0] * xy[0] + n[1] * xy[1];
            float P, dP[2];
            float r2 = r * r;
            if (!gf->yukawa) {
                P = (float)((double)nd / (TWO_PI_D * (double)r2));
                float c = 2.0f * (nd / r2);
                float s = (float)(TWO_PI_D * (double)r2);
                for (int k = 0; k < 2; k++) dP[k] = (n[k] - c * xy[k]) / s;
            } else {
                float Qr = gf->sqrtLambda * K1;
                P = (float)((double)(nd * Qr) / (TWO_PI_D * (double)r));
                float Qr1 = gf->sqrtLambda * K1;
                float Qr2 = gf->lambda * (K0 + K2) / 2.0f;
                float c = (nd / r2) * (Qr1 + r * Qr2);
                float s = (float)(TWO_PI_D * (double)r);
                for (int k = 0; k < 2; k++) dP[k] = (n[k] * Qr1 - c * xy[k]) / s;
            }
            float dPNorm = sqrtf(dP[0] * dP[0] + dP[1] * dP[1]);
            if (!(isfinite(G) && isfinite(P) && isfinite(dGNorm) && isfinite(dPNorm))) continue;
            if (reg > 0.0f) { r /= reg; P *= 1.0f - m_expf(-r * r); }
            float ndv = R[6];
            est = (G * ndv - P * value) / pdf;
            for (int k = 0; k < 2; k++) ge[k] = (dG[k] * ndv - dP[k] * value) / pdf;
        } else {
            if (!(isfinite(G) && isfinite(dGNorm))) continue;
            est = (G * value) / pdf;
            for (int k = 0; k < 2; k++) ge[k] = (dG[k] * value) / pdf;
        }
        sstat_add(&st[slot], est, ge);
    }
    float v = st[0].mean; v += st[1].mean; v += st[2].mean;
    *sol = v;
    for (int k = 0; k < 2; k++) { float a = st[0].g[k]; a += st[1].g[k]; a += st[2].g[k]; grad[k] = a; }
}

int oracle_bvc(const oracle_scene_desc *scene, const oracle_params *prm, const oracle_bvc_params *bp,
               float *solution, float *grad, float *samples, int64_t samples_capacity, int64_t *counts,
               oracle_stats *stats)
{
    if (!scene || !prm || !bp || !solution || !grad) return -1;
    if (scene->dim != 2 || scene->n_prims + scene->n_dprims <= 0 || bp->grid_res < 1 || bp->n_walks_solution < 1 ||
        (scene->n_dprims > 0 && bp->n_walks_gradient < 1)) return -2;
    scene_t sc;
    g_libm = prm->math_mode == 1;
    g_robust = prm->robust_float != 0;
    if (scene_build(&sc, scene)) { scene_free(&sc); return -3; }
    const geom_t *g = &sc.neu;
    bseg_t B; bseg_build(&sc, &B);
    recbuf_t rb = {0};
    /* ---- boundary samples (BoundarySampler::initialize + generateSamples, demo.cpp:316-318) */
    pcg_t bs; pcg_seed(&bs, oracle_seed32(prm->seed, 0, 0, 4), 1u);
    float *t_main = malloc(sizeof(float) * ((size_t)B.ns + 1)), *t_al = malloc(sizeof(float) * ((size_t)B.ns + 1));
    float a_main = bvc_table(&B, &sc, -1.0f * bp->normal_offset, t_main);
    int nb_main, nb_al = 0;
    if (sc.double_sided) {
        float a_al = bvc_table(&B, &sc, bp->normal_offset, t_al);
        float total = a_main + a_al;
        int n_main = (int)ceilf((float)bp->boundary_cache_size * a_main / total);
        int n_al = (int)ceilf((float)bp->boundary_cache_size * a_al / total);
        bvc_gen_boundary(&B, t_main, n_main, a_main, -1.0f * bp->normal_offset, 0, &bs, &rb, 1.0f / a_main);
        nb_main = rb.n;
        bvc_gen_boundary(&B, t_al, n_al, a_al, bp->normal_offset, 1, &bs, &rb, 1.0f / a_al);
        nb_al = rb.n - nb_main;
    } else {
        bvc_gen_boundary(&B, t_main, bp->boundary_cache_size, a_main, -1.0f * bp->normal_offset, 0, &bs, &rb,
                         1.0f / a_main);
        nb_main = rb.n;
    }
    free(t_main); free(t_al);
    /* ---- estimates at the boundary samples (BoundarySampler::computeEstimates :121-190):
     * Neumann samples estimateSolution (nWalksForCachedSolutionEstimates, walks tag 6);
     * Dirichlet samples estimateSolutionAndGradient along their normal (nWalksForCachedGradient-
     * Estimates, keyed by the sample index) -> solution and normal derivative, or with
     * useFiniteDifferences estimateSolution in the domain (tag 8) and (g(proj) - u)/|d| */
    pcount_t pc; memset(&pc, 0, sizeof(pc));
    for (int i = 0; i < rb.n; i++) {
        float *R = rb.rec + 8 * (size_t)i;
        int kind = (int)R[7], al = kind == KB_NEUMANN_ALIGNED || kind == KB_DIRICHLET_ALIGNED;
        if (kind == KB_NEUMANN || kind == KB_NEUMANN_ALIGNED) {
            R[5] = bvc_estimate(&sc, prm, R, R + 2, al, 1, bp->n_walks_solution, (uint64_t)i, 6u, &pc);
            /* normalDerivative = pde.neumann(pt) (boundary_sampler.h:126-133): 0 in the reference's
             * scenes (scene.h:176-181), the image-valued h when given */
            R[6] = prm->ignore_neumann ? 0.0f : neumann_value(&sc, R);
            continue;
        }
        float x[3] = {R[0], R[1], 0.0f};
        if (bp->use_finite_differences) {
            R[5] = bvc_estimate(&sc, prm, R, R + 2, al, 0, bp->n_walks_gradient, (uint64_t)i, 8u, &pc);
            cp_t c;
            float gv = sc.g_dirichlet, sd = 0.0f;
            if (closest_point(&sc.dir, x, &c, sc.double_sided) >= 0) {
                gv = dirichlet_value(&sc, x);
                sd = sc.double_sided ? signed_distance(&c, x) : c.d;
            }
            R[6] = (gv - R[5]) / fabsf(sd);
            continue;
        }
        float dir[3] = {R[2], R[3], 0.0f};
        if (sc.double_sided && al) { dir[0] *= -1.0f; dir[1] *= -1.0f; }
        stats_t S;
        oracle_params wp = *prm;
        wp.n_walks = bp->n_walks_gradient;
        estimate_point(&sc, &wp, x, (uint64_t)i, dist_dirichlet(&sc, x, 0), dist_neumann(&sc, x, 0), &S, &pc, dir);
        R[5] = S.solMean;
        R[6] = S.totalDeriv / (float)(S.nSol > 1 ? S.nSol : 1);
    }
    /* ---- domain samples (DomainSampler::generateSamples) */
    int nd_kept = 0;
    if (!prm->ignore_source && bp->domain_cache_size > 0) {
        float ext[2] = {sc.pmax[0] - sc.pmin[0], sc.pmax[1] - sc.pmin[1]};
        float vol;
        if (sc.double_sided) vol = ext[0] * ext[1];
        else {
            /* getSolveRegionVolume (scene.h:92-100): |signed area of the Dirichlet part + the Neumann part| */
            float sv = 0.0f;
            const geom_t *parts[2] = {&sc.dir, g};
            for (int q = 0; q < 2; q++) {
                float sq = 0.0f;
                for (int p = 0; p < parts[q]->np; p++) {
                    const float *pa = parts[q]->v[parts[q]->ix[p][0]], *pb = parts[q]->v[parts[q]->ix[p][1]];
                    sq += 0.5f * (pa[0] * pb[1] - pa[1] * pb[0]);
                }
                sv += sq;
            }
            vol = fabsf(sv);
        }
        float pdf = 1.0f / vol;
        int nstrat = bp->domain_cache_size;
        if (vol > 0.0f) nstrat = (int)((float)nstrat * (ext[0] * ext[1] * pdf));
        if (nstrat > 0) {
            pcg_t ds; pcg_seed(&ds, oracle_seed32(prm->seed, 0, 0, 5), 1u);
            float *strat = malloc(sizeof(float) * 2 * (size_t)nstrat);
            gen_stratified(strat, nstrat, 2, &ds);
            for (int i = 0; i < nstrat; i++) {
                float x[3] = {sc.pmin[0] + ext[0] * strat[2 * i], sc.pmin[1] + ext[1] * strat[2 * i + 1], 0.0f};
                int keep = sc.double_sided ? !outside_bbox(&sc, x) : inside_domain(&sc, x);
                if (!keep) continue;
                float r[8] = {x[0], x[1], 0.0f, 0.0f, pdf, source_value(&sc, x), 0.0f, 2.0f};
                rec_push(&rb, r);
                nd_kept++;
            }
            free(strat);
        }
    }
    /* ---- splat onto the evaluation grid (createEvaluationGrid grid.h:352-368, saveEvaluationGrid 370-414)
     * over bp->grid_box (x0, y0, ex, ey; extent 0: the scene's box); points closer to the Dirichlet
     * boundary than normalOffset take a pointwise estimateSolution instead (splatter.h:160-196,
     * nWalksForCachedSolutionEstimates, walks seed32(key, rank, w, 7)) with a zero gradient */
    fs2_t gf = {sc.absorption > 0.0f, sc.absorption, sqrtf(sc.absorption)};
    const int res = bp->grid_res;
    float gmin[2] = {sc.pmin[0], sc.pmin[1]};
    float ext[2] = {sc.pmax[0] - sc.pmin[0], sc.pmax[1] - sc.pmin[1]};
    if (bp->grid_box[2] > 0.0f && bp->grid_box[3] > 0.0f) {
        gmin[0] = bp->grid_box[0]; gmin[1] = bp->grid_box[1]; ext[0] = bp->grid_box[2]; ext[1] = bp->grid_box[3];
    }
    uint64_t n_near = 0;  /* rank of an evaluation point among those near the Dirichlet boundary: its walks' key */
    for (int i = 0; i < res; i++) for (int j = 0; j < res; j++) {
        size_t q = (size_t)i * res + j;
        float x[3] = {((float)i / (float)res) * ext[0] + gmin[0], ((float)j / (float)res) * ext[1] + gmin[1], 0.0f};
        float dDist = dist_dirichlet(&sc, x, 0), nDist = dist_neumann(&sc, x, 0);
        float v = 0.0f, gv[2] = {0.0f, 0.0f};
        if (!(dDist < bp->normal_offset)) bvc_splat_point(&gf, x, &rb, bp->radius_clamp, bp->kernel_regularization, &v, gv);
        else if (sc.dir.np > 0) {
            static const float zero[2] = {0.0f, 0.0f};
            v = bvc_estimate(&sc, prm, x, zero, 0, 0, bp->n_walks_solution, n_near++, 7u, &pc);
        }
        int in = inside_domain(&sc, x);
        int masked = (!in && !sc.double_sided) || sminf(fabsf(dDist), fabsf(nDist)) < prm->boundary_distance_mask;
        solution[q] = masked ? 0.0f : v;
        grad[2 * q] = masked ? 0.0f : gv[0];
        grad[2 * q + 1] = masked ? 0.0f : gv[1];
    }
    if (counts) { counts[0] = nb_main; counts[1] = nb_al; counts[2] = nd_kept; counts[3] = rb.n; }
    int rc = 0;
    if (samples) {
        if (samples_capacity < rb.n) rc = -4;
        else memcpy(samples, rb.rec, sizeof(float) * 8 * (size_t)rb.n);
    }
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        stats->walk_steps = pc.steps; stats->wasted_steps = pc.wasted; stats->walks_recorded = pc.rec;
        stats->walks_escaped = pc.esc; stats->walks_max_length = pc.maxl; stats->walks_rr = pc.rr;
        stats->walks_dirichlet = pc.dir; stats->points_estimated = (uint64_t)(nb_main + nb_al);
        stats->rejection_iters = pc.iters;
    }
    free(rb.rec);
    bseg_free(&B);
    scene_free(&sc);
    return rc;
}
