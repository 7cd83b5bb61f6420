/*
 * oracle/detmath.h -- TEST INFRASTRUCTURE ONLY (part of the parity oracle).
 *
 * Deterministic, portable transcendental functions used by the oracle in its
 * "det" math mode.  The reference (zombie, walk_on_stars.h / distributions.h /
 * bessel.hpp / sampling.h) calls glibc's expf/logf/cosf/sinf/exp/log/cbrtf/
 * atan2f.  Those are not reproducible on a GPU, so the product (HIP) and this
 * oracle both implement the SAME algorithms below with only IEEE +,-,*,/,sqrt
 * (compiled with -ffp-contract=off on both sides).  The oracle's "libm" mode
 * calls glibc instead; tests check det-vs-libm agreement to bound the effect.
 *
 * Algorithms: fdlibm-style Cody-Waite reduction + polynomial (exp, log,
 * sin/cos kernels); float functions are evaluated in double and rounded once.
 * This file is an independent C restatement; the product's copy lives in
 * neural-monte-carlo-fluid-simulation_amd/csrc/wos_detmath.h and must stay
 * operation-for-operation identical (the GPU parity tests enforce that).
 */
#ifndef ORACLE_DETMATH_H
#define ORACLE_DETMATH_H

#include <stdint.h>
#include <string.h>
#include <math.h>

static inline double dm_bits2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static inline uint64_t dm_d2bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

/* 2^k for k in [-1022, 1023], exact */
static inline double dm_pow2i(int k) { return dm_bits2d((uint64_t)(k + 1023) << 52); }

static inline double dm_exp(double x)
{
    if (x != x) return x;
    if (x > 709.782712893384) return INFINITY;
    if (x < -745.1332191019412) return 0.0;
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double inv_ln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    double kd = floor(x * inv_ln2 + 0.5);
    int k = (int)kd;
    double hi = x - kd * ln2_hi;
    double lo = kd * ln2_lo;
    double r = hi - lo;
    double t = r * r;
    double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    if (k > 1023) return (y * dm_pow2i(1023)) * 2.0;
    if (k >= -1021) return y * dm_pow2i(k);
    return (y * dm_pow2i(k + 1000)) * dm_pow2i(-1000);
}

static inline double dm_log(double x)
{
    if (x != x) return x;
    if (x < 0.0) return NAN;
    if (x == 0.0) return -INFINITY;
    if (x == INFINITY) return x;
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    int k = 0;
    if (x < 2.2250738585072014e-308) { x *= 18014398509481984.0; k = -54; } /* 2^54 */
    uint64_t u = dm_d2bits(x);
    int e = (int)((u >> 52) & 0x7ff) - 1023;
    uint64_t mant = u & 0x000fffffffffffffULL;
    double m = dm_bits2d(mant | 0x3ff0000000000000ULL); /* [1,2) */
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    k += e;
    double f = m - 1.0;
    double s = f / (2.0 + f);
    double z = s * s;
    double w = z * z;
    double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    double R = t2 + t1;
    double hfsq = 0.5 * f * f;
    double dk = (double)k;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

/* sin and cos of a double argument (|x| < ~2^19*pi/2 for full accuracy) */
static inline void dm_sincos(double x, double *sp, double *cp)
{
    if (x != x || x == INFINITY || x == -INFINITY) { *sp = NAN; *cp = NAN; return; }
    const double two_over_pi = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;
    const double pio2_2 = 6.07710050630396597660e-11;
    const double pio2_3 = 2.02226624871116645580e-21;
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double kd = floor(x * two_over_pi + 0.5);
    double r = ((x - kd * pio2_1) - kd * pio2_2) - kd * pio2_3;
    double z = r * r;
    double s = r + (z * r) * (S1 + z * (S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)))));
    double c = (1.0 - 0.5 * z) + (z * z) * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    int64_t ki = (int64_t)kd;
    int q = (int)(ki & 3);
    switch (q) {
    case 0: *sp = s; *cp = c; break;
    case 1: *sp = c; *cp = -s; break;
    case 2: *sp = -s; *cp = -c; break;
    default: *sp = -c; *cp = s; break;
    }
}

/* atan for double, |err| ~ 1 ulp (fdlibm s_atan.c structure) */
static inline double dm_atan(double x)
{
    const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                              9.82793723247329054082e-01, 1.57079632679489655800e+00};
    const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                              1.39033110312309984516e-17, 6.12323399573676603587e-17};
    const double aT[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01,
                           1.42857142725034663711e-01, -1.11111104054623557880e-01,
                           9.09088713343650656196e-02, -7.69187620504482999495e-02,
                           6.66107313738753120669e-02, -5.83357013379057348645e-02,
                           4.97687799461593236017e-02, -3.65315727442169155270e-02,
                           1.62858201153657823623e-02};
    if (x != x) return x;
    double sgn = 1.0;
    if (x < 0.0) { x = -x; sgn = -1.0; }
    if (x == INFINITY) return sgn * (atanhi[3] + atanlo[3]);
    int id;
    if (x < 0.4375) {
        id = -1;
    } else if (x < 1.1875) {
        if (x < 0.6875) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }
        else { id = 1; x = (x - 1.0) / (x + 1.0); }
    } else if (x < 2.4375) {
        id = 2; x = (x - 1.5) / (1.0 + 1.5 * x);
    } else {
        id = 3; x = -1.0 / x;
    }
    double z = x * x;
    double w = z * z;
    double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return sgn * (x - x * (s1 + s2));
    double r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return sgn * r;
}

static inline double dm_atan2(double y, double x)
{
    const double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
    if (x != x || y != y) return x + y;
    if (y == 0.0) {
        if (signbit(x)) return signbit(y) ? -pi : pi;
        return y;
    }
    if (x == 0.0) return y > 0.0 ? pi * 0.5 : -pi * 0.5;
    double a = dm_atan(fabs(y / x));
    if (x > 0.0) return y > 0.0 ? a : -a;
    double r = pi - (a - pi_lo);
    return y > 0.0 ? r : -r;
}

/* float wrappers: evaluate in double, round once */
static inline float dm_expf(float x) { return (float)dm_exp((double)x); }
static inline float dm_logf(float x) { return (float)dm_log((double)x); }
static inline float dm_cosf(float x) { double s, c; dm_sincos((double)x, &s, &c); return (float)c; }
static inline float dm_sinf(float x) { double s, c; dm_sincos((double)x, &s, &c); return (float)s; }
static inline float dm_atan2f(float y, float x) { return (float)dm_atan2((double)y, (double)x); }
static inline float dm_cbrtf(float xf)
{
    double x = (double)xf;
    if (x == 0.0 || x != x) return xf;
    double ax = fabs(x);
    double y = dm_exp(dm_log(ax) / 3.0);
    y = y - (y * y * y - ax) / (3.0 * y * y);
    return (float)(x < 0.0 ? -y : y);
}

#endif
