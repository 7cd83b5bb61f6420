// wos_detmath.h -- deterministic scalar math shared by the gfx950 kernels and the
// host-side scene preparation.  Everything here uses only IEEE-correctly-rounded
// +,-,*,/,sqrt (built with -ffp-contract=off), so the GPU produces bit-identical
// results to the CPU oracle in "det" math mode.
//
//   * exp/log/sin/cos/atan: fdlibm-structured Cody-Waite reduction + polynomial,
//     float variants evaluated in double and rounded once.
//   * modified Bessel I0, I1, K0, K1 (double): the polynomial approximations the
//     reference uses (bindings/zombie/deps/bessel/bessel.hpp:373-555, Abramowitz &
//     Stegun 9.8), same Horner order.
//   * PCG32 (deps/pcg32/pcg32.h:53-112) and the counter-based seed hash that
//     replaces the reference's std::chrono::system_clock seeds
//     (walk_on_stars.h:498,639).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define WOS_HD __host__ __device__ __forceinline__
#else
// plain host C++ (g++): the scene preparation is also built this way by the CPU
// test suite (tests/test_host_scene.py), which checks the culling records
#define WOS_HD inline
#endif

namespace wos {

constexpr double kPi = 3.141592653589793;
constexpr double kTwoPi = 6.283185307179586;    // 2.0f*M_PI evaluated in double
constexpr double kFourPi = 12.566370614359172;  // 4.0f*M_PI evaluated in double
constexpr float kFltEps = 1.1920928955078125e-07f;
constexpr float kFltMax = 3.4028234663852886e+38f;

WOS_HD double bits_to_double(uint64_t u) { return __builtin_bit_cast(double, u); }
WOS_HD uint64_t double_to_bits(double d) { return __builtin_bit_cast(uint64_t, d); }
WOS_HD float bits_to_float(uint32_t u) { return __builtin_bit_cast(float, u); }
WOS_HD uint32_t float_to_bits(float f) { return __builtin_bit_cast(uint32_t, f); }

WOS_HD double pow2i(int k) { return bits_to_double((uint64_t)(k + 1023) << 52); }

WOS_HD double dexp(double x) {
  if (x != x) return x;
  if (x > 709.782712893384) return __builtin_inf();
  if (x < -745.1332191019412) return 0.0;
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  const double inv_ln2 = 1.44269504088896338700e+00;
  const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  double kd = __builtin_floor(x * inv_ln2 + 0.5);
  int k = (int)kd;
  double hi = x - kd * ln2_hi;
  double lo = kd * ln2_lo;
  double r = hi - lo;
  double t = r * r;
  double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
  if (k > 1023) return (y * pow2i(1023)) * 2.0;
  if (k >= -1021) return y * pow2i(k);
  return (y * pow2i(k + 1000)) * pow2i(-1000);
}

WOS_HD double dlog(double x) {
  if (x != x) return x;
  if (x < 0.0) return __builtin_nan("");
  if (x == 0.0) return -__builtin_inf();
  if (x == __builtin_inf()) return x;
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  int k = 0;
  if (x < 2.2250738585072014e-308) { x *= 18014398509481984.0; k = -54; }
  uint64_t u = double_to_bits(x);
  int e = (int)((u >> 52) & 0x7ff) - 1023;
  double m = bits_to_double((u & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL);
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

WOS_HD void dsincos(double x, double* sp, double* cp) {
  if (x != x || x == __builtin_inf() || x == -__builtin_inf()) {
    *sp = __builtin_nan(""); *cp = __builtin_nan(""); return;
  }
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
  double kd = __builtin_floor(x * two_over_pi + 0.5);
  double r = ((x - kd * pio2_1) - kd * pio2_2) - kd * pio2_3;
  double z = r * r;
  double s = r + (z * r) * (S1 + z * (S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)))));
  double c = (1.0 - 0.5 * z) + (z * z) * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  int64_t ki = (int64_t)kd;
  int q = (int)(ki & 3);
  if (q == 0) { *sp = s; *cp = c; }
  else if (q == 1) { *sp = c; *cp = -s; }
  else if (q == 2) { *sp = -s; *cp = -c; }
  else { *sp = -c; *cp = s; }
}

WOS_HD double datan(double x) {
  const double atanhi0 = 4.63647609000806093515e-01, atanhi1 = 7.85398163397448278999e-01,
               atanhi2 = 9.82793723247329054082e-01, atanhi3 = 1.57079632679489655800e+00;
  const double atanlo0 = 2.26987774529616870924e-17, atanlo1 = 3.06161699786838301793e-17,
               atanlo2 = 1.39033110312309984516e-17, atanlo3 = 6.12323399573676603587e-17;
  const double a0 = 3.33333333333329318027e-01, a1 = -1.99999999998764832476e-01,
               a2 = 1.42857142725034663711e-01, a3 = -1.11111104054623557880e-01,
               a4 = 9.09088713343650656196e-02, a5 = -7.69187620504482999495e-02,
               a6 = 6.66107313738753120669e-02, a7 = -5.83357013379057348645e-02,
               a8 = 4.97687799461593236017e-02, a9 = -3.65315727442169155270e-02,
               a10 = 1.62858201153657823623e-02;
  if (x != x) return x;
  double sgn = 1.0;
  if (x < 0.0) { x = -x; sgn = -1.0; }
  if (x == __builtin_inf()) return sgn * (atanhi3 + atanlo3);
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
  double s1 = z * (a0 + w * (a2 + w * (a4 + w * (a6 + w * (a8 + w * a10)))));
  double s2 = w * (a1 + w * (a3 + w * (a5 + w * (a7 + w * a9))));
  if (id < 0) return sgn * (x - x * (s1 + s2));
  double hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  double lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  double r = hi - ((x * (s1 + s2) - lo) - x);
  return sgn * r;
}

WOS_HD double datan2(double y, double x) {
  const double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
  if (x != x || y != y) return x + y;
  if (y == 0.0) {
    if (__builtin_signbit(x)) return __builtin_signbit(y) ? -pi : pi;
    return y;
  }
  if (x == 0.0) return y > 0.0 ? pi * 0.5 : -pi * 0.5;
  double a = datan(__builtin_fabs(y / x));
  if (x > 0.0) return y > 0.0 ? a : -a;
  double r = pi - (a - pi_lo);
  return y > 0.0 ? r : -r;
}

WOS_HD float fexp(float x) { return (float)dexp((double)x); }
WOS_HD float flog(float x) { return (float)dlog((double)x); }
WOS_HD float fcos(float x) { double s, c; dsincos((double)x, &s, &c); return (float)c; }
WOS_HD float fsin(float x) { double s, c; dsincos((double)x, &s, &c); return (float)s; }
WOS_HD void fsincos(float x, float* s, float* c) {
  double sd, cd; dsincos((double)x, &sd, &cd); *s = (float)sd; *c = (float)cd;
}
WOS_HD float fatan2(float y, float x) { return (float)datan2((double)y, (double)x); }
WOS_HD float fcbrt(float xf) {
  double x = (double)xf;
  if (x == 0.0 || x != x) return xf;
  double ax = __builtin_fabs(x);
  double y = dexp(dlog(ax) / 3.0);
  y = y - (y * y * y - ax) / (3.0 * y * y);
  return (float)(x < 0.0 ? -y : y);
}

// std::max / std::min / std::clamp semantics
WOS_HD float smax(float a, float b) { return (a < b) ? b : a; }
WOS_HD float smin(float a, float b) { return (b < a) ? b : a; }
WOS_HD int sclamp(int v, int lo, int hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }
// int(float) with x86 cvttss2si semantics (NaN / out of range -> INT_MIN)
WOS_HD int cvt_trunc(float x) {
  if (!(x > -2147483904.0f && x < 2147483648.0f)) return (int)0x80000000u;
  return (int)x;
}

// ---------------------------------------------------------------------------
// Modified Bessel functions in double (bessel.hpp:373-555)
// ---------------------------------------------------------------------------
WOS_HD double bessi0(double x) {
  double ax = __builtin_fabs(x), y;
  if (ax < 3.75) {
    y = x / 3.75; y = y * y;
    return 1.0 + y * (3.5156229 + y * (3.0899424 + y * (1.2067492 + y * (0.2659732 +
           y * (0.360768e-1 + y * 0.45813e-2)))));
  }
  y = 3.75 / ax;
  return (dexp(ax) / __builtin_sqrt(ax)) * (0.39894228 + y * (0.1328592e-1 + y * (0.225319e-2 +
         y * (-0.157565e-2 + y * (0.916281e-2 + y * (-0.2057706e-1 + y * (0.2635537e-1 +
         y * (-0.1647633e-1 + y * 0.392377e-2))))))));
}

WOS_HD double bessi1(double x) {
  double ax = __builtin_fabs(x), y, ans;
  if (ax < 3.75) {
    y = x / 3.75; y = y * y;
    ans = ax * (0.5 + y * (0.87890594 + y * (0.51498869 + y * (0.15084934 + y * (0.2658733e-1 +
          y * (0.301532e-2 + y * 0.32411e-3))))));
  } else {
    y = 3.75 / ax;
    ans = 0.2282967e-1 + y * (-0.2895312e-1 + y * (0.1787654e-1 - y * 0.420059e-2));
    ans = 0.39894228 + y * (-0.3988024e-1 + y * (-0.362018e-2 + y * (0.163801e-2 +
          y * (-0.1031555e-1 + y * ans))));
    ans *= (dexp(ax) / __builtin_sqrt(ax));
  }
  return x < 0.0 ? -ans : ans;
}

WOS_HD double bessk0(double x) {
  double y;
  if (x <= 2.0) {
    y = x * x / 4.0;
    return (-dlog(x / 2.0) * bessi0(x)) + (-0.57721566 + y * (0.42278420 + y * (0.23069756 +
           y * (0.3488590e-1 + y * (0.262698e-2 + y * (0.10750e-3 + y * 0.74e-5))))));
  }
  y = 2.0 / x;
  return (dexp(-x) / __builtin_sqrt(x)) * (1.25331414 + y * (-0.7832358e-1 + y * (0.2189568e-1 +
         y * (-0.1062446e-1 + y * (0.587872e-2 + y * (-0.251540e-2 + y * 0.53208e-3))))));
}

WOS_HD double bessk1(double x) {
  double y;
  if (x <= 2.0) {
    y = x * x / 4.0;
    return (dlog(x / 2.0) * bessi1(x)) + (1.0 / x) * (1.0 + y * (0.15443144 + y * (-0.67278579 +
           y * (-0.18156897 + y * (-0.1919402e-1 + y * (-0.110404e-2 + y * (-0.4686e-4)))))));
  }
  y = 2.0 / x;
  return (dexp(-x) / __builtin_sqrt(x)) * (1.25331414 + y * (0.23498619 + y * (-0.3655620e-1 +
         y * (0.1504268e-1 + y * (-0.780353e-2 + y * (0.325614e-2 + y * (-0.68245e-3)))))));
}

// I and K of order 0 and/or 1 at the same x >= 0, the shared pieces evaluated once:
// the operations of bessi0 / bessi1 / bessk0 / bessk1 above, operand for operand, so
// the values are identical -- y and dexp(x)/sqrt(x) of the I's, dlog(x/2) and
// I0 / I1 reused by the K's for x <= 2, 2/x and dexp(-x)/sqrt(x) of the K's for
// x > 2.  (The ball update needs all four at mu R; the Green's function, its
// gradient and the direction-sampled Poisson kernel need one order at mu r.)
template <bool N0, bool N1>
WOS_HD void bessel_ik(double x, double* i0, double* k0, double* i1, double* k1) {
  const double ax = __builtin_fabs(x);
  double vi0 = 0.0, vi1 = 0.0;
  if (ax < 3.75) {
    double y = x / 3.75;
    y = y * y;
    if (N0)
      vi0 = 1.0 + y * (3.5156229 + y * (3.0899424 + y * (1.2067492 + y * (0.2659732 +
            y * (0.360768e-1 + y * 0.45813e-2)))));
    if (N1)
      vi1 = ax * (0.5 + y * (0.87890594 + y * (0.51498869 + y * (0.15084934 + y * (0.2658733e-1 +
            y * (0.301532e-2 + y * 0.32411e-3))))));
  } else {
    const double y = 3.75 / ax;
    const double e = dexp(ax) / __builtin_sqrt(ax);
    if (N0)
      vi0 = e * (0.39894228 + y * (0.1328592e-1 + y * (0.225319e-2 +
            y * (-0.157565e-2 + y * (0.916281e-2 + y * (-0.2057706e-1 + y * (0.2635537e-1 +
            y * (-0.1647633e-1 + y * 0.392377e-2))))))));
    if (N1) {
      double ans = 0.2282967e-1 + y * (-0.2895312e-1 + y * (0.1787654e-1 - y * 0.420059e-2));
      ans = 0.39894228 + y * (-0.3988024e-1 + y * (-0.362018e-2 + y * (0.163801e-2 +
            y * (-0.1031555e-1 + y * ans))));
      vi1 = ans * e;
    }
  }
  if (N1 && x < 0.0) vi1 = -vi1;
  if (x <= 2.0) {
    const double y = x * x / 4.0;
    const double l = dlog(x / 2.0);
    if (N0)
      *k0 = (-l * vi0) + (-0.57721566 + y * (0.42278420 + y * (0.23069756 +
            y * (0.3488590e-1 + y * (0.262698e-2 + y * (0.10750e-3 + y * 0.74e-5))))));
    if (N1)
      *k1 = (l * vi1) + (1.0 / x) * (1.0 + y * (0.15443144 + y * (-0.67278579 +
            y * (-0.18156897 + y * (-0.1919402e-1 + y * (-0.110404e-2 + y * (-0.4686e-4)))))));
  } else {
    const double y = 2.0 / x;
    const double e = dexp(-x) / __builtin_sqrt(x);
    if (N0)
      *k0 = e * (1.25331414 + y * (-0.7832358e-1 + y * (0.2189568e-1 +
            y * (-0.1062446e-1 + y * (0.587872e-2 + y * (-0.251540e-2 + y * 0.53208e-3))))));
    if (N1)
      *k1 = e * (1.25331414 + y * (0.23498619 + y * (-0.3655620e-1 +
            y * (0.1504268e-1 + y * (-0.780353e-2 + y * (0.325614e-2 + y * (-0.68245e-3)))))));
  }
  if (N0) *i0 = vi0;
  if (N1) *i1 = vi1;
}

// Robust float semantics (wos_solver_params.robust_float): exponentially scaled A&S
// functions ie_v(x) = e^-x I_v(x), ke_v(x) = e^x K_v(x), x > 0 -- the polynomials above
// without the exponential (large x) or times the compensating exponential (small x),
// so nothing overflows.  Operation for operation as oracle/wos_oracle.c bess_scaled.
WOS_HD void bessel_scaled(double x, double* ie0, double* ke0, double* ie1, double* ke1) {
  if (x < 3.75) {
    const double e = dexp(-x);
    *ie0 = bessi0(x) * e;
    *ie1 = bessi1(x) * e;
  } else {
    const double y = 3.75 / x, sx = __builtin_sqrt(x);
    *ie0 = (0.39894228 + y * (0.1328592e-1 + y * (0.225319e-2 + y * (-0.157565e-2 + y * (0.916281e-2 +
           y * (-0.2057706e-1 + y * (0.2635537e-1 + y * (-0.1647633e-1 + y * 0.392377e-2)))))))) / sx;
    double a = 0.2282967e-1 + y * (-0.2895312e-1 + y * (0.1787654e-1 - y * 0.420059e-2));
    a = 0.39894228 + y * (-0.3988024e-1 + y * (-0.362018e-2 + y * (0.163801e-2 + y * (-0.1031555e-1 + y * a))));
    *ie1 = a / sx;
  }
  if (x <= 2.0) {
    const double e = dexp(x);
    *ke0 = bessk0(x) * e;
    *ke1 = bessk1(x) * e;
  } else {
    const double y = 2.0 / x, sx = __builtin_sqrt(x);
    *ke0 = (1.25331414 + y * (-0.7832358e-1 + y * (0.2189568e-1 + y * (-0.1062446e-1 + y * (0.587872e-2 +
           y * (-0.251540e-2 + y * 0.53208e-3)))))) / sx;
    *ke1 = (1.25331414 + y * (0.23498619 + y * (-0.3655620e-1 + y * (0.1504268e-1 + y * (-0.780353e-2 +
           y * (0.325614e-2 + y * (-0.68245e-3))))))) / sx;
  }
}

// 3D robust member: (cosh x - sinh x / x) e^-x
WOS_HD double i32_scaled(double x) {
  const double e2 = dexp(-2.0 * x);
  return 0.5 * ((1.0 + e2) - (1.0 - e2) / x);
}

// ---------------------------------------------------------------------------
// PCG32 (pcg32.h) + counter-based seeding
// ---------------------------------------------------------------------------
constexpr uint64_t kPcgMult = 0x5851f42d4c957f2dULL;
// every stream is seeded with initseq = 1 (the counter-based seed32 key selects
// the stream through initstate), so the increment is the constant (1 << 1) | 1
// and a generator is one 64-bit register pair.
constexpr uint64_t kPcgInc = 3u;
// two steps at once: state * kPcgMult2 + kPcgInc2 == (state * kPcgMult + kPcgInc) * kPcgMult + kPcgInc
constexpr uint64_t kPcgMult2 = kPcgMult * kPcgMult;
constexpr uint64_t kPcgInc2 = kPcgInc * kPcgMult + kPcgInc;

struct Pcg32 {
  uint64_t state;
  WOS_HD void seed(uint64_t initstate) {
    state = 0u;
    next(); state += initstate; next();
  }
  WOS_HD uint32_t next() {
    uint64_t old = state;
    state = old * kPcgMult + kPcgInc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((~rot + 1u) & 31));
  }
  WOS_HD float nextf() { return bits_to_float((next() >> 9) | 0x3f800000u) - 1.0f; }
  WOS_HD uint32_t bounded(uint32_t bound) {
    uint32_t th = (~bound + 1u) % bound;
    for (;;) { uint32_t r = next(); if (r >= th) return r % bound; }
  }
};

WOS_HD uint32_t pcg_output(uint64_t old) {
  uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
  uint32_t rot = (uint32_t)(old >> 59u);
  return (xs >> rot) | (xs << ((~rot + 1u) & 31));
}

WOS_HD uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// tag 0: per-point stratified-sample stream; 1: per-pair first-ball stream;
// 2: per-pair walk stream (shared by both antithetic members).
WOS_HD uint32_t seed32(uint64_t key, uint64_t idx, uint64_t pair, uint32_t tag) {
  uint64_t h = mix64(key ^ mix64(idx * 0x9E3779B97F4A7C15ULL + pair * 0xD1B54A32D192ED03ULL +
                                 (uint64_t)tag * 0x8CB92BA72F3D8DD7ULL + 0x632BE59BD9B4E019ULL));
  return (uint32_t)(h >> 32);
}

}  // namespace wos
