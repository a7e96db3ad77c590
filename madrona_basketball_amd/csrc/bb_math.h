// bb_math.h -- deterministic scalar math for the basketball step, identical
// bit-for-bit on the host (CPU exec mode) and on gfx950.
//
// The reference calls libm: sinf/cosf/atan2f/atanf/acosf on floats and the
// double overloads of erf/acos/exp (src/game.cpp:302,345,435,746,806,808,868;
// src/helper.cpp:39,135-136).  Its two executors disagree with each other in
// the last ulp (glibc on the CPU executor, CUDA libdevice under NVRTC), so this
// build fixes one platform-independent definition:
//
//     float  f(float x)   :=  (float) f_binary64(x)
//
// where f_binary64 is evaluated here from IEEE-754 binary64 add/mul/fma/div/
// sqrt only (Cody-Waite reduction + Taylor/Horner kernels, tables from
// tools/gen_math_tables.py).  Every f_binary64 is within ~1 ulp of the true
// value, so the float result is the correctly rounded one except for inputs
// within ~2^-28 relative of a float rounding boundary (tested against
// (float)libm_double(x) in tests/test_math.py).  Compile with
// -ffp-contract=off: every product and sum below is meant to round on its own.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BB_HD __host__ __device__ __forceinline__
#else
#define BB_HD static inline
#endif

namespace bbm {

BB_HD double fma_d(double a, double b, double c) { return __builtin_fma(a, b, c); }
BB_HD double rint_d(double x) { return __builtin_rint(x); }
BB_HD double fabs_d(double x) { return __builtin_fabs(x); }
BB_HD double sqrt_d(double x) { return __builtin_sqrt(x); }
BB_HD double ldexp_d(double x, int k) { return __builtin_ldexp(x, k); }
BB_HD bool isnan_d(double x) { return x != x; }
BB_HD bool signbit_d(double x) { return __builtin_signbit(x); }
BB_HD double nan_d() { return __builtin_nan(""); }
BB_HD double inf_d() { return __builtin_inf(); }

// ---------------------------------------------------------------- tables
// atan(i/8), i = 0..8  (tools/gen_math_tables.py)
static constexpr double ATAN_HI[9] = {
    0.0, 0.12435499454676144, 0.24497866312686414, 0.35877067027057225, 0.4636476090008061,
    0.5585993153435624, 0.6435011087932844, 0.7188299996216245, 0.7853981633974483};
static constexpr double ATAN_LO[9] = {
    0.0, -3.1253241424539383e-18, 1.0698755618734451e-17, -2.4623815582638635e-17,
    2.2698777452961687e-17, -5.4556305485916264e-18, 1.5834785051444286e-17,
    -2.1478388444456983e-17, 3.061616997868383e-17};
static constexpr double PI_HI = 3.141592653589793;
static constexpr double PI_LO = 1.2246467991473532e-16;
static constexpr double PIO2_HI = 1.5707963267948966;
static constexpr double PIO2_LO = 6.123233995736766e-17;

// pi/2 split in 33-bit pieces (Cody-Waite), 2/pi, ln2 split (32-bit high part).
static constexpr double INV_PIO2 = 6.36619772367581382433e-01;
static constexpr double PIO2_1 = 1.57079632673412561417e+00;
static constexpr double PIO2_2 = 6.07710050630396597660e-11;
static constexpr double PIO2_3 = 2.02226624871116645580e-21;
static constexpr double INV_LN2 = 1.44269504088896338700e+00;
static constexpr double LN2_HI = 6.93147180369123816490e-01;
static constexpr double LN2_LO = 1.90821492927058770002e-10;
static constexpr double TWO_OVER_SQRTPI = 1.1283791670955126;   // 2/sqrt(pi)
static constexpr double INV_SQRTPI = 0.5641895835477563;        // 1/sqrt(pi)

// ---------------------------------------------------------------- sin / cos
// Kernels on |r| <= pi/4 (+ rounding slack): Taylor to r^23 / r^22.
BB_HD double sin_kernel(double r)
{
    const double z = r * r;
    double p = -1.0 / 25852016738884976640000.0;   // -1/23!
    p = fma_d(p, z, 1.0 / 51090942171709440000.0);  // 1/21!
    p = fma_d(p, z, -1.0 / 121645100408832000.0);   // -1/19!
    p = fma_d(p, z, 1.0 / 355687428096000.0);       // 1/17!
    p = fma_d(p, z, -1.0 / 1307674368000.0);        // -1/15!
    p = fma_d(p, z, 1.0 / 6227020800.0);            // 1/13!
    p = fma_d(p, z, -1.0 / 39916800.0);             // -1/11!
    p = fma_d(p, z, 1.0 / 362880.0);                // 1/9!
    p = fma_d(p, z, -1.0 / 5040.0);                 // -1/7!
    p = fma_d(p, z, 1.0 / 120.0);                   // 1/5!
    p = fma_d(p, z, -1.0 / 6.0);                    // -1/3!
    return fma_d(r * z, p, r);
}

BB_HD double cos_kernel(double r)
{
    const double z = r * r;
    double q = -1.0 / 1124000727777607680000.0;     // -1/22!
    q = fma_d(q, z, 1.0 / 2432902008176640000.0);   // 1/20!
    q = fma_d(q, z, -1.0 / 6402373705728000.0);     // -1/18!
    q = fma_d(q, z, 1.0 / 20922789888000.0);        // 1/16!
    q = fma_d(q, z, -1.0 / 87178291200.0);          // -1/14!
    q = fma_d(q, z, 1.0 / 479001600.0);             // 1/12!
    q = fma_d(q, z, -1.0 / 3628800.0);              // -1/10!
    q = fma_d(q, z, 1.0 / 40320.0);                 // 1/8!
    q = fma_d(q, z, -1.0 / 720.0);                  // -1/6!
    q = fma_d(q, z, 1.0 / 24.0);                    // 1/4!
    // cos r = 1 - z/2 + z^2 q, with the 1 - z/2 split kept exact (fdlibm style)
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    return w + fma_d(z * z, q, (1.0 - w) - hz);
}

// x -> (r, quadrant) with x = r + k pi/2; exact-enough for |x| < 2^20 pi/2.
BB_HD double reduce_pio2(double x, int *quadrant)
{
    const double k = rint_d(x * INV_PIO2);
    double r = fma_d(-k, PIO2_1, x);
    r = fma_d(-k, PIO2_2, r);
    r = fma_d(-k, PIO2_3, r);
    *quadrant = (int)((int64_t)k & 3);
    return r;
}

BB_HD void sincos_d(double x, double *s, double *c)
{
    if (!(fabs_d(x) <= 1.0e15)) {   // NaN, inf, absurd angles: deterministic junk
        *s = x - x; *c = x - x;
        return;
    }
    int q;
    const double r = reduce_pio2(x, &q);
    const double sr = sin_kernel(r), cr = cos_kernel(r);
    switch (q) {
    case 0: *s = sr; *c = cr; break;
    case 1: *s = cr; *c = -sr; break;
    case 2: *s = -sr; *c = -cr; break;
    default: *s = -cr; *c = sr; break;
    }
}

BB_HD double sin_d(double x) { double s, c; sincos_d(x, &s, &c); return s; }
BB_HD double cos_d(double x) { double s, c; sincos_d(x, &s, &c); return c; }

// ---------------------------------------------------------------- atan family
// atan on [0, 1]: atan(t) = atan(c) + atan((t - c) / (1 + t c)), c = i/8.
BB_HD double atan01(double t)
{
    const int i = (int)(t * 8.0 + 0.5);
    const double c = (double)i * 0.125;
    const double u = (t - c) / fma_d(t, c, 1.0);
    const double z = u * u;
    double p = 1.0 / 21.0;
    p = fma_d(p, z, -1.0 / 19.0);
    p = fma_d(p, z, 1.0 / 17.0);
    p = fma_d(p, z, -1.0 / 15.0);
    p = fma_d(p, z, 1.0 / 13.0);
    p = fma_d(p, z, -1.0 / 11.0);
    p = fma_d(p, z, 1.0 / 9.0);
    p = fma_d(p, z, -1.0 / 7.0);
    p = fma_d(p, z, 1.0 / 5.0);
    p = fma_d(p, z, -1.0 / 3.0);
    const double at = fma_d(u * z, p, u);
    return ATAN_HI[i] + (ATAN_LO[i] + at);
}

BB_HD double atan_d(double x)
{
    if (isnan_d(x)) return x;
    const double t = fabs_d(x);
    double r;
    if (t <= 1.0) r = atan01(t);
    else r = PIO2_HI - (atan01(1.0 / t) - PIO2_LO);
    return signbit_d(x) ? -r : r;
}

BB_HD double atan2_d(double y, double x)
{
    if (isnan_d(x) || isnan_d(y)) return x + y;
    const double ax = fabs_d(x), ay = fabs_d(y);
    const bool xneg = signbit_d(x);
    double r;
    if (ay == 0.0) {
        r = xneg ? PI_HI : 0.0;
    } else if (ax == 0.0) {
        r = PIO2_HI;
    } else if (ax == inf_d() && ay == inf_d()) {
        r = xneg ? 3.0 * (PIO2_HI * 0.5) : PIO2_HI * 0.5;
    } else {
        if (ay <= ax) r = atan01(ay / ax);
        else r = PIO2_HI - (atan01(ax / ay) - PIO2_LO);
        if (xneg) r = PI_HI - (r - PI_LO);
    }
    return signbit_d(y) ? -r : r;
}

BB_HD double acos_d(double x)
{
    if (isnan_d(x)) return x;
    if (x > 1.0 || x < -1.0) return nan_d();
    const double s = sqrt_d((1.0 - x) * (1.0 + x));
    return atan2_d(s, x);
}

// ---------------------------------------------------------------- exp / erf
BB_HD double exp_d(double x)
{
    if (isnan_d(x)) return x;
    if (x > 709.782712893384) return inf_d();
    if (x < -745.1332191019412) return 0.0;
    const double k = rint_d(x * INV_LN2);
    double r = fma_d(-k, LN2_HI, x);
    r = fma_d(-k, LN2_LO, r);
    // exp(r), |r| <= 0.3466: Taylor to r^14
    double p = 1.0 / 87178291200.0;          // 1/14!
    p = fma_d(p, r, 1.0 / 6227020800.0);     // 1/13!
    p = fma_d(p, r, 1.0 / 479001600.0);
    p = fma_d(p, r, 1.0 / 39916800.0);
    p = fma_d(p, r, 1.0 / 3628800.0);
    p = fma_d(p, r, 1.0 / 362880.0);
    p = fma_d(p, r, 1.0 / 40320.0);
    p = fma_d(p, r, 1.0 / 5040.0);
    p = fma_d(p, r, 1.0 / 720.0);
    p = fma_d(p, r, 1.0 / 120.0);
    p = fma_d(p, r, 1.0 / 24.0);
    p = fma_d(p, r, 1.0 / 6.0);
    p = fma_d(p, r, 0.5);
    p = fma_d(p, r, 1.0);
    p = fma_d(p, r, 1.0);
    return ldexp_d(p, (int)k);
}

// Maclaurin coefficients of erf(x) sqrt(pi)/(2x) in z = x^2: (-1)^n / (n! (2n+1)),
// folded at compile time (identical on host and device).
static constexpr int ERF_NT = 56;
struct ErfCoef {
    double c[ERF_NT];
    constexpr ErfCoef() : c()
    {
        double f = 1.0;
        for (int n = 0; n < ERF_NT; n++) {
            c[n] = ((n & 1) ? -f : f) / (double)(2 * n + 1);
            f = f / (double)(n + 1);
        }
    }
};
static constexpr ErfCoef ERF_COEF{};

// erf: Maclaurin series (Horner in x^2) below 3, 1 - erfc by the Laplace
// continued fraction from 3 to 6, 1 above.  Absolute error < 1e-12 (the
// reference only rounds it to float, src/game.cpp:808).
BB_HD double erf_d(double x)
{
    if (isnan_d(x)) return x;
    const double ax = fabs_d(x);
    double r;
    if (ax < 3.0) {
        // erf x = 2/sqrt(pi) * x * sum_n (-1)^n z^n / (n! (2n+1)), z = x^2
        const double z = ax * ax;
        double p = ERF_COEF.c[ERF_NT - 1];
#pragma unroll
        for (int n = ERF_NT - 2; n >= 0; n--) p = fma_d(p, z, ERF_COEF.c[n]);
        r = TWO_OVER_SQRTPI * (ax * p);
    } else if (ax < 6.0) {
        // erfc x = exp(-x^2)/sqrt(pi) * 1/(x + (1/2)/(x + 1/(x + (3/2)/(x + ...))))
        double f = ax;
        for (int k = 40; k >= 1; k--) f = ax + (0.5 * (double)k) / f;
        r = 1.0 - exp_d(-(ax * ax)) * INV_SQRTPI / f;
    } else {
        r = 1.0;
    }
    return signbit_d(x) ? -r : r;
}

// ---------------------------------------------------------------- float API
BB_HD float sinf_(float x) { return (float)sin_d((double)x); }
BB_HD float cosf_(float x) { return (float)cos_d((double)x); }
BB_HD void sincosf_(float x, float *s, float *c)
{
    double sd, cd;
    sincos_d((double)x, &sd, &cd);
    *s = (float)sd; *c = (float)cd;
}
BB_HD float atan2f_(float y, float x) { return (float)atan2_d((double)y, (double)x); }
BB_HD float atanf_(float x) { return (float)atan_d((double)x); }
BB_HD float acosf_(float x) { return (float)acos_d((double)x); }
BB_HD float sqrtf_(float x) { return __builtin_sqrtf(x); }

}  // namespace bbm
