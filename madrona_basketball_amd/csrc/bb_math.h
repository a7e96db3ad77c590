// bb_math.h -- deterministic scalar math for the basketball step, identical
// bit-for-bit on the host (CPU exec mode) and on gfx950.
//
// The reference calls libm: sinf/cosf/atan2f/atanf/acosf on floats and the
// double overloads of erf/acos/exp (src/game.cpp:302,345,435,746,806,808,868;
// src/helper.cpp:39,135-136).  Its CPU TaskGraph executor -- the north_star's
// parity target -- gets them from glibc.  So:
//
//   * the float functions are glibc 2.35's own algorithms, restated operation
//     for operation (section "float API" below; exhaustively equal to the
//     host libm on every float input, tests/test_math.py);
//   * the double functions (erf, exp, acos on a float argument, rounded back
//     to float by the reference) are evaluated here from IEEE-754 binary64
//     add/mul/fma/div/sqrt only (Horner / Taylor kernels, tables from
//     tools/gen_math_tables.py), within ~1 double ulp of libm's: their float
//     results equal libm's except within ~2^-29 relative of a float rounding
//     boundary (tests/test_math.py).
//
// Compile with -ffp-contract=off: every product and sum below is meant to
// round on its own; fused multiply-adds are written as fma_d.
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

// ln2 split (32-bit high part).
static constexpr double INV_LN2 = 1.44269504088896338700e+00;
static constexpr double LN2_HI = 6.93147180369123816490e-01;
static constexpr double LN2_LO = 1.90821492927058770002e-10;
static constexpr double TWO_OVER_SQRTPI = 1.1283791670955126;   // 2/sqrt(pi)
static constexpr double TWO_OVER_SQRTPI_M1 = 1.28379167095512586316e-01;  // 2/sqrt(pi) - 1
static constexpr double INV_SQRTPI = 0.5641895835477563;        // 1/sqrt(pi)

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
    // table entry by register selects (a per-lane table load would wait on memory)
    double hi = ATAN_HI[0], lo = ATAN_LO[0];
#pragma unroll
    for (int j = 1; j < 9; j++) {
        hi = (i == j) ? ATAN_HI[j] : hi;
        lo = (i == j) ? ATAN_LO[j] : lo;
    }
    return hi + (lo + at);
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

// log (double; the policy's own f32 log is pol_logf, bb_policy.h): x = m 2^e with
// m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s), s = (m - 1)/(m + 1), |s| <= 0.1716:
// odd series to s^25 (next term < 2^-60).
BB_HD double log_d(double x)
{
    if (isnan_d(x) || x < 0.0) return nan_d();
    if (x == 0.0) return -inf_d();
    if (x == inf_d()) return x;
    int e = 0;
    double m = __builtin_frexp(x, &e);  // [0.5, 1)
    if (m < 0.7071067811865476) { m = m * 2.0; e -= 1; }
    const double s = (m - 1.0) / (m + 1.0);
    const double z = s * s;
    double p = 1.0 / 25.0;
    p = fma_d(p, z, 1.0 / 23.0);
    p = fma_d(p, z, 1.0 / 21.0);
    p = fma_d(p, z, 1.0 / 19.0);
    p = fma_d(p, z, 1.0 / 17.0);
    p = fma_d(p, z, 1.0 / 15.0);
    p = fma_d(p, z, 1.0 / 13.0);
    p = fma_d(p, z, 1.0 / 11.0);
    p = fma_d(p, z, 1.0 / 9.0);
    p = fma_d(p, z, 1.0 / 7.0);
    p = fma_d(p, z, 1.0 / 5.0);
    p = fma_d(p, z, 1.0 / 3.0);
    const double lm = 2.0 * fma_d(s * z, p, s);
    const double k = (double)e;
    return fma_d(k, LN2_HI, fma_d(k, LN2_LO, lm));
}

// Maclaurin coefficients of erf(x) sqrt(pi)/(2x) in z = x^2: (-1)^n / (n! (2n+1)),
// folded at compile time (identical on host and device).
static constexpr int ERF_NT = 17;  // z <= 0.5625: term 17 < 1e-19
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

// erf Taylor coefficients at c_k = 0.875 + k/4 (k = 0..12), degree 16
static constexpr int ERF_TK = 13, ERF_TD = 16;
static constexpr double ERF_TAYLOR[13][17] = {
    {0.7840750610598597, 0.5247450452901482, -0.45915191462887966, 0.09292360177013041, 0.11239656243519451, -0.0672158773833572, -0.010367785745906018, 0.018595726765847267, -0.0018461468559063715, -0.0032568627602662854, 0.000898154868541066, 0.0003900529044120407, -0.00019296678621782653, -2.903116273391371e-05, 2.9075064952881173e-05, 2.0224352255317938e-07, -3.4142112964487243e-06},
    {0.8883882317017078, 0.3182739585007693, -0.35805820331336546, 0.16245233298476766, 0.027973297133856677, -0.061323683605665806, 0.015536835449762896, 0.009606894225829976, -0.006031260883106729, -0.0003601919898013683, 0.0011532673547020597, -0.0001769550878579247, -0.0001415583990117997, 4.9455696834570095e-05, 1.0718804636659436e-05, -7.730906970255213e-06, -1.633684149181282e-07},
    {0.9481700727820903, 0.1703597736875156, -0.23424468882033395, 0.15793770685613426, -0.03050061052348098, -0.030605976268925736, 0.022161235262852557, -0.001419062360662139, -0.004261033441276509, 0.001577911232741016, 0.00032359146722315554, -0.0003391015230725006, 2.8681755518788118e-05, 4.175471522740388e-05, -1.1984028581486832e-05, -2.9725595025012275e-06, 1.909045332332529e-06},
    {0.9784437332399837, 0.08047225902251116, -0.13076742091158064, 0.11484061964670864, -0.049718863159090555, -0.0021349248406037306, 0.014414781131084502, -0.006184261515478821, -0.000576525430283408, 0.0014106850333898903, -0.00035597922602355293, -0.00012566368868411414, 8.79701620524859e-05, -4.270738262797687e-06, -1.0609039547562964e-05, 2.8273833059374034e-06, 6.634090465304774e-07},
    {0.9919900576701199, 0.03354582842421607, -0.06289842829540514, 0.0674410925611844, -0.04225988151097533, 0.011462583364876176, 0.004105187133212477, -0.004928393908239107, 0.001430501687370122, 0.00036225644575338666, -0.0003901575782455417, 7.37299378240623e-05, 3.607417901263836e-05, -2.0803824921141647e-05, 8.154185088040366e-07, 2.3718570297022424e-06, -6.51036150696934e-07},
    {0.9973459706405177, 0.012340820614333696, -0.026224243805459103, 0.033037405186289164, -0.026360828408612536, 0.012495482591433906, -0.0018214125933023405, -0.0018692572567887945, 0.0013833456162338344, -0.0002897798521792673, -0.00012277167237649306, 9.485303104752515e-05, -1.4992013287438935e-05, -8.475474393501074e-06, 4.549880654612466e-06, -2.397884034210181e-07, -4.671256150460798e-07},
    {0.9992170617821089, 0.004006477861670219, -0.009515384921466771, 0.013730533505098981, -0.013133213563482782, 0.00835739283377895, -0.0031140790431462596, 0.0001232696283780691, 0.0005941113102532914, -0.00033752784148497275, 5.4705936215888043e-05, 3.1608810695225705e-05, -2.0800599114722e-05, 3.1425661169499264e-06, 1.6767083573168686e-06, -9.200372609631897e-07, 7.752008682814561e-08},
    {0.9997946242638588, 0.001147875125882675, -0.003013172205442022, 0.004890426317562647, -0.005414293806653633, 0.004217880601717521, -0.0022468338447285286, 0.0006808680974231771, 3.464470636501039e-05, -0.00015260043098965162, 7.395616736023192e-05, -1.0326282078167697e-05, -6.687731493867075e-06, 4.157085191239199e-06, -6.770082881827777e-07, -2.7773383709897626e-07, 1.701157155860923e-07},
    {0.9999521451602562, 0.00029022828286249803, -0.0008344063132296819, 0.001502536006069391, -0.001881760070981522, 0.0017132632798079331, -0.0011400746242208634, 0.0005285700413700108, -0.00013560801204451028, -1.6139055904620542e-05, 3.338804817529197e-05, -1.4811906943601079e-05, 2.0385768990676424e-06, 1.1871804277151051e-06, -7.564152887325688e-07, 1.429749505827574e-07, 3.6866827486454585e-08},
    {0.9999901032653747, 6.475868323471298e-05, -0.00020237088510847805, 0.0004000197828977583, -0.0005575739490749213, 0.0005769615014743242, -0.00045231517761577534, 0.00026648105109162697, -0.00011126364024766743, 2.5450656904174918e-05, 3.873542145587109e-06, -6.36552916703948e-06, 2.7284794494107734e-06, -4.1406613481371433e-07, -1.7494853479255093e-07, 1.241605538071656e-07, -2.8089553938459793e-08},
    {0.9999981847185726, 1.2751740799765088e-05, -4.303712519920718e-05, 9.258295143162778e-05, -0.00014188802214113615, 0.00016377394446104548, -0.0001464088816143732, 0.0001021861966850395, -5.484627167849354e-05, 2.126516551455692e-05, -4.603538423927069e-06, -6.548557786086127e-07, 1.0658621972744764e-06, -4.6107699262719935e-07, 8.175172180466655e-08, 2.0297448084600926e-08, -1.8100686787902113e-08},
    {0.9999997048598075, 2.2159202846331124e-06, -8.032711031795032e-06, 1.8673744898626958e-05, -3.1168592284829685e-05, 3.959233534341495e-05, -3.952911393067182e-05, 3.151412148928749e-05, -2.0089148185951398e-05, 1.0055179082432725e-05, -3.7186007128168107e-06, 8.055029835948156e-07, 7.676629783825506e-08, -1.5640854840393676e-07, 7.087425570853251e-08, -1.4891022361493784e-08, -1.5211686584435892e-09},
    {0.999999957486056, 3.398223817809154e-07, -1.3168117294010471e-06, 3.2884895070257334e-06, -5.9325111767286764e-06, 8.208845471821727e-06, -9.021089087308752e-06, 8.033147329562849e-06, -5.849020956804992e-06, 3.4746560653893003e-06, -1.6530325028002647e-06, 5.960564526364828e-07, -1.3449365553980958e-07, -3.880333287181606e-09, 1.9883468745269102e-08, -9.792703301880837e-09, 2.4236026415671354e-09},
};

// erf: Maclaurin series (Horner in x^2) below 0.75; Taylor polynomials at the
// centres of 13 quarter-unit intervals on [0.75, 4) (no cancellation: every
// value there is > 0.7); 1 from 4 on, where erfc < 2^-25 and the float result
// is 1.  Absolute error ~2e-16 (the reference rounds erf to float,
// src/game.cpp:808).
// tab: ERF_TAYLOR's 13 x 17 coefficients (the kernels pass a copy in LDS: a
// per-lane table read there is an LDS read, not a memory load).
BB_HD double erf_d(double x, const double *tab = &ERF_TAYLOR[0][0])
{
    if (isnan_d(x)) return x;
    const double ax = fabs_d(x);
    double r;
    if (ax < 0.75) {
        // erf x = 2/sqrt(pi) * x * sum_n (-1)^n z^n / (n! (2n+1)), z = x^2,
        // evaluated as x + x*y with y = (2/sqrt(pi) - 1) + 2/sqrt(pi) z q(z)
        // (q: the series from n = 1 on): the leading x is exact and one fma
        // rounds the sum, so (float)erf_d equals glibc's (float)erf on every
        // float below 0.75 (tests/test_math.py, exhaustive; the plain product
        // form differed on one input, 1.8398030e-4).
        const double z = ax * ax;
        double q = ERF_COEF.c[ERF_NT - 1];
#pragma unroll
        for (int n = ERF_NT - 2; n >= 1; n--) q = fma_d(q, z, ERF_COEF.c[n]);
        const double y = fma_d(TWO_OVER_SQRTPI * z, q, TWO_OVER_SQRTPI_M1);
        r = fma_d(ax, y, ax);
    } else if (ax < 4.0) {
        const int k = (int)((ax - 0.75) * 4.0);
        const double t = ax - (0.875 + 0.25 * (double)k);  // exact, |t| <= 1/8
        const double *a = tab + k * (ERF_TD + 1);
        double p = a[ERF_TD];
#pragma unroll
        for (int n = ERF_TD - 1; n >= 0; n--) p = fma_d(p, t, a[n]);
        r = p;
    } else {
        r = 1.0;
    }
    return signbit_d(x) ? -r : r;
}

// ------------------------------------------------ float API: glibc 2.35 libm
// The reference CPU executor calls glibc's float functions (sinf/cosf/atan2f/
// atanf/acosf; src/game.cpp:302,345,435,806, src/helper.cpp:39,135-136).
// What follows restates glibc 2.35's x86-64 implementations operation for
// operation, so the step computes exactly what the reference CPU executor
// computes on the same inputs:
//   * sinf / cosf: the double-precision polynomial implementation
//     (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h) in its FMA ifunc
//     variant (selected on every AVX2+FMA host): the fused multiply-adds below
//     are exactly those of that variant; coefficient table __sincosf_table;
//   * atanf, atan2f, acosf: the single-precision fdlibm implementations
//     (s_atanf.c, e_atan2f.c, e_acosf.c; no ifunc variants), every float
//     operation rounding on its own (-ffp-contract=off).
// Constants are the words the library holds.  Pinned exhaustively (every
// float input) against the host's libm by tests/test_math.py.
//
// Attribution.  The atanf / atan2f / acosf algorithms and constants below
// follow fdlibm (float versions by Ian Lance Taylor, Cygnus Support), whose
// notice reads:
//   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//   Developed at SunPro, a Sun Microsystems, Inc. business.
//   Permission to use, copy, modify, and distribute this software is freely
//   granted, provided that this notice is preserved.
// The sinf / cosf algorithm and its __sincosf_table coefficients are those of
// glibc's sysdeps/ieee754/flt-32 (Szabolcs Nagy, ARM Ltd; contributed to glibc
// from ARM's optimized-routines), here restated, not copied.
BB_HD uint32_t f2u(float x) { return __builtin_bit_cast(uint32_t, x); }
BB_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
BB_HD double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }

// __sincosf_table[0]: 2/pi 2^24, pi/2 and the polynomial coefficients.
// __sincosf_table[1] (quadrants 2-3) holds the cosine coefficients negated:
// every fused step of the cosine polynomial then yields the exact negation,
// so it is applied as one sign flip of the result (no per-lane table reads).
static constexpr double GLIBC_HPI_INV = 10680707.430881744, GLIBC_HPI = 1.5707963267948966;
static constexpr double GLIBC_C0 = 1.0, GLIBC_C1 = -0.49999999725108224, GLIBC_C2 = 0.041666623324344516,
                        GLIBC_C3 = -0.001388676379437604, GLIBC_C4 = 2.4390450703564542e-05;
static constexpr double GLIBC_S1 = -0.16666654943701084, GLIBC_S2 = 0.008332178146138854,
                        GLIBC_S3 = -0.00019517298981385725;
// __inv_pio4: 4/pi in 32-bit words, for the |x| >= 120 reduction
static constexpr uint32_t GLIBC_INV_PIO4[24] = {
    0xa2, 0xa2f9, 0xa2f983, 0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041,
};

// sinf_poly's two branches (sincosf.h)
BB_HD float glibc_sin_poly(double x, double x2)
{
    const double x3 = x2 * x;
    const double s1 = fma_d(x2, GLIBC_S3, GLIBC_S2);
    const double x5 = x2 * x3;
    const double s = fma_d(x3, GLIBC_S1, x);
    return (float)fma_d(s1, x5, s);
}
BB_HD float glibc_cos_poly(double x2)
{
    const double x4 = x2 * x2;
    const double c1 = fma_d(x2, GLIBC_C1, GLIBC_C0);
    const double c2 = fma_d(x2, GLIBC_C4, GLIBC_C3);
    const double x6 = x2 * x4;
    const double c = fma_d(x4, GLIBC_C2, c1);
    return (float)fma_d(c2, x6, c);
}
// x = n pi/2 + r for |x| < 120: n = round(x 2/pi) from the 2^24-scaled
// product, r by one fused multiply-add (reduce_fast).
BB_HD double glibc_reduce_fast(double x, int *np)
{
    const double r = x * GLIBC_HPI_INV;
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return fma_d(-(double)n, GLIBC_HPI, x);
}
// |x| >= 120: 4/pi in fixed point times the significand (reduce_large).
BB_HD double glibc_reduce_large(uint32_t xi, int *np)
{
    const uint32_t *arr = &GLIBC_INV_PIO4[(xi >> 26) & 15];
    const int shift = (xi >> 23) & 7;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    uint64_t res0 = (uint64_t)(uint32_t)(xi * arr[0]);
    const uint64_t res1 = (uint64_t)xi * arr[4];
    const uint64_t res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ull << 61)) >> 62;
    res0 -= n << 62;
    *np = (int)n;
    return (double)(int64_t)res0 * u2d(0x3c1921fb54442d18ull);  // pi / 2^63
}
// sinf (cos = false) or cosf (cos = true)
BB_HD float glibc_sincosf_one(float y, bool cos)
{
    const uint32_t top = (f2u(y) >> 20) & 0x7ff;
    double x = (double)y;
    if (top < 0x3f4) {  // |y| < pi/4
        const double x2 = x * x;
        if (top < 0x398) return cos ? 1.0f : y;  // |y| < 2^-12
        return cos ? glibc_cos_poly(x2) : glibc_sin_poly(x, x2);
    }
    int n, q;  // q selects the sign and the table: n, plus the sign of y on the large path
    if (top < 0x42f) {  // |y| < 120
        x = glibc_reduce_fast(x, &n);
        q = n;
    } else if (top < 0x7f8) {
        x = glibc_reduce_large(f2u(y), &n);
        q = n + (int)(f2u(y) >> 31);
    } else {
        return (y - y) / (y - y);  // inf / nan: invalid
    }
    const double x2 = x * x;
    if (((n & 1) != 0) != cos) {
        const float c = glibc_cos_poly(x2);
        return (q & 2) ? -c : c;
    }
    return glibc_sin_poly(((q + 1) & 2) ? -x : x, x2);  // sign[q & 3] = {1, -1, -1, 1}
}

// fdlibm s_atanf.c as glibc builds it
BB_HD float glibc_atanf(float x)
{
    const uint32_t hx = f2u(x), ix = hx & 0x7fffffff;
    const float aT[11] = {u2f(0x3eaaaaab), u2f(0xbe4ccccd), u2f(0x3e124925), u2f(0xbde38e38), u2f(0x3dba2e6e),
                          u2f(0xbd9d8795), u2f(0x3d886b35), u2f(0xbd6ef16b), u2f(0x3d4bda59), u2f(0xbd15a221),
                          u2f(0x3c8569d7)};
    // atanhi / atanlo[id] by selects (no per-lane table)
    const auto hi = [](int id) {
        return u2f(id == 0 ? 0x3eed6338u : id == 1 ? 0x3f490fdau : id == 2 ? 0x3f7b985eu : 0x3fc90fdau);
    };
    const auto lo = [](int id) {
        return u2f(id == 0 ? 0x31ac3769u : id == 1 ? 0x33222168u : id == 2 ? 0x33140fb4u : 0x33a22168u);
    };
    if (ix >= 0x4c000000) {  // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;
        return (int32_t)hx > 0 ? lo(3) + hi(3) : -hi(3) - lo(3);
    }
    int id;
    if (ix < 0x3ee00000) {  // |x| < 0.4375
        if (ix < 0x31000000) return x;  // |x| < 2^-29 (huge + x > one)
        id = -1;
    } else {
        x = __builtin_fabsf(x);
        if (ix < 0x3f980000) {      // |x| < 1.1875
            if (ix < 0x3f300000) {  // 7/16 <= |x| < 11/16
                id = 0; x = ((x + x) - 1.0f) / (x + 2.0f);
            } else {                // 11/16 <= |x| < 19/16
                id = 1; x = (x - 1.0f) / (x + 1.0f);
            }
        } else if (ix < 0x401c0000) {  // |x| < 2.4375
            id = 2; x = (x - 1.5f) / (x * 1.5f + 1.0f);
        } else {                       // 2.4375 <= |x| < 2^25
            id = 3; x = -1.0f / x;
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = hi(id) - ((x * (s1 + s2) - lo(id)) - x);
    return (int32_t)hx < 0 ? -r : r;
}

// fdlibm e_atan2f.c as glibc builds it (__ieee754_atan2f; the wrapper only
// sets errno)
BB_HD float glibc_atan2f(float y, float x)
{
    const float tiny = u2f(0x0da24260), pi_o_4 = u2f(0x3f490fdb), pi_o_2 = u2f(0x3fc90fdb),
                pi = u2f(0x40490fdb), pi_lo = u2f(0xb3bbbd2e);
    const uint32_t hx = f2u(x), ix = hx & 0x7fffffff, hy = f2u(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return glibc_atanf(y);
    const int m = (int)((hy >> 31) & 1) | (int)((hx >> 30) & 2);
    if (iy == 0) {
        switch (m) {
        case 0: case 1: return y;
        case 2: return pi + tiny;
        default: return -pi - tiny;
        }
    }
    if (ix == 0) return (int32_t)hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
            case 0: return pi_o_4 + tiny;
            case 1: return -pi_o_4 - tiny;
            case 2: return 3.0f * pi_o_4 + tiny;
            default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
        case 0: return 0.0f;
        case 1: return -0.0f;
        case 2: return pi + tiny;
        default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return (int32_t)hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = ((int32_t)iy - (int32_t)ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 - u2f(0x333bbd2e);           // pi_o_2 + 0.5 pi_lo, folded
    else if ((int32_t)hx < 0 && k < -60) z = 0.0f;
    else z = glibc_atanf(__builtin_fabsf(y / x));
    switch (m) {
    case 0: return z;
    case 1: return u2f(f2u(z) ^ 0x80000000u);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
    }
}

// fdlibm e_acosf.c as glibc builds it
BB_HD float glibc_acosf(float x)
{
    const float pi = u2f(0x40490fda), pio2_hi = u2f(0x3fc90fda), pio2_lo = u2f(0x33a22168);
    const float pS0 = u2f(0x3e2aaaab), pS1 = u2f(0xbea6b090), pS2 = u2f(0x3e4e0aa8), pS3 = u2f(0xbd241146),
                pS4 = u2f(0x3a4f7f04), pS5 = u2f(0x3811ef08);
    const float qS1 = u2f(0xc019d139), qS2 = u2f(0x4001572d), qS3 = u2f(0xbf303361), qS4 = u2f(0x3d9dc62e);
    const uint32_t hx = f2u(x), ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) return (int32_t)hx > 0 ? 0.0f : pi + u2f(0x34222168);  // pi + 2 pio2_lo
    if (ix > 0x3f800000) return (x - x) / (x - x);
    if (ix < 0x3f000000) {  // |x| < 0.5
        if (ix <= 0x32800000) return pio2_hi + pio2_lo;
        const float z = x * x;
        const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const float r = p / q;
        return pio2_hi - (x - (pio2_lo - x * r));
    }
    if ((int32_t)hx < 0) {  // x < -0.5
        const float z = (1.0f + x) * 0.5f;
        const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const float s = __builtin_sqrtf(z);
        const float r = p / q;
        const float w = r * s - pio2_lo;
        return pi - 2.0f * (s + w);
    }
    const float z = (1.0f - x) * 0.5f;  // x > 0.5
    const float s = __builtin_sqrtf(z);
    const float df = u2f(f2u(s) & 0xfffff000u);
    const float c = (z - df * df) / (s + df);
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float r = p / q;
    const float w = r * s + c;
    return 2.0f * (df + w);
}

BB_HD float sinf_(float x) { return glibc_sincosf_one(x, false); }
BB_HD float cosf_(float x) { return glibc_sincosf_one(x, true); }
BB_HD void sincosf_(float x, float *s, float *c)
{
    *s = glibc_sincosf_one(x, false);
    *c = glibc_sincosf_one(x, true);
}
BB_HD float atan2f_(float y, float x) { return glibc_atan2f(y, x); }
BB_HD float atanf_(float x) { return glibc_atanf(x); }
BB_HD float acosf_(float x) { return glibc_acosf(x); }
BB_HD float sqrtf_(float x) { return __builtin_sqrtf(x); }
}  // namespace bbm
