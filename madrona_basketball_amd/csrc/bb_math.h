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

// log (the policy's logsumexp and Gumbel noise, bb_policy.h): x = m 2^e with
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
        // erf x = 2/sqrt(pi) * x * sum_n (-1)^n z^n / (n! (2n+1)), z = x^2
        const double z = ax * ax;
        double p = ERF_COEF.c[ERF_NT - 1];
#pragma unroll
        for (int n = ERF_NT - 2; n >= 0; n--) p = fma_d(p, z, ERF_COEF.c[n]);
        r = TWO_OVER_SQRTPI * (ax * p);
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
