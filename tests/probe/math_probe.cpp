// Host build of the product math (madrona_basketball_amd/csrc/bb_math.h) next
// to the host libm it restates, for tests/test_math.py.
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <thread>
#include <vector>
#include "../../madrona_basketball_amd/csrc/bb_math.h"

extern "C" {
#define VEC1(name, expr) \
    void name(const float *x, float *out, int64_t n) { for (int64_t i = 0; i < n; i++) { const float v = x[i]; out[i] = (expr); } }
VEC1(bb_sinf, bbm::sinf_(v))
VEC1(bb_cosf, bbm::cosf_(v))
VEC1(bb_atanf, bbm::atanf_(v))
VEC1(bb_acosf, bbm::acosf_(v))
VEC1(glibc_sinf, sinf(v))
VEC1(glibc_cosf, cosf(v))
VEC1(glibc_atanf, atanf(v))
VEC1(glibc_acosf, acosf(v))
VEC1(cr_sinf, (float)sin((double)v))
// the device probe's float-valued forms of the double functions (bb_diag_math 5-7)
VEC1(bb_erff, (float)bbm::erf_d((double)v))
VEC1(bb_acospred, ((float)bbm::acos_d((double)v) > 3.14159265358979323846f / 8.f) ? 1.f : 0.f)
VEC1(bb_expm1sum, (float)(-1.0 + bbm::exp_d((double)v)))
void bb_atan2f(const float *y, const float *x, float *out, int64_t n) { for (int64_t i = 0; i < n; i++) out[i] = bbm::atan2f_(y[i], x[i]); }
void glibc_atan2f(const float *y, const float *x, float *out, int64_t n) { for (int64_t i = 0; i < n; i++) out[i] = atan2f(y[i], x[i]); }
#define VECD(name, expr) \
    void name(const double *x, double *out, int64_t n) { for (int64_t i = 0; i < n; i++) { const double v = x[i]; out[i] = (expr); } }
VECD(bb_exp, bbm::exp_d(v))
VECD(bb_erf, bbm::erf_d(v))
VECD(bb_acos, bbm::acos_d(v))
VECD(bb_atan, bbm::atan_d(v))

static bool same_bits(float a, float b)
{
    uint32_t ua, ub;
    memcpy(&ua, &a, 4);
    memcpy(&ub, &b, 4);
    if (ua == ub) return true;
    return a != a && b != b;  // any NaN matches any NaN
}

// Mismatches of the restatement against the host libm over every 32-bit
// pattern (fn: 0 sinf, 1 cosf, 2 atanf, 3 acosf, 4 glibc sincosf vs sinf/cosf);
// first mismatching input in *first (or 0).
int64_t exhaustive_mismatches(int fn, int threads, uint32_t *first)
{
    std::vector<int64_t> bad(threads, 0);
    std::vector<uint32_t> f(threads, 0);
    std::vector<std::thread> pool;
    const uint64_t total = 1ull << 32, chunk = total / threads;
    for (int t = 0; t < threads; t++) {
        pool.emplace_back([&, t] {
            const uint64_t lo = chunk * t, hi = t + 1 == threads ? total : lo + chunk;
            for (uint64_t i = lo; i < hi; i++) {
                float x;
                const uint32_t u = (uint32_t)i;
                memcpy(&x, &u, 4);
                bool ok;
                switch (fn) {
                case 0: ok = same_bits(bbm::sinf_(x), sinf(x)); break;
                case 1: ok = same_bits(bbm::cosf_(x), cosf(x)); break;
                case 2: ok = same_bits(bbm::atanf_(x), atanf(x)); break;
                case 3: ok = same_bits(bbm::acosf_(x), acosf(x)); break;
                default: {
                    float s, c;
                    sincosf(x, &s, &c);
                    ok = same_bits(s, sinf(x)) && same_bits(c, cosf(x));
                }
                }
                if (!ok && bad[t]++ == 0) f[t] = u;
            }
        });
    }
    for (auto &th : pool) th.join();
    int64_t n = 0;
    *first = 0;
    for (int t = 0; t < threads; t++) {
        if (bad[t] && !n) *first = f[t];
        n += bad[t];
    }
    return n;
}

// The double functions of the step take a float argument and their result
// ends in a float (or a float comparison), so their agreement with glibc is
// decidable input by input.  Over the 32-bit patterns [lo, hi):
//   5  erf : (float)erf_d((double)x) == (float)erf((double)x)    (game.cpp:808)
//   6  exp : exp_d((double)x) == exp((double)x), as doubles       (game.cpp:868)
//   7  acos: ((float)acos_d((double)c) > pi/8) == ((float)acos((double)c) > pi/8)
//                                                                  (game.cpp:746-747)
//   8  exp : (float)((double)r + exp_d(x)) == (float)((double)r + exp(x)) for the
//            reward bases r the step can hold there (see tests/test_math.py)
static bool double_check(int fn, float x)
{
    switch (fn) {
    case 5: return same_bits((float)bbm::erf_d((double)x), (float)erf((double)x));
    case 6: {
        const double a = bbm::exp_d((double)x), b = exp((double)x);
        uint64_t ua, ub;
        memcpy(&ua, &a, 8);
        memcpy(&ub, &b, 8);
        return ua == ub || (a != a && b != b);
    }
    case 7: {
        const float pi8 = 3.14159265358979323846f / 8.f;
        return ((float)bbm::acos_d((double)x) > pi8) == ((float)acos((double)x) > pi8);
    }
    default: {
        const double a = bbm::exp_d((double)x), b = exp((double)x);
        if (a == b) return true;
        // reward before the exp term: -1 + (the tag / out-of-bounds / clock
        // terms of that step): 0, +-10, -100, +10 - 10, ...
        static const float base[] = {-1.f, -11.f, 9.f, -101.f, -111.f, -91.f, 19.f, -21.f};
        for (float r : base)
            if (!same_bits((float)((double)r + a), (float)((double)r + b))) return false;
        return true;
    }
    }
}

int64_t exhaustive_double_mismatches(int fn, int threads, uint32_t lo, uint32_t hi, uint32_t *first)
{
    std::vector<int64_t> bad(threads, 0);
    std::vector<uint32_t> f(threads, 0);
    std::vector<std::thread> pool;
    const uint64_t total = (uint64_t)hi - lo, chunk = total / threads;
    for (int t = 0; t < threads; t++) {
        pool.emplace_back([&, t] {
            const uint64_t a = lo + chunk * t, b = t + 1 == threads ? (uint64_t)hi : a + chunk;
            for (uint64_t i = a; i < b; i++) {
                float x;
                const uint32_t u = (uint32_t)i;
                memcpy(&x, &u, 4);
                if (!double_check(fn, x) && bad[t]++ == 0) f[t] = u;
            }
        });
    }
    for (auto &th : pool) th.join();
    int64_t n = 0;
    *first = 0;
    for (int t = 0; t < threads; t++) {
        if (bad[t] && !n) *first = f[t];
        n += bad[t];
    }
    return n;
}
}
