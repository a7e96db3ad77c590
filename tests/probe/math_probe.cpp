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
}
