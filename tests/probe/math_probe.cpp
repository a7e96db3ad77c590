// Host build of the product math (madrona_basketball_amd/csrc/bb_math.h) next
// to the libm-based definition it targets, for tests/test_math.py.
#include <math.h>
#include <stdint.h>
#include "../../madrona_basketball_amd/csrc/bb_math.h"

extern "C" {
#define VEC1(name, expr) \
    void name(const float *x, float *out, int64_t n) { for (int64_t i = 0; i < n; i++) { const float v = x[i]; out[i] = (expr); } }
VEC1(bb_sinf, bbm::sinf_(v))
VEC1(bb_cosf, bbm::cosf_(v))
VEC1(bb_atanf, bbm::atanf_(v))
VEC1(bb_acosf, bbm::acosf_(v))
VEC1(ref_sinf, (float)sin((double)v))
VEC1(ref_cosf, (float)cos((double)v))
VEC1(ref_atanf, (float)atan((double)v))
VEC1(ref_acosf, (float)acos((double)v))
VEC1(glibc_sinf, sinf(v))
VEC1(glibc_atanf, atanf(v))
void bb_atan2f(const float *y, const float *x, float *out, int64_t n) { for (int64_t i = 0; i < n; i++) out[i] = bbm::atan2f_(y[i], x[i]); }
void ref_atan2f(const float *y, const float *x, float *out, int64_t n) { for (int64_t i = 0; i < n; i++) out[i] = (float)atan2((double)y[i], (double)x[i]); }
#define VECD(name, expr) \
    void name(const double *x, double *out, int64_t n) { for (int64_t i = 0; i < n; i++) { const double v = x[i]; out[i] = (expr); } }
VECD(bb_exp, bbm::exp_d(v))
VECD(bb_erf, bbm::erf_d(v))
VECD(bb_acos, bbm::acos_d(v))
VECD(bb_sin, bbm::sin_d(v))
VECD(bb_atan, bbm::atan_d(v))
}
