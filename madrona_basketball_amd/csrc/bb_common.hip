// bb_common.hip -- small kernels shared by every agent count: the synthetic
// action workload, device-side pokes (set_action / trigger_reset), a
// streaming probe for roofline calibration, and the N dispatch.
#include <hip/hip_runtime.h>
#include "bb_launch.h"
#include "bb_rng.h"

namespace bb {

int diag_override[DIAG_KEYS] = {-1, -1, -1, -1, -1, -1, -1, -1, -1};

// one lane = one (world, agent) action row (24 B); N compile-time so the
// row -> (world, agent) split is a multiply, not a 64-bit division
template <int N>
__global__ __launch_bounds__(256) void k_random_actions(int32_t *action, int32_t rows, int64_t world_offset,
                                                        uint32_t seed, uint32_t step)
{
    const int32_t r = (int32_t)blockIdx.x * 256 + (int32_t)threadIdx.x;
    if (r >= rows) return;
    const int32_t w = r / N;
    const int32_t a = r - w * N;
    int32_t act[6];
    random_action(seed, step, (uint32_t)(world_offset + w), (uint32_t)a, act);
    int2 *dst = (int2 *)(action + (int64_t)r * 6);
    dst[0] = make_int2(act[0], act[1]);
    dst[1] = make_int2(act[2], act[3]);
    dst[2] = make_int2(act[4], act[5]);
}

struct Poke { int32_t v[16]; };
__global__ void k_poke(int32_t *dst, int32_t count, Poke vals)
{
    const int k = threadIdx.x;
    if (k < count) dst[k] = vals.v[k];
}

// Trajectory recorder: one lane per record word; consecutive lanes write
// consecutive words of the ring slot (the source reads are the scattered side,
// a few hundred bytes per world).
int32_t record_words(int n) { return 18 * n + 27; }

RecordArgs record_args(const Params &p, int n)
{
    const Columns &c = p.c;
    RecordArgs a;
    const void *src[RECORD_SEGS] = {c.agent_pos, c.ball_pos, c.ball_vel, c.orientation, c.ball_physics,
                                    c.possession, c.game_state, c.reward, c.action, c.done};
    const int32_t wpw[RECORD_SEGS] = {3 * n, 3, 3, 4 * n, 7, 3 * n, 14, n, 6 * n, n};
    a.off[0] = 0;
    for (int k = 0; k < RECORD_SEGS; k++) {
        a.src[k] = (const uint32_t *)src[k];
        a.wpw[k] = wpw[k];
        a.off[k + 1] = a.off[k] + wpw[k];
    }
    return a;
}

__host__ __device__ inline uint32_t record_word(const RecordArgs &a, int64_t world, int32_t q)
{
    int k = 0;
#pragma unroll
    for (int j = 1; j < RECORD_SEGS; j++) k += q >= a.off[j] ? 1 : 0;
    // (select chain: a per-lane index into the kernel-argument arrays stays in scalars)
    const uint32_t *src = a.src[0];
    int32_t wpw = a.wpw[0], off = a.off[0];
#pragma unroll
    for (int j = 1; j < RECORD_SEGS; j++) {
        if (k == j) { src = a.src[j]; wpw = a.wpw[j]; off = a.off[j]; }
    }
    return src[world * wpw + (q - off)];
}

__global__ __launch_bounds__(256) void k_record(const RecordArgs a, int64_t world0, int64_t total, uint32_t *dst)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const int32_t words = a.off[RECORD_SEGS];
    const int64_t wl = i / words;
    dst[i] = record_word(a, world0 + wl, (int32_t)(i - wl * words));
}

void host_record(const RecordArgs &a, int64_t world0, int32_t count, uint32_t *dst)
{
    const int32_t words = a.off[RECORD_SEGS];
    for (int64_t wl = 0; wl < count; wl++)
        for (int32_t q = 0; q < words; q++) dst[wl * words + q] = record_word(a, world0 + wl, q);
}

// Coalesced streaming probe: item i reads read_q float4 and writes write_q
// float4.  pattern 0 lays them out [q][item] (the waves resident at once
// sweep one contiguous window); pattern 1 gives each wave a region of its own
// that it reads/writes front to back (as k_step's rows: 64 pieces of one
// region per instruction).  Every wave instruction is 1 KiB contiguous; nt:
// non-temporal stores.
__global__ __launch_bounds__(256) void k_stream_probe(const float4 *src, float4 *dst, int64_t items, int read_q,
                                                     int write_q, int pattern, int nt)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= items) return;
    const int64_t wave = i >> 6, lane = i & 63;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = 0; q < read_q; q++) {
        const int64_t at = pattern ? (wave * read_q + q) * 64 + lane : (int64_t)q * items + i;
        const float4 v = src[at];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    for (int q = 0; q < write_q; q++) {
        const int64_t at = pattern ? (wave * write_q + q) * 64 + lane : (int64_t)q * items + i;
        typedef float v4 __attribute__((ext_vector_type(4)));
        const v4 a = {acc.x, acc.y, acc.z, acc.w};
        if (nt) __builtin_nontemporal_store(a, (v4 *)&dst[at]);
        else *(v4 *)&dst[at] = a;
    }
}

// Diagnostics (tests/test_gpu_math.py): the step's scalar math evaluated on
// gfx950 over caller inputs, to compare bit for bit with the host build of
// the same header.  fn: 0 sinf, 1 cosf, 2 atanf, 3 acosf, 4 atan2f(x, y),
// 5 (float)erf_d, 6 acos_d(c) > pi/8 as 0/1, 7 (float)(-1 + exp_d(x)).
__global__ __launch_bounds__(256) void k_math_probe(int fn, const float *x, const float *y, float *out, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float v = x[i];
    float r;
    switch (fn) {
    case 0: r = bbm::sinf_(v); break;
    case 1: r = bbm::cosf_(v); break;
    case 2: r = bbm::atanf_(v); break;
    case 3: r = bbm::acosf_(v); break;
    case 4: r = bbm::atan2f_(v, y[i]); break;
    case 5: r = (float)bbm::erf_d((double)v); break;
    case 6: r = ((float)bbm::acos_d((double)v) > PI_OVER_8) ? 1.f : 0.f; break;
    default: r = (float)(-1.0 + bbm::exp_d((double)v)); break;
    }
    out[i] = r;
}

// Diagnostics (tests/test_gpu_math.py): shorter
// sequences for the step's correctly rounded f32 quotients and square roots,
// against the IEEE operations hipcc compiles.  The compiler's expansions serve
// every input (operand scaling for extreme exponents, special values: 10-11
// instructions per quotient, ~14 per root); these are its own sequences
// without the scaling, valid well inside the exponent range:
//   rcp_refined(b):  v_rcp_f32 then one Newton step by fma;
//   div_short<C>:    q = a y, then C residual corrections q + (a - b q) y
//                    (C = 1 Markstein's, C = 2 the expansion's);
//   sqrt_short(x):   v_sqrt_f32 then the expansion's neighbour selection.
// Measured (round 4, profiles/r04/a_divsqrt_*): exact on every input tried
// (rcp on all 2^32 floats of its range, div on 2^32 random pairs), but with
// the wave-uniform range guards the step got slower (65 536 x 2 21.0 ->
// 21.5 us), and even unguarded non-IEEE fast division / roots save only
// 0.35 us: the product keeps the IEEE operators.
// mode 0 sqrt_short, 1 rcp_refined, 2 rcp_short<1>, 3 div_short<1>,
// 4 div_short<2>, 5 the bare v_sqrt_f32.  Modes 0-2 and 5 take the float bit
// patterns start + i, i < count, skipping those outside the short path's
// range; modes 3-4 take pseudo-random operand pairs (index i, seed) with
// exponents in [2^-47, 2^48).  Per workgroup: the mismatch count and one
// mismatching input (a bits, b bits).
__device__ __forceinline__ bool exp_in(float x, uint32_t lo, uint32_t hi)
{
    return ((bbm::f2u(x) >> 23) & 0xffu) - lo <= hi - lo;
}
__device__ __forceinline__ float rcp_refined(float b)
{
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y0, 1.0f);
    return __builtin_fmaf(e, y0, y0);
}
template <int C>
__device__ __forceinline__ float div_short(float a, float b)
{
    const float y = rcp_refined(b);
    float q = a * y;
#pragma unroll
    for (int k = 0; k < C; k++) q = __builtin_fmaf(__builtin_fmaf(-b, q, a), y, q);
    return q;
}
template <int C>
__device__ __forceinline__ float rcp_short(float b)
{
    const float y = rcp_refined(b);
    float q = y;
#pragma unroll
    for (int k = 0; k < C; k++) q = __builtin_fmaf(__builtin_fmaf(-b, q, 1.0f), y, q);
    return q;
}
__device__ __forceinline__ float sqrt_short(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float lo = bbm::u2f(bbm::f2u(s) - 1u), hi = bbm::u2f(bbm::f2u(s) + 1u);
    const float rlo = __builtin_fmaf(-lo, s, x), rhi = __builtin_fmaf(-hi, s, x);
    float r = rlo <= 0.0f ? lo : s;
    r = rhi > 0.0f ? hi : r;
    return r;
}
__device__ __forceinline__ uint32_t probe_hash(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ float probe_operand(uint32_t h, uint32_t e_lo, uint32_t e_hi)
{
    const uint32_t e = e_lo + (uint32_t)(((uint64_t)(h >> 8) * (e_hi - e_lo + 1)) >> 24);
    return __builtin_bit_cast(float, (h & 0x80000000u) | (e << 23) | (probe_hash(h) & 0x7fffffu));
}
__global__ __launch_bounds__(256) void k_divsqrt_probe(int mode, uint64_t start, uint64_t count, uint32_t seed,
                                                       uint32_t *counts, uint32_t *ex)
{
    const uint64_t nth = (uint64_t)gridDim.x * 256;
    uint32_t bad = 0, ea = 0, eb = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += nth) {
        float a = 0.f, b = 0.f, got = 0.f, want = 0.f;
        bool in = true;
        if (mode == 3 || mode == 4) {
            const uint32_t h = probe_hash((uint32_t)i ^ probe_hash(seed + (uint32_t)(i >> 32)));
            a = probe_operand(h, 80u, 174u);
            b = probe_operand(probe_hash(h ^ 0x9e3779b9u), 80u, 174u);
            got = mode == 3 ? div_short<1>(a, b) : div_short<2>(a, b);
            want = a / b;
        } else {
            b = __builtin_bit_cast(float, (uint32_t)(start + i));
            if (mode == 0 || mode == 5) {
                in = !(bbm::f2u(b) >> 31) && exp_in(b, mode == 0 ? 32u : 1u, 254u);
                got = mode == 0 ? sqrt_short(b) : __builtin_amdgcn_sqrtf(b);
                want = __builtin_sqrtf(b);
            } else {
                in = exp_in(b, 2u, 252u);
                got = mode == 1 ? rcp_refined(b) : rcp_short<1>(b);
                want = 1.0f / b;
            }
        }
        if (in && bbm::f2u(got) != bbm::f2u(want)) {
            bad++;
            ea = bbm::f2u(a);
            eb = bbm::f2u(b);
        }
    }
    __shared__ uint32_t sbad[256], sa[256], sb[256];
    sbad[threadIdx.x] = bad; sa[threadIdx.x] = ea; sb[threadIdx.x] = eb;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0, xa = 0, xb = 0;
        for (int k = 0; k < 256; k++) {
            t += sbad[k];
            if (sbad[k]) { xa = sa[k]; xb = sb[k]; }
        }
        counts[blockIdx.x] = t;
        ex[2 * blockIdx.x] = xa;
        ex[2 * blockIdx.x + 1] = xb;
    }
}

hipError_t launch_divsqrt_probe(int mode, uint64_t start, uint64_t count, uint32_t seed, uint32_t *counts,
                                uint32_t *ex, int blocks, hipStream_t s)
{
    if (mode < 0 || mode > 5 || blocks <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_divsqrt_probe, dim3((unsigned)blocks), dim3(256), 0, s, mode, start, count, seed, counts, ex);
    return hipGetLastError();
}

static inline dim3 grid_for(int64_t items, int block) { return dim3((unsigned)((items + block - 1) / block)); }

template <int N>
hipError_t launch_random_actions_t(const Params &p, uint32_t seed, uint32_t step, hipStream_t s)
{
    const int64_t rows = p.num_worlds * N;
    if (rows > INT32_MAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_random_actions<N>, grid_for(rows, 256), dim3(256), 0, s, p.c.action, (int32_t)rows,
                       p.world_offset, seed, step);
    return hipGetLastError();
}

hipError_t launch_poke(int32_t *dst, int count, const int32_t *vals, hipStream_t s)
{
    if (count < 0 || count > 16) return hipErrorInvalidValue;
    Poke pk;
    for (int k = 0; k < 16; k++) pk.v[k] = k < count ? vals[k] : 0;
    hipLaunchKernelGGL(k_poke, dim3(1), dim3(64), 0, s, dst, count, pk);
    return hipGetLastError();
}

hipError_t launch_record(const RecordArgs &a, int64_t world0, int32_t count, uint32_t *dst, hipStream_t s)
{
    const int64_t total = (int64_t)count * a.off[RECORD_SEGS];
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_record, grid_for(total, 256), dim3(256), 0, s, a, world0, total, dst);
    return hipGetLastError();
}

hipError_t launch_math_probe(int fn, const float *x, const float *y, float *out, int64_t n, hipStream_t s)
{
    if (fn < 0 || fn > 7 || n < 0) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_math_probe, grid_for(n, 256), dim3(256), 0, s, fn, x, y, out, n);
    return hipGetLastError();
}

hipError_t launch_stream_probe(const float4 *src, float4 *dst, int64_t items, int read_q, int write_q, int pattern,
                               int nt, hipStream_t s)
{
    hipLaunchKernelGGL(k_stream_probe, grid_for(items, 256), dim3(256), 0, s, src, dst, items, read_q, write_q, pattern,
                       nt);
    return hipGetLastError();
}

#define BB_DISPATCH_N(n, call)                  \
    switch (n) {                                \
    case 2: return call(2);                     \
    case 4: return call(4);                     \
    case 6: return call(6);                     \
    case 8: return call(8);                     \
    case 10: return call(10);                   \
    default: return hipErrorInvalidValue;       \
    }

hipError_t launch_random_actions(int n, const Params &p, uint32_t seed, uint32_t step, hipStream_t s)
{
#define CALL(k) launch_random_actions_t<k>(p, seed, step, s)
    BB_DISPATCH_N(n, CALL)
#undef CALL
}

hipError_t launch_step(int n, const Params &p, hipStream_t s, int mode, hipEvent_t ev0, hipEvent_t ev1)
{
#define CALL(k) launch_step_t<k>(p, mode, s, ev0, ev1)
    BB_DISPATCH_N(n, CALL)
#undef CALL
}

bool resident_staged_n(int n, int64_t num_worlds)
{
    switch (n) {
    case 2: return resident_staged<2>(num_worlds);
    case 4: return resident_staged<4>(num_worlds);
    case 6: return resident_staged<6>(num_worlds);
    case 8: return resident_staged<8>(num_worlds);
    case 10: return resident_staged<10>(num_worlds);
    default: return false;
    }
}

int step_grid_n(int n, int64_t num_worlds)
{
#define CALL(k) step_grid<k>(num_worlds)
    BB_DISPATCH_N(n, CALL)
#undef CALL
}

hipError_t launch_rollout(int n, const Params &p, const RolloutArgs &r, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1)
{
#define CALL(k) launch_rollout_t<k>(p, r, s, ev0, ev1)
    BB_DISPATCH_N(n, CALL)
#undef CALL
}

hipError_t launch_rollout_policy(int n, const Params &p, const PolicyRolloutArgs &r, hipStream_t s)
{
#define CALL(k) launch_rollout_policy_t<k>(p, r, s)
    BB_DISPATCH_N(n, CALL)
#undef CALL
}

hipError_t launch_step_ppo_2(const Params &p, const PpoStepArgs &a, hipStream_t s);  // bb_kernels.hip (N = 2)
hipError_t launch_rollout_ppo_2(const Params &p, const PpoStepArgs &a, int32_t steps, hipStream_t s);
hipError_t launch_rollout_ppo(int n, const Params &p, const PpoStepArgs &a, int32_t steps, hipStream_t s)
{
    return n == 2 ? launch_rollout_ppo_2(p, a, steps, s) : hipErrorNotSupported;
}
hipError_t launch_step_ppo(int n, const Params &p, const PpoStepArgs &a, hipStream_t s)
{
    return n == 2 ? launch_step_ppo_2(p, a, s) : hipErrorNotSupported;
}

bool step_records(int n)
{
    switch (n) {
    case 2: return step_records_t<2>();
    case 4: return step_records_t<4>();
    case 6: return step_records_t<6>();
    case 8: return step_records_t<8>();
    case 10: return step_records_t<10>();
    default: return false;
    }
}

// The K-step rollout kernel at N >= 4 agents (k_rollout_shared: the world in
// LDS across the steps) is taken up to this many agents.  At N = 4 it keeps
// 1/4 of the world's words per lane in registers across the row pass and
// beats per-step launches (65 536 worlds: 45.3 vs 62.7 us per step); from
// N = 6 the row-source table sits beside the world instead (the register copy
// spills), which costs occupancy: N = 10 396 vs 290 us per step
// (profiles/r05/g_*, h_*).  DIAG_ROLLOUT_SHARED_MAX_N overrides it (tests).
bool fused_rollout_n(int n)
{
    if (n >= 4 && n > diag_or(DIAG_ROLLOUT_SHARED_MAX_N, 4)) return false;
    switch (n) {
    case 2: return fused_rollout<2>();
    case 4: return fused_rollout<4>();
    case 6: return fused_rollout<6>();
    case 8: return fused_rollout<8>();
    case 10: return fused_rollout<10>();
    default: return false;
    }
}

int rollout_kernel_n(int n, int64_t num_worlds)
{
    switch (n) {
    case 2: return rollout_kernel_t<2>(num_worlds);
    case 4: return rollout_kernel_t<4>(num_worlds);
    case 6: return rollout_kernel_t<6>(num_worlds);
    case 8: return rollout_kernel_t<8>(num_worlds);
    case 10: return rollout_kernel_t<10>(num_worlds);
    default: return RK_NONE;
    }
}

hipError_t launch_init(int n, const Params &p, hipStream_t s)
{
#define CALL(k) launch_init_t<k>(p, s)
    BB_DISPATCH_N(n, CALL)
#undef CALL
}

hipError_t launch_step_loop(int n, const Params &p, int32_t *actions, int32_t steps, hipStream_t s, hipEvent_t ev0,
                            hipEvent_t ev1)
{
#define CALL(k) launch_step_loop_t<k>(p, actions, steps, s, ev0, ev1)
    BB_DISPATCH_N(n, CALL)
#undef CALL
}

}  // namespace bb
