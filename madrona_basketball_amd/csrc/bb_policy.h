// bb_policy.h -- the reference's policy network (scripts/agent.py:108-154 with
// num_channels = 32, num_layers = 2, env.py:107 / infer.py:182,203) for one
// observation row, shared by the host executor and the gfx950 kernel
// (bb_policy.hip) so that both give the same bits.
//
//   x  = clamp((obs - mean) * rsqrt(var + 1e-5), -5, 5)        RunningMeanStd, agent.py:28-38
//   h1 = relu(LN(W1 x + b1)),  h2 = relu(LN(W2 h1 + b2))       backbone, agent.py:115-124
//   logits = Wa h2 + ba (19),  value = Wc h2 + bc              heads, agent.py:127-128
//   per bucket [2,8,3,2,2,2] (env.py:102): action = argmax (best(), action.py:21-23) or a
//   categorical sample (inverse CDF of softmax); log_prob = logit - logsumexp (Categorical,
//   action.py:16-33), summed.
//
// Arithmetic order (fixed, -ffp-contract=off): each matrix product is the k-ordered
// fmaf chain the gfx950 f32 MFMA computes (v_mfma_f32_16x16x4_f32: one rounding per
// product), over the k permutation the kernel's operand layout gives -- k = 32q + j for
// the 128-wide layer (j outer, q inner), k = 8q + j for the 32-wide ones; LayerNorm
// sums are the kernel's butterfly tree (DPP), exp / log fixed f32 sequences (below).
#pragma once
#include "bb_math.h"
#include "bb_rng.h"

namespace bb {

constexpr int POL_IN = 128;     // observation width read (obs row: agent.py input_dim)
constexpr int POL_HID = 32;     // num_channels
constexpr int POL_LOGITS = 19;  // sum of the buckets
constexpr int POL_HEAD = 32;    // head rows: 19 actor + 1 critic + 12 zero
constexpr int POL_BUCKETS = 6;
BB_HD constexpr int pol_bucket(int b) { return b == 1 ? 8 : (b == 2 ? 3 : 2); }  // [2, 8, 3, 2, 2, 2]

// Device (or host) pointers, fp32, row-major [out][in].
struct PolicyWeights {
    const float *obs_mean, *obs_inv;           // [128]: mean, rsqrt(var + eps) as torch computes it
    const float *w1, *b1, *ln1_w, *ln1_b;      // [32][128], [32] x3
    const float *w2, *b2, *ln2_w, *ln2_b;      // [32][32], [32] x3
    const float *head_w, *head_b;              // [32][32], [32]
};

struct PolicyArgs {
    PolicyWeights w;
    const float *obs;      // row r at obs + r * obs_stride
    int64_t obs_stride;    // floats
    int64_t rows;
    int32_t *actions;      // row r at actions + r * act_stride (6 int32)
    int64_t act_stride;    // int32 words
    float *log_prob;       // [rows] (optional)
    float *value;          // [rows] (optional)
    int32_t stochastic;    // 0: argmax (best), 1: categorical sample (inverse CDF)
    uint32_t seed, step;   // sample key: threefry({seed, step}, {row, logit})
    // actions == nullptr: no actions written (value only, agent.evaluate).
    // Rollout recording (bb_rollout_policy, scripts/ppo.py:129-134; all optional):
    float *obs_out;                   // row r's 128 observation floats -> obs_out + r * 128
    int32_t *act_out;                 // row r's 6 actions -> act_out + r * 6
    const float *rew_src, *done_src;  // the previous step's reward / done of row r at src + r * rd_stride
    int64_t rd_stride;
    float *rew_out, *done_out;        // -> rew_out[r], done_out[r]
    uint64_t *diag_ts;                // diagnostics only: POL_TRACE_POINTS clocks of each wave's first tile
    uint32_t key_row0;                // sampling key of row r: key_row0 + r (a part of a larger call keeps its rows' keys)
    int32_t mt;                       // k_policy<mt> forced (1, 2, 4; bb_rollout_policy's split halves), 0: by row count
};

constexpr int POL_TRACE_POINTS = 8;

// exp / log in f32 from a fixed sequence of f32 operations (identical bits on
// host and gfx950; ~1 ulp): the policy is compared with torch's fp32 forward
// within a tolerance, so the step's correctly-rounded double route (bb_math)
// is not needed here, and these are 4-8x cheaper.  The polynomials run as
// explicit fused multiply-adds (correctly rounded on both sides: v_fma_f32 /
// the host's fmaf), half the instructions of the separately rounded mul + add
// chains (the translation units build with -ffp-contract=off) -- the bucket
// pass evaluates 19 of these per row (round 5).
//
// Branch-free: the special cases (NaN, overflow, underflow; log of 0, inf or
// a negative) are selected at the end, the polynomial path runs on an input
// clamped into its range -- equal to the input wherever that path's result is
// the one returned, so every value is the same as with early returns.  (With
// early returns each call was three nested exec-mask branches on the device,
// and the bucket pass's 8 exps of a bucket ran one after another.)
BB_HD float pol_expf(float x)
{
    const float xc = __builtin_fminf(__builtin_fmaxf(x, -104.0f), 89.0f);  // (NaN -> -104)
    const float k = __builtin_rintf(xc * 1.44269504f);
    float r = __builtin_fmaf(-k, 0.693145752f, xc);   // ln2 high part
    r = __builtin_fmaf(-k, 1.42860677e-06f, r);        // ln2 low part
    float p = 1.0f / 5040.0f;                          // Taylor to r^7 on |r| <= 0.347
    p = __builtin_fmaf(p, r, 1.0f / 720.0f);
    p = __builtin_fmaf(p, r, 1.0f / 120.0f);
    p = __builtin_fmaf(p, r, 1.0f / 24.0f);
    p = __builtin_fmaf(p, r, 1.0f / 6.0f);
    p = __builtin_fmaf(p, r, 0.5f);
    p = __builtin_fmaf(p, r, 1.0f);
    p = __builtin_fmaf(p, r, 1.0f);
    float y = __builtin_ldexpf(p, (int)k);
    y = x < -103.9f ? 0.f : y;
    y = x > 88.7f ? __builtin_inff() : y;
    return x != x ? x : y;
}
BB_HD float pol_logf(float x)
{
    // the polynomial path on a finite positive stand-in where x is special
    const bool special = !(x > 0.f) || x == __builtin_inff();  // NaN, <= 0, inf
    const float xs = special ? 1.0f : x;
    int e = 0;
    float m = __builtin_frexpf(xs, &e);      // [0.5, 1)
    const bool lo = m < 0.707106781f;
    m = lo ? m * 2.0f : m;
    e = lo ? e - 1 : e;
    const float s = (m - 1.0f) / (m + 1.0f);  // |s| <= 0.1716
    const float z = s * s;
    float p = 1.0f / 11.0f;
    p = __builtin_fmaf(p, z, 1.0f / 9.0f);
    p = __builtin_fmaf(p, z, 1.0f / 7.0f);
    p = __builtin_fmaf(p, z, 1.0f / 5.0f);
    p = __builtin_fmaf(p, z, 1.0f / 3.0f);
    const float lm = 2.0f * __builtin_fmaf(s * z, p, s);
    const float k = (float)e;
    const float y = __builtin_fmaf(k, 0.693145752f, __builtin_fmaf(k, 1.42860677e-06f, lm));
    if (!special) return y;
    return x == 0.f ? -__builtin_inff() : (x == __builtin_inff() ? x : __builtin_nanf(""));
}
BB_HD float pol_clamp(float x) { return __builtin_fminf(__builtin_fmaxf(x, -5.f), 5.f); }  // v_max / v_min
BB_HD float pol_relu(float x) { return x > 0.f ? x : 0.f; }

// Sampling (Categorical.sample, action.py:29-33) by inverse CDF: bucket b of
// row r draws one uniform u in [0, 1) -- word b & 1 of threefry({seed, step},
// {r, b >> 1}) -- and takes the first action whose running sum of
// exp(logit - max) (the terms and order of the bucket's logsumexp) exceeds
// u * sum, the last one if rounding leaves none: 6 uniforms and no logarithm
// per row (a Gumbel-max draw needs 19 uniforms and 38 logarithms).
BB_HD float pol_u01(uint32_t bits) { return (float)(bits >> 8) * (1.0f / 16777216.0f); }
BB_HD float pol_bucket_u(uint32_t seed, uint32_t step, uint32_t row, int b)
{
    uint32_t b0, b1;
    threefry2x32(seed, step, row, (uint32_t)(b >> 1), &b0, &b1);
    return pol_u01((b & 1) ? b1 : b0);
}
// The action of one bucket from its exp terms e[0..nb) (sum s) and uniform u.
template <int NB>
BB_HD int pol_inverse_cdf(const float (&e)[NB], int nb, float s, float u)
{
    const float t = u * s;
    float c = 0.f;
    int a = nb - 1;
#pragma unroll
    for (int i = 0; i < NB; i++) {  // (selects, no branches)
        const bool in = i < nb - 1;
        const float ci = c + e[i];
        a = (in && a == nb - 1 && ci > t) ? i : a;
        c = in ? ci : c;
    }
    return a;
}

// Bucket sampling / scoring of one row's logits (fully unrolled: the bucket
// sizes and offsets are compile-time, so logit[] stays in registers).
// Logit offset of bucket b ([2, 8, 3, 2, 2, 2]).
BB_HD constexpr int pol_bucket_off(int b) { return b == 0 ? 0 : (b == 1 ? 2 : (b == 2 ? 10 : 13 + 2 * (b - 3))); }

// Bucket B of one row: its action (argmax or inverse-CDF sample) and the
// log-prob term logit[a] - logsumexp(bucket).
// u: the bucket's uniform (pol_bucket_u), read only when stochastic.
template <int B>
BB_HD void pol_bucket_term(const float *logit, bool stochastic, float u, int32_t *act, float *term)
{
    constexpr int o = pol_bucket_off(B), nb = pol_bucket(B);
    float mx = logit[o];
#pragma unroll
    for (int i = 1; i < nb; i++) mx = logit[o + i] > mx ? logit[o + i] : mx;
    float e[nb], s = 0.f;
#pragma unroll
    for (int i = 0; i < nb; i++) {
        e[i] = pol_expf(logit[o + i] - mx);
        s = s + e[i];
    }
    int a = 0;
    if (stochastic) {
        a = pol_inverse_cdf(e, nb, s, u);
    } else {
        float best = logit[o];
#pragma unroll
        for (int i = 1; i < nb; i++)
            if (logit[o + i] > best) { best = logit[o + i]; a = i; }  // first maximum (torch argmax)
    }
    const float lse = mx + pol_logf(s);
    float la = logit[o];
#pragma unroll
    for (int i = 1; i < nb; i++) la = a == i ? logit[o + i] : la;
    *act = a;
    *term = la - lse;
}

// Summed log-prob of the six bucket terms, in bucket order.
BB_HD float pol_logp_sum(const float (&term)[POL_BUCKETS])
{
    float total = 0.f;
#pragma unroll
    for (int b = 0; b < POL_BUCKETS; b++) total = total + term[b];
    return total;
}

// Bucket sampling / scoring of one row's logits (fully unrolled: the bucket
// sizes and offsets are compile-time, so logit[] stays in registers).
BB_HD void pol_select(const float *logit, bool stochastic, uint32_t seed, uint32_t step, uint32_t row,
                      int32_t act[6], float *logp_sum)
{
    // the six uniforms (pol_bucket_u's values): one threefry call per bucket pair
    float u[POL_BUCKETS] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (stochastic) {
#pragma unroll
        for (int p = 0; p < POL_BUCKETS / 2; p++) {
            uint32_t b0, b1;
            threefry2x32(seed, step, row, (uint32_t)p, &b0, &b1);
            u[2 * p] = pol_u01(b0);
            u[2 * p + 1] = pol_u01(b1);
        }
    }
    float term[POL_BUCKETS];
    pol_bucket_term<0>(logit, stochastic, u[0], &act[0], &term[0]);
    pol_bucket_term<1>(logit, stochastic, u[1], &act[1], &term[1]);
    pol_bucket_term<2>(logit, stochastic, u[2], &act[2], &term[2]);
    pol_bucket_term<3>(logit, stochastic, u[3], &act[3], &term[3]);
    pol_bucket_term<4>(logit, stochastic, u[4], &act[4], &term[4]);
    pol_bucket_term<5>(logit, stochastic, u[5], &act[5], &term[5]);
    *logp_sum = pol_logp_sum(term);
}

// Sum of 32 values in the kernel's order: t_c = v_c + v_{c+16}, then the xor
// butterfly over c in [0, 16) (every lane ends with the same bits).
BB_HD float pol_sum32(const float *v)
{
    float t[16];
    for (int c = 0; c < 16; c++) t[c] = v[c] + v[c + 16];
    for (int m = 1; m < 16; m <<= 1) {
        float u[16];
        for (int c = 0; c < 16; c++) u[c] = t[c] + t[c ^ m];
        for (int c = 0; c < 16; c++) t[c] = u[c];
    }
    return t[0];
}

// relu(LayerNorm(h)) in place (torch: biased variance, eps 1e-5).
BB_HD void pol_layernorm_relu(float *h, const float *w, const float *b)
{
    const float mean = pol_sum32(h) * (1.0f / 32.0f);
    float d[32];
    for (int c = 0; c < 32; c++) d[c] = h[c] - mean;
    float sq[32];
    for (int c = 0; c < 32; c++) sq[c] = d[c] * d[c];
    const float var = pol_sum32(sq) * (1.0f / 32.0f);
    const float inv = 1.0f / bbm::sqrtf_(var + 1e-5f);
    for (int c = 0; c < 32; c++) h[c] = pol_relu(((d[c] * inv) * w[c]) + b[c]);
}

// One row on the host, in the kernel's arithmetic order.
inline void policy_row_host(const PolicyArgs &a, int64_t r)
{
    const PolicyWeights &W = a.w;
    const float *o = a.obs + r * a.obs_stride;
    float x[POL_IN];
    for (int k = 0; k < POL_IN; k++) x[k] = pol_clamp((o[k] - W.obs_mean[k]) * W.obs_inv[k]);
    float h1[POL_HID], h2[POL_HID], out[POL_HEAD];
    for (int n = 0; n < POL_HID; n++) {
        float acc = 0.f;
        for (int j = 0; j < 32; j++)
            for (int q = 0; q < 4; q++) acc = __builtin_fmaf(x[32 * q + j], W.w1[n * POL_IN + 32 * q + j], acc);
        h1[n] = acc + W.b1[n];
    }
    pol_layernorm_relu(h1, W.ln1_w, W.ln1_b);
    for (int n = 0; n < POL_HID; n++) {
        float acc = 0.f;
        for (int j = 0; j < 8; j++)
            for (int q = 0; q < 4; q++) acc = __builtin_fmaf(h1[8 * q + j], W.w2[n * POL_HID + 8 * q + j], acc);
        h2[n] = acc + W.b2[n];
    }
    pol_layernorm_relu(h2, W.ln2_w, W.ln2_b);
    for (int n = 0; n < POL_HEAD; n++) {
        float acc = 0.f;
        for (int j = 0; j < 8; j++)
            for (int q = 0; q < 4; q++) acc = __builtin_fmaf(h2[8 * q + j], W.head_w[n * POL_HID + 8 * q + j], acc);
        out[n] = acc + W.head_b[n];
    }
    int32_t act[6];
    float lp;
    pol_select(out, a.stochastic != 0, a.seed, a.step, (uint32_t)r + a.key_row0, act, &lp);
    if (a.obs_out)
        for (int k = 0; k < POL_IN; k++) a.obs_out[r * POL_IN + k] = o[k];
    if (a.actions) {
        int32_t *d = a.actions + r * a.act_stride;
        for (int b = 0; b < 6; b++) d[b] = act[b];
    }
    if (a.act_out)
        for (int b = 0; b < 6; b++) a.act_out[r * 6 + b] = act[b];
    if (a.log_prob) a.log_prob[r] = lp;
    if (a.value) a.value[r] = out[POL_LOGITS];
    if (a.rew_out) {
        a.rew_out[r] = a.rew_src[r * a.rd_stride];
        a.done_out[r] = a.done_src[r * a.rd_stride];
    }
}

}  // namespace bb
