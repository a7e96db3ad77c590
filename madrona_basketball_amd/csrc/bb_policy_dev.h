// bb_policy_dev.h -- device building blocks of the policy network on gfx950
// (bb_policy.h has the row math and the reference lines): the MFMA layers of
// one 16 MT-row tile and the bucket pass, shared by k_policy (bb_policy.hip)
// and the fused PPO rollout kernel (bb_kernels.hip k_rollout_policy), so that
// both compute the very same bits.
//
// The three matrix products run on v_mfma_f32_16x16x4_f32 (exact f32, a
// k-ordered fmaf chain):
//   layer 1  [16 x 128] x [128 x 32]: lane (r = l & 15, q = l >> 4) feeds
//            A = x[r][32q + j] and B = W1[n][32q + j] for j = 0..31 (32
//            contiguous floats of its row; its 64 weights in registers);
//   layer 2 / heads  [16 x 32] x [32 x 32]: k = 8q + j, the hidden tile
//            transposed through a 16 x 33 LDS tile.
// The C/D layout (col = l & 15, row = 4q + i) puts a row's 32 outputs on the 16
// lanes of one quarter-wave: LayerNorm is a 4-step xor butterfly there.
// Synchronisation inside a tile is wave-local (pol_wave_sync): the LDS words a
// wave exchanges are its own, so the pieces run in multi-wave workgroups too.
#pragma once
#include <hip/hip_runtime.h>
#include "bb_policy.h"
#include <type_traits>

namespace bb {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Ordering of LDS words written and read by different lanes of the wave.
__device__ __forceinline__ void pol_wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}



// Sum over the 16 lanes of a DPP row, the same tree as bb_policy.h pol_sum32's
// xor butterfly (partners 1, 2, then the other quad / half: once a quad holds
// equal values any cross-quad partner gives the same bits): four DPP adds.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ float quarter_sum(float t)
{
    t = t + dpp_f<0xB1>(t);   // quad_perm [1,0,3,2]: xor 1
    t = t + dpp_f<0x4E>(t);   // quad_perm [2,3,0,1]: xor 2
    t = t + dpp_f<0x141>(t);  // row_half_mirror: the other quad of the 8
    t = t + dpp_f<0x140>(t);  // row_mirror: the other 8 of the 16
    return t;
}

// 1 / sqrt(var[i] + eps) of the 4 rows a lane holds: every lane of a 16-lane
// row group holds the same four variances, so lane c evaluates only row
// (c & 3)'s (the correctly rounded square root and quotient are ~25
// instructions) and the quad's lanes exchange them by DPP broadcasts.  The
// values are the ones each lane would compute itself.
__device__ __forceinline__ void ln_inv4(const float (&var)[4], int c, float (&inv)[4])
{
    // var[c & 3] by bit masks behind an empty asm: as a select chain the
    // compiler turned it into an indexed private array (a scratch round trip)
    uint32_t me = (uint32_t)(c & 3);
    __asm__ volatile("" : "+v"(me));
    uint32_t v = __builtin_bit_cast(uint32_t, var[0]);
#pragma unroll
    for (int i = 1; i < 4; i++) {
        const uint32_t m = 0u - (uint32_t)(me == (uint32_t)i);
        v = (v & ~m) | (__builtin_bit_cast(uint32_t, var[i]) & m);
    }
    const float mine = 1.0f / bbm::sqrtf_(__builtin_bit_cast(float, v) + 1e-5f);
    inv[0] = dpp_f<0x00>(mine);  // quad_perm [0,0,0,0]
    inv[1] = dpp_f<0x55>(mine);  // [1,1,1,1]
    inv[2] = dpp_f<0xAA>(mine);  // [2,2,2,2]
    inv[3] = dpp_f<0xFF>(mine);  // [3,3,3,3]
}

// LayerNorm + ReLU of the 4 rows a lane holds (cols c and c + 16), then the
// result into the LDS tile [row][col].  SPREAD: the inverse deviations by
// ln_inv4 (k_policy: 25.3 -> 25.2 us at 65 536 rows); k_policy_wg keeps one
// per lane and row (with ln_inv4 it measured 28.0 -> 51.6 us, profiles/r04/k_*).
template <bool SPREAD = true>
__device__ __forceinline__ void ln_relu_to_tile(f32x4 a0, f32x4 a1, float bias0, float bias1, float w0, float w1,
                                                float lb0, float lb1, float (*tile)[33], int c, int q)
{
    if constexpr (SPREAD) {
        float d0[4], d1[4], var[4], inv[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const float h0 = a0[i] + bias0, h1 = a1[i] + bias1;
            const float mean = quarter_sum(h0 + h1) * (1.0f / 32.0f);
            d0[i] = h0 - mean;
            d1[i] = h1 - mean;
            var[i] = quarter_sum((d0[i] * d0[i]) + (d1[i] * d1[i])) * (1.0f / 32.0f);
        }
        ln_inv4(var, c, inv);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            tile[4 * q + i][c] = pol_relu(((d0[i] * inv[i]) * w0) + lb0);
            tile[4 * q + i][c + 16] = pol_relu(((d1[i] * inv[i]) * w1) + lb1);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const float h0 = a0[i] + bias0, h1 = a1[i] + bias1;
            const float mean = quarter_sum(h0 + h1) * (1.0f / 32.0f);
            const float d0 = h0 - mean, d1 = h1 - mean;
            const float var = quarter_sum((d0 * d0) + (d1 * d1)) * (1.0f / 32.0f);
            const float inv = 1.0f / bbm::sqrtf_(var + 1e-5f);
            tile[4 * q + i][c] = pol_relu(((d0 * inv) * w0) + lb0);
            tile[4 * q + i][c + 16] = pol_relu(((d1 * inv) * w1) + lb1);
        }
    }
}

// Bucket pass of R < 64 rows: LPR = 64 / R lanes per row,
// every step the same instructions on different data (no divergent roles):
//   B  lane part p: buckets p, p + LPR, ...: the bucket's logits, maximum,
//      exp terms and their sum in logit order, the action (first maximum, or
//      the inverse-CDF draw over the terms in logit order), logit -
//      logsumexp, into LDS;
//   C  lane part 0: the six terms summed in bucket order, the outputs.
// Every value is the one pol_bucket_term / pol_select computes (same
// operations on the same inputs), so rows are bit-identical to MT = 4's.
// (Until round 5 the maxima and the exp terms were separate phases with an
// LDS round trip between them: 8 192-world PPO trace 0.64 + 0.48 + 0.84 us.)
// The largest bucket among round j's (buckets p + lpr j, p < lpr).
__host__ __device__ constexpr int bucket_round_max(int lpr, int j)
{
    int m = 0;
    for (int p = 0; p < lpr; p++) {
        const int b = p + lpr * j;
        if (b < POL_BUCKETS && pol_bucket(b) > m) m = pol_bucket(b);
    }
    return m;
}
static_assert(bucket_round_max(2, 0) == 8 && bucket_round_max(2, 1) == 3 && bucket_round_max(2, 2) == 2 &&
                  bucket_round_max(4, 1) == 2 && bucket_round_max(8, 0) == 8,
              "bucket rounds");

// The bucket pass's LDS exchange of one wave (R rows).
template <int R>
struct BucketLds {
    float t[R][POL_BUCKETS];
    int32_t a[R][POL_BUCKETS];
};

// The uniforms a lane of the R-row bucket pass draws: buckets part + LPR j
// (pol_bucket_u's values).  They depend only on (seed, step, row, bucket), so
// a caller may draw them ahead of the logits.
template <int R>
struct BucketNoise {
    static constexpr int LPR = 64 / R, BPL = (POL_BUCKETS + LPR - 1) / LPR;
    float u[BPL];
};
template <int R>
__device__ __forceinline__ void bucket_noise(BucketNoise<R> &n, uint32_t seed, uint32_t step, int64_t row0, int64_t rows,
                                             int lane, uint32_t key0 = 0)
{
    using BN = BucketNoise<R>;
    const int r = lane / BN::LPR, part = lane % BN::LPR;
    const int64_t rr = row0 + r;
    if constexpr (R == 16) {
        // 4 lanes per row (a DPP quad), buckets part and part + 4: three
        // threefry calls per row, one per lane -- part 0 the pair of buckets
        // 0 / 1, part 1 buckets 4 / 5, parts 2 and 3 buckets 2 / 3 -- and the
        // words handed over by quad_perm moves (one call per lane instead of
        // two; the same words pol_bucket_u draws)
        uint32_t pm = part == 0 ? 0u : (part == 1 ? 2u : 1u);
        uint32_t w0, w1;
        threefry2x32(seed, step, (uint32_t)rr + key0, pm, &w0, &w1);
        const bool odd = (part & 1) != 0, live = rr < rows;
        const uint32_t a0 = dpp_u<0xA0>(w0), a1 = dpp_u<0xA0>(w1);  // quad_perm [0,0,2,2]: buckets 0-3
        const uint32_t c0 = dpp_u<0x55>(w0), c1 = dpp_u<0x55>(w1);  // quad_perm [1,1,1,1]: buckets 4, 5
        n.u[0] = live ? pol_u01(odd ? a1 : a0) : 0.f;
        n.u[1] = (live && part < 2) ? pol_u01(odd ? c1 : c0) : 0.f;
        return;
    }
    if constexpr (R == 32) {
        // 2 lanes per row, buckets part, part + 2, part + 4 (words `part` of
        // pairs 0, 1, 2): pair `part` and pair 2 per lane, pair 1 - part's
        // words from the row's other lane (quad_perm [1,0,3,2]): two threefry
        // calls per lane instead of three
        uint32_t a0, a1, b0, b1;
        threefry2x32(seed, step, (uint32_t)rr + key0, (uint32_t)part, &a0, &a1);
        threefry2x32(seed, step, (uint32_t)rr + key0, 2u, &b0, &b1);
        const uint32_t x0 = dpp_u<0xB1>(a0), x1 = dpp_u<0xB1>(a1);
        const bool live = rr < rows;
        n.u[0] = live ? pol_u01(part ? x1 : a0) : 0.f;
        n.u[1] = live ? pol_u01(part ? a1 : x0) : 0.f;
        n.u[2] = live ? pol_u01(part ? b1 : b0) : 0.f;
        return;
    }
#pragma unroll
    for (int j = 0; j < BN::BPL; j++) {
        const int b = part + BN::LPR * j;
        n.u[j] = (b < POL_BUCKETS && rr < rows) ? pol_bucket_u(seed, step, (uint32_t)rr + key0, b) : 0.f;
    }
}

// R rows (8, 16 or 32) over the wave's 64 lanes.  act_local (optional): row
// r's six actions also into act_local[r] (LDS).  pre (optional): this
// lane's uniforms, drawn ahead by bucket_noise with a's seed and step.
// PRE (compile-time, so that the uniforms stay in registers: a runtime-null
// pointer to them would put them in scratch): `pre` holds this lane's draws.
// STOCH: -1 a.stochastic at run time, 0 / 1 fixed at compile time.
template <int R, bool PRE = false, int STOCH = -1>
__device__ __forceinline__ void bucket_pass_spread(const PolicyArgs &a, float (*tile)[33], int64_t row0, int lane,
                                                   BucketLds<R> &buf, int32_t (*act_local)[6] = nullptr,
                                                   const BucketNoise<R> *pre = nullptr)
{
    static_assert(R == 8 || R == 16 || R == 32, "rows per bucket pass");
    constexpr int LPR = 64 / R;
    constexpr int BPL = (POL_BUCKETS + LPR - 1) / LPR;
    float (*tbuf)[POL_BUCKETS] = buf.t;
    int32_t (*abuf)[POL_BUCKETS] = buf.a;
    const int r = lane / LPR, part = lane % LPR;
    const int64_t rr = row0 + r;
    const bool live = rr < a.rows;
    const bool stochastic = STOCH < 0 ? a.stochastic != 0 : STOCH == 1;
    const float *lg = tile[r];
    // this lane's uniforms, drawn before the LDS work (in pass B the threefry
    // chain raised k_policy_wg over its register budget)
    BucketNoise<R> own;
    if constexpr (!PRE) {
        if (stochastic) bucket_noise<R>(own, a.seed, a.step, row0, a.rows, lane, a.key_row0);
    }
    // one phase per bucket: lane part p takes buckets p, p + LPR, ...: its
    // logits (up to 8) into registers, the maximum, exp(logit - max) of each,
    // their sum in logit order, the action (first maximum, or the inverse-CDF
    // draw over the terms in logit order), logit[a] - (max + log(sum)) --
    // pol_bucket_term's operations, the terms never leave the registers
    // round j: every lane's bucket part + LPR j; the loops run to the largest
    // bucket of the round (compile time: 8, then 3 and 2 at LPR 2), not to 8
    const auto round = [&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (j < BPL) {
            constexpr int NBM = bucket_round_max(LPR, j);
            const int b = part + LPR * j;
            if (b < POL_BUCKETS) {
                const int o = pol_bucket_off(b), nb = pol_bucket(b);
                float l[NBM];
#pragma unroll
                for (int i = 0; i < NBM; i++) {  // (in the row: o + NBM <= 21 of its 33 floats)
                    const float li = lg[o + i];
                    l[i] = i < nb ? li : 0.f;
                }
                float mx = l[0];
#pragma unroll
                for (int i = 1; i < NBM; i++)
                    if (i < nb) mx = l[i] > mx ? l[i] : mx;
                float e[NBM];
#pragma unroll
                for (int i = 0; i < NBM; i++) e[i] = pol_expf(l[i] - mx);
                float sum = e[0];
#pragma unroll
                for (int i = 1; i < NBM; i++)
                    if (i < nb) sum = sum + e[i];
                int act = 0;
                if (stochastic) {
                    const float u = PRE ? pre->u[j] : own.u[j];
                    const float t = u * sum;
                    float cs = 0.f;
                    act = nb - 1;
#pragma unroll
                    for (int i = 0; i < NBM - 1; i++) {  // (selects, no branches)
                        const bool in = i < nb - 1;
                        const float ci = cs + e[i];
                        act = (in && act == nb - 1 && ci > t) ? i : act;
                        cs = in ? ci : cs;
                    }
                } else {
                    float best = l[0];
#pragma unroll
                    for (int i = 1; i < NBM; i++) {  // first maximum
                        const bool up = i < nb && l[i] > best;
                        best = up ? l[i] : best;
                        act = up ? i : act;
                    }
                }
                const float lse = mx + pol_logf(sum);
                float la = l[0];
#pragma unroll
                for (int i = 1; i < NBM; i++) la = act == i ? l[i] : la;
                abuf[r][b] = act;
                tbuf[r][b] = la - lse;
            }
        }
    };
    round(std::integral_constant<int, 0>());
    round(std::integral_constant<int, 1>());
    round(std::integral_constant<int, 2>());
    pol_wave_sync();
    if (part == 0 && live) {
        float term[POL_BUCKETS];
        int32_t act[POL_BUCKETS];
#pragma unroll
        for (int b = 0; b < POL_BUCKETS; b++) { term[b] = tbuf[r][b]; act[b] = abuf[r][b]; }
        const float lp = pol_logp_sum(term);
        if (act_local)
#pragma unroll
            for (int b = 0; b < 6; b++) act_local[r][b] = act[b];
        if (a.actions) {
            int32_t *d = a.actions + rr * a.act_stride;
#pragma unroll
            for (int b = 0; b < 6; b++) d[b] = act[b];
        }
        if (a.act_out) {
            int2 *d = (int2 *)(a.act_out + rr * 6);
            d[0] = make_int2(act[0], act[1]);
            d[1] = make_int2(act[2], act[3]);
            d[2] = make_int2(act[4], act[5]);
        }
        if (a.log_prob) a.log_prob[rr] = lp;
        if (a.value) a.value[rr] = lg[POL_LOGITS];
        if (a.rew_out) {  // the previous step's outcome of this row (buffer.rewards / not_dones)
            a.rew_out[rr] = a.rew_src[rr * a.rd_stride];
            a.done_out[rr] = a.done_src[rr * a.rd_stride];
        }
    }
}

// bucket_pass_spread in two halves, for a caller whose consumer needs the
// actions before the log-probabilities (the fused PPO rollout: the sim wave
// waits for the actions only).  bucket_pass_act runs every bucket's logits,
// maximum, exp terms, sum and action and puts the row's six actions into
// act_local; what the log-probability needs (maximum, sum, the chosen logit)
// stays in the lane's registers (BucketHold).  bucket_pass_out then computes
// logit - (max + log(sum)) per bucket and the outputs -- the same operations
// on the same values as bucket_pass_spread, so rows are bit-identical; only
// the order of the two halves around the caller's hand-off differs.
template <int R>
struct BucketHold {
    static constexpr int BPL = (POL_BUCKETS + 64 / R - 1) / (64 / R);
    float mx[BPL], sum[BPL], la[BPL];
};

template <int R, bool PRE = false>
__device__ __forceinline__ void bucket_pass_act(const PolicyArgs &a, float (*tile)[33], int64_t row0, int lane,
                                                BucketLds<R> &buf, int32_t (*act_local)[6], const BucketNoise<R> *pre,
                                                BucketHold<R> &hold)
{
    static_assert(R == 8 || R == 16 || R == 32, "rows per bucket pass");
    constexpr int LPR = 64 / R;
    constexpr int BPL = (POL_BUCKETS + LPR - 1) / LPR;
    int32_t (*abuf)[POL_BUCKETS] = buf.a;
    const int r = lane / LPR, part = lane % LPR;
    const int64_t rr = row0 + r;
    const bool live = rr < a.rows;
    const bool stochastic = a.stochastic != 0;
    const float *lg = tile[r];
    BucketNoise<R> own;
    if constexpr (!PRE) {
        if (stochastic) bucket_noise<R>(own, a.seed, a.step, row0, a.rows, lane, a.key_row0);
    }
    const auto round = [&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (j < BPL) {
            constexpr int NBM = bucket_round_max(LPR, j);
            const int b = part + LPR * j;
            hold.mx[j] = 0.f; hold.sum[j] = 1.f; hold.la[j] = 0.f;
            if (b < POL_BUCKETS) {
                const int o = pol_bucket_off(b), nb = pol_bucket(b);
                float l[NBM];
#pragma unroll
                for (int i = 0; i < NBM; i++) {
                    const float li = lg[o + i];
                    l[i] = i < nb ? li : 0.f;
                }
                float mx = l[0];
#pragma unroll
                for (int i = 1; i < NBM; i++)
                    if (i < nb) mx = l[i] > mx ? l[i] : mx;
                float e[NBM];
#pragma unroll
                for (int i = 0; i < NBM; i++) e[i] = pol_expf(l[i] - mx);
                float sum = e[0];
#pragma unroll
                for (int i = 1; i < NBM; i++)
                    if (i < nb) sum = sum + e[i];
                int act = 0;
                if (stochastic) {
                    const float u = PRE ? pre->u[j] : own.u[j];
                    const float t = u * sum;
                    float cs = 0.f;
                    act = nb - 1;
#pragma unroll
                    for (int i = 0; i < NBM - 1; i++) {
                        const bool in = i < nb - 1;
                        const float ci = cs + e[i];
                        act = (in && act == nb - 1 && ci > t) ? i : act;
                        cs = in ? ci : cs;
                    }
                } else {
                    float best = l[0];
#pragma unroll
                    for (int i = 1; i < NBM; i++) {
                        const bool up = i < nb && l[i] > best;
                        best = up ? l[i] : best;
                        act = up ? i : act;
                    }
                }
                float la = l[0];
#pragma unroll
                for (int i = 1; i < NBM; i++) la = act == i ? l[i] : la;
                abuf[r][b] = act;
                hold.mx[j] = mx; hold.sum[j] = sum; hold.la[j] = la;
            }
        }
    };
    round(std::integral_constant<int, 0>());
    round(std::integral_constant<int, 1>());
    round(std::integral_constant<int, 2>());
    pol_wave_sync();
    if (part == 0 && live) {
#pragma unroll
        for (int b = 0; b < 6; b++) act_local[r][b] = abuf[r][b];
    }
}

template <int R>
__device__ __forceinline__ void bucket_pass_out(const PolicyArgs &a, float (*tile)[33], int64_t row0, int lane,
                                                BucketLds<R> &buf, const BucketHold<R> &hold)
{
    constexpr int LPR = 64 / R;
    constexpr int BPL = (POL_BUCKETS + LPR - 1) / LPR;
    float (*tbuf)[POL_BUCKETS] = buf.t;
    int32_t (*abuf)[POL_BUCKETS] = buf.a;
    const int r = lane / LPR, part = lane % LPR;
    const int64_t rr = row0 + r;
    const bool live = rr < a.rows;
#pragma unroll
    for (int j = 0; j < BPL; j++) {
        const int b = part + LPR * j;
        if (b < POL_BUCKETS) {
            const float lse = hold.mx[j] + pol_logf(hold.sum[j]);
            tbuf[r][b] = hold.la[j] - lse;
        }
    }
    pol_wave_sync();
    if (part == 0 && live) {
        float term[POL_BUCKETS];
        int32_t act[POL_BUCKETS];
#pragma unroll
        for (int b = 0; b < POL_BUCKETS; b++) { term[b] = tbuf[r][b]; act[b] = abuf[r][b]; }
        const float lp = pol_logp_sum(term);
        if (a.act_out) {
            int2 *d = (int2 *)(a.act_out + rr * 6);
            d[0] = make_int2(act[0], act[1]);
            d[1] = make_int2(act[2], act[3]);
            d[2] = make_int2(act[4], act[5]);
        }
        if (a.log_prob) a.log_prob[rr] = lp;
        if (a.value) a.value[rr] = tile[r][POL_LOGITS];
    }
}

// The network's weights in LDS, shared by the waves of a workgroup (k_policy_wg,
// k_step_ppo): images conflict-free for the lanes' 16-byte reads (lane (c, q)
// reads W[16t + c][k-chunk q]): planes [q][n][j] padded to 36 / 12 floats
// (every ds_read_b128 lane group of 16 lanes covers the 64 banks once).
constexpr int PWG_P1 = 36, PWG_P2 = 12;
struct PolicyLdsWeights {
    float w1[4][32][PWG_P1];  // W1[n][32q + j]
    float w2[4][32][PWG_P2];  // W2[n][8q + j]
    float wh[4][32][PWG_P2];  // head_w[n][8q + j]
    float norm[2][POL_IN];    // obs_mean, obs_inv
    float cst[7][32];         // b1, ln1_w, ln1_b, b2, ln2_w, ln2_b, head_b
};

// Thread tid of nt copies its share of the weights into L (the caller orders
// the writes before their first read with a workgroup barrier).
__device__ __forceinline__ void policy_weights_to_lds(PolicyLdsWeights &L, const PolicyWeights &W, int tid, int nt)
{
    for (int i = tid; i < 32 * 32; i += nt) {  // W1 [32][128] as float4
        const int n = i >> 5, k = 4 * (i & 31);
        *(float4 *)&L.w1[k >> 5][n][k & 31] = ((const float4 *)W.w1)[i];
    }
    for (int i = tid; i < 32 * 8; i += nt) {  // W2, head_w [32][32] as float4
        const int n = i >> 3, k = 4 * (i & 7);
        *(float4 *)&L.w2[k >> 3][n][k & 7] = ((const float4 *)W.w2)[i];
        *(float4 *)&L.wh[k >> 3][n][k & 7] = ((const float4 *)W.head_w)[i];
    }
    for (int k = tid; k < POL_IN; k += nt) {
        L.norm[0][k] = W.obs_mean[k];
        L.norm[1][k] = W.obs_inv[k];
    }
    for (int k = tid; k < 7 * 32; k += nt) {
        const float *src[7] = {W.b1, W.ln1_w, W.ln1_b, W.b2, W.ln2_w, W.ln2_b, W.head_b};
        L.cst[k >> 5][k & 31] = src[k >> 5][k & 31];
    }
}

// Layer 2 + LayerNorm + ReLU, then the heads, of one 16-row M-tile whose
// layer-1 output is in tm[16][33], with the weights in LDS: row r's 19 logits
// and value into tm[r][0..19].  The same operands in the same order as
// policy_layers' second loop (lane (c, q): k = 8q + j).
__device__ __forceinline__ void policy_tail_lds(const PolicyLdsWeights &L, float (*tm)[33], int c, int q)
{
#pragma unroll
    for (int layer = 0; layer < 2; layer++) {
        const float (*wl)[32][PWG_P2] = layer == 0 ? L.w2 : L.wh;
        float h[8];
#pragma unroll
        for (int j = 0; j < 8; j++) h[j] = tm[c][8 * q + j];
        pol_wave_sync();
        float w0[8], w1[8];
#pragma unroll
        for (int v = 0; v < 2; v++) {
            const float4 u0 = *(const float4 *)&wl[q][c][4 * v];
            const float4 u1 = *(const float4 *)&wl[q][16 + c][4 * v];
            w0[4 * v] = u0.x; w0[4 * v + 1] = u0.y; w0[4 * v + 2] = u0.z; w0[4 * v + 3] = u0.w;
            w1[4 * v] = u1.x; w1[4 * v + 1] = u1.y; w1[4 * v + 2] = u1.z; w1[4 * v + 3] = u1.w;
        }
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 8; j++) {
            a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], w0[j], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], w1[j], a1, 0, 0, 0);
        }
        if (layer == 0) {
            ln_relu_to_tile(a0, a1, L.cst[3][c], L.cst[3][c + 16], L.cst[4][c], L.cst[4][c + 16], L.cst[5][c],
                            L.cst[5][c + 16], tm, c, q);
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                tm[4 * q + i][c] = a0[i] + L.cst[6][c];
                tm[4 * q + i][c + 16] = a1[i] + L.cst[6][c + 16];
            }
        }
        pol_wave_sync();
    }
}

// policy_tail_lds for two M-tiles at once (rows 0..31 of t[32][33]): each
// layer's MFMA chains of both tiles are issued before the first tile's
// LayerNorm, so that tile's VALU work runs while the matrix pipe works
// through the second tile's chains.  The same operations on the same values.
__device__ __forceinline__ void policy_tail_lds2(const PolicyLdsWeights &L, float (*t)[33], int c, int q)
{
#pragma unroll
    for (int layer = 0; layer < 2; layer++) {
        const float (*wl)[32][PWG_P2] = layer == 0 ? L.w2 : L.wh;
        float h[2][8];
#pragma unroll
        for (int m = 0; m < 2; m++)
#pragma unroll
            for (int j = 0; j < 8; j++) h[m][j] = t[16 * m + c][8 * q + j];
        pol_wave_sync();
        float w0[8], w1[8];
#pragma unroll
        for (int v = 0; v < 2; v++) {
            const float4 u0 = *(const float4 *)&wl[q][c][4 * v];
            const float4 u1 = *(const float4 *)&wl[q][16 + c][4 * v];
            w0[4 * v] = u0.x; w0[4 * v + 1] = u0.y; w0[4 * v + 2] = u0.z; w0[4 * v + 3] = u0.w;
            w1[4 * v] = u1.x; w1[4 * v + 1] = u1.y; w1[4 * v + 2] = u1.z; w1[4 * v + 3] = u1.w;
        }
        f32x4 a[2][2];
#pragma unroll
        for (int m = 0; m < 2; m++) {
            a[m][0] = a[m][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 8; j++) {
                a[m][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(h[m][j], w0[j], a[m][0], 0, 0, 0);
                a[m][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(h[m][j], w1[j], a[m][1], 0, 0, 0);
            }
        }
#pragma unroll
        for (int m = 0; m < 2; m++) {
            float (*tm)[33] = t + 16 * m;
            if (layer == 0) {
                ln_relu_to_tile(a[m][0], a[m][1], L.cst[3][c], L.cst[3][c + 16], L.cst[4][c], L.cst[4][c + 16],
                                L.cst[5][c], L.cst[5][c + 16], tm, c, q);
            } else {
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    tm[4 * q + i][c] = a[m][0][i] + L.cst[6][c];
                    tm[4 * q + i][c + 16] = a[m][1][i] + L.cst[6][c + 16];
                }
            }
        }
        pol_wave_sync();
    }
}

// The B operands and the per-column constants of one lane, loaded once per
// wave and kept in registers for every tile it processes.
struct PolicyRegs {
    float w1[2][32], w2[2][8], wh[2][8];
    float b1_0, b1_1, l1w0, l1w1, l1b0, l1b1, b2_0, b2_1, l2w0, l2w1, l2b0, l2b1, bh0, bh1;
};

__device__ __forceinline__ void load_policy_regs(PolicyRegs &R, const PolicyWeights &W, int c, int q)
{
#pragma unroll
    for (int t = 0; t < 2; t++) {
        const float4 *src = (const float4 *)(W.w1 + (16 * t + c) * POL_IN + 32 * q);
#pragma unroll
        for (int v = 0; v < 8; v++) {
            const float4 x = src[v];
            R.w1[t][4 * v] = x.x; R.w1[t][4 * v + 1] = x.y; R.w1[t][4 * v + 2] = x.z; R.w1[t][4 * v + 3] = x.w;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            R.w2[t][j] = W.w2[(16 * t + c) * POL_HID + 8 * q + j];
            R.wh[t][j] = W.head_w[(16 * t + c) * POL_HID + 8 * q + j];
        }
    }
    R.b1_0 = W.b1[c]; R.b1_1 = W.b1[c + 16]; R.l1w0 = W.ln1_w[c]; R.l1w1 = W.ln1_w[c + 16];
    R.l1b0 = W.ln1_b[c]; R.l1b1 = W.ln1_b[c + 16];
    R.b2_0 = W.b2[c]; R.b2_1 = W.b2[c + 16]; R.l2w0 = W.ln2_w[c]; R.l2w1 = W.ln2_w[c + 16];
    R.l2b0 = W.ln2_b[c]; R.l2b1 = W.ln2_b[c + 16];
    R.bh0 = W.head_b[c]; R.bh1 = W.head_b[c + 16];
}

// Layer 2 + LayerNorm + ReLU, then the heads, of one 16-row M-tile whose
// layer-1 output is in tm[16][33] (policy_layers' second loop; the B operands
// in registers): row r's 19 logits and value into tm[r][0..19].
__device__ __forceinline__ void policy_tail_regs(const PolicyRegs &R, float (*tm)[33], int c, int q)
{
    float h[8];
#pragma unroll
    for (int j = 0; j < 8; j++) h[j] = tm[c][8 * q + j];
    pol_wave_sync();
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 8; j++) {
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], R.w2[0][j], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], R.w2[1][j], a1, 0, 0, 0);
    }
    ln_relu_to_tile(a0, a1, R.b2_0, R.b2_1, R.l2w0, R.l2w1, R.l2b0, R.l2b1, tm, c, q);
    pol_wave_sync();
#pragma unroll
    for (int j = 0; j < 8; j++) h[j] = tm[c][8 * q + j];
    pol_wave_sync();
    a0 = f32x4{0.f, 0.f, 0.f, 0.f};
    a1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 8; j++) {
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], R.wh[0][j], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], R.wh[1][j], a1, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        tm[4 * q + i][c] = a0[i] + R.bh0;
        tm[4 * q + i][c + 16] = a1[i] + R.bh1;
    }
}

// The network on one tile of 16 MT rows: x[m][j] = observation float 32q + j
// of row 16m + c (lane (c, q)); norm = {mean, rsqrt(var + eps)} in LDS.
// Leaves each row's 19 logits and value (column 19) in tile[row][0..19].
template <int MT>
__device__ __forceinline__ void policy_layers(float (&x)[MT][32], const PolicyRegs &R, const float (*norm)[POL_IN],
                                              float (*tile)[33], int c, int q)
{
    // layer 1 (two independent accumulators per M-tile keep the MFMA pipe full)
    float nm[32], ni[32];
#pragma unroll
    for (int v = 0; v < 8; v++) {
        const float4 a4 = *(const float4 *)&norm[0][32 * q + 4 * v];
        const float4 b4 = *(const float4 *)&norm[1][32 * q + 4 * v];
        nm[4 * v] = a4.x; nm[4 * v + 1] = a4.y; nm[4 * v + 2] = a4.z; nm[4 * v + 3] = a4.w;
        ni[4 * v] = b4.x; ni[4 * v + 1] = b4.y; ni[4 * v + 2] = b4.z; ni[4 * v + 3] = b4.w;
    }
    // Software-pipelined over the M-tiles: the MFMA chain of tile m is issued
    // before the VALU work of tile m - 1 (its LayerNorm) and of tile m + 1
    // (its normalisation), which then run while the matrix pipe works
    // through tile m.  Blocks fenced by scheduling barriers, so each keeps its
    // place: the normalisation as one block, then the MFMA chain back to back
    // (interleaved, every MFMA waits out a VALU-write hazard).
    f32x4 acc[MT][2];
#pragma unroll
    for (int j = 0; j < 32; j++) x[0][j] = pol_clamp((x[0][j] - nm[j]) * ni[j]);
#pragma unroll
    for (int m = 0; m < MT; m++) {
        __builtin_amdgcn_sched_barrier(0);
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 32; j++) {
            a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[m][j], R.w1[0][j], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[m][j], R.w1[1][j], a1, 0, 0, 0);
        }
        acc[m][0] = a0;
        acc[m][1] = a1;
        __builtin_amdgcn_sched_barrier(0);
        if (m + 1 < MT) {
#pragma unroll
            for (int j = 0; j < 32; j++) x[m + 1][j] = pol_clamp((x[m + 1][j] - nm[j]) * ni[j]);
        }
        if (m > 0) {
            __builtin_amdgcn_sched_barrier(0);
            ln_relu_to_tile(acc[m - 1][0], acc[m - 1][1], R.b1_0, R.b1_1, R.l1w0, R.l1w1, R.l1b0, R.l1b1,
                            tile + 16 * (m - 1), c, q);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    ln_relu_to_tile(acc[MT - 1][0], acc[MT - 1][1], R.b1_0, R.b1_1, R.l1w0, R.l1w1, R.l1b0, R.l1b1,
                    tile + 16 * (MT - 1), c, q);
    pol_wave_sync();
    // layer 2 and heads, per M-tile through its 16 rows of the tile
#pragma unroll
    for (int m = 0; m < MT; m++) policy_tail_regs(R, tile + 16 * m, c, q);
    pol_wave_sync();
}

// policy_layers<1> with the rows arriving in two halves (as
// policy_layers_half_split): lane group q's floats 32q + [0, 16) of row c are
// in LDS at xrow when called, 32q + [16, 32) after mid().  Layer 1's two
// accumulator chains take steps 0..15 before mid(), 16..31 after; then the
// LayerNorm, layer 2 and the heads of policy_layers.  The same bits.
template <class Mid>
__device__ __forceinline__ void policy_layers1_split(const float *xrow, const PolicyRegs &R,
                                                     const float (*norm)[POL_IN], float (*tile)[33], int c, int q,
                                                     Mid mid)
{
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int half = 0; half < 2; half++) {
        if (half == 1) mid();
        float x[16];
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int k = 32 * q + 16 * half + 4 * v;
            const float4 o = *(const float4 *)(xrow + k);
            const float4 a4 = *(const float4 *)&norm[0][k];
            const float4 b4 = *(const float4 *)&norm[1][k];
            x[4 * v] = pol_clamp((o.x - a4.x) * b4.x);
            x[4 * v + 1] = pol_clamp((o.y - a4.y) * b4.y);
            x[4 * v + 2] = pol_clamp((o.z - a4.z) * b4.z);
            x[4 * v + 3] = pol_clamp((o.w - a4.w) * b4.w);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 16; j++) {
            a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[j], R.w1[0][16 * half + j], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[j], R.w1[1][16 * half + j], a1, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    ln_relu_to_tile(a0, a1, R.b1_0, R.b1_1, R.l1w0, R.l1w1, R.l1b0, R.l1b1, tile, c, q);
    pol_wave_sync();
    policy_tail_regs(R, tile, c, q);
    pol_wave_sync();
}

// LayerNorm + ReLU of rows 4q + i, i in [I0, I1), of a lane's accumulators
// (the rows ln_relu_to_tile covers, the same operations).
template <int I0, int I1>
__device__ __forceinline__ void ln_relu_rows(f32x4 a0, f32x4 a1, float bias0, float bias1, float w0, float w1,
                                             float lb0, float lb1, float (*tile)[33], int c, int q)
{
#pragma unroll
    for (int i = I0; i < I1; i++) {
        const float h0 = a0[i] + bias0, h1 = a1[i] + bias1;
        const float mean = quarter_sum(h0 + h1) * (1.0f / 32.0f);
        const float d0 = h0 - mean, d1 = h1 - mean;
        const float var = quarter_sum((d0 * d0) + (d1 * d1)) * (1.0f / 32.0f);
        const float inv = 1.0f / bbm::sqrtf_(var + 1e-5f);
        tile[4 * q + i][c] = pol_relu(((d0 * inv) * w0) + lb0);
        tile[4 * q + i][c + 16] = pol_relu(((d1 * inv) * w1) + lb1);
    }
}

// policy_layers<1> on one 16-row M-tile by two waves, h = 0 and 1: wave h
// runs the accumulator chain of output columns 16h..16h+15 of every product
// (the a0 / a1 chain of policy_layers, the same MFMA sequence) and the
// LayerNorm of rows 4q + 2h, 4q + 2h + 1 (the same operations), the two halves
// exchanged through `ex`.  bar(): a workgroup barrier both waves pass (5
// calls).  Leaves row r's logits and value in ltile[r][0..19].
struct HalfExchange {
    f32x4 acc[2][64];  // [h][lane]
};
// The part of policy_layers_half after layer 1's chain (acc: the wave's half
// of the M-tile's layer-1 outputs).
template <class Bar>
__device__ __forceinline__ void policy_layers_half_rest(f32x4 acc, const PolicyRegs &R, float (*tile)[33],
                                                        float (*ltile)[33], HalfExchange &ex, int c, int q, int lane,
                                                        int h, Bar bar)
{
    ex.acc[h][lane] = acc;
    bar();
    if (h == 0)
        ln_relu_rows<0, 2>(ex.acc[0][lane], ex.acc[1][lane], R.b1_0, R.b1_1, R.l1w0, R.l1w1, R.l1b0, R.l1b1, tile, c, q);
    else
        ln_relu_rows<2, 4>(ex.acc[0][lane], ex.acc[1][lane], R.b1_0, R.b1_1, R.l1w0, R.l1w1, R.l1b0, R.l1b1, tile, c, q);
    bar();
    float hh[8];
#pragma unroll
    for (int j = 0; j < 8; j++) hh[j] = tile[c][8 * q + j];
    acc = f32x4{0.f, 0.f, 0.f, 0.f};
    if (h == 0) {
#pragma unroll
        for (int j = 0; j < 8; j++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(hh[j], R.w2[0][j], acc, 0, 0, 0);
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(hh[j], R.w2[1][j], acc, 0, 0, 0);
    }
    ex.acc[h][lane] = acc;
    bar();
    if (h == 0)
        ln_relu_rows<0, 2>(ex.acc[0][lane], ex.acc[1][lane], R.b2_0, R.b2_1, R.l2w0, R.l2w1, R.l2b0, R.l2b1, tile, c, q);
    else
        ln_relu_rows<2, 4>(ex.acc[0][lane], ex.acc[1][lane], R.b2_0, R.b2_1, R.l2w0, R.l2w1, R.l2b0, R.l2b1, tile, c, q);
    bar();
#pragma unroll
    for (int j = 0; j < 8; j++) hh[j] = tile[c][8 * q + j];
    acc = f32x4{0.f, 0.f, 0.f, 0.f};
    if (h == 0) {
#pragma unroll
        for (int j = 0; j < 8; j++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(hh[j], R.wh[0][j], acc, 0, 0, 0);
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(hh[j], R.wh[1][j], acc, 0, 0, 0);
    }
    const float bh = h == 0 ? R.bh0 : R.bh1;
#pragma unroll
    for (int i = 0; i < 4; i++) ltile[4 * q + i][c + 16 * h] = acc[i] + bh;
    bar();
}

template <class Bar>
__device__ __forceinline__ void policy_layers_half(float (&x)[32], const PolicyRegs &R, const float (*norm)[POL_IN],
                                                   float (*tile)[33], float (*ltile)[33], HalfExchange &ex, int c,
                                                   int q, int lane, int h, Bar bar)
{
    float nm[32], ni[32];
#pragma unroll
    for (int v = 0; v < 8; v++) {
        const float4 a4 = *(const float4 *)&norm[0][32 * q + 4 * v];
        const float4 b4 = *(const float4 *)&norm[1][32 * q + 4 * v];
        nm[4 * v] = a4.x; nm[4 * v + 1] = a4.y; nm[4 * v + 2] = a4.z; nm[4 * v + 3] = a4.w;
        ni[4 * v] = b4.x; ni[4 * v + 1] = b4.y; ni[4 * v + 2] = b4.z; ni[4 * v + 3] = b4.w;
    }
#pragma unroll
    for (int j = 0; j < 32; j++) x[j] = pol_clamp((x[j] - nm[j]) * ni[j]);
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (h == 0) {
#pragma unroll
        for (int j = 0; j < 32; j++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[j], R.w1[0][j], acc, 0, 0, 0);
    } else {
#pragma unroll
        for (int j = 0; j < 32; j++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[j], R.w1[1][j], acc, 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    policy_layers_half_rest(acc, R, tile, ltile, ex, c, q, lane, h, bar);
}

// policy_layers_half with the rows arriving in two halves: lane group q's
// floats 32q + [0, 16) are in LDS at xrow (row c of the M-tile) when called,
// floats 32q + [16, 32) after mid() (a workgroup barrier: the hand-off of the
// second half).  Layer 1's chain steps 0..15 run before mid(), 16..31 after --
// the same chain, the same bits.
template <class Mid, class Bar>
__device__ __forceinline__ void policy_layers_half_split(const float *xrow, const PolicyRegs &R,
                                                         const float (*norm)[POL_IN], float (*tile)[33],
                                                         float (*ltile)[33], HalfExchange &ex, int c, int q, int lane,
                                                         int h, Mid mid, Bar bar)
{
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int half = 0; half < 2; half++) {
        if (half == 1) mid();
        float x[16];
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int k = 32 * q + 16 * half + 4 * v;
            const float4 o = *(const float4 *)(xrow + k);
            const float4 a4 = *(const float4 *)&norm[0][k];
            const float4 b4 = *(const float4 *)&norm[1][k];
            x[4 * v] = pol_clamp((o.x - a4.x) * b4.x);
            x[4 * v + 1] = pol_clamp((o.y - a4.y) * b4.y);
            x[4 * v + 2] = pol_clamp((o.z - a4.z) * b4.z);
            x[4 * v + 3] = pol_clamp((o.w - a4.w) * b4.w);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (h == 0) {
#pragma unroll
            for (int j = 0; j < 16; j++)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[j], R.w1[0][16 * half + j], acc, 0, 0, 0);
        } else {
#pragma unroll
            for (int j = 0; j < 16; j++)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[j], R.w1[1][16 * half + j], acc, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    policy_layers_half_rest(acc, R, tile, ltile, ex, c, q, lane, h, bar);
}

}  // namespace bb
