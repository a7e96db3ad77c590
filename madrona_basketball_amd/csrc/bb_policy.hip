// bb_policy.hip -- fused policy inference on gfx950:
// observation rows -> RunningMeanStd -> 2 x (Linear + LayerNorm + ReLU) ->
// actor/critic heads -> per-bucket argmax or categorical sample, log-prob and
// value, written straight into the simulator's action tensor (bb_policy.h has
// the row math and the reference lines).
//
// One wave per workgroup, 64 rows per tile (4 MFMA row blocks of 16), grid-stride.  The three matrix
// products run on v_mfma_f32_16x16x4_f32 (exact f32, a k-ordered fmaf chain):
//   layer 1  [16 x 128] x [128 x 32]: lane (r = l & 15, q = l >> 4) feeds
//            A = x[r][32q + j] and B = W1[n][32q + j] for j = 0..31, so each
//            lane reads 32 contiguous floats of its row (8 x 16-byte loads)
//            and keeps its 64 weights in registers for the whole launch;
//   layer 2 / heads  [16 x 32] x [32 x 32]: k = 8q + j, the hidden tile
//            transposed through a 16 x 33 LDS tile.
// The C/D layout (col = l & 15, row = 4q + i) puts a row's 32 outputs on the 16
// lanes of one quarter-wave: LayerNorm is a 4-step xor butterfly there.
#include <hip/hip_runtime.h>
#include "bb_launch.h"
#include "bb_policy.h"
#include "bb_policy_dev.h"

namespace bb {

// diagnostics (PolicyArgs::diag_ts): the clock at phase boundaries of the
// wave's first tile -- 0 start, 1 weights loaded, 2 rows loaded, 3 layer 1,
// 4 layer 2 + heads, 5 bucket pass done
__device__ __forceinline__ void pol_trace(const PolicyArgs &a, bool first, int point, bool wait_mem)
{
    if (a.diag_ts && first) {
        if (wait_mem) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t t = wall_clock64();
        if (threadIdx.x == 0) a.diag_ts[(int64_t)blockIdx.x * POL_TRACE_POINTS + point] = t;
    }
}

// the same clocks for k_policy_wg, indexed by the wave's global id
__device__ __forceinline__ void pol_trace_wg(const PolicyArgs &a, int64_t gw, int point, bool wait_mem)
{
    if (a.diag_ts) {
        if (wait_mem) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t t = wall_clock64();
        if ((threadIdx.x & 63) == 0) a.diag_ts[gw * POL_TRACE_POINTS + point] = t;
    }
}

template <int MT>
__global__ __launch_bounds__(64) void k_policy(const PolicyArgs a)
{
    // MT: 16-row M-tiles per tile
    pol_trace(a, true, 0, false);
    __shared__ __attribute__((aligned(16))) float norm[2][POL_IN];
    __shared__ float tile[16 * MT][33];
    const int lane = threadIdx.x, c = lane & 15, q = lane >> 4;
    const PolicyWeights &W = a.w;
    for (int k = lane; k < POL_IN; k += 64) {
        norm[0][k] = W.obs_mean[k];
        norm[1][k] = W.obs_inv[k];
    }
    // B operands, loaded once per (persistent) wave
    PolicyRegs R;
    load_policy_regs(R, W, c, q);
    pol_wave_sync();
    pol_trace(a, true, 1, true);

    const int64_t tiles = (a.rows + 16 * MT - 1) / (16 * MT);
    // every M-tile's 32 observation floats per lane, loads issued together;
    // in a grid-stride loop the next tile's rows are loaded while this tile
    // is computed
    auto load_rows = [&](int64_t row0, float (&x)[MT][32]) {
#pragma unroll
        for (int m = 0; m < MT; m++) {
            const int64_t r = row0 + 16 * m + c;
            if (r < a.rows) {
                const float4 *src = (const float4 *)(a.obs + r * a.obs_stride + 32 * q);
#pragma unroll
                for (int v = 0; v < 8; v++) {
                    const float4 o = src[v];
                    x[m][4 * v] = o.x; x[m][4 * v + 1] = o.y; x[m][4 * v + 2] = o.z; x[m][4 * v + 3] = o.w;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 32; j++) x[m][j] = 0.f;
            }
        }
    };
    // (PREFETCH: 64-row tiles, whose kernel holds a wave per SIMD anyway; at
    // MT = 1 the second row set would cost the two waves per SIMD)
    constexpr bool PREFETCH = MT == 4;
    float xn[PREFETCH ? MT : 1][32];
    if constexpr (PREFETCH)
        if ((int64_t)blockIdx.x < tiles) load_rows((int64_t)blockIdx.x * 16 * MT, xn);
    for (int64_t tl = blockIdx.x; tl < tiles; tl += gridDim.x) {
        const int64_t row0 = tl * 16 * MT;
        const bool first = tl == blockIdx.x;
        float x[MT][32];
        if constexpr (PREFETCH) {
#pragma unroll
            for (int m = 0; m < MT; m++)
#pragma unroll
                for (int j = 0; j < 32; j++) x[m][j] = xn[m][j];
            if (tl + gridDim.x < tiles) load_rows((tl + gridDim.x) * 16 * MT, xn);
        } else {
            load_rows(row0, x);
        }
        if (a.obs_out) {  // the rollout's record of the observed rows (buffer.obs, ppo.py:129)
#pragma unroll
            for (int m = 0; m < MT; m++) {
                const int64_t r = row0 + 16 * m + c;
                if (r < a.rows) {
                    float4 *dst = (float4 *)(a.obs_out + r * POL_IN + 32 * q);
#pragma unroll
                    for (int v = 0; v < 8; v++)
                        dst[v] = make_float4(x[m][4 * v], x[m][4 * v + 1], x[m][4 * v + 2], x[m][4 * v + 3]);
                }
            }
        }
        pol_trace(a, first, 2, true);
        policy_layers<MT>(x, R, norm, tile, c, q);
        pol_trace(a, first, 4, false);
        if constexpr (16 * MT < 64) {
            __shared__ BucketLds<16 * MT> bl;
            bucket_pass_spread<16 * MT>(a, tile, row0, lane, bl);
            pol_wave_sync();
            pol_trace(a, first, 5, false);
            continue;
        }
        // one row per lane: buckets, log-prob, value
        const int64_t rr = row0 + lane;
        if (lane < 16 * MT && rr < a.rows) {
            float logit[POL_LOGITS + 1];
#pragma unroll
            for (int i = 0; i <= POL_LOGITS; i++) logit[i] = tile[lane][i];
            int32_t act[6];
            float lp;
            pol_select(logit, a.stochastic != 0, a.seed, a.step, (uint32_t)rr + a.key_row0, act, &lp);
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
            if (a.value) a.value[rr] = logit[POL_LOGITS];
            if (a.rew_out) {  // the previous step's outcome of this row (buffer.rewards / not_dones)
                a.rew_out[rr] = a.rew_src[rr * a.rd_stride];
                a.done_out[rr] = a.done_src[rr * a.rd_stride];
            }
        }
        pol_wave_sync();
        pol_trace(a, first, 5, false);
    }
}

// ---------------------------------------------------------------------------
// k_policy_wg: the network's B operands in LDS, shared by a workgroup of up
// to 12 waves (one workgroup per CU, three waves per SIMD),
// 16-row tiles per wave in a grid-stride loop.  With the weights in
// registers (k_policy) a wave needs 238-480 VGPRs, so a SIMD holds one or two
// waves and each wave's chain -- row loads, 96 dependent-pair MFMAs, the
// LayerNorm DPP trees, the bucket pass -- runs alone; here three waves per
// SIMD overlap one wave's MFMAs with the others' VALU / LDS / memory work.
// Every value is computed as k_policy<1> computes it (the same MFMA operands
// in the same order, the same LayerNorm and bucket pass), so the outputs are
// bit-identical.
//
// The weights' LDS images: PolicyLdsWeights (bb_policy_dev.h).
#ifndef BB_PWG_WAVES
#define BB_PWG_WAVES 12  // 3 per SIMD: 141-159 VGPRs (at 16 the 128-VGPR budget spills 16-104 B)
#endif
constexpr int PWG_WAVES = BB_PWG_WAVES;
struct PolicyWgLds {
    PolicyLdsWeights wt;
    float tile[PWG_WAVES][16][33];
    BucketLds<16> bl[PWG_WAVES];
};

template <bool PREFETCH, int STOCH>
__global__ __launch_bounds__(64 * PWG_WAVES) void k_policy_wg(const PolicyArgs a)
{
    __shared__ __attribute__((aligned(16))) PolicyWgLds L;
    const int tid = (int)threadIdx.x, wave = tid >> 6, lane = tid & 63, c = lane & 15, q = lane >> 4;
    const int nw = (int)(blockDim.x >> 6);
    const int64_t tiles = (a.rows + 15) / 16;
    const int64_t tw0 = (int64_t)blockIdx.x * nw + wave, tstride = (int64_t)gridDim.x * nw;
    pol_trace_wg(a, tw0, 0, false);
    const PolicyWeights &W = a.w;
    // lane (c, q): observation floats 32q .. 32q + 31 of row row0 + c
    auto load_rows = [&](int64_t row0, float (&x)[32]) {
        const int64_t r = row0 + c;
        if (r < a.rows) {
            const float4 *src = (const float4 *)(a.obs + r * a.obs_stride + 32 * q);
#pragma unroll
            for (int v = 0; v < 8; v++) {
                const float4 o = src[v];
                x[4 * v] = o.x; x[4 * v + 1] = o.y; x[4 * v + 2] = o.z; x[4 * v + 3] = o.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 32; j++) x[j] = 0.f;
        }
    };
    // the first tile's rows in flight under the weight copy
    float xn[32];
    if (tw0 < tiles) load_rows(tw0 * 16, xn);
    policy_weights_to_lds(L.wt, W, tid, (int)blockDim.x);
    __syncthreads();
    pol_trace_wg(a, tw0, 1, true);
    float (*tile)[33] = L.tile[wave];

    for (int64_t tl = tw0; tl < tiles; tl += tstride) {
        const int64_t row0 = tl * 16;
        const bool first = tl == tw0;
        float x[32];
#pragma unroll
        for (int j = 0; j < 32; j++) x[j] = xn[j];
        if (PREFETCH && tl + tstride < tiles) load_rows((tl + tstride) * 16, xn);
        if (a.obs_out) {  // the rollout's record of the observed rows (buffer.obs, ppo.py:129)
            const int64_t r = row0 + c;
            if (r < a.rows) {
                float4 *dst = (float4 *)(a.obs_out + r * POL_IN + 32 * q);
#pragma unroll
                for (int v = 0; v < 8; v++) dst[v] = make_float4(x[4 * v], x[4 * v + 1], x[4 * v + 2], x[4 * v + 3]);
            }
        }
        if (first) pol_trace_wg(a, tw0, 2, true);
        // an offset the compiler cannot see through: the LDS operand reads stay
        // inside the loop instead of being hoisted into 128 live registers
        int z = 0;
        __asm__ volatile("" : "+v"(z));
        const float (*nrm)[POL_IN] = (const float (*)[POL_IN])(&L.wt.norm[0][0] + z);
        const float (*w1l)[32][PWG_P1] = (const float (*)[32][PWG_P1])(&L.wt.w1[0][0][0] + z);
        const float (*w2l)[32][PWG_P2] = (const float (*)[32][PWG_P2])(&L.wt.w2[0][0][0] + z);
        const float (*whl)[32][PWG_P2] = (const float (*)[32][PWG_P2])(&L.wt.wh[0][0][0] + z);
        const float (*cs)[32] = (const float (*)[32])(&L.wt.cst[0][0] + z);
        // layer 1: normalisation, then the two accumulator chains (policy_layers).
        // The LDS operands are read one 4-float group ahead of their use and the
        // groups fenced with scheduling barriers: hoisted all at once they would
        // take 64 more registers (spills at four waves per SIMD).
#pragma unroll
        for (int v = 0; v < 8; v++) {
            const float4 m4 = *(const float4 *)&nrm[0][32 * q + 4 * v];
            const float4 i4 = *(const float4 *)&nrm[1][32 * q + 4 * v];
            x[4 * v] = pol_clamp((x[4 * v] - m4.x) * i4.x);
            x[4 * v + 1] = pol_clamp((x[4 * v + 1] - m4.y) * i4.y);
            x[4 * v + 2] = pol_clamp((x[4 * v + 2] - m4.z) * i4.z);
            x[4 * v + 3] = pol_clamp((x[4 * v + 3] - m4.w) * i4.w);
            if (v & 1) __builtin_amdgcn_sched_barrier(0);
        }
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
        float4 n0 = *(const float4 *)&w1l[q][c][0], n1 = *(const float4 *)&w1l[q][16 + c][0];
#pragma unroll
        for (int v = 0; v < 8; v++) {
            const float w0[4] = {n0.x, n0.y, n0.z, n0.w}, w1[4] = {n1.x, n1.y, n1.z, n1.w};
            if (v + 1 < 8) {
                n0 = *(const float4 *)&w1l[q][c][4 * v + 4];
                n1 = *(const float4 *)&w1l[q][16 + c][4 * v + 4];
            }
#pragma unroll
            for (int e = 0; e < 4; e++) {
                a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[4 * v + e], w0[e], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[4 * v + e], w1[e], a1, 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        ln_relu_to_tile<false>(a0, a1, cs[0][c], cs[0][c + 16], cs[1][c], cs[1][c + 16], cs[2][c], cs[2][c + 16], tile, c, q);
        pol_wave_sync();
        // layer 2, then the heads (k = 8q + j)
#pragma unroll
        for (int layer = 0; layer < 2; layer++) {
            const float (*wl)[32][PWG_P2] = layer == 0 ? w2l : whl;
            float h[8];
#pragma unroll
            for (int j = 0; j < 8; j++) h[j] = tile[c][8 * q + j];
            pol_wave_sync();
            float w0[8], w1[8];
#pragma unroll
            for (int v = 0; v < 2; v++) {
                const float4 u0 = *(const float4 *)&wl[q][c][4 * v];
                const float4 u1 = *(const float4 *)&wl[q][16 + c][4 * v];
                w0[4 * v] = u0.x; w0[4 * v + 1] = u0.y; w0[4 * v + 2] = u0.z; w0[4 * v + 3] = u0.w;
                w1[4 * v] = u1.x; w1[4 * v + 1] = u1.y; w1[4 * v + 2] = u1.z; w1[4 * v + 3] = u1.w;
            }
            a0 = f32x4{0.f, 0.f, 0.f, 0.f};
            a1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 8; j++) {
                a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], w0[j], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], w1[j], a1, 0, 0, 0);
            }
            if (layer == 0) {
                ln_relu_to_tile<false>(a0, a1, cs[3][c], cs[3][c + 16], cs[4][c], cs[4][c + 16], cs[5][c], cs[5][c + 16], tile, c, q);
            } else {
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    tile[4 * q + i][c] = a0[i] + cs[6][c];
                    tile[4 * q + i][c + 16] = a1[i] + cs[6][c + 16];
                }
            }
            pol_wave_sync();
        }
        if (first) pol_trace_wg(a, tw0, 4, false);
        bucket_pass_spread<16, false, STOCH>(a, tile, row0, lane, L.bl[wave]);
        pol_wave_sync();
        if (first) pol_trace_wg(a, tw0, 5, false);
    }
}

// Waves per workgroup and workgroups of a k_policy_wg launch: one workgroup
// per CU (256) once there are 12 tiles per CU, fewer waves per workgroup
// below that so that every CU gets work.
struct PolicyWgGrid {
    int waves;
    unsigned groups;
};
inline PolicyWgGrid policy_wg_grid(int64_t tiles)
{
    constexpr int64_t CUS = 256;
    int64_t w = (tiles + CUS - 1) / CUS;
    w = w < 1 ? 1 : (w > PWG_WAVES ? PWG_WAVES : w);
    int64_t g = (tiles + w - 1) / w;
    g = g > CUS ? CUS : g;
    return {(int)w, (unsigned)g};
}

// M-tiles per wave.  4: 64 rows per wave, one row per lane in the bucket
// pass, each lane's buckets in series; 2: 32 rows, 2 lanes per row; 1: 16
// rows per wave, 4 lanes per row in the bucket pass.  Measured
// (profiles/r03/e_policy_mt_ab.txt, profiles/r04/mt_sweep_rows.txt; sampled,
// us per launch): 16 384 rows MT 1 10.9 / MT 2 12.6 / MT 4 17.5; 24 576
// 14.2 / 13.9 / 19.6; 32 768 16.4 / 15.3 / 19.9; 49 152 24.3 / 27.6 / 22.0;
// 65 536 27.0 / 27.7 / 23.5 -- MT 2 while its waves (276 registers, one per
// SIMD) fit one round, MT 4 above.
#ifndef POLICY_MT2_ROWS
#define POLICY_MT2_ROWS 20480
#endif
#ifndef POLICY_MT4_ROWS
#define POLICY_MT4_ROWS 32769
#endif
inline int policy_mt(int64_t rows)
{
    return rows < POLICY_MT2_ROWS ? 1 : (rows < POLICY_MT4_ROWS ? 2 : 4);
}

template <int MT>
static hipError_t launch_policy_mt(const PolicyArgs &a, hipStream_t s)
{
    const int64_t tiles = (a.rows + 16 * MT - 1) / (16 * MT);
    if (tiles <= 0) return hipSuccess;
    // grid-stride beyond this many waves: 64-row tiles one wave per SIMD
    // (1 024 on the 256 CUs), the next tile's rows loaded under this one's
    // network (131 072 rows: 46.8 -> 43.5 us argmax, 57.1 -> 54.4 sampled;
    // profiles/r03/ah_policy_grid_ab.txt)
    const int64_t cap = MT == 4 ? 1024 : 16384;
    const unsigned grid = (unsigned)(tiles < cap ? tiles : cap);
    hipLaunchKernelGGL(k_policy<MT>, dim3(grid), dim3(64), 0, s, a);
    return hipGetLastError();
}

// k_policy_wg from POLICY_WG_MIN_ROWS rows on: measured (profiles/r03/ap_policy_ab.txt)
// 131 072 rows 43.2 -> 38.4 us argmax, 53.9 -> 49.1 sampled; at 65 536 rows the
// register-weight kernel is ahead (25.3 vs 27.1, 30.3 vs 34.3: its 64-row
// tiles amortise the bucket pass's per-tile exchanges).  DIAG_POLICY_WG = 1 / 0
// forces it on / off (tests).
#ifndef POLICY_WG_MIN_ROWS
#define POLICY_WG_MIN_ROWS 98304
#endif
static bool policy_wg_enabled(int64_t rows)
{
    const int forced = diag_or(DIAG_POLICY_WG, -1);
    return forced >= 0 ? forced == 1 : rows >= POLICY_WG_MIN_ROWS;
}

hipError_t launch_policy(const PolicyArgs &a, hipStream_t s)
{
    if (a.rows <= 0) return hipSuccess;
    switch (a.mt) {  // the caller's choice
    case 1: return launch_policy_mt<1>(a, s);
    case 2: return launch_policy_mt<2>(a, s);
    case 4: return launch_policy_mt<4>(a, s);
    default: break;
    }
    if (policy_wg_enabled(a.rows)) {
        const int64_t tiles = (a.rows + 15) / 16;
        if (tiles <= 0) return hipSuccess;
        const PolicyWgGrid g = policy_wg_grid(tiles);
        // the next tile's rows under this one's network once a wave has two
        const bool pre = tiles > (int64_t)g.groups * g.waves;
        const dim3 grid(g.groups), block(64 * g.waves);
        if (a.stochastic) {
            if (pre) hipLaunchKernelGGL((k_policy_wg<true, 1>), grid, block, 0, s, a);
            else hipLaunchKernelGGL((k_policy_wg<false, 1>), grid, block, 0, s, a);
        } else {
            if (pre) hipLaunchKernelGGL((k_policy_wg<true, 0>), grid, block, 0, s, a);
            else hipLaunchKernelGGL((k_policy_wg<false, 0>), grid, block, 0, s, a);
        }
        return hipGetLastError();
    }
    switch (policy_mt(a.rows)) {
    case 1: return launch_policy_mt<1>(a, s);
    case 2: return launch_policy_mt<2>(a, s);
    default: return launch_policy_mt<4>(a, s);
    }
}

void host_policy(const PolicyArgs &a)
{
    for (int64_t r = 0; r < a.rows; r++) policy_row_host(a, r);
}

}  // namespace bb
