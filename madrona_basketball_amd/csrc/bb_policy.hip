// bb_policy.hip -- fused policy inference on gfx950:
// observation rows -> RunningMeanStd -> 2 x (Linear + LayerNorm + ReLU) ->
// actor/critic heads -> per-bucket argmax or Gumbel-max sample, log-prob and
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
#include <cstdlib>
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
            pol_select(logit, a.stochastic != 0, a.seed, a.step, (uint32_t)rr, act, &lp);
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

// M-tiles per wave.  4: 64 rows per wave, one row per lane in the bucket
// pass, each lane's 19 Gumbel draws in series; 1: 16 rows per wave, 4 lanes
// per row in the bucket pass.  Measured (profiles/r03/e_policy_mt_ab.txt):
// 8 192 rows 18.1 (MT 4) -> 13.9-18.6 us (MT 1), 65 536 rows 24.8 (MT 4) vs
// 28.8 us (MT 1): MT = 1 below POLICY_MT4_ROWS rows.  MADRONA_BB_POLICY_MT
// forces one (A/B timing).
#ifndef POLICY_MT4_ROWS
#define POLICY_MT4_ROWS 32768
#endif
inline int policy_mt(int64_t rows)
{
    static const int forced = [] {
        const char *e = getenv("MADRONA_BB_POLICY_MT");
        const int m = e && *e ? atoi(e) : 0;
        return (m == 1 || m == 2 || m == 4) ? m : 0;
    }();
    if (forced) return forced;
    return rows < POLICY_MT4_ROWS ? 1 : 4;
}

template <int MT>
static hipError_t launch_policy_mt(const PolicyArgs &a, hipStream_t s)
{
    const int64_t tiles = (a.rows + 16 * MT - 1) / (16 * MT);
    if (tiles <= 0) return hipSuccess;
    // grid-stride beyond this many waves: 64-row tiles one wave per SIMD
    // (1 024 on the 256 CUs), the next tile's rows loaded under this one's
    // network (131 072 rows: 46.8 -> 43.5 us argmax, 57.1 -> 54.4 sampled;
    // profiles/r03/ah_policy_grid_ab.txt); MADRONA_BB_POLICY_GRID overrides
    static const int64_t forced = [] {
        const char *e = getenv("MADRONA_BB_POLICY_GRID");
        const long g = e && *e ? atol(e) : 0;
        return (int64_t)(g > 0 ? g : 0);
    }();
    const int64_t cap = forced ? forced : (MT == 4 ? 1024 : 16384);
    const unsigned grid = (unsigned)(tiles < cap ? tiles : cap);
    hipLaunchKernelGGL(k_policy<MT>, dim3(grid), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_policy(const PolicyArgs &a, hipStream_t s)
{
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
