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
#include "bb_launch.h"
#include "bb_policy.h"

namespace bb {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 16-row MFMA blocks per tile: 4 -> 64 rows per wave pass, one row per lane in the bucket pass
// (measured 25.2 us for 65 536 argmax rows vs 29.9 at 2 blocks and 2 waves per SIMD)
#ifndef POLICY_MT
#define POLICY_MT 4
#endif

// Sum over the 16 lanes of a DPP row, the same tree as bb_policy.h pol_sum32's
// xor butterfly (partners 1, 2, then the other quad / half: once a quad holds
// equal values any cross-quad partner gives the same bits): four DPP adds.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float quarter_sum(float t)
{
    t = t + dpp_f<0xB1>(t);   // quad_perm [1,0,3,2]: xor 1
    t = t + dpp_f<0x4E>(t);   // quad_perm [2,3,0,1]: xor 2
    t = t + dpp_f<0x141>(t);  // row_half_mirror: the other quad of the 8
    t = t + dpp_f<0x140>(t);  // row_mirror: the other 8 of the 16
    return t;
}

// LayerNorm + ReLU of the 4 rows a lane holds (cols c and c + 16), then the
// result into the LDS tile [row][col].
__device__ __forceinline__ void ln_relu_to_tile(f32x4 a0, f32x4 a1, float bias0, float bias1, float w0, float w1,
                                                float lb0, float lb1, float (*tile)[33], int c, int q)
{
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

__global__ __launch_bounds__(64) void k_policy(const PolicyArgs a)
{
    constexpr int MT = POLICY_MT;  // 16-row M-tiles per tile
    __shared__ __attribute__((aligned(16))) float norm[2][POL_IN];
    __shared__ float tile[16 * MT][33];
    const int lane = threadIdx.x, c = lane & 15, q = lane >> 4;
    const PolicyWeights &W = a.w;
    for (int k = lane; k < POL_IN; k += 64) {
        norm[0][k] = W.obs_mean[k];
        norm[1][k] = W.obs_inv[k];
    }
    // B operands, loaded once per (persistent) wave
    float w1[2][32], w2[2][8], wh[2][8];
#pragma unroll
    for (int t = 0; t < 2; t++) {
        const float4 *src = (const float4 *)(W.w1 + (16 * t + c) * POL_IN + 32 * q);
#pragma unroll
        for (int v = 0; v < 8; v++) {
            const float4 x = src[v];
            w1[t][4 * v] = x.x; w1[t][4 * v + 1] = x.y; w1[t][4 * v + 2] = x.z; w1[t][4 * v + 3] = x.w;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            w2[t][j] = W.w2[(16 * t + c) * POL_HID + 8 * q + j];
            wh[t][j] = W.head_w[(16 * t + c) * POL_HID + 8 * q + j];
        }
    }
    const float b1_0 = W.b1[c], b1_1 = W.b1[c + 16], l1w0 = W.ln1_w[c], l1w1 = W.ln1_w[c + 16];
    const float l1b0 = W.ln1_b[c], l1b1 = W.ln1_b[c + 16];
    const float b2_0 = W.b2[c], b2_1 = W.b2[c + 16], l2w0 = W.ln2_w[c], l2w1 = W.ln2_w[c + 16];
    const float l2b0 = W.ln2_b[c], l2b1 = W.ln2_b[c + 16];
    const float bh0 = W.head_b[c], bh1 = W.head_b[c + 16];
    __syncthreads();

    const int64_t tiles = (a.rows + 16 * MT - 1) / (16 * MT);
    for (int64_t tl = blockIdx.x; tl < tiles; tl += gridDim.x) {
        const int64_t row0 = tl * 16 * MT;
        // every M-tile's 32 observation floats per lane, loads issued together
        float x[MT][32];
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
                if (a.obs_out) {  // the rollout's record of the observed row (buffer.obs, ppo.py:129)
                    float4 *dst = (float4 *)(a.obs_out + r * POL_IN + 32 * q);
#pragma unroll
                    for (int v = 0; v < 8; v++)
                        dst[v] = make_float4(x[m][4 * v], x[m][4 * v + 1], x[m][4 * v + 2], x[m][4 * v + 3]);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 32; j++) x[m][j] = 0.f;
            }
        }
        // layer 1 (two independent accumulators per M-tile keep the MFMA pipe full)
        float nm[32], ni[32];
#pragma unroll
        for (int v = 0; v < 8; v++) {
            const float4 a4 = *(const float4 *)&norm[0][32 * q + 4 * v];
            const float4 b4 = *(const float4 *)&norm[1][32 * q + 4 * v];
            nm[4 * v] = a4.x; nm[4 * v + 1] = a4.y; nm[4 * v + 2] = a4.z; nm[4 * v + 3] = a4.w;
            ni[4 * v] = b4.x; ni[4 * v + 1] = b4.y; ni[4 * v + 2] = b4.z; ni[4 * v + 3] = b4.w;
        }
#pragma unroll
        for (int m = 0; m < MT; m++) {
            // the VALU normalisation as one block, then the MFMA chain back to back
            // (interleaved, every MFMA waits out a VALU-write hazard)
#pragma unroll
            for (int j = 0; j < 32; j++) x[m][j] = pol_clamp((x[m][j] - nm[j]) * ni[j]);
            __builtin_amdgcn_sched_barrier(0);
            f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 32; j++) {
                a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[m][j], w1[0][j], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[m][j], w1[1][j], a1, 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            ln_relu_to_tile(a0, a1, b1_0, b1_1, l1w0, l1w1, l1b0, l1b1, tile + 16 * m, c, q);
        }
        __syncthreads();
        // layer 2 and heads, per M-tile through its 16 rows of the tile
#pragma unroll
        for (int m = 0; m < MT; m++) {
            float (*tm)[33] = tile + 16 * m;
            float h[8];
#pragma unroll
            for (int j = 0; j < 8; j++) h[j] = tm[c][8 * q + j];
            __syncthreads();
            f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 8; j++) {
                a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], w2[0][j], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], w2[1][j], a1, 0, 0, 0);
            }
            ln_relu_to_tile(a0, a1, b2_0, b2_1, l2w0, l2w1, l2b0, l2b1, tm, c, q);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 8; j++) h[j] = tm[c][8 * q + j];
            __syncthreads();
            a0 = f32x4{0.f, 0.f, 0.f, 0.f};
            a1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 8; j++) {
                a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], wh[0][j], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], wh[1][j], a1, 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                tm[4 * q + i][c] = a0[i] + bh0;
                tm[4 * q + i][c + 16] = a1[i] + bh1;
            }
        }
        __syncthreads();
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
        __syncthreads();
    }
}

hipError_t launch_policy(const PolicyArgs &a, hipStream_t s)
{
    const int64_t tiles = (a.rows + 16 * POLICY_MT - 1) / (16 * POLICY_MT);
    if (tiles <= 0) return hipSuccess;
    const unsigned grid = (unsigned)(tiles < 4096 ? tiles : 4096);  // grid-stride beyond
    hipLaunchKernelGGL(k_policy, dim3(grid), dim3(64), 0, s, a);
    return hipGetLastError();
}

void host_policy(const PolicyArgs &a)
{
    for (int64_t r = 0; r < a.rows; r++) policy_row_host(a, r);
}

}  // namespace bb
