// bb_policy.hip -- fused policy inference on gfx950:
// observation rows -> RunningMeanStd -> 2 x (Linear + LayerNorm + ReLU) ->
// actor/critic heads -> per-bucket argmax or Gumbel-max sample, log-prob and
// value, written straight into the simulator's action tensor (bb_policy.h has
// the row math and the reference lines).
//
// One wave per workgroup, 16 rows per tile (grid-stride).  The three matrix
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

__device__ __forceinline__ float quarter_sum(float t)
{
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) t = t + __shfl_xor(t, m, 64);
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
    __shared__ float norm[2][POL_IN];
    __shared__ float tile[16][33];
    const int lane = threadIdx.x, c = lane & 15, q = lane >> 4;
    const PolicyWeights &W = a.w;
    for (int k = lane; k < POL_IN; k += 64) {
        norm[0][k] = W.obs_mean[k];
        norm[1][k] = W.obs_inv[k];
    }
    // B operands for the whole launch
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

    const int64_t tiles = (a.rows + 15) / 16;
    for (int64_t tl = blockIdx.x; tl < tiles; tl += gridDim.x) {
        const int64_t row0 = tl * 16;
        // layer 1 A operand: 32 normalised floats of row row0 + c
        float x[32];
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
#pragma unroll
        for (int j = 0; j < 32; j++) x[j] = pol_clamp((x[j] - norm[0][32 * q + j]) * norm[1][32 * q + j]);
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 32; j++) {
            a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[j], w1[0][j], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x[j], w1[1][j], a1, 0, 0, 0);
        }
        ln_relu_to_tile(a0, a1, b1_0, b1_1, l1w0, l1w1, l1b0, l1b1, tile, c, q);
        __syncthreads();
        // layer 2
        float h[8];
#pragma unroll
        for (int j = 0; j < 8; j++) h[j] = tile[c][8 * q + j];
        __syncthreads();
        a0 = f32x4{0.f, 0.f, 0.f, 0.f};
        a1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 8; j++) {
            a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], w2[0][j], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(h[j], w2[1][j], a1, 0, 0, 0);
        }
        ln_relu_to_tile(a0, a1, b2_0, b2_1, l2w0, l2w1, l2b0, l2b1, tile, c, q);
        __syncthreads();
        // heads
#pragma unroll
        for (int j = 0; j < 8; j++) h[j] = tile[c][8 * q + j];
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
            tile[4 * q + i][c] = a0[i] + bh0;
            tile[4 * q + i][c + 16] = a1[i] + bh1;
        }
        __syncthreads();
        // one lane per row: buckets, log-prob, value
        if (lane < 16 && row0 + lane < a.rows) {
            const int64_t rr = row0 + lane;
            float logit[POL_LOGITS + 1];
#pragma unroll
            for (int i = 0; i <= POL_LOGITS; i++) logit[i] = tile[lane][i];
            int32_t act[6];
            float lp;
            pol_select(logit, a.stochastic != 0, a.seed, a.step, (uint32_t)rr, act, &lp);
            int32_t *d = a.actions + rr * a.act_stride;
#pragma unroll
            for (int b = 0; b < 6; b++) d[b] = act[b];
            if (a.log_prob) a.log_prob[rr] = lp;
            if (a.value) a.value[rr] = logit[POL_LOGITS];
        }
        __syncthreads();
    }
}

hipError_t launch_policy(const PolicyArgs &a, hipStream_t s)
{
    const int64_t tiles = (a.rows + 15) / 16;
    if (tiles <= 0) return hipSuccess;
    const unsigned grid = (unsigned)(tiles < 8192 ? tiles : 8192);  // 8 waves per CU, grid-stride beyond
    hipLaunchKernelGGL(k_policy, dim3(grid), dim3(64), 0, s, a);
    return hipGetLastError();
}

void host_policy(const PolicyArgs &a)
{
    for (int64_t r = 0; r < a.rows; r++) policy_row_host(a, r);
}

}  // namespace bb
