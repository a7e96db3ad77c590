// bb_kernels.hip -- gfx950 step kernel of the basketball simulator; compiled
// once per agent count (-DBB_N=2,4,6,8,10).
//
// k_step<N>: one lane = one world, one wave = one workgroup of 64 worlds.
//   1. the lane loads its world's columns (16/8-byte vector loads where the
//      per-world chunk allows) into a register-resident World<N>;
//   2. systems 1-17 of src/game.cpp:1463-1526 run on registers (bb_sim.h);
//   3. fillObservations (game.cpp:1175-1461): for each agent slot the lane
//      writes its row into an LDS tile (conflict-free ds_write_b128, row
//      stride 4 mod 8 dwords), then the wave stores the 64 rows back as
//      consecutive 16-byte pieces, so every 1 KiB store instruction covers
//      whole 128-byte lines instead of 64 scattered ones;
//   4. rewardSystem, then every modified column is stored.
// Replaces the reference's 19 ParallelFor megakernel nodes + 3 sort nodes per
// step (src/game.cpp:1467-1523, src/sim.cpp:99-124) with one launch.
#include <hip/hip_runtime.h>
#include "bb_launch.h"
#include "bb_sim.h"

#ifndef BB_N
#error "compile bb_kernels.hip with -DBB_N=<agents>"
#endif

namespace bb {

constexpr int WAVE = 64;

template <int N>
struct ObsTile {
    static constexpr int QW = (obs_used(N) + 3) / 4;  // float4 pieces of a used row
    static constexpr int RS = QW * 4 + 4;             // LDS row stride (floats): == 4 mod 8
    // LDS-staged rows only while the tile leaves room for >= 2 waves per CU
    static constexpr bool STAGED = (WAVE * RS * 4) <= 64 * 1024;
    static constexpr int FLOATS = STAGED ? WAVE * RS : 4;
};

template <int N, int MODE>
__global__ __launch_bounds__(WAVE, 2) void k_step(const Params p)
{
    using T = ObsTile<N>;
    __shared__ float4 tile4[T::FLOATS / 4];
    float *tile = (float *)tile4;
    const int lane = threadIdx.x;
    const int64_t w0 = (int64_t)blockIdx.x * WAVE;
    const int64_t w = w0 + lane;
    const bool active = w < p.num_worlds;

    World<N> s;
    Ctx c;
    c.p = &p; c.w = w; c.key_ready = false; c.k0 = c.k1 = 0;
    if (active) {
        load_world(s, p, w);
        if constexpr (MODE != MODE_IO && MODE != MODE_IO_OBS) step_world_pre_obs(s, c);
    }
    if constexpr (MODE == MODE_IO) {
        if (active) store_world(s, p, w);
        return;
    }
    if constexpr (MODE == MODE_DIRECT_OBS || !T::STAGED) {
        if (active) sys_fill_obs(s, c);
    } else if constexpr (MODE != MODE_NO_OBS) {
        constexpr int OW = obs_width(N);
#pragma unroll
        for (int a = 0; a < N; a++) {
            const bool fast = active && canonical_slots(s, a);
            if (fast) fill_obs_fast(s, c, a, tile + lane * T::RS);
            else if (active) fill_obs_slow(s, c, a, p.c.obs + (w * N + a) * (int64_t)OW);
            __syncthreads();
            const uint64_t staged = __ballot(fast);
            float *obs_a = p.c.obs + (w0 * N + a) * (int64_t)OW;
            for (int f = lane; f < WAVE * T::QW; f += WAVE) {
                const int r = f / T::QW, q = f - r * T::QW;
                if ((staged >> r) & 1ull) {
                    const float4 v = *(const float4 *)(tile + r * T::RS + 4 * q);
                    *(float4 *)(obs_a + (int64_t)r * N * OW + 4 * q) = v;
                }
            }
            __syncthreads();
        }
    }
    if (active) {
        if constexpr (MODE != MODE_IO_OBS) sys_reward(s);
        store_world(s, p, w);
    }
}

template <int N>
__global__ __launch_bounds__(256) void k_init(const Params p)
{
    const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (w >= p.num_worlds) return;
    init_world<N>(p, w);
}

template <int N>
hipError_t launch_step_t(const Params &p, int mode, hipStream_t s)
{
    const dim3 grid((unsigned)((p.num_worlds + WAVE - 1) / WAVE)), block(WAVE);
    switch (mode) {
    case MODE_FULL: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step<N, MODE_FULL>), grid, block, 0, s, p); break;
    case MODE_IO: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step<N, MODE_IO>), grid, block, 0, s, p); break;
    case MODE_IO_OBS: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step<N, MODE_IO_OBS>), grid, block, 0, s, p); break;
    case MODE_DIRECT_OBS: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step<N, MODE_DIRECT_OBS>), grid, block, 0, s, p); break;
    case MODE_NO_OBS: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step<N, MODE_NO_OBS>), grid, block, 0, s, p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int N>
hipError_t launch_init_t(const Params &p, hipStream_t s)
{
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_init<N>), dim3((unsigned)((p.num_worlds + 255) / 256)), dim3(256), 0, s, p);
    return hipGetLastError();
}

template hipError_t launch_step_t<BB_N>(const Params &, int, hipStream_t);
template hipError_t launch_init_t<BB_N>(const Params &, hipStream_t);

}  // namespace bb
