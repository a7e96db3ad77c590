// bb_kernels.hip -- gfx950 step kernel of the basketball simulator; compiled
// once per agent count (-DBB_N=2,4,6,8,10).
//
// k_step<N>: one wave = one 64-lane workgroup; at N = 2 and 4 one lane per
// agent (64/N worlds per wave), otherwise one lane per world.
//   1. every lane loads its world's columns (16/8-byte vector loads where the
//      per-world chunk allows) into a register-resident World<N>;
//   2. systems 1-17 of src/game.cpp:1463-1526 run on registers (bb_sim.h),
//      identically in the N lanes of a world;
//   3. fillObservations (game.cpp:1175-1461): each lane writes its agent's
//      row into an LDS tile (conflict-free ds_write_b128, row stride 4 mod 8
//      dwords); the wave then stores the 64 rows -- consecutive in memory --
//      as consecutive 16-byte pieces (whole 128-byte lines per instruction
//      instead of 64 scattered ones);
//   4. rewardSystem for the lane's agent, then the lane stores its agent's
//      columns and the agent-0 lane the world columns.
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

// Lanes per world: with one lane per agent (N = 2, 4) the lanes of a world
// all hold the full world state and run systems 1-17 identically, but each
// computes and stores only its own agent's observation row, reward and
// per-agent columns; the world-level columns are stored by the agent-0 lane.
#ifndef BB_AGENT_LANES
#define BB_AGENT_LANES 0  // measured slower at N=2 (duplicated systems, LDS-limited residency)
#endif
template <int N>
struct Lanes {
    static constexpr int LPW = (BB_AGENT_LANES && (N == 2 || N == 4)) ? N : 1;
    static constexpr int WPB = WAVE / LPW;  // worlds per 64-lane workgroup
};

// Copy the wave's 64 staged rows (tile row r -> obs row base_row + r*stride)
// as consecutive 16-byte pieces; rows whose bit is clear in `staged` were
// written directly (generic layout) or belong to no world.
template <int N>
__device__ __forceinline__ void flush_tile(const float *tile, float *obs, int64_t row0, int64_t row_stride,
                                           uint64_t staged, int lane)
{
    using T = ObsTile<N>;
    constexpr int OW = obs_width(N);
    for (int f = lane; f < WAVE * T::QW; f += WAVE) {
        const int r = f / T::QW, q = f - r * T::QW;
        if ((staged >> r) & 1ull) {
            const float4 v = *(const float4 *)(tile + r * T::RS + 4 * q);
            *(float4 *)(obs + (row0 + (int64_t)r * row_stride) * OW + 4 * q) = v;
        }
    }
}

template <int N, int MODE>
__global__ __launch_bounds__(WAVE, 2) void k_step(const Params p)
{
    using T = ObsTile<N>;
    constexpr int LPW = Lanes<N>::LPW, WPB = Lanes<N>::WPB;
    constexpr int OW = obs_width(N);
    __shared__ float4 tile4[T::FLOATS / 4];
    float *tile = (float *)tile4;
    const int lane = threadIdx.x;
    const int k = lane % LPW;  // this lane's agent when LPW == N
    const int64_t w0 = (int64_t)blockIdx.x * WPB;
    const int64_t w = w0 + lane / LPW;
    const bool active = w < p.num_worlds;

    World<N> s;
    Ctx c = make_ctx(p, w, k == 0);
    if (active) {
        load_world(s, p, w);
        if constexpr (MODE == MODE_SKIP) step_world_pre_obs_diag(s, c, p.diag_skip);
        else if constexpr (MODE != MODE_IO && MODE != MODE_IO_OBS) step_world_pre_obs(s, c);
    }
    // ---------------------------------------------------------- observations
    // view of the world with this lane's agent in slot 0 (LPW == N)
    World<N> v;
    int32_t ib = -1;
    if constexpr (LPW == N) {
        if (active) {
            ib = inbounder_id(s);
            agent_view(s, v, k);
        }
    }
    if constexpr (LPW != N && (MODE == MODE_IO || MODE == MODE_NO_OBS)) {
        if (active) {
            if constexpr (MODE == MODE_NO_OBS) sys_reward(s);
            store_world(s, p, w);
        }
        return;
    } else if constexpr (MODE == MODE_IO || MODE == MODE_NO_OBS) {
    } else if constexpr (LPW == N) {
        float *grow = p.c.obs + (w * N + k) * (int64_t)OW;
        if constexpr (MODE == MODE_DIRECT_OBS || !T::STAGED) {
            if (active) {
                if (canonical_slots(v, 0)) fill_obs_fast(v, c, 0, grow, ib);
                else fill_obs_slow(v, c, 0, grow, ib);
            }
        } else {
            const bool fast = active && canonical_slots(v, 0);
            if (fast) fill_obs_fast(v, c, 0, tile + lane * T::RS, ib);
            else if (active) fill_obs_slow(v, c, 0, grow, ib);
            __syncthreads();
            // lane = (w - w0) * N + k: the wave's rows are consecutive in memory
            flush_tile<N>(tile, p.c.obs, w0 * N, 1, __ballot(fast), lane);
        }
    } else {
        // one lane per world: reward + state columns first, so their stores
        // drain while the observation rows are built
        if (active) {
            if constexpr (MODE != MODE_IO_OBS) sys_reward(s);
            store_world(s, p, w);
        }
        if constexpr (MODE == MODE_DIRECT_OBS || !T::STAGED) {
            if (active) sys_fill_obs(s, c);
        } else {
            const int32_t ib1 = active ? inbounder_id(s) : -1;
            const bool share = active && obs_sharable(s);
            SharedObs<N> sh;
            if (share) shared_obs_prepare(s, c, sh);
#pragma unroll
            for (int a = 0; a < N; a++) {
                float *trow = tile + lane * T::RS;
                const bool fast = active && (share || canonical_slots(s, a));
                if (share) {
                    RowSink o;
                    o.row = trow; o.idx = 0; o.b0 = o.b1 = o.b2 = o.b3 = 0.f;
                    emit_row_shared(s, c, sh, a, o, ib1);
                } else if (fast) {
                    fill_obs_fast(s, c, a, trow, ib1);
                } else if (active) {
                    fill_obs_slow(s, c, a, p.c.obs + (w * N + a) * (int64_t)OW, ib1);
                }
                __syncthreads();
                flush_tile<N>(tile, p.c.obs, w0 * N + a, N, __ballot(fast), lane);
                __syncthreads();
            }
        }
        return;
    }
    // ---------------------------------------------------------- reward + store
    if (!active) return;
    if constexpr (LPW == N) {
        if constexpr (MODE != MODE_IO && MODE != MODE_IO_OBS) sys_reward_agent(v, 0, AGENT0_ID + k);
        store_world_agent(v, p, w * N + k, 0);
        if (k == 0) store_world_shared(s, p, w);
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
    constexpr int WPB = Lanes<N>::WPB;
    const dim3 grid((unsigned)((p.num_worlds + WPB - 1) / WPB)), block(WAVE);
    switch (mode) {
    case MODE_FULL: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step<N, MODE_FULL>), grid, block, 0, s, p); break;
    case MODE_IO: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step<N, MODE_IO>), grid, block, 0, s, p); break;
    case MODE_IO_OBS: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step<N, MODE_IO_OBS>), grid, block, 0, s, p); break;
    case MODE_DIRECT_OBS: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step<N, MODE_DIRECT_OBS>), grid, block, 0, s, p); break;
    case MODE_NO_OBS: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step<N, MODE_NO_OBS>), grid, block, 0, s, p); break;
    case MODE_SKIP: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step<N, MODE_SKIP>), grid, block, 0, s, p); break;
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
