// bb_kernels.hip -- gfx950 kernels of the basketball step.
//
// k_step<N>: one lane = one world.  The lane loads its world's columns
// (16/8-byte vector loads where the per-world chunk allows), runs the 19
// systems of src/game.cpp:1463-1526 on registers (bb_sim.h), and writes the
// columns back; observation rows are written as float4 stores.  Replaces the
// reference's 19 ParallelFor megakernel nodes + 3 sort nodes per step
// (src/game.cpp:1467-1523, src/sim.cpp:99-124) with one launch.
#include <hip/hip_runtime.h>
#include "bb_sim.h"
#include "bb_launch.h"

namespace bb {

constexpr int STEP_BLOCK = 256;

template <int N>
__global__ __launch_bounds__(STEP_BLOCK) void k_step(const Params p)
{
    const int64_t w = (int64_t)blockIdx.x * STEP_BLOCK + threadIdx.x;
    if (w >= p.num_worlds) return;
    step_one_world<N>(p, w);
}

template <int N>
__global__ __launch_bounds__(STEP_BLOCK) void k_init(const Params p)
{
    const int64_t w = (int64_t)blockIdx.x * STEP_BLOCK + threadIdx.x;
    if (w >= p.num_worlds) return;
    init_world<N>(p, w);
}

// one lane = one (world, agent) action row (24 B)
__global__ __launch_bounds__(256) void k_random_actions(int32_t *action, int64_t rows, int32_t n,
                                                        int64_t world_offset, uint32_t seed,
                                                        uint32_t step)
{
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    const int64_t w = r / n;
    const int32_t a = (int32_t)(r - w * n);
    int32_t act[6];
    random_action(seed, step, (uint32_t)(world_offset + w), (uint32_t)a, act);
    int2 *dst = (int2 *)(action + r * 6);
    dst[0] = make_int2(act[0], act[1]);
    dst[1] = make_int2(act[2], act[3]);
    dst[2] = make_int2(act[4], act[5]);
}

struct Poke { int32_t v[8]; };
__global__ void k_poke(int32_t *dst, int32_t count, Poke vals)
{
    const int k = threadIdx.x;
    if (k < count) dst[k] = vals.v[k];
}

static inline dim3 grid_for(int64_t items, int block) { return dim3((unsigned)((items + block - 1) / block)); }

template <int N>
static hipError_t launch_step_n(const Params &p, hipStream_t s)
{
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_step<N>), grid_for(p.num_worlds, STEP_BLOCK), dim3(STEP_BLOCK), 0, s, p);
    return hipGetLastError();
}

template <int N>
static hipError_t launch_init_n(const Params &p, hipStream_t s)
{
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_init<N>), grid_for(p.num_worlds, STEP_BLOCK), dim3(STEP_BLOCK), 0, s, p);
    return hipGetLastError();
}

#define BB_DISPATCH_N(n, fn, ...)                       \
    switch (n) {                                        \
    case 2: return fn<2>(__VA_ARGS__);                  \
    case 4: return fn<4>(__VA_ARGS__);                  \
    case 6: return fn<6>(__VA_ARGS__);                  \
    case 8: return fn<8>(__VA_ARGS__);                  \
    case 10: return fn<10>(__VA_ARGS__);                \
    default: return hipErrorInvalidValue;               \
    }

hipError_t launch_step(int n, const Params &p, hipStream_t s) { BB_DISPATCH_N(n, launch_step_n, p, s) }
hipError_t launch_init(int n, const Params &p, hipStream_t s) { BB_DISPATCH_N(n, launch_init_n, p, s) }

hipError_t launch_random_actions(int n, const Params &p, uint32_t seed, uint32_t step, hipStream_t s)
{
    const int64_t rows = p.num_worlds * n;
    hipLaunchKernelGGL(k_random_actions, grid_for(rows, 256), dim3(256), 0, s, p.c.action, rows, n,
                       p.world_offset, seed, step);
    return hipGetLastError();
}

hipError_t launch_poke(int32_t *dst, int count, const int32_t *vals, hipStream_t s)
{
    Poke pk;
    for (int k = 0; k < 8; k++) pk.v[k] = k < count ? vals[k] : 0;
    hipLaunchKernelGGL(k_poke, dim3(1), dim3(64), 0, s, dst, count, pk);
    return hipGetLastError();
}

}  // namespace bb
