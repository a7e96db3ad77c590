// bb_launch.h -- host-side entry points into the gfx950 kernels (bb_kernels.hip)
// and the host executor (bb_host.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "bb_sim.h"

namespace bb {

hipError_t launch_step(int n, const Params &p, hipStream_t s);
hipError_t launch_init(int n, const Params &p, hipStream_t s);
hipError_t launch_random_actions(int n, const Params &p, uint32_t seed, uint32_t step, hipStream_t s);
hipError_t launch_poke(int32_t *dst, int count, const int32_t *vals, hipStream_t s);

// Host executor (ExecMode.CPU): the same step_one_world<N> over a thread pool.
int host_step(int n, const Params &p, int threads);
int host_init(int n, const Params &p);
int host_random_actions(int n, const Params &p, uint32_t seed, uint32_t step);

}  // namespace bb
