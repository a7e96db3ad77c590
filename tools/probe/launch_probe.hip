// Per-launch overhead of a kernel that uses scratch (private segment) vs one
// that does not: the same short loop, 256 workgroups of 320 threads and
// 47 KB of LDS (the PPO rollout's launch shape), launched back to back.
// Standalone diagnostic: hipcc --offload-arch=gfx950 -O3 -o launch_probe launch_probe.hip
//   ./launch_probe <iters per launch> <launches>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <bool SCRATCH>
__global__ __launch_bounds__(320, 1) void k_probe(float *out, int iters, int idx)
{
    __shared__ float lds[11 * 1024];
    float acc = threadIdx.x;
    if constexpr (SCRATCH) {
        // the private array is touched only when iters > 0: at iters = 0 the
        // launch carries a scratch allocation and no scratch traffic
        volatile float priv[40];
        for (int i = 0; i < iters && i < 40; i++) priv[i] = acc + i;
        for (int i = 0; i < iters; i++) acc = acc * 0.999f + priv[(i + idx) % 40];
    } else {
        for (int i = 0; i < iters; i++) acc = acc * 0.999f + (float)((i + idx) % 40);
    }
    lds[threadIdx.x] = acc;
    __syncthreads();
    if (acc == 1234.5f) out[blockIdx.x] = lds[(threadIdx.x + 1) % 320];
}

template <bool S>
static float run(float *out, int iters, int launches)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_probe<S>, dim3(256), dim3(320), 0, 0, out, iters, 3);
    hipDeviceSynchronize();
    float total = 0.f;
    for (int l = 0; l < launches; l++) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_probe<S>, dim3(256), dim3(320), 0, 0, out, iters, l);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        total += ms;
    }
    return total * 1e3f / launches;
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 1000;
    const int launches = argc > 2 ? atoi(argv[2]) : 50;
    float *out;
    hipMalloc(&out, 4096);
    for (int rep = 0; rep < 2; rep++) {
        const float a = run<false>(out, iters, launches), b = run<true>(out, iters, launches);
        printf("iters %d: no scratch %.1f us per launch, scratch %.1f us per launch\n", iters, a, b);
    }
    return 0;
}
