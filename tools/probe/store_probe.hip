// Store-stream calibration for the resident loop (k_rollout<2, 2, 1, true>):
// the same per-step store pattern with no systems, to tell which part of the
// loop's 15.3 us per step the written bytes alone cost.  Standalone diagnostic
// (not product code):
//   hipcc --offload-arch=gfx950 -O3 -o store_probe tools/probe/store_probe.hip
//   ./store_probe <worlds> <steps> <rows> <line3> <cols> <valu> <rowaux> <wait>
// rows:  1 = every row's 4 lines (512 B, whole lines), 0 = none
// line3: 0 = store line 3 (floats 96..127) of every row, 1 = of no row,
//        2 = of 2 % of rows (per-lane hash; the measured change rate)
// cols:  0 = no state columns, 1 = every column every step (524 B per world),
//        2 = the rarely-changing columns (236 B per world) in 35 % of waves only
// valu:  per lane per step before the stores, 4 independent FMA chains x valu
//        (4 * valu VALU instructions; 0 = none)
// wait:  1 = s_waitcnt vmcnt(0) after the VALU, before the step's stores (every
//        store of the previous step retired, as a load or spill reload issued
//        after them forces); 2 = the same wait halfway through the VALU
// rowaux: cache-policy bits of the row stores (2 = non-temporal)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef float vf4 __attribute__((ext_vector_type(4)));
typedef uint32_t vu4 __attribute__((ext_vector_type(4)));
constexpr int WAVE = 64;

struct Cols {
    // agent-level columns [W][2][words], world-level [W][words]
    float *ag[15];
    float *wd[7];
};
constexpr int AG_WORDS[15] = {3, 3, 4, 5, 2, 6, 4, 10, 1, 1, 2, 1, 1, 1, 6};
constexpr int AG_RARE[15] = {0, 0, 0, 0, 0, 1, 1, 1, 1, 0, 1, 1, 0, 1, 0};
constexpr int WD_WORDS[7] = {14, 3, 3, 7, 2, 1, 1};
constexpr int WD_RARE[7] = {0, 0, 1, 1, 1, 1, 1};

__device__ __forceinline__ void store_aux(char *base, uint32_t off, vf4 v, int aux)
{
    const uint64_t b = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    char *ub = (char *)(((uint64_t)hi << 32) | lo);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(ub, 0, 0x7fffffff, 0x00020000);
    if (aux == 2) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(vu4, v), rs, (int)off, 0, 2);
    else if (aux == 16) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(vu4, v), rs, (int)off, 0, 16);
    else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(vu4, v), rs, (int)off, 0, 0);
}

template <int WORDS>
__device__ __forceinline__ void store_col(float *col, int64_t idx, float x)
{
    float *p = col + idx * WORDS;
#pragma unroll
    for (int i = 0; i < WORDS; i++) p[i] = x + i;
}
template <int J>
__device__ __forceinline__ void store_ag(const Cols &c, int64_t idx, float x, bool rare)
{
    if constexpr (J < 15) {
        if (!AG_RARE[J] || rare) store_col<AG_WORDS[J]>(c.ag[J], idx, x);
        store_ag<J + 1>(c, idx, x, rare);
    }
}
template <int J>
__device__ __forceinline__ void store_wd(const Cols &c, int64_t idx, float x, bool rare)
{
    if constexpr (J < 7) {
        if (!WD_RARE[J] || rare) store_col<WD_WORDS[J]>(c.wd[J], idx, x);
        store_wd<J + 1>(c, idx, x, rare);
    }
}

__global__ __launch_bounds__(WAVE, 2) void k_probe(float *obs, Cols c, int64_t W, int steps, int rows, int line3,
                                                    int cols, int valu, int rowaux, int wait)
{
    const int lane = threadIdx.x;
    const int64_t w0 = (int64_t)blockIdx.x * 32;
    const int64_t w = w0 + lane / 2;
    const int k = lane & 1;
    if (w0 >= W) return;
    float x = (float)lane * 1e-3f, y = 1.0f, z = 0.25f, u = 0.5f;
    for (int t = 0; t < steps; t++) {
        if (wait == 3) {
            // rows interleaved with the VALU: one row store instruction every valu/32 FMA groups
            char *base = (char *)(obs + w0 * 2 * 128);
            for (int i = 0; i < 32; i++) {
                const vf4 v = {x, y, (float)t, 0.f};
                store_aux(base, (uint32_t)((i * WAVE + lane) * 16), v, rowaux);
#pragma unroll 8
                for (int j = 0; j < valu / 32; j++) {
                    __asm__ volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(x));
                    __asm__ volatile("v_fma_f32 %0, %0, %0, 0.5" : "+v"(y));
                    __asm__ volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(z));
                    __asm__ volatile("v_fma_f32 %0, %0, %0, 0.5" : "+v"(u));
                }
            }
        }
        for (int h = 0; h < 2 && wait != 3; h++) {
            if (wait == 2 && h == 1) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#pragma unroll 16
            for (int i = 0; i < valu / 2; i++) {
                __asm__ volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(x));
                __asm__ volatile("v_fma_f32 %0, %0, %0, 0.5" : "+v"(y));
                __asm__ volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(z));
                __asm__ volatile("v_fma_f32 %0, %0, %0, 0.5" : "+v"(u));
            }
        }
        if (wait == 1) __builtin_amdgcn_s_waitcnt(0x0F70);
        x += z + u;
        const vf4 v = {x, y, (float)t, 0.f};
        if (cols) {
            const bool wave_rare = cols == 1 || ((blockIdx.x * 2654435761u + (uint32_t)t * 40503u) >> 16) % 100 < 35;
            store_ag<0>(c, w * 2 + k, x, wave_rare);
            if (k == 0) store_wd<0>(c, w, y, wave_rare);
        }
        if (rows && wait != 3) {
            // the wave's 64 rows: 2048 pieces of 16 B, 32 store instructions,
            // consecutive lanes on consecutive pieces (1 KB per instruction)
            char *base = (char *)(obs + w0 * 2 * 128);
            const bool my_l3 = line3 == 0 ||
                               (line3 == 2 && ((uint32_t)(w * 2 + k) * 2654435761u + (uint32_t)t * 97u) % 100 < 2);
            const uint64_t l3mask = __ballot(my_l3);
            if (rows == 1) {
#pragma unroll
                for (int i = 0; i < 32; i++) {
                    const int f = i * WAVE + lane, r = f >> 5, q = f & 31;
                    if (q < 24 || ((l3mask >> r) & 1ull)) store_aux(base, (uint32_t)(f * 16), v, rowaux);
                }
            } else {
                // the resident loop's order: pass 0 = lines 0-1 of the 64 rows, pass 1 = lines 2-3
                // (16 pieces of 4 rows per instruction)
#pragma unroll
                for (int ps = 0; ps < 2; ps++) {
                    if (rows == 3 && ps == 1) __builtin_amdgcn_s_sleep(8);
#pragma unroll
                    for (int i = 0; i < 16; i++) {
                        const int r = i * 4 + (lane >> 4), q = 16 * ps + (lane & 15);
                        if (q < 24 || ((l3mask >> r) & 1ull)) store_aux(base, (uint32_t)((r * 32 + q) * 16), v, rowaux);
                    }
                }
            }
        }
    }
    if (x == 12345.f) obs[0] = y;
}

int main(int argc, char **argv)
{
    const int64_t W = argc > 1 ? atoll(argv[1]) : 65536;
    const int steps = argc > 2 ? atoi(argv[2]) : 200;
    const int rows = argc > 3 ? atoi(argv[3]) : 1;
    const int line3 = argc > 4 ? atoi(argv[4]) : 0;
    const int cols = argc > 5 ? atoi(argv[5]) : 1;
    const int valu = argc > 6 ? atoi(argv[6]) : 0;
    const int rowaux = argc > 7 ? atoi(argv[7]) : 2;
    const int wait = argc > 8 ? atoi(argv[8]) : 0;
    const int agw[15] = {3, 3, 4, 5, 2, 6, 4, 10, 1, 1, 2, 1, 1, 1, 6};
    const int wdw[7] = {14, 3, 3, 7, 2, 1, 1};
    float *obs;
    Cols c;
    hipMalloc(&obs, W * 2 * 128 * 4);
    hipMemset(obs, 0, W * 2 * 128 * 4);
    for (int j = 0; j < 15; j++) hipMalloc(&c.ag[j], W * 2 * agw[j] * 4);
    for (int j = 0; j < 7; j++) hipMalloc(&c.wd[j], W * wdw[j] * 4);
    const int grid = (int)((W + 31) / 32);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_probe, dim3(grid), dim3(WAVE), 0, 0, obs, c, W, 10, rows, line3, cols, valu, rowaux, wait);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_probe, dim3(grid), dim3(WAVE), 0, 0, obs, c, W, steps, rows, line3, cols, valu, rowaux, wait);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double us = best * 1e3 / steps;
    double bytes = 0;
    if (rows) bytes += W * 2.0 * (384 + (line3 == 0 ? 128 : line3 == 2 ? 128 * 0.02 : 0));
    if (cols) bytes += W * (cols == 1 ? 524.0 : 288.0 + 0.35 * 236.0);
    printf("worlds %lld rows %d line3 %d cols %d valu %d aux %d wait %d: %.2f us/step, %.1f MB/step, %.0f GB/s\n",
           (long long)W, rows, line3, cols, valu, rowaux, wait, us, bytes / 1e6, bytes / us / 1e3);
    return hipGetLastError() != hipSuccess;
}
