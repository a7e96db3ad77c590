// bb_rng.h -- counter-based RNG of the basketball step (host + device).
//
// The reference's per-world Sim::rng (src/sim.cpp:89, madrona::RNG) lives in
// the un-vendored Madrona engine, so its bit stream is not reproducible here.
// This build defines it as threefry2x32-20 (Salmon et al., SC'11; the
// Random123 / JAX known-answer vectors are checked in tests/test_oracle.py):
//
//   world key   = {seed, k}, k = 0 for every world (reference-compatible:
//                 every world's rng is split_i(initKey(0), 0, 0)), or k = the
//                 global world index with BB_FLAG_PER_WORLD_RNG;
//   draw j      = threefry(world key, ctr = {j, 0}).x;  U = (draw >> 8) * 2^-24.
//
// sampleUniform(min, max) = min + (max - min) * U  (src/helper.cpp:8-11).
#pragma once
#include <stdint.h>
#include "bb_math.h"

namespace bb {

BB_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

BB_HD void threefry2x32(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1,
                        uint32_t *o0, uint32_t *o1)
{
    const uint32_t k2 = 0x1BD11BDAu ^ k0 ^ k1;
    uint32_t x0 = c0 + k0, x1 = c1 + k1;
#define BB_TF_ROUND(r) x0 += x1; x1 = rotl32(x1, r); x1 ^= x0;
#define BB_TF_INJECT(a, b, s) x0 += (a); x1 += (b) + (s);
    BB_TF_ROUND(13) BB_TF_ROUND(15) BB_TF_ROUND(26) BB_TF_ROUND(6)  BB_TF_INJECT(k1, k2, 1u)
    BB_TF_ROUND(17) BB_TF_ROUND(29) BB_TF_ROUND(16) BB_TF_ROUND(24) BB_TF_INJECT(k2, k0, 2u)
    BB_TF_ROUND(13) BB_TF_ROUND(15) BB_TF_ROUND(26) BB_TF_ROUND(6)  BB_TF_INJECT(k0, k1, 3u)
    BB_TF_ROUND(17) BB_TF_ROUND(29) BB_TF_ROUND(16) BB_TF_ROUND(24) BB_TF_INJECT(k1, k2, 4u)
    BB_TF_ROUND(13) BB_TF_ROUND(15) BB_TF_ROUND(26) BB_TF_ROUND(6)  BB_TF_INJECT(k2, k0, 5u)
#undef BB_TF_ROUND
#undef BB_TF_INJECT
    *o0 = x0; *o1 = x1;
}

BB_HD float u01_from_bits(uint32_t bits) { return (float)(bits >> 8) * (1.0f / 16777216.0f); }

// Synthetic action workload (bench + tests): buckets [2, 8, 3, 2, 2, 2] of
// scripts/env.py:102 from one threefry draw keyed {seed, step}, ctr {world, agent}.
BB_HD void random_action(uint32_t seed, uint32_t step, uint32_t world, uint32_t agent,
                         int32_t act[6])
{
    uint32_t r0, r1;
    threefry2x32(seed, step, world, agent, &r0, &r1);
    act[0] = (int32_t)(r0 & 1u);
    act[1] = (int32_t)((r0 >> 1) & 7u);
    act[2] = (int32_t)(((r0 >> 4) & 0xFFFFu) % 3u);
    act[3] = (int32_t)((r0 >> 20) & 1u);
    act[4] = (int32_t)((r0 >> 21) & 1u);
    act[5] = (int32_t)((r0 >> 22) & 1u);
}

}  // namespace bb
