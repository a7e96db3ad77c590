// Static instruction cost of each system of the step (diagnostics): one
// kernel per system = load world + tick + actionMask + that system + store
// world; the VALU count of each kernel minus the kernel without a system
// estimates the system's cost (static: every branch counted once).  hipcc -S -DBB_N=2 tools/probe/sys_cost.hip, then tools/sys_cost.py.
#include <hip/hip_runtime.h>
#include "../../madrona_basketball_amd/csrc/bb_sim.h"

namespace bb {
#define BB_SYS_KERNEL(name, stmt)                                          \
    __global__ __launch_bounds__(64) void k_##name(const Params p)         \
    {                                                                      \
        const int64_t w = (int64_t)blockIdx.x * 64 + threadIdx.x;          \
        if (w >= p.num_worlds) return;                                     \
        constexpr int N = BB_N;                                            \
        World<N> s;                                                        \
        Ctx c = make_ctx(p, w, true);                                      \
        load_world(s, p, w);                                               \
        sys_tick(s);                                                       \
        sys_action_mask(s, p.flags);                                       \
        { stmt; }                                                          \
        store_world(s, p, w);                                              \
    }
BB_SYS_KERNEL(none, (void)c)
BB_SYS_KERNEL(move, sys_move_agents(s, c, EachAgent()))
BB_SYS_KERNEL(grab, for (int i = 0; i < N; i++) sys_grab(s, c, i))
BB_SYS_KERNEL(pass, for (int i = 0; i < N; i++) sys_pass(s, i))
BB_SYS_KERNEL(shoot, sys_shoot(s, c, EachAgent()))
BB_SYS_KERNEL(move_ball, sys_move_ball(s, c))
BB_SYS_KERNEL(shot_pct, sys_shot_percentage(s, c, EachAgent()))
BB_SYS_KERNEL(score, sys_score(s, c, 0); sys_score(s, c, 1))
BB_SYS_KERNEL(oob, sys_out_of_bounds(s, c))
BB_SYS_KERNEL(last_touch, sys_last_touch(s, c))
BB_SYS_KERNEL(clock, sys_clock(s))
BB_SYS_KERNEL(inbound_violation, sys_inbound_violation(s, c))
BB_SYS_KERNEL(reset, if (s.reset_now != 0) { reset_world(s, c); s.reset_now = 0; })
BB_SYS_KERNEL(points_worth, sys_points_worth(s, c, EachAgent()))
BB_SYS_KERNEL(collisions, sys_collisions(s))
BB_SYS_KERNEL(defense, sys_defense(s, c, EachAgent()))
BB_SYS_KERNEL(reward, sys_reward(s))
BB_SYS_KERNEL(all, step_world_pre_obs(s, c, EachAgent(), 6u); sys_reward(s))  // tick + mask not repeated
}  // namespace bb
