"""Fused PPO rollout timing A/B: events per bb_rollout_policy call with all
buffers vs without one of them (diagnostics: what the recorded outputs and the
kernel's setup / drain cost).

python tools/ppo_ab.py [--worlds 8192] [--steps 32] [--reps 20]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import madrona_basketball_amd as mba
    from madrona_basketball_amd.policy import FusedPolicy, make_agent
    sim = mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, a.worlds, 0,
                                       per_world_rng=True)
    pol = FusedPolicy.from_agent(make_agent(0).cuda())
    full = pol.rollout_buffers(sim, a.steps)
    variants = {"all buffers": full,
                "no obs": {**full, "obs": None},
                "no obs/actions": {**full, "obs": None, "actions": None},
                "nothing recorded": {k: None for k in full}}
    for i in range(3):
        pol.rollout(sim, a.steps, full, seed=1, step0=i * a.steps)
    res = {k: [] for k in variants}
    step0 = 3 * a.steps
    for r in range(a.reps):
        for k, b in variants.items():
            res[k].append(pol.rollout(sim, a.steps, b, seed=1, step0=step0, time_kernels=True) * 1e3)
            step0 += a.steps
    for k, v in res.items():
        print(f"{k:18s} median {statistics.median(v):8.1f} us  min {min(v):8.1f}  per step {statistics.median(v) / a.steps:6.2f}")
    # fixed cost per launch: event time against K (fused PPO rollout and the
    # staged-action k_rollout)
    for K in (1, 2, 4, 8, 16, 32):
        b = pol.rollout_buffers(sim, K)
        v = []
        for r in range(a.reps):
            v.append(pol.rollout(sim, K, b, seed=1, step0=step0, time_kernels=True) * 1e3)
            step0 += K
        acts = sim.stage_random_actions(K * a.reps, action_seed=1, step0=step0)
        rb = sim.rollout_buffers(K)
        u = [sim.rollout(acts[i * K:(i + 1) * K], rb["obs"], rb["reward"], rb["done"], time_kernels=True) * 1e3
             for i in range(a.reps)]
        print(f"K={K:3d}  PPO rollout {statistics.median(v):8.1f} us   k_rollout {statistics.median(u):8.1f} us")


if __name__ == "__main__":
    main()
