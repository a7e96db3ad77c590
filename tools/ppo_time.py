"""PPO rollout (bb_rollout_policy) time per step with different sets of the
buffer records (scripts/ppo.py:129-134) turned off -- which records cost what.

python tools/ppo_time.py [--worlds 65536] [--rollouts 6]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=65536)
    ap.add_argument("--rollouts", type=int, default=6)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--host", action="store_true", help="also time the host's enqueue of one rollout")
    a = ap.parse_args()
    import madrona_basketball_amd as mba
    from madrona_basketball_amd.policy import FusedPolicy, make_agent
    sim = mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, a.worlds, 0,
                                       per_world_rng=True)
    pol = FusedPolicy.from_agent(make_agent(0).cuda())
    full = pol.rollout_buffers(sim, a.k)
    sets = {"all records": full,
            "no obs": {k: (None if k == "obs" else v) for k, v in full.items()},
            "no obs/actions": {k: (None if k in ("obs", "actions") else v) for k, v in full.items()},
            "value + next_value only": {"value": full["value"], "next_value": full["next_value"]}}
    for name, bufs in sets.items():
        for per_step in (False, True):
            pol.rollout(sim, a.k, bufs, seed=1, step0=0, per_step=per_step)
            torch.cuda.synchronize()
            ms = sum(pol.rollout(sim, a.k, bufs, seed=1, step0=(i + 1) * a.k, per_step=per_step, time_kernels=True)
                     for i in range(a.rollouts)) / a.rollouts
            print(f"{name:26s} per_step={int(per_step)}  {ms * 1e3 / a.k:8.2f} us/step", flush=True)
            if a.host:  # host time to enqueue one rollout (the call returns once its launches are queued)
                t0 = time.perf_counter()
                pol.rollout(sim, a.k, bufs, seed=1, step0=99 * a.k, per_step=per_step)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                print(f"{name:26s} per_step={int(per_step)}  host enqueue {(t1 - t0) * 1e6 / a.k:8.2f} us/step, "
                      f"enqueue + drain {(t2 - t0) * 1e6 / a.k:8.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
