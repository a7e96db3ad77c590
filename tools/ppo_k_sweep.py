"""PPO rollout (bb_rollout_policy) time per call against its length K: the
per-call intercept (launch, setup, next-value pass, tail) and the per-step
slope, from back-to-back calls (wall) and per-call events.

python tools/ppo_k_sweep.py [--worlds 8192] [--ks 1,2,4,8,16,32,64] [--calls 20]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=8192)
    ap.add_argument("--ks", default="1,2,4,8,16,32,64")
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--pw", type=int, default=-1, help="k_rollout_policy's policy waves (2 or 4; -1 the rule)")
    a = ap.parse_args()
    import madrona_basketball_amd as mba
    from madrona_basketball_amd import _lib
    from madrona_basketball_amd.policy import FusedPolicy, make_agent
    if a.pw > 0:
        _lib.diag_set("ppo_pwaves", a.pw)
    sim = mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, a.worlds, 0,
                                       per_world_rng=True)
    pol = FusedPolicy.from_agent(make_agent(0).cuda())
    pts = []
    step0 = 0
    for k in [int(x) for x in a.ks.split(",")]:
        bufs = pol.rollout_buffers(sim, k)
        for _ in range(3):
            pol.rollout(sim, k, bufs, seed=1, step0=step0)
            step0 += k
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.calls):
            pol.rollout(sim, k, bufs, seed=1, step0=step0)
            step0 += k
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.calls * 1e6
        ev = 0.0
        for _ in range(a.calls):
            ev += pol.rollout(sim, k, bufs, seed=1, step0=step0, time_kernels=True) * 1e3
            step0 += k
        ev /= a.calls
        pts.append((k, wall, ev))
        print(f"worlds {a.worlds} pw {a.pw} K {k:3d}: wall {wall:9.1f} us per call ({wall / k:7.2f} per step), "
              f"events {ev:9.1f} us ({ev / k:7.2f} per step)", flush=True)
        del bufs
    n = len(pts)
    for col, name in ((1, "wall"), (2, "events")):
        mx = sum(p[0] for p in pts) / n
        my = sum(p[col] for p in pts) / n
        sl = sum((p[0] - mx) * (p[col] - my) for p in pts) / sum((p[0] - mx) ** 2 for p in pts)
        print(f"{name}: {my - sl * mx:.1f} us per call + {sl:.2f} us per step")


if __name__ == "__main__":
    main()
