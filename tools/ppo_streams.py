"""Does PPO's per-step path gain from two concurrent world halves?  One
65 536-world simulator on one stream (policy launch + step launch per step)
against two 32 768-world simulators on two streams (same launches each).

python tools/ppo_streams.py [--worlds 65536] [--steps 64]
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
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import madrona_basketball_amd as mba
    from madrona_basketball_amd.policy import FusedPolicy, make_agent
    mk = lambda W, off: mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, W, 0,
                                                     per_world_rng=True, world_offset=off)
    pol = FusedPolicy.from_agent(make_agent(0).cuda())
    one = mk(a.worlds, 0)
    h = a.worlds // 2
    halves = [mk(h, 0), mk(a.worlds - h, h)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def run_one():
        for t in range(a.steps):
            pol.act(one, 0, stochastic=True, seed=1, step=t)
            one.step()

    def run_two():
        for t in range(a.steps):
            for sim, st in zip(halves, streams):
                with torch.cuda.stream(st):
                    pol.act(sim, 0, stochastic=True, seed=1, step=t)
                    sim.step()

    for name, fn in (("one stream, 65536 worlds", run_one), ("two streams, 2 x 32768", run_two)):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        print(f"{name}: {best * 1e6 / a.steps:.2f} us per step (wall, best of {a.reps})", flush=True)


if __name__ == "__main__":
    main()
