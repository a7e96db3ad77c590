"""bb_step_n_staged as one k_step_loop launch vs one k_step launch per step,
per-step kernel time (events) across world counts.

python tools/step_loop_sweep.py [--worlds 16384,32768,...] [--steps 200] [--reps 3]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import madrona_basketball_amd as mba
    from madrona_basketball_amd import _lib
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="8192,16384,32768,49152,65536,81920,98304,131072,196608,262144")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--agents", type=int, default=2)
    a = ap.parse_args()
    L = _lib.load()
    for W in [int(x) for x in a.worlds.split(",")]:
        sim = mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, W, 0,
                                           num_agents=a.agents, per_world_rng=True)
        sim.step_n(10, random_actions=True)
        res = {}
        for loop in (1, 0):
            L.bb_diag_step_loop(loop)
            ts = []
            for r in range(a.reps):
                acts = sim.stage_random_actions(a.steps, action_seed=5, step0=100 + r * a.steps)
                ts.append(sim.step_n_staged(acts, time_kernels=True) * 1e3 / a.steps)
                del acts
            res[loop] = statistics.median(ts)
        L.bb_diag_step_loop(-1)
        print(f"worlds {W:7d} x {a.agents}  loop {res[1]:8.2f} us/step   one launch per step {res[0]:8.2f} us/step   "
              f"ratio {res[1] / res[0]:.3f}", flush=True)
        del sim
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
