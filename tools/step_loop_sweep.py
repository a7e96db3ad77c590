"""bb_step_n_staged per-step kernel time (events) across world counts, by
kind (bb_diag_step_loop): 2 register-resident rollout launch with per-step
state stores, 1 one k_step_loop launch, 0 one k_step launch per step.  With
--check every column and the written-back action rows of each kind are
compared with kind 0's (same initial state, same staged rows).

python tools/step_loop_sweep.py [--worlds 16384,32768,...] [--steps 200] [--reps 3] [--kinds 2,1,0] [--check]
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
    ap.add_argument("--kinds", default="2,1,0")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--minw", type=int, default=-1, help="rollout_minw path override (3: k_rollout2)")
    a = ap.parse_args()
    kinds = [int(x) for x in a.kinds.split(",")]
    L = _lib.load()
    if a.minw >= 0:
        _lib.diag_set("rollout_minw", a.minw)
    for W in [int(x) for x in a.worlds.split(",")]:
        sim = mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, W, 0,
                                           num_agents=a.agents, per_world_rng=True)
        sim.step_n(10, random_actions=True)
        if a.check:
            ref = None
            for kind in [0] + [k for k in kinds if k != 0]:
                c = mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, W, 0,
                                                 num_agents=a.agents, per_world_rng=True)
                c.step_n(7, random_actions=True)
                acts = c.stage_random_actions(37, action_seed=9, step0=50)
                L.bb_diag_step_loop(kind)
                c.step_n_staged(acts)
                torch.cuda.synchronize()
                got = {n: t.clone() for n, t in c._views.items()}
                got["staged"] = acts.clone()
                if ref is None:
                    ref = got
                else:
                    bad = [n for n in ref if not torch.equal(ref[n], got[n])]
                    print(f"worlds {W:7d} kind {kind} vs 0: {'EQUAL' if not bad else 'DIFF ' + ','.join(bad)}",
                          flush=True)
                del c, acts
            L.bb_diag_step_loop(-1)
        res = {}
        for kind in kinds:
            L.bb_diag_step_loop(kind)
            ts = []
            for r in range(a.reps):
                acts = sim.stage_random_actions(a.steps, action_seed=5, step0=100 + r * a.steps)
                ts.append(sim.step_n_staged(acts, time_kernels=True) * 1e3 / a.steps)
                del acts
            res[kind] = statistics.median(ts)
        L.bb_diag_step_loop(-1)
        print(f"worlds {W:7d} x {a.agents} minw {a.minw} {_lib.kernel_name(sim._h, 1, a.steps)}  " + "   ".join(f"kind {k} {res[k]:8.2f} us/step" for k in kinds),
              flush=True)
        del sim
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
