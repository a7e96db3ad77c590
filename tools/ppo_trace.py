"""Per-step phase clocks of the fused PPO rollout kernel (workgroup 0):
S = the sim wave's step (systems + reward, then the observation rows), P = the
policy waves' pass (network + buckets) that precedes it.

python tools/ppo_trace.py [--worlds 8192] [--steps 32]
"""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=32)
    a = ap.parse_args()
    path = os.path.join(tempfile.mkdtemp(), "ppo_trace.txt")
    os.environ["MADRONA_BB_PPO_TRACE"] = path
    import numpy as np
    import torch
    import madrona_basketball_amd as mba
    from madrona_basketball_amd.policy import FusedPolicy, make_agent
    sim = mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, a.worlds, 0,
                                       per_world_rng=True)
    pol = FusedPolicy.from_agent(make_agent(0).cuda())
    b = pol.rollout_buffers(sim, a.steps)
    for i in range(3):
        pol.rollout(sim, a.steps, b, seed=1, step0=i * a.steps)
    torch.cuda.synchronize()
    rows = np.loadtxt(path, dtype=np.int64)[-a.steps:]
    t = rows[:, 1:5]
    d_sys = (t[:, 1] - t[:, 0]) * 10
    d_obs = (t[:, 2] - t[:, 1]) * 10
    d_pol = (t[1:, 3] - t[:-1, 2]) * 10  # policy for step k+1 after the rows of step k
    step = (t[1:, 0] - t[:-1, 0]) * 10
    pct = lambda x: [int(np.percentile(x, q)) for q in (0, 50, 100)]
    print(f"worlds {a.worlds}: ns per step {pct(step)}; S systems+reward {pct(d_sys)}; S rows {pct(d_obs)}; "
          f"P policy {pct(d_pol)}; barrier hand-offs {pct(step[:] - d_sys[1:] - d_obs[1:] - d_pol)}")


if __name__ == "__main__":
    main()
