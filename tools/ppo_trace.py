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
    ap.add_argument("--reps", type=int, default=3)
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
    ev = []
    for i in range(a.reps):
        ev.append(pol.rollout(sim, a.steps, b, seed=1, step0=i * a.steps, time_kernels=True) * 1e3)
    torch.cuda.synchronize()
    print(f"event us per rollout (first, median, last of {a.reps}): {ev[0]:.1f} {sorted(ev)[len(ev) // 2]:.1f} {ev[-1]:.1f}")
    lines = open(path).read().split("\n")
    steps = [l for l in lines if l and not l.startswith("wg")]
    wgs = [l for l in lines if l.startswith("wg")]
    G = (a.worlds + 31) // 32
    rows = np.array([[int(x) for x in l.split()] for l in steps[-a.steps:]], dtype=np.int64)
    # the first policy wave's pass for step k (points 4..12): obs_out record,
    # X into registers, layer 1 + its barrier, LayerNorm 1, layer 2, LayerNorm
    # 2, heads, bucket pass
    P = rows[:, 5:17]
    names = ["(start)", "X -> registers", "layer 1 MFMA", "LN 1 (+bar)", "layer 2 MFMA (+bar)",
             "LN 2 (+bar)", "heads (+bar)", "bucket maxima", "bucket per-logit", "bucket per-bucket",
             "bucket outputs"]
    sub = {n: [int(np.percentile((P[:, i + 1] - P[:, i]) * 10, q)) for q in (0, 50, 100)] for i, n in enumerate(names)}
    wg = np.array([[int(x) for x in l.split()[1:]] for l in wgs[-G:]], dtype=np.int64)
    t = rows[:, 1:5]
    d_sys = (t[:, 1] - t[:, 0]) * 10
    d_obs = (t[:, 2] - t[:, 1]) * 10
    d_pol = (t[1:, 3] - t[:-1, 2]) * 10  # policy for step k+1 after the rows of step k
    step = (t[1:, 0] - t[:-1, 0]) * 10
    pct = lambda x: [int(np.percentile(x, q)) for q in (0, 50, 100)]
    print(f"worlds {a.worlds}: ns per step {pct(step)}; S systems {pct(d_sys)}; S X free + rows {pct(d_obs)}; "
          f"P policy {pct(d_pol)}; barrier hand-offs {pct(step[:] - d_sys[1:] - d_obs[1:] - d_pol)}")
    wait = (P[1:, 0] - t[:-1, 2]) * 10  # S's rows done -> P's pass starts
    print(f"  P pass ns (min, median, max): rows ready -> P start {pct(wait)}; "
          + "; ".join(f"{n} {v}" for n, v in sub.items()))
    t0 = wg[:, 1].min()
    span = (wg[:, 2] - wg[:, 1]) * 10
    start = (wg[:, 1] - t0) * 10
    end = (wg[:, 2] - t0) * 10
    pq = lambda x: [int(np.percentile(x, q)) for q in (0, 10, 50, 90, 100)]
    w0 = wg[wg[:, 0] == 0][0]
    print(f"  workgroups {G}: start ns {pq(start)}; span ns {pq(span)}; end ns {pq(end)}; "
          f"wg0 setup {(t[0, 0] - w0[1]) * 10} ns, steps {(t[-1, 2] - t[0, 0]) * 10} ns, "
          f"tail {(w0[2] - t[-1, 2]) * 10} ns")


if __name__ == "__main__":
    main()
