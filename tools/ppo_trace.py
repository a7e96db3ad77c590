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
    T = rows[:, 1:]  # clock points of each step (PPO_TRACE_POINTS, bb_kernels.hip)
    pct = lambda x: [int(np.percentile(x, q)) for q in (0, 50, 100)]
    if T.shape[1] == 16:  # the round-4 kernel (one hand-off of the rows): its layout
        old = [(5, 6, "X -> registers"), (6, 7, "layer 1 MFMA"), (7, 8, "LN 1 (+bar)"), (8, 9, "layer 2 (+bar)"),
               (9, 10, "LN 2 (+bar)"), (10, 11, "heads (+bar)"), (11, 12, "bucket maxima"),
               (12, 13, "bucket per-logit"), (13, 14, "bucket per-bucket"), (14, 15, "bucket outputs"),
               (15, 3, "to actions")]
        step = (T[1:, 0] - T[:-1, 0]) * 10
        print(f"worlds {a.worlds} (round-4 layout): ns per step {pct(step)}; S systems {pct((T[:, 1] - T[:, 0]) * 10)}; "
              f"S X free + rows {pct((T[:, 2] - T[:, 1]) * 10)}; P {pct((T[1:, 3] - T[:-1, 2]) * 10)}")
        print("  P: " + "; ".join(f"{n} {pct((T[1:, j] - T[1:, i]) * 10)}" for i, j, n in old))
        return
    ns = lambda i, j, sl=slice(None): (T[sl, j] - T[sl, i]) * 10
    # S (sim wave): 0 actions in, 1 systems done, 20 row sources done, 21 pass 0
    # of X written, 2 rows complete
    step = (T[1:, 0] - T[:-1, 0]) * 10
    print(f"worlds {a.worlds}: ns per step {pct(step)}")
    print(f"  S: systems {pct(ns(0, 1))}; row sources {pct(ns(1, 20))}; X free + pass 0 {pct(ns(20, 21))}; "
          f"pass 1 (+ last-step rows) {pct(ns(21, 2))}")
    # P (first policy wave), pass of step k + 1 against S's rows of step k
    names = [(4, 6, "layer 1, steps 0-15"), (6, 7, "wait: rows' second half"),
             (7, 12, "layer 1 steps 16-31, LN 1, layer 2, LN 2, heads"),
             (12, 13, "bucket: uniforms (drawn ahead: 0)"), (13, 14, "bucket per-bucket"),
             (15, 16, "bucket outputs"), (16, 3, "to actions")]
    print("  P: " + "; ".join(f"{n} {pct(ns(i, j, slice(1, None)))}" for i, j, n in names))
    # the overlap: P's layer 1 on pass 0 of step k's rows starts before S has
    # finished pass 1 of them
    lead = (T[:-1, 2] - T[1:, 4]) * 10
    print(f"  overlap: P starts layer 1 this many ns before S's rows are complete {pct(lead)}; "
          f"P pass (start -> actions) {pct((T[1:, 3] - T[1:, 4]) * 10)}; "
          f"S (actions in -> rows complete) {pct(ns(0, 2))}")
    wg = np.array([[int(x) for x in l.split()[1:]] for l in wgs[-G:]], dtype=np.int64)
    t = T[:, [0, 1, 2, 3]]
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
