"""Where a k_step_ppo launch's time goes (the fused PPO step, bb_rollout_policy
from 32 768 worlds).

1. Per-wave phase clocks of every launch of one rollout
   (MADRONA_BB_PPO_STEP_TRACE; 10 ns ticks of the constant-rate clock): median
   and spread over the waves of a middle step of each phase -- load, systems,
   state stores, pass 0 (rows into LDS, layer-1 MFMAs + stores), pass 1, the
   layers, the bucket pass, the stores' drain.
2. Attribution by leaving parts out (MADRONA_BB_PPO_STEP_DIAG, read once per
   process, so each variant runs in a child process): us per step of the whole
   rollout with the bucket pass, the layers, the layer-1 MFMAs and the
   buffer.obs stores skipped (outputs then wrong; timing only).

python tools/ppo_step_trace.py [--worlds 65536] [--k 32]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
POINTS = 12
PHASES = ["load", "systems", "reward+state stores", "pass 0 rows->LDS", "pass 0 MFMA+stores",
          "pass 1 rows->LDS", "pass 1 MFMA+stores", "LN / layer 2 / heads", "bucket pass", "stores retire"]

CHILD = r'''
import sys, json, torch
sys.path.insert(0, {root!r})
import madrona_basketball_amd as mba
from madrona_basketball_amd.policy import FusedPolicy, make_agent
W, K, R = {W}, {K}, {R}
sim = mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, W, 0, per_world_rng=True)
pol = FusedPolicy.from_agent(make_agent(0).cuda())
b = pol.rollout_buffers(sim, K)
pol.rollout(sim, K, b, seed=1, step0=0)
torch.cuda.synchronize()
ms = sorted(pol.rollout(sim, K, b, seed=1, step0=(i + 1) * K, time_kernels=True) for i in range(R))
print(json.dumps({{"us_per_step": ms[len(ms) // 2] * 1e3 / K}}))
'''


def child(W, K, R, env_extra):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, W=W, K=K, R=R)], env=env,
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-3000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=65536)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-ablate", action="store_true")
    ap.add_argument("--skews", default="", help="comma list: the upper half of each workgroup's waves starts "
                                                 "k s_sleep(127) later (timing experiment, diag bits 8-15)")
    a = ap.parse_args()
    W, K = a.worlds, a.k
    waves = (W + 31) // 32
    path = os.path.join(tempfile.mkdtemp(), "pps_trace.bin")
    child(W, K, 1, {"MADRONA_BB_PPO_STEP_TRACE": path})
    ts = np.fromfile(path, dtype=np.uint64).astype(np.int64).reshape(K, waves, POINTS)
    t = ts[K // 2]  # a middle step
    t0 = t[:, 0].min()
    print(f"worlds {W}: step {K // 2} of {K}, {waves} waves; clock ticks of 10 ns")
    print(f"  wave start (us from the first): median {np.median(t[:, 0] - t0) / 100:.2f}, "
          f"p90 {np.percentile(t[:, 0] - t0, 90) / 100:.2f}, max {(t[:, 0] - t0).max() / 100:.2f}")
    print(f"  wave end   (us from the first start): median {np.median(t[:, 10] - t0) / 100:.2f}, "
          f"max {(t[:, 10] - t0).max() / 100:.2f}; wave life median {np.median(t[:, 10] - t[:, 0]) / 100:.2f}")
    for i, name in enumerate(PHASES):
        d = (t[:, i + 1] - t[:, i]) / 100.0
        print(f"  {name:24s} median {np.median(d):6.2f} us  p10 {np.percentile(d, 10):6.2f}  p90 {np.percentile(d, 90):6.2f}")
    if a.skews:
        print("start skew of half the waves (us per step, median of the rollouts):")
        for k in [int(x) for x in a.skews.split(",")]:
            r = child(W, K, a.reps, {"MADRONA_BB_PPO_STEP_DIAG": str(k << 8)})
            print(f"  skew {k:2d} x s_sleep(127) {r['us_per_step']:7.2f}", flush=True)
    if a.no_ablate:
        return
    print("attribution (parts skipped; us per step, median of the rollouts):")
    for diag, name in [(0, "product"), (8, "no buffer.obs stores"), (1, "no bucket pass"),
                       (3, "no bucket pass, no layers 2 / heads"), (7, "no policy (no MFMAs)"),
                       (15, "no policy, no buffer.obs stores")]:
        r = child(W, K, a.reps, {"MADRONA_BB_PPO_STEP_DIAG": str(diag)})
        print(f"  diag {diag:2d} {name:38s} {r['us_per_step']:7.2f}", flush=True)


if __name__ == "__main__":
    main()
