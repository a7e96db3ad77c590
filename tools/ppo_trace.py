"""Per-step phase times of the fused PPO rollout (k_rollout_policy) from a
diagnostic variant build that stamps s_memrealtime (100 MHz) into the value
buffer (build.py --variant ppotrace with the stamps of
profiles/r06/r_ppo_trace.diff; never the product):

MADRONA_BB_LIB=.../_variants/ppotrace/libmadrona_basketball_amd.so python tools/ppo_trace.py [--worlds 8192]

S (sim wave): actions in -> systems done -> X pass 0 written -> X complete;
P (policy wave 0): X pass 0 in -> logits ready -> actions written.
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=8192)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--pw", type=int, default=-1)
    a = ap.parse_args()
    import madrona_basketball_amd as mba
    from madrona_basketball_amd import _lib
    from madrona_basketball_amd.policy import FusedPolicy, make_agent
    if a.pw > 0:
        _lib.diag_set("ppo_pwaves", a.pw)
    sim = mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, a.worlds, 0,
                                       per_world_rng=True)
    pol = FusedPolicy.from_agent(make_agent(0).cuda())
    bufs = pol.rollout_buffers(sim, a.k)
    for i in range(4):
        pol.rollout(sim, a.k, bufs, seed=1, step0=i * a.k)
    torch.cuda.synchronize()
    v = bufs["value"].view(torch.int32).cpu().numpy().astype(np.uint64) & 0xFFFFFFFF  # [K, W]
    G = a.worlds // 32
    v = v[:, :G * 32].reshape(a.k, G, 32)
    ts = (v[:, :, 0:14:2] | (v[:, :, 1:14:2] << np.uint64(32))).astype(np.int64)  # [K, G, 7]
    sa, sb, sc, sd, pa, pb, pc = [ts[:, :, i] for i in range(7)]
    ns = 10.0
    def q(x):
        x = np.asarray(x, dtype=np.float64).ravel() * ns
        return f"{np.percentile(x, 10):7.0f} {np.median(x):7.0f} {np.percentile(x, 90):7.0f}"
    print(f"worlds {a.worlds} pw {a.pw}: ns per step, 10th / median / 90th percentile over steps and workgroups")
    print(f"  step period (sa[t+1] - sa[t])         {q(sa[1:] - sa[:-1])}")
    print(f"  S systems (sb - sa)                   {q(sb - sa)}")
    print(f"  S rows pass 0 (sc - sb)               {q(sc - sb)}")
    print(f"  S pass 0 -> X complete (sd - sc)      {q(sd - sc)}")
    print(f"  P start after pass 0 (pa - sc)        {q(pa - sc)}")
    print(f"  P layers (pb - pa)                    {q(pb - pa)}")
    print(f"  P bucket pass (pc - pb)               {q(pc - pb)}")
    print(f"  actions -> S (sa[t+1] - pc[t])        {q(sa[1:] - pc[:-1])}")
    print(f"  P chain (pc - pa)                     {q(pc - pa)}")
    print(f"  S chain (sd - sa)                     {q(sd - sa)}")


if __name__ == "__main__":
    main()
