"""Average k_policy time (torch events on the current stream) for argmax and
sampling, over a simulator's real observation rows.

python tools/policy_time.py [--worlds 65536] [--iters 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only-argmax", action="store_true", help="agent-0 rows, argmax only (PMC runs)")
    ap.add_argument("--trace", action="store_true", help="per-wave phase clocks of one launch (agent-0 rows)")
    a = ap.parse_args()
    import madrona_basketball_amd as mba
    from madrona_basketball_amd.policy import FusedPolicy, make_agent
    sim = mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, a.worlds, 0,
                                       per_world_rng=True)
    sim.step_n(100, random_actions=True)
    pol = FusedPolicy.from_agent(make_agent(0).cuda())
    obs_all = sim.observations_tensor().to_torch()
    cases = [("agent 0 rows", obs_all[:, 0])]
    if not a.only_argmax:
        cases.append(("all agents", obs_all.view(-1, obs_all.shape[-1])))
    if a.trace:
        import ctypes
        import numpy as np
        from madrona_basketball_amd import _lib
        L = _lib.load()
        L.bb_diag_policy_trace.restype = ctypes.c_int
        L.bb_diag_policy_trace.argtypes = [ctypes.POINTER(_lib.PolicyWeights), ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
        obs = obs_all[:, 0]
        for stoch in (0, 1):
            buf = np.zeros((1 << 16, 8), np.uint64)
            nw = ctypes.c_int64()
            rc = L.bb_diag_policy_trace(ctypes.byref(pol._w), 0, obs.data_ptr(), obs.shape[0], obs.stride(0), stoch,
                                        torch.cuda.current_stream().cuda_stream, buf.ctypes.data, buf.shape[0],
                                        ctypes.byref(nw))
            assert rc == 0, L.bb_last_error()
            t = buf[:, :6].astype(np.int64)
            t = t[t[:, 0] > 0]
            t -= t[:, 0].min()
            pct = lambda x: [int(np.percentile(x, q)) for q in (0, 10, 50, 90, 100)]
            print(f"trace rows {obs.shape[0]} stochastic={stoch} waves {len(t)} (10 ns ticks) start {pct(t[:, 0])} "
                  f"end {pct(t[:, 5])}", flush=True)
            for n, i, j in (("weights", 0, 1), ("rows", 1, 2), ("layers", 2, 4), ("buckets", 4, 5)):
                print(f"  {n:14s} {pct(t[:, j] - t[:, i])}", flush=True)
    for label, obs in cases:
        rows = obs.shape[0]
        act = torch.empty((rows, 6), dtype=torch.int32, device="cuda")
        lp = torch.empty(rows, device="cuda")
        v = torch.empty(rows, device="cuda")
        for stoch in ((False,) if a.only_argmax else (False, True)):
            pol.forward_into(obs, act, lp, v, stochastic=stoch)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for t in range(a.iters):
                pol.forward_into(obs, act, lp, v, stochastic=stoch, step=t)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            print(f"{label:14s} rows {rows:7d} stochastic={int(stoch)}  {us:8.2f} us/launch  "
                  f"{rows * 512 / us / 1e3:7.1f} GB/s of obs rows", flush=True)


if __name__ == "__main__":
    main()
