"""Time k_step variants (bb::StepMode) and a coalesced streaming probe with the
same per-world traffic, interleaved in one process (guide §5.4 rule 24).

python tools/ablate.py [--worlds 65536] [--agents 2] [--iters 200] [--rounds 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MODES = {0: "full (LDS-staged obs)", 1: "io only", 2: "io + obs rows", 3: "full (lane-strided obs, v1)",
         4: "full minus obs", 100: "stream probe (same bytes, coalesced)",
         101: "stream probe, per-wave regions", 102: "stream probe, nt stores",
         103: "stream probe, per-wave regions, nt"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=65536)
    ap.add_argument("--agents", type=int, default=2)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", type=int, nargs="*", default=None, help="time only these modes, no trace")
    args = ap.parse_args()
    import torch
    import madrona_basketball_amd as mba
    from madrona_basketball_amd import _lib
    L = _lib.load()
    L.bb_diag_time.restype = ctypes.c_int
    L.bb_diag_time.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                               ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
    sim = mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, args.worlds, 0,
                                       num_agents=args.agents, per_world_rng=True)
    sim.step_n(50, random_actions=True)  # realistic, diverged state
    torch.cuda.synchronize()
    N = args.agents
    B = L.bb_algorithmic_bytes_per_world(N)
    obs_b = N * 4 * (61 + 38 * (N - 1) + 2 * N)  # observation bytes of B
    reads = N * 144 + 120                          # per-agent and per-world reads of B
    # the probe moves B in 16-byte pieces: its reads, then the rest as writes
    read_q, write_q = (reads + 15) // 16, (B - reads + 15) // 16
    # algorithmic bytes each mode moves per world: the variants without the
    # observation pass do not write the rows, the probe moves its own pieces
    moved = {0: B, 1: B - obs_b, 2: B, 3: B, 4: B - obs_b, **{m: 16 * (read_q + write_q) for m in (100, 101, 102, 103)}}
    modes = {m: MODES[m] for m in (args.only if args.only is not None else MODES)}
    res = {m: [] for m in modes}
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for r in range(args.rounds):
        for m in modes:
            ms = ctypes.c_float()
            rc = L.bb_diag_time(sim._h, m, args.iters, read_q, write_q, stream, ctypes.byref(ms))
            assert rc == 0, L.bb_last_error()
            res[m].append(ms.value * 1e3)
    out = {}
    for m, v in res.items():
        med = statistics.median(v)
        gbs = moved[m] * args.worlds / (med * 1e-6) / 1e9
        out[MODES[m]] = {"median_us": med, "min_us": min(v), "bytes_per_world": moved[m], "GBps": gbs}
        # above the HBM peak the bytes did not all come from / go to HBM
        # (Infinity-Cache-resident state): say so instead of quoting a rate
        note = "  (> 8 TB/s HBM peak: cache-resident, not an HBM rate)" if gbs > 8000 else ""
        print(f"{MODES[m]:40s} median {med:8.2f} us  min {min(v):8.2f} us  "
              f"{moved[m]:6d} B/world  {gbs:7.0f} GB/s{note}", flush=True)
    if args.only is None:
        out["trace"] = trace(L, sim, stream)
    print(json.dumps({"worlds": args.worlds, "agents": args.agents, "results": out}))


def trace(L, sim, stream):
    """Per-wave phase clocks of one MODE_TRACE launch (wall_clock64 ticks,
    100 MHz on gfx950): when waves start/end and how long each phase takes."""
    import numpy as np
    L.bb_diag_trace.restype = ctypes.c_int
    L.bb_diag_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                ctypes.POINTER(ctypes.c_int64)]
    cap = 1 << 20
    buf = np.zeros((cap, 12), dtype=np.uint64)
    nw = ctypes.c_int64()
    rc = L.bb_diag_trace(sim._h, stream, buf.ctypes.data, cap, ctypes.byref(nw))
    assert rc == 0, L.bb_last_error()
    pct = lambda x: [int(np.percentile(x, q)) for q in (0, 10, 50, 90, 100)]
    # one wave per 64 // N worlds (N = 2: 32 worlds of agent lanes; N >= 4:
    # 64 // N worlds of the LDS-world kernel, the lanes past them idle)
    wpw = 64 // sim.num_agents
    ngrid = (sim.num_worlds + wpw - 1) // wpw
    if nw.value != ngrid and nw.value % ngrid:
        raise RuntimeError(f"trace: {nw.value} wave records for a {ngrid}-wave grid")
    if nw.value != ngrid:  # k_step_wide: WAVES waves per workgroup, per-role phases
        waves = nw.value // ngrid
        t = buf[: nw.value, :10].astype(np.int64).reshape(ngrid, waves, 10)
        t -= t[:, :, 0].min()
        roles = ["DEF", "PCT", "STORE"] + [f"OBS{i}" for i in range(waves - 3)]
        res = {"waves": int(nw.value), "tick_ns": 10, "kernel_span": int(t[:, :, 9].max() - t[:, :, 0].min())}
        for r, name in enumerate(roles):
            x = t[:, r]
            res[name] = {"start": pct(x[:, 0]), "load": pct(x[:, 1] - x[:, 0]), "b0_wait": pct(x[:, 2] - x[:, 1]),
                         "systems": pct(x[:, 3] - x[:, 2]), "b1_wait": pct(x[:, 4] - x[:, 3]),
                         "tail": pct(x[:, 9] - x[:, 4]), "end": pct(x[:, 9])}
        for k, v in res.items():
            print(f"trace {k:6s} {v}", flush=True)
        return res
    t = buf[: nw.value, :10].astype(np.int64)
    resets = buf[: nw.value, 10].astype(np.int64)
    t -= t[:, 0].min()
    names = ["load", "tick..move", "grab..shoot", "ball..score", "oob..inbound", "reset", "points..defense",
             "reward+store", "obs"]
    res = {"waves": int(nw.value), "tick_ns": 10, "start_pct": pct(t[:, 0]), "end_pct": pct(t[:, 9]),
           "lifetime_pct": pct(t[:, 9] - t[:, 0]), "waves_with_reset": int((resets > 0).sum()),
           "reset_lanes": int(resets.sum())}
    for i, n in enumerate(names):
        res[f"{n}_pct"] = pct(t[:, i + 1] - t[:, i])
    sel = resets > 0
    if sel.any() and (~sel).any():
        res["reset_phase_with_reset_pct"] = pct(t[sel, 6] - t[sel, 5])
        res["reset_phase_without_pct"] = pct(t[~sel, 6] - t[~sel, 5])
    for k, v in res.items():
        print(f"trace {k:14s} {v}", flush=True)
    return res


if __name__ == "__main__":
    main()
