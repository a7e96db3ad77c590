"""Per-system time attribution (MODE_SKIP variants of k_step, timing only):
  skip: the kernel without one system (its state effects are lost, so later
        systems see a different trajectory -- confounded);
  dup:  the kernel with one system run a second time on a copy whose result
        is dropped (same trajectory; the added time is the system's cost)."""
import argparse, ctypes, os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAMES = {1: "tick", 2: "actionMask", 3: "moveAgent", 4: "grab", 5: "pass", 6: "shoot", 7: "moveBall",
         8: "shotPct", 9: "score", 10: "outOfBounds", 11: "lastTouch", 12: "clock", 13: "inboundViol",
         14: "reset", 15: "pointsWorth", 16: "collision", 17: "defense"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, default=65536)
    ap.add_argument("--agents", type=int, default=2)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import madrona_basketball_amd as mba
    from madrona_basketball_amd import _lib
    L = _lib.load()
    L.bb_diag_time.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                               ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
    sim = mba.SimpleGridworldSimulator(32, 17, 15.7575, 8.382, 39600, mba.ExecMode.CUDA, a.worlds, 0,
                                       num_agents=a.agents, per_world_rng=True)
    sim.step_n(50, random_actions=True)
    torch.cuda.synchronize()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    snap = sim.snapshot()

    def t(mode, skip=0, dup=0):
        v = []
        for _ in range(a.rounds):
            sim.restore(snap)
            ms = ctypes.c_float()
            assert L.bb_diag_time(sim._h, mode, a.iters, skip, dup, st, ctypes.byref(ms)) == 0, L.bb_last_error()
            v.append(ms.value * 1e3)
        return statistics.median(v)
    base = t(5)  # MODE_SKIP with empty mask == full
    full = t(0)
    print(f"full {full:.2f} us, skip-mode baseline {base:.2f} us, no-obs {t(4):.2f}, io {t(1):.2f}")
    for b, n in NAMES.items():
        x = t(5, 1 << b)
        print(f"  without {n:12s} {x:8.2f} us   saves {base - x:6.2f} us")
    for combo in ((8, 17), (8, 17, 6), (6, 8)):
        x = t(5, sum(1 << b for b in combo))
        print(f"  without {'+'.join(NAMES[b] for b in combo):24s} {x:8.2f} us   saves {base - x:6.2f} us")
    allsys = t(5, sum(1 << b for b in NAMES))
    print(f"  without all systems {allsys:.2f} us")
    for b, n in NAMES.items():
        x = t(5, 0, 1 << b)
        print(f"  twice   {n:12s} {x:8.2f} us   adds  {x - base:6.2f} us")
    x = t(5, 0, sum(1 << b for b in NAMES))
    print(f"  all systems twice {x:.2f} us   adds {x - base:.2f} us")


if __name__ == "__main__":
    main()
