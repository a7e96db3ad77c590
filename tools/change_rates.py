"""Per step, the fraction of worlds and of 32-world waves (one resident-loop
wave at N = 2) whose state columns / observation-row 128-byte lines change,
on the oracle (random play, per-world RNG): what a store-only-on-change
scheme can skip.  python tools/change_rates.py"""
import numpy as np, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.oracle import Oracle, FLAG_PER_WORLD_RNG
W = 8192; G = 32
o = Oracle(W, flags=FLAG_PER_WORLD_RNG)
for t in range(50):
    o.random_actions(321, t); o.step()
cols = ["reset", "action_mask", "agent_possession", "inbounding", "attributes", "grab_cooldown", "game_state",
        "world_clock", "rng_counter", "ball_physics", "ball_grabbed", "action", "agent_pos", "ball_pos", "ball_velocity",
        "orientation", "agent_velocity", "cur_step", "done", "reward"]
def grab():
    d = {c: o.export(c).copy().view(np.uint32).reshape(W, -1) for c in cols}
    a = d["attributes"].reshape(W, 2, 10)
    d["attr_event"] = np.concatenate([a[:, :, :5], a[:, :, 9:]], axis=2).reshape(W, -1)
    d["attr_5_8"] = a[:, :, 5:9].reshape(W, -1)
    g = d["game_state"]
    d["game_nonclock"] = np.concatenate([g[:, :8], g[:, 10:]], axis=1)
    d["game_clocks"] = g[:, 8:10]
    return d
prev = grab()
acc = {}
steps = 300
for t in range(50, 50 + steps):
    o.random_actions(321, t); o.step()
    cur = grab()
    for k in cur:
        ch = (cur[k] != prev[k]).any(axis=1)
        acc.setdefault(k, [0, 0])
        acc[k][0] += ch.mean()
        acc[k][1] += ch.reshape(W // G, G).any(axis=1).mean()
    prev = cur
for k, (w, g) in sorted(acc.items(), key=lambda x: x[1][1]):
    print(f"{k:16s} worlds changed {w/steps:7.4f}   32-world waves changed {g/steps:7.4f}")
print("--- observation row lines (128 B each), fraction of 32-world waves with any change")
o2 = Oracle(W, flags=FLAG_PER_WORLD_RNG)
for t in range(50):
    o2.random_actions(321, t); o2.step()
prev = o2.export("observations").copy().view(np.uint32)
acc = np.zeros(4); accw = np.zeros(4)
for t in range(50, 50 + steps):
    o2.random_actions(321, t); o2.step()
    cur = o2.export("observations").copy().view(np.uint32)
    for l in range(4):
        ch = (cur[:, :, 32*l:32*l+32] != prev[:, :, 32*l:32*l+32]).any(axis=(1, 2))
        accw[l] += ch.mean(); acc[l] += ch.reshape(W // G, G).any(axis=1).mean()
    prev = cur
for l in range(4):
    print(f"line {l}: worlds {accw[l]/steps:.4f}  waves {acc[l]/steps:.4f}")
