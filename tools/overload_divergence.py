"""How far a reference built with the float overloads of game.cpp's unqualified
acos / erf / exp (src/game.cpp:746,808,868) would diverge from the double
reading this build takes.

Two oracles run in lockstep on identical actions: MATH_LIBM (the reference CPU
executor's glibc float calls, the unqualified calls bound to C's double
functions -- the product's reading, bit-identical to the HIP path on every
column) and MATH_LIBM_FLOAT (the same, but acosf / erff / expf).  Per case the
script records the first step at which any column differs, the columns that
differ then, and at checkpoints the fraction of worlds with any differing
column, of worlds whose integer / score / done state differs, and of worlds
outside the north_star float bar.  Test infrastructure: CPU only (the oracle).

python tools/overload_divergence.py [--out profiles/r05/overload_divergence.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.oracle import MATH_LIBM, MATH_LIBM_FLOAT, Oracle  # noqa: E402
from tests.helpers import ALL_COLUMNS, EXACT_COLUMNS, FLOAT_ATOL, oracle_flags  # noqa: E402

CASES = {
    "random_8192x1000": dict(W=8192, steps=1000),
    "tag_heavy_4096x800": dict(W=4096, steps=800, sparse=True),
    "full_game_2048x800": dict(W=2048, steps=800, flags=dict(one_on_one=False)),
}
CHECKPOINTS = (50, 100, 200, 400, 800, 1000)


def world_masks(a: Oracle, b: Oracle):
    """Per world: any column differs in a bit; an exact column differs; a float
    column is outside the north_star bar (1e-5 + 1e-6 |x|)."""
    W = a.w
    anyd = np.zeros(W, bool)
    exact = np.zeros(W, bool)
    outside = np.zeros(W, bool)
    cols = []
    maxdiff = {}
    for n in ALL_COLUMNS:
        x, y = a.export(n), b.export(n)
        d = (x.view(np.uint32) != y.view(np.uint32)).reshape(W, -1).any(axis=1)
        if d.any():
            cols.append(n)
            anyd |= d
            if n in EXACT_COLUMNS or x.dtype != np.float32:
                exact |= d
            else:
                diff = np.abs(x.astype(np.float64) - y.astype(np.float64))
                tol = FLOAT_ATOL + 1e-6 * np.abs(y.astype(np.float64))
                outside |= (diff > tol).reshape(W, -1).any(axis=1)
                maxdiff[n] = float(np.nanmax(diff))
    return anyd, exact, outside, cols, maxdiff


def run_case(name: str, c: dict, seed: int = 321) -> dict:
    W, steps = c["W"], c["steps"]
    fl = oracle_flags(per_world_rng=True, **c.get("flags", {}))
    a = Oracle(W, flags=fl, math_mode=MATH_LIBM)
    b = Oracle(W, flags=fl, math_mode=MATH_LIBM_FLOAT)
    rng = np.random.default_rng(5)
    hi = np.array([2, 8, 3, 2, 2, 2])
    first = None
    first_cols: list = []
    ever = np.zeros(W, bool)
    maxabs: dict = {}
    checks = {}
    for t in range(steps):
        if c.get("sparse"):
            # tests/helpers.py sparse_actions: a mostly idle offence the defence AI tags
            act = a.export("action").copy()
            r = (rng.random((W, 6)) * hi).astype(np.int32)
            r[rng.random(W) >= 0.02] = 0
            act[:, 0] = r
            bact = b.export("action").copy()
            bact[:, 0] = r
            a.set_actions(act)
            b.set_actions(bact)
        else:
            a.random_actions(seed, t)
            b.random_actions(seed, t)
        a.step()
        b.step()
        anyd, exact, outside, cols, md = world_masks(a, b)
        for n, v in md.items():
            maxabs[n] = max(maxabs.get(n, 0.0), v)
        ever |= anyd
        if first is None and anyd.any():
            first, first_cols = t + 1, cols
        if (t + 1) in CHECKPOINTS or t + 1 == steps:
            checks[t + 1] = {"worlds_any_bit": float(anyd.mean()), "worlds_exact_state": float(exact.mean()),
                             "worlds_outside_float_bar": float(outside.mean()), "columns": cols}
    return {"case": name, "worlds": W, "steps": steps, "flags": c.get("flags", {}),
            "first_diverging_step": first, "first_diverging_columns": first_cols,
            "worlds_ever_diverged": float(ever.mean()), "max_abs_float_diff": maxabs, "checkpoints": checks}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05", "overload_divergence.jsonl"))
    ap.add_argument("--case", action="append", default=None)
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        for name in args.case or list(CASES):
            rep = run_case(name, CASES[name])
            print(json.dumps(rep), flush=True)
            f.write(json.dumps(rep) + "\n")


if __name__ == "__main__":
    main()
