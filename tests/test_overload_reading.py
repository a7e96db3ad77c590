"""The one unpinned choice of the build: game.cpp's unqualified
acos / erf / exp on float arguments (src/game.cpp:746,808,868) bind to the
double functions here; a reference built with headers that put the float
overloads in the global namespace would call acosf / erff / expf instead.

tools/overload_divergence.py runs the two readings in lockstep on the oracle
(MATH_LIBM vs MATH_LIBM_FLOAT) at 8 192 worlds x 1 000 random steps, in the
tag-heavy scenario and in the full game; profiles/r05/overload_divergence.jsonl
holds what it measured.  These tests re-measure a small case and check the
recorded numbers: the two readings differ in the last bits of float columns
(reward, the shot-percentage attribute and the observations that carry it)
from the first step on, in a few to ~40 % of worlds at any time, but never in
integer / score / done state and never by more than the north_star float bar
(1e-5 + 1e-6 |x|): no trajectory forks within these runs."""
import json
import os

import pytest

from tools.overload_divergence import run_case

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RECORD = os.path.join(ROOT, "profiles", "r05", "overload_divergence.jsonl")
FLOAT_COLUMNS = {"reward", "observations", "attributes"}


def test_overload_readings_small_case(oracle_lib):
    rep = run_case("random_1024x200", dict(W=1024, steps=200))
    assert rep["first_diverging_step"] == 1
    assert set(rep["first_diverging_columns"]) <= FLOAT_COLUMNS
    for cp in rep["checkpoints"].values():
        assert set(cp["columns"]) <= FLOAT_COLUMNS
        assert cp["worlds_exact_state"] == 0.0
        assert cp["worlds_outside_float_bar"] == 0.0
        assert 0.0 < cp["worlds_any_bit"] < 0.2
    assert max(rep["max_abs_float_diff"].values()) < 1e-6


def test_recorded_overload_measurement():
    recs = [json.loads(line) for line in open(RECORD)]
    cases = {r["case"]: r for r in recs}
    assert set(cases) == {"random_8192x1000", "tag_heavy_4096x800", "full_game_2048x800"}
    for r in recs:
        assert r["first_diverging_step"] == 1
        assert set(r["max_abs_float_diff"]) <= FLOAT_COLUMNS
        assert max(r["max_abs_float_diff"].values()) < 1e-6
        for cp in r["checkpoints"].values():
            assert cp["worlds_exact_state"] == 0.0, (r["case"], cp)
            assert cp["worlds_outside_float_bar"] == 0.0, (r["case"], cp)
    # the share of worlds with a differing bit at the last checkpoint
    last = {k: v["checkpoints"][str(v["steps"])]["worlds_any_bit"] for k, v in cases.items()}
    assert last["random_8192x1000"] == pytest.approx(0.0348, abs=1e-3)
    assert last["tag_heavy_4096x800"] == pytest.approx(0.1709, abs=1e-3)
    assert last["full_game_2048x800"] == pytest.approx(0.4263, abs=1e-3)
