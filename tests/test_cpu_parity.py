"""Host executor (ExecMode.CPU, the same step code the gfx950 kernel runs)
vs the oracle, across the reference's configurations and edge cases."""
import numpy as np
import pytest
import torch

from madrona_basketball_amd import ExecMode
from oracle.oracle import Oracle
from tests.helpers import compare, count_tags, make_sim, oracle_flags, run_lockstep, sim_np, sparse_actions


@pytest.fixture(scope="module", autouse=True)
def _libs(native_lib, oracle_lib):
    pass


def test_generation_matches():
    sim = make_sim(ExecMode.CPU, 16)
    bad, ident = compare(sim, Oracle(16))
    assert not bad, bad
    assert min(ident.values()) == 1.0


def test_single_world_scripted_config0():
    """configs[0]: 1 world, CPU executor, scripted actions."""
    sim = make_sim(ExecMode.CPU, 1)
    o = Oracle(1)
    script = np.zeros((700, 1, 2, 6), np.int32)
    script[5:60, 0, 0] = [1, 2, 0, 0, 0, 0]      # offence runs right
    script[60:80, 0, 0] = [1, 6, 1, 0, 0, 0]     # back left while turning
    script[80, 0, 0] = [0, 0, 0, 0, 0, 1]        # shoot
    script[200:260, 0, 1] = [1, 4, 2, 1, 1, 1]   # defender inputs (overridden by defence AI)
    run_lockstep(sim, o, 700, check_every=1, actions_fn=lambda t: script[t])


@pytest.mark.parametrize("per_world_rng", [False, True])
def test_random_rollout(per_world_rng):
    W = 256
    sim = make_sim(ExecMode.CPU, W, per_world_rng=per_world_rng)
    o = Oracle(W, flags=oracle_flags(per_world_rng=per_world_rng))
    worst = run_lockstep(sim, o, 1500, check_every=50)
    assert worst["observations"] == 1.0


def test_staged_actions_equal_per_step_writes():
    """bb_step_n_staged (actions resident in a [n,W,N,6] buffer, the bench
    path) == bb_step_n with the same synthetic actions written before each
    step, on every column."""
    W, n = 128, 300
    a = make_sim(ExecMode.CPU, W, per_world_rng=True)
    b = make_sim(ExecMode.CPU, W, per_world_rng=True)
    a.step_n(n, random_actions=True, action_seed=321, step0=7)
    staged = b.stage_random_actions(n, action_seed=321, step0=7)
    b.step_n_staged(staged)
    for name in a._views:
        assert torch.equal(a._views[name], b._views[name]), name


def test_tag_heavy_rollout():
    """Mostly idle offenders: the defence AI tags them (SAT contact, -10/+10,
    delayed reset) -- the contact path random play almost never reaches."""
    W = 256
    sim = make_sim(ExecMode.CPU, W, per_world_rng=True)
    o = Oracle(W, flags=oracle_flags(per_world_rng=True))
    tags = [0]
    run_lockstep(sim, o, 800, check_every=20, actions_fn=sparse_actions(o),
                 on_step=lambda t: tags.__setitem__(0, tags[0] + count_tags(o)))
    assert tags[0] >= 100, tags[0]


@pytest.mark.parametrize("n_agents", [4, 6, 8, 10])
def test_more_agents(n_agents):
    W = 64
    sim = make_sim(ExecMode.CPU, W, num_agents=n_agents, per_world_rng=True)
    o = Oracle(W, num_agents=n_agents, flags=oracle_flags(per_world_rng=True))
    assert sim.observations_tensor().to_torch().shape == (W, n_agents, O_width(n_agents))
    run_lockstep(sim, o, 600, check_every=50)


def O_width(n):
    from oracle.oracle import obs_width
    return obs_width(n)


@pytest.mark.parametrize("flags", [dict(tag_mask=False), dict(one_on_one=False),
                                   dict(tag_mask=False, one_on_one=False)])
def test_game_variants(flags):
    """grab / pass / steal (tag override off) and the full-game inbound,
    period and violation paths (isOneOnOne = 0)."""
    W = 256
    sim = make_sim(ExecMode.CPU, W, per_world_rng=True, **flags)
    o = Oracle(W, flags=oracle_flags(per_world_rng=True, **flags))
    seen_grab = False
    for chunk in range(24):
        run_lockstep(sim, o, 50, check_every=50, step0=chunk * 50)
        seen_grab |= bool((sim_np(sim, "grab_cooldown") > 0).any())
    if not flags.get("tag_mask", True):
        assert seen_grab  # grabs happened


def test_full_game_reaches_period_logic():
    """isOneOnOne = 0 with no one moving: the clock expiry takes the
    end-of-period branch of resetWorld (gen.cpp:221-236)."""
    W = 4
    sim = make_sim(ExecMode.CPU, W, one_on_one=False)
    o = Oracle(W, flags=oracle_flags(one_on_one=False))
    run_lockstep(sim, o, 1400, check_every=20, actions_fn=lambda t: np.zeros((W, 2, 6), np.int32))
    assert sim_np(sim, "game_state")[0, 2] >= 2  # period advanced


def test_full_game_inbound_scenario():
    """Forced rare paths: grab, shot, out-of-bounds inbound, inbound
    violation turnover, pass (tests/scenarios.py)."""
    from tests.scenarios import FullGameInbound
    W = 4
    sim = make_sim(ExecMode.CPU, W, tag_mask=False, one_on_one=False)
    o = Oracle(W, flags=oracle_flags(tag_mask=False, one_on_one=False))
    sc = FullGameInbound(W)
    sc.prepare(o, sim.internal_tensor("attributes"))
    seen = {"inbound": False, "violation": False, "pass": False}
    prev_oob = np.zeros(W)
    for t in range(1000):
        a = sc.actions(o, t)
        run_lockstep(sim, o, 1, check_every=1, actions_fn=lambda _: a)
        gs = sim_np(sim, "game_state")
        gi = gs.view(np.int32)
        seen["inbound"] |= bool((gi[:, 0] == 1).any())
        seen["violation"] |= bool(((gs[:, 11] > prev_oob) & (gi[:, 1] == 0) & (gs[:, 11] >= 2)).any())
        seen["pass"] |= bool(((gi[:, 0] == 0) & (gs[:, 11] >= 1) & (sim_np(sim, "ball_grabbed")[:, 0, 0] == 0)).any())
        prev_oob = gs[:, 11].copy()
    assert all(seen.values()), seen


def test_non_canonical_teams_take_the_generic_obs_path():
    """A Team edit that leaves the opponent slot empty exercises the 37-float
    padding path of fillObservations (game.cpp:1428-1437)."""
    W = 8
    sim = make_sim(ExecMode.CPU, W)
    o = Oracle(W)
    team = sim_np(sim, "team").copy()
    team[::2, 1, 0] = 0  # even worlds: both agents on team 0
    sim.agent_team_tensor().to_torch().copy_(torch.from_numpy(team))
    o.import_("team", team)
    run_lockstep(sim, o, 300, check_every=10)


def test_env_reset_pattern_and_pokes():
    """scripts/env.py:178-185 (resets.fill_(1); step; fill_(0)),
    trigger_reset (mgr.cpp:297-311), set_action (mgr.cpp:270-293)."""
    W = 16
    sim = make_sim(ExecMode.CPU, W)
    o = Oracle(W)
    resets = sim.reset_tensor().to_torch()
    for t in range(200):
        if t % 29 == 0:
            resets.fill_(1)
            o.import_("reset", np.ones((W, 2, 1), np.int32))
        sim.write_random_actions(3, t)
        o.random_actions(3, t)
        if t == 40:
            sim.set_action(2, 0, 1, 3, 2, 1, 1, 0)
            a = o.export("action")
            a[2, 0] = [1, 3, 2, 1, 1, 0]
            o.set_actions(a)
        if t == 77:
            sim.trigger_reset(4)
            sim.trigger_reset(W + 5)  # out of range: ignored, as in the reference
            r = o.export("reset")
            r[4] = 1
            o.import_("reset", r)
        sim.step()
        o.step()
        if t % 29 == 0:
            resets.fill_(0)
            o.import_("reset", np.zeros((W, 2, 1), np.int32))
        bad, _ = compare(sim, o)
        assert not bad, (t, bad)
        if 77 <= t < 86:
            # Reset flag only marks done and zeroes CurStep (game.cpp:978-980);
            # it does not regenerate the world, so it stays set every step
            assert (sim_np(sim, "done")[4] == 1).all()
            assert (sim_np(sim, "cur_step")[4] == 0).all()


def test_set_action_bad_index_reports(capsys):
    sim = make_sim(ExecMode.CPU, 2)
    sim.set_action(5, 0, 1, 1, 1, 1, 1, 1)
    assert "Invalid indices" in capsys.readouterr().out


def test_sharded_worlds_equal_unsharded():
    """World-level sharding (bench --gpus N): a world's trajectory depends only
    on its global index, so shards concatenate to the unsharded run."""
    W = 64
    full = make_sim(ExecMode.CPU, W, per_world_rng=True)
    parts = [make_sim(ExecMode.CPU, W // 4, per_world_rng=True, world_offset=k * W // 4) for k in range(4)]
    full.step_n(300, random_actions=True, action_seed=17)
    for p in parts:
        p.step_n(300, random_actions=True, action_seed=17)
    for n in ("agent_pos", "observations", "game_state", "reward", "done", "rng_counter"):
        cat = np.concatenate([sim_np(p, n) for p in parts])
        assert np.array_equal(cat.view(np.uint32), sim_np(full, n).view(np.uint32)), n


def test_snapshot_restore_replays_identically():
    sim = make_sim(ExecMode.CPU, 32, per_world_rng=True)
    sim.step_n(50, random_actions=True, action_seed=1)
    snap = sim.snapshot()
    sim.step_n(100, random_actions=True, action_seed=1, step0=50)
    a = {k: v.clone() for k, v in sim.snapshot().items()}
    sim.restore(snap)
    sim.step_n(100, random_actions=True, action_seed=1, step0=50)
    for k, v in sim.snapshot().items():
        assert torch.equal(v.view(torch.int32), a[k].view(torch.int32)), k
