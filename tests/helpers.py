"""Shared comparison helpers for the parity tests (oracle = checker only)."""
from __future__ import annotations

import numpy as np
import torch

from oracle.oracle import Oracle

ALL_COLUMNS = [
    "reset", "game_state", "action", "action_mask", "agent_pos", "observations", "reward", "done",
    "agent_entity_id", "agent_possession", "orientation", "team", "agent_stats", "ball_pos",
    "ball_physics", "ball_entity_id", "ball_grabbed", "ball_velocity", "hoop_pos",
    "agent_velocity", "grab_cooldown", "cur_step", "inbounding", "attributes", "world_clock",
    "rng_counter",
]
# Columns whose payload is integer (or integer-valued) state: must match exactly.
# game_state mixes int and float fields (scores and flags are exact; clocks are
# compared exactly too since they are pure repeated subtraction).
EXACT_COLUMNS = {
    "reset", "game_state", "action", "action_mask", "done", "agent_entity_id", "agent_possession",
    "team", "agent_stats", "ball_physics", "ball_entity_id", "ball_grabbed", "cur_step",
    "inbounding", "world_clock", "rng_counter", "hoop_pos",
}
# Float tolerance of north_star ("within 1e-5 on float positions").
FLOAT_ATOL = 1e-5


def sim_np(sim, name: str, world=None) -> np.ndarray:
    v = sim._views[name]
    if world is not None:
        v = v[world:world + 1]
    return v.detach().cpu().numpy()


def compare(sim, oracle: Oracle, names=ALL_COLUMNS, atol: float = FLOAT_ATOL, world=None):
    """Return ({name: description} of mismatches, {name: bit-identical fraction}).
    world: compare only that world of the simulator with a one-world oracle
    (Oracle(1, world_offset=world), the same global world index)."""
    bad, ident = {}, {}
    for n in names:
        a = sim_np(sim, n, world)
        b = oracle.export(n)
        if a.shape != b.shape:
            bad[n] = f"shape {a.shape} vs {b.shape}"
            continue
        same_bits = a.view(np.uint32) == b.view(np.uint32)
        ident[n] = float(same_bits.mean()) if same_bits.size else 1.0
        if n in EXACT_COLUMNS or a.dtype != np.float32:
            ok = same_bits | (a == b)  # +0 / -0
            if not ok.all():
                idx = np.argwhere(~ok)[:3].tolist()
                bad[n] = f"exact mismatch at {idx}"
        else:
            diff = np.abs(a.astype(np.float64) - b.astype(np.float64))
            both_nan = np.isnan(a) & np.isnan(b)
            tol = atol + 1e-6 * np.abs(b.astype(np.float64))
            ok = (diff <= tol) | both_nan
            if not ok.all():
                idx = np.argwhere(~ok)[:3].tolist()
                bad[n] = f"max |diff| {np.nanmax(diff):.3g} at {idx}"
    return bad, ident


def make_sim(mode, num_worlds, num_agents=2, **kw):
    import madrona_basketball_amd as m
    from oracle.oracle import ENV_DISCRETE_X, ENV_DISCRETE_Y, ENV_START_X, ENV_START_Y
    return m.SimpleGridworldSimulator(
        discrete_x=ENV_DISCRETE_X, discrete_y=ENV_DISCRETE_Y, start_x=ENV_START_X, start_y=ENV_START_Y,
        max_episode_length=39600, exec_mode=mode, num_worlds=num_worlds, gpu_id=0,
        num_agents=num_agents, **kw)


def oracle_flags(per_world_rng=False, tag_mask=True, one_on_one=True):
    from oracle import oracle as O
    return ((O.FLAG_PER_WORLD_RNG if per_world_rng else 0) | (0 if tag_mask else O.FLAG_NO_TAG_MASK)
            | (0 if one_on_one else O.FLAG_FULL_GAME))


def sparse_actions(oracle: Oracle, p_act: float = 0.02, seed: int = 5):
    """actions_fn of a mostly idle offence: agent 0 of every world stands still
    with probability 1 - p_act, else takes a uniform action over the
    [2,8,3,2,2,2] buckets; the other agents keep the actions the defence AI
    wrote (hardCodeDefenseSystem, game.cpp:651-755), so it reaches the
    offender and tags it (agentCollisionSystem)."""
    rng = np.random.default_rng(seed)
    hi = np.array([2, 8, 3, 2, 2, 2])

    def fn(t):
        a = oracle.export("action").copy()
        W = a.shape[0]
        r = (rng.random((W, 6)) * hi).astype(np.int32)
        r[rng.random(W) >= p_act] = 0
        a[:, 0] = r
        return a
    return fn


def count_tags(oracle: Oracle) -> int:
    """Worlds whose offender was just tagged (-10 / +10 pair, game.cpp:626-629)."""
    r = oracle.export("reward")
    return int(((r <= -9.0).any(axis=1) & (r >= 9.0).any(axis=1)).sum())


def run_lockstep(sim, oracle: Oracle, steps: int, seed: int = 321, check_every: int = 50,
                 actions_fn=None, atol: float = FLOAT_ATOL, step0: int = 0, on_step=None):
    """Drive sim and oracle with identical actions; assert parity every
    `check_every` steps and at the end.  actions_fn(t) -> int32 array
    [W,N,6] or None for the synthetic threefry workload; on_step(t) is
    called after each step (e.g. to count events on the oracle)."""
    worst = {}
    for t in range(steps):
        if actions_fn is None:
            sim.write_random_actions(seed, step0 + t)
            oracle.random_actions(seed, step0 + t)
        else:
            a = actions_fn(t)
            if a is not None:
                sim.action_tensor().to_torch().copy_(torch.from_numpy(np.ascontiguousarray(a)))
                oracle.set_actions(a)
        sim.step()
        oracle.step()
        if on_step is not None:
            on_step(t)
        if (t + 1) % check_every == 0 or t + 1 == steps:
            bad, ident = compare(sim, oracle, atol=atol)
            assert not bad, f"step {t + 1}: {bad}"
            for k, v in ident.items():
                worst[k] = min(worst.get(k, 1.0), v)
    return worst
