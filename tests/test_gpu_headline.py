"""The headline kernel at the length the bench times, and env.py's exact call
sequence on the GPU (VERDICT r5 "next round" items 1 and 6).

bench.py times the staged steps as ONE launch of the resident loop
(k_rollout<2, 2, 1, true> at 65 536 worlds): 100 warmup steps in one launch,
then 1 000 timed steps in a second.  Every world reaches the 620-live-step
clock expiry (src/game.cpp:1009-1020) and its resetWorld (src/gen.cpp:216-316)
inside those launches, so the tests here run the same chained launches and
check them, column by column, against one k_step launch per step, and a sample
of worlds against the oracle replaying them by global world index.  The same
at 262 144 worlds (beyond the Infinity Cache) for 700 steps, and for the two
other resident kernels a grid size picks (k_rollout<2, 1, 1, true> at 32 768
worlds, k_rollout_split<2, true> at 8 192).
"""
import numpy as np
import pytest
import torch

from madrona_basketball_amd import ExecMode, _lib
from oracle.oracle import Oracle
from tests.helpers import ALL_COLUMNS, compare, make_sim, oracle_flags

pytestmark = pytest.mark.gpu
SEED = 321


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(native_lib, oracle_lib):
    assert torch.cuda.is_available(), "GPU tests selected but no HIP device is visible"


def staged_run(W, chunks, kind, agents=2):
    """A simulator stepped through bb_step_n_staged in `chunks` = [(steps,
    step0)] (one call each), with the staged launch kind forced (None: the
    product's rule); returns the simulator and every chunk's staged rows after
    the call (with the defence AI's overrides written back)."""
    sim = make_sim(ExecMode.CUDA, W, num_agents=agents, per_world_rng=True)
    rows = []
    with _lib.diag(**({} if kind is None else {"step_loop": kind})):
        for n, step0 in chunks:
            acts = sim.stage_random_actions(n, action_seed=SEED, step0=step0)
            if kind == 2:
                assert _lib.load().bb_step_staged_path(sim._h, n) == 2
            sim.step_n_staged(acts)
            rows.append(acts)
    torch.cuda.synchronize()
    return sim, rows


def sampled_worlds_match_oracle(sim, W, steps, count=16, agents=2):
    rng = np.random.default_rng(W)
    worlds = [0, W - 1] + [int(w) for w in rng.choice(np.arange(1, W - 1), size=count - 2, replace=False)]
    for w in worlds:
        o = Oracle(1, num_agents=agents, flags=oracle_flags(per_world_rng=True), world_offset=w)
        for t in range(steps):
            o.random_actions(SEED, t)
            o.step()
        bad, _ = compare(sim, o, world=w)
        assert not bad, (w, bad)


@pytest.mark.parametrize("W,kernel", [(65536, "bb::k_rollout<2, 2, 1, true>"), (32768, "bb::k_rollout<2, 1, 1, true>"),
                                      (8192, "bb::k_rollout_split<2, true>")])
def test_gpu_resident_loop_bench_length_chained_launches(W, kernel):
    """bench.py's headline shape: a 100-step resident launch, then a 1 000-step
    one (each world crosses the clock-expiry reset inside the second) ==
    1 100 k_step launches, every column and every staged write-back; 16
    worlds == the oracle."""
    chunks = [(100, 0), (1000, 100)]
    probe = make_sim(ExecMode.CUDA, W, per_world_rng=True)
    assert _lib.kernel_name(probe._h, 1, 1000) == kernel
    del probe
    a, rows_a = staged_run(W, chunks, 2)
    b, rows_b = staged_run(W, chunks, 0)
    for name in a._views:
        assert torch.equal(a._views[name], b._views[name]), name
    for ra, rb in zip(rows_a, rows_b):
        assert torch.equal(ra, rb), "staged write-backs"
    # every world reset inside the timed launch (clock expiry at <= 620 live steps)
    cur = a.internal_tensor("cur_step")
    assert int(cur.max()) < 1000, int(cur.max())
    assert int((a._views["rng_counter"] > 0).sum()) == W  # every world drew from its RNG
    del rows_a, rows_b, b
    sampled_worlds_match_oracle(a, W, 1100)


def test_gpu_resident_loop_beyond_the_cache_700_steps():
    """262 144 worlds (436 MB of state and rows: beyond the Infinity Cache),
    700 steps in one resident launch == 700 k_step launches; 16 worlds ==
    the oracle."""
    W = 262144
    a, rows_a = staged_run(W, [(700, 0)], 2)
    b, rows_b = staged_run(W, [(700, 0)], 0)
    for name in a._views:
        assert torch.equal(a._views[name], b._views[name]), name
    assert torch.equal(rows_a[0], rows_b[0])
    assert int(a.internal_tensor("cur_step").max()) < 700
    del rows_a, rows_b, b
    sampled_worlds_match_oracle(a, W, 700)


@pytest.mark.parametrize("agents,kernel", [(4, "bb::k_rollout_shared<4, true>"), (10, "bb::k_step_loop<10>")])
def test_gpu_more_agents_bench_configs_at_bench_length(agents, kernel):
    """The bench line's 65 536 x 4 ("2v2", the resident shared-world loop) and
    65 536 x 10 ("5v5", C5: the reloading step loop) objects at their timed
    length: 20 + 200 staged steps in two launches, as bench.py's config lines
    run them == 220 k_step launches on every column and staged write-back; 8
    worlds == the oracle."""
    W, chunks = 65536, [(20, 0), (200, 20)]
    probe = make_sim(ExecMode.CUDA, W, num_agents=agents, per_world_rng=True)
    assert _lib.kernel_name(probe._h, 1, 200) == kernel
    del probe
    a, rows_a = staged_run(W, chunks, None, agents)
    b, rows_b = staged_run(W, chunks, 0, agents)
    for name in a._views:
        assert torch.equal(a._views[name], b._views[name]), name
    for ra, rb in zip(rows_a, rows_b):
        assert torch.equal(ra, rb), "staged write-backs"
    del rows_a, rows_b, b
    torch.cuda.empty_cache()
    sampled_worlds_match_oracle(a, W, 220, count=8, agents=agents)


@pytest.mark.parametrize("agent_idx", [0, 1])
def test_gpu_env_py_call_sequence_matches_oracle(agent_idx):
    """scripts/env.py's calls on ExecMode.CUDA, issued on a non-default torch
    stream: int64 trainee actions slice-assigned into actions[:, agent_idx]
    (env.py:147), step() (env.py:155), the three .clone()s (env.py:167-170);
    reset = resets.fill_(1) / step / fill_(0) every 33 steps (env.py:178-185,
    ppo.py's rollout).  The clones and every column == the oracle."""
    W = 4096
    sim = make_sim(ExecMode.CUDA, W)
    o = Oracle(W)
    observations = sim.observations_tensor().to_torch()
    actions = sim.action_tensor().to_torch()
    dones = sim.done_tensor().to_torch()
    rewards = sim.reward_tensor().to_torch()
    resets = sim.reset_tensor().to_torch()
    buckets = [2, 8, 3, 2, 2, 2]
    gen = torch.Generator().manual_seed(agent_idx)
    side = torch.cuda.Stream()

    def env_step(trainee_cpu):
        trainee = trainee_cpu.to(sim.device, non_blocking=False)  # int64, as the policy returns it
        actions[:, agent_idx] = trainee
        a = o.export("action")
        a[:, agent_idx] = trainee_cpu.numpy()
        o.set_actions(a)
        sim.step()
        o.step()
        return (observations[:, agent_idx].detach().clone(), rewards[:, agent_idx].detach().clone(),
                dones[:, agent_idx].detach().clone())

    def env_reset():
        resets.fill_(1)
        o.import_("reset", np.ones((W, 2, 1), np.int32))
        out = env_step(torch.zeros((W, 6), dtype=torch.int64))
        resets.fill_(0)
        o.import_("reset", np.zeros((W, 2, 1), np.int32))
        return out

    def check(out):
        obs, rew, done = (x.cpu().numpy() for x in out)
        np.testing.assert_allclose(obs, o.export("observations")[:, agent_idx], atol=1e-5, rtol=1e-6)
        np.testing.assert_allclose(rew, o.export("reward")[:, agent_idx], atol=1e-5, rtol=1e-6)
        assert np.array_equal(done, o.export("done")[:, agent_idx])

    with torch.cuda.stream(side):
        for it in range(8):  # ppo.py's rollouts: reset + 32 steps
            out = env_reset()
            side.synchronize()
            assert (out[2] == 1).all()
            check(out)
            for t in range(32):
                trainee = torch.stack([torch.randint(0, b, (W,), generator=gen) for b in buckets], dim=-1)
                out = env_step(trainee)
                side.synchronize()
                check(out)
            bad, _ = compare(sim, o)
            assert not bad, (it, bad)


@pytest.mark.parametrize("W", [4194304, 4194303])
def test_gpu_maximum_size_staged_and_per_call(W):
    """Maximum sizes: 4 194 304 worlds (7 GB of state and rows, 8.4 M agent
    rows) and a ragged 4 194 303 -- the resident loop (one launch, 24 steps) ==
    24 k_step launches in every column and write-back, and sampled worlds
    (the last one included) == the oracle."""
    a, rows_a = staged_run(W, [(24, 0)], 2)
    b, rows_b = staged_run(W, [(24, 0)], 0)
    for name in a._views:
        assert torch.equal(a._views[name], b._views[name]), name
    assert torch.equal(rows_a[0], rows_b[0])
    del rows_a, rows_b, b
    torch.cuda.empty_cache()
    sampled_worlds_match_oracle(a, W, 24, count=8)
