"""Forced rare-path scenarios on the gfx950 kernels.

The scripted scenarios of tests/scenarios.py drive the branches random play
never reaches -- full-game inbound / turnover / 5-s violation
(src/game.cpp:14-53, 1083-1111, 1116-1157), the full-game make -> inbound
(game.cpp:905-950), end-of-period and game-over resets (src/gen.cpp:221-236),
the padded observation row (game.cpp:1428-1437) -- through every kernel the
product ships, in lockstep with the oracle:

  step     k_step<2>       agent lanes + DPP exchange (one launch per step)
  rollout  k_rollout<2>    registers-resident world, one K=1 launch per step
  shared4  k_step<4>       world in LDS shared by its agent lanes
  shared10 k_step<10>      same kernel family, 5v5

and through bb_step_n_staged's multi-step launches, the scenario's actions
(closed-loop on the oracle's state) staged in chunks of CHUNK steps, every
column checked after each chunk:

  staged_split   k_rollout_split<2, true>    resident loop, sim wave + row wave
  staged_minw1   k_rollout<2, 1, 1, true>    resident loop, whole register file
  staged_minw2   k_rollout<2, 2, 1, true>    resident loop, the bench's kernel
  staged_loop    k_step_loop<2>              reloading loop
  staged4        k_rollout_shared<4, true>   resident loop, world in LDS
  staged10       k_rollout_shared<10, true>

Each test also asserts, from the oracle's event counters, that the branch
under test was actually taken (count > 0).
"""
import numpy as np
import pytest
import torch

from madrona_basketball_amd import ExecMode
from oracle.oracle import Oracle
from tests.helpers import compare, make_sim, oracle_flags

pytestmark = pytest.mark.gpu

KERNELS = [("step", 2), ("rollout", 2), ("shared4", 4), ("shared10", 10), ("staged_split", 2), ("staged_minw1", 2),
           ("staged_minw2", 2), ("staged_loop", 2), ("staged4", 4), ("staged10", 10)]
CHUNK = 16
# the path overrides that make bb_step_n_staged launch each staged kernel on
# the scenarios' small grids, and the kernel that must then be launched
STAGED = {
    "staged_split": (dict(step_loop=2), "bb::k_rollout_split<2, true>"),
    "staged_minw1": (dict(step_loop=2, rollout_split=0), "bb::k_rollout<2, 1, 1, true>"),
    "staged_minw2": (dict(step_loop=2, rollout_split=0, rollout_minw=2), "bb::k_rollout<2, 2, 1, true>"),
    "staged_loop": (dict(step_loop=1), "bb::k_step_loop<2>"),
    "staged4": (dict(step_loop=2), "bb::k_rollout_shared<4, true>"),
    "staged10": (dict(step_loop=2), "bb::k_rollout_shared<10, true>"),
}
KERNEL_IDS = [k for k, _ in KERNELS]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(native_lib, oracle_lib):
    assert torch.cuda.is_available(), "GPU tests selected but no HIP device is visible"


class Driver:
    """Steps a CUDA simulator through the chosen kernel with the same actions
    as the oracle, and checks every column (and, for the rollout kernel, the
    recorded outputs) when `check` is set -- one step at a time, or for the
    staged kernels in chunks of CHUNK steps through bb_step_n_staged (the
    oracle steps at once, so the scenario's closed-loop actions come from
    its state; every column is checked after each chunk and by finish())."""

    def __init__(self, kernel: str, sim, oracle: Oracle):
        self.kernel, self.sim, self.o = kernel, sim, oracle
        if kernel == "rollout":
            self.buf = sim.rollout_buffers(1)
        self.pending, self.oracle_rows = [], []
        self.chunks = 0

    def _flush(self, t):
        from madrona_basketball_amd import _lib
        if not self.pending:
            return
        overrides, kernel = STAGED[self.kernel]
        staged = torch.tensor(np.stack(self.pending), device=self.sim.device)
        with _lib.diag(**overrides):
            if len(self.pending) >= 2:
                assert _lib.kernel_name(self.sim._h, 1, len(self.pending)) == kernel
                self.chunks += 1
            self.sim.step_n_staged(staged)
        bad, _ = compare(self.sim, self.o)
        assert not bad, f"{self.kernel} chunk ending at step {t}: {bad}"
        # the defence AI's overrides written back into the staged rows == the
        # oracle's action column after each of those steps
        assert np.array_equal(staged.cpu().numpy(), np.stack(self.oracle_rows)), (t, "staged write-backs")
        self.pending, self.oracle_rows = [], []

    def finish(self, t: int = -1):
        if self.kernel in STAGED:
            self._flush(t)
            assert self.chunks > 0

    def step(self, actions: np.ndarray, t: int, check: bool = True):
        sim, o = self.sim, self.o
        if self.kernel in STAGED:
            self.pending.append(np.asarray(actions, dtype=np.int32).copy())
            o.set_actions(actions)
            o.step()
            self.oracle_rows.append(o.export("action").copy())
            if len(self.pending) == CHUNK:
                self._flush(t)
            return
        a = torch.tensor(np.asarray(actions, dtype=np.int32), device=sim.device)  # a copy (overrides land in it)
        if self.kernel == "rollout":
            staged = a[None].contiguous()
            sim.rollout(staged, self.buf["obs"], self.buf["reward"], self.buf["done"])
        else:
            sim.action_tensor().to_torch().copy_(a)
            sim.step()
        o.set_actions(actions)
        o.step()
        if not check:
            return
        bad, _ = compare(sim, o)
        assert not bad, f"{self.kernel} step {t}: {bad}"
        if self.kernel == "rollout":
            for name, key in (("observations", "obs"), ("reward", "reward"), ("done", "done")):
                got = self.buf[key][0].cpu().numpy()
                exp = o.export(name)
                assert np.allclose(got, exp, atol=1e-5, rtol=1e-6), (t, name)
            assert np.array_equal(staged[0].cpu().numpy(), o.export("action")), (t, "action written back")


@pytest.mark.parametrize("kernel,n", KERNELS, ids=KERNEL_IDS)
def test_gpu_full_game_inbound_violation_pass(kernel, n):
    """grab -> shot out of bounds -> turnover inbound (game.cpp:1083-1111) ->
    5-s inbound violation turnover (game.cpp:1116-1157) -> pass."""
    from tests.scenarios import FullGameInbound
    W = 6
    sim = make_sim(ExecMode.CUDA, W, num_agents=n, tag_mask=False, one_on_one=False)
    o = Oracle(W, num_agents=n, flags=oracle_flags(tag_mask=False, one_on_one=False))
    sc = FullGameInbound(W, n)
    sc.prepare(o, sim.internal_tensor("attributes"))
    d = Driver(kernel, sim, o)
    for t in range(1000):
        d.step(sc.actions(o, t), t, check=(t % 5 == 0 or t > 590))
    d.finish()
    ev = o.events()
    for k in ("grab", "shot", "oob_turnover", "inbound_start", "inbound_violation", "pass"):
        assert ev[k] > 0, (k, ev)


@pytest.mark.parametrize("kernel,n", KERNELS, ids=KERNEL_IDS)
def test_gpu_full_game_make_then_inbound(kernel, n):
    """Carry the ball to the hoop and shoot: the full-game branch of
    scoreSystem (score, baseline spot, assignInbounder, game.cpp:905-950),
    then the inbounder's pass.  At 10 agents the carrier is tagged on the way
    (contact path) instead; both are checked against the oracle."""
    from tests.scenarios import FullGameScore
    W = 6
    sim = make_sim(ExecMode.CUDA, W, num_agents=n, tag_mask=False, one_on_one=False)
    o = Oracle(W, num_agents=n, flags=oracle_flags(tag_mask=False, one_on_one=False))
    sc = FullGameScore(W, n)
    sc.prepare(o, sim.internal_tensor("attributes"))
    d = Driver(kernel, sim, o)
    for t in range(700):
        d.step(sc.actions(o, t), t, check=(t % 5 == 0))
    d.finish()
    ev = o.events()
    if n <= 4:
        for k in ("grab", "shot_going_in", "make", "inbound_start", "pass"):
            assert ev[k] > 0, (k, ev)
    else:
        assert ev["grab"] > 0 and ev["tag"] > 0, ev


@pytest.mark.parametrize("kernel,n", KERNELS, ids=KERNEL_IDS)
def test_gpu_full_game_period_and_game_end(kernel, n):
    """No one moves in a full game: the clock expiry takes the end-of-period
    branch of resetWorld; worlds started in period 4 with unequal scores take
    the game-over branch (liveBall = 0, gen.cpp:221-236) and then stand
    still."""
    W = 4
    sim = make_sim(ExecMode.CUDA, W, num_agents=n, one_on_one=False)
    o = Oracle(W, num_agents=n, flags=oracle_flags(one_on_one=False))
    gs = o.export("game_state")
    gs[2:, 2] = 4.0   # period 4
    gs[2:, 5] = 3.0   # team 0 leads 3 - 0
    o.import_("game_state", gs)
    sim.game_state_tensor().to_torch().copy_(torch.from_numpy(gs).to(sim.device))
    d = Driver(kernel, sim, o)
    zeros = np.zeros((W, n, 6), np.int32)
    for t in range(1400):
        d.step(zeros, t, check=(t % 10 == 0 or 610 <= t <= 630 or 1235 <= t <= 1250))
    d.finish()
    ev = o.events()
    assert ev["period_advance"] > 0 and ev["game_end"] > 0 and ev["clock_expiry"] > 0, ev
    g = sim.game_state_tensor().to_torch().cpu().numpy()
    assert (g[:2, 2] >= 3).all()                    # two periods advanced
    assert (g[2:].view(np.int32)[:, 1] == 0).all()  # game over: ball dead


@pytest.mark.parametrize("kernel,n", KERNELS, ids=KERNEL_IDS)
def test_gpu_non_canonical_teams_padded_rows(kernel, n):
    """A Team edit that leaves opponent slots empty: the 37-float padding path
    of fillObservations (game.cpp:1428-1437) and the generic row writer."""
    W = 64
    sim = make_sim(ExecMode.CUDA, W, num_agents=n, per_world_rng=True)
    o = Oracle(W, num_agents=n, flags=oracle_flags(per_world_rng=True))
    team = o.export("team")
    team[::2, 1, 0] = 0  # even worlds: agent 1 joins team 0
    sim.agent_team_tensor().to_torch().copy_(torch.from_numpy(team).to(sim.device))
    o.import_("team", team)
    d = Driver(kernel, sim, o)
    gen = np.random.default_rng(12)
    hi = np.array([2, 8, 3, 2, 2, 2])
    for t in range(300):
        a = (gen.random((W, n, 6)) * hi).astype(np.int32)
        d.step(a, t, check=(t % 10 == 0))
    d.finish()
    assert o.events()["obs_padded_row"] > 0


@pytest.mark.parametrize("kernel", ["step", "rollout", "staged_split", "staged_minw1", "staged_minw2", "staged_loop"])
def test_gpu_single_world_scripted_config0(kernel):
    """configs[0] on the GPU kernels: 1 world, scripted actions, 700 steps
    (clock expiry at step 620, +10 to the offence, done), every step checked."""
    sim = make_sim(ExecMode.CUDA, 1)
    o = Oracle(1)
    script = np.zeros((700, 1, 2, 6), np.int32)
    script[5:60, 0, 0] = [1, 2, 0, 0, 0, 0]
    script[60:80, 0, 0] = [1, 6, 1, 0, 0, 0]
    script[80, 0, 0] = [0, 0, 0, 0, 0, 1]
    script[200:260, 0, 1] = [1, 4, 2, 1, 1, 1]
    d = Driver(kernel, sim, o)
    for t in range(700):
        d.step(script[t], t)
    d.finish()
    ev = o.events()
    assert ev["shot"] == 1 and ev["world_reset"] >= 1, ev
