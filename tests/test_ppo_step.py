"""k_rollout_ppo<2> / k_step_ppo<2>: PPO's rollout loop with the trainee's
policy pass fused behind the world step (bb_rollout_policy above 16 384 worlds;
scripts/ppo.py:65-134 over scripts/env.py:126-170), the whole rollout in one
launch (each wave steps its worlds K times; default) or one launch per step
(the ppo_step_loop path override = 0).  Every recorded output
(buffer.obs / actions / log_probs / values / rewards / not_dones, next_value)
and every simulator column must equal the per-step launches (k_policy +
k_step, the `per_step` flag) and the loop of FusedPolicy.act + step, bit for
bit: the row passes feed layer 1's MFMA chain in its own k order, so the
policy sees the same floats in the same order.

The fused step is taken by row count: small and ragged grids run it with the
path overrides ppo_step_fused_min_worlds = 1 and ppo_fused_max_worlds = 0
(partial waves, inactive waves of the last workgroup, 4-wave workgroups)."""
import pytest
import torch

from madrona_basketball_amd import ExecMode, _lib
from madrona_basketball_amd.policy import FusedPolicy, make_agent
from tests.helpers import make_sim
from tests.test_policy_rollout import assert_same, reference_loop, run_pair



def fused_vs_per_step(W, n, trainee, stochastic, seed=7, step0=3, partial=False, flags=None):
    sims = [make_sim(ExecMode.CUDA, W, per_world_rng=True, **(flags or {})) for _ in range(2)]
    for s in sims:
        s.step_n(9, random_actions=True, action_seed=321, step0=0)
    pol = FusedPolicy.from_agent(make_agent(5).cuda())
    bufs = [pol.rollout_buffers(s, n) for s in sims]
    if partial:  # value / reward / done only (buffer.obs, actions, log-probs not recorded)
        bufs = [{k: b[k] for k in ("value", "reward", "done", "next_value")} for b in bufs]
    pol.rollout(sims[0], n, bufs[0], trainee=trainee, stochastic=stochastic, seed=seed, step0=step0)
    pol.rollout(sims[1], n, bufs[1], trainee=trainee, stochastic=stochastic, seed=seed, step0=step0, per_step=True)
    torch.cuda.synchronize()
    assert_same(bufs[0], bufs[1])
    for name in sims[0]._views:
        assert torch.equal(sims[0]._views[name], sims[1]._views[name]), name
    return bufs[0]


@pytest.mark.gpu
@pytest.mark.parametrize("W,n,trainee,stochastic", [(65536, 6, 0, True), (65536, 5, 1, False),
                                                    (65536, 32, 1, True), (32768, 8, 1, True),
                                                    (40001, 4, 0, True), (131072, 3, 0, False),
                                                    (24576, 6, 1, True), (16385, 4, 0, False)])
def test_gpu_fused_ppo_step_equals_per_step_launches(native_lib, W, n, trainee, stochastic):
    assert torch.cuda.is_available()
    b = fused_vs_per_step(W, n, trainee, stochastic)
    assert b["obs"].abs().sum() > 0 and (b["actions"] != 0).any()


@pytest.mark.gpu
def test_gpu_fused_ppo_step_partial_outputs(native_lib):
    """Only value / reward / done / next_value recorded (no buffer.obs): the
    policy still reads its rows from LDS, the outputs equal the per-step loop's."""
    assert torch.cuda.is_available()
    fused_vs_per_step(65536, 4, 0, True, partial=True)


@pytest.mark.gpu
def test_gpu_fused_ppo_step_equals_the_ppo_loop(native_lib):
    """At 40 000 worlds (4-wave workgroups) == FusedPolicy.act + step per step."""
    assert torch.cuda.is_available()
    run_pair(ExecMode.CUDA, 40000, 5, 1, True, False, "cuda")


@pytest.mark.gpu
def test_gpu_fused_ppo_step_single_step(native_lib):
    """n = 1: the policy pass of step 0, then the last step's value pass only."""
    assert torch.cuda.is_available()
    fused_vs_per_step(65536, 1, 1, True)


@pytest.mark.gpu
def test_gpu_fused_ppo_step_forced_on_small_grids(native_lib):
    with _lib.diag(ppo_step_fused_min_worlds=1, ppo_fused_max_worlds=0):
        for W, n, trainee, stoch in [(1000, 6, 1, True), (64, 3, 0, False), (12345, 5, 0, True), (31, 4, 1, True),
                                     (8192, 4, 0, True)]:
            fused_vs_per_step(W, n, trainee, stoch)


@pytest.mark.gpu
def test_gpu_fused_ppo_step_one_launch_per_step(native_lib):
    """ppo_step_loop = 0: one k_step_ppo launch per step, equal to the
    per-step launches (and so to the one-launch rollout)."""
    with _lib.diag(ppo_step_loop=0):
        for W, n, trainee, stoch in [(65536, 6, 1, True), (40001, 4, 0, True), (65536, 1, 0, False)]:
            fused_vs_per_step(W, n, trainee, stoch)


@pytest.mark.gpu
@pytest.mark.parametrize("W,n,flags", [(8192, 700, {}), (65536, 640, {}),
                                       (4096, 300, dict(one_on_one=False, tag_mask=False)),
                                       (2000, 200, dict(tag_mask=False))])
def test_gpu_fused_ppo_step_long_rollouts_and_full_game(native_lib, W, n, flags):
    """k_rollout_ppo as one launch over 640-700 steps (every world crosses the
    620-step clock expiry and its resetWorld inside the launch), and on the
    full-game / grab-and-pass rules (one_on_one=False, tag_mask=False), ==
    k_policy + k_step per step, every record and every column."""
    with _lib.diag(ppo_step_fused_min_worlds=1, ppo_fused_max_worlds=0):
        sims_probe = make_sim(ExecMode.CUDA, W, per_world_rng=True, **flags)
        assert _lib.load().bb_rollout_policy_path(sims_probe._h, 0, 0) == 2  # BB_PPO_PATH_FUSED_STEP
        del sims_probe
        b = fused_vs_per_step(W, n, 0, True, flags=flags)
    assert (b["done"] == 1).any()  # resets happened inside the launch


@pytest.mark.gpu
def test_gpu_fused_ppo_step_on_a_side_stream(native_lib):
    """Issued on a torch side stream: clones enqueued on that stream right after
    the call see every record and the final state, equal to the PPO loop."""
    assert torch.cuda.is_available()
    W, n = 65536, 3
    sims = [make_sim(ExecMode.CUDA, W, per_world_rng=True) for _ in range(2)]
    for s in sims:
        s.step_n(5, random_actions=True, action_seed=321, step0=0)
    torch.cuda.synchronize()
    pol = FusedPolicy.from_agent(make_agent(6).cuda())
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        bufs = pol.rollout_buffers(sims[0], n)
        pol.rollout(sims[0], n, bufs, stochastic=True, seed=9, step0=2)
        snap = {k: v.clone() for k, v in bufs.items()}
        views = {k: v.clone() for k, v in sims[0]._views.items()}
    ref = reference_loop(sims[1], pol, n, stochastic=True, seed=9, step0=2)
    torch.cuda.synchronize()
    assert_same(snap, ref)
    for name in views:
        assert torch.equal(views[name], sims[1]._views[name]), name
