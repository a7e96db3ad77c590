"""PPO's rollout on the device (bb_rollout_policy, FusedPolicy.rollout) vs the
loop it replaces, scripts/ppo.py:61-141 over scripts/env.py:126-170:

    obs = trainee observations
    for k in range(n):
        actions, log_probs, values = agent(obs)     -> FusedPolicy.act (trainee rows)
        [frozen opponent acts]                       -> opponent.act (other rows)
        obs_, rews, dones = env.step(actions)        -> sim.step + clones
        buffer.*[k] = obs, actions, values, log_probs, rews, dones
        obs = obs_
    next_value = agent.evaluate(obs_)

bit for bit (same kernels, same reads), on the host executor and on gfx950; on
step 0 the recorded policy outputs are pinned to the reference's own Agent
through tests/golden/policy_golden.npz (same bars as test_policy_golden.py).
"""
import numpy as np
import pytest
import torch

from madrona_basketball_amd import ExecMode
from madrona_basketball_amd.policy import FusedPolicy, agent_from_state_dict, make_agent
from tests.helpers import make_sim
from tests.test_policy_golden import MIN_DECISIVE, check, load_case


def reference_loop(sim, pol, n, trainee=0, stochastic=True, seed=0, step0=0, opponent=None):
    """The PPO loop with the per-step primitives (FusedPolicy.act + step)."""
    W, dev = sim.num_worlds, sim.device
    obs_t = sim.observations_tensor().to_torch()
    rew_t = sim.reward_tensor().to_torch()
    done_t = sim.done_tensor().to_torch()
    act_t = sim.action_tensor().to_torch()
    out = {k: [] for k in ("obs", "actions", "log_prob", "value", "reward", "done")}
    lp = torch.empty((W,), dtype=torch.float32, device=dev)
    val = torch.empty((W,), dtype=torch.float32, device=dev)
    for k in range(n):
        out["obs"].append(obs_t[:, trainee, :128].clone())
        pol.act(sim, trainee, lp, val, stochastic=stochastic, seed=seed, step=step0 + k)
        out["actions"].append(act_t[:, trainee].clone())
        out["log_prob"].append(lp.clone())
        out["value"].append(val.clone())
        if opponent is not None:
            opponent.act(sim, 1 - trainee, stochastic=True, seed=(seed ^ 0x9E3779B9) & 0xFFFFFFFF, step=step0 + k)
        sim.step()
        out["reward"].append(rew_t[:, trainee].clone())
        out["done"].append(done_t[:, trainee].clone())
    res = {k: torch.stack(v) for k, v in out.items()}
    nv = torch.empty((W,), dtype=torch.float32, device=dev)
    a = torch.empty((W, 6), dtype=torch.int32, device=dev)
    pol.forward_into(obs_t[:, trainee], a, None, nv, stochastic=stochastic, seed=seed, step=step0 + n)
    res["next_value"] = nv
    return res


def assert_same(a: dict, b: dict):
    for k in b:
        x, y = a[k], b[k]
        assert x.shape == y.shape, (k, x.shape, y.shape)
        assert torch.equal(x.cpu().contiguous().view(torch.int32), y.cpu().contiguous().view(torch.int32)), k


def run_pair(mode, W, n, trainee, stochastic, with_opponent, device):
    sims = [make_sim(mode, W, per_world_rng=True) for _ in range(2)]
    for s in sims:
        s.step_n(7, random_actions=True, action_seed=321, step0=0)
    pol = FusedPolicy.from_agent(make_agent(3).to(device))
    opp = FusedPolicy.from_agent(make_agent(4).to(device)) if with_opponent else None
    bufs = pol.rollout_buffers(sims[0], n)
    pol.rollout(sims[0], n, bufs, trainee=trainee, stochastic=stochastic, seed=11, step0=5, opponent=opp)
    ref = reference_loop(sims[1], pol, n, trainee, stochastic, seed=11, step0=5, opponent=opp)
    if device != "cpu":
        torch.cuda.synchronize()
    assert_same(bufs, ref)
    for name in sims[0]._views:  # and the simulators end in the same state
        assert torch.equal(sims[0]._views[name], sims[1]._views[name]), name
    return bufs


@pytest.mark.parametrize("trainee,stochastic,opp", [(0, True, False), (1, False, False), (0, True, True)])
def test_host_policy_rollout_equals_the_ppo_loop(native_lib, trainee, stochastic, opp):
    bufs = run_pair(ExecMode.CPU, 64, 12, trainee, stochastic, opp, "cpu")
    assert bufs["done"].sum() >= 0 and bufs["obs"].abs().sum() > 0


def test_policy_rollout_partial_outputs(native_lib):
    """Outputs left as None are not recorded; the ones given still match."""
    sims = [make_sim(ExecMode.CPU, 32, per_world_rng=True) for _ in range(2)]
    pol = FusedPolicy.from_agent(make_agent(1))
    bufs = pol.rollout_buffers(sims[0], 6)
    part = {"value": bufs["value"], "reward": bufs["reward"], "done": bufs["done"]}
    pol.rollout(sims[0], 6, part, seed=2)
    ref = reference_loop(sims[1], pol, 6, seed=2)
    assert_same(part, {k: ref[k] for k in part})
    with pytest.raises(ValueError):
        pol.rollout(sims[0], 6, {"reward": bufs["reward"]})


@pytest.mark.gpu
@pytest.mark.parametrize("trainee,stochastic,opp", [(0, True, False), (1, False, False), (0, True, True)])
def test_gpu_policy_rollout_equals_the_ppo_loop(native_lib, trainee, stochastic, opp):
    assert torch.cuda.is_available()
    run_pair(ExecMode.CUDA, 8192, 32, trainee, stochastic, opp, "cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("W,n,trainee,stochastic", [(8192, 32, 0, True), (1000, 20, 1, False), (64, 3, 0, True),
                                                    (16384, 16, 1, True), (12345, 8, 0, False)])
def test_gpu_fused_policy_rollout_equals_per_step_launches(native_lib, W, n, trainee, stochastic):
    """The fused PPO rollout kernel (one launch, k_rollout_policy) == a policy
    launch + a step launch per step, every output and every column, bit for bit
    (a partial last workgroup included: W = 1000, 64, 12345; 16 384 = the fused
    kernel's default bound, two workgroups per CU)."""
    assert torch.cuda.is_available()
    sims = [make_sim(ExecMode.CUDA, W, per_world_rng=True) for _ in range(2)]
    for s in sims:
        s.step_n(9, random_actions=True, action_seed=321, step0=0)
    pol = FusedPolicy.from_agent(make_agent(5).cuda())
    bufs = [pol.rollout_buffers(s, n) for s in sims]
    pol.rollout(sims[0], n, bufs[0], trainee=trainee, stochastic=stochastic, seed=7, step0=3)
    pol.rollout(sims[1], n, bufs[1], trainee=trainee, stochastic=stochastic, seed=7, step0=3, per_step=True)
    torch.cuda.synchronize()
    assert_same(bufs[0], bufs[1])
    for name in sims[0]._views:
        assert torch.equal(sims[0]._views[name], sims[1]._views[name]), name


@pytest.mark.gpu
@pytest.mark.parametrize("pw", [2, 4])
def test_gpu_fused_policy_rollout_policy_wave_counts(native_lib, pw):
    """k_rollout_policy with its policy waves forced to 2 (one per M-tile) or 4
    (two per M-tile, one output half each) at any grid (the ppo_pwaves path
    override) == the per-step launches."""
    from madrona_basketball_amd import _lib
    with _lib.diag(ppo_pwaves=pw):
        for W, n, tr, st in [(8192, 12, 1, True), (1000, 10, 0, False), (16384, 6, 0, True)]:
            test_gpu_fused_policy_rollout_equals_per_step_launches(native_lib, W, n, tr, st)


@pytest.mark.gpu
def test_gpu_policy_rollout_at_65536_worlds_equals_the_ppo_loop(native_lib):
    """BASELINE configs[2]'s world count (the bench's ppo_rollout32_65536x2
    line): the default rollout path at 65 536 worlds == FusedPolicy.act +
    step per step, every output and every column."""
    assert torch.cuda.is_available()
    run_pair(ExecMode.CUDA, 65536, 8, 0, True, False, "cuda")


@pytest.mark.gpu
def test_gpu_split_policy_rollout_odd_worlds_with_opponent(native_lib):
    """From 32 768 worlds the per-step rollout runs the two world halves on two
    streams (bb_host.hip, shard_params): an odd count (halves of 20 001 and
    20 000 worlds), the frozen opponent and a deterministic trainee, still ==
    FusedPolicy.act + step per step, every output and every column."""
    assert torch.cuda.is_available()
    run_pair(ExecMode.CUDA, 40001, 6, 1, False, True, "cuda")


@pytest.mark.gpu
def test_gpu_split_policy_rollout_on_a_side_stream(native_lib):
    """The split rollout (from 32 768 worlds: a second stream inside the call)
    issued on a torch side stream: clones enqueued on that stream right after
    the call see every part's records and final state, equal to the PPO loop."""
    assert torch.cuda.is_available()
    W, n = 32768, 4
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


@pytest.mark.gpu
def test_gpu_policy_rollout_equals_host_executor(native_lib):
    """Device rollout == host-executor rollout (policy and step), bit for bit."""
    assert torch.cuda.is_available()
    outs = []
    for mode, dev in ((ExecMode.CUDA, "cuda"), (ExecMode.CPU, "cpu")):
        sim = make_sim(mode, 1024, per_world_rng=True)
        sim.step_n(3, random_actions=True, action_seed=321, step0=0)
        pol = FusedPolicy.from_agent(make_agent(8).to(dev))
        bufs = pol.rollout_buffers(sim, 16)
        pol.rollout(sim, 16, bufs, stochastic=True, seed=3)
        outs.append(bufs)
    torch.cuda.synchronize()
    assert_same(outs[0], outs[1])


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["init", "scaled"])
def test_gpu_policy_rollout_step0_pinned_to_reference_agent(native_lib, case):
    """The golden rows are both agents' observations of 256 oracle worlds after
    150 random steps (make_policy_golden.py); the simulator reproduces that
    state, so step 0 of a rollout with the fixture's weights must give the
    reference Agent's best() actions, log-probs and values on the trainee rows."""
    assert torch.cuda.is_available()
    obs, sd, ref = load_case(case)
    sim = make_sim(ExecMode.CUDA, 256, per_world_rng=True)
    sim.step_n(150, random_actions=True, action_seed=321, step0=0)
    torch.cuda.synchronize()
    rows = sim.observations_tensor().to_torch().reshape(-1, 128).cpu()
    assert torch.equal(rows, obs), "simulator state differs from the fixture's"
    pol = FusedPolicy.from_agent(agent_from_state_dict(sd, "cuda"))
    for trainee in (0, 1):
        s2 = make_sim(ExecMode.CUDA, 256, per_world_rng=True)
        s2.step_n(150, random_actions=True, action_seed=321, step0=0)
        bufs = pol.rollout_buffers(s2, 2)
        pol.rollout(s2, 2, bufs, trainee=trainee, stochastic=False)
        torch.cuda.synchronize()
        sel = {k: v[trainee::2] for k, v in ref.items()}
        assert torch.equal(bufs["obs"][0].cpu(), obs[trainee::2])
        check(bufs["actions"][0], bufs["log_prob"][0], bufs["value"][0], sel, MIN_DECISIVE[case] * 0.9)
