"""k_rollout_ppo<2> / k_step_ppo<2>: PPO's rollout loop with the trainee's
policy pass fused behind the world step (bb_rollout_policy above 16 384 worlds;
scripts/ppo.py:65-134 over scripts/env.py:126-170), the whole rollout in one
launch (each wave steps its worlds K times; default) or one launch per step
(MADRONA_BB_PPO_STEP_LOOP=0, child process).  Every recorded output
(buffer.obs / actions / log_probs / values / rewards / not_dones, next_value)
and every simulator column must equal the per-step launches (k_policy +
k_step, the `per_step` flag) and the loop of FusedPolicy.act + step, bit for
bit: the row passes feed layer 1's MFMA chain in its own k order, so the
policy sees the same floats in the same order.

The fused step is taken by row count (MADRONA_BB_PPO_STEP_FUSED_MIN_WORLDS,
read once per process): small and ragged grids run it in a child process with
the bound lowered to 1 (partial waves, inactive waves of the last workgroup,
4-wave workgroups)."""
import os
import subprocess
import sys

import pytest
import torch

from madrona_basketball_amd import ExecMode
from madrona_basketball_amd.policy import FusedPolicy, make_agent
from tests.helpers import make_sim
from tests.test_policy_rollout import assert_same, reference_loop, run_pair

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fused_vs_per_step(W, n, trainee, stochastic, seed=7, step0=3, partial=False):
    sims = [make_sim(ExecMode.CUDA, W, per_world_rng=True) for _ in range(2)]
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


CHILD = r'''
import torch
from tests.test_ppo_step import fused_vs_per_step
for W, n, trainee, stoch in [(1000, 6, 1, True), (64, 3, 0, False), (12345, 5, 0, True), (31, 4, 1, True),
                             (8192, 4, 0, True)]:
    fused_vs_per_step(W, n, trainee, stoch)
print("PPO_STEP_OK")
'''


@pytest.mark.gpu
def test_gpu_fused_ppo_step_forced_on_small_grids(native_lib):
    env = dict(os.environ, MADRONA_BB_PPO_STEP_FUSED_MIN_WORLDS="1", MADRONA_BB_PPO_FUSED_MAX_WORLDS="0",
               PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "PPO_STEP_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


STEP_LAUNCHES_CHILD = r'''
import torch
from tests.test_ppo_step import fused_vs_per_step
for W, n, trainee, stoch in [(65536, 6, 1, True), (40001, 4, 0, True), (65536, 1, 0, False)]:
    fused_vs_per_step(W, n, trainee, stoch)
print("PPO_STEP_OK")
'''


@pytest.mark.gpu
def test_gpu_fused_ppo_step_one_launch_per_step(native_lib):
    """MADRONA_BB_PPO_STEP_LOOP=0: one k_step_ppo launch per step, equal to the
    per-step launches (and so to the one-launch rollout)."""
    env = dict(os.environ, MADRONA_BB_PPO_STEP_LOOP="0", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", STEP_LAUNCHES_CHILD], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "PPO_STEP_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


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
