"""The Python surface the reference's scripts bind to (src/bindings.cpp:14-101,
scripts/env.py), on the host executor (no GPU needed)."""
import inspect
import math

import numpy as np
import pytest
import torch

import madrona_basketball as mba
from oracle.oracle import Oracle
from tests.helpers import compare

GETTERS = ["reset_tensor", "game_state_tensor", "action_tensor", "action_mask_tensor", "agent_pos_tensor",
           "observations_tensor", "reward_tensor", "done_tensor", "agent_possession_tensor",
           "agent_entity_id_tensor", "agent_team_tensor", "orientation_tensor", "agent_stats_tensor",
           "basketball_pos_tensor", "ball_physics_tensor", "ball_grabbed_tensor", "ball_entity_id_tensor",
           "ball_velocity_tensor", "hoop_pos_tensor"]


@pytest.fixture(scope="module", autouse=True)
def _libs(native_lib, oracle_lib):
    pass


def make(num_worlds=4, **kw):
    # exactly the arguments scripts/env.py:20-35 passes (src/constants.py dims)
    w, h = 28.65 * 1.1, 15.24 * 1.1
    return mba.SimpleGridworldSimulator(
        discrete_x=math.ceil(w), discrete_y=math.ceil(h), start_x=w / 2.0, start_y=h / 2.0,
        max_episode_length=39600, exec_mode=mba.madrona.ExecMode.CPU, num_worlds=num_worlds, gpu_id=0, **kw)


def test_module_surface():
    assert int(mba.madrona.ExecMode.CPU) == 0 and int(mba.madrona.ExecMode.CUDA) == 1
    params = list(inspect.signature(mba.SimpleGridworldSimulator.__init__).parameters)
    assert params[1:9] == ["discrete_x", "discrete_y", "start_x", "start_y", "max_episode_length", "exec_mode",
                           "num_worlds", "gpu_id"]
    sim = make()
    for g in GETTERS + ["step", "set_action", "trigger_reset"]:
        assert callable(getattr(sim, g))


def test_tensor_shapes_and_dtypes():
    """src/mgr.cpp:317-445 shapes; torch dtypes of the exported element types."""
    W = 3
    sim = make(W)
    i32, f32 = torch.int32, torch.float32
    expect = {
        "reset_tensor": ((W, 2, 1), i32), "game_state_tensor": ((W, 14), f32), "action_tensor": ((W, 2, 6), i32),
        "action_mask_tensor": ((W, 2, 4), i32), "agent_pos_tensor": ((W, 2, 3), f32),
        "observations_tensor": ((W, 2, 128), f32), "reward_tensor": ((W, 2), f32), "done_tensor": ((W, 2), f32),
        "agent_possession_tensor": ((W, 2, 3), i32), "agent_entity_id_tensor": ((W, 2), i32),
        "agent_team_tensor": ((W, 2, 5), i32), "orientation_tensor": ((W, 2, 4), f32),
        "agent_stats_tensor": ((W, 2, 2), i32), "basketball_pos_tensor": ((W, 1, 3), f32),
        "ball_physics_tensor": ((W, 1, 7), i32), "ball_grabbed_tensor": ((W, 1, 2), i32),
        "ball_entity_id_tensor": ((W, 1), i32), "ball_velocity_tensor": ((W, 1, 3), f32),
        "hoop_pos_tensor": ((W, 2, 3), f32),
    }
    for g, (shape, dt) in expect.items():
        t = getattr(sim, g)().to_torch()
        assert tuple(t.shape) == shape and t.dtype == dt, g


def test_views_alias_live_state():
    sim = make(2)
    obs = sim.observations_tensor().to_torch()
    before = obs.clone()
    sim.step()
    assert not torch.equal(before, obs)  # same storage, updated in place
    act = sim.action_tensor().to_torch()
    act[0, 0] = torch.tensor([1, 2, 1, 0, 0, 0], dtype=torch.int32)
    assert torch.equal(sim.action_tensor().to_torch()[0, 0], act[0, 0])


def test_env_py_call_sequence_matches_oracle():
    """Replays what EnvWrapper does (scripts/env.py:75-79, 125-170, 178-185):
    int64 trainee actions written into one agent slot, step, clone the
    trainee's obs/reward/done; reset = resets.fill_(1), step, fill_(0)."""
    W, agent_idx = 16, 1
    sim = make(W)
    o = Oracle(W)
    observations = sim.observations_tensor().to_torch()
    actions = sim.action_tensor().to_torch()
    dones = sim.done_tensor().to_torch()
    rewards = sim.reward_tensor().to_torch()
    resets = sim.reset_tensor().to_torch()
    buckets = [2, 8, 3, 2, 2, 2]
    gen = torch.Generator().manual_seed(0)

    def env_step(trainee):
        actions[:, agent_idx] = trainee
        a = o.export("action")
        a[:, agent_idx] = trainee.numpy()
        o.set_actions(a)
        sim.step()
        o.step()
        return (observations[:, agent_idx].detach().clone(), rewards[:, agent_idx].detach().clone(),
                dones[:, agent_idx].detach().clone())

    def env_reset():
        resets.fill_(1)
        o.import_("reset", np.ones((W, 2, 1), np.int32))
        out = env_step(torch.zeros_like(actions[:, agent_idx]))
        resets.fill_(0)
        o.import_("reset", np.zeros((W, 2, 1), np.int32))
        return out

    for it in range(6):           # ppo.py rollout: reset + 32 steps
        obs, rew, done = env_reset()
        assert (done == 1).all()
        for _ in range(32):
            trainee = torch.stack([torch.randint(0, b, (W,), generator=gen) for b in buckets], dim=-1)  # int64
            obs, rew, done = env_step(trainee)
            assert obs.shape == (W, 128) and rew.shape == (W,) and done.shape == (W,)
        bad, _ = compare(sim, o)
        assert not bad, bad


def test_viewer_and_logger_getters_work():
    """scripts/viewer.py:198-300 and scripts/ppo.py:94-104 read these every step."""
    sim = make(2)
    sim.step()
    log = {k: getattr(sim, k)().to_torch()[:1].cpu().numpy().copy() for k in GETTERS}
    assert log["hoop_pos_tensor"].shape == (1, 2, 3)
    sim.trigger_reset(0)
    sim.step()
    assert (sim.done_tensor().to_torch()[0] == 1).all()
