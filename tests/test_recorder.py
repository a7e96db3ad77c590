"""Device-side trajectory recorder (bb_record) against
the reference's own logging: per step, ten `.to_torch()[w0:w1].cpu().numpy()`
copies (scripts/ppo.py:94-105, scripts/infer.py:117-128), stacked with
np.array([step[key] for step in log]) and saved with np.savez_compressed."""
import numpy as np
import pytest
import torch

from madrona_basketball_amd import ExecMode, TrajectoryRecorder
from madrona_basketball_amd.recorder import KEYS
from tests.helpers import make_sim

GETTER = {
    "agent_pos": "agent_pos_tensor", "ball_pos": "basketball_pos_tensor", "ball_vel": "ball_velocity_tensor",
    "orientation": "orientation_tensor", "ball_physics": "ball_physics_tensor",
    "agent_possession": "agent_possession_tensor", "game_state": "game_state_tensor",
    "rewards": "reward_tensor", "actions": "action_tensor", "done": "done_tensor",
}


def reference_log(sim, w0, nw, steps, seed):
    """What the reference's logger stores: host copies after every step."""
    log = []
    for t in range(steps):
        sim.write_random_actions(seed, t)
        sim.step()
        log.append({k: getattr(sim, GETTER[k])().to_torch()[w0:w0 + nw].cpu().numpy().copy() for k, _, _ in KEYS})
    return {k: np.array([step[k] for step in log]) for k, _, _ in KEYS}


def recorded_log(sim, w0, nw, steps, seed, capacity=None):
    rec = TrajectoryRecorder(sim, capacity or steps, world0=w0, num_worlds=nw)
    for t in range(steps):
        sim.write_random_actions(seed, t)
        sim.step()
        rec.record()
    return rec


def check_same(a: dict, b: dict):
    assert list(a) == list(b)
    for k in a:
        assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape, (k, a[k].dtype, b[k].dtype, a[k].shape, b[k].shape)
        assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)), k


@pytest.mark.parametrize("num_agents,w0,nw", [(2, 0, 1), (2, 5, 7), (4, 3, 4)])
def test_host_recorder_equals_reference_logging(native_lib, num_agents, w0, nw):
    W, T = 16, 90
    a = make_sim(ExecMode.CPU, W, num_agents=num_agents, per_world_rng=True)
    b = make_sim(ExecMode.CPU, W, num_agents=num_agents, per_world_rng=True)
    ref = reference_log(a, w0, nw, T, 3)
    rec = recorded_log(b, w0, nw, T, 3)
    check_same(rec.episode_log(), ref)


def test_recorder_npz_and_limits(native_lib, tmp_path):
    W, T = 8, 12
    sim = make_sim(ExecMode.CPU, W)
    rec = recorded_log(sim, 0, 1, T, 1)
    with pytest.raises(RuntimeError):
        rec.record()  # full
    hoop = sim.hoop_pos_tensor().to_torch()[:1].numpy().copy()
    path = tmp_path / "episode.npz"
    rec.save_npz(str(path), done_agent=0, hoop_pos=hoop)
    with np.load(path) as z:  # allow_pickle=False (default)
        assert sorted(z.files) == sorted([k for k, _, _ in KEYS] + ["hoop_pos"])
        assert z["done"].shape == (T, 1) and z["agent_pos"].shape == (T, 1, 2, 3)
        assert z["game_state"].shape == (T, 1, 14) and z["actions"].dtype == np.int32
    rec.clear()
    assert rec.length == 0
    with pytest.raises(ValueError):
        TrajectoryRecorder(sim, 4, world0=7, num_worlds=2)


@pytest.mark.gpu
def test_gpu_recorder_equals_reference_logging(native_lib):
    assert torch.cuda.is_available()
    W, T = 4096, 200
    a = make_sim(ExecMode.CUDA, W, per_world_rng=True)
    b = make_sim(ExecMode.CUDA, W, per_world_rng=True)
    ref = reference_log(a, 100, 33, T, 9)
    rec = recorded_log(b, 100, 33, T, 9)
    check_same(rec.episode_log(), ref)
    # and the whole-batch logger of scripts/infer.py (every world)
    c = make_sim(ExecMode.CUDA, W, per_world_rng=True)
    d = make_sim(ExecMode.CUDA, W, per_world_rng=True)
    check_same(recorded_log(d, 0, W, 20, 4).episode_log(), reference_log(c, 0, W, 20, 4))
