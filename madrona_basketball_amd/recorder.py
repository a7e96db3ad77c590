"""Device-side trajectory recorder.

The reference logs a trajectory by copying ten exported tensors to the host
every step (scripts/ppo.py:93-106 for world 0, scripts/infer.py:116-129 for
all worlds) and saving them with np.savez_compressed (scripts/ppo.py:108-119,
scripts/infer.py:142-149).  Here each step's record is one launch of
bb_record into a device ring ([capacity, worlds, words] int32, no host sync);
the host copy happens once, in episode_log() / save_npz(), whose arrays have
the keys, dtypes and shapes the reference's np.array([step[key] ...]) gives.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

# scripts/ppo.py:94-105 key order -> (export column, dtype, per-world shape(N))
KEYS = (
    ("agent_pos", np.float32, lambda n: (n, 3)),
    ("ball_pos", np.float32, lambda n: (1, 3)),
    ("ball_vel", np.float32, lambda n: (1, 3)),
    ("orientation", np.float32, lambda n: (n, 4)),
    ("ball_physics", np.int32, lambda n: (1, 7)),
    ("agent_possession", np.int32, lambda n: (n, 3)),
    ("game_state", np.float32, lambda n: (14,)),
    ("rewards", np.float32, lambda n: (n,)),
    ("actions", np.int32, lambda n: (n, 6)),
    ("done", np.float32, lambda n: (n,)),
)


class TrajectoryRecorder:
    """Records worlds [world0, world0 + num_worlds) of `sim` after each step.

    record() enqueues one copy on the sim's stream; episode_log() returns
    {key: array[T, num_worlds, ...]} (done: all agents, or the trainee's
    column with done_agent=i as env.step returns it, scripts/env.py:169);
    save_npz(path, **static) writes them like the reference's logger.
    """

    def __init__(self, sim, capacity: int, world0: int = 0, num_worlds: int = 1):
        self.sim = sim
        self.capacity = int(capacity)
        self.world0 = int(world0)
        self.num_worlds = int(num_worlds)
        if self.world0 < 0 or self.world0 + self.num_worlds > sim.num_worlds or self.capacity < 1:
            raise ValueError("recorded worlds must lie inside the simulator and capacity >= 1")
        self.n = sim.num_agents
        self.words = int(_lib.load().bb_record_words(self.n))
        self.ring = torch.zeros((self.capacity, self.num_worlds, self.words), dtype=torch.int32, device=sim.device)
        self.length = 0

    def record(self) -> None:
        if self.length >= self.capacity:
            raise RuntimeError(f"TrajectoryRecorder full ({self.capacity} steps); clear() or save first")
        _lib.check(_lib.load().bb_record(self.sim._h, self.world0, self.num_worlds,
                                         ctypes.c_void_p(self.ring.data_ptr()), self.length, self.sim._stream()),
                   "record")
        self.length += 1

    def clear(self) -> None:
        self.length = 0

    def episode_log(self, done_agent: int | None = None) -> dict:
        raw = self.ring[:self.length].cpu().numpy()  # one device -> host copy
        out, q = {}, 0
        for key, dtype, shape in KEYS:
            shp = shape(self.n)
            width = int(np.prod(shp))
            a = np.ascontiguousarray(raw[:, :, q:q + width]).view(dtype).reshape((self.length, self.num_worlds) + shp)
            out[key] = a
            q += width
        if done_agent is not None:
            out["done"] = np.ascontiguousarray(out["done"][:, :, done_agent])
        return out

    def save_npz(self, path: str, done_agent: int | None = None, **static) -> None:
        np.savez_compressed(path, **static, **self.episode_log(done_agent))
