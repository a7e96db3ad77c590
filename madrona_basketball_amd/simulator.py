"""SimpleGridworldSimulator: the reference's Python class, MI355X-native.

Mirrors `madrona_basketball.SimpleGridworldSimulator` (src/bindings.cpp:17-101):
same constructor arguments and keyword names, `step()`, `set_action(...)`,
`trigger_reset(world_idx)` and the 19 `*_tensor()` getters whose
`.to_torch()` is a zero-copy view aliasing the live simulator state
(scripts/env.py:75-79 writes `actions` in place and reads
observations/rewards/dones after `step()`).

Storage is allocated by torch (on `cuda:gpu_id` for ExecMode.CUDA, host for
ExecMode.CPU) and handed to the native library, so every view is an ordinary
torch tensor that keeps its storage alive on its own.  In CUDA mode all work
is enqueued on torch's current stream of the simulator's device.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .madrona import ExecMode


class Tensor:
    """Stand-in for madrona::py::Tensor: `.to_torch()` returns the live view."""

    __slots__ = ("_t",)

    def __init__(self, t: torch.Tensor):
        self._t = t

    def to_torch(self) -> torch.Tensor:
        return self._t

    def __dlpack__(self, *args, **kwargs):
        return self._t.__dlpack__(*args, **kwargs)

    def __dlpack_device__(self):
        return self._t.__dlpack_device__()

    @property
    def shape(self):
        return tuple(self._t.shape)

    def __repr__(self):
        return f"Tensor({tuple(self._t.shape)}, {self._t.dtype}, {self._t.device})"


_TORCH_DTYPE = {_lib.DTYPE_INT32: torch.int32, _lib.DTYPE_FLOAT32: torch.float32}


def _raw_stream(device_index: int) -> int:
    """Torch's current HIP stream on the device, as a raw handle."""
    get = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if get is not None:
        return get(device_index)
    return torch.cuda.current_stream(device_index).cuda_stream


class SimpleGridworldSimulator:
    def __init__(self, discrete_x: int, discrete_y: int, start_x: float, start_y: float,
                 max_episode_length: int, exec_mode, num_worlds: int, gpu_id: int = -1,
                 *, num_agents: int = 2, rand_seed: int = 0, per_world_rng: bool = False,
                 tag_mask: bool = True, one_on_one: bool = True, world_offset: int = 0):
        L = _lib.load()
        mode = int(ExecMode(int(exec_mode)))
        cfg = _lib.Config()
        _lib.check(L.bb_default_config(ctypes.byref(cfg)), "bb_default_config")
        cfg.discrete_x = int(discrete_x)
        cfg.discrete_y = int(discrete_y)
        cfg.start_x = float(start_x)
        cfg.start_y = float(start_y)
        cfg.max_episode_length = int(max_episode_length)
        cfg.exec_mode = mode
        cfg.num_worlds = int(num_worlds)
        cfg.world_offset = int(world_offset)
        cfg.rand_seed = int(rand_seed) & 0xFFFFFFFF  # reference: 0 (src/bindings.cpp:37)
        cfg.num_agents = int(num_agents)
        cfg.flags = ((_lib.FLAG_PER_WORLD_RNG if per_world_rng else 0)
                     | (0 if tag_mask else _lib.FLAG_NO_TAG_MASK)
                     | (0 if one_on_one else _lib.FLAG_FULL_GAME))
        if mode == ExecMode.CUDA:
            if not torch.cuda.is_available():
                raise RuntimeError("ExecMode.CUDA requested but no HIP device is visible to torch")
            dev_index = torch.cuda.current_device() if int(gpu_id) < 0 else int(gpu_id)
            self._device = torch.device("cuda", dev_index)
            cfg.gpu_id = dev_index
        else:
            self._device = torch.device("cpu")
            cfg.gpu_id = -1
        self._cfg = cfg
        self._num_worlds = cfg.num_worlds
        self._num_agents = cfg.num_agents

        # torch-owned storage, one flat buffer per export / internal column
        self._raw = {}
        bufs = (ctypes.c_void_p * _lib.NUM_SLOTS)()
        for name, eid in _lib.EXPORT_IDS.items():
            nbytes = ctypes.c_int64()
            _lib.check(L.bb_buffer_bytes(ctypes.byref(cfg), eid, ctypes.byref(nbytes)), "bb_buffer_bytes")
            raw = torch.zeros(max(1, (nbytes.value + 3) // 4), dtype=torch.int32, device=self._device)
            self._raw[name] = raw
            bufs[eid] = raw.data_ptr()
        if mode == ExecMode.CUDA:
            torch.cuda.synchronize(self._device)
        handle = ctypes.c_void_p()
        _lib.check(L.bb_create_with_buffers(ctypes.byref(cfg), bufs, _lib.NUM_SLOTS, ctypes.byref(handle)),
                   "SimpleGridworldSimulator")
        self._h = handle
        self._bb_step = L.bb_step
        self._views = {}
        for name, eid in _lib.EXPORT_IDS.items():
            ptr = ctypes.c_void_p()
            dt = ctypes.c_int32()
            nd = ctypes.c_int32()
            dims = (ctypes.c_int64 * 4)()
            _lib.check(L.bb_export(self._h, eid, ctypes.byref(ptr), ctypes.byref(dt), ctypes.byref(nd), dims),
                       "bb_export")
            shape = tuple(int(dims[k]) for k in range(nd.value))
            raw = self._raw[name]
            numel = 1
            for d in shape:
                numel *= d
            self._views[name] = raw[:numel].view(_TORCH_DTYPE[dt.value]).view(shape)

    # ------------------------------------------------------------ lifecycle
    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.load().bb_destroy(h)
            except Exception:
                pass
            self._h = None

    def _stream(self):
        if self._device.type == "cuda":
            return ctypes.c_void_p(_raw_stream(self._device.index))
        return ctypes.c_void_p(None)

    # ------------------------------------------------------------ reference API
    def step(self) -> None:
        """Manager::step (src/mgr.cpp:243-246).  The per-call Python work is one
        ctypes call with torch's current raw stream (env.py calls this once per
        environment step)."""
        stream = _raw_stream(self._device.index) if self._device.type == "cuda" else None
        rc = self._bb_step(self._h, stream)
        if rc != _lib.OK:
            _lib.check(rc, "step")

    def set_action(self, world_idx: int, agent_idx: int, move_speed: int, move_angle: int, rotate: int,
                   grab: int, pass_: int = None, shoot: int = None, **kw) -> None:
        """Manager::setAction (src/mgr.cpp:270-293); `pass` is a keyword in the binding."""
        if pass_ is None:
            pass_ = kw.pop("pass")
        if shoot is None:
            shoot = kw.pop("shoot")
        rc = _lib.load().bb_set_action(self._h, int(world_idx), int(agent_idx), int(move_speed), int(move_angle),
                                       int(rotate), int(grab), int(pass_), int(shoot), self._stream())
        if rc != _lib.OK:
            # the reference prints and continues on bad indices (src/mgr.cpp:289-292)
            print("ERROR:", _lib.load().bb_last_error().decode())

    def trigger_reset(self, world_idx: int) -> None:
        """Manager::triggerReset (src/mgr.cpp:297-311), device-side in CUDA mode."""
        _lib.check(_lib.load().bb_trigger_reset(self._h, int(world_idx), self._stream()), "trigger_reset")

    def _t(self, name: str) -> Tensor:
        return Tensor(self._views[name])

    def reset_tensor(self): return self._t("reset")
    def game_state_tensor(self): return self._t("game_state")
    def action_tensor(self): return self._t("action")
    def action_mask_tensor(self): return self._t("action_mask")
    def agent_pos_tensor(self): return self._t("agent_pos")
    def observations_tensor(self): return self._t("observations")
    def reward_tensor(self): return self._t("reward")
    def done_tensor(self): return self._t("done")
    def agent_possession_tensor(self): return self._t("agent_possession")
    def agent_entity_id_tensor(self): return self._t("agent_entity_id")
    def agent_team_tensor(self): return self._t("team")
    def orientation_tensor(self): return self._t("orientation")
    def agent_stats_tensor(self): return self._t("agent_stats")
    def basketball_pos_tensor(self): return self._t("ball_pos")
    def ball_physics_tensor(self): return self._t("ball_physics")
    def ball_grabbed_tensor(self): return self._t("ball_grabbed")
    def ball_entity_id_tensor(self): return self._t("ball_entity_id")
    def ball_velocity_tensor(self): return self._t("ball_velocity")
    def hoop_pos_tensor(self): return self._t("hoop_pos")

    # ------------------------------------------------------------ build extensions
    def internal_tensor(self, name: str) -> torch.Tensor:
        """Build-internal state columns (velocity, cooldown, cur_step, inbounding,
        attributes, world_clock, rng_counter) for tests and snapshots."""
        return self._views[name]

    def step_n(self, n: int, random_actions: bool = False, action_seed: int = 321, step0: int = 0,
               time_kernels: bool = False):
        """n steps in one native call (optionally with the on-device synthetic
        random-action workload before each); returns summed step-kernel ms
        when time_kernels (CUDA mode)."""
        ms = ctypes.c_float(0.0)
        _lib.check(_lib.load().bb_step_n(self._h, int(n), 1 if random_actions else 0, int(action_seed) & 0xFFFFFFFF,
                                         int(step0) & 0xFFFFFFFF, self._stream(),
                                         ctypes.byref(ms) if time_kernels else None), "step_n")
        return ms.value if time_kernels else None

    def stage_random_actions(self, n: int, action_seed: int = 321, step0: int = 0) -> torch.Tensor:
        """[n, W, N, 6] int32 tensor (on the sim's device) holding the synthetic
        workload of step_n(random_actions=True) for steps step0..step0+n-1."""
        buf = torch.empty((n, self._num_worlds, self._num_agents, 6), dtype=torch.int32, device=self._device)
        _lib.check(_lib.load().bb_fill_random_actions(self._h, ctypes.c_void_p(buf.data_ptr()), int(n),
                                                      int(action_seed) & 0xFFFFFFFF, int(step0) & 0xFFFFFFFF,
                                                      self._stream()), "fill_random_actions")
        return buf

    def step_n_staged(self, actions: torch.Tensor, time_kernels: bool = False):
        """len(actions) steps, step k reading actions[k] ([W, N, 6] int32, on the
        sim's device) in place of the action tensor (the defence AI's
        overrides are written back into actions[k]); returns summed
        step-kernel ms when time_kernels (CUDA mode)."""
        n = actions.shape[0]
        if (tuple(actions.shape[1:]) != (self._num_worlds, self._num_agents, 6) or actions.dtype != torch.int32
                or not actions.is_contiguous() or actions.device != self._device):
            raise ValueError("actions must be a contiguous int32 [n, num_worlds, num_agents, 6] tensor "
                             "on the simulator's device")
        ms = ctypes.c_float(0.0)
        _lib.check(_lib.load().bb_step_n_staged(self._h, int(n), ctypes.c_void_p(actions.data_ptr()), self._stream(),
                                                ctypes.byref(ms) if time_kernels else None), "step_n_staged")
        return ms.value if time_kernels else None

    def rollout_buffers(self, n: int) -> dict:
        """Zeroed [n, W, N, ...] outputs for rollout() on the sim's device:
        obs float32 [n, W, N, OBSW], reward / done float32 [n, W, N] (the
        storage of scripts/ppo.py:63-70's rollout buffers)."""
        W, N = self._num_worlds, self._num_agents
        ow = self._views["observations"].shape[-1]
        return {
            "obs": torch.zeros((n, W, N, ow), dtype=torch.float32, device=self._device),
            "reward": torch.zeros((n, W, N), dtype=torch.float32, device=self._device),
            "done": torch.zeros((n, W, N), dtype=torch.float32, device=self._device),
        }

    def rollout(self, actions: torch.Tensor, obs: torch.Tensor = None, reward: torch.Tensor = None,
                done: torch.Tensor = None, per_step: bool = False, time_kernels: bool = False):
        """len(actions) steps in one native call (bb_rollout): step k takes
        actions[k] ([W, N, 6] int32; the defence AI's overrides are written
        back) and its observations / rewards / done flags land in obs[k],
        reward[k], done[k] (rollout_buffers(); None: not recorded).  One
        launch for all steps on gfx950 at 2 agents (worlds held in registers);
        per_step=True forces one step launch per step.  Afterwards every
        tensor of the simulator holds the state after the last step."""
        n = actions.shape[0]
        W, N = self._num_worlds, self._num_agents
        ow = self._views["observations"].shape[-1]

        def ok(t, shape, dtype):
            return (t is None or (tuple(t.shape) == shape and t.dtype == dtype and t.is_contiguous()
                                  and t.device == self._device))
        if not ok(actions, (n, W, N, 6), torch.int32):
            raise ValueError("actions must be a contiguous int32 [n, num_worlds, num_agents, 6] tensor "
                             "on the simulator's device")
        if not (ok(obs, (n, W, N, ow), torch.float32) and ok(reward, (n, W, N), torch.float32)
                and ok(done, (n, W, N), torch.float32)):
            raise ValueError("rollout outputs must be contiguous float32 tensors shaped like rollout_buffers(n)")
        if (reward is None) != (done is None):
            raise ValueError("reward and done are recorded together")

        def ptr(t):
            return ctypes.c_void_p(None if t is None else t.data_ptr())
        ms = ctypes.c_float(0.0)
        _lib.check(_lib.load().bb_rollout(self._h, int(n), ptr(actions), ptr(obs), ptr(reward), ptr(done),
                                          _lib.ROLLOUT_PER_STEP if per_step else 0, self._stream(),
                                          ctypes.byref(ms) if time_kernels else None), "rollout")
        return ms.value if time_kernels else None

    def write_random_actions(self, action_seed: int, step: int) -> None:
        _lib.check(_lib.load().bb_write_random_actions(self._h, int(action_seed) & 0xFFFFFFFF,
                                                       int(step) & 0xFFFFFFFF, self._stream()),
                   "write_random_actions")

    def snapshot(self) -> dict:
        """Copy of every column (exports + internal state)."""
        return {k: v.clone() for k, v in self._views.items()}

    def restore(self, snap: dict) -> None:
        for k, v in snap.items():
            self._views[k].copy_(v)

    @property
    def num_worlds(self) -> int:
        return self._num_worlds

    @property
    def num_agents(self) -> int:
        return self._num_agents

    @property
    def device(self) -> torch.device:
        return self._device
