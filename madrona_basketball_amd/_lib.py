"""ctypes binding of libmadrona_basketball_amd.so (include/madrona_basketball_amd.h).

Loaded after `import torch`, so the library resolves libamdhip64.so.7 to the
HIP runtime torch already loaded (one runtime per process, shared streams).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime first)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmadrona_basketball_amd.so")

OK = 0
EXEC_CPU = 0
EXEC_CUDA = 1
DTYPE_INT32 = 0
DTYPE_FLOAT32 = 1
FLAG_PER_WORLD_RNG = 0x1
FLAG_NO_TAG_MASK = 0x2
FLAG_FULL_GAME = 0x4
ROLLOUT_PER_STEP = 0x1
NUM_REFERENCE_EXPORTS = 19
INTERNAL_FIRST = 32
INTERNAL_LAST = 38
NUM_SLOTS = INTERNAL_LAST + 1

EXPORT_IDS = {
    "reset": 0, "game_state": 1, "action": 2, "action_mask": 3, "agent_pos": 4,
    "observations": 5, "reward": 6, "done": 7, "agent_entity_id": 8,
    "agent_possession": 9, "orientation": 10, "team": 11, "agent_stats": 12,
    "ball_pos": 13, "ball_physics": 14, "ball_entity_id": 15, "ball_grabbed": 16,
    "ball_velocity": 17, "hoop_pos": 18,
    "agent_velocity": 32, "grab_cooldown": 33, "cur_step": 34, "inbounding": 35,
    "attributes": 36, "world_clock": 37, "rng_counter": 38,
}

# every symbol include/madrona_basketball_amd.h declares
ABI_SYMBOLS = [
    "bb_default_config", "bb_obs_width", "bb_buffer_bytes", "bb_create",
    "bb_create_with_buffers", "bb_destroy", "bb_step", "bb_step_n",
    "bb_write_random_actions", "bb_step_n_staged", "bb_fill_random_actions", "bb_rollout",
    "bb_record_words", "bb_record", "bb_policy_forward", "bb_rollout_policy",
    "bb_set_action", "bb_trigger_reset", "bb_export",
    "bb_num_worlds", "bb_num_agents", "bb_exec_mode", "bb_algorithmic_bytes_per_world",
    "bb_rollout_policy_path", "bb_rollout_policy_bytes", "bb_step_staged_path", "bb_step_staged_bytes",
    "bb_rollout_fused", "bb_rollout_bytes_per_world_step", "bb_rollout_state_bytes_per_world",
    "bb_last_error",
]


class Config(ctypes.Structure):
    _fields_ = [
        ("discrete_x", ctypes.c_int64), ("discrete_y", ctypes.c_int64),
        ("start_x", ctypes.c_float), ("start_y", ctypes.c_float),
        ("max_episode_length", ctypes.c_int64),
        ("exec_mode", ctypes.c_int32), ("gpu_id", ctypes.c_int32),
        ("num_worlds", ctypes.c_int64), ("world_offset", ctypes.c_int64),
        ("rand_seed", ctypes.c_uint32), ("flags", ctypes.c_uint32),
        ("num_agents", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]


class PolicyWeights(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("obs_mean", "obs_inv", "w1", "b1", "ln1_w", "ln1_b", "w2", "b2",
                                               "ln2_w", "ln2_b", "head_w", "head_b")]


class PolicyRolloutBuffers(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("obs", "actions", "log_prob", "value", "reward", "done",
                                               "next_value")]


_lib = None


class BBError(RuntimeError):
    pass


def load():
    """Load (never silently replace) the native library."""
    global _lib
    if _lib is not None:
        return _lib
    # MADRONA_BB_LIB: a diagnostic variant build (build.py --variant), for A/B timing
    path = os.environ.get("MADRONA_BB_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `python -m madrona_basketball_amd.build` "
            "(hipcc --offload-arch=gfx950). There is no Python fallback.")
    L = ctypes.CDLL(path)
    vp, i32, i64, u32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32
    cfgp = ctypes.POINTER(Config)
    sig = {
        "bb_default_config": (ctypes.c_int, [cfgp]),
        "bb_obs_width": (i32, [i32]),
        "bb_buffer_bytes": (ctypes.c_int, [cfgp, i32, ctypes.POINTER(i64)]),
        "bb_create": (ctypes.c_int, [cfgp, ctypes.POINTER(vp)]),
        "bb_create_with_buffers": (ctypes.c_int, [cfgp, ctypes.POINTER(vp), i32, ctypes.POINTER(vp)]),
        "bb_destroy": (ctypes.c_int, [vp]),
        "bb_step": (ctypes.c_int, [vp, vp]),
        "bb_step_n": (ctypes.c_int, [vp, i32, i32, u32, u32, vp, ctypes.POINTER(ctypes.c_float)]),
        "bb_write_random_actions": (ctypes.c_int, [vp, u32, u32, vp]),
        "bb_step_n_staged": (ctypes.c_int, [vp, i32, vp, vp, ctypes.POINTER(ctypes.c_float)]),
        "bb_fill_random_actions": (ctypes.c_int, [vp, vp, i32, u32, u32, vp]),
        "bb_rollout": (ctypes.c_int, [vp, i32, vp, vp, vp, vp, u32, vp, ctypes.POINTER(ctypes.c_float)]),
        "bb_record_words": (i32, [i32]),
        "bb_policy_forward": (ctypes.c_int, [ctypes.POINTER(PolicyWeights), i32, i32, vp, i64, i64, vp, i64, vp, vp,
                                             i32, u32, u32, vp]),
        "bb_record": (ctypes.c_int, [vp, i64, i32, vp, i64, vp]),
        "bb_rollout_policy": (ctypes.c_int, [vp, ctypes.POINTER(PolicyWeights), ctypes.POINTER(PolicyWeights), i32,
                                             i32, i32, u32, u32, ctypes.POINTER(PolicyRolloutBuffers), u32, vp,
                                             ctypes.POINTER(ctypes.c_float)]),
        "bb_set_action": (ctypes.c_int, [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp]),
        "bb_trigger_reset": (ctypes.c_int, [vp, i32, vp]),
        "bb_export": (ctypes.c_int, [vp, i32, ctypes.POINTER(vp), ctypes.POINTER(i32),
                                     ctypes.POINTER(i32), ctypes.POINTER(i64)]),
        "bb_num_worlds": (i64, [vp]),
        "bb_num_agents": (i32, [vp]),
        "bb_exec_mode": (i32, [vp]),
        "bb_algorithmic_bytes_per_world": (i64, [i32]),
        "bb_rollout_policy_path": (i32, [vp, i32, ctypes.c_uint32]),
        "bb_step_staged_path": (i32, [vp, i32]),
        "bb_step_staged_bytes": (i64, [vp, i32]),
        "bb_rollout_policy_bytes": (i64, [vp, i32, ctypes.c_uint32, i32]),
        "bb_rollout_fused": (i32, [i32]),
        "bb_rollout_bytes_per_world_step": (i64, [i32]),
        "bb_rollout_state_bytes_per_world": (i64, [i32]),
        "bb_last_error": (ctypes.c_char_p, []),
        "bb_diag_set": (ctypes.c_int, [i32, i32]),
        "bb_diag_kernel_name": (ctypes.c_char_p, [vp, i32, i32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


# Path overrides of the library (bb_launch.h DiagKey, set through the
# diagnostic bb_diag_set; -1 restores the product's own rule).  Tests and A/B
# timing only: the library reads no environment variable to pick a kernel.
DIAG_KEYS = {
    "step_loop": 0,                  # bb_step_n_staged's launch kind (BB_STAGED_*)
    "rollout_split": 1,              # k_rollout_split: 0 never, 1 always
    "rollout_minw": 2,               # k_rollout's register budget: 1 or 2 waves per SIMD
    "rollout_shared_max_n": 3,       # the N >= 4 K-step rollout kernel up to this many agents
    "ppo_pwaves": 4,                 # k_rollout_policy's policy waves: 2 or 4
    "ppo_fused_max_worlds": 5,       # k_rollout_policy up to this many worlds
    "ppo_step_fused_min_worlds": 6,  # the fused PPO step from this many worlds (0: never)
    "ppo_step_loop": 7,              # 0: one k_step_ppo launch per step
    "policy_wg": 8,                  # k_policy_wg: 0 never, 1 always
}


def diag_set(name: str, value: int) -> None:
    check(load().bb_diag_set(DIAG_KEYS[name], int(value)), f"bb_diag_set({name}, {value})")


class diag:
    """Context manager: `with diag(step_loop=0): ...` sets path overrides for
    the block and restores the product's rules (-1) after it."""

    def __init__(self, **overrides):
        self.overrides = overrides

    def __enter__(self):
        for k, v in self.overrides.items():
            diag_set(k, v)
        return self

    def __exit__(self, *exc):
        for k in self.overrides:
            diag_set(k, -1)
        return False


def kernel_name(sim_handle, what: int, n: int) -> str:
    """The kernel a call launches (0 bb_step, 1 bb_step_n_staged of n steps,
    2 bb_rollout of n steps), from the library's own selection rules."""
    return load().bb_diag_kernel_name(sim_handle, int(what), int(n)).decode()


def check(rc: int, what: str) -> None:
    if rc != OK:
        msg = load().bb_last_error().decode(errors="replace")
        raise BBError(f"{what} failed ({rc}): {msg}")
