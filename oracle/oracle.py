"""ctypes wrapper for the CPU oracle (liboracle_bb.so).

TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg are the only callers.  The product package never imports this
module.  See bb_oracle.h for the parity status of the restatement.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MADRONA_BB_ORACLE_LIB: a sanitizer build of the same source (tools/sanitize.sh)
LIB_PATH = os.environ.get("MADRONA_BB_ORACLE_LIB") or os.path.join(HERE, "liboracle_bb.so")

# Export ids (reference src/types.hpp:10-42) and build-internal state ids.
EXPORTS = {
    "reset": 0, "game_state": 1, "action": 2, "action_mask": 3, "agent_pos": 4,
    "observations": 5, "reward": 6, "done": 7, "agent_entity_id": 8,
    "agent_possession": 9, "orientation": 10, "team": 11, "agent_stats": 12,
    "ball_pos": 13, "ball_physics": 14, "ball_entity_id": 15, "ball_grabbed": 16,
    "ball_velocity": 17, "hoop_pos": 18,
    "agent_velocity": 32, "grab_cooldown": 33, "cur_step": 34, "inbounding": 35,
    "attributes": 36, "world_clock": 37, "rng_counter": 38,
}

FLAG_PER_WORLD_RNG = 0x1
FLAG_NO_TAG_MASK = 0x2
FLAG_FULL_GAME = 0x4
MATH_CR = 0
MATH_LIBM = 1
MATH_LIBM_FLOAT = 2  # the float-overload reading of game.cpp:746,808,868

# Cumulative event counters (bb_oracle.h OR_EV_*), in enum order.
EVENTS = [
    "shot", "shot_going_in", "make", "oob_1v1", "oob_turnover", "tag", "contact", "inbound_start",
    "inbound_violation", "period_advance", "game_end", "world_reset", "clock_expiry", "grab", "pass",
    "defender_grab_reset", "obs_padded_row",
]


def obs_width(n: int) -> int:
    used = 61 + 38 * (n - 1) + 2 * n
    return max(128, (used + 3) & ~3)


def export_layout(name: str, n: int):
    """(numpy dtype, per-world shape) of an export in the reference layout
    (src/mgr.cpp:317-445)."""
    f, i = np.float32, np.int32
    table = {
        "reset": (i, (n, 1)), "game_state": (f, (14,)), "action": (i, (n, 6)),
        "action_mask": (i, (n, 4)), "agent_pos": (f, (n, 3)),
        "observations": (f, (n, obs_width(n))), "reward": (f, (n,)), "done": (f, (n,)),
        "agent_entity_id": (i, (n,)), "agent_possession": (i, (n, 3)),
        "orientation": (f, (n, 4)), "team": (i, (n, 5)), "agent_stats": (i, (n, 2)),
        "ball_pos": (f, (1, 3)), "ball_physics": (i, (1, 7)), "ball_entity_id": (i, (1,)),
        "ball_grabbed": (i, (1, 2)), "ball_velocity": (f, (1, 3)), "hoop_pos": (f, (2, 3)),
        "agent_velocity": (f, (n, 3)), "grab_cooldown": (f, (n,)), "cur_step": (i, (n,)),
        "inbounding": (i, (n, 2)), "attributes": (f, (n, 10)), "world_clock": (i, ()),
        "rng_counter": (i, ()),
    }
    return table[name]


class _Cfg(ctypes.Structure):
    _fields_ = [
        ("num_agents", ctypes.c_int32), ("num_worlds", ctypes.c_int64),
        ("discrete_x", ctypes.c_int32), ("discrete_y", ctypes.c_int32),
        ("start_x", ctypes.c_float), ("start_y", ctypes.c_float),
        ("seed", ctypes.c_uint32), ("flags", ctypes.c_uint32),
        ("world_offset", ctypes.c_int64), ("math_mode", ctypes.c_int32),
    ]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_create.restype = ctypes.c_void_p
        L.oracle_create.argtypes = [ctypes.POINTER(_Cfg)]
        L.oracle_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_step.argtypes = [ctypes.c_void_p]
        L.oracle_export.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
        L.oracle_import.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
        L.oracle_export_bytes.restype = ctypes.c_int64
        L.oracle_export_bytes.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.oracle_random_actions.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_events.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
        L.oracle_run_random.restype = ctypes.c_double
        L.oracle_run_random.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_threefry2x32.argtypes = [ctypes.c_uint32] * 4 + [ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_shot_point_value.restype = ctypes.c_int32
        L.oracle_shot_point_value.argtypes = [ctypes.c_float] * 6
        L.oracle_rotate_vec.argtypes = [ctypes.POINTER(ctypes.c_float)] * 3
        L.oracle_court_constants.argtypes = [ctypes.POINTER(ctypes.c_float)]
        L.oracle_obs_width.restype = ctypes.c_int32
        L.oracle_obs_width.argtypes = [ctypes.c_int32]
        _lib = L
    return _lib


# Constructor inputs scripts/env.py:20-35 derives from src/constants.py
# (WORLD_WIDTH_M = 31.515, WORLD_HEIGHT_M = 16.764): ceil -> 32 x 17 cells,
# start = width/2, height/2 rounded to float by the nanobind float args.
ENV_DISCRETE_X = 32
ENV_DISCRETE_Y = 17
ENV_START_X = float(np.float32(31.515 / 2.0))
ENV_START_Y = float(np.float32(16.764000000000003 / 2.0))


class Oracle:
    def __init__(self, num_worlds: int, num_agents: int = 2, seed: int = 0, flags: int = 0,
                 world_offset: int = 0, math_mode: int = MATH_LIBM,
                 discrete_x: int = ENV_DISCRETE_X, discrete_y: int = ENV_DISCRETE_Y,
                 start_x: float = ENV_START_X, start_y: float = ENV_START_Y):
        self.n = num_agents
        self.w = num_worlds
        cfg = _Cfg(num_agents, num_worlds, discrete_x, discrete_y, start_x, start_y,
                   seed, flags, world_offset, math_mode)
        self._h = lib().oracle_create(ctypes.byref(cfg))
        if not self._h:
            raise ValueError("oracle_create rejected the config")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().oracle_destroy(h)
            self._h = None

    def step(self, n: int = 1):
        for _ in range(n):
            lib().oracle_step(self._h)

    def export(self, name: str) -> np.ndarray:
        dt, shape = export_layout(name, self.n)
        out = np.zeros((self.w,) + shape, dtype=dt)
        lib().oracle_export(self._h, EXPORTS[name], out.ctypes.data)
        return out

    def import_(self, name: str, arr) -> None:
        dt, shape = export_layout(name, self.n)
        a = np.ascontiguousarray(np.asarray(arr).reshape((self.w,) + shape).astype(dt, copy=False))
        lib().oracle_import(self._h, EXPORTS[name], a.ctypes.data)

    def set_actions(self, actions) -> None:
        self.import_("action", actions)

    def random_actions(self, seed: int, step: int) -> None:
        lib().oracle_random_actions(self._h, seed, step)

    def run_random(self, steps: int, seed: int, step0: int = 0) -> float:
        return lib().oracle_run_random(self._h, steps, seed, step0)

    def events(self) -> dict:
        """Cumulative counts of the rare branches taken since creation."""
        out = (ctypes.c_int64 * len(EVENTS))()
        lib().oracle_events(self._h, out)
        return {k: int(out[i]) for i, k in enumerate(EVENTS)}

    def snapshot(self, names=None) -> dict:
        names = names or list(EXPORTS)
        return {k: self.export(k) for k in names}


def threefry2x32(k0, k1, c0, c1):
    out = (ctypes.c_uint32 * 2)()
    lib().oracle_threefry2x32(k0, k1, c0, c1, out)
    return int(out[0]), int(out[1])


def shot_point_value(p, h) -> int:
    return int(lib().oracle_shot_point_value(*[float(x) for x in p], *[float(x) for x in h]))


def rotate_vec(q, v):
    qa = (ctypes.c_float * 4)(*q)
    va = (ctypes.c_float * 3)(*v)
    out = (ctypes.c_float * 3)()
    lib().oracle_rotate_vec(qa, va, out)
    return np.array(list(out), dtype=np.float32)


def court_constants():
    out = (ctypes.c_float * 8)()
    lib().oracle_court_constants(out)
    keys = ["world_w", "world_h", "court_min_x", "court_max_x", "court_min_y", "court_max_y",
            "ts", "pi"]
    return dict(zip(keys, [np.float32(x) for x in out]))
