"""The C-ABI library: loads without a GPU, exports every symbol
include/madrona_basketball_amd.h declares, and reports errors instead of
aborting (the reference aborts via FATAL/REQ_CUDA, src/mgr.cpp:191,198)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "madrona_basketball_amd.h")


@pytest.fixture(scope="module")
def L(native_lib):
    return native_lib


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(bb_\w+)\s*\(", text, flags=re.M)))


def test_header_and_binding_agree():
    from madrona_basketball_amd._lib import ABI_SYMBOLS
    assert declared_functions() == sorted(ABI_SYMBOLS)


def test_library_exports_every_declared_symbol(L):
    from madrona_basketball_amd._lib import LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in declared_functions() if s not in exported]
    assert not missing, missing
    for s in declared_functions():
        assert hasattr(L, s)


def cfg_default(L):
    from madrona_basketball_amd._lib import Config
    c = Config()
    assert L.bb_default_config(ctypes.byref(c)) == 0
    return c


def test_defaults_are_the_env_py_constructor(L):
    c = cfg_default(L)
    assert (c.discrete_x, c.discrete_y, c.max_episode_length, c.num_agents, c.rand_seed) == (32, 17, 39600, 2, 0)
    assert np.float32(c.start_x) == np.float32(31.515 / 2) and np.float32(c.start_y) == np.float32(16.764000000000003 / 2)


def test_errors_are_reported_not_fatal(L):
    c = cfg_default(L)
    h = ctypes.c_void_p()
    c.num_agents = 3
    assert L.bb_create(ctypes.byref(c), ctypes.byref(h)) < 0
    assert b"num_agents" in L.bb_last_error()
    c = cfg_default(L)
    c.num_worlds = 0
    assert L.bb_create(ctypes.byref(c), ctypes.byref(h)) < 0
    c = cfg_default(L)
    c.flags = 0x80
    assert L.bb_create(ctypes.byref(c), ctypes.byref(h)) < 0


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="only meaningful where no GPU is visible")
def test_cuda_mode_without_gpu_is_an_error(L):
    c = cfg_default(L)
    c.exec_mode = 1
    h = ctypes.c_void_p()
    assert L.bb_create(ctypes.byref(c), ctypes.byref(h)) < 0
    assert b"HIP" in L.bb_last_error() or b"device" in L.bb_last_error()


def test_self_allocating_path_and_exports(L):
    c = cfg_default(L)
    c.num_worlds = 8
    h = ctypes.c_void_p()
    assert L.bb_create(ctypes.byref(c), ctypes.byref(h)) == 0, L.bb_last_error()
    try:
        assert L.bb_num_worlds(h) == 8 and L.bb_num_agents(h) == 2 and L.bb_exec_mode(h) == 0
        for _ in range(3):
            assert L.bb_step(h, None) == 0
        expected = {0: (0, 3, (8, 2, 1)), 1: (1, 2, (8, 14)), 2: (0, 3, (8, 2, 6)), 5: (1, 3, (8, 2, 128)),
                    6: (1, 2, (8, 2)), 11: (0, 3, (8, 2, 5)), 12: (0, 3, (8, 2, 2)), 13: (1, 3, (8, 1, 3)),
                    14: (0, 3, (8, 1, 7)), 15: (0, 2, (8, 1)), 18: (1, 3, (8, 2, 3))}
        for eid, (dt, nd, shape) in expected.items():
            p, d, n = ctypes.c_void_p(), ctypes.c_int32(), ctypes.c_int32()
            dims = (ctypes.c_int64 * 4)()
            assert L.bb_export(h, eid, ctypes.byref(p), ctypes.byref(d), ctypes.byref(n), dims) == 0
            assert (d.value, n.value) == (dt, nd) and tuple(dims[:nd]) == shape and p.value
        p = ctypes.c_void_p()
        assert L.bb_export(h, 99, ctypes.byref(p), None, None, None) < 0
        # out-of-range trigger_reset is ignored, bad set_action is an error
        assert L.bb_trigger_reset(h, 100, None) == 0
        assert L.bb_set_action(h, 100, 0, 1, 1, 1, 1, 1, 1, None) < 0
    finally:
        L.bb_destroy(h)


def test_algorithmic_bytes(L):
    assert L.bb_algorithmic_bytes_per_world(2) == 1512
    assert L.bb_algorithmic_bytes_per_world(10) == 19752
    assert L.bb_obs_width(2) == 128 and L.bb_obs_width(4) == 184 and L.bb_obs_width(10) == 424


def test_kernel_choices_are_not_read_from_the_environment(L):
    """The library picks its kernels by its own rules; the only overrides are
    the diagnostic bb_diag_set table (tests, A/B timing).  Its one environment
    variable is BB_CPU_THREADS (the host executor's thread count)."""
    from madrona_basketball_amd._lib import DIAG_KEYS, LIB_PATH
    blob = open(LIB_PATH, "rb").read()
    names = set(re.findall(rb"(?:MADRONA_BB|BB)_[A-Z0-9_]{3,}", blob))
    env_like = {n for n in names if n.startswith(b"MADRONA_BB_")}
    assert not env_like, env_like
    assert b"BB_CPU_THREADS" in blob
    # every key accepted, restored with -1; out-of-range keys / values refused
    for k in DIAG_KEYS.values():
        assert L.bb_diag_set(k, -1) == 0
    assert L.bb_diag_set(len(DIAG_KEYS), 0) < 0 and L.bb_diag_set(0, -2) < 0
    assert b"bb_diag_set" in L.bb_last_error()
