"""Host build of the product math (csrc/bb_math.h) next to the host libm it
restates (tests/probe/math_probe.cpp): built in-tree here, loaded by
tests/test_math.py and tests/test_gpu_math.py."""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "probe", "math_probe.cpp")
LIB = os.path.join(HERE, "probe", "libmath_probe.so")
HDR = os.path.join(HERE, "..", "madrona_basketball_amd", "csrc", "bb_math.h")


def load_math_probe():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(SRC), os.path.getmtime(HDR)):
        # -mfma (where the CPU has it) only speeds up fma_d; fma is exact either way
        fma = ["-mfma"] if "fma" in open("/proc/cpuinfo").read().split() else []
        # built under a per-process name and renamed into place: concurrent
        # test workers never load a half-written library
        tmp = f"{LIB}.{os.getpid()}.tmp"
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
                        *fma, "-pthread", "-o", tmp, SRC, "-lm"], check=True)
        os.replace(tmp, LIB)
    L = ctypes.CDLL(LIB)
    L.exhaustive_mismatches.restype = ctypes.c_int64
    L.exhaustive_double_mismatches.restype = ctypes.c_int64
    L.exhaustive_double_mismatches.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.POINTER(ctypes.c_uint32)]
    return L
