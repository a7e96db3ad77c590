"""The product's deterministic math (csrc/bb_math.h) vs the host libm it
restates: glibc 2.35's float functions, which the reference CPU executor calls
(src/game.cpp:302,345,435,806; src/helper.cpp:39,135-136), bit for bit on
every input; the double functions (erf/exp/acos, rounded to float by the
reference) within a few double ulps (DESIGN.md "Numerics")."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "probe", "math_probe.cpp")
LIB = os.path.join(HERE, "probe", "libmath_probe.so")


@pytest.fixture(scope="module")
def P():
    hdr = os.path.join(HERE, "..", "madrona_basketball_amd", "csrc", "bb_math.h")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(SRC), os.path.getmtime(hdr)):
        # -mfma (where the CPU has it) only speeds up fma_d; fma is exact either way
        fma = ["-mfma"] if "fma" in open("/proc/cpuinfo").read().split() else []
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
                        *fma, "-pthread", "-o", LIB, SRC, "-lm"], check=True)
    L = ctypes.CDLL(LIB)
    L.exhaustive_mismatches.restype = ctypes.c_int64
    return L


def call(P, name, x, dtype=np.float32):
    x = np.ascontiguousarray(x, dtype=dtype)
    out = np.empty_like(x)
    getattr(P, name)(x.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(x.size))
    return out


def ulp_diff(a, b):
    ai = a.view(np.int32).astype(np.int64)
    bi = b.view(np.int32).astype(np.int64)
    ai = np.where(ai < 0, -(ai & 0x7FFFFFFF), ai)
    bi = np.where(bi < 0, -(bi & 0x7FFFFFFF), bi)
    return np.abs(ai - bi)


def inputs(lo, hi, n=400_000, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.uniform(lo, hi, n).astype(np.float32)
    specials = np.array([0.0, -0.0, 1e-30, -1e-30, 1e-8, lo, hi, np.float32(np.pi), np.float32(np.pi / 4),
                         np.float32(-np.pi / 2), np.float32(np.pi / 8)], np.float32)
    return np.concatenate([x, specials[(specials >= lo) & (specials <= hi)]])


def _threads():
    return max(1, min(8, os.cpu_count() or 1))


@pytest.mark.parametrize("fn", ["sinf", "cosf", "atanf", "acosf"])
def test_float_functions_equal_glibc_on_every_input(P, fn):
    """bb_math.h's restatement of glibc 2.35's float functions == the host
    libm, bit for bit, on all 2^32 inputs (NaNs compared as NaN)."""
    first = ctypes.c_uint32()
    n = P.exhaustive_mismatches(["sinf", "cosf", "atanf", "acosf"].index(fn), _threads(), ctypes.byref(first))
    assert n == 0, (fn, n, hex(first.value))


def test_glibc_sincosf_equals_sinf_and_cosf(P):
    """A compiler may fuse the reference's sinf/cosf pairs (game.cpp:345,
    helper.cpp:135-136) into sincosf: glibc's gives the same bits."""
    first = ctypes.c_uint32()
    assert P.exhaustive_mismatches(4, _threads(), ctypes.byref(first)) == 0, hex(first.value)


def _atan2(P, name, y, x):
    y = np.ascontiguousarray(y, np.float32)
    x = np.ascontiguousarray(x, np.float32)
    o = np.empty_like(x)
    getattr(P, name)(y.ctypes.data_as(ctypes.c_void_p), x.ctypes.data_as(ctypes.c_void_p),
                     o.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(x.size))
    return o


def test_atan2f_equals_glibc(P):
    rng = np.random.default_rng(1)
    n = 2_000_000
    bits = rng.integers(0, 2**32, size=(2, n), dtype=np.uint64).astype(np.uint32)
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-30, -1e-30, 1e30, 3.0, 1e-45], np.float32)
    sy, sx = np.meshgrid(sp, sp)
    e = rng.integers(-60, 60, n)
    e2 = np.clip(e + rng.integers(-70, 70, n), -125, 125)
    ys = [rng.uniform(-40, 40, n), bits[0].view(np.float32), sy.ravel(), rng.uniform(-1, 1, n) * 2.0 ** e]
    xs = [rng.uniform(-40, 40, n), bits[1].view(np.float32), sx.ravel(), rng.uniform(-1, 1, n) * 2.0 ** e2]
    for y, x in zip(ys, xs):
        a, b = _atan2(P, "bb_atan2f", y, x), _atan2(P, "glibc_atan2f", y, x)
        same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
        assert same.all(), (y[~same][:3], x[~same][:3])


@pytest.mark.parametrize("fn,lo,hi,rel", [("exp", -40, 0, 4e-16), ("acos", -1, 1, 4e-16), ("atan", -100, 100, 4e-16)])
def test_double_kernels_near_libm(P, fn, lo, hi, rel):
    x = np.random.default_rng(2).uniform(lo, hi, 200_000)
    got = call(P, "bb_" + fn, x, np.float64)
    ref = getattr(np, {"acos": "arccos", "atan": "arctan"}.get(fn, fn))(x)
    err = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300)
    assert np.quantile(err, 0.999) < rel and err.max() < 8 * rel, (fn, err.max())


def test_erf_absolute_error(P):
    import math
    # double accuracy below 4; from 4 on erf_d returns 1 (erfc(4) < 2^-25)
    x = np.concatenate([np.linspace(-3.999, 3.999, 20001), np.random.default_rng(3).uniform(-4, 4, 200000)])
    got = call(P, "bb_erf", x, np.float64)
    ref = np.array([math.erf(v) for v in x])
    assert np.abs(got - ref).max() < 4e-16
    # the float the step keeps ((float)erf, src/game.cpp:808) equals libm's
    xf = np.concatenate([np.random.default_rng(4).uniform(-4.5, 4.5, 200000), np.linspace(-7, 7, 20001)])
    xf = xf.astype(np.float32).astype(np.float64)
    got_f = call(P, "bb_erf", xf, np.float64).astype(np.float32)
    ref_f = np.array([math.erf(v) for v in xf]).astype(np.float32)
    assert (got_f == ref_f).all()


def test_glibc_float_functions_are_not_correctly_rounded(P):
    """Why the float functions restate glibc instead of computing the
    correctly rounded value: glibc's sinf differs from (float)sin((double)x) on
    ~1% of inputs, and one flip can fork a rollout."""
    x = inputs(-50, 50, seed=7)
    frac = (call(P, "glibc_sinf", x) != call(P, "cr_sinf", x)).mean()
    assert 0 < frac < 0.05, frac
