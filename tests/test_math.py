"""The product's deterministic math (csrc/bb_math.h) vs the host libm it
restates: glibc 2.35's float functions, which the reference CPU executor calls
(src/game.cpp:302,345,435,806; src/helper.cpp:39,135-136), bit for bit on
every input; the double functions (erf/exp/acos, rounded to float by the
reference) within a few double ulps (DESIGN.md "Numerics")."""
import ctypes
import os

import numpy as np
import pytest

from tests.math_probe import load_math_probe


@pytest.fixture(scope="module")
def P():
    return load_math_probe()


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


def _fbits(x: float) -> int:
    return int(np.array([x], np.float32).view(np.uint32)[0])


# (check id of math_probe.cpp exhaustive_double_mismatches, [lo, hi) of 32-bit patterns)
_DOUBLE_DOMAINS = {
    # (float)erf((double)x) over every float (game.cpp:808 rounds it to float)
    "erf_pos": (5, 0x00000000, 0x7F800001),
    "erf_neg": (5, 0x80000000, 0xFF800001),
    # acos(c) > pi/8 for every float c in [-1, 1] (game.cpp:746-747; the step
    # compares c against the threshold Params.rot_thresh derived from acos_d)
    "acos_pred_pos": (7, 0x00000000, _fbits(1.0) + 1),
    "acos_pred_neg": (7, 0x80000000, _fbits(-1.0) + 1),
    # reward += exp(-0.4 dist) (game.cpp:868): every float x in [-104, 0]
    # (below that both are 0), summed onto the rewards a defender can hold
    # at that point of the step
    "exp_reward": (8, 0x80000000, _fbits(-104.0) + 1),
}


@pytest.mark.parametrize("dom", list(_DOUBLE_DOMAINS))
def test_double_functions_round_like_glibc_on_every_float(P, dom):
    """The step's double functions take a float and end in a float (or a
    float comparison): their float outcome equals glibc's on every input of
    the domain the step reaches (exhaustive), so the HIP path is bit-exact
    against the reference CPU executor's erf / acos / exp."""
    fn, lo, hi = _DOUBLE_DOMAINS[dom]
    first = ctypes.c_uint32()
    n = P.exhaustive_double_mismatches(fn, _threads(), lo, hi, ctypes.byref(first))
    assert n == 0, (dom, n, hex(first.value))


def test_exp_d_is_not_glibc_exp_in_double(P):
    """exp_d is not glibc's exp bit for bit in double (so the reward check
    above is on the float sums the step forms, not on the doubles)."""
    first = ctypes.c_uint32()
    n = P.exhaustive_double_mismatches(6, _threads(), 0x80000000, _fbits(-1.0), ctypes.byref(first))
    assert n > 0
