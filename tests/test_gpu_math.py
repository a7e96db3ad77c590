"""The step's scalar math on gfx950 == the host build of the same header
(csrc/bb_math.h), bit for bit, over a strided sweep of every float (the
|x| >= 120 reduction of sinf/cosf, subnormals, infinities and NaNs
included), plus atan2f edge grids.  tests/test_math.py pins the host build
against glibc on every input; this closes the loop to the device code, whose
gameplay inputs never reach most of these paths."""
import ctypes

import numpy as np
import pytest
import torch

from tests.math_probe import load_math_probe

pytestmark = pytest.mark.gpu

# bb_diag_math fn ids (bb_common.hip k_math_probe) -> host probe function
FNS = {0: "bb_sinf", 1: "bb_cosf", 2: "bb_atanf", 3: "bb_acosf", 5: "bb_erff", 6: "bb_acospred", 7: "bb_expm1sum"}
STRIDE = 97  # 44 M of the 2^32 patterns


@pytest.fixture(scope="module")
def dev(native_lib):
    assert torch.cuda.is_available(), "GPU tests selected but no HIP device is visible"
    L = native_lib
    L.bb_diag_math.restype = ctypes.c_int
    L.bb_diag_math.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                               ctypes.c_int32, ctypes.c_void_p]
    return L


def device_eval(L, fn, x, y=None):
    xd = torch.from_numpy(x).cuda()
    yd = torch.from_numpy(y).cuda() if y is not None else None
    out = torch.empty_like(xd)
    rc = L.bb_diag_math(fn, xd.data_ptr(), yd.data_ptr() if yd is not None else None, out.data_ptr(), xd.numel(), 0,
                        torch.cuda.current_stream().cuda_stream)
    assert rc == 0, L.bb_last_error()
    torch.cuda.synchronize()
    return out.cpu().numpy()


def host_eval(P, name, x, y=None):
    out = np.empty_like(x)
    if y is None:
        getattr(P, name)(x.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(x.size))
    else:
        getattr(P, name)(y.ctypes.data_as(ctypes.c_void_p), x.ctypes.data_as(ctypes.c_void_p),
                         out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(x.size))
    return out


def same(a, b):
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


@pytest.mark.parametrize("fn", list(FNS))
def test_device_math_equals_host_build(dev, fn):
    P = load_math_probe()
    for start in (0, 41):
        bits = np.arange(start, 2**32, STRIDE, dtype=np.uint64).astype(np.uint32)
        x = bits.view(np.float32)
        if fn == 6:
            x = x[np.abs(x) <= 1.0]  # acos's domain
        x = np.ascontiguousarray(x)
        a, b = device_eval(dev, fn, x), host_eval(P, FNS[fn], x)
        ok = same(a, b)
        assert ok.all(), (FNS[fn], x[~ok][:4], a[~ok][:4], b[~ok][:4])


def test_device_atan2f_equals_host_build(dev):
    """atan2f(x, y) of bb_diag_math 4 is bbm::atan2f_(x, y): the host probe's
    bb_atan2f(y, x) argument order."""
    P = load_math_probe()
    rng = np.random.default_rng(11)
    n = 4_000_000
    bits = rng.integers(0, 2**32, size=(2, n), dtype=np.uint64).astype(np.uint32)
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-30, -1e-30, 1e30, 3.0, 1e-45, -1e-45,
                   3.4e38, -3.4e38], np.float32)
    gy, gx = np.meshgrid(sp, sp)
    e = rng.integers(-60, 60, n)
    cases = [(bits[0].view(np.float32), bits[1].view(np.float32)), (gy.ravel(), gx.ravel()),
             (rng.uniform(-40, 40, n), rng.uniform(-40, 40, n)),
             (rng.uniform(-1, 1, n) * 2.0 ** e, rng.uniform(-1, 1, n) * 2.0 ** np.clip(e + rng.integers(-70, 70, n),
                                                                                       -125, 125))]
    for y, x in cases:
        y = np.ascontiguousarray(y, np.float32)
        x = np.ascontiguousarray(x, np.float32)
        # device: atan2f_(first, second) with first = y
        a = device_eval(dev, 4, y, x)
        b = host_eval(P, "bb_atan2f", x, y)  # bb_atan2f(y, x) = atan2f_(y, x)
        ok = same(a, b)
        assert ok.all(), (y[~ok][:3], x[~ok][:3])


# bb_diag_divsqrt modes (bb_common.hip k_divsqrt_probe)
DIVSQRT = {"sqrt_short": 0, "rcp_refined": 1, "rcp_short1": 2, "div_short1": 3, "div_short2": 4, "v_sqrt_f32": 5}


def divsqrt_mismatches(L, mode, start, count, seed=0, blocks=8192):
    L.bb_diag_divsqrt.restype = ctypes.c_int
    L.bb_diag_divsqrt.argtypes = [ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
    counts = torch.zeros(blocks, dtype=torch.int32, device="cuda")
    ex = torch.zeros(2 * blocks, dtype=torch.int32, device="cuda")
    rc = L.bb_diag_divsqrt(mode, start, count, seed, counts.data_ptr(), ex.data_ptr(), blocks, 0,
                           torch.cuda.current_stream().cuda_stream)
    assert rc == 0, L.bb_last_error()
    torch.cuda.synchronize()
    c = counts.cpu().numpy().astype(np.int64)
    e = ex.cpu().numpy().view(np.uint32).reshape(-1, 2)
    bad = int(c.sum())
    examples = [(hex(a), hex(b)) for a, b in e[c > 0][:4]]
    return bad, examples


@pytest.mark.parametrize("name", ["sqrt_short", "rcp_short1"])
def test_short_path_divide_sqrt_equal_ieee_on_every_input(dev, name):
    """The short square root and reciprocal sequences of k_divsqrt_probe
    (bb_common.hip) == the IEEE operations (hipcc's correctly rounded
    expansions) on every float of their ranges (2^32 patterns, the rest
    skipped).  Diagnostic: the product keeps the IEEE operators."""
    bad, ex = divsqrt_mismatches(dev, DIVSQRT[name], 0, 2**32)
    assert bad == 0, (name, bad, ex)


def test_short_path_quotient_equals_ieee(dev):
    """The short quotient (two residual corrections) == a / b on 2^36
    pseudo-random operand pairs with both exponents in [2^-47, 2^48)."""
    for seed in range(16):
        bad, ex = divsqrt_mismatches(dev, DIVSQRT["div_short2"], 0, 2**32, seed=seed)
        assert bad == 0, (seed, bad, ex)


def test_divsqrt_variants_report(dev):
    """Which cheaper sequences would also be exact (reported, not asserted):
    the bare v_sqrt_f32, the refined reciprocal alone, Markstein's single
    correction."""
    out = {}
    for name in ("v_sqrt_f32", "rcp_refined"):
        out[name] = divsqrt_mismatches(dev, DIVSQRT[name], 0, 2**32)
    out["div_short1"] = divsqrt_mismatches(dev, DIVSQRT["div_short1"], 0, 2**32, seed=99)
    print("divsqrt variants:", out)
