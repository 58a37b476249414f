"""The decoder's two NumPy scalar-math restatements, checked exhaustively on the CPU.

cifcaf.py:139 scores a CAF column as `np.exp(-0.5 * d**2 / sigma**2) * v` in float32:
- np.exp of a float32 array runs NumPy's SIMD routine (AVX512F / FMA3; the fixtures record
  AVX512_SKX, tests/golden/meta.json), which is not correctly rounded;
- `sigma**2` of a NumPy float32 SCALAR calls the C library's powf(sigma, 2.0f), glibc 2.35's
  FMA build, which is not always sigma * sigma.
The product restates both (pp_common.hpp np_exp_f32 / np_pow2_f32, used by the kernels and,
through pp_np_exp_cpu / pp_np_square_cpu, by these host twins); the oracle restates the exp
and calls libm's powf.  Here: every float32 in [-104, 0] through the product's exp and the
oracle's against np.exp itself, and every float32 >= 0 (2^31 values, zero, subnormals, inf
and NaN included) through the product's square against libm's powf, plus a sample of
NumPy's own scalar power (to pin that it is libm's powf).  The device forms are checked
against these host twins in tests/test_gpu_np_exp.py.
"""
import concurrent.futures
import ctypes
import os

import numpy as np
import pytest

import oracle

CHUNK = 1 << 24
THREADS = max(1, min(8, os.cpu_count() or 1))


def _product():
    from openpifpaf_amd._lib import load
    return load()


def _bits(lo, hi):
    return np.arange(lo, hi, dtype=np.uint64).astype(np.uint32).view(np.float32)


def _chunks(lo, hi):
    return [(s, min(hi, s + CHUNK)) for s in range(lo, hi, CHUNK)]


def _run_chunks(lo, hi, check):
    with concurrent.futures.ThreadPoolExecutor(THREADS) as ex:
        return sum(ex.map(lambda c: check(*c), _chunks(lo, hi)))


def test_exp_numpy_simd_exhaustive():
    """Every float32 in [-104, 0]: product host twin and oracle == np.exp, bit for bit."""
    lib, orc = _product(), oracle.lib()
    lo, hi = 0x80000000, int(np.float32(-104.0).view(np.uint32)) + 1

    def check(a, b):
        x = _bits(a, b)
        want = np.exp(x).view(np.uint32)
        got = np.empty_like(x)
        assert lib.pp_np_exp_cpu(x.ctypes.data, got.ctypes.data, len(x), 0) == 0
        orc_y = np.empty_like(x)
        orc.orc_np_exp(x.ctypes.data_as(ctypes.c_void_p), orc_y.ctypes.data_as(ctypes.c_void_p),
                       ctypes.c_long(len(x)))
        bad = np.count_nonzero(got.view(np.uint32) != want)
        bad_o = np.count_nonzero(orc_y.view(np.uint32) != want)
        assert bad == 0 and bad_o == 0, (hex(a), bad, bad_o)
        return len(x)

    assert _run_chunks(lo, hi, check) == hi - lo == 1120927745


def test_exp_edges_and_correct_mode():
    """NaN, +-inf, the overflow / underflow thresholds, positive arguments; exp_mode 1 is
    the correctly rounded exp (through float64)."""
    lib = _product()
    x = np.array([np.nan, np.inf, -np.inf, 0.0, -0.0, 88.72283935546875, 88.7228317,
                  -103.97208404541015625, -103.972076, 1.5, 10.0, 80.0, -87.5, -100.0,
                  np.float32(1e-30), -np.float32(1e-38)], np.float32)
    got = np.empty_like(x)
    assert lib.pp_np_exp_cpu(x.ctypes.data, got.ctypes.data, len(x), 0) == 0
    with np.errstate(over='ignore'):
        want = np.exp(x)
    assert np.array_equal(got, want, equal_nan=True)
    rng = np.random.default_rng(3)
    y = (-104 * rng.random(1 << 20)).astype(np.float32)
    got = np.empty_like(y)
    assert lib.pp_np_exp_cpu(y.ctypes.data, got.ctypes.data, len(y), 1) == 0
    assert np.array_equal(got, np.exp(y.astype(np.float64)).astype(np.float32))
    # the two modes differ (NumPy's SIMD exp is not correctly rounded)
    simd = np.empty_like(y)
    lib.pp_np_exp_cpu(y.ctypes.data, simd.ctypes.data, len(y), 0)
    assert 0.2 < np.mean(simd != got) < 0.5


def test_square_matches_libm_powf_exhaustive():
    """Every non-negative float32 (2^31 bit patterns): pp_np_square_cpu == libm powf(x, 2)."""
    lib, orc = _product(), oracle.lib()

    def check(a, b):
        x = _bits(a, b)
        got = np.empty_like(x)
        want = np.empty_like(x)
        assert lib.pp_np_square_cpu(x.ctypes.data, got.ctypes.data, len(x)) == 0
        orc.orc_np_square(x.ctypes.data_as(ctypes.c_void_p), want.ctypes.data_as(ctypes.c_void_p),
                          ctypes.c_long(len(x)))
        g, w = got.view(np.uint32), want.view(np.uint32)
        nan = np.isnan(got) & np.isnan(want)
        bad = np.count_nonzero((g != w) & ~nan)
        assert bad == 0, (hex(a), bad)
        return len(x)

    assert _run_chunks(0, 1 << 31, check) == 1 << 31


def test_square_is_numpys_scalar_power():
    """NumPy's float32 scalar `** 2` is libm's powf (sampled), and differs from x * x."""
    lib = _product()
    rng = np.random.default_rng(11)
    x = rng.integers(0x30000000, 0x48000000, size=200000, dtype=np.uint32).view(np.float32)
    numpy_scalar = np.array([v ** 2 for v in x], np.float32)
    got = np.empty_like(x)
    assert lib.pp_np_square_cpu(x.ctypes.data, got.ctypes.data, len(x)) == 0
    assert np.array_equal(got, numpy_scalar)
    assert np.count_nonzero(numpy_scalar != x * x) > 20


@pytest.mark.parametrize('mode', [0, 1])
def test_exp_rejects_bad_arguments(mode):
    lib = _product()
    x = np.zeros(4, np.float32)
    assert lib.pp_np_exp_cpu(x.ctypes.data, x.ctypes.data, 4, 2) != 0
    assert lib.pp_np_exp_cpu(None, x.ctypes.data, 4, mode) != 0
    assert lib.pp_np_square_cpu(x.ctypes.data, None, 4) != 0
