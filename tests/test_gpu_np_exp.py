"""The device forms of the decoder's NumPy scalar-math restatements (pp_common.hpp
np_exp_f32 / np_pow2_f32 through pp_np_exp / pp_np_square) against np.exp and against the
host twins, which tests/test_np_exp.py checks exhaustively against np.exp and libm's powf.
gfx950 must give the same bits: fused multiply-adds, IEEE division, ldexp to subnormals."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHUNK = 1 << 26


def _dev_bits(lo, hi, step=1):
    import torch
    return torch.arange(lo, hi, step, dtype=torch.int64, device='cuda').to(torch.int32).view(
        torch.float32)


def _call(name, x, *args):
    import torch
    from openpifpaf_amd import _device
    from openpifpaf_amd._lib import call
    y = torch.empty_like(x)
    call(name, _device.ptr(x), _device.ptr(y), ctypes.c_int64(x.numel()), *args,
         _device.stream())
    return y


@pytest.mark.parametrize('step', [3])
def test_device_exp_matches_numpy(step):
    """Every 3rd float32 in [-104, 0] and every one in [-104, -87] (subnormal results)."""
    lo, hi = 0x80000000, int(np.float32(-104.0).view(np.uint32)) + 1
    sub_lo = int(np.float32(-87.0).view(np.uint32))
    n = 0
    for a, b, s in [(c, min(hi, c + CHUNK * step), step) for c in range(lo, hi, CHUNK * step)] + \
                   [(c, min(hi, c + CHUNK), 1) for c in range(sub_lo, hi, CHUNK)]:
        x = _dev_bits(a, b, s)
        got = _call('pp_np_exp', x, 0).cpu().numpy()
        want = np.exp(x.cpu().numpy())
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), hex(a)
        n += x.numel()
    assert n > 1120927745 // step


def test_device_exp_correct_mode_and_edges():
    import torch
    x = torch.tensor([float('nan'), float('inf'), -float('inf'), 0.0, -0.0, 88.72283935546875,
                      -103.97208404541015625, 1.5, 80.0], dtype=torch.float32, device='cuda')
    got = _call('pp_np_exp', x, 0).cpu().numpy()
    with np.errstate(over='ignore'):
        assert np.array_equal(got, np.exp(x.cpu().numpy()), equal_nan=True)
    y = -104 * torch.rand(1 << 22, device='cuda')
    got = _call('pp_np_exp', y, 1).cpu().numpy()
    assert np.array_equal(got, np.exp(y.cpu().numpy().astype(np.float64)).astype(np.float32))


def test_device_square_matches_host_twin():
    """Every 61st non-negative float32 bit pattern (zero, subnormals, inf and NaN included)
    and every float32 in [0.25, 64) (the decoder's sigma range): device == host twin."""
    from openpifpaf_amd._lib import load
    lib = load()
    ranges = [(c, min(1 << 31, c + CHUNK * 61), 61) for c in range(0, 1 << 31, CHUNK * 61)]
    lo, hi = int(np.float32(0.25).view(np.uint32)), int(np.float32(64.0).view(np.uint32))
    ranges += [(c, min(hi, c + CHUNK), 1) for c in range(lo, hi, CHUNK)]
    for a, b, s in ranges:
        x = _dev_bits(a, b, s)
        got = _call('pp_np_square', x).cpu().numpy()
        xh = x.cpu().numpy()
        want = np.empty_like(xh)
        assert lib.pp_np_square_cpu(xh.ctypes.data, want.ctypes.data, len(xh)) == 0
        same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
        assert same.all(), hex(a)
