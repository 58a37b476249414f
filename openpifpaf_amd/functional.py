"""Drop-in for `openpifpaf.functional` (openpifpaf/functional.pyx), executed on gfx950.

Same names, signatures, defaults, return types and in-place semantics as the reference's
Cython module; same ValueError messages for buffers of the wrong dtype, rank or
writability (the typed-memoryview checks of functional.pyx).  Arrays may be NumPy
(copied to the device, computed by HIP kernels, copied back in place) or torch device
tensors (computed in place, results stay on the device).  There is no CPU path.
"""
import ctypes

import numpy as np
import torch

from . import _device
from ._abi import EXP_MODES
from ._lib import call

_CTYPE_NAMES = {
    np.dtype(np.float32): 'float', np.dtype(np.float64): 'double', np.dtype(np.int64): 'long',
    np.dtype(np.int32): 'int', np.dtype(np.int16): 'short', np.dtype(np.int8): 'signed char',
    np.dtype(np.uint8): 'unsigned char', np.dtype(np.uint16): 'unsigned short',
    np.dtype(np.uint32): 'unsigned int', np.dtype(np.uint64): 'unsigned long',
    np.dtype(np.float16): 'half', np.dtype(np.bool_): "'bool'",
}
_TORCH_NP = {torch.float32: np.float32, torch.float64: np.float64, torch.uint8: np.uint8,
             torch.int32: np.int32, torch.int64: np.int64}


def _buf(a, ndim, ctype='float'):
    """Typed-memoryview admission check (functional.pyx argument types)."""
    want = np.dtype(np.float32 if ctype == 'float' else np.uint8)
    if isinstance(a, torch.Tensor):
        got = np.dtype(_TORCH_NP.get(a.dtype, np.float64))
        nd = a.dim()
    else:
        if not isinstance(a, np.ndarray):
            a = np.asarray(a)
        if not a.flags.writeable:
            raise ValueError('buffer source array is read-only')
        got = a.dtype
        nd = a.ndim
    if nd != ndim:
        raise ValueError('Buffer has wrong number of dimensions (expected {}, got {})'
                         .format(ndim, nd))
    if got != want:
        raise ValueError("Buffer dtype mismatch, expected '{}' but got '{}'".format(
            _CTYPE_NAMES[want], _CTYPE_NAMES.get(got, str(got))))
    return a


def _on_device(*arrays):
    return any(_device.is_device(a) for a in arrays)


class _Field:
    """A 2-D field on the device (contiguous working copy when needed), written back on
    exit when the caller passed a host array or a non-contiguous tensor."""

    def __init__(self, a, dtype=torch.float32):
        self.src = a
        if _device.is_device(a) and a.is_contiguous():
            self.t = a
        else:
            self.t = _device.to_device(a, dtype)

    def finish(self):
        if self.t is self.src:
            return
        if isinstance(self.src, torch.Tensor):
            self.src.copy_(self.t)
        else:
            np.copyto(self.src, self.t.cpu().numpy())

    @property
    def args(self):
        h, w = self.t.shape
        return (ctypes.c_int64(h), ctypes.c_int64(w), ctypes.c_int64(w))


def _points(*arrays):
    return [_device.to_device(a) for a in arrays]


def _square(name, field, pts, *scalars):
    field = _buf(field, 2)
    pts = [_buf(p, 1) for p in pts]
    n = len(pts[0])
    f = _Field(field)
    d = _points(*pts)
    call(name, _device.ptr(f.t), *f.args, *[_device.ptr(t) for t in d], ctypes.c_int64(n),
         *scalars, _device.stream())
    f.finish()


def scalar_square_add_constant(field, x, y, width, v):
    """functional.pyx:7-26 (returns None, mutates field)."""
    _square('pp_scalar_square_add_constant', field, (x, y, width, v))


def cumulative_average(cuma, cumw, x, y, width, v, w):
    """functional.pyx:29-54."""
    cuma = _buf(cuma, 2)
    cumw = _buf(cumw, 2)
    pts = [_buf(p, 1) for p in (x, y, width, v, w)]
    fa, fw = _Field(cuma), _Field(cumw)
    d = _points(*pts)
    call('pp_cumulative_average', _device.ptr(fa.t), _device.ptr(fw.t), *fa.args,
         *[_device.ptr(t) for t in d], ctypes.c_int64(len(pts[0])), _device.stream())
    fa.finish()
    fw.finish()


def scalar_square_add_gauss(field, x, y, sigma, v, truncate=2.0):
    """functional.pyx:71-102."""
    _square('pp_scalar_square_add_gauss', field, (x, y, sigma, v), ctypes.c_float(truncate))


def scalar_square_add_gauss_with_max(field, x, y, sigma, v, truncate=2.0, max_value=1.0):
    """functional.pyx:105-141 (the CifHr splat)."""
    _square('pp_scalar_square_add_gauss_with_max', field, (x, y, sigma, v),
            ctypes.c_float(truncate), ctypes.c_float(max_value))


def scalar_square_max_gauss(field, x, y, sigma, v, truncate=2.0):
    """functional.pyx:144-169."""
    _square('pp_scalar_square_max_gauss', field, (x, y, sigma, v), ctypes.c_float(truncate))


def weiszfeld_nd(x_np, y_np, weights=None, epsilon=1e-8, max_steps=20):
    """functional.pyx:172-211: weighted Weiszfeld; mutates y_np, returns (y_np, denom)."""
    if weights is None:
        weights = np.ones(x_np.shape[0])  # float64 -> the reference's ValueError below
    weights = _buf(weights, 1)
    x = _buf(x_np, 2)
    y = _buf(y_np, 1)
    dev = _on_device(x, y, weights)
    xd = _device.to_device(x)
    yf = _Field.__new__(_Field)
    yf.src = y
    yf.t = y if (_device.is_device(y) and y.is_contiguous()) else _device.to_device(y)
    wd = _device.to_device(weights)
    denom = torch.zeros_like(wd)
    call('pp_weiszfeld_nd', _device.ptr(xd), ctypes.c_int64(xd.shape[0]),
         ctypes.c_int64(xd.shape[1]), ctypes.c_int64(xd.shape[1]), _device.ptr(yf.t),
         _device.ptr(wd), ctypes.c_float(epsilon), ctypes.c_int64(int(max_steps)),
         _device.ptr(denom), _device.stream())
    yf.finish()
    return y_np, (denom if dev else denom.cpu().numpy())


def _filter(field, x, y, sigma, mode, rows_min):
    field = _buf(field, 2)
    dev = _on_device(field)
    f = _device.to_device(field)
    rows, n = f.shape
    if mode == 3:
        out = torch.zeros(n, dtype=torch.uint8, device=f.device)
        pitch = n
    else:
        out = torch.empty((rows, n), dtype=torch.float32, device=f.device)
        pitch = n
    count = torch.zeros(1, dtype=torch.int32, device=f.device)
    if rows < rows_min:
        raise IndexError('Out of bounds on buffer access (axis 0)')
    call('pp_center_filter', _device.ptr(f), ctypes.c_int64(rows), ctypes.c_int64(n),
         ctypes.c_int64(n), ctypes.c_int32(mode), ctypes.c_float(x), ctypes.c_float(y),
         ctypes.c_float(sigma), _device.ptr(out), ctypes.c_int64(pitch), _device.ptr(count),
         _device.stream())
    if mode == 3:
        mask = out != 0
        return mask if dev else mask.cpu().numpy()
    k = int(count.item())
    res = out if dev else out.cpu().numpy()
    return res[:, :k]  # a view of a new (rows, n) array, like result_np[:, :result_i]


def paf_mask_center(paf_field, x, y, sigma=1.0):
    """functional.pyx:214-228."""
    return _filter(paf_field, x, y, sigma, 3, 4)


def scalar_values(field, x, y, default=-1):
    """functional.pyx:231-244: new float32 array of field[int(y), int(x)] or default."""
    field = _buf(field, 2)
    x = _buf(x, 1)
    y = _buf(y, 1)
    dev = _on_device(field, x, y)
    f = _Field(field)
    xd, yd = _points(x, y)
    out = torch.empty(len(x), dtype=torch.float32, device=f.t.device)
    call('pp_scalar_values', _device.ptr(f.t), *f.args, _device.ptr(xd), _device.ptr(yd),
         ctypes.c_int64(len(x)), ctypes.c_float(default), _device.ptr(out), _device.stream())
    return out if dev else out.cpu().numpy()


def _lookup(field, x, y, mode, default=0.0, r=1.0, ctype='float'):
    field = _buf(field, 2, ctype)
    dt = torch.float32 if ctype == 'float' else torch.uint8
    f = _Field(field, dt)
    xd = _device.to_device(np.array([x], np.float32))
    yd = _device.to_device(np.array([y], np.float32))
    out = torch.empty(1, dtype=dt, device=f.t.device)
    call('pp_scalar_lookup', _device.ptr(f.t), *f.args, ctypes.c_int32(mode), _device.ptr(xd),
         _device.ptr(yd), ctypes.c_int64(1), ctypes.c_float(default), ctypes.c_float(r),
         _device.ptr(out), _device.stream())
    v = out.item()
    return float(v) if ctype == 'float' else int(v)


def scalar_value(field, x, y, default=-1):
    """functional.pyx:247-253."""
    return _lookup(field, x, y, 0, default)


def scalar_value_clipped(field, x, y):
    """functional.pyx:256-261."""
    return _lookup(field, x, y, 1)


def scalar_nonzero(field, x, y, default=0):
    """functional.pyx:264-270."""
    return _lookup(field, x, y, 2, default, ctype='uchar')


def scalar_nonzero_clipped(field, x, y):
    """functional.pyx:273-278."""
    return _lookup(field, x, y, 3, ctype='uchar')


def scalar_nonzero_clipped_with_reduction(field, x, y, r):
    """functional.pyx:281-286."""
    return _lookup(field, x, y, 4, r=r, ctype='uchar')


def paf_center_b(paf_field, x, y, sigma=1.0):
    """functional.pyx:289-310."""
    return _filter(paf_field, x, y, sigma, 2, 4)


def paf_center(paf_field, x, y, sigma):
    """functional.pyx:313-335."""
    return _filter(paf_field, x, y, sigma, 1, 3)


def caf_center_s(caf_field, x, y, sigma):
    """functional.pyx:338-359 (the column filter inside _grow_connection)."""
    return _filter(caf_field, x, y, sigma, 0, 3)


__all__ = [
    'scalar_square_add_constant', 'cumulative_average', 'scalar_square_add_gauss',
    'scalar_square_add_gauss_with_max', 'scalar_square_max_gauss', 'weiszfeld_nd',
    'paf_mask_center', 'scalar_values', 'scalar_value', 'scalar_value_clipped',
    'scalar_nonzero', 'scalar_nonzero_clipped', 'scalar_nonzero_clipped_with_reduction',
    'paf_center_b', 'paf_center', 'caf_center_s',
]


def grow_connection_blend(caf_field, x, y, xy_scale, connection_method='blend',
                          exp_mode='numpy_simd'):
    """CifCaf._grow_connection + _target_with_blend (cifcaf.py:124-192), named
    `grow_connection_blend` by the north star.  caf_field: (9, N) column set (a CafScored
    forward/backward entry).  Returns (x, y, scale, score) as float32 scalars, or
    (0, 0, 0, 0) when no column lies within 2 * xy_scale of (x, y).  exp_mode: the
    scores' np.exp ('numpy_simd', NumPy's float32 SIMD routine, or 'correct';
    _abi.make_config)."""
    caf_field = _buf(caf_field, 2)
    method = {'blend': 0, 'max': 1}.get(connection_method)
    if method is None:
        raise Exception('connection method not known')
    if exp_mode not in EXP_MODES:
        raise ValueError('exp_mode must be one of {}'.format(sorted(EXP_MODES)))
    method |= EXP_MODES[exp_mode] << 1
    f = _device.to_device(caf_field)
    if f.shape[0] != 9:
        raise AssertionError('caf_field must have 9 rows')
    n = f.shape[1]
    out = torch.zeros(4, dtype=torch.float32, device=f.device)
    call('pp_grow_connection', _device.ptr(f), ctypes.c_int64(n), ctypes.c_int64(n),
         ctypes.c_float(x), ctypes.c_float(y), ctypes.c_float(xy_scale), ctypes.c_int32(method),
         _device.ptr(out), _device.stream())
    r = out.cpu().numpy()
    if not r.any():
        return 0, 0, 0, 0
    return tuple(np.float32(v) for v in r)


__all__.append('grow_connection_blend')
