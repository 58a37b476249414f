"""Host twins of `openpifpaf.functional` (functional.pyx): the `pp_*_cpu` entry points of
libpifpaf_amd.so (csrc/functional_cpu.hip), on NumPy arrays, in place, on the calling
thread -- SURVEY.md §8(b)'s `_cpu` variants.

Same names, signatures, defaults, return types and ValueError messages as
`openpifpaf_amd.functional` (the device API) and the reference's Cython module.  This is an
explicit choice of the caller: `openpifpaf_amd.functional` and the decoder never fall back
to it, and it raises, like every other entry point, when the library is missing.
(grow_connection_blend is decoder-internal, cifcaf.py:124-192, and stays device-only.)
"""
import ctypes

import numpy as np

from ._lib import call
from .functional import _buf


def _host(a):
    if not isinstance(a, np.ndarray):
        raise TypeError('functional_cpu takes NumPy arrays (openpifpaf_amd.functional takes '
                        'device tensors)')
    return a


class _Work:
    """A C-contiguous working copy of a (possibly strided) 2-D array, copied back on exit:
    the ABI takes a row pitch; the reference's memoryviews take any strides."""

    def __init__(self, a, dtype=np.float32):
        self.src = a
        self.a = a if a.flags.c_contiguous else np.ascontiguousarray(a, dtype)

    def finish(self):
        if self.a is not self.src:
            np.copyto(self.src, self.a)

    def args(self):
        h, w = self.a.shape
        return (self.a.ctypes.data, ctypes.c_int64(h), ctypes.c_int64(w), ctypes.c_int64(w))


def _pts(*arrays):
    out = [np.ascontiguousarray(_host(_buf(p, 1))) for p in arrays]
    return out, [p.ctypes.data for p in out]


def _square(name, field, pts, *scalars):
    f = _Work(_host(_buf(field, 2)))
    keep, ptrs = _pts(*pts)
    call(name, *f.args(), *ptrs, ctypes.c_int64(len(keep[0])), *scalars)
    f.finish()


def scalar_square_add_constant(field, x, y, width, v):
    """functional.pyx:7-26 (returns None, mutates field)."""
    _square('pp_scalar_square_add_constant_cpu', field, (x, y, width, v))


def cumulative_average(cuma, cumw, x, y, width, v, w):
    """functional.pyx:29-54."""
    fa, fw = _Work(_host(_buf(cuma, 2))), _Work(_host(_buf(cumw, 2)))
    keep, ptrs = _pts(x, y, width, v, w)
    call('pp_cumulative_average_cpu', fa.a.ctypes.data, fw.a.ctypes.data, *fa.args()[1:], *ptrs,
         ctypes.c_int64(len(keep[0])))
    fa.finish()
    fw.finish()


def scalar_square_add_gauss(field, x, y, sigma, v, truncate=2.0):
    """functional.pyx:71-102."""
    _square('pp_scalar_square_add_gauss_cpu', field, (x, y, sigma, v), ctypes.c_float(truncate))


def scalar_square_add_gauss_with_max(field, x, y, sigma, v, truncate=2.0, max_value=1.0):
    """functional.pyx:105-141 (the CifHr splat)."""
    _square('pp_scalar_square_add_gauss_with_max_cpu', field, (x, y, sigma, v),
            ctypes.c_float(truncate), ctypes.c_float(max_value))


def scalar_square_max_gauss(field, x, y, sigma, v, truncate=2.0):
    """functional.pyx:144-169."""
    _square('pp_scalar_square_max_gauss_cpu', field, (x, y, sigma, v), ctypes.c_float(truncate))


def weiszfeld_nd(x_np, y_np, weights=None, epsilon=1e-8, max_steps=20):
    """functional.pyx:172-211: weighted Weiszfeld; mutates y_np, returns (y_np, denom)."""
    if weights is None:
        weights = np.ones(x_np.shape[0])  # float64 -> the reference's ValueError below
    weights = _host(_buf(weights, 1))
    x = _Work(_host(_buf(x_np, 2)))
    y = _Work(_host(_buf(y_np, 1)))
    w = np.ascontiguousarray(weights)
    denom = np.zeros(len(w), np.float32)
    n, d = x.a.shape
    call('pp_weiszfeld_nd_cpu', x.a.ctypes.data, ctypes.c_int64(n), ctypes.c_int64(d),
         ctypes.c_int64(d), y.a.ctypes.data, w.ctypes.data, ctypes.c_float(epsilon),
         ctypes.c_int64(int(max_steps)), denom.ctypes.data, None)
    y.finish()
    return y_np, denom


def _filter(field, x, y, sigma, mode, rows_min):
    f = np.ascontiguousarray(_host(_buf(field, 2)))
    rows, n = f.shape
    if rows < rows_min:
        raise IndexError('Out of bounds on buffer access (axis 0)')
    out = np.zeros(n, np.uint8) if mode == 3 else np.empty((rows, n), np.float32)
    count = np.zeros(1, np.int32)
    call('pp_center_filter_cpu', f.ctypes.data, ctypes.c_int64(rows), ctypes.c_int64(n),
         ctypes.c_int64(n), ctypes.c_int32(mode), ctypes.c_float(x), ctypes.c_float(y),
         ctypes.c_float(sigma), out.ctypes.data, ctypes.c_int64(n), count.ctypes.data)
    if mode == 3:
        return out != 0
    return out[:, :int(count[0])]  # a view of a new (rows, n) array, like result_np[:, :result_i]


def paf_mask_center(paf_field, x, y, sigma=1.0):
    """functional.pyx:214-228."""
    return _filter(paf_field, x, y, sigma, 3, 4)


def scalar_values(field, x, y, default=-1):
    """functional.pyx:231-244: new float32 array of field[int(y), int(x)] or default."""
    f = _Work(_host(_buf(field, 2)))
    keep, ptrs = _pts(x, y)
    out = np.empty(len(keep[0]), np.float32)
    call('pp_scalar_values_cpu', *f.args(), *ptrs, ctypes.c_int64(len(out)),
         ctypes.c_float(default), out.ctypes.data)
    return out


def _lookup(field, x, y, mode, default=0.0, r=1.0, ctype='float'):
    dt = np.float32 if ctype == 'float' else np.uint8
    f = _Work(_host(_buf(field, 2, ctype)), dt)
    px, py = np.array([x], np.float32), np.array([y], np.float32)
    out = np.zeros(1, dt)
    call('pp_scalar_lookup_cpu', *f.args(), ctypes.c_int32(mode), px.ctypes.data,
         py.ctypes.data, ctypes.c_int64(1), ctypes.c_float(default), ctypes.c_float(r),
         out.ctypes.data)
    return float(out[0]) if ctype == 'float' else int(out[0])


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


def occupancy_set(occ, f, x, y, sigma, reduction=2.0, min_scale_reduced=2.0):
    """Occupancy.set for marks in order (occupancy.py:36-44 + decoder/utils.py:61-66) on a
    (planes, h, w) uint8 grid, in place (pp_occupancy_set_cpu)."""
    occ = _host(occ)
    if occ.dtype != np.uint8 or occ.ndim != 3 or not occ.flags.c_contiguous:
        raise ValueError('occupancy grid must be a C-contiguous (planes, h, w) uint8 array')
    fs = np.ascontiguousarray(f, np.int32)
    (xs, ys, ss), ptrs = _pts(*[np.ascontiguousarray(a, np.float32) for a in (x, y, sigma)])
    n_planes, h, w = occ.shape
    call('pp_occupancy_set_cpu', occ.ctypes.data, ctypes.c_int32(n_planes), ctypes.c_int64(h),
         ctypes.c_int64(w), ctypes.c_int64(w), fs.ctypes.data, *ptrs, ctypes.c_int64(len(fs)),
         ctypes.c_float(reduction), ctypes.c_float(min_scale_reduced))


__all__ = [
    'scalar_square_add_constant', 'cumulative_average', 'scalar_square_add_gauss',
    'scalar_square_add_gauss_with_max', 'scalar_square_max_gauss', 'weiszfeld_nd',
    'paf_mask_center', 'scalar_values', 'scalar_value', 'scalar_value_clipped',
    'scalar_nonzero', 'scalar_nonzero_clipped', 'scalar_nonzero_clipped_with_reduction',
    'paf_center_b', 'paf_center', 'caf_center_s', 'occupancy_set',
]
