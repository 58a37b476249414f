"""Occupancy grid (decoder/occupancy.py:10-47) held in device memory.

The decoder's own occupancy lives inside the seed-loop kernel (csrc/grow.hip).  This class
serves callers of the reference API: the grid is a (fields, H / r, W / r) u8 device tensor,
`set` marks boxes with pp_occupancy_set (decoder/utils.py:61-66 semantics: the box around
the rounded reduced position, u8 add that wraps) and `get` reads with
scalar_nonzero_clipped_with_reduction (pp_scalar_lookup).  `mark` takes arrays of marks in
one launch.
"""
import ctypes

import numpy as np
import torch

from .. import _device
from .._lib import call
from ..functional import scalar_nonzero_clipped_with_reduction


class Occupancy():
    def __init__(self, shape, reduction, *, min_scale=None):
        assert len(shape) == 3
        if min_scale is None:
            min_scale = reduction
        assert min_scale >= reduction
        self.reduction = reduction
        self.min_scale = min_scale
        self.min_scale_reduced = min_scale / reduction
        grid = (shape[0], int(shape[1] / reduction), int(shape[2] / reduction))
        self.occupancy = torch.zeros(grid, dtype=torch.uint8, device=_device.require())

    def __len__(self):
        return len(self.occupancy)

    def mark(self, fields, xs, ys, sigmas):
        """Occupancy.set for every (f, x, y, sigma), in order, in one device launch: x, y and
        sigma as float32 (the division and rounding run in f32 on the device, as the
        reference computes them for the decoder's float32 coordinates); f in range."""
        f = torch.as_tensor(np.asarray(fields, np.int32), device=self.occupancy.device)
        pts = [torch.as_tensor(np.asarray(a, np.float32), device=self.occupancy.device)
               for a in (xs, ys, sigmas)]
        _, h, w = self.occupancy.shape
        call('pp_occupancy_set', _device.ptr(self.occupancy), len(self.occupancy), h, w, w,
             _device.ptr(f), *[_device.ptr(t) for t in pts], ctypes.c_int64(len(f)),
             ctypes.c_float(self.reduction), ctypes.c_float(self.min_scale_reduced),
             _device.stream())

    def _plane(self, f):
        """self.occupancy[f] of the reference: negative f counts from the end."""
        n = len(self.occupancy)
        if not -n <= f < n:
            raise IndexError('index {} is out of bounds for axis 0 with size {}'.format(f, n))
        return f + n if f < 0 else f

    def set(self, f, x, y, sigma):
        """Setting is centered at the rounded (x, y) (u8 += 1 on the box, wrapping).  The
        box corners are rounded here exactly as occupancy.py:36-39 does (Python round() on
        the operands' own types: f32 for numpy float32 inputs, f64 for Python floats), then
        marked on the device."""
        if f >= len(self.occupancy):
            return
        f = self._plane(f)
        xi = round(x / self.reduction)
        yi = round(y / self.reduction)
        si = round(max(self.min_scale_reduced, sigma / self.reduction))
        # the kernel's own rounding of the already integral values is the identity
        _, h, w = self.occupancy.shape
        fa = torch.tensor([f], dtype=torch.int32, device=self.occupancy.device)
        pts = [torch.tensor([float(v)], dtype=torch.float32, device=self.occupancy.device)
               for v in (xi, yi, si)]
        call('pp_occupancy_set', _device.ptr(self.occupancy), len(self.occupancy), h, w, w,
             _device.ptr(fa), *[_device.ptr(t) for t in pts], ctypes.c_int64(1),
             ctypes.c_float(1.0), ctypes.c_float(0.0), _device.stream())

    def get(self, f, x, y):
        """Read at the floor of (x, y) / reduction, clipped to the grid."""
        if f >= len(self.occupancy):
            return 1.0
        return scalar_nonzero_clipped_with_reduction(self.occupancy[self._plane(f)], x, y,
                                                     self.reduction)
