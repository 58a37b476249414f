"""CafScored (caf_scored.py:13-98) on gfx950 (pp_caf_scored): per CAF field the forward
and backward (9, N) column sets, rescored with CifHr at both ends, row-major order."""
import ctypes

import numpy as np
import torch

from .. import _device
from .._abi import make_config, skeleton_array
from .._lib import call
from ._fields import batch1, head_scales, pitched_hr
from .field_config import FieldConfig


class CafScored:
    default_score_th = 0.1

    def __init__(self, cifhr, config: FieldConfig, skeleton, *, score_th=None, cif_floor=0.1):
        self.cifhr = cifhr
        self.config = config
        self.skeleton = skeleton
        self.score_th = score_th or self.default_score_th
        self.cif_floor = cif_floor
        self.forward = None
        self.backward = None

    def directed(self, caf_i, forward):
        if forward:
            return self.forward[caf_i], self.backward[caf_i]
        return self.backward[caf_i], self.forward[caf_i]

    def fill_caf(self, caf, stride, min_distance=0.0, max_distance=None):
        if min_distance or max_distance:
            raise NotImplementedError('CAF distance masks (multi-scale) are not implemented')
        if self.forward is not None:
            raise NotImplementedError('several CAF heads (multi-scale) are not implemented')
        c = batch1(caf)
        _, n_caf, _, h, w = c.shape
        hr = pitched_hr(self.cifhr)
        k = hr.shape[1]
        skel = skeleton_array(self.skeleton)[:n_caf]
        cols = torch.empty((1, n_caf, 2, 9, h * w), dtype=torch.float32, device=c.device)
        counts = torch.zeros((1, n_caf, 2), dtype=torch.int32, device=c.device)
        cfg = make_config(cif_floor=self.cif_floor, stride=int(stride))
        call('pp_caf_scored', _device.ptr(c), _device.ptr(hr), 1, k, n_caf, h, w,
             skel.ctypes.data_as(ctypes.c_void_p), ctypes.c_float(self.score_th),
             ctypes.byref(cfg), _device.ptr(cols), _device.ptr(counts), _device.stream())
        return self._set_columns(cols, counts, n_caf, not _device.is_device(caf))

    def _set_columns(self, cols, counts, n_caf, host):
        cnt = counts.cpu().numpy()[0]
        data = cols.cpu().numpy()[0] if host else cols[0]
        self.forward = [data[i, 1, :, :cnt[i, 1]] for i in range(n_caf)]
        self.backward = [data[i, 0, :, :cnt[i, 0]] for i in range(n_caf)]
        if host:
            self.forward = [np.ascontiguousarray(a) for a in self.forward]
            self.backward = [np.ascontiguousarray(a) for a in self.backward]
        return self

    def fill(self, fields):
        """caf_scored.py:88-98: every CAF head of the FieldConfig, columns concatenated."""
        if self.config.is_single_scale():
            _, caf_i, stride = self.config.single_scale()
            return self.fill_caf(fields[caf_i], stride)
        if self.forward is not None:
            raise NotImplementedError('several fill() calls are not implemented')
        arr, ts = head_scales(fields, self.config, 'caf')
        n_caf = ts[0].shape[1]
        cap = sum(t.shape[3] * t.shape[4] for t in ts)
        hr = pitched_hr(self.cifhr)
        k = hr.shape[1]
        skel = skeleton_array(self.skeleton)[:n_caf]
        cols = torch.empty((1, n_caf, 2, 9, cap), dtype=torch.float32, device=ts[0].device)
        counts = torch.zeros((1, n_caf, 2), dtype=torch.int32, device=ts[0].device)
        cfg = make_config(cif_floor=self.cif_floor)
        call('pp_caf_scored_multi', arr, len(arr), _device.ptr(hr), 1, k, n_caf,
             skel.ctypes.data_as(ctypes.c_void_p), ctypes.c_float(self.score_th),
             ctypes.byref(cfg), _device.ptr(cols), ctypes.c_int64(cap), _device.ptr(counts),
             _device.stream())
        host = not any(_device.is_device(fields[i]) for i in self.config.caf_indices)
        return self._set_columns(cols, counts, n_caf, host)
