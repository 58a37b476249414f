"""CafScored (caf_scored.py:13-98) on gfx950 (pp_caf_scored): per CAF field the forward
and backward (9, N) column sets, rescored with CifHr at both ends, row-major order."""
import ctypes

import numpy as np
import torch

from .. import _device
from .._abi import make_config, scale_list, skeleton_array
from .._lib import call
from ._fields import batch1, head_scales, pitched_hr, with_geometry
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
        """caf_scored.py:32-86 for one head at `stride` with its distance masks; the
        columns are appended to those of earlier calls (np.concatenate per field)."""
        c = batch1(caf)
        _, n_caf, _, h, w = c.shape
        arr = scale_list([], [(c.data_ptr(), h, w)], [], [int(stride)], None, [min_distance],
                         [max_distance])
        return self._run(with_geometry(arr, self.cifhr.shape), n_caf, h * w, c.device,
                         not _device.is_device(caf))

    def _run(self, arr, n_caf, cap, device, host):
        hr = pitched_hr(self.cifhr)
        k = hr.shape[1]
        skel = skeleton_array(self.skeleton)[:n_caf]
        cols = torch.empty((1, n_caf, 2, 9, max(1, cap)), dtype=torch.float32, device=device)
        counts = torch.zeros((1, n_caf, 2), dtype=torch.int32, device=device)
        cfg = make_config(cif_floor=self.cif_floor)
        call('pp_caf_scored_multi', arr, len(arr), _device.ptr(hr), 1, k, n_caf,
             skel.ctypes.data_as(ctypes.c_void_p), ctypes.c_float(self.score_th),
             ctypes.byref(cfg), _device.ptr(cols), ctypes.c_int64(max(1, cap)),
             _device.ptr(counts), _device.stream())
        cnt = counts.cpu().numpy()[0]
        data = cols.cpu().numpy()[0] if host else cols[0]
        fwd = [data[i, 1, :, :cnt[i, 1]] for i in range(n_caf)]
        bwd = [data[i, 0, :, :cnt[i, 0]] for i in range(n_caf)]
        if host:
            fwd = [np.ascontiguousarray(a) for a in fwd]
            bwd = [np.ascontiguousarray(a) for a in bwd]
        if self.forward is None:
            self.forward, self.backward = fwd, bwd
        else:
            cat = (lambda a, b: np.concatenate((a, np.asarray(b)), axis=1)) if host else \
                (lambda a, b: torch.cat((_device.to_device(a), b), dim=1))
            self.forward = [cat(a, b) for a, b in zip(self.forward, fwd)]
            self.backward = [cat(a, b) for a, b in zip(self.backward, bwd)]
        return self

    def fill(self, fields):
        """caf_scored.py:88-98: every CAF head of the FieldConfig, columns concatenated."""
        if self.config.is_single_scale():
            _, caf_i, stride = self.config.single_scale()
            return self.fill_caf(fields[caf_i], stride)
        arr, ts = head_scales(fields, self.config, 'caf')
        cap = sum(t.shape[3] * t.shape[4] for t in ts)
        host = not any(_device.is_device(fields[i]) for i in self.config.caf_indices)
        return self._run(with_geometry(arr, self.cifhr.shape), ts[0].shape[1], cap,
                         ts[0].device, host)
