"""CifHr: the high-resolution CIF confidence map (cif_hr.py:14-81) on gfx950.

`fill(fields)` runs pp_cifhr (splat compaction + LDS-tiled gather-fold, bit-exact with
scalar_square_add_gauss_with_max in ascending splat order).  `.accumulated` is a NumPy
(K, H', W') array for host inputs, a device tensor view for device inputs.
"""
import ctypes

import numpy as np
import torch

from .. import _device
from .._abi import make_config, scale_list
from .._lib import call, load
from ..functional import scalar_square_add_gauss_with_max
from ._fields import batch1, head_scales, hr_geometry, with_geometry
from .field_config import FieldConfig


def cifhr_device(cif, stride, v_threshold, neighbors):
    """cif (n, K, 5, H, W) device tensor -> (n, K, H', pitch) device tensor."""
    n, k, _, h, w = cif.shape
    hh, _, pitch = hr_geometry(h, w, stride)
    lib = load()
    out = torch.empty((n, k, hh, pitch), dtype=torch.float32, device=cif.device)
    ws = torch.empty(lib.pp_cifhr_workspace_size(n, k, h, w), dtype=torch.uint8,
                     device=cif.device)
    cfg = make_config(cif_threshold=v_threshold, stride=stride, cif_neighbors=neighbors)
    call('pp_cifhr', _device.ptr(cif), n, k, h, w, ctypes.byref(cfg), _device.ptr(out),
         _device.ptr(ws), ctypes.c_size_t(ws.numel()), _device.stream())
    return out


def cifhr_sparse_device(cif, stride, v_threshold, neighbors):
    """cif (n, K, 5, H, W) device tensor -> the decoder's block-sparse CifHr
    (pp_cifhr_sparse): (map (n, K, T, 64, 64) f32, masks (n, K, T) int64 block bits)."""
    n, k, _, h, w = cif.shape
    lib = load()
    t = int(lib.pp_cifhr_sparse_tiles(h, w, stride))
    hmap = torch.empty((n, k, t, 64, 64), dtype=torch.float32, device=cif.device)
    masks = torch.empty((n, k, t), dtype=torch.int64, device=cif.device)
    ws = torch.empty(max(1, lib.pp_cifhr_sparse_workspace_size(n, k, h, w)), dtype=torch.uint8,
                     device=cif.device)
    cfg = make_config(cif_threshold=v_threshold, stride=stride, cif_neighbors=neighbors)
    call('pp_cifhr_sparse', _device.ptr(cif), n, k, h, w, ctypes.byref(cfg), _device.ptr(hmap),
         _device.ptr(masks), _device.ptr(ws), ctypes.c_size_t(ws.numel()), _device.stream())
    return hmap, masks


def sparse_to_dense(hmap, masks, hh, ww):
    """Host (numpy) expansion of a block-sparse CifHr (cifhr_sparse_device) to (..., hh, ww);
    blocks whose mask bit is clear read as 0, as HrMap::at does."""
    import numpy as np
    hmap = np.asarray(hmap)
    bits = np.asarray(masks).view(np.uint64)
    lead, t = hmap.shape[:-3], hmap.shape[-3]
    pitch = -(-ww // 32) * 32
    tx = -(-pitch // 64)
    ty = t // tx
    blk = hmap.reshape(lead + (t, 8, 8, 8, 8))  # (tile, by, bx, py, px)
    on = ((bits[..., None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool)
    blk = np.where(on.reshape(lead + (t, 8, 8, 1, 1)), blk, np.float32(0))
    full = blk.reshape(lead + (ty, tx, 8, 8, 8, 8)).transpose(
        tuple(range(len(lead))) + tuple(len(lead) + i for i in (0, 2, 4, 1, 3, 5)))
    full = full.reshape(lead + (ty * 64, tx * 64))
    return full[..., :hh, :ww]


def cifdet_hr_device(det, stride, v_threshold, neighbors):
    """det (n, K, 7, H, W) device tensor -> (n, K, H', pitch) device tensor (pp_cifdet_hr)."""
    n, k, _, h, w = det.shape
    hh, _, pitch = hr_geometry(h, w, stride)
    lib = load()
    out = torch.empty((n, k, hh, pitch), dtype=torch.float32, device=det.device)
    ws = torch.empty(lib.pp_cifhr_workspace_size(n, k, h, w), dtype=torch.uint8,
                     device=det.device)
    cfg = make_config(cif_threshold=v_threshold, stride=stride, cif_neighbors=neighbors)
    call('pp_cifdet_hr', _device.ptr(det), n, k, h, w, ctypes.byref(cfg), _device.ptr(out),
         _device.ptr(ws), ctypes.c_size_t(ws.numel()), _device.stream())
    return out


class CifHr:
    neighbors = 16
    v_threshold = 0.1
    _multi_entry = 'pp_cifhr_multi'  # the head-list launcher (_run_multi)

    def __init__(self, config: FieldConfig):
        self.config = config
        self.accumulated = None

    def accumulate(self, len_cifs, t, p, stride, min_scale):
        """cif_hr.py:26-40, for one field p (5, H, W) into t (H', W') in place."""
        p = p[:, p[0] > self.v_threshold]
        if min_scale:
            p = p[:, p[4] > min_scale / stride]
        v, x, y, _, scale = p
        x = x * stride
        y = y * stride
        sigma = np.maximum(1.0, 0.5 * scale * stride)
        scalar_square_add_gauss_with_max(t, x, y, sigma, v / self.neighbors / len_cifs,
                                         truncate=1.0)

    def fill_cif(self, cif, stride, min_scale=0.0):
        return self.fill_multiple([cif], stride, min_scale)

    def fill_multiple(self, cifs, stride, min_scale=0.0):
        """cif_hr.py:42-57: the heads accumulated into one zero map with len_cifs =
        len(cifs) (pp_cifhr_multi, one group of len(cifs) heads), at the size of the
        existing map if there is one (else from cifs[0] and stride), then combined with it
        by np.maximum."""
        ts = [batch1(c) for c in cifs]
        k, h, w = ts[0].shape[1], ts[0].shape[3], ts[0].shape[4]
        if self.accumulated is None:
            hh, ww, _ = hr_geometry(h, w, int(stride))
        else:
            if self.accumulated.shape[0] != k:
                raise ValueError('CIF heads with {} fields into a map of {}'.format(
                    k, self.accumulated.shape[0]))
            hh, ww = self.accumulated.shape[1:]
        n = len(ts)
        arr = scale_list([(t.data_ptr(), t.shape[3], t.shape[4]) for t in ts], [],
                         [int(stride)] * n, [], [min_scale] * n)
        arr = with_geometry(arr, (hh, ww))
        groups = n if n > 1 else 0  # one group of all n heads
        ta = self._run_multi(arr, groups, k, hh, ww, ts[0].device)
        device = any(_device.is_device(c) for c in cifs) or _device.is_device(self.accumulated)
        if self.accumulated is None:
            self.accumulated = ta if device else np.ascontiguousarray(ta.cpu().numpy())
        elif device:
            self.accumulated = torch.maximum(ta, _device.to_device(self.accumulated))
        else:  # np.maximum(ta, accumulated): NaN propagates, as torch.maximum does
            self.accumulated = np.maximum(ta.cpu().numpy(), self.accumulated)
        return self

    def _run_multi(self, arr, groups, k, hh, ww, device):
        """pp_cifhr_multi (pp_cifdet_hr_multi for CifDetHr) -> the (K, hh, ww) device view
        of its pitched output."""
        lib = load()
        pitch = int(lib.pp_cifhr_pitch(ww))
        out = torch.empty((1, k, hh, pitch), dtype=torch.float32, device=device)
        ws = torch.empty(max(1, int(lib.pp_cifhr_multi_workspace_size(arr, len(arr), groups, 1,
                                                                      k))),
                         dtype=torch.uint8, device=device)
        cfg = make_config(cif_threshold=self.v_threshold, cif_neighbors=self.neighbors)
        call(self._multi_entry, arr, len(arr), groups, 1, k, ctypes.byref(cfg), _device.ptr(out),
             _device.ptr(ws), ctypes.c_size_t(ws.numel()), _device.stream())
        return out[0, :, :, :ww]

    def fill(self, fields):
        """cif_hr.py:59-73: every CIF head of the FieldConfig, pairs when there are 10 (one
        pp_cifhr_multi call; the groups' maps are combined by np.maximum on the device)."""
        if self.config.is_single_scale():
            cif_i, _, stride = self.config.single_scale()
            return self.fill_cif(fields[cif_i], stride)
        if self.accumulated is not None:  # into an existing map: head group by head group
            if len(self.config.cif_indices) == 10:
                for i1, i2, stride, ms in zip(self.config.cif_indices[:5],
                                              self.config.cif_indices[5:],
                                              self.config.cif_strides[:5],
                                              self.config.cif_min_scales[:5]):
                    self.fill_multiple([fields[i1], fields[i2]], stride, min_scale=ms)
            else:
                for i, stride, ms in zip(self.config.cif_indices, self.config.cif_strides,
                                         self.config.cif_min_scales):
                    self.fill_cif(fields[i], stride, min_scale=ms)
            return self
        arr, ts = head_scales(fields, self.config, 'cif')
        _, k, _, h, w = ts[0].shape
        hh, ww, _ = hr_geometry(h, w, int(self.config.cif_strides[0]))
        acc = self._run_multi(arr, int(len(self.config.cif_indices) == 10), k, hh, ww,
                              ts[0].device)
        host = not any(_device.is_device(fields[i]) for i in self.config.cif_indices)
        self.accumulated = np.ascontiguousarray(acc.cpu().numpy()) if host else acc
        return self


class CifDetHr(CifHr):
    """cif_hr.py:84-100: detection fields (K, 7, H, W), min-scale masks on w and h,
    sigma = max(1, 0.1 min(w, h) stride).  fill_cif / fill_multiple / fill are CifHr's (the
    reference's CifDetHr inherits them): one head, several heads combined by np.maximum, the
    10-head pairs, on pp_cifdet_hr_multi."""
    _multi_entry = 'pp_cifdet_hr_multi'

    def accumulate(self, len_cifs, t, p, stride, min_scale):
        p = p[:, p[0] > self.v_threshold]
        if min_scale:
            p = p[:, p[4] > min_scale / stride]
            p = p[:, p[5] > min_scale / stride]
        v, x, y, _, w, h, _ = p
        x = x * stride
        y = y * stride
        sigma = np.maximum(1.0, 0.1 * np.minimum(w, h) * stride)
        scalar_square_add_gauss_with_max(t, x, y, sigma, v / self.neighbors / len_cifs,
                                         truncate=1.0)
