"""CifSeeds (cif_seeds.py:13-64) on gfx950: threshold, CifHr rescore, ballot compaction
and the sorted(seeds, reverse=True) order, all in one kernel per image (pp_seeds)."""
import numpy as np
import torch

from .. import _device
from .._abi import SEED_DTYPE, check_seed_mask, make_config, scale_list
from .._lib import call
from ._fields import batch1, cfg_ptr, head_scales, pitched_hr, with_geometry
from .field_config import FieldConfig


class CifSeeds:
    threshold = None
    score_scale = 1.0

    def __init__(self, cifhr, config: FieldConfig):
        self.cifhr = cifhr
        self.config = config
        self.seeds = []

    def fill_cif(self, cif, stride, *, min_scale=0.0, seed_mask=None):
        """cif_seeds.py:23-50 for one head at `stride` (any stride: CifHr lookups go through
        the map's own geometry), appended to the seeds of earlier calls."""
        self._check_threshold()
        c = batch1(cif)
        _, k, _, h, w = c.shape
        arr = scale_list([(c.data_ptr(), h, w)], [], [int(stride)], [], [min_scale])
        self._run(with_geometry(arr, self.cifhr.shape), k, k * h * w, c.device, seed_mask)
        return self

    def _check_threshold(self):
        if self.threshold is None:
            raise TypeError("'>' not supported between instances of 'numpy.ndarray' and "
                            "'NoneType' (CifSeeds.threshold is not configured)")

    def _run(self, arr, k, cap, device, seed_mask):
        """pp_seeds_multi over the CIF entries of `arr`; the seeds of fields whose
        seed_mask entry is falsy are dropped (cif_seeds.py:28-29; the kernel's order is
        the sorted order, which dropping entries keeps)."""
        check_seed_mask(seed_mask, k)
        hr = pitched_hr(self.cifhr)
        out = torch.empty(max(1, cap) * SEED_DTYPE.itemsize, dtype=torch.uint8, device=device)
        count = torch.zeros(1, dtype=torch.int32, device=device)
        cfg = make_config(seed_threshold=self.threshold, seed_score_scale=self.score_scale)
        call('pp_seeds_multi', arr, len(arr), _device.ptr(hr), 1, k, cfg_ptr(cfg),
             _device.ptr(out), max(1, cap), _device.ptr(count), _device.stream())
        n = int(count.item())
        recs = np.frombuffer(out[:n * SEED_DTYPE.itemsize].cpu().numpy().tobytes(),
                             dtype=SEED_DTYPE)
        if seed_mask is not None:
            keep = np.array([bool(m) for m in seed_mask[:k]])
            recs = recs[keep[recs['field']]]
        self.seeds.extend((v, int(f), x, y, s) for v, f, x, y, s in
                          zip(recs['v'], recs['field'], recs['x'], recs['y'], recs['s']))

    def get(self):
        """cif_seeds.py:52-54 (the kernel already emits this order)."""
        return sorted(self.seeds, reverse=True)

    def fill(self, fields):
        """cif_seeds.py:56-64: every CIF head of the FieldConfig, in order."""
        self._check_threshold()
        if self.config.is_single_scale():
            cif_i, _, stride = self.config.single_scale()
            return self.fill_cif(fields[cif_i], stride, seed_mask=self.config.seed_mask)
        arr, ts = head_scales(fields, self.config, 'cif')
        k = ts[0].shape[1]
        cap = k * sum(t.shape[3] * t.shape[4] for t in ts)
        self._run(with_geometry(arr, self.cifhr.shape), k, cap, ts[0].device,
                  self.config.seed_mask)
        return self


class CifDetSeeds(CifSeeds):
    """cif_seeds.py:67-90: (v, field, x, y, w, h) seeds of detection fields."""

    def fill_cif(self, cif, stride, *, min_scale=0.0, seed_mask=None):
        """cif_seeds.py:68-90 for one detection head at `stride` (min-scale masks on p[4] and
        p[5]; CifHr lookups through the map's own geometry, which may be another head's),
        appended to the seeds of earlier calls (pp_cifdet_seeds_multi)."""
        if self.threshold is None:
            raise TypeError("'>' not supported between instances of 'float' and 'NoneType' "
                            "(CifSeeds.threshold is not configured)")
        c = batch1(cif)
        _, k, _, h, w = c.shape
        hr = pitched_hr(self.cifhr)
        arr = scale_list([(c.data_ptr(), h, w)], [], [int(stride)], [], [min_scale])
        arr = with_geometry(arr, self.cifhr.shape)
        seg = torch.empty((k, 5, h * w), dtype=torch.float32, device=c.device)
        counts = torch.zeros(k, dtype=torch.int32, device=c.device)
        cfg = make_config(seed_threshold=self.threshold, seed_score_scale=self.score_scale,
                          stride=int(stride), seed_mask=seed_mask)
        call('pp_cifdet_seeds_multi', arr, len(arr), _device.ptr(hr), 1, k, cfg_ptr(cfg),
             _device.ptr(seg), _device.ptr(counts), _device.stream())
        seg, counts = seg.cpu().numpy(), counts.cpu().numpy()
        for f in range(k):  # emission order: fields in order, cells in row-major order
            n = int(counts[f])
            self.seeds.extend((v, f, x, y, ww, hh) for v, x, y, ww, hh in zip(*seg[f, :, :n]))
        return self

    def fill(self, fields):
        """cif_seeds.py:56-64: every detection head of the FieldConfig, in order."""
        for cif_i, stride, min_scale in zip(self.config.cif_indices, self.config.cif_strides,
                                            self.config.cif_min_scales):
            self.fill_cif(fields[cif_i], stride, min_scale=min_scale,
                          seed_mask=self.config.seed_mask)
        return self
