"""CifSeeds (cif_seeds.py:13-64) on gfx950: threshold, CifHr rescore, ballot compaction
and the sorted(seeds, reverse=True) order, all in one kernel per image (pp_seeds)."""
import numpy as np
import torch

from .. import _device
from .._abi import SEED_DTYPE, make_config
from .._lib import call
from ._fields import batch1, cfg_ptr, head_scales, pitched_hr
from .field_config import FieldConfig


class CifSeeds:
    threshold = None
    score_scale = 1.0

    def __init__(self, cifhr, config: FieldConfig):
        self.cifhr = cifhr
        self.config = config
        self.seeds = []

    def fill_cif(self, cif, stride, *, min_scale=0.0, seed_mask=None):
        if self.threshold is None:
            raise TypeError("'>' not supported between instances of 'numpy.ndarray' and "
                            "'NoneType' (CifSeeds.threshold is not configured)")
        if min_scale or seed_mask is not None:
            raise NotImplementedError('min_scale / seed_mask are not implemented')
        c = batch1(cif)
        _, k, _, h, w = c.shape
        hr = pitched_hr(self.cifhr)
        cap = k * h * w
        out = torch.empty(cap * SEED_DTYPE.itemsize, dtype=torch.uint8, device=c.device)
        count = torch.zeros(1, dtype=torch.int32, device=c.device)
        cfg = make_config(seed_threshold=self.threshold, seed_score_scale=self.score_scale,
                          stride=int(stride))
        call('pp_seeds', _device.ptr(c), _device.ptr(hr), 1, k, h, w, cfg_ptr(cfg),
             _device.ptr(out), cap, _device.ptr(count), _device.stream())
        n = int(count.item())
        recs = np.frombuffer(out[:n * SEED_DTYPE.itemsize].cpu().numpy().tobytes(),
                             dtype=SEED_DTYPE)
        self.seeds.extend((v, int(f), x, y, s) for v, f, x, y, s in
                          zip(recs['v'], recs['field'], recs['x'], recs['y'], recs['s']))
        return self

    def get(self):
        """cif_seeds.py:52-54 (the kernel already emits this order)."""
        return sorted(self.seeds, reverse=True)

    def fill(self, fields):
        """cif_seeds.py:56-64: every CIF head of the FieldConfig, in order."""
        if self.config.is_single_scale():
            cif_i, _, stride = self.config.single_scale()
            return self.fill_cif(fields[cif_i], stride, seed_mask=self.config.seed_mask)
        if self.threshold is None:
            raise TypeError("'>' not supported between instances of 'numpy.ndarray' and "
                            "'NoneType' (CifSeeds.threshold is not configured)")
        if self.config.seed_mask is not None:
            raise NotImplementedError('seed_mask is not implemented')
        arr, ts = head_scales(fields, self.config, 'cif')
        k = ts[0].shape[1]
        cap = k * sum(t.shape[3] * t.shape[4] for t in ts)
        hr = pitched_hr(self.cifhr)
        out = torch.empty(cap * SEED_DTYPE.itemsize, dtype=torch.uint8, device=ts[0].device)
        count = torch.zeros(1, dtype=torch.int32, device=ts[0].device)
        cfg = make_config(seed_threshold=self.threshold, seed_score_scale=self.score_scale)
        call('pp_seeds_multi', arr, len(arr), _device.ptr(hr), 1, k, cfg_ptr(cfg),
             _device.ptr(out), cap, _device.ptr(count), _device.stream())
        n = int(count.item())
        recs = np.frombuffer(out[:n * SEED_DTYPE.itemsize].cpu().numpy().tobytes(),
                             dtype=SEED_DTYPE)
        self.seeds.extend((v, int(f), x, y, s) for v, f, x, y, s in
                          zip(recs['v'], recs['field'], recs['x'], recs['y'], recs['s']))
        return self


class CifDetSeeds(CifSeeds):
    """cif_seeds.py:67-90: (v, field, x, y, w, h) seeds of detection fields."""

    def fill_cif(self, cif, stride, *, min_scale=0.0, seed_mask=None):
        if self.threshold is None:
            raise TypeError("'>' not supported between instances of 'float' and 'NoneType' "
                            "(CifSeeds.threshold is not configured)")
        if min_scale or seed_mask is not None:
            raise NotImplementedError('min_scale / seed_mask are not implemented')
        c = batch1(cif)
        _, k, _, h, w = c.shape
        hr = pitched_hr(self.cifhr)
        seg = torch.empty((k, 5, h * w), dtype=torch.float32, device=c.device)
        counts = torch.zeros(k, dtype=torch.int32, device=c.device)
        cfg = make_config(seed_threshold=self.threshold, seed_score_scale=self.score_scale,
                          stride=int(stride))
        call('pp_cifdet_seeds', _device.ptr(c), _device.ptr(hr), 1, k, h, w, cfg_ptr(cfg),
             _device.ptr(seg), _device.ptr(counts), _device.stream())
        seg, counts = seg.cpu().numpy(), counts.cpu().numpy()
        for f in range(k):  # emission order: fields in order, cells in row-major order
            n = int(counts[f])
            self.seeds.extend((v, f, x, y, ww, hh) for v, x, y, ww, hh in zip(*seg[f, :, :n]))
        return self
