"""Preprocess inverse transforms (transforms/preprocess.py:15-95) on the device.

`Preprocess.annotations_inverse(annotations, meta)` maps decoded Annotation /
AnnotationDet objects from network-input to image coordinates exactly as the reference
(float64 offset / scale steps rounded to float32, float32 rotation), through
pp_annotations_inverse / pp_dets_inverse.  `inverse_records` applies the same kernels to
whole device batches of decoder records (one meta per image) without leaving the GPU.
"""
import copy
import ctypes

import numpy as np
import torch

from . import _device
from ._abi import ANN_DTYPE, DET_DTYPE
from ._lib import PPError, call
from .annotation import AnnotationDet


class InverseMeta(ctypes.Structure):
    """pp_inverse_meta (include/pifpaf_amd.h)."""
    _fields_ = [('offset', ctypes.c_double * 2), ('scale', ctypes.c_double * 2),
                ('rotation_angle', ctypes.c_double), ('rotation_width', ctypes.c_double),
                ('rotation_height', ctypes.c_double), ('width', ctypes.c_double),
                ('hflip', ctypes.c_int32), ('pad_', ctypes.c_int32)]


META_DTYPE = np.dtype([('offset', '<f8', (2,)), ('scale', '<f8', (2,)), ('rotation_angle', '<f8'),
                       ('rotation_width', '<f8'), ('rotation_height', '<f8'), ('width', '<f8'),
                       ('hflip', '<i4'), ('pad_', '<i4')])
assert META_DTYPE.itemsize == ctypes.sizeof(InverseMeta)


class _HorizontalSwap:
    """transforms/hflip.py:12-29: target row of each keypoint under a horizontal flip."""

    def __init__(self, keypoints, hflip):
        self.keypoints = keypoints
        self.hflip = hflip

    def __call__(self, keypoints):
        target = np.zeros(keypoints.shape)
        for source_i, xyv in enumerate(keypoints):
            target_name = self.hflip.get(self.keypoints[source_i])
            target_i = self.keypoints.index(target_name) if target_name else source_i
            target[target_i] = xyv
        return target


def swap_table(swap, k):
    """Target row of every source row of a row-permuting `horizontal_swap` callable, found
    by applying it once to rows that hold their own index."""
    probe = np.repeat(np.arange(1, k + 1, dtype=np.float64)[:, None], 3, axis=1)
    out = np.asarray(swap(probe))
    table = np.zeros(k, np.int32)
    seen = np.zeros(k, bool)
    for t in range(k):
        s = int(round(out[t, 0])) - 1
        if s >= 0:
            table[s] = t
            seen[s] = True
    if not seen.all():
        raise NotImplementedError('horizontal_swap that drops keypoints')
    return table


def meta_record(meta):
    rot = meta.get('rotation') or {'angle': 0.0, 'width': None, 'height': None}
    m = np.zeros(1, META_DTYPE)
    m['offset'] = np.asarray(meta['offset'], np.float64)
    m['scale'] = np.asarray(meta['scale'], np.float64)
    m['rotation_angle'] = rot['angle']
    m['rotation_width'] = rot['width'] if rot['width'] is not None else 0.0
    m['rotation_height'] = rot['height'] if rot['height'] is not None else 0.0
    m['width'] = float(meta['width_height'][0])
    m['hflip'] = 1 if meta['hflip'] else 0
    return m


def inverse_records(recs, counts, metas, k=17, hswap=None, det=False):
    """In place on device record batches (n_img, cap, record bytes) with per-image counts
    (device int32) and metas (device META_DTYPE bytes).  Returns per-image NaN flags."""
    n, cap = recs.shape[0], recs.shape[1]
    if det:
        call('pp_dets_inverse', _device.ptr(recs), _device.ptr(counts), n, cap,
             _device.ptr(metas), _device.stream())
        return None
    flags = torch.zeros(n, dtype=torch.int32, device=recs.device)
    call('pp_annotations_inverse', _device.ptr(recs), _device.ptr(counts), n, cap, k,
         _device.ptr(metas), _device.ptr(hswap), _device.ptr(flags), _device.stream())
    return flags


class Preprocess:
    @staticmethod
    def keypoint_sets_inverse(keypoint_sets, meta):
        """preprocess.py:15-32 on an (n, K, 3) array (a copy)."""
        kps = np.asarray(keypoint_sets, np.float32)
        n, k, _ = kps.shape
        if n == 0:
            return kps.copy()
        meta2 = dict(meta, rotation={'angle': 0.0, 'width': None, 'height': None})
        recs = np.zeros(n, ANN_DTYPE)
        recs['data'][:, :k] = kps
        out, _ = _run_poses(recs, k, meta2)
        return out['data'][:, :k].copy()

    @staticmethod
    def annotations_inverse(annotations, meta):
        """preprocess.py:35-82: deep copies, mapped to image coordinates."""
        annotations = copy.deepcopy(annotations)
        poses = [a for a in annotations if not isinstance(a, AnnotationDet)]
        dets = [a for a in annotations if isinstance(a, AnnotationDet)]
        if poses:
            k = len(poses[0].data)
            recs = np.zeros(len(poses), ANN_DTYPE)
            for i, a in enumerate(poses):
                recs[i]['data'][:k] = a.data
                recs[i]['joint_scales'][:k] = a.joint_scales
                nd = min(len(a.decoding_order), recs['decoding_xyv'].shape[1])
                recs[i]['n_decoding'] = nd
                for t in range(nd):
                    recs[i]['decoding_xyv'][t, :3] = a.decoding_order[t][2][:3]
                    recs[i]['decoding_xyv'][t, 3:] = a.decoding_order[t][3][:3]
            out, nan = _run_poses(recs, k, meta)
            if nan:
                raise AssertionError('NaN in annotation data (preprocess.py:67)')
            for i, a in enumerate(poses):
                a.data = out[i]['data'][:k].copy()
                a.joint_scales = out[i]['joint_scales'][:k].copy()
                for t, (j1, j2, c1, c2) in enumerate(a.decoding_order[:out[i]['n_decoding']]):
                    c1[:2] = out[i]['decoding_xyv'][t, 0:2]
                    c2[:2] = out[i]['decoding_xyv'][t, 3:5]
        if dets:
            recs = np.zeros(len(dets), DET_DTYPE)
            for i, a in enumerate(dets):
                recs[i]['field'] = a.field_i
                recs[i]['bbox'] = np.asarray(a.bbox, np.float32)
            dev = _device.require()
            w = DET_DTYPE.itemsize
            d = torch.from_numpy(recs.view(np.uint8).reshape(1, len(dets), w)).to(dev)
            counts = torch.tensor([len(dets)], dtype=torch.int32, device=dev)
            m = torch.from_numpy(meta_record(meta).view(np.uint8)).to(dev)
            inverse_records(d, counts, m, det=True)
            out = np.frombuffer(d.cpu().numpy().tobytes(), dtype=DET_DTYPE)
            for i, a in enumerate(dets):
                a.bbox = out[i]['bbox'].copy()
        return annotations


def _run_poses(recs, k, meta):
    dev = _device.require()
    n, w = len(recs), ANN_DTYPE.itemsize
    recs['n_keypoints'] = k
    d = torch.from_numpy(recs.view(np.uint8).reshape(1, n, w)).to(dev)
    counts = torch.tensor([n], dtype=torch.int32, device=dev)
    m = torch.from_numpy(meta_record(meta).view(np.uint8)).to(dev)
    hswap = None
    if meta['hflip'] and meta.get('horizontal_swap'):
        hswap = torch.from_numpy(swap_table(meta['horizontal_swap'], k)).to(dev)
    flags = inverse_records(d, counts, m, k=k, hswap=hswap)
    if flags is None:
        raise PPError('pp_annotations_inverse failed')
    out = np.frombuffer(d.cpu().numpy().tobytes(), dtype=ANN_DTYPE)
    return out, bool(flags.cpu().numpy().any())
