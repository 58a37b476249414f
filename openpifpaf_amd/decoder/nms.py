"""Keypoint and detection NMS (nms.py:11-102).

Inside the device decode the suppression runs after the seed loop and force-complete
(csrc/grow.hip, nms_kernel), configured from these class attributes exactly as the
reference's CifCaf(nms=nms.Keypoints()) is.  `Keypoints().annotations(anns)` runs the
same kernel over a host list of Annotation objects (pp_nms_keypoints): it mutates their
data in place as the reference does and returns the survivors, sorted by -score.  Each
annotation's own score() is honoured (fixed_score, suppress_score_index, score_weights:
pp_nms_keypoints_scored).
"""
import ctypes

import numpy as np
import torch

from .. import _device
from .._abi import ANN_DTYPE, DET_DTYPE, DetNms, make_config
from .._lib import call, load
from ..annotation import NOTSET


def _default_weights(k):
    w = np.ones((k,))
    w[:3] = 3.0
    return w / np.sum(w)


def _score_spec(anns, k):
    """Each annotation's Annotation.score() inputs (annotation.py:60-71) for
    pp_nms_keypoints_scored: (spec int32 (n,), score_weights float64 (n, k), fixed float64
    (n,)), or None when every annotation scores the default way."""
    default = _default_weights(k)
    custom = False
    for ann in anns:
        w = getattr(ann, 'score_weights', None)
        if (ann.fixed_score != NOTSET or ann.suppress_score_index is not None
                or w is None or not np.array_equal(np.asarray(w, np.float64), default)):
            custom = True
            break
    if not custom:
        return None
    n = len(anns)
    spec = np.full(n, -1, np.int32)
    sw = np.zeros((n, k), np.float64)
    fixed = np.zeros(n, np.float64)
    for i, ann in enumerate(anns):
        if ann.fixed_score != NOTSET:
            spec[i] = -2
            fixed[i] = float(ann.fixed_score)
            continue
        w = np.asarray(ann.score_weights, np.float64)
        if w.shape != (k,):
            raise ValueError('score_weights of length {} for {} keypoints'.format(len(w), k))
        sw[i] = w
        j = ann.suppress_score_index
        if j is not None:
            j = int(j)
            if not -k <= j < k:  # v[j] = 0.0 raises in the reference too
                raise IndexError('suppress_score_index {} is out of bounds for {} keypoints'
                                 .format(j, k))
            spec[i] = j % k
    return spec, sw, fixed


class Keypoints:
    suppression = 0.0
    instance_threshold = 0.0
    keypoint_threshold = 0.0
    occupancy_visualizer = None

    def config(self):
        return make_config(nms_keypoint_threshold=self.keypoint_threshold,
                           nms_instance_threshold=self.instance_threshold,
                           nms_suppression=self.suppression)

    def annotations(self, anns):
        if not anns:
            return anns
        k = len(anns[0].data)
        for ann in anns:
            if len(ann.data) != k:
                raise ValueError('annotations with different keypoint counts')
        if k > ANN_DTYPE['data'].shape[0]:
            raise ValueError('more keypoints than PP_MAX_KP')
        n = len(anns)
        spec = _score_spec(anns, k)
        recs = np.zeros(n, ANN_DTYPE)
        for i, ann in enumerate(anns):
            recs['data'][i, :k] = ann.data
            recs['joint_scales'][i, :k] = ann.joint_scales
        recs['n_keypoints'] = k
        dev = _device.require()
        width = ANN_DTYPE.itemsize
        d_in = torch.from_numpy(recs.view(np.uint8).reshape(n, width)).to(dev)
        d_out = torch.empty_like(d_in)
        d_counts = torch.tensor([n], dtype=torch.int32, device=dev)
        d_out_counts = torch.empty(1, dtype=torch.int32, device=dev)
        d_out_index = torch.empty(n, dtype=torch.int32, device=dev)
        ws = torch.empty(int(load().pp_nms_workspace_size(1, n)), dtype=torch.uint8, device=dev)
        cfg = self.config()
        # the float64 instance threshold the reference compares score() with (nms.py:21, 53)
        d_spec = d_sw = d_fixed = None
        if spec is not None:
            d_spec, d_sw, d_fixed = (torch.from_numpy(a).to(dev) for a in spec)
        call('pp_nms_keypoints_scored', _device.ptr(d_in), _device.ptr(d_counts), 1, k, n,
             ctypes.byref(cfg), float(self.instance_threshold), _device.ptr(d_spec),
             _device.ptr(d_sw), _device.ptr(d_fixed), _device.ptr(d_out),
             _device.ptr(d_out_counts), _device.ptr(d_out_index), _device.ptr(ws),
             ctypes.c_size_t(ws.numel()), _device.stream())
        mutated = np.frombuffer(d_in.cpu().numpy().tobytes(), dtype=ANN_DTYPE)
        m = int(d_out_counts.cpu().item())
        order = d_out_index[:m].cpu().numpy()
        for i, ann in enumerate(anns):  # the reference edits ann.data in place
            ann.data[:] = mutated['data'][i, :k]
        return [anns[int(i)] for i in order]


class Detection:
    """nms.py:60-102.  `annotations(anns)` runs pp_nms_detection on a host list of
    AnnotationDet (scores and order as the reference; scores edited in place)."""
    suppression = 0.1
    suppression_soft = 0.3
    instance_threshold = 0.1
    iou_threshold = 0.7
    iou_threshold_soft = 0.5

    @staticmethod
    def bbox_iou(box, other_boxes):
        """nms.py:67-77 (host arrays, as the reference)."""
        box = np.expand_dims(box, 0)
        x1 = np.maximum(box[:, 0], other_boxes[:, 0])
        y1 = np.maximum(box[:, 1], other_boxes[:, 1])
        x2 = np.minimum(box[:, 0] + box[:, 2], other_boxes[:, 0] + other_boxes[:, 2])
        y2 = np.minimum(box[:, 1] + box[:, 3], other_boxes[:, 1] + other_boxes[:, 3])
        inter_area = np.maximum(0.0, x2 - x1) * np.maximum(0.0, y2 - y1)
        box_area = box[:, 2] * box[:, 3]
        other_areas = other_boxes[:, 2] * other_boxes[:, 3]
        return inter_area / (box_area + other_areas - inter_area + 1e-5)

    def config(self):
        return DetNms(self.suppression, self.suppression_soft, self.instance_threshold,
                      self.iou_threshold, self.iou_threshold_soft, 1)

    def annotations(self, anns):
        if not anns:
            return anns
        n = len(anns)
        recs = np.zeros(n, DET_DTYPE)
        for i, a in enumerate(anns):
            recs[i]['field'] = a.field_i
            recs[i]['score'] = a.score
            recs[i]['bbox'] = np.asarray(a.bbox, dtype=np.float32)
        dev = _device.require()
        w = DET_DTYPE.itemsize
        d_in = torch.from_numpy(recs.view(np.uint8).reshape(n, w)).to(dev)
        d_out = torch.empty_like(d_in)
        d_counts = torch.tensor([n], dtype=torch.int32, device=dev)
        d_out_counts = torch.empty(1, dtype=torch.int32, device=dev)
        d_out_index = torch.empty(n, dtype=torch.int32, device=dev)
        d_scores = torch.empty(n, dtype=torch.float32, device=dev)
        ws = torch.empty(int(load().pp_nms_detection_workspace_size(1, n)), dtype=torch.uint8,
                         device=dev)
        z = self.config()
        call('pp_nms_detection', _device.ptr(d_in), _device.ptr(d_counts), 1, n,
             ctypes.byref(z), _device.ptr(d_out), _device.ptr(d_out_counts),
             _device.ptr(d_out_index), _device.ptr(d_scores), _device.ptr(ws),
             ctypes.c_size_t(ws.numel()), _device.stream())
        m = int(d_out_counts.cpu().item())
        order = d_out_index[:m].cpu().numpy()
        # the reference edits every annotation's score in place (nms.py:90-99)
        scores = d_scores.cpu().numpy()
        for ann, sc in zip(anns, scores):
            if ann.score >= self.instance_threshold:
                ann.score = np.float32(sc)
        return [anns[int(i)] for i in order]
