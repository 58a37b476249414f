"""Keypoint NMS (nms.py:11-57).

Inside the device decode the suppression runs after the seed loop and force-complete
(csrc/grow.hip, nms_kernel), configured from these class attributes exactly as the
reference's CifCaf(nms=nms.Keypoints()) is.  `Keypoints().annotations(anns)` runs the
same kernel over a host list of Annotation objects (pp_nms_keypoints): it mutates their
data in place as the reference does and returns the survivors, sorted by -score.
"""
import ctypes

import numpy as np
import torch

from .. import _device
from .._abi import ANN_DTYPE, make_config
from .._lib import call, load
from ..annotation import NOTSET


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
            if ann.fixed_score != NOTSET or ann.suppress_score_index is not None:
                raise NotImplementedError('device NMS scores with the default Annotation.score()'
                                          ' (no fixed_score / suppress_score_index)')
            if len(ann.data) != k:
                raise ValueError('annotations with different keypoint counts')
        if k > ANN_DTYPE['data'].shape[0]:
            raise ValueError('more keypoints than PP_MAX_KP')
        n = len(anns)
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
        call('pp_nms_keypoints', _device.ptr(d_in), _device.ptr(d_counts), 1, k, n,
             ctypes.byref(cfg), _device.ptr(d_out), _device.ptr(d_out_counts),
             _device.ptr(d_out_index), _device.ptr(ws), ctypes.c_size_t(ws.numel()),
             _device.stream())
        mutated = np.frombuffer(d_in.cpu().numpy().tobytes(), dtype=ANN_DTYPE)
        m = int(d_out_counts.cpu().item())
        order = d_out_index[:m].cpu().numpy()
        for i, ann in enumerate(anns):  # the reference edits ann.data in place
            ann.data[:] = mutated['data'][i, :k]
        return [anns[int(i)] for i in order]
