"""CifDet (decoder/generator/cifdet.py:17-52) on gfx950.

Same constructor and call signature as the reference.  One call runs CifDetHr, CifDetSeeds,
the occupancy loop and nms.Detection on the device for one image (`__call__`) or a whole
batch (`decode_batch`), configured from the CifHr / CifSeeds / nms.Detection class
attributes as the reference's decoder.configure() sets them.
"""
import ctypes

import numpy as np
import torch

from ... import _device
from ..._abi import DET_DTYPE, DetNms, check_seed_mask, make_config, scale_list
from ..._lib import PPError, call, load
from ...annotation import AnnotationDet
from .. import nms
from ..cif_hr import CifHr
from ..cif_seeds import CifSeeds
from ..field_config import FieldConfig
from .generator import Generator

PP_ST_ANN_OVERFLOW = 1


def det_nms_config(cls=None):
    cls = cls or nms.Detection
    return DetNms(cls.suppression, cls.suppression_soft, cls.instance_threshold,
                  cls.iou_threshold, cls.iou_threshold_soft, 1)


class CifDet(Generator):
    occupancy_visualizer = None
    supports_sharding = True

    def __init__(self, field_config: FieldConfig, categories, *, worker_pool=None):
        super().__init__(worker_pool)
        self.field_config = field_config
        self.categories = categories
        self._ws = None

    def single_head(self):
        """One detection head without a min scale: pp_cifdet_decode; anything else (several
        heads, min-scale masks) runs pp_cifdet_decode_multi."""
        fc = self.field_config
        return len(fc.cif_indices) == 1 and not fc.cif_min_scales[0]

    def head_fields(self, fields):
        """The FieldConfig's detection heads of a field list, in cif_indices order."""
        return [fields[i] for i in self.field_config.cif_indices]

    def config(self):
        if CifSeeds.threshold is None:
            raise TypeError("'>' not supported between instances of 'float' and 'NoneType' "
                            "(CifSeeds.threshold is not configured)")
        stride = int(self.field_config.cif_strides[0])
        check_seed_mask(self.field_config.seed_mask, len(self.categories))
        return make_config(cif_threshold=CifHr.v_threshold, seed_threshold=CifSeeds.threshold,
                           seed_score_scale=CifSeeds.score_scale, stride=int(stride),
                           cif_neighbors=CifHr.neighbors, seed_mask=self.field_config.seed_mask)

    def decode_records(self, det_batch, cap=None):
        """det_batch (B, K, 7, H, W), or with several heads / min scales the list of the
        FieldConfig's heads (each (B, K, 7, H_m, W_m), cif_indices order) -> (pp_det
        records, per-image offsets)."""
        heads = [_device.to_device(t) for t in
                 (det_batch if isinstance(det_batch, (list, tuple)) else [det_batch])]
        for det in heads:
            if det.dim() != 5 or det.shape[2] != 7:
                raise ValueError('expected CifDet fields (B, K, 7, H, W)')
        if len(heads) != len(self.field_config.cif_indices):
            raise ValueError('expected {} CifDet heads, got {}'.format(
                len(self.field_config.cif_indices), len(heads)))
        det = heads[0]
        b, k, _, h, w = det.shape
        if any(t.shape[:3] != det.shape[:3] for t in heads):
            raise ValueError('CifDet heads differ in batch or field count')
        cfg = self.config()
        z = det_nms_config()
        cells = sum(t.shape[3] * t.shape[4] for t in heads)
        fc = self.field_config
        multi = not self.single_head()
        arr = scale_list([(t.data_ptr(), t.shape[3], t.shape[4]) for t in heads], [],
                         fc.cif_strides, [], fc.cif_min_scales) if multi else None
        pairs = int(len(heads) == 10)  # CifHr.fill's 10-head layout (cif_hr.py:68-73)
        cap = cap or max(64, h * w)
        while True:
            if multi:
                size = int(load().pp_cifdet_multi_workspace_size(arr, len(arr), pairs, b, k, cap))
            else:
                size = int(load().pp_cifdet_workspace_size(b, k, h, w, ctypes.byref(cfg), cap))
            if self._ws is None or self._ws.numel() < size:
                self._ws = torch.empty(size, dtype=torch.uint8, device=det.device)
            out = torch.empty((b, cap, DET_DTYPE.itemsize), dtype=torch.uint8, device=det.device)
            counts = torch.empty(b, dtype=torch.int32, device=det.device)
            status = torch.empty(b, dtype=torch.int32, device=det.device)
            if multi:
                call('pp_cifdet_decode_multi', arr, len(arr), pairs, b, k, ctypes.byref(cfg),
                     ctypes.byref(z), _device.ptr(None), _device.ptr(out), cap,
                     _device.ptr(counts), _device.ptr(status), _device.ptr(self._ws),
                     ctypes.c_size_t(self._ws.numel()), _device.stream())
            else:
                call('pp_cifdet_decode', _device.ptr(det), b, k, h, w, ctypes.byref(cfg),
                     ctypes.byref(z), _device.ptr(None), _device.ptr(out), cap,
                     _device.ptr(counts), _device.ptr(status), _device.ptr(self._ws),
                     ctypes.c_size_t(self._ws.numel()), _device.stream())
            st = status.cpu().numpy()
            if not (st & PP_ST_ANN_OVERFLOW).any():
                break
            if cap >= k * cells:
                raise PPError('CifDet: detection capacity overflow')
            cap = min(k * cells, 2 * cap)
        counts = counts.cpu().numpy().astype(np.int64)
        offsets = np.concatenate([[0], np.cumsum(counts)])
        host = out.cpu().numpy()
        recs = np.concatenate([host[i, :counts[i]].reshape(-1) for i in range(b)])
        return np.frombuffer(recs.tobytes(), dtype=DET_DTYPE), offsets

    def annotations_from_records(self, recs, offsets):
        return [[AnnotationDet.from_record(r, self.categories)
                 for r in recs[offsets[i]:offsets[i + 1]]] for i in range(len(offsets) - 1)]

    def decode_batch(self, det_batch, *, group=None, dst=0, local=False):
        """(B, K, 7, H, W) -> one list of AnnotationDet per image.

        With a torch.distributed process `group`, the batch is image-sharded as in
        CifCaf.decode_batch: each rank decodes its contiguous `distributed.shard` of the
        images (`local=True`: det_batch is already this rank's share, possibly None), and
        rank `dst` returns the detections of all images in rank order, gathered as pp_det
        records whose digests it checks (distributed.gather_records; GatherMismatch on a
        mismatch).  Other ranks return None.  Replaces the reference's
        worker_pool.starmap over the batch (generator.py:96-97)."""
        if group is None:
            return self.annotations_from_records(*self.decode_records(det_batch))
        import torch.distributed as dist  # pylint: disable=import-outside-toplevel
        from ...distributed import GatherMismatch, gather_records, shard
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        several = isinstance(det_batch, (list, tuple))
        n = 0 if det_batch is None else len(det_batch[0] if several else det_batch)
        a, b = (0, n) if local else shard(n, rank, world)
        if b > a:
            recs, offsets = self.decode_records([t[a:b] for t in det_batch] if several
                                                else det_batch[a:b])
        else:
            recs, offsets = np.zeros(0, DET_DTYPE), np.zeros(1, np.int64)
        nccl = dist.get_backend(group) == 'nccl'
        device = (torch.device('cuda', torch.cuda.current_device()) if nccl
                  else torch.device('cpu'))
        self.last_gather = {}
        recs, offsets = gather_records(recs, offsets, dist, device, dst=dst,
                                       report=self.last_gather, group=group)
        if recs is None:
            return None
        if self.last_gather['ranks_verified'] != world:
            raise GatherMismatch('gathered detections of {} of {} ranks do not match their '
                                 'digests'.format(world - self.last_gather['ranks_verified'],
                                                  world))
        return self.annotations_from_records(recs, offsets)

    def decode_heads(self, heads, *, group=None, dst=0, local=False):
        """Generator.batch: the model's head list (each (B, ...)); reads the CifDet head
        (`group` / `dst` / `local`: image-sharded, as decode_batch)."""
        kw = {} if group is None else {'group': group, 'dst': dst, 'local': local}
        if heads is None:  # this rank's shard of a sharded batch is empty
            return self.decode_batch(None, **kw)
        heads = self.head_fields(heads)
        return self.decode_batch(heads[0] if self.single_head() else heads, **kw)

    def __call__(self, fields):
        """generator/cifdet.py:27-52 for one image's field list."""
        heads = [_device.to_device(t)[None] for t in self.head_fields(fields)]
        return self.decode_batch(heads[0] if self.single_head() else heads)[0]
