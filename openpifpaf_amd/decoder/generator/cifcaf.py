"""CifCaf greedy pose decoder (decoder/generator/cifcaf.py:24-351) on gfx950.

Same constructor, class attributes and call signature as the reference.  One call runs the
whole per-image pipeline on the device (engine.DecodeEngine -> pp_decode_stages):
CifHr -> CifSeeds -> CafScored (both thresholds) -> seed loop with occupancy and the
frontier grow -> complete_annotations / flood fill -> nms.Keypoints, and returns
Annotation objects.  `decode_batch` decodes a whole (B, ...) batch of device fields in
one launch sequence, which is how `batch()` (generator.py:84-101) is served.
"""
from collections import defaultdict
import logging
import time

import numpy as np

from ... import _device
from ..._abi import PACK_ALL, check_seed_mask, make_config, skeleton_array
from ...annotation import Annotation
from ...distributed import decode_sharded, shard
from ...engine import HeadSet, InitialAnnotations, engine
from ...functional import grow_connection_blend
from .. import nms as nms_module
from ..caf_scored import CafScored
from ..cif_hr import CifHr
from ..cif_seeds import CifSeeds
from ..field_config import FieldConfig
from .generator import Generator

LOG = logging.getLogger(__name__)


class CifCaf(Generator):
    """Generate CifCaf poses from fields.

    :param: nms: set to None to switch off non-maximum suppression.
    """
    connection_method = 'blend'
    supports_sharding = True
    force_complete = False
    greedy = False
    keypoint_threshold = 0.0

    def __init__(self, field_config: FieldConfig, *, keypoints, skeleton, out_skeleton=None,
                 confidence_scales=None, worker_pool=None, nms=True):
        super().__init__(worker_pool)
        if nms is True:
            nms = nms_module.Keypoints()
        # nms.Keypoints (its own annotations()) runs inside the device decode; any other
        # object with an annotations(list) method (cifcaf.py:117-118) runs on the host over
        # each image's decoded list, which the device then leaves unsuppressed
        if nms is not None and not callable(getattr(nms, 'annotations', None)):
            raise TypeError('nms must provide annotations(annotations)')
        # confidence_scales (cifcaf.py:39,52): per-CAF weights on the frontier priorities
        # of _grow (cifcaf.py:259-260, 282-284), applied on the device (pp_config).  The
        # reference indexes it per CAF while growing; a list shorter than the skeleton
        # raises its IndexError here, before any decode -- deliberately stricter than the
        # reference (see config(), which checks again for lists replaced after __init__).
        if confidence_scales is not None and len(confidence_scales) < len(skeleton):
            raise IndexError('list index out of range (confidence_scales has {} entries for '
                             '{} CAF fields)'.format(len(confidence_scales), len(skeleton)))
        self.field_config = field_config
        self.keypoints = keypoints
        self.skeleton = skeleton
        self.skeleton_m1 = np.asarray(skeleton) - 1
        self.out_skeleton = out_skeleton or skeleton
        self.confidence_scales = confidence_scales
        self.nms = nms
        self.timers = defaultdict(float)
        # cifcaf.py:57-65 (kept for API parity; the kernel builds the same tables)
        self.by_target = defaultdict(dict)
        for caf_i, (j1, j2) in enumerate(self.skeleton_m1):
            self.by_target[j2][j1] = (caf_i, True)
            self.by_target[j1][j2] = (caf_i, False)
        self.by_source = defaultdict(dict)
        for caf_i, (j1, j2) in enumerate(self.skeleton_m1):
            self.by_source[j1][j2] = (caf_i, True)
            self.by_source[j2][j1] = (caf_i, False)

    # -- configuration -------------------------------------------------------------------
    def config(self):
        """pp_config from the class attributes decoder.configure() writes (factory.py:64-98)."""
        stride = int(self.field_config.cif_strides[0])  # multi-scale heads carry their own
        if CifSeeds.threshold is None:
            raise TypeError('CifSeeds.threshold is not configured (decoder.configure sets it)')
        nms = self.nms if self._device_nms() else None
        check_seed_mask(self.field_config.seed_mask, len(self.keypoints))
        # Deliberately stricter than the reference: it indexes confidence_scales per CAF
        # inside _grow and raises IndexError only when a grow reaches an edge past the end
        # of the list (cifcaf.py:259-260, 282-284), so a decode that never grows such an
        # edge succeeds there.  The device table needs every edge's weight up front, so a
        # short list raises the same IndexError here, at the start of every decode.
        cs = self.confidence_scales
        if cs is not None and len(cs) < len(self.skeleton):
            raise IndexError('list index out of range (confidence_scales has {} entries for '
                             '{} CAF fields)'.format(len(cs), len(self.skeleton)))
        return make_config(
            cif_threshold=CifHr.v_threshold,
            seed_threshold=CifSeeds.threshold,
            seed_score_scale=CifSeeds.score_scale,
            caf_threshold=CafScored.default_score_th,
            complete_caf_threshold=0.0001,
            keypoint_threshold=self.keypoint_threshold,
            nms_keypoint_threshold=nms.keypoint_threshold if nms else 0.0,
            nms_instance_threshold=nms.instance_threshold if nms else 0.0,
            nms_suppression=nms.suppression if nms else 0.0,
            stride=stride,
            cif_neighbors=CifHr.neighbors,
            force_complete=self.force_complete,
            greedy=self.greedy,
            connection_method=self.connection_method,
            apply_nms=nms is not None,
            seed_mask=self.field_config.seed_mask,
            confidence_scales=self.confidence_scales,
        )

    def _device_nms(self):
        """nms.Keypoints (not a subclass overriding annotations()) runs on the device."""
        return (isinstance(self.nms, nms_module.Keypoints) and
                type(self.nms).annotations is nms_module.Keypoints.annotations)

    def _host_nms(self, anns):
        """cifcaf.py:117-118 for an NMS object other than nms.Keypoints."""
        if self.nms is None or self._device_nms():
            return anns
        return self.nms.annotations(anns)

    # -- decoding ------------------------------------------------------------------------
    def __call__(self, fields, initial_annotations=None):
        """One image: fields = the head outputs [cif (K, 5, H, W), caf (C, 9, H, W), ...]
        (numpy or device), read through the FieldConfig (single- or multi-scale)."""
        start = time.perf_counter()
        if initial_annotations:
            anns = self._call_initial(fields, list(initial_annotations))
            LOG.debug('%d annotations, %.3fs', len(anns), time.perf_counter() - start)
            return anns
        if self.field_config.is_single_scale():
            cif_i, caf_i, _ = self.field_config.single_scale()
            anns = self.decode_batch(_device.to_device(fields[cif_i])[None],
                                     _device.to_device(fields[caf_i])[None])[0]
        else:
            used = set(self.field_config.cif_indices) | set(self.field_config.caf_indices)
            batched = [_device.to_device(f)[None] if i in used else None
                       for i, f in enumerate(fields)]
            anns = self.decode_fields_batch(batched)[0]
        LOG.debug('%d annotations, %.3fs', len(anns), time.perf_counter() - start)
        return anns

    def _call_initial(self, fields, initial):
        """cifcaf.py:67-71, 95-98: the initial annotations are grown first, marked occupied
        and kept in the annotation list (pp_decode_initial).  As in the reference, the
        returned list holds the same initial Annotation objects, mutated (grown, completed,
        NMS-suppressed); one that NMS drops is mutated too (the reference edits the objects
        in place before filtering, nms.py:20-53), from the decode's working records
        (pp_decode_multi_work_offset)."""
        init = InitialAnnotations([np.stack([a.to_record() for a in initial])],
                                  _device.require())
        skel = skeleton_array(self.skeleton)
        if self.field_config.is_single_scale():
            cif_i, caf_i, _ = self.field_config.single_scale()
            recs, offsets, b = engine().decode(_device.to_device(fields[cif_i])[None],
                                               _device.to_device(fields[caf_i])[None], skel,
                                               self.config(), initial=init)
        else:
            used = set(self.field_config.cif_indices) | set(self.field_config.caf_indices)
            heads = HeadSet([_device.to_device(f)[None] if i in used else None
                             for i, f in enumerate(fields)], self.field_config)
            recs, offsets, b = engine().decode(None, None, skel, self.config(), heads=heads,
                                               initial=init)
        n = int(offsets[1])
        index = b.out_index[:n].cpu().numpy()
        out = []
        for rec, idx in zip(recs[:n], index):
            if 0 <= idx < len(initial):
                out.append(initial[idx].update_from_record(rec))
            else:
                out.append(Annotation.from_record(rec, self.keypoints, self.out_skeleton))
        dropped = sorted(set(range(len(initial))) - set(int(i) for i in index))
        if dropped:
            for i, rec in zip(dropped, b.work_records(0, dropped)):
                initial[i].update_from_record(rec)
        return self._host_nms(out)

    def decode_records(self, cif_batch, caf_batch, keep_cifhr=False, compact=None):
        """Device decode of a batch -> (packed records, per-image offsets, buffers): full
        pp_ann records, or compact ones (pp_pack_compact) with `compact` flags."""
        cif = _device.to_device(cif_batch)
        caf = _device.to_device(caf_batch)
        return engine().decode(cif, caf, skeleton_array(self.skeleton), self.config(),
                               keep_cifhr=keep_cifhr, compact=compact)

    def decode_fields_records(self, fields_batch, keep_cifhr=False, compact=None):
        """Multi-scale device decode (pp_decode_multi): fields_batch is the head output list
        with a batch dimension, indexed by the FieldConfig (factory.py:153-180)."""
        heads = HeadSet([None if f is None else _device.to_device(f) for f in fields_batch],
                        self.field_config)
        return engine().decode(None, None, skeleton_array(self.skeleton), self.config(),
                               keep_cifhr=keep_cifhr, heads=heads, compact=compact)

    def annotations_from_records(self, recs, offsets):
        """Full or compact records + per-image offsets -> one list of Annotation per image."""
        out = []
        for i in range(len(offsets) - 1):
            out.append(self._host_nms([Annotation.from_any(r, self.keypoints, self.out_skeleton)
                                       for r in recs[offsets[i]:offsets[i + 1]]]))
        return out

    def decode_heads(self, heads, *, group=None, dst=0, local=False):
        """Generator.batch: the model's head list (each (B, ...)) through the FieldConfig.
        `group` / `dst` / `local`: image-sharded over a process group (decode_batch)."""
        kw = {} if group is None else {'group': group, 'dst': dst, 'local': local}
        if heads is None:  # this rank's shard of a sharded batch is empty
            return self.decode_batch(None, None, **kw)
        if self.field_config.is_single_scale():
            cif_i, caf_i, _ = self.field_config.single_scale()
            return self.decode_batch(heads[cif_i], heads[caf_i], **kw)
        used = set(self.field_config.cif_indices) | set(self.field_config.caf_indices)
        return self.decode_fields_batch([h if i in used else None for i, h in enumerate(heads)],
                                        **kw)

    def decode_batch(self, cif_batch, caf_batch, *, group=None, dst=0, local=False):
        """(B, K, 5, H, W) + (B, C, 9, H, W) -> one list of Annotation per image.

        With a torch.distributed process `group` (e.g. `dist.group.WORLD`: one rank per
        GPU, nccl = RCCL over xGMI, or gloo; the nccl leg has not yet run on hardware with
        more than one GPU), the batch is image-sharded: each rank decodes
        its contiguous `distributed.shard` of the B images (every rank passes the whole
        batch; `local=True`: the arguments are already this rank's images, possibly None
        for none), and rank `dst` returns the annotation lists of all images in rank order,
        gathered as compact records whose digests it checks (distributed.decode_sharded;
        GatherMismatch on a mismatch).  Other ranks return None.  This replaces the
        reference's worker_pool.starmap over the batch (generator.py:96-97)."""
        if group is None:
            recs, offsets, _ = self.decode_records(cif_batch, caf_batch, compact=PACK_ALL)
            return self.annotations_from_records(recs, offsets)
        n = 0 if cif_batch is None else len(cif_batch)
        return self._decode_sharded(
            n, lambda a, b: (_device.to_device(cif_batch[a:b]).contiguous(),
                             _device.to_device(caf_batch[a:b]).contiguous(), None),
            group, dst, local)

    def decode_fields_batch(self, fields_batch, *, group=None, dst=0, local=False):
        """Batched head outputs of any FieldConfig -> one list of Annotation per image
        (`group` / `dst` / `local`: image-sharded, as decode_batch)."""
        if group is None:
            recs, offsets, _ = self.decode_fields_records(fields_batch, compact=PACK_ALL)
            return self.annotations_from_records(recs, offsets)
        n = 0 if fields_batch is None else len(
            fields_batch[self.field_config.cif_indices[0]])

        def take(a, b):
            fields = [None if f is None else _device.to_device(f[a:b]).contiguous()
                      for f in fields_batch]
            return None, None, HeadSet(fields, self.field_config)
        return self._decode_sharded(n, take, group, dst, local)

    def _decode_sharded(self, n, take, group, dst, local):
        import torch.distributed as dist  # pylint: disable=import-outside-toplevel
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        a, b = (0, n) if local else shard(n, rank, world)
        cfg, skel = self.config(), skeleton_array(self.skeleton)

        def decode_local(device_out):
            cif, caf, heads = take(a, b)
            _, pending = engine().decode_async(cif, caf, skel, cfg, heads=heads,
                                               compact=PACK_ALL, device_out=device_out)
            return pending
        self.last_gather = {}
        recs, offsets = decode_sharded(decode_local, b - a, dist, group=group, dst=dst,
                                       report=self.last_gather)
        if recs is None:
            return None
        return self.annotations_from_records(recs, offsets)

    # -- reference building blocks, on the device ------------------------------------------
    def _grow_connection(self, xy, xy_scale, caf_field):
        assert len(xy) == 2
        assert caf_field.shape[0] == 9
        return grow_connection_blend(caf_field, xy[0], xy[1], xy_scale,
                                     connection_method=self.connection_method)
