"""Batched device decode: fields resident in HBM -> packed annotation records.

The engine owns the per-shape workspace (zeroed once at allocation, see the workspace
contract in include/pifpaf_amd.h) and drives pp_decode_stages on torch's current stream.
Records come back as a NumPy structured array (openpifpaf_amd._abi.ANN_DTYPE) packed over
the whole batch plus per-image offsets; decoder/generator/cifcaf.py turns them into
Annotation objects.
"""
import ctypes
import logging

import numpy as np
import torch

from . import _device
from ._abi import (ANN_DTYPE, PACK_ALL, PP_ST_ANN_OVERFLOW, PP_ST_DEC_OVERFLOW,
                   PP_ST_NMS_OVERFLOW, packed_dtype, scale_list, skeleton_array)
from ._lib import PPError, call, load

LOG = logging.getLogger(__name__)

STAGE_CIFHR, STAGE_SEEDS, STAGE_CAF, STAGE_GROW = 1, 2, 4, 8
STAGE_ALL = 15
# PP_STAGE_COMPLETE_SETS_EARLY: the force-complete column sets with the CAF stage
STAGE_COMPLETE_EARLY = 16
# PP_STAGE_SEED_LOOP_ONLY / PP_STAGE_AFTER_SEED_LOOP: stage 8 in two calls (same slot)
STAGE_SEED_LOOP_ONLY, STAGE_AFTER_SEED_LOOP = 32, 64
# PP_STAGE_COMPLETE_ONLY / PP_STAGE_NMS_ONLY: the after-seed-loop part in two calls
STAGE_COMPLETE_ONLY, STAGE_NMS_ONLY = 128, 256
# PP_STAGE_NMS_WIDE: NMS in 8-wave workgroups (dense batches; the 4-wave default fits beside
# a seed loop on a CU)
STAGE_NMS_WIDE = 512
# PP_STAGE_NMS_BITMAP: NMS planes as LDS bitmaps, one wave per (image, plane) (opt-in)
STAGE_NMS_BITMAP = 1024


def default_ann_capacity(h, w):
    """Annotations per image the first attempt reserves (doubles on overflow)."""
    return int(min(8192, max(128, (h * w) // 8)))


class DecodeBuffers:
    """Workspace + outputs for one (batch shape, config) combination.  `heads` (a HeadSet)
    selects the multi-scale entry points."""

    def __init__(self, key, n, k, c, h, w, cfg, cap, device, heads=None):
        lib = load()
        self.key = key
        self.n, self.k, self.c, self.cap = n, k, c, cap
        if heads is None:
            size = lib.pp_decode_workspace_size(n, k, c, h, w, ctypes.byref(cfg), cap)
            zero_off = lib.pp_decode_workspace_zero_offset(n, k, c, h, w, ctypes.byref(cfg), cap)
            self.work_off = lib.pp_decode_work_offset(n, k, c, h, w, ctypes.byref(cfg), cap)
            stride = cfg.stride
        else:
            args = (heads.arr, len(heads.arr), heads.pairs, n, k, c, ctypes.byref(cfg), cap)
            size = lib.pp_decode_multi_workspace_size(*args)
            zero_off = lib.pp_decode_multi_workspace_zero_offset(*args)
            self.work_off = lib.pp_decode_multi_work_offset(*args)
            stride = heads.stride0
        if size == 0:
            raise PPError('pp_decode_workspace_size rejected the shape: ' +
                          lib.pp_last_error().decode())
        self.ws = torch.empty(size, dtype=torch.uint8, device=device)
        self.ws[zero_off:].zero_()
        # two output slots (records, counts, status): a decode with the grow stage writes the
        # slot after the previous one, so records of decode i can still be packed / fetched
        # while decode i + 1 runs (DecodeEngine.fetch_async)
        self._slots = [(torch.empty(n * cap * ANN_DTYPE.itemsize, dtype=torch.uint8, device=device),
                        torch.zeros(n, dtype=torch.int32, device=device),
                        torch.zeros(n, dtype=torch.int32, device=device)) for _ in range(2)]
        self._cur = 0
        self._free = [None, None]  # per slot: event after which its records were packed
        self.hh = (h - 1) * stride + 1
        self.ww = (w - 1) * stride + 1
        self.pitch = int(lib.pp_cifhr_pitch(self.ww))
        self.cifhr = None
        self.out_index = None  # pp_decode_initial's (n, cap) positions before NMS

    def work_records(self, img, positions):
        """pp_decode_work_offset: image img's annotations at `positions` of its list before
        NMS, in the state NMS left them (ANN_DTYPE, host), after a decode with the grow
        stage and before the next decode into this workspace."""
        rows = self.ws[self.work_off:self.work_off + self.n * self.cap * ANN_DTYPE.itemsize]
        rows = rows.view(self.n * self.cap, ANN_DTYPE.itemsize)
        idx = torch.as_tensor([img * self.cap + int(p) for p in positions], dtype=torch.int64,
                              device=rows.device)
        return rows.index_select(0, idx).cpu().numpy().reshape(-1).view(ANN_DTYPE)

    anns = property(lambda self: self._slots[self._cur][0])
    counts = property(lambda self: self._slots[self._cur][1])
    status = property(lambda self: self._slots[self._cur][2])

    def next_slot(self):
        """Switch to the other output slot; the current stream waits until that slot's
        previous records have been packed (fetch_async packs on a side stream)."""
        self._cur ^= 1
        if self._free[self._cur] is not None:
            torch.cuda.current_stream().wait_event(self._free[self._cur])
            self._free[self._cur] = None

    def cifhr_buffer(self):
        if self.cifhr is None:
            self.cifhr = torch.empty((self.n, self.k, self.hh, self.pitch), dtype=torch.float32,
                                     device=self.ws.device)
        return self.cifhr


class InitialAnnotations:
    """Per-image initial annotations (CifCaf.__call__'s initial_annotations,
    cifcaf.py:67-71) as device pp_ann records for pp_decode_initial: `records` (n, cap)
    ANN_DTYPE rows, `counts` (n) int32.  `per_image`: one list of ANN_DTYPE record arrays
    per image."""

    def __init__(self, per_image, device):
        self.n = len(per_image)
        self.cap = max(1, max((len(r) for r in per_image), default=0))
        host = np.zeros((self.n, self.cap), ANN_DTYPE)
        for i, r in enumerate(per_image):
            host[i, :len(r)] = r
        self.records = torch.from_numpy(host.view(np.uint8).reshape(-1)).to(device)
        self.counts = torch.tensor([len(r) for r in per_image], dtype=torch.int32,
                                   device=device)


class HeadSet:
    """The CIF and CAF heads of a FieldConfig for one batch of device fields
    (field_config.py:7-13): `fields` is the head-network output list with a leading batch
    dimension on every tensor.  Builds the pp_scale list of pp_decode_multi."""

    def __init__(self, fields, fc):
        self.cifs = [fields[i] for i in fc.cif_indices]
        self.cafs = [fields[i] for i in fc.caf_indices]
        for t in self.cifs + self.cafs:
            if not _device.is_device(t) or t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError('multi-scale fields must be contiguous float32 device tensors')
            if t.dim() != 5:
                raise ValueError('expected batched fields (B, n_fields, channels, H, W)')
        if any(t.shape[2] != 5 for t in self.cifs) or any(t.shape[2] != 9 for t in self.cafs):
            raise ValueError('expected CIF heads (B, K, 5, H, W) and CAF heads (B, C, 9, H, W)')
        self.n = self.cifs[0].shape[0]
        self.k = self.cifs[0].shape[1]
        self.c = self.cafs[0].shape[1]
        if any(t.shape[0] != self.n for t in self.cifs + self.cafs):
            raise ValueError('heads have different batch sizes')
        if any(t.shape[1] != self.k for t in self.cifs) or any(t.shape[1] != self.c for t in self.cafs):
            raise ValueError('heads have different field counts')
        self.h, self.w = self.cifs[0].shape[3], self.cifs[0].shape[4]
        self.stride0 = int(fc.cif_strides[0])
        self.pairs = int(len(fc.cif_indices) == 10)  # cif_hr.py:63
        self.arr = scale_list([(t.data_ptr(), t.shape[3], t.shape[4]) for t in self.cifs],
                              [(t.data_ptr(), t.shape[3], t.shape[4]) for t in self.cafs],
                              fc.cif_strides, fc.caf_strides, fc.cif_min_scales,
                              fc.caf_min_distances, fc.caf_max_distances)
        self.shape_key = (self.pairs,) + tuple(
            (s.H, s.W, s.stride, s.role) for s in self.arr)


def _buffer_key(n, k, c, shape, cap, cfg):
    return (n, k, c, shape, cap, cfg.force_complete, cfg.stride, cfg.occupancy_reduction)


class DecodeEngine:
    def __init__(self):
        self._bufs = None
        # annotations per image of the last checked decode: dense batches (>= 32) get the
        # 8-wave NMS (PP_STAGE_NMS_WIDE) in the next one, as DecodePipeline does
        self.density = 0.0

    def buffers(self, n, k, c, h, w, cfg, cap, heads=None):
        shape = (h, w) if heads is None else heads.shape_key
        key = _buffer_key(n, k, c, shape, cap, cfg)
        if self._bufs is None or self._bufs.key != key:
            self._bufs = None  # free the previous workspace first
            self._bufs = DecodeBuffers(key, n, k, c, h, w, cfg, cap, _device.require(), heads)
        return self._bufs

    def launch(self, cif, caf, skeleton, cfg, cap=None, keep_cifhr=False, stages=STAGE_ALL,
               initial=None):
        """Enqueue the decode on the current stream; returns the DecodeBuffers.  `initial`
        (InitialAnnotations) selects pp_decode_initial."""
        if cif.dim() != 5 or caf.dim() != 5 or cif.shape[2] != 5 or caf.shape[2] != 9:
            raise ValueError('expected cif (B, K, 5, H, W) and caf (B, C, 9, H, W)')
        n, k, _, h, w = cif.shape
        c = caf.shape[1]
        if caf.shape[0] != n or caf.shape[3:] != cif.shape[3:]:
            raise ValueError('cif and caf batch / spatial shapes differ')
        skel = skeleton_array(skeleton)
        if len(skel) != c:
            raise ValueError('skeleton has {} edges but caf has {} fields'.format(len(skel), c))
        cap = cap or default_ann_capacity(h, w)
        b = self.buffers(n, k, c, h, w, cfg, cap)
        if stages & STAGE_GROW and not stages & STAGE_AFTER_SEED_LOOP:
            b.next_slot()
        hr = b.cifhr_buffer() if keep_cifhr else None
        if initial is not None:
            arr = scale_list([(cif.data_ptr(), h, w)], [(caf.data_ptr(), h, w)], [cfg.stride],
                             [cfg.stride])
            self._launch_initial(b, arr, 0, n, k, c, skel, cfg, hr, cap, initial, stages)
            return b
        call('pp_decode_stages', _device.ptr(cif), _device.ptr(caf), n, k, c, h, w,
             skel.ctypes.data_as(ctypes.c_void_p), ctypes.byref(cfg), _device.ptr(hr),
             _device.ptr(b.anns), cap, _device.ptr(b.counts), _device.ptr(b.status),
             _device.ptr(b.ws), ctypes.c_size_t(b.ws.numel()), ctypes.c_uint32(stages),
             _device.stream())
        return b

    @staticmethod
    def _launch_initial(b, arr, pairs, n, k, c, skel, cfg, hr, cap, initial, stages):
        if initial.n != n:
            raise ValueError('initial annotations for {} images, batch has {}'.format(
                initial.n, n))
        # out_index is exactly (n * cap) long, image i's rows at [i * cap, (i + 1) * cap) as
        # the kernel writes them (the store behind it only grows)
        store = getattr(b, '_out_index_store', None)
        if store is None or store.numel() < n * cap:
            store = b._out_index_store = torch.empty(n * cap, dtype=torch.int32,
                                                     device=b.ws.device)
        b.out_index = store[:n * cap]
        b.out_index_cap = cap
        call('pp_decode_initial', arr, len(arr), pairs, n, k, c,
             skel.ctypes.data_as(ctypes.c_void_p), ctypes.byref(cfg), _device.ptr(hr),
             _device.ptr(b.anns), cap, _device.ptr(b.counts), _device.ptr(b.status),
             _device.ptr(initial.records), _device.ptr(initial.counts), initial.cap,
             _device.ptr(b.out_index), _device.ptr(b.ws), ctypes.c_size_t(b.ws.numel()),
             ctypes.c_uint32(stages), _device.stream())

    def launch_multi(self, heads, skeleton, cfg, cap=None, keep_cifhr=False, stages=STAGE_ALL,
                     initial=None):
        """pp_decode_multi over a HeadSet (pp_decode_initial with `initial`); returns the
        DecodeBuffers."""
        skel = skeleton_array(skeleton)
        if len(skel) != heads.c:
            raise ValueError('skeleton has {} edges but caf has {} fields'.format(len(skel),
                                                                                  heads.c))
        cap = cap or default_ann_capacity(heads.h, heads.w)
        b = self.buffers(heads.n, heads.k, heads.c, heads.h, heads.w, cfg, cap, heads)
        if stages & STAGE_GROW and not stages & STAGE_AFTER_SEED_LOOP:
            b.next_slot()
        hr = b.cifhr_buffer() if keep_cifhr else None
        if initial is not None:
            self._launch_initial(b, heads.arr, heads.pairs, heads.n, heads.k, heads.c, skel, cfg,
                                 hr, cap, initial, stages)
            return b
        call('pp_decode_multi', heads.arr, len(heads.arr), heads.pairs, heads.n, heads.k,
             heads.c, skel.ctypes.data_as(ctypes.c_void_p), ctypes.byref(cfg), _device.ptr(hr),
             _device.ptr(b.anns), cap, _device.ptr(b.counts), _device.ptr(b.status),
             _device.ptr(b.ws), ctypes.c_size_t(b.ws.numel()), ctypes.c_uint32(stages),
             _device.stream())
        return b

    def launch_checked(self, cif, caf, skeleton, cfg, cap=None, keep_cifhr=False, heads=None,
                       initial=None):
        """launch / launch_multi with overflow retry (the annotation capacity doubles until
        no image overflows); returns the DecodeBuffers of a decode whose records are
        complete.  Raises PPError on the overflows a retry cannot fix."""
        h, w = (cif.shape[3], cif.shape[4]) if heads is None else (heads.h, heads.w)
        cap = cap or default_ann_capacity(h, w)
        stages = STAGE_ALL | (STAGE_NMS_WIDE if self.density >= _B_FIRST_DENSITY else 0)
        while True:
            if heads is None:
                b = self.launch(cif, caf, skeleton, cfg, cap=cap, keep_cifhr=keep_cifhr,
                                stages=stages, initial=initial)
            else:
                b = self.launch_multi(heads, skeleton, cfg, cap=cap, keep_cifhr=keep_cifhr,
                                      stages=stages, initial=initial)
            status = b.status.cpu().numpy()
            if len(status):
                self.density = float(b.counts[:len(status)].float().mean())
            if not (status & PP_ST_ANN_OVERFLOW).any():
                break
            cap *= 2
            LOG.info('annotation capacity overflow, retrying with %d per image', cap)
        if (status & PP_ST_NMS_OVERFLOW).any():
            raise PPError('NMS occupancy grid exceeds the workspace (keypoints far outside '
                          'the field); status={}'.format(status.tolist()))
        if (status & PP_ST_DEC_OVERFLOW).any():
            raise PPError('decoding/frontier order exceeded the record capacity')
        return b

    def decode(self, cif, caf, skeleton, cfg, cap=None, keep_cifhr=False, heads=None,
               compact=None, initial=None):
        """Full decode with overflow retry.  Returns (records, offsets, buffers).  With a
        HeadSet `heads`, cif / caf are ignored and the multi-scale decode runs.  `compact`
        flags (e.g. _abi.PACK_ALL) fetch compact records (pp_pack_compact) instead of full
        pp_ann records.  `initial` (InitialAnnotations): grown before the seed loop; the
        buffers then hold out_index (see pp_decode_initial)."""
        b = self.launch_checked(cif, caf, skeleton, cfg, cap=cap, keep_cifhr=keep_cifhr,
                                heads=heads, initial=initial)
        k = cif.shape[1] if heads is None else heads.k
        recs, offsets = self.fetch(b, None if compact is None else
                                   (k, len(skeleton_array(skeleton)), compact))
        return recs, offsets, b

    def decode_async(self, cif, caf, skeleton, cfg, heads=None, compact=PACK_ALL,
                     device_out=False):
        """decode() up to the record pack: (buffers, PendingRecords of compact records, or
        full ones with compact=None).  `device_out` packs into device memory (what a
        multi-GPU rank sends, distributed.decode_sharded)."""
        b = self.launch_checked(cif, caf, skeleton, cfg, heads=heads)
        k = cif.shape[1] if heads is None else heads.k
        spec = None if compact is None else (k, len(skeleton_array(skeleton)), compact)
        return b, self.fetch_async(b, spec, device_out=device_out)

    @staticmethod
    def fetch(b, compact=None):
        """Packed records of all images and per-image offsets of the last decode into `b`
        (fetch_async(b).result())."""
        return DecodeEngine.fetch_async(b, compact).result()

    @staticmethod
    def fetch_async(b, compact=None, device_out=False, capacity=0, stream=None):
        """Enqueue the record fetch of the last decode into `b` on a side stream and return a
        PendingRecords; its result() waits for it.

        The records are packed image after image straight into a pinned host block
        (zero-copy through its mapped device address) together with the per-image counts,
        so one synchronisation hands over everything.  `compact` = (K, C, flags) selects
        pp_pack_compact's compact records (include/pifpaf_amd.h); None the full pp_ann
        records (pp_pack_records).  `device_out` packs the records into a device buffer
        instead (the multi-GPU gather sends them from there); the counts still land in
        pinned host memory.  The block is sized from the largest batch seen so far
        (`capacity` = records to reserve at least); result() re-packs a batch that outgrew
        it, and fetches full records when a compact record is flagged PP_PACK_REFETCH.  The
        slot stays valid until the second decode after this one, so a caller may launch the
        next decode before calling result().  `stream`: pack there instead of on the
        engine's pack stream."""
        est = max(getattr(b, 'pack_cap', 0), 16 * b.n, capacity)
        decoded = torch.cuda.Event()
        decoded.record()
        p = DecodeEngine._pack(b, b.anns, b.counts, b.status, compact, device_out, est, decoded,
                               stream)
        b._free[b._cur] = p.done_event
        return p

    @staticmethod
    def _pack(b, anns, counts, status, compact, device_out, est, after, stream=None):
        n = b.n
        dtype = ANN_DTYPE if compact is None else packed_dtype(*compact)
        width = dtype.itemsize
        # head: counts (n int32), the slot's status (n int32), per-image refetch flags
        # (n int32, pp_pack_compact's out_flags), then the records
        head = -(-12 * n // 256) * 256
        host = torch.empty(head + (0 if device_out else est * width), dtype=torch.uint8,
                           pin_memory=True)
        if compact is None:
            host[8 * n:12 * n].zero_()
        dev = (torch.empty(est * width, dtype=torch.uint8, device=anns.device)
               if device_out else None)
        out_ptr = dev.data_ptr() if device_out else host.data_ptr() + head
        # the pack runs on a side stream after the decode, so its PCIe writes overlap the
        # next decode; the slot is not rewritten before it is done (DecodeBuffers.next_slot)
        side = DecodeEngine._pack_stream(anns.device) if stream is None else stream
        side.wait_event(after)
        with torch.cuda.stream(side):
            if compact is None:
                call('pp_pack_records', _device.ptr(anns), _device.ptr(counts), n, b.cap,
                     ctypes.c_void_p(out_ptr), est, ctypes.c_void_p(host.data_ptr()),
                     _device.stream())
            else:
                k, c, flags = compact
                call('pp_pack_compact', _device.ptr(anns), _device.ptr(counts), n, b.cap,
                     k, c, ctypes.c_uint32(flags), ctypes.c_void_p(out_ptr), est,
                     ctypes.c_void_p(host.data_ptr()),
                     ctypes.c_void_p(host.data_ptr() + 8 * n), _device.stream())
            host[4 * n:8 * n].copy_(status.view(torch.uint8), non_blocking=True)
            done = torch.cuda.Event()
            done.record()
            if dev is not None:
                dev.record_stream(side)
        return PendingRecords(b, (anns, counts, status), host, head, est, done, dtype, dev,
                              compact, device_out)

    _pack_streams = {}

    @staticmethod
    def _pack_stream(device):
        if device not in DecodeEngine._pack_streams:
            DecodeEngine._pack_streams[device] = torch.cuda.Stream(device=device)
        return DecodeEngine._pack_streams[device]

    @staticmethod
    def fetch_gather(b, anns=None, counts=None):
        """Packed records of all images (one gather + one D2H copy) and per-image offsets;
        `anns` / `counts` select an output slot (default: the last decode's)."""
        anns = b.anns if anns is None else anns
        counts = (b.counts if counts is None else counts).cpu().numpy().astype(np.int64)
        offsets = np.concatenate([[0], np.cumsum(counts)])
        total = int(offsets[-1])
        if total == 0:
            return np.zeros(0, ANN_DTYPE), offsets
        # row of record r of image i is i * cap + r: one vectorised gather index
        idx = np.arange(total, dtype=np.int64) + np.repeat(
            np.arange(len(counts), dtype=np.int64) * b.cap - offsets[:-1], counts)
        rows = anns.view(b.n * b.cap, ANN_DTYPE.itemsize)
        sel = rows.index_select(0, torch.from_numpy(idx).to(rows.device))
        # pinned destination from torch's caching host allocator: full-rate D2H, and the
        # returned array owns the block (released to the cache when the caller drops it)
        host = torch.empty(sel.shape, dtype=torch.uint8, pin_memory=True)
        host.copy_(sel, non_blocking=True)
        torch.cuda.current_stream(rows.device).synchronize()
        return host.numpy().reshape(-1).view(ANN_DTYPE), offsets


class PendingRecords:
    """A record fetch enqueued by DecodeEngine.fetch_async."""

    def __init__(self, b, slot, host, head, est, done, dtype, dev=None, compact=None,
                 device_out=False):
        self._b, self._slot = b, slot
        self._host, self._head, self._est, self._done = host, head, est, done
        self.dtype, self.device_records = dtype, dev
        self._compact, self._device_out = compact, device_out
        self._waited = False
        self.on_counts = None  # callback(counts) once the pack is waited for

    def __del__(self):
        # the pinned block goes back to torch's host cache when this object dies; the raw
        # pack kernel must have finished writing it by then
        if not self._waited and self._done is not None:
            try:
                self._done.synchronize()
            except Exception:  # pylint: disable=broad-except
                pass

    def wait(self):
        """Wait for the pack; per-image counts (int64).  Raises PPError when the decode set
        an overflow bit (its records are truncated)."""
        n = self._b.n
        self._done.synchronize()
        self._waited = True
        status = self._host[4 * n:8 * n].numpy().view(np.int32)
        if self.on_counts is not None:
            self.on_counts(self._host[:4 * n].numpy().view(np.int32))
        bad = status & (PP_ST_ANN_OVERFLOW | PP_ST_DEC_OVERFLOW | PP_ST_NMS_OVERFLOW)
        if bad.any():
            raise PPError('decode status flags set (records truncated; decode() retries with '
                          'more capacity): {}'.format(status[bad != 0][:8].tolist()))
        return self._host[:4 * n].numpy().view(np.int32).astype(np.int64)

    @property
    def done_event(self):
        return self._done

    @property
    def refetch(self):
        """True when a compact record of this fetch is flagged PP_PACK_REFETCH (valid after
        wait(); from pp_pack_compact's per-image flags, so device-resident records need not
        be read)."""
        n = self._b.n
        return bool(self._host[8 * n:12 * n].numpy().view(np.int32).any())

    def host_records(self):
        """The pinned block's record area (a CPU uint8 tensor; valid after wait())."""
        return self._host[self._head:]

    def fits(self, total):
        return total <= self._est

    def result(self):
        """(records, offsets) once the fetch has completed (waits for it).  Records are
        self.dtype, or full ANN_DTYPE records after a refetch."""
        width = self.dtype.itemsize
        counts = self.wait()
        offsets = np.concatenate([[0], np.cumsum(counts)])
        total = int(offsets[-1])
        if total > self._est:  # outgrew the block: pack again into one that fits
            self._b.pack_cap = 2 * total
            after = torch.cuda.Event()
            after.record(DecodeEngine._pack_stream(self._slot[0].device))
            return DecodeEngine._pack(self._b, *self._slot, self._compact, self._device_out,
                                      2 * total, after).result()
        if self.device_records is not None:
            host = torch.empty(total * width, dtype=torch.uint8, pin_memory=True)
            host.copy_(self.device_records[:total * width])
            recs = host.numpy().view(self.dtype)
        else:
            recs = self._host[self._head:self._head + total * width].numpy().view(self.dtype)
        if self.refetch:
            return DecodeEngine.fetch_gather(self._b, self._slot[0], self._slot[1])
        return recs, offsets

    def full_device_records(self):
        """The decode's full pp_ann records as one device uint8 tensor (image after image;
        what a multi-GPU rank sends instead of compact records after a refetch)."""
        b, anns = self._b, self._slot[0]
        counts = self.wait()
        offsets = np.concatenate([[0], np.cumsum(counts)])
        idx = np.arange(int(offsets[-1]), dtype=np.int64) + np.repeat(
            np.arange(len(counts), dtype=np.int64) * b.cap - offsets[:-1], counts)
        rows = anns.view(b.n * b.cap, ANN_DTYPE.itemsize)
        return rows.index_select(0, torch.from_numpy(idx).to(rows.device)).reshape(-1)


# The pipeline's scheduling choices are module constants, not environment switches (tests
# set them to check that every order gives the same records).
# _B_FIRST: the force-complete set order of DecodePipeline, True / False / 'lazy' (gated
# after the seed loop, on the tail stream); None: auto below
_B_FIRST = None
# auto: lazy sets (only the (field, direction) pairs force-complete needs, on the tail
# stream) until a batch averaged this many annotations per image, then sets first.  Round 4,
# with the tail split: planted cfg3 0.687-0.691 (lazy) vs 0.801-0.811 ms (first) per step,
# uniform 14.7k vs 15.1-15.2k images/s, cfg5 planted equal, cfg5 uniform 1180 vs 1200
_B_FIRST_DENSITY = 32.0
# workspaces in flight: batch i + depth's front half waits for batch i's tail
_PIPE_DEPTH = 2
# the tail as two calls (force-complete, then NMS): a workspace's next front half waits only
# for the force-complete, its next seed loop for the NMS (False: one call, the front half
# waits for both)
_SPLIT_TAIL = True
# Sparse batches: batch i's seed loop and tail share the back stream of its workspace
# (i % 2), so a seed loop starts beside the previous batch's slowest images (cfg5 planted
# 30.5k -> 41.7k images/s, cfg3 planted equal); dense ones: one stream for the seed loops
# and one for the tails (cfg3 uniform 15.5k vs 14.6k images/s); True / False forces either.
# The same two streams serve both (current + the library's side stream + two: four
# hardware queues).
_BACK2 = None


class DecodePipeline:
    """Decodes a sequence of batches with consecutive batches overlapped on the device.

    A decode has a bandwidth-bound front half (CifHr, seeds, CafScored: stages 1 | 2 | 4,
    here with the force-complete column sets too, STAGE_COMPLETE_EARLY) and a
    latency-bound back half: the seed loop, then force-complete and NMS (stage 8 in two
    calls).  Batch i's front half runs on the caller's current stream, its seed loop on a
    back stream that waits for it, and its force-complete, NMS and record pack on a tail
    stream that waits for the seed loop.  So batch i + 1's front half runs beside batch i's
    seed loop, and batch i + 1's seed loop beside batch i's tail.  Two engines (two
    workspaces) alternate; a workspace's front half waits until the tail that last used it
    is done, and its output slots are released by their record packs as in DecodeEngine.
    The tail is two calls (STAGE_COMPLETE_ONLY, then STAGE_NMS_ONLY): the workspace's next
    front half waits only for the force-complete (the last reader of the stage 1-4 buffers),
    its next seed loop for the NMS.
    (The front half stays on the current stream and the pack on the tail stream so that
    the streams in use -- current, back, tail, the library's CafScored side stream -- each
    get a hardware queue of their own: HIP shares 4 per process between streams.)
    For sparse batches the same two streams are used per workspace instead: batch i's seed
    loop and its tail both go on stream i % 2, so batch i + 1's seed loop can start on the
    CUs that batch i's finished images left (the loop ends with its slowest image); every
    order between batches is an event either way.

    The force-complete sets are lazy for sparse batches (built after the seed loop on the
    tail stream, only for the (field, direction) pairs an annotation left unset), and go
    first for dense ones, on the side stream before the CifHr map (they read only the CAF
    fields), then set A after them, beside the CifHr map and the seeds on the current
    stream (_B_FIRST = True / False / 'lazy' forces first / after set A / lazy).  Every order
    gives the same records.

    submit() returns (buffers, PendingRecords of the batch: DecodeEngine.fetch_async).
    The current stream does not wait for the back half; the fields must stay unchanged
    until the batch's records are fetched."""

    def __init__(self, device=None, depth=None):
        self.device = _device.require() if device is None else device
        if depth is None:
            depth = _PIPE_DEPTH
        self.depth = max(2, depth)  # workspaces in flight (3 or 4 measured slower)
        self.engines = tuple(DecodeEngine() for _ in range(self.depth))
        # dense batches: seed loops on `back`, tails on `tail`; sparse ones: each workspace's
        # loop and tail on one of the two (_BACK2 above, per submit)
        # (a high HIP priority for the back, tail or a separate front stream measured no
        # better: planted 385-389k / 373-382k / 365-389k vs 390-391k images/s, round 4)
        self.back = torch.cuda.Stream(device=self.device)
        self.tail = torch.cuda.Stream(device=self.device)
        self._back_done = [None] * self.depth
        self._sets_done = [None] * self.depth  # end of force-complete (last reader of 1-4)
        self._i = 0
        self.density = 0.0  # annotations per image of the last batch whose records were read

    def submit(self, cif, caf, skeleton, cfg, cap=None, heads=None, compact=None,
               device_out=False, events=None):
        """Enqueue one batch (cif / caf, or a multi-scale HeadSet `heads`).  `events`
        (five torch.cuda.Events, optional) are recorded around the CifHr stage, the other
        front stages (front stream), at the seed loop's start (back stream) and at the end
        of NMS (tail stream); a sixth one, if given, at the seed loop's end (back stream)."""
        par = self._i % self.depth
        self._i += 1
        eng = self.engines[par]
        front = torch.cuda.current_stream(self.device)

        def launch(stages):
            if heads is None:
                return eng.launch(cif, caf, skeleton, cfg, cap=cap, stages=stages)
            return eng.launch_multi(heads, skeleton, cfg, cap=cap, stages=stages)

        if self._sets_done[par] is not None:  # the workspace's previous force-complete
            front.wait_event(self._sets_done[par])
        with torch.cuda.stream(front):
            if events:
                events[0].record()
            dense = self.density >= _B_FIRST_DENSITY
            b_first = _B_FIRST if _B_FIRST is not None else (True if dense else 'lazy')
            # dense batches: the 8-wave NMS (uniform cfg3 15.1-15.3k vs 14.4-14.5k images/s);
            # sparse ones: the 4-wave NMS runs beside the next seed loop (planted 370-375k
            # vs 385-394k, A/B on one box)
            wide = STAGE_NMS_WIDE if dense else 0
            early = 0 if b_first == 'lazy' else STAGE_COMPLETE_EARLY
            if b_first == 'lazy':
                launch(STAGE_CIFHR)
            elif b_first:
                # the force-complete sets start on the library's side stream before the
                # CifHr map (they read only the CAF fields); the next call's join covers them
                launch(STAGE_CIFHR | STAGE_COMPLETE_EARLY)
            else:
                launch(STAGE_CIFHR)
            if events:
                events[1].record()
            launch(STAGE_SEEDS | STAGE_CAF | (0 if b_first else early))
            if events:
                events[2].record()
            front_done = torch.cuda.Event()
            front_done.record()
        per_ws = _BACK2 if _BACK2 is not None else not dense
        if per_ws:  # loop + tail on the workspace's stream (every cross-batch order is an event)
            back = tail = (self.back, self.tail)[par % 2]
        else:
            back, tail = self.back, self.tail
        back.wait_event(front_done)
        if self._back_done[par] is not None:  # the workspace's previous NMS (records)
            back.wait_event(self._back_done[par])
        with torch.cuda.stream(back):
            if events:
                events[3].record()
            launch(STAGE_GROW | early | STAGE_SEED_LOOP_ONLY)
            if events and len(events) > 5:
                events[5].record()
            loop_done = torch.cuda.Event()
            loop_done.record()
        if tail is not back:
            tail.wait_event(loop_done)
        with torch.cuda.stream(tail):
            if _SPLIT_TAIL:
                launch(STAGE_GROW | early | STAGE_AFTER_SEED_LOOP | STAGE_COMPLETE_ONLY | wide)
                sets_done = torch.cuda.Event()
                sets_done.record()
                b = launch(STAGE_GROW | early | STAGE_AFTER_SEED_LOOP | STAGE_NMS_ONLY | wide)
            else:
                b = launch(STAGE_GROW | early | STAGE_AFTER_SEED_LOOP | wide)
                sets_done = None
            if events:
                events[4].record()
            back_done = torch.cuda.Event()
            back_done.record()
            pending = DecodeEngine.fetch_async(b, compact, device_out=device_out,
                                               stream=tail)
        pending.on_counts = self._note_counts
        self._back_done[par] = back_done
        self._sets_done[par] = sets_done or back_done
        return b, pending

    def _note_counts(self, counts):
        self.density = float(counts.mean()) if len(counts) else 0.0


_ENGINE = None


def engine():
    global _ENGINE  # pylint: disable=global-statement
    if _ENGINE is None:
        _ENGINE = DecodeEngine()
    return _ENGINE
