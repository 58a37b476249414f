"""Host twins of decoder stages on NumPy arrays: pp_cifhr_cpu, pp_seeds_cpu,
pp_caf_scored_cpu and pp_nms_keypoints_cpu (csrc/stages_cpu.hip) -- CifHr.fill
(cif_hr.py:23-81), CifSeeds.fill + get (cif_seeds.py:23-64) and CafScored.fill
(caf_scored.py:32-98) for one CIF and one CAF head, and nms.Keypoints.annotations
(nms.py:17-57), on the calling thread -- and the whole decode, pp_decode_batch_cpu
(csrc/decode_cpu.hip: CifCaf.__call__, cifcaf.py:67-122, with the seed loop, _grow,
complete_annotations and the NMS), on host threads.

An explicit host API, like openpifpaf_amd.functional_cpu: the decoder classes compute on the
device and never fall back to it, and it raises when the library is missing.  `cfg` is a
pp_config (openpifpaf_amd._abi.make_config); the outputs match the device stages bit for bit
(tests/test_stages_cpu.py pins them to the reference's own fixtures).
"""
import ctypes

import numpy as np

from ._abi import ANN_DTYPE, PP_ST_ANN_OVERFLOW, PP_ST_DEC_OVERFLOW, SEED_DTYPE
from ._lib import PPError, call


def _f32(a, ndim, what):
    if not isinstance(a, np.ndarray) or a.ndim != ndim:
        raise ValueError('{} must be a {}-d NumPy array'.format(what, ndim))
    return np.ascontiguousarray(a, dtype=np.float32)


def _hr_shape(h, w, stride):
    hh, ww = (h - 1) * stride + 1, (w - 1) * stride + 1
    return hh, ww, (ww + 31) // 32 * 32


def cifhr(cif, cfg):
    """cif (n, K, 5, H, W) -> the CifHr maps (n, K, H', pitch) float32 (columns past W' are
    zero); `[..., :W']` is CifHr.accumulated of each image."""
    cif = _f32(cif, 5, 'cif')
    n, k, _, h, w = cif.shape
    hh, _, pitch = _hr_shape(h, w, cfg.stride)
    out = np.empty((n, k, hh, pitch), np.float32)
    call('pp_cifhr_cpu', cif.ctypes.data, n, k, h, w, ctypes.byref(cfg), out.ctypes.data)
    return out


def seeds(cif, hr, cfg):
    """cif (n, K, 5, H, W), hr (n, K, H', pitch) from cifhr() -> per image a SEED_DTYPE array
    in CifSeeds.get() order (v, field, x, y, s)."""
    cif = _f32(cif, 5, 'cif')
    hr = _f32(hr, 4, 'hr')
    n, k, _, h, w = cif.shape
    if hr.shape != (n, k) + _hr_shape(h, w, cfg.stride)[::2]:
        raise ValueError('hr must be (n, K, H\', pitch) for these fields')
    cap = max(1, k * h * w)
    out = np.empty((n, cap), SEED_DTYPE)
    counts = np.empty(n, np.int32)
    call('pp_seeds_cpu', cif.ctypes.data, hr.ctypes.data, n, k, h, w, ctypes.byref(cfg),
         out.ctypes.data, cap, counts.ctypes.data)
    return [out[i, :counts[i]].copy() for i in range(n)]


def caf_scored(caf, hr, skeleton, score_th, cfg):
    """caf (n, C, 9, H, W), hr (n, K, H', pitch), 1-based skeleton (C, 2) -> per image
    (forward, backward): lists over the C fields of (9, N) float32 column sets, as
    CafScored(score_th=...).fill() holds them."""
    caf = _f32(caf, 5, 'caf')
    hr = _f32(hr, 4, 'hr')
    n, c, _, h, w = caf.shape
    k = hr.shape[1]
    if hr.shape != (n, k) + _hr_shape(h, w, cfg.stride)[::2]:
        raise ValueError('hr must be (n, K, H\', pitch) for these fields')
    sk = np.ascontiguousarray(skeleton, dtype=np.int32).reshape(-1, 2)
    if len(sk) != c:
        raise ValueError('skeleton has {} pairs for {} CAF fields'.format(len(sk), c))
    cols = np.empty((n, c, 2, 9, h * w), np.float32)
    counts = np.empty((n, c, 2), np.int32)
    call('pp_caf_scored_cpu', caf.ctypes.data, hr.ctypes.data, n, k, c, h, w, sk.ctypes.data,
         ctypes.c_float(score_th), ctypes.byref(cfg), cols.ctypes.data, counts.ctypes.data)
    out = []
    for i in range(n):
        fwd = [cols[i, f, 1, :, :counts[i, f, 1]].copy() for f in range(c)]
        bwd = [cols[i, f, 0, :, :counts[i, f, 0]].copy() for f in range(c)]
        out.append((fwd, bwd))
    return out


def nms_keypoints(data, joint_scales, cfg, *, score_spec=None, instance_threshold=None):
    """nms.Keypoints.annotations over one list of annotations given as data (N, K, 3) float32
    (edited in place as the reference edits ann.data) and joint_scales (N, K), with cfg's
    nms_* thresholds -> (input indices of the survivors in output order, their scores).
    score_spec = (spec (N,) int32, score_weights (N, K) float64, fixed (N,) float64) as
    decoder.nms builds it: each annotation's own score() (pp_nms_keypoints_scored_cpu), with
    instance_threshold (float64) replacing cfg's float32 one."""
    if not isinstance(data, np.ndarray) or data.dtype != np.float32 or data.ndim != 3:
        raise ValueError('data must be a float32 (N, K, 3) NumPy array')
    n, k, _ = data.shape
    recs = np.zeros(max(1, n), ANN_DTYPE)
    recs['data'][:n, :k] = data
    recs['joint_scales'][:n, :k] = joint_scales
    recs['n_keypoints'] = k
    out = np.zeros_like(recs)
    counts = np.array([n], np.int32)
    out_counts = np.zeros(1, np.int32)
    index = np.zeros(len(recs), np.int32)
    if score_spec is None:
        call('pp_nms_keypoints_cpu', recs.ctypes.data, counts.ctypes.data, 1, k, len(recs),
             ctypes.byref(cfg), out.ctypes.data, out_counts.ctypes.data, index.ctypes.data)
    else:
        spec, sw, fixed = (np.ascontiguousarray(a, t) for a, t in
                           zip(score_spec, (np.int32, np.float64, np.float64)))
        if spec.shape != (n,) or sw.shape != (n, k) or fixed.shape != (n,):
            raise ValueError('score_spec must be (N,), (N, K), (N,) arrays')
        it = (float(cfg.nms_instance_threshold) if instance_threshold is None
              else float(instance_threshold))
        call('pp_nms_keypoints_scored_cpu', recs.ctypes.data, counts.ctypes.data, 1, k,
             len(recs), ctypes.byref(cfg), it, spec.ctypes.data, sw.ctypes.data,
             fixed.ctypes.data, out.ctypes.data, out_counts.ctypes.data, index.ctypes.data)
    data[...] = recs['data'][:n, :k]
    m = int(out_counts[0])
    return index[:m].tolist(), out['score'][:m].copy()


def decode_batch(cif, caf, skeleton, cfg, *, n_threads=0, cap=None):
    """The whole CifCaf decode on host threads (pp_decode_batch_cpu, csrc/decode_cpu.hip):
    cif (n, K, 5, H, W), caf (n, C, 9, H, W), 1-based skeleton (C, 2) -> (records, offsets)
    as engine.DecodeEngine.decode returns them: ANN_DTYPE records of all images packed in
    image order (each image's in nms.Keypoints order, `score` = Annotation.score()) and
    per-image offsets (n + 1).  n_threads 0: one per hardware thread.  The annotation
    capacity doubles until no image overflows, as the device decode's does."""
    cif = _f32(cif, 5, 'cif')
    caf = _f32(caf, 5, 'caf')
    n, k, _, h, w = cif.shape
    c = caf.shape[1]
    if caf.shape[0] != n or caf.shape[3:] != cif.shape[3:]:
        raise ValueError('cif and caf batch / spatial shapes differ')
    sk = np.ascontiguousarray(skeleton, dtype=np.int32).reshape(-1, 2)
    if len(sk) != c:
        raise ValueError('skeleton has {} pairs for {} CAF fields'.format(len(sk), c))
    cap = cap or int(min(8192, max(128, (h * w) // 8)))  # engine.default_ann_capacity
    while True:
        anns = np.zeros((max(1, n), cap), ANN_DTYPE)
        counts = np.zeros(max(1, n), np.int32)
        status = np.zeros(max(1, n), np.int32)
        call('pp_decode_batch_cpu', cif.ctypes.data, caf.ctypes.data, n, k, c, h, w,
             sk.ctypes.data, ctypes.byref(cfg), anns.ctypes.data, cap, counts.ctypes.data,
             status.ctypes.data, int(n_threads))
        if not (status[:n] & PP_ST_ANN_OVERFLOW).any():
            break
        cap *= 2
    if (status[:n] & PP_ST_DEC_OVERFLOW).any():
        raise PPError('decoding/frontier order exceeded the record capacity')
    offsets = np.concatenate([[0], np.cumsum(counts[:n])]).astype(np.int64)
    recs = np.concatenate([anns[i, :counts[i]] for i in range(n)]) if n else \
        np.zeros(0, ANN_DTYPE)
    return recs, offsets
