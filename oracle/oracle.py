"""ctypes wrapper over oracle/liboracle.so (oracle/pp_oracle.c).

TEST INFRASTRUCTURE: the CPU restatement of the reference decoder used as the parity
checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product
package never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

from openpifpaf_amd._abi import (ANN_DTYPE, ROLE_HRMAP, SEED_DTYPE, Scale, make_config, scale_list,
                                 skeleton_array)

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags='C_CONTIGUOUS')
_vp = ctypes.c_void_p
_l = ctypes.c_long
_i = ctypes.c_int
_f = ctypes.c_float


def build():
    subprocess.check_call(['make', '-s', '-C', HERE])


def lib():
    global _LIB  # pylint: disable=global-statement
    if _LIB is None:
        path = os.path.join(HERE, 'liboracle.so')
        if not os.path.exists(path):
            build()
        _LIB = ctypes.CDLL(path)
        _LIB.orc_decode.restype = ctypes.c_long
        _LIB.orc_seeds.restype = ctypes.c_long
        _LIB.orc_weiszfeld_nd.restype = ctypes.c_long
        _LIB.orc_center_filter.restype = ctypes.c_long
        _LIB.orc_ann_score.restype = ctypes.c_double
        _LIB.orc_nms_keypoints.restype = ctypes.c_long
        _LIB.orc_cifdet_seeds.restype = ctypes.c_long
        _LIB.orc_cifdet_decode.restype = ctypes.c_long
        _LIB.orc_seeds_multi.restype = ctypes.c_long
        _LIB.orc_decode_multi.restype = ctypes.c_long
        _LIB.orc_decode_initial.restype = ctypes.c_long
        assert _LIB.orc_sizeof_ann() == ANN_DTYPE.itemsize
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _c32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def hr_shape(h, w, stride=8):
    return (h - 1) * stride + 1, (w - 1) * stride + 1


def cifhr(cif, cfg=None):
    cfg = cfg or make_config()
    cif = _c32(cif)
    k, _, h, w = cif.shape
    hh, ww = hr_shape(h, w, cfg.stride)
    out = np.empty((k, hh, ww), np.float32)
    lib().orc_cifhr(_p(cif), _i(k), _i(h), _i(w), ctypes.byref(cfg), _p(out))
    return out


def seeds(cif, hr, cfg=None):
    cfg = cfg or make_config()
    cif = _c32(cif)
    hr = _c32(hr)
    k, _, h, w = cif.shape
    cap = k * h * w
    out = np.empty(cap, SEED_DTYPE)
    n = lib().orc_seeds(_p(cif), _p(hr), _l(hr.shape[-1]), _i(k), _i(h), _i(w),
                        ctypes.byref(cfg), _p(out), _l(cap))
    return out[:n]


def caf_scored(caf, hr, skeleton, score_th, cfg=None):
    """Returns (forward, backward): lists of (9, N_i) arrays (caf_scored.py:23-24)."""
    cfg = cfg or make_config()
    caf = _c32(caf)
    hr = _c32(hr)
    c, _, h, w = caf.shape
    k = hr.shape[0]
    skel = skeleton_array(skeleton)
    cols = np.zeros((c, 2, 9, h * w), np.float32)
    counts = np.zeros((c, 2), np.int32)
    lib().orc_caf_scored(_p(caf), _p(hr), _l(hr.shape[-1]), _i(k), _i(c), _i(h), _i(w),
                         _p(skel), _f(score_th), ctypes.byref(cfg), _p(cols), _p(counts))
    forward = [cols[i, 1, :, :counts[i, 1]].copy() for i in range(c)]
    backward = [cols[i, 0, :, :counts[i, 0]].copy() for i in range(c)]
    return forward, backward


def decode(cif, caf, skeleton, cfg=None):
    """One image, CifCaf.__call__ -> structured array of pp_ann records."""
    cfg = cfg or make_config()
    cif = _c32(cif)
    caf = _c32(caf)
    k, _, h, w = cif.shape
    c = caf.shape[0]
    skel = skeleton_array(skeleton)
    cap = 64
    while True:
        out = np.zeros(cap, ANN_DTYPE)
        n = lib().orc_decode(_p(cif), _p(caf), _i(k), _i(c), _i(h), _i(w), _p(skel),
                             ctypes.byref(cfg), _p(out), _l(cap))
        if n < 0:
            raise ValueError('oracle decode rejected the shapes')
        if n <= cap:
            return out[:n]
        cap = int(n)


class Members:
    """The heads of a multi-scale FieldConfig for the oracle: fields list + FieldConfig
    lists (cif_indices, caf_indices, strides, cif_min_scales, caf min / max distances)."""

    def __init__(self, fields, *, cif_indices, caf_indices, cif_strides, caf_strides,
                 cif_min_scales=None, caf_min_distances=None, caf_max_distances=None, **_):
        self.cifs = [_c32(fields[i]) for i in cif_indices]
        self.cafs = [_c32(fields[i]) for i in caf_indices]
        self.arr = scale_list([(c.ctypes.data, c.shape[-2], c.shape[-1]) for c in self.cifs],
                              [(c.ctypes.data, c.shape[-2], c.shape[-1]) for c in self.cafs],
                              cif_strides, caf_strides, cif_min_scales, caf_min_distances,
                              caf_max_distances)
        self.n = len(self.arr)
        self.pairs = int(len(cif_indices) == 10)  # cif_hr.py:63
        self.k = self.cifs[0].shape[0]
        self.c = self.cafs[0].shape[0]
        self.hr_shape = (self.k,) + hr_shape(self.cifs[0].shape[-2], self.cifs[0].shape[-1],
                                             int(cif_strides[0]))


def cifhr_multi(members, cfg=None):
    cfg = cfg or make_config()
    out = np.empty(members.hr_shape, np.float32)
    lib().orc_cifhr_multi(members.arr, _i(members.n), _i(members.pairs), _i(members.k),
                          ctypes.byref(cfg), _p(out))
    return out


def seeds_multi(members, hr, cfg=None):
    cfg = cfg or make_config()
    hr = _c32(hr)
    cap = sum(c.shape[0] * c.shape[2] * c.shape[3] for c in members.cifs)
    out = np.empty(max(cap, 1), SEED_DTYPE)
    n = lib().orc_seeds_multi(members.arr, _i(members.n), _i(members.k), _p(hr),
                              _l(hr.shape[1]), _l(hr.shape[2]), ctypes.byref(cfg), _p(out),
                              _l(cap))
    return out[:n]


def caf_scored_multi(members, hr, skeleton, score_th, cfg=None):
    """(forward, backward) lists of (9, N_i) arrays, every head's columns concatenated."""
    cfg = cfg or make_config()
    hr = _c32(hr)
    skel = skeleton_array(skeleton)
    cap = sum(c.shape[2] * c.shape[3] for c in members.cafs)
    c = members.c
    cols = np.zeros((c, 2, 9, cap), np.float32)
    counts = np.zeros((c, 2), np.int32)
    lib().orc_caf_scored_multi(members.arr, _i(members.n), _i(hr.shape[0]), _i(c), _p(hr),
                               _l(hr.shape[1]), _l(hr.shape[2]), _p(skel), _f(score_th),
                               ctypes.byref(cfg), _p(cols), _l(cap), _p(counts))
    forward = [cols[i, 1, :, :counts[i, 1]].copy() for i in range(c)]
    backward = [cols[i, 0, :, :counts[i, 0]].copy() for i in range(c)]
    return forward, backward


def decode_multi(members, skeleton, cfg=None):
    """One image, CifCaf.__call__ over a multi-scale FieldConfig -> pp_ann records."""
    cfg = cfg or make_config()
    skel = skeleton_array(skeleton)
    cap = 64
    while True:
        out = np.zeros(cap, ANN_DTYPE)
        n = lib().orc_decode_multi(members.arr, _i(members.n), _i(members.pairs),
                                   _i(members.k), _i(members.c), _p(skel), ctypes.byref(cfg),
                                   _p(out), _l(cap))
        if n < 0:
            raise ValueError('oracle decode rejected the shapes')
        if n <= cap:
            return out[:n]
        cap = int(n)


def decode_initial(cif, caf, skeleton, initial, cfg=None):
    """One image, CifCaf.__call__(fields, initial_annotations) (cifcaf.py:67-122): `initial`
    pp_ann records grown and marked before the seed loop.  Returns (records, index of each
    record in the annotation list before NMS)."""
    cfg = cfg or make_config()
    cif, caf = _c32(cif), _c32(caf)
    k, _, h, w = cif.shape
    c = caf.shape[0]
    arr = scale_list([(cif.ctypes.data, h, w)], [(caf.ctypes.data, h, w)], [cfg.stride],
                     [cfg.stride])
    init = np.ascontiguousarray(initial, ANN_DTYPE)
    skel = skeleton_array(skeleton)
    cap = 64 + len(init)
    while True:
        out = np.zeros(cap, ANN_DTYPE)
        idx = np.zeros(cap, np.int32)
        n = lib().orc_decode_initial(arr, _i(len(arr)), _i(0), _i(k), _i(c), _p(skel),
                                     ctypes.byref(cfg), _p(init), _l(len(init)), _p(out),
                                     _l(cap), _p(idx))
        if n < 0:
            raise ValueError('oracle decode rejected the shapes')
        if n <= cap:
            return out[:n], idx[:n]
        cap = int(n)


def _geometry_entry(hr_shape_):
    """pp_scale entry naming a CifHr map of (hh, ww) (PP_ROLE_HRMAP, stride 1)."""
    return Scale(None, None, int(hr_shape_[-2]), int(hr_shape_[-1]), 1, 0.0, 0.0, 0.0, ROLE_HRMAP)


def cifhr_group(cifs, stride, min_scale=0.0, hr_shape_=None, cfg=None):
    """CifHr.fill_multiple(cifs, stride, min_scale)'s `ta` (cif_hr.py:42-57): the heads
    accumulated into one zero map with len_cifs = len(cifs), map size hr_shape_ (K, hh, ww)
    or from cifs[0] and stride."""
    cfg = cfg or make_config()
    cifs = [_c32(c) for c in cifs]
    k = cifs[0].shape[0]
    arr = scale_list([(c.ctypes.data, c.shape[-2], c.shape[-1]) for c in cifs], [],
                     [stride] * len(cifs), [], [min_scale] * len(cifs))
    if hr_shape_ is None:
        hr_shape_ = (k,) + hr_shape(cifs[0].shape[-2], cifs[0].shape[-1], int(stride))
    full = (Scale * (len(arr) + 1))(*arr, _geometry_entry(hr_shape_))
    out = np.empty(tuple(hr_shape_), np.float32)
    lib().orc_cifhr_multi(full, _i(len(full)), _i(len(cifs) if len(cifs) > 1 else 0), _i(k),
                          ctypes.byref(cfg), _p(out))
    return out


def seeds_head(cif, stride, hr, min_scale=0.0, cfg=None):
    """CifSeeds.fill_cif(cif, stride, min_scale=...) (cif_seeds.py:23-50), sorted."""
    cfg = cfg or make_config()
    cif, hr = _c32(cif), _c32(hr)
    k, _, h, w = cif.shape
    arr = scale_list([(cif.ctypes.data, h, w)], [], [stride], [], [min_scale])
    out = np.empty(max(1, k * h * w), SEED_DTYPE)
    n = lib().orc_seeds_multi(arr, _i(1), _i(k), _p(hr), _l(hr.shape[1]), _l(hr.shape[2]),
                              ctypes.byref(cfg), _p(out), _l(k * h * w))
    return out[:n]


def caf_scored_head(caf, stride, hr, skeleton, score_th, min_distance=0.0, max_distance=None,
                    cfg=None):
    """CafScored.fill_caf(caf, stride, min_distance, max_distance)'s columns of one head
    (caf_scored.py:32-86): (forward, backward) lists of (9, N_i) arrays."""
    cfg = cfg or make_config()
    caf, hr = _c32(caf), _c32(hr)
    c, _, h, w = caf.shape
    arr = scale_list([], [(caf.ctypes.data, h, w)], [], [stride], None, [min_distance],
                     [max_distance])
    skel = skeleton_array(skeleton)
    cols = np.zeros((c, 2, 9, h * w), np.float32)
    counts = np.zeros((c, 2), np.int32)
    lib().orc_caf_scored_multi(arr, _i(1), _i(hr.shape[0]), _i(c), _p(hr), _l(hr.shape[1]),
                               _l(hr.shape[2]), _p(skel), _f(score_th), ctypes.byref(cfg),
                               _p(cols), _l(h * w), _p(counts))
    forward = [cols[i, 1, :, :counts[i, 1]].copy() for i in range(c)]
    backward = [cols[i, 0, :, :counts[i, 0]].copy() for i in range(c)]
    return forward, backward


def nms_keypoints(data, scales, keypoint_threshold, instance_threshold, suppression):
    """nms.Keypoints().annotations on n annotations (data (n, K, 3), scales (n, K)).
    Returns (order: survivors' input indices, survivor records)."""
    n, k, _ = data.shape
    recs = np.zeros(n, ANN_DTYPE)
    recs['data'][:, :k] = data
    recs['joint_scales'][:, :k] = scales
    recs['n_keypoints'] = k
    recs['image'] = np.arange(n)
    cfg = make_config(nms_keypoint_threshold=keypoint_threshold,
                      nms_instance_threshold=instance_threshold, nms_suppression=suppression)
    m = lib().orc_nms_keypoints(recs.ctypes.data_as(_vp), _l(n), _i(k), ctypes.byref(cfg))
    return recs['image'][:m].astype(np.int64), recs[:m]


def ann_score(v):
    """Annotation.score() of joint confidences v (K,) (orc_ann_score reads v with stride 3)."""
    v = _c32(np.stack([v, np.zeros_like(v), np.zeros_like(v)], axis=1))
    return lib().orc_ann_score(_p(v.reshape(-1)), _i(len(v)))


# ---- functional.pyx primitives (field arrays mutated in place, like the reference) ----

def _field_args(field):
    assert field.dtype == np.float32 or field.dtype == np.uint8
    item = field.dtype.itemsize
    return (_l(field.shape[0]), _l(field.shape[1]),
            _l(field.strides[0] // item), _l(field.strides[1] // item))


def scalar_square_add_gauss_with_max(field, x, y, sigma, v, truncate=2.0, max_value=1.0):
    x, y, sigma, v = map(_c32, (x, y, sigma, v))
    lib().orc_scalar_square_add_gauss_with_max(
        _p(field), *_field_args(field), _p(x), _p(y), _p(sigma), _p(v), _l(len(x)),
        _f(truncate), _f(max_value))


def scalar_square_add_gauss(field, x, y, sigma, v, truncate=2.0):
    x, y, sigma, v = map(_c32, (x, y, sigma, v))
    lib().orc_scalar_square_add_gauss(
        _p(field), *_field_args(field), _p(x), _p(y), _p(sigma), _p(v), _l(len(x)),
        _f(truncate))


def scalar_square_max_gauss(field, x, y, sigma, v, truncate=2.0):
    x, y, sigma, v = map(_c32, (x, y, sigma, v))
    lib().orc_scalar_square_max_gauss(
        _p(field), *_field_args(field), _p(x), _p(y), _p(sigma), _p(v), _l(len(x)),
        _f(truncate))


def scalar_square_add_constant(field, x, y, width, v):
    x, y, width, v = map(_c32, (x, y, width, v))
    lib().orc_scalar_square_add_constant(
        _p(field), *_field_args(field), _p(x), _p(y), _p(width), _p(v), _l(len(x)))


def cumulative_average(cuma, cumw, x, y, width, v, w):
    assert cuma.strides == cumw.strides
    x, y, width, v, w = map(_c32, (x, y, width, v, w))
    lib().orc_cumulative_average(
        _p(cuma), _p(cumw), *_field_args(cuma), _p(x), _p(y), _p(width), _p(v), _p(w),
        _l(len(x)))


def weiszfeld_nd(x_np, y_np, weights, epsilon=1e-8, max_steps=20):
    x = _c32(x_np)
    weights = _c32(weights)
    denom = np.zeros_like(weights)
    lib().orc_weiszfeld_nd(_p(x), _l(x.shape[0]), _l(x.shape[1]), _l(x.shape[1]), _l(1),
                           _p(y_np), _p(weights), _f(epsilon), _l(max_steps), _p(denom))
    return y_np, denom


def scalar_values(field, x, y, default=-1):
    x, y = _c32(x), _c32(y)
    out = np.empty(len(x), np.float32)
    lib().orc_scalar_values(_p(field), *_field_args(field), _p(x), _p(y), _l(len(x)),
                            _f(default), _p(out))
    return out


def scalar_lookup(field, x, y, mode, default=0.0, reduction=1.0):
    x, y = _c32(np.atleast_1d(x)), _c32(np.atleast_1d(y))
    out = np.empty(len(x), np.float32 if mode < 2 else np.uint8)
    lib().orc_scalar_lookup(_p(field), *_field_args(field), _i(mode), _p(x), _p(y),
                            _l(len(x)), _f(default), _f(reduction), _p(out))
    return out


def center_filter(field, x, y, sigma, mode):
    rows, n = field.shape
    item = field.dtype.itemsize
    if mode == 3:
        out = np.zeros(n, np.uint8)
    else:
        out = np.zeros((rows, n), np.float32)
    k = lib().orc_center_filter(_p(field), _l(rows), _l(n), _l(field.strides[0] // item),
                                _l(field.strides[1] // item), _i(mode), _f(x), _f(y),
                                _f(sigma), _p(out))
    if mode == 3:
        return out != 0
    return out[:, :k]


# ---- network/heads.py field ingestion (numpy restatement, test infrastructure) -------------

_INGEST = {  # (n_conf, n_vec, n_scales), output channel -> concatenated channel
    'cif': ((1, 1, 1), (0, 1, 2, 3, 4)),
    'caf': ((1, 2, 2), (0, 1, 2, 5, 7, 3, 4, 6, 8)),        # heads.py:87
    'cifdet': ((1, 2, 0), (0, 1, 2, 5, 3, 4, 6)),           # heads.py:142
}


def fields_from_conv(conv, n_fields, kind, quad):
    """CompositeFieldFused.forward (eval, heads.py:406-455) after its conv, then the
    collector (heads.py:65-88 / 127-144).  sigmoid / exp in float64, rounded to float32."""
    (nc, nv, ns), perm = _INGEST[kind]
    x = np.asarray(conv, np.float32)
    for _ in range(quad):  # PixelShuffle(2), then [:, :, :-1, :-1]
        b, c, h, w = x.shape
        x = x.reshape(b, c // 4, 2, 2, h, w).transpose(0, 1, 4, 2, 5, 3).reshape(
            b, c // 4, 2 * h, 2 * w)[:, :, :-1, :-1]
    b, _, h, w = x.shape
    f0, f1, f2 = nc * n_fields, (nc + 2 * nv) * n_fields, (nc + 3 * nv) * n_fields
    conf = 1.0 / (1.0 + np.exp(-x[:, :f0].astype(np.float64)))
    parts = [conf.astype(np.float32).reshape(b, n_fields, nc, h, w),
             x[:, f0:f1].reshape(b, n_fields, 2 * nv, h, w),
             x[:, f1:f2].reshape(b, n_fields, nv, h, w)]
    if ns:
        parts.append(np.exp(x[:, f2:].astype(np.float64)).astype(np.float32).reshape(
            b, n_fields, ns, h, w))
    cat = np.concatenate(parts, axis=2)
    yy, xx = np.indices((h, w), dtype=np.float32)
    vec_pairs = 1 if kind == 'cifdet' else nv
    for v in range(vec_pairs):  # index_field_torch added to the vector components
        cat[:, :, 1 + 2 * v] += xx
        cat[:, :, 2 + 2 * v] += yy
    return np.ascontiguousarray(cat[:, :, list(perm)])


# ---- CifDet (decoder/generator/cifdet.py) --------------------------------------------------

DET_DTYPE = np.dtype([('field', '<i4'), ('score', '<f4'), ('bbox', '<f4', (4,)), ('image', '<i4'),
                      ('pad_', '<i4')])


class DetNms(ctypes.Structure):
    """pp_det_nms: nms.Detection class attributes (nms.py:60-65)."""
    _fields_ = [('suppression', ctypes.c_float), ('suppression_soft', ctypes.c_float),
                ('instance_threshold', ctypes.c_float), ('iou_threshold', ctypes.c_float),
                ('iou_threshold_soft', ctypes.c_float), ('apply', ctypes.c_int32)]


def det_nms_defaults():
    return DetNms(0.1, 0.3, 0.1, 0.7, 0.5, 1)


def cifdet_hr(det, cfg=None):
    cfg = cfg or make_config()
    det = _c32(det)
    k, _, h, w = det.shape
    hh, ww = hr_shape(h, w, cfg.stride)
    out = np.empty((k, hh, ww), np.float32)
    lib().orc_cifdet_hr(_p(det), _i(k), _i(h), _i(w), ctypes.byref(cfg), _p(out))
    return out


def cifdet_seeds(det, hr, cfg=None):
    """(n, 7): v, field, x, y, w, h, emission index; sorted as the reference."""
    cfg = cfg or make_config()
    det, hr = _c32(det), _c32(hr)
    k, _, h, w = det.shape
    cap = k * h * w
    out = np.empty((cap, 7), np.float32)
    n = lib().orc_cifdet_seeds(_p(det), _p(hr), _l(hr.shape[-1]), _i(k), _i(h), _i(w),
                               ctypes.byref(cfg), _p(out), _l(cap))
    return out[:n]


def cifdet_decode(det, cfg=None, nms=None):
    cfg = cfg or make_config()
    nms = nms or det_nms_defaults()
    det = _c32(det)
    k, _, h, w = det.shape
    cap = k * h * w
    out = np.zeros(cap, DET_DTYPE)
    n = lib().orc_cifdet_decode(_p(det), _i(k), _i(h), _i(w), ctypes.byref(cfg),
                                ctypes.byref(nms), out.ctypes.data_as(_vp), _l(cap))
    return out[:n]


# ---- Preprocess.annotations_inverse (transforms/preprocess.py:35-95), numpy restatement ----

def annotations_inverse(data, scales, dxyv, nd, meta, hswap=None):
    """Poses (n, K, 3) / (n, K) / decoding xyv (n, T, 6) with nd[i] valid rows."""
    data, scales, dxyv = data.copy(), scales.copy(), dxyv.copy()
    off = np.asarray(meta['offset'], np.float64)
    sc = np.asarray(meta['scale'], np.float64)
    angle = -meta['rotation']['angle']
    if angle != 0.0:
        rw, rh = meta['rotation']['width'], meta['rotation']['height']
        c = np.float32(np.cos(angle / 180.0 * np.pi))
        s = np.float32(np.sin(angle / 180.0 * np.pi))
        hw, hh = np.float32((rw - 1) / 2), np.float32((rh - 1) / 2)
        xo, yo = data[:, :, 0] - hw, data[:, :, 1] - hh
        data[:, :, 0] = (hw + c * xo) + s * yo
        data[:, :, 1] = (hh - s * xo) + c * yo
    data[:, :, 0] = (data[:, :, 0].astype(np.float64) + off[0]).astype(np.float32)
    data[:, :, 1] = (data[:, :, 1].astype(np.float64) + off[1]).astype(np.float32)
    data[:, :, 0] = (data[:, :, 0].astype(np.float64) / sc[0]).astype(np.float32)
    data[:, :, 1] = (data[:, :, 1].astype(np.float64) / sc[1]).astype(np.float32)
    scales = (scales.astype(np.float64) / sc[0]).astype(np.float32)
    if meta['hflip']:
        w = float(meta['width_height'][0])
        data[:, :, 0] = (-data[:, :, 0].astype(np.float64) + (w - 1)).astype(np.float32)
        if hswap is not None:
            t = np.zeros_like(data)
            for src, dst in enumerate(hswap):
                t[:, dst] = data[:, src]
            data = t
    for i in range(len(dxyv)):
        for col in (0, 1, 3, 4):
            v = dxyv[i, :nd[i], col].astype(np.float64) + off[col % 3]
            v = v.astype(np.float32).astype(np.float64) / sc[col % 3]
            dxyv[i, :nd[i], col] = v.astype(np.float32)
    return data, scales, dxyv
