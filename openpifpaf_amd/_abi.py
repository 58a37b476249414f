"""NumPy / ctypes mirrors of the plain-data types in include/pifpaf_amd.h."""
import ctypes

import numpy as np

PP_ABI_VERSION = 4
PP_MAX_KP = 24
PP_MAX_EDGES = 64
PP_MAX_FRONTIER = 4 * PP_MAX_EDGES

PP_ST_ANN_OVERFLOW = 1
PP_ST_NMS_OVERFLOW = 2
PP_ST_SEED_OVERFLOW = 4
PP_ST_DEC_OVERFLOW = 8

STATUS_NAMES = {
    0: 'PP_OK', -1: 'PP_EINVAL', -2: 'PP_ESHAPE', -3: 'PP_EOVERFLOW', -4: 'PP_EHIP',
    -5: 'PP_ENOMEM',
}

ANN_DTYPE = np.dtype([
    ('data', np.float32, (PP_MAX_KP, 3)),
    ('joint_scales', np.float32, (PP_MAX_KP,)),
    ('score', np.float64),
    ('n_keypoints', np.int32),
    ('n_decoding', np.int32),
    ('n_frontier', np.int32),
    ('image', np.int32),
    ('decoding_pairs', np.uint8, (PP_MAX_KP, 2)),
    ('decoding_xyv', np.float32, (PP_MAX_KP, 6)),
    ('frontier_pairs', np.uint8, (PP_MAX_FRONTIER, 2)),
], align=True)
assert ANN_DTYPE.itemsize == 1544, ANN_DTYPE.itemsize

PP_PACK_DECODING = 1
PP_PACK_FRONTIER = 2
PP_PACK_REFETCH = 0x8000
PACK_ALL = PP_PACK_DECODING | PP_PACK_FRONTIER


def _up(n, m):
    return -(-n // m) * m


def packed_dtype(k, c, flags=PACK_ALL):
    """Compact record of pp_pack_compact (include/pifpaf_amd.h) for K keypoints and C
    skeleton edges; the layout pp_packed_record_size(K, C, flags) sizes."""
    f = min(PP_MAX_FRONTIER, 4 * c)
    names = ['score', 'image', 'n_decoding', 'n_frontier', 'data', 'joint_scales']
    formats = ['<f8', '<i4', '<u2', '<u2', ('<f4', (k, 3)), ('<f4', (k,))]
    offsets = [0, 8, 12, 14, 16, 16 + 12 * k]
    o = 16 + 16 * k
    if flags & PP_PACK_DECODING:
        names += ['decoding_pairs', 'decoding_v', 'decoding_xy']
        formats += [('u1', (k, 2)), ('<f4', (k, 2)), ('<f4', (k, 2))]
        offsets += [o, o + _up(2 * k, 4), o + _up(2 * k, 4) + 8 * k]
        o += _up(2 * k, 4) + 16 * k
    if flags & PP_PACK_FRONTIER:
        names.append('frontier_pairs')
        formats.append(('u1', (f, 2)))
        offsets.append(o)
        o += _up(2 * f, 4)
    return np.dtype({'names': names, 'formats': formats, 'offsets': offsets,
                     'itemsize': _up(o, 16)})


SEED_DTYPE = np.dtype([
    ('v', np.float32), ('field', np.int32), ('x', np.float32), ('y', np.float32),
    ('s', np.float32),
])


class PPConfig(ctypes.Structure):
    """struct pp_config (include/pifpaf_amd.h)."""
    _fields_ = [
        ('cif_threshold', ctypes.c_float),
        ('seed_threshold', ctypes.c_float),
        ('seed_score_scale', ctypes.c_float),
        ('caf_threshold', ctypes.c_float),
        ('complete_caf_threshold', ctypes.c_float),
        ('cif_floor', ctypes.c_float),
        ('keypoint_threshold', ctypes.c_float),
        ('nms_keypoint_threshold', ctypes.c_float),
        ('nms_instance_threshold', ctypes.c_float),
        ('nms_suppression', ctypes.c_float),
        ('stride', ctypes.c_int32),
        ('cif_neighbors', ctypes.c_int32),
        ('force_complete', ctypes.c_int32),
        ('greedy', ctypes.c_int32),
        ('connection_method', ctypes.c_int32),
        ('apply_nms', ctypes.c_int32),
        ('occupancy_reduction', ctypes.c_int32),
        ('occupancy_min_scale', ctypes.c_int32),
        ('seed_skip_mask', ctypes.c_uint32),
        ('exp_mode', ctypes.c_int32),
        ('confidence_scales', ctypes.POINTER(ctypes.c_float)),
    ]


EXP_MODES = {'numpy_simd': 0, 'correct': 1}


def make_config(*, cif_threshold=0.1, seed_threshold=0.2, seed_score_scale=1.0,
                caf_threshold=0.1, complete_caf_threshold=0.0001, cif_floor=0.1,
                keypoint_threshold=0.0, nms_keypoint_threshold=0.0,
                nms_instance_threshold=0.0, nms_suppression=0.0, stride=8, cif_neighbors=16,
                force_complete=True, greedy=False, connection_method='blend', apply_nms=True,
                occupancy_reduction=2, occupancy_min_scale=4, seed_mask=None,
                confidence_scales=None, exp_mode='numpy_simd'):
    """Defaults = eval_coco defaults (decoder/factory.py:17-22, eval_coco.py:215).
    confidence_scales: CifCaf's per-CAF frontier weights (cifcaf.py:259-260, 282-284) as
    float32, the type NumPy multiplies a float32 score by a Python float in; the array is
    kept alive on the returned struct.  exp_mode: how np.exp of the CAF scores rounds
    (cifcaf.py:139): 'numpy_simd' (default) is NumPy's float32 SIMD exp, the routine the
    reference runs on any x86-64 with FMA3; 'correct' rounds correctly (NumPy's scalar
    loop)."""
    if connection_method not in ('blend', 'max'):
        raise Exception('connection method not known')
    if exp_mode not in EXP_MODES:
        raise ValueError('exp_mode must be one of {}'.format(sorted(EXP_MODES)))
    cfg = PPConfig(
        cif_threshold, seed_threshold, seed_score_scale, caf_threshold,
        complete_caf_threshold, cif_floor, keypoint_threshold, nms_keypoint_threshold,
        nms_instance_threshold, nms_suppression, int(stride), int(cif_neighbors),
        int(bool(force_complete)), int(bool(greedy)),
        0 if connection_method == 'blend' else 1, int(bool(apply_nms)),
        int(occupancy_reduction), int(occupancy_min_scale), seed_skip_mask(seed_mask),
        EXP_MODES[exp_mode])
    if confidence_scales is not None:
        cs = np.ascontiguousarray([float(v) for v in confidence_scales], dtype=np.float32)
        cfg._confidence_scales = cs  # the struct points into it
        cfg.confidence_scales = cs.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    return cfg


def check_seed_mask(seed_mask, k):
    """The reference indexes seed_mask[field_i] for every one of the K fields
    (cif_seeds.py:28-29): a shorter mask raises its IndexError on every path here too."""
    if seed_mask is not None and len(seed_mask) < k:
        raise IndexError('list index out of range (seed_mask has {} entries for {} fields)'
                         .format(len(seed_mask), k))


def seed_skip_mask(seed_mask):
    """pp_config.seed_skip_mask of FieldConfig.seed_mask: bit f set where seed_mask[f] is
    falsy (cif_seeds.py:28-29); None = every field seeds."""
    if seed_mask is None:
        return 0
    if len(seed_mask) > 32:
        raise ValueError('seed_mask longer than 32 fields')
    return sum(1 << f for f, m in enumerate(seed_mask) if not m)


EVAL_CONFIG = dict(seed_threshold=0.2, force_complete=True, keypoint_threshold=0.0,
                   nms_keypoint_threshold=0.0, nms_instance_threshold=0.0)
PREDICT_CONFIG = dict(seed_threshold=0.5, force_complete=False, keypoint_threshold=0.001,
                      nms_keypoint_threshold=0.001, nms_instance_threshold=0.1)


def skeleton_array(skeleton):
    return np.ascontiguousarray(np.asarray(skeleton, dtype=np.int32).reshape(-1, 2))


# pp_det: one AnnotationDet (annotation.py:122-137) with its image
DET_DTYPE = np.dtype([('field', '<i4'), ('score', '<f4'), ('bbox', '<f4', (4,)), ('image', '<i4'),
                      ('pad_', '<i4')])
assert DET_DTYPE.itemsize == 32


class DetNms(ctypes.Structure):
    """pp_det_nms: nms.Detection class attributes (nms.py:60-65)."""
    _fields_ = [('suppression', ctypes.c_float), ('suppression_soft', ctypes.c_float),
                ('instance_threshold', ctypes.c_float), ('iou_threshold', ctypes.c_float),
                ('iou_threshold_soft', ctypes.c_float), ('apply', ctypes.c_int32)]


ROLE_CIF, ROLE_CAF, ROLE_HRMAP = 1, 2, 4


class Scale(ctypes.Structure):
    """pp_scale: one head of a multi-scale FieldConfig (field_config.py:7-13).  role
    ROLE_CIF / ROLE_CAF bits say which head list the entry joins (0 = both).  0.0 for a
    min scale / distance means unused (the reference tests them for truthiness)."""
    _fields_ = [('cif', ctypes.c_void_p), ('caf', ctypes.c_void_p), ('H', ctypes.c_int32),
                ('W', ctypes.c_int32), ('stride', ctypes.c_int32),
                ('cif_min_scale', ctypes.c_float), ('caf_min_distance', ctypes.c_float),
                ('caf_max_distance', ctypes.c_float), ('role', ctypes.c_int32)]


def scale_list(cifs, cafs, cif_strides, caf_strides, cif_min_scales=None,
               caf_min_distances=None, caf_max_distances=None):
    """pp_scale array of a FieldConfig: the CIF heads (role CIF) then the CAF heads (role
    CAF).  cifs / cafs: (pointer, H, W) per head."""
    nc, na = len(cifs), len(cafs)
    arr = (Scale * (nc + na))()
    for m, (ptr, h, w) in enumerate(cifs):
        ms = (cif_min_scales or [0.0] * nc)[m] or 0.0
        arr[m] = Scale(ptr, None, h, w, int(cif_strides[m]), float(ms), 0.0, 0.0, ROLE_CIF)
    for m, (ptr, h, w) in enumerate(cafs):
        dmin = (caf_min_distances or [0.0] * na)[m] or 0.0
        dmax = (caf_max_distances or [None] * na)[m] or 0.0
        arr[nc + m] = Scale(None, ptr, h, w, int(caf_strides[m]), 0.0, float(dmin),
                            float(dmax), ROLE_CAF)
    return arr
