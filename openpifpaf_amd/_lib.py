"""ctypes binding of libpifpaf_amd.so (include/pifpaf_amd.h).

There is no fallback: if the HIP library is missing or no HIP device is visible, every
entry point raises.  The library is built in-tree by `python -m openpifpaf_amd.build`
(or __graft_entry__.build()).
"""
import ctypes
import os
import threading

from ._abi import PP_ABI_VERSION, STATUS_NAMES

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libpifpaf_amd.so')
if os.environ.get('PP_LIB_VARIANT'):  # diagnostic builds (e.g. 'stamps'); never the default
    LIB_PATH = LIB_PATH.replace('.so', '_{}.so'.format(os.environ['PP_LIB_VARIANT']))

_lock = threading.Lock()
_lib = None

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_f = ctypes.c_float
_f64 = ctypes.c_double
_sz = ctypes.c_size_t

_SIGNATURES = {
    'pp_version': ([], ctypes.c_int),
    'pp_last_error': ([], ctypes.c_char_p),
    'pp_default_config': ([_vp], None),
    'pp_cifhr_pitch': ([_i64], _i64),
    'pp_cifhr_workspace_size': ([_i32, _i32, _i32, _i32], _sz),
    'pp_cifhr_sparse_tiles': ([_i32, _i32, _i32], _i32),
    'pp_cifhr_sparse_workspace_size': ([_i32, _i32, _i32, _i32], _sz),
    'pp_cifhr': ([_vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _sz, _vp], ctypes.c_int),
    'pp_cifhr_sparse': ([_vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _sz, _vp],
                        ctypes.c_int),
    'pp_seeds': ([_vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _i32, _vp, _vp], ctypes.c_int),
    'pp_caf_scored': ([_vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _f, _vp, _vp, _vp, _vp],
                      ctypes.c_int),
    'pp_pack_records': ([_vp, _vp, _i32, _i32, _vp, _i64, _vp, _vp], ctypes.c_int),
    'pp_packed_record_size': ([_i32, _i32, _u32], _i64),
    'pp_pack_compact': ([_vp, _vp, _i32, _i32, _i32, _i32, _u32, _vp, _i64, _vp, _vp, _vp],
                        ctypes.c_int),
    'pp_decode_workspace_size': ([_i32, _i32, _i32, _i32, _i32, _vp, _i32], _sz),
    'pp_decode_workspace_zero_offset': ([_i32, _i32, _i32, _i32, _i32, _vp, _i32], _sz),
    'pp_decode_work_offset': ([_i32, _i32, _i32, _i32, _i32, _vp, _i32], _sz),
    'pp_decode_multi_work_offset': ([_vp, _i32, _i32, _i32, _i32, _i32, _vp, _i32], _sz),
    'pp_decode_batch': ([_vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _vp,
                         _vp, _vp, _sz, _vp], ctypes.c_int),
    'pp_decode_stages': ([_vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _vp,
                          _vp, _vp, _sz, _u32, _vp], ctypes.c_int),
    'pp_cifhr_multi_workspace_size': ([_vp, _i32, _i32, _i32, _i32], _sz),
    'pp_cifhr_multi': ([_vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _sz, _vp], ctypes.c_int),
    'pp_seeds_multi': ([_vp, _i32, _vp, _i32, _i32, _vp, _vp, _i32, _vp, _vp], ctypes.c_int),
    'pp_caf_scored_multi': ([_vp, _i32, _vp, _i32, _i32, _i32, _vp, _f, _vp, _vp, _i64, _vp,
                             _vp], ctypes.c_int),
    'pp_decode_multi_workspace_size': ([_vp, _i32, _i32, _i32, _i32, _i32, _vp, _i32], _sz),
    'pp_decode_multi_workspace_zero_offset': ([_vp, _i32, _i32, _i32, _i32, _i32, _vp, _i32],
                                              _sz),
    'pp_decode_multi': ([_vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _vp, _vp,
                         _vp, _sz, _u32, _vp], ctypes.c_int),
    'pp_decode_initial': ([_vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _vp,
                           _vp, _vp, _vp, _i32, _vp, _vp, _sz, _u32, _vp], ctypes.c_int),
    'pp_scalar_square_add_gauss_with_max': ([_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _f,
                                             _f, _vp], ctypes.c_int),
    'pp_scalar_square_add_gauss': ([_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _f, _vp],
                                   ctypes.c_int),
    'pp_scalar_square_add_constant': ([_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp],
                                      ctypes.c_int),
    'pp_scalar_square_max_gauss': ([_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _f, _vp],
                                   ctypes.c_int),
    'pp_cumulative_average': ([_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _vp],
                              ctypes.c_int),
    'pp_weiszfeld_nd': ([_vp, _i64, _i64, _i64, _vp, _vp, _f, _i64, _vp, _vp], ctypes.c_int),
    'pp_scalar_values': ([_vp, _i64, _i64, _i64, _vp, _vp, _i64, _f, _vp, _vp], ctypes.c_int),
    'pp_scalar_lookup': ([_vp, _i64, _i64, _i64, _i32, _vp, _vp, _i64, _f, _f, _vp, _vp],
                         ctypes.c_int),
    'pp_grow_connection': ([_vp, _i64, _i64, _f, _f, _f, _i32, _vp, _vp], ctypes.c_int),
    'pp_np_exp': ([_vp, _vp, _i64, _i32, _vp], ctypes.c_int),
    'pp_np_square': ([_vp, _vp, _i64, _vp], ctypes.c_int),
    'pp_nms_workspace_size': ([_i32, _i32], _sz),
    'pp_fields_dim': ([_i64, _i32], _i64),
    'pp_default_det_nms': ([_vp], None),
    'pp_annotations_inverse': ([_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp], ctypes.c_int),
    'pp_dets_inverse': ([_vp, _vp, _i32, _i32, _vp, _vp], ctypes.c_int),
    'pp_cifdet_hr': ([_vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _sz, _vp], ctypes.c_int),
    'pp_cifdet_seeds': ([_vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp], ctypes.c_int),
    'pp_cifdet_hr_multi': ([_vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _sz, _vp], ctypes.c_int),
    'pp_cifdet_seeds_multi': ([_vp, _i32, _vp, _i32, _i32, _vp, _vp, _vp, _vp], ctypes.c_int),
    'pp_cifdet_multi_workspace_size': ([_vp, _i32, _i32, _i32, _i32, _i32], _sz),
    'pp_cifdet_decode_multi': ([_vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _vp,
                                _vp, _vp, _sz, _vp], ctypes.c_int),
    'pp_nms_detection_workspace_size': ([_i32, _i32], _sz),
    'pp_nms_detection': ([_vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp],
                         ctypes.c_int),
    'pp_cifdet_workspace_size': ([_i32, _i32, _i32, _i32, _vp, _i32], _sz),
    'pp_cifdet_decode': ([_vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp,
                          _sz, _vp], ctypes.c_int),
    'pp_fields_from_conv': ([_vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp], ctypes.c_int),
    'pp_nms_keypoints': ([_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _sz, _vp],
                         ctypes.c_int),
    'pp_nms_keypoints_scored': ([_vp, _vp, _i32, _i32, _i32, _vp, _f64, _vp, _vp, _vp, _vp,
                                 _vp, _vp, _vp, _sz, _vp], ctypes.c_int),
    'pp_occupancy_set': ([_vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _f, _f, _vp],
                         ctypes.c_int),
    'pp_center_filter': ([_vp, _i64, _i64, _i64, _i32, _f, _f, _f, _vp, _i64, _vp, _vp],
                         ctypes.c_int),
    # host twins of the functional primitives (csrc/functional_cpu.hip): host pointers
    'pp_scalar_square_add_gauss_with_max_cpu': ([_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp,
                                                 _i64, _f, _f], ctypes.c_int),
    'pp_scalar_square_add_gauss_cpu': ([_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _f],
                                       ctypes.c_int),
    'pp_scalar_square_max_gauss_cpu': ([_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _f],
                                       ctypes.c_int),
    'pp_scalar_square_add_constant_cpu': ([_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64],
                                          ctypes.c_int),
    'pp_cumulative_average_cpu': ([_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _i64],
                                  ctypes.c_int),
    'pp_weiszfeld_nd_cpu': ([_vp, _i64, _i64, _i64, _vp, _vp, _f, _i64, _vp, _vp],
                            ctypes.c_int),
    'pp_scalar_values_cpu': ([_vp, _i64, _i64, _i64, _vp, _vp, _i64, _f, _vp], ctypes.c_int),
    'pp_scalar_lookup_cpu': ([_vp, _i64, _i64, _i64, _i32, _vp, _vp, _i64, _f, _f, _vp],
                             ctypes.c_int),
    'pp_occupancy_set_cpu': ([_vp, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _f, _f],
                             ctypes.c_int),
    'pp_center_filter_cpu': ([_vp, _i64, _i64, _i64, _i32, _f, _f, _f, _vp, _i64, _vp],
                             ctypes.c_int),
    'pp_np_exp_cpu': ([_vp, _vp, _i64, _i32], ctypes.c_int),
    'pp_np_square_cpu': ([_vp, _vp, _i64], ctypes.c_int),
    # host twins of the front stages (csrc/stages_cpu.hip)
    'pp_cifhr_cpu': ([_vp, _i32, _i32, _i32, _i32, _vp, _vp], ctypes.c_int),
    'pp_seeds_cpu': ([_vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _i32, _vp], ctypes.c_int),
    'pp_caf_scored_cpu': ([_vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _f, _vp, _vp, _vp],
                          ctypes.c_int),
    'pp_nms_keypoints_cpu': ([_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp], ctypes.c_int),
    'pp_nms_keypoints_scored_cpu': ([_vp, _vp, _i32, _i32, _i32, _vp, _f64, _vp, _vp, _vp, _vp,
                                     _vp, _vp], ctypes.c_int),
    # host twin of the whole decode (csrc/decode_cpu.hip)
    'pp_decode_batch_cpu': ([_vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _i32, _vp,
                             _vp, _i32], ctypes.c_int),
}

EXPORTED = tuple(_SIGNATURES)


class PPError(RuntimeError):
    pass


def load():
    """Load the library (raises if it is missing; never falls back to CPU)."""
    global _lib  # pylint: disable=global-statement
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise PPError('libpifpaf_amd.so not built ({}); run `python -m openpifpaf_amd.build`'
                          .format(LIB_PATH))
        lib = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        if lib.pp_version() != PP_ABI_VERSION:
            raise PPError('libpifpaf_amd ABI version mismatch')
        _lib = lib
        return lib


def check(rc, what=''):
    if rc != 0:
        msg = load().pp_last_error().decode(errors='replace')
        raise PPError('{} failed: {} ({})'.format(what, STATUS_NAMES.get(rc, rc), msg))
    return rc


def call(name, *args):
    return check(getattr(load(), name)(*args), name)
