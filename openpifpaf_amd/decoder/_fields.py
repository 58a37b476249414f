"""Shared plumbing of the single-image stage classes: field tensors and the pitched
high-resolution CIF layout (n, K, H', pitch) the kernels use."""
import ctypes

import torch

from .. import _device
from .._lib import load


def hr_geometry(h, w, stride):
    hh = (h - 1) * stride + 1
    ww = (w - 1) * stride + 1
    return hh, ww, int(load().pp_cifhr_pitch(ww))


def batch1(field):
    """(1, ...) contiguous float32 device tensor of one image's field."""
    return _device.to_device(field)[None]


def pitched_hr(cifhr, stride_unused=None):
    """CifHr map as a (1, K, H', pitch) device tensor.  Views of a decoder-made map are
    used in place; other arrays are copied into a fresh pitched buffer."""
    k, hh, ww = cifhr.shape
    pitch = int(load().pp_cifhr_pitch(ww))
    if (_device.is_device(cifhr) and cifhr.dtype == torch.float32
            and tuple(cifhr.stride()) == (hh * pitch, pitch, 1)):
        base = cifhr.storage_offset()
        if cifhr.untyped_storage().nbytes() >= 4 * (base + k * hh * pitch):
            return torch.as_strided(cifhr, (1, k, hh, pitch), (k * hh * pitch, hh * pitch, pitch, 1))
    dev = _device.require()
    out = torch.zeros((1, k, hh, pitch), dtype=torch.float32, device=dev)
    out[0, :, :, :ww] = _device.to_device(cifhr)
    return out


def cfg_ptr(cfg):
    return ctypes.byref(cfg)


def head_scales(fields, config, role):
    """pp_scale list of a FieldConfig's heads for one image: (array, the batch-1 device
    tensors it points into).  role 'cif' lists the CIF heads; 'caf' the CAF heads after the
    CIF heads' shapes (CIF head 0 gives the CifHr geometry; their fields are not read)."""
    from .._abi import scale_list  # pylint: disable=import-outside-toplevel
    if role == 'cif':
        ts = [batch1(fields[i]) for i in config.cif_indices]
        arr = scale_list([(t.data_ptr(), t.shape[3], t.shape[4]) for t in ts], [],
                         config.cif_strides, [], config.cif_min_scales)
        return arr, ts
    ts = [batch1(fields[i]) for i in config.caf_indices]
    geo = [(None, fields[i].shape[-2], fields[i].shape[-1]) for i in config.cif_indices]
    arr = scale_list(geo, [(t.data_ptr(), t.shape[3], t.shape[4]) for t in ts],
                     config.cif_strides, config.caf_strides, None, config.caf_min_distances,
                     config.caf_max_distances)
    return arr, ts


def geometry_entry(hr_shape):
    """pp_scale entry (PP_ROLE_HRMAP) naming a CifHr map of hr_shape[-2:] = (hh, ww): the
    stage entry points then read / write a map made at another head's size."""
    from .._abi import ROLE_HRMAP, Scale  # pylint: disable=import-outside-toplevel
    return Scale(None, None, int(hr_shape[-2]), int(hr_shape[-1]), 1, 0.0, 0.0, 0.0, ROLE_HRMAP)


def with_geometry(arr, hr_shape):
    """A pp_scale array followed by the geometry entry of hr_shape."""
    from .._abi import Scale  # pylint: disable=import-outside-toplevel
    return (Scale * (len(arr) + 1))(*arr, geometry_entry(hr_shape))
