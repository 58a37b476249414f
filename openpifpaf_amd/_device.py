"""Device-memory plumbing (torch owns HIP memory and streams; the kernels are ours)."""
import ctypes

import numpy as np
import torch

from ._lib import PPError


def require():
    if not torch.cuda.is_available():
        raise PPError('openpifpaf_amd needs a HIP device (MI355X); none is visible')
    return torch.device('cuda', torch.cuda.current_device())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    if t is None:
        return ctypes.c_void_p(0)
    return ctypes.c_void_p(t.data_ptr())


def is_device(a):
    return isinstance(a, torch.Tensor) and a.is_cuda


def to_device(a, dtype=torch.float32):
    """Contiguous device tensor of `dtype` (copies host arrays; no-op for suitable tensors)."""
    dev = require()
    if isinstance(a, torch.Tensor):
        return a.to(device=dev, dtype=dtype).contiguous()
    np_dtype = {torch.float32: np.float32, torch.uint8: np.uint8, torch.int32: np.int32}[dtype]
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np_dtype)).to(dev)
