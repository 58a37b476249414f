"""Time the CifHr entry points on a resident batch with HIP events: the dense map of the
reference API (pp_cifhr, CifHr.accumulated) and the decoder's block-sparse map
(pp_cifhr_sparse).  python tools/hr_time.py [planted|uniform] [n]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import synthetic  # noqa: E402
from openpifpaf_amd.decoder.cif_hr import cifhr_device, cifhr_sparse_device  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else 'planted'
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
cif, _ = synthetic.batch(kind, n, 80, 80)
c = torch.from_numpy(cif).cuda()
k, h, w = cif.shape[1], cif.shape[3], cif.shape[4]
hh = (h - 1) * 8 + 1
alg = 4 * n * k * (5 * h * w + hh * hh)
for name, fn in (('dense pp_cifhr', lambda: cifhr_device(c, 8, 0.1, 16)),
                 ('sparse pp_cifhr_sparse', lambda: cifhr_sparse_device(c, 8, 0.1, 16))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print('{:24s} {:8.3f} ms  dense-equivalent {:7.1f} GB/s'.format(name, ms, alg / ms / 1e6))
