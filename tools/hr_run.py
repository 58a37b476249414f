"""Run one CifHr entry point alone on a resident batch, for rocprofv3 counter passes:
python tools/hr_run.py [planted|uniform] [n] [sparse|dense]
sparse = the decoder's pp_cifhr_sparse, dense = pp_cifhr (CifHr.accumulated)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import synthetic  # noqa: E402
from openpifpaf_amd.decoder.cif_hr import cifhr_device, cifhr_sparse_device  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else 'planted'
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
which = sys.argv[3] if len(sys.argv) > 3 else 'sparse'
cif, _ = synthetic.batch(kind, n, 80, 80)
c = torch.from_numpy(cif).cuda()
fn = cifhr_sparse_device if which == 'sparse' else cifhr_device
for _ in range(3):
    fn(c, 8, 0.1, 16)
torch.cuda.synchronize()
print('ok')
