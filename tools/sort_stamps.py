"""Diagnostic: per-phase cycles of seeds_sort_kernel (stamps build).

    PP_LIB_VARIANT=stamps PP_SORT_STAMPS_OUT=gpurun_out/sort.bin python tools/sort_stamps.py \
        [kind:n ...]   (default planted:1 planted:256)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import constants, synthetic  # noqa: E402
from openpifpaf_amd._abi import EVAL_CONFIG, make_config  # noqa: E402
from openpifpaf_amd.engine import STAGE_CIFHR, STAGE_SEEDS, DecodeEngine  # noqa: E402

out = os.environ.get('PP_SORT_STAMPS_OUT', 'pp_sort_stamps.bin')
cases = [(c.split(':')[0], int(c.split(':')[1])) for c in sys.argv[1:]] or [('planted', 1),
                                                                           ('planted', 256)]
for kind, n in cases:
    cif, caf = synthetic.batch(kind, n, 80, 80)
    c, f = torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda()
    eng = DecodeEngine()
    cfg = make_config(**EVAL_CONFIG)
    sk = constants.COCO_PERSON_SKELETON
    for _ in range(3):
        if os.path.exists(out):
            os.remove(out)
        eng.launch(c, f, sk, cfg, stages=STAGE_CIFHR | STAGE_SEEDS)
        torch.cuda.synchronize()
    st = np.fromfile(out, dtype=np.uint64).reshape(-1, 6).astype(np.int64)
    d = np.diff(st[:, :5], axis=1)
    print('== {} n={} (shader cycles, mean over images; keys mean {:.0f})'.format(kind, n, st[:, 5].mean()))
    for name, col in zip(('offsets', 'load keys', 'bitonic', 'finish'), d.T):
        print('  {:10s} {:9.0f}'.format(name, col.mean()))
    print('  total      {:9.0f}'.format((st[:, 4] - st[:, 0]).mean()))
