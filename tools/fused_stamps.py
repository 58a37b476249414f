"""Diagnostic: per-workgroup phases of the decoder's cifhr_fused_kernel<true> (stamps build).

    PP_LIB_VARIANT=stamps PP_HR_STAMPS_OUT=gpurun_out/fused.bin python tools/fused_stamps.py \
        [kind:n ...]   (default planted:256)

One workgroup per (image, field): phase 1 (list + seed candidates), phase 2 (fold of the
touched tiles), phase 3 (seeds from the map).  Times in us (s_memrealtime, 100 MHz).
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import constants, synthetic  # noqa: E402
from openpifpaf_amd._abi import EVAL_CONFIG, make_config  # noqa: E402
from openpifpaf_amd.engine import STAGE_CIFHR, STAGE_SEEDS, DecodeEngine  # noqa: E402

KHRST = 12
out = os.environ.get('PP_HR_STAMPS_OUT', 'pp_hr_stamps.bin')
cases = [(c.split(':')[0], int(c.split(':')[1])) for c in sys.argv[1:]] or [('planted', 256)]
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
    st = np.fromfile(out, dtype=np.uint64).reshape(-1, KHRST).astype(np.int64)
    t0 = st[:, 0].min()
    s0, s1, s2, s3 = (st[:, q] - t0 for q in range(4))
    print('== {} n={} workgroups={} (us)'.format(kind, n, len(st)))
    print('  kernel span {:.1f}  list mean {:.0f}  seed candidates mean {:.0f}'.format(
        s3.max() / 100, st[:, 8].mean(), st[:, 9].mean()))
    for name, v in (('lifetime', s3 - s0), ('phase1', s1 - s0), ('phase2', s2 - s1),
                    ('phase3', s3 - s2), ('start', s0)):
        q = np.percentile(v, [10, 50, 90, 99]) / 100
        print('  {:10s} mean {:7.2f}  p10 {:7.2f} p50 {:7.2f} p90 {:7.2f} p99 {:7.2f}'.format(
            name, v.mean() / 100, *q))
    ts = np.linspace(0, s3.max(), 12)[1:-1]
    alive = [int(((s0 <= t) & (s3 > t)).sum()) for t in ts]
    print('  workgroups alive over the span:', alive)
