"""Diagnostic: per-workgroup timeline of cifhr_sparse_kernel (stamps build).

    PP_LIB_VARIANT=stamps PP_HR_STAMPS_OUT=gpurun_out/hr_stamps.bin python tools/hr_stamps.py \
        [kind:n ...]   (default planted:256 uniform:64)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import synthetic  # noqa: E402
from openpifpaf_amd.decoder.cif_hr import cifhr_sparse_device  # noqa: E402

out = os.environ.get('PP_HR_STAMPS_OUT', 'pp_hr_stamps.bin')
cases = [(c.split(':')[0], int(c.split(':')[1])) for c in sys.argv[1:]] or [('planted', 256),
                                                                           ('uniform', 64)]
for kind, n in cases:
    if os.path.exists(out):
        os.remove(out)
    cif, _ = synthetic.batch(kind, n, 80, 80)
    c = torch.from_numpy(cif).cuda()
    for _ in range(3):
        cifhr_sparse_device(c, 8, 0.1, 16)
    torch.cuda.synchronize()
    st = np.fromfile(out, dtype=np.uint64).reshape(3, -1, 12)[-1].astype(np.int64)
    t0 = st[:, 0].min()
    start, p1, ends = st[:, 0] - t0, st[:, 1] - t0, st[:, 2:6] - t0
    end = ends.max(axis=1)
    life = end - start
    print('== {} n={} fields={} (times in us, 100 MHz ticks)'.format(kind, n, len(st)))
    print('  kernel span {:.1f}'.format(end.max() / 100))
    for name, v in (('lifetime', life), ('phase1', p1 - start), ('phase2', end - p1),
                    ('wave spread', ends.max(axis=1) - ends.min(axis=1))):
        q = np.percentile(v, [10, 50, 90, 99]) / 100
        print('  {:12s} mean {:7.2f}  p10 {:7.2f} p50 {:7.2f} p90 {:7.2f} p99 {:7.2f}'.format(
            name, v.mean() / 100, *q))
    # concurrency: workgroups alive over time
    ts = np.linspace(0, end.max(), 20)
    alive = [int(((start <= t) & (end > t)).sum()) for t in ts]
    print('  alive over time:', alive)
    hw = st[:, 6]
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    xcc = st[:, 7] & 0xF
    print('  distinct (xcc, se, cu):', len(set(zip(xcc.tolist(), se.tolist(), cu.tolist()))))
    print('  splats per field mean {:.1f} max {}'.format(st[:, 8].mean(), st[:, 8].max()))
    u = np.maximum(st[:, 11], 1)
    print('  wave 0: units mean {:.2f} max {}; per unit shader cycles: staging {:.0f}, fold {:.0f}'
          .format(st[:, 11].mean(), st[:, 11].max(), (st[:, 9] / u).mean(), (st[:, 10] / u).mean()))
    print('  wave 0 cycles per workgroup: staging {:.0f} fold {:.0f} (p90 {:.0f} / {:.0f})'.format(
        st[:, 9].mean(), st[:, 10].mean(), np.percentile(st[:, 9], 90), np.percentile(st[:, 10], 90)))
    order = np.argsort(start)
    print('  start of wg 0/1000/2000/3000/last: ',
          [round(start[order[i]] / 100, 1) for i in (0, 1000, 2000, 3000, len(st) - 1)
           if i < len(st)])
