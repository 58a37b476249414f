"""Diagnostic: where the non-kernel time of a bench step goes (host launch, device time,
record fetch pieces).  python tools/host_timing.py [--generator planted|uniform]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import constants, synthetic  # noqa: E402
from openpifpaf_amd._abi import ANN_DTYPE, EVAL_CONFIG, make_config  # noqa: E402
from openpifpaf_amd.engine import DecodeEngine  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument('--generator', default='planted')
p.add_argument('--n', type=int, default=256)
args = p.parse_args()

cif, caf = synthetic.batch(args.generator, args.n, 80, 80)
c, f = torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda()
eng = DecodeEngine()
cfg = make_config(**EVAL_CONFIG)
sk = constants.COCO_PERSON_SKELETON
for _ in range(3):
    b = eng.launch(c, f, sk, cfg)
    eng.fetch(b)
torch.cuda.synchronize()

acc = np.zeros(7)
reps = 20
for _ in range(reps):
    t0 = time.perf_counter()
    b = eng.launch(c, f, sk, cfg)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    counts = b.counts.cpu().numpy().astype(np.int64)
    t3 = time.perf_counter()
    offs = np.concatenate([[0], np.cumsum(counts)])
    idx = np.arange(offs[-1], dtype=np.int64) + np.repeat(
        np.arange(len(counts), dtype=np.int64) * b.cap - offs[:-1], counts)
    rows = b.anns.view(b.n * b.cap, ANN_DTYPE.itemsize)
    sel = rows.index_select(0, torch.from_numpy(idx).to(rows.device))
    t4 = time.perf_counter()
    host = torch.empty(sel.shape, dtype=torch.uint8, pin_memory=True)
    t5 = time.perf_counter()
    host.copy_(sel, non_blocking=True)
    torch.cuda.current_stream().synchronize()
    t6 = time.perf_counter()
    _ = host.numpy().reshape(-1).view(ANN_DTYPE)
    t7 = time.perf_counter()
    acc += np.diff([t0, t1, t2, t3, t4, t5, t6, t7])
names = ['launch (host)', 'device wait', 'counts D2H', 'idx + index_select', 'pinned alloc',
         'records D2H', 'view']
for n_, v in zip(names, acc / reps * 1e3):
    print('{:22s} {:8.3f} ms'.format(n_, v))
print('records per step', int(counts.sum()), 'bytes', int(counts.sum()) * ANN_DTYPE.itemsize)
