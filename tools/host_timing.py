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

acc = np.zeros(5)
reps = 20
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
pack_ms = 0.0
for _ in range(reps):
    t0 = time.perf_counter()
    ev[0].record()
    b = eng.launch(c, f, sk, cfg)
    ev[1].record()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    recs, offs = eng.fetch(b)  # pp_pack_records into pinned memory + one sync
    ev[2].record()
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    pack_ms += ev[1].elapsed_time(ev[2])
    t4 = time.perf_counter()
    recs = None
    b = eng.launch(c, f, sk, cfg)
    t5 = time.perf_counter()  # one full bench-like step: launch .. fetch
    eng.fetch(b)
    t6 = time.perf_counter()
    acc += np.array([t1 - t0, t2 - t1, t3 - t2, t5 - t4, (t6 - t4)])
names = ['launch (host)', 'device wait', 'fetch (pack + sync)', 'launch again', 'step']
for n_, v in zip(names, acc / reps * 1e3):
    print('{:22s} {:8.3f} ms'.format(n_, v))
print('pack kernel (events)   {:8.3f} ms'.format(pack_ms / reps))
print('records per step', len(offs) and int(offs[-1]), 'bytes', int(offs[-1]) * ANN_DTYPE.itemsize)
