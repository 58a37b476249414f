"""Diagnostic: host time of the bench's overlapped loop (DecodePipeline, 3 steps in flight):
per step, the host time inside submit(), the time blocked waiting for the records, and
the host time of the rest of result().  If submit + result approach the step time, the
host, not the device, sets the pace.

    python tools/host_pipe.py [--generator planted] [--steps 60]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import constants, synthetic  # noqa: E402
from openpifpaf_amd._abi import EVAL_CONFIG, PACK_ALL, make_config  # noqa: E402
from openpifpaf_amd.engine import DecodePipeline  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument('--generator', default='planted')
p.add_argument('--n', type=int, default=256)
p.add_argument('--steps', type=int, default=60)
p.add_argument('--depth', type=int, default=3, help='steps in flight on the host')
args = p.parse_args()

cif, caf = synthetic.batch(args.generator, args.n, 80, 80)
c, f = torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda()
cfg = make_config(**EVAL_CONFIG)
sk = constants.COCO_PERSON_SKELETON
compact = (17, len(sk), PACK_ALL)
pipe = DecodePipeline()
for _ in range(3):
    pipe.submit(c, f, sk, cfg, compact=compact)[1].result()
warm = []  # then 3 in flight, as timed (the pinned record blocks get allocated here)
for _ in range(5):
    warm.append(pipe.submit(c, f, sk, cfg, compact=compact)[1])
    if len(warm) >= 3:
        warm.pop(0).result()
while warm:
    warm.pop(0).result()
torch.cuda.synchronize()


# host time inside the library calls and the record-pack setup, per step
from openpifpaf_amd import engine as _engine  # noqa: E402
acc = {}


def _timed(name, fn):
    def w(*a, **k):
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc.setdefault(name, []).append(time.perf_counter() - t)
    return w


_engine.call = _timed('library calls', _engine.call)
_engine.DecodeEngine._pack = staticmethod(_timed('_pack (incl. its library call)',
                                                 _engine.DecodeEngine._pack))
_orig_empty = torch.empty
torch.empty = _timed('torch.empty', _orig_empty)

t_sub, t_wait, t_res = [], [], []
inflight = []
t0 = time.perf_counter()
for k in range(args.steps):
    a = time.perf_counter()
    inflight.append(pipe.submit(c, f, sk, cfg, compact=compact)[1])
    t_sub.append(time.perf_counter() - a)
    if len(inflight) >= args.depth:
        q = inflight.pop(0)
        a = time.perf_counter()
        q.wait()
        b = time.perf_counter()
        q.result()
        t_wait.append(b - a)
        t_res.append(time.perf_counter() - b)
while inflight:
    inflight.pop(0).result()
torch.cuda.synchronize()
total = time.perf_counter() - t0
print('{} n={} depth={}: {:.3f} ms per step'.format(args.generator, args.n, args.depth,
                                                    1e3 * total / args.steps))
for name, v in (('submit (host)', t_sub), ('blocked on records', t_wait),
                ('result after wait (host)', t_res)):
    v = 1e3 * np.array(v)
    print('  {:26s} mean {:.3f}  p50 {:.3f}  p90 {:.3f} ms'.format(name, v.mean(),
                                                                 np.median(v),
                                                                 np.percentile(v, 90)))
for name, v in acc.items():
    v = 1e3 * np.array(v)
    print('  {:30s} per step {:.3f} ms  (calls {}, max {:.3f} ms)'.format(
        name, v.sum() / args.steps, len(v), v.max()))
