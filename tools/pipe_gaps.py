"""Diagnostic: where the overlapped pipeline's step time goes (DecodePipeline, the bench's
3 steps in flight), from HIP events on the three streams: per step the front half
(CifHr + seeds + CafScored, current stream), the seed loop (back stream), the tail
(force-complete + NMS, tail stream), the back stream's idle gap before each seed loop, and
which dependency the seed loop waited for last: its own front half, or the NMS of the
batch that last used its workspace (two steps back).

    python tools/pipe_gaps.py [--generator planted] [--steps 40]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import constants, synthetic  # noqa: E402
from openpifpaf_amd._abi import EVAL_CONFIG, PACK_ALL, make_config  # noqa: E402
from openpifpaf_amd.engine import DecodePipeline  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument('--generator', default='planted')
p.add_argument('--n', type=int, default=256)
p.add_argument('--steps', type=int, default=40)
p.add_argument('--pipe-depth', type=int, default=2, help='workspaces in flight')
p.add_argument('--host-depth', type=int, default=3, help='steps in flight on the host')
args = p.parse_args()

kw = {'n_caf': 19} if args.generator == 'uniform' else {}
cif, caf = synthetic.batch(args.generator, args.n, 80, 80, **kw)
c, f = torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda()
cfg = make_config(**EVAL_CONFIG)
sk = constants.COCO_PERSON_SKELETON
compact = (17, len(sk), PACK_ALL)
pipe = DecodePipeline(depth=args.pipe_depth)
for _ in range(3):
    pipe.submit(c, f, sk, cfg, compact=compact)[1].result()
evs = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(args.steps)]
inflight = []
torch.cuda.synchronize()
for k in range(args.steps):
    inflight.append(pipe.submit(c, f, sk, cfg, compact=compact, events=evs[k])[1])
    if len(inflight) >= args.host_depth:
        inflight.pop(0).result()
while inflight:
    inflight.pop(0).result()
torch.cuda.synchronize()
e0 = evs[0][0]
t = np.array([[e0.elapsed_time(e) for e in ev] for ev in evs])  # ms since step 0's front start
# columns: 0 front start, 1 CifHr end, 2 front end, 3 loop start, 4 NMS end, 5 loop end
rows = []
for k in range(4, args.steps):
    gap = t[k, 3] - t[k - 1, 5]
    dep_front = t[k, 2]
    dep_nms = t[k - args.pipe_depth, 4]
    rows.append((t[k, 3] - t[k - 1, 3], t[k, 2] - t[k, 0], t[k, 5] - t[k, 3],
                 t[k, 4] - t[k, 5], gap, 1e3 * (t[k, 3] - max(dep_front, dep_nms, t[k - 1, 5])),
                 'front' if dep_front >= max(dep_nms, t[k - 1, 5]) else
                 'nms(k-2)' if dep_nms >= t[k - 1, 5] else 'loop(k-1)',
                 t[k, 0] - t[k - 1, 0]))
print('{} n={} workspaces {} host depth {}: mean step (loop start to loop start) {:.3f} ms'.format(
    args.generator, args.n, args.pipe_depth, args.host_depth, np.mean([r[0] for r in rows])))
names = ('step', 'front', 'loop', 'tail after loop', 'back idle before loop')
for i, nm in enumerate(names):
    v = np.array([r[i] for r in rows])
    print('  {:24s} mean {:.3f}  p50 {:.3f}  min {:.3f}  max {:.3f} ms'.format(
        nm, v.mean(), np.median(v), v.min(), v.max()))
lag = np.array([r[5] for r in rows])
print('  loop start after its last dependency: mean {:.1f} us'.format(lag.mean()))
from collections import Counter  # noqa: E402
print('  last dependency of the seed loop:', dict(Counter(r[6] for r in rows)))
print('  front-start spacing mean {:.3f} ms'.format(np.mean([r[7] for r in rows])))
for r in rows[:12]:
    print('   step {:.3f} front {:.3f} loop {:.3f} tail {:.3f} idle {:.3f} lag {:5.1f}us last={}'.format(*r[:7]))
