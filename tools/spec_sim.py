"""Diagnostic (CPU, build container): how many of the seed loop's first speculative picks
are seeds the loop really commits, for the plan rule of seed_loop_kernel's spec_plan at
kernel start (wave 0 grows seed 0, the 7 helpers take the first free seeds of the next
kSpecScan = 128 that lie kSpecFar = 4 joint scales from every seed in flight).  The
committed seeds come from the oracle's decode (force-complete and NMS off: the annotations
in seed order), matched to the sorted seed list by (field, x, y, v); planted seeds of one
joint patch share x and y.  'fldR' variants keep seeds of other fields R joint scales away.

    python tools/spec_sim.py [n_images]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'oracle'))
import oracle  # noqa: E402
from openpifpaf_amd import constants, synthetic  # noqa: E402
from openpifpaf_amd._abi import EVAL_CONFIG, make_config  # noqa: E402

kw = dict(EVAL_CONFIG)
kw.update(force_complete=0, apply_nms=0)
cfg = make_config(**kw)
sk = constants.COCO_PERSON_SKELETON
N = int(sys.argv[1]) if len(sys.argv) > 1 else 24
cif, caf = synthetic.batch('planted', N, 80, 80)
res = {}
for i in range(N):
    hr = oracle.cifhr(cif[i], cfg)
    sd = oracle.seeds(cif[i], hr, cfg)
    order = sorted(range(len(sd)), key=lambda j: (float(sd['v'][j]), int(sd['field'][j]),
                                                  float(sd['x'][j]), float(sd['y'][j]),
                                                  float(sd['s'][j])), reverse=True)
    sd = sd[np.array(order)]
    recs = oracle.decode(cif[i], caf[i], sk, cfg)
    key = {}
    for j, (f, x, y, v) in enumerate(zip(sd['field'], sd['x'], sd['y'], sd['v'])):
        key.setdefault((int(f), float(x), float(y), float(v)), j)
    committed = []
    for r in recs:
        nd = r['n_decoding']
        f = int(r['decoding_pairs'][0][0]) if nd > 0 else int(np.nonzero(r['data'][:17, 2])[0][0])
        committed.append(key[(f, float(r['data'][f][0]), float(r['data'][f][1]),
                              float(r['data'][f][2]))])
    committed.sort()
    cset = set(committed)
    if i < 4:
        print('image', i, 'seeds', len(sd), 'committed seed indices', committed)

    def far(a, b, k):
        r = k * max(sd['s'][a], sd['s'][b], 1.0)
        return abs(sd['x'][a] - sd['x'][b]) > r or abs(sd['y'][a] - sd['y'][b]) > r

    for name, R in (('far4', None), ('fld6', 6), ('fld8', 8), ('fld12', 12)):
        fly, picks = [committed[0]], []
        for c in range(committed[0] + 1, min(len(sd), committed[0] + 1 + 128)):
            ok = True
            for q in fly:
                ok = ok and far(c, q, 4.0 if R is None or sd['field'][c] == sd['field'][q] else R)
            if ok:
                picks.append(c)
                fly.append(c)
            if len(picks) == 7:
                break
        res.setdefault(name, []).append((sum(1 for p in picks if p in cset), len(picks),
                                         len(committed)))
for name, v in res.items():
    v = np.array(v)
    print('{:6s} first picks useful / made {:.2f} / {:.2f}, committed per image {:.2f}'.format(
        name, *v.mean(axis=0)))
