"""Helpers to load the golden fixtures and compare decoder outputs against them."""
import glob
import hashlib
import json
import os

import numpy as np

from openpifpaf_amd import constants, synthetic
from openpifpaf_amd._abi import EVAL_CONFIG, PREDICT_CONFIG, make_config

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')

# keypoint (x, y, v) and joint-scale tolerance: BASELINE.json north_star "within 1e-4"
# (absolute), plus 1e-5 relative: hi-res pixel coordinates reach 1273 px where one f32 ulp is
# 1.2e-4, and the reference's SIMD np.exp differs from a correctly rounded exp by up to
# 2 ulp, which the blend propagates by a few ulp.
ATOL = 1e-4
RTOL = 1e-5


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def case_names():
    return sorted(os.path.basename(p)[len('decode_'):-len('.npz')]
                  for p in glob.glob(os.path.join(GOLDEN, 'decode_*.npz')))


def load_case(name):
    with np.load(os.path.join(GOLDEN, 'decode_%s.npz' % name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def load_primitives():
    with np.load(os.path.join(GOLDEN, 'primitives.npz'), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def load_errors():
    with open(os.path.join(GOLDEN, 'errors.json')) as fh:
        return json.load(fh)


def case_inputs(g):
    gen = str(g['generator'])
    h, w, seed = int(g['H']), int(g['W']), int(g['seed'])
    skeleton = [tuple(int(t) for t in e) for e in g['skeleton']]
    if gen == 'zero':
        cif = np.zeros((17, 5, h, w), np.float32)
        caf = np.zeros((len(skeleton), 9, h, w), np.float32)
    elif gen == 'uniform':
        cif, caf = synthetic.uniform(h, w, n_caf=len(skeleton), seed=seed)
    else:
        cif, caf = synthetic.planted(h, w, n_people=int(g['n_people']), seed=seed,
                                     skeleton=skeleton)
    assert sha(cif, caf) == str(g['input_sha']), 'synthetic generator drifted from the fixture'
    return cif, caf, skeleton


def case_config(g):
    mode = str(g['mode'])
    kw = dict(EVAL_CONFIG if mode == 'eval' else PREDICT_CONFIG)
    kw['connection_method'] = str(g['connection_method'])
    kw['greedy'] = bool(int(g['greedy']))
    return make_config(**kw)


def seeds_as_rows(seeds):
    """pp_seed structured array -> (n, 5) float32 rows (v, f, x, y, s)."""
    if len(seeds) == 0:
        return np.zeros((0, 5), np.float32)
    return np.stack([seeds['v'], seeds['field'].astype(np.float32), seeds['x'], seeds['y'],
                     seeds['s']], axis=1).astype(np.float32)


def compare_annotations(g, recs, k=17):
    """Compare pp_ann records with the golden annotation list.

    Connectivity (decoding_order / frontier_order pairs) must match exactly; (x, y, v),
    joint scales and the decoding_order xyv copies within ATOL/RTOL; score to 1e-6.
    Returns a list of human-readable mismatch strings (empty = parity).
    """
    errs = []
    n = len(g['ann_score'])
    if len(recs) != n:
        return ['annotation count %d != golden %d' % (len(recs), n)]
    for i in range(n):
        r = recs[i]
        gd = g['ann_decoding_pairs'][i]
        nd = int((gd[:, 0] >= 0).sum())
        if int(r['n_decoding']) != nd or not np.array_equal(
                r['decoding_pairs'][:nd].astype(np.int16), gd[:nd]):
            errs.append('ann %d decoding_order differs' % i)
        gf = g['ann_frontier_pairs'][i]
        nf = int((gf[:, 0] >= 0).sum())
        if int(r['n_frontier']) != nf or not np.array_equal(
                r['frontier_pairs'][:nf].astype(np.int16), gf[:nf]):
            errs.append('ann %d frontier_order differs' % i)
        if not np.allclose(r['data'][:k], g['ann_data'][i], atol=ATOL, rtol=RTOL):
            errs.append('ann %d data max|d|=%g' % (
                i, np.abs(r['data'][:k] - g['ann_data'][i]).max()))
        if not np.allclose(r['joint_scales'][:k], g['ann_joint_scales'][i], atol=ATOL, rtol=RTOL):
            errs.append('ann %d joint_scales differ' % i)
        if nd and not np.allclose(r['decoding_xyv'][:nd], g['ann_decoding_xyv'][i][:nd],
                                  atol=ATOL, rtol=RTOL):
            errs.append('ann %d decoding_order xyv differ' % i)
        if not np.isclose(r['score'], g['ann_score'][i], rtol=RTOL, atol=1e-9):
            errs.append('ann %d score %r != %r' % (i, r['score'], g['ann_score'][i]))
    return errs


DENSE = constants.DENSE_DECODE_SKELETON
