"""Helpers to load the golden fixtures and compare decoder outputs against them."""
import glob
import hashlib
import json
import os

import numpy as np

from openpifpaf_amd import constants, synthetic
from openpifpaf_amd._abi import EVAL_CONFIG, PREDICT_CONFIG, make_config

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')

# Grow-stage comparison against the reference's own outputs (BASELINE.json north_star
# "within 1e-4"): EXACT.  The decoder restates the two places where the
# reference's float32 arithmetic is not IEEE-correct rounding (tests/test_np_exp.py): np.exp
# (NumPy's SIMD routine) and the scalar `sigma**2` (libm powf), cifcaf.py:139; with them
# every fixture matches bit for bit (x, y, v, joint scales, decoding_order copies).  Until
# round 5 the device's correctly rounded exp left up to 2 ulp (2.4e-4 at x ~ 1236).  The
# tolerances below stay as parameters of xy_close / compare_annotations: ulps and absolute
# deviations allowed, all zero, and the f64 score (records and Annotation.score()) exact.
XY_ULPS = 0
ATOL = 0.0
SCALE_RTOL = 0.0
SCORE_ATOL = 0.0


def ulp_distance(a, b):
    """Number of representable f32 values between a and b (elementwise; NaN == NaN -> 0)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)

    def ordered(x):
        i = x.view(np.int32).astype(np.int64)
        return np.where(i < 0, -(i & 0x7fffffff), i)

    d = np.abs(ordered(a) - ordered(b))
    return np.where(np.isnan(a) & np.isnan(b), 0, d)


def xy_close(got, ref):
    """(ok, max ulps) for keypoint coordinates: within ATOL absolute or XY_ULPS ulps."""
    got = np.asarray(got, np.float32)
    ref = np.asarray(ref, np.float32)
    u = ulp_distance(got, ref)
    ok = (u <= XY_ULPS) | (np.abs(got.astype(np.float64) - ref) <= ATOL)
    return bool(ok.all()), int(u.max(initial=0))


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


def confscale_config(g):
    """case_config plus an api_confscales fixture's CifCaf(confidence_scales=...)."""
    cfg = case_config(g)
    scales = [float(v) for v in g['confidence_scales']]
    out = make_config(**dict(EVAL_CONFIG if str(g['mode']) == 'eval' else PREDICT_CONFIG,
                             confidence_scales=scales))
    assert bytes(memoryview(out))[:-8] == bytes(memoryview(cfg))[:-8]  # only the weights differ
    return out


CONFSCALE_NAMES = ('p40_eval', 'u20_eval', 'dense_p80_eval')


def configure_decoder(dec, g):
    """Decoder class attributes of a fixture's mode (what decoder.configure() writes)."""
    mode = str(g['mode'])
    dec.CifHr.v_threshold = 0.1
    dec.CafScored.default_score_th = 0.1
    dec.CifSeeds.threshold = 0.2 if mode == 'eval' else 0.5
    dec.CifCaf.force_complete = mode == 'eval'
    dec.CifCaf.keypoint_threshold = 0.0 if mode == 'eval' else 0.001
    dec.CifCaf.greedy = bool(int(g['greedy']))
    dec.CifCaf.connection_method = str(g['connection_method'])
    dec.nms.Keypoints.instance_threshold = 0.0 if mode == 'eval' else 0.1
    dec.nms.Keypoints.keypoint_threshold = 0.0 if mode == 'eval' else 0.001


def annotations_as_records(anns, k=17):
    """Annotation objects -> pp_ann records (for compare_annotations / oracle checks)."""
    from openpifpaf_amd._abi import ANN_DTYPE
    recs = np.zeros(len(anns), ANN_DTYPE)
    for i, a in enumerate(anns):
        r = recs[i]
        r['data'][:k] = a.data
        r['joint_scales'][:k] = a.joint_scales
        r['score'] = a.score()
        r['n_keypoints'] = k
        r['n_decoding'] = len(a.decoding_order)
        for t, (js, jt, xa, xb) in enumerate(a.decoding_order):
            r['decoding_pairs'][t] = (js, jt)
            r['decoding_xyv'][t, :3] = xa
            r['decoding_xyv'][t, 3:] = xb
        r['n_frontier'] = len(a.frontier_order)
        for t, pair in enumerate(a.frontier_order):
            r['frontier_pairs'][t] = pair
    return recs


def seeds_as_rows(seeds):
    """pp_seed structured array -> (n, 5) float32 rows (v, f, x, y, s)."""
    if len(seeds) == 0:
        return np.zeros((0, 5), np.float32)
    return np.stack([seeds['v'], seeds['field'].astype(np.float32), seeds['x'], seeds['y'],
                     seeds['s']], axis=1).astype(np.float32)


def compare_annotations(g, recs, k=17, stats=None):
    """Compare pp_ann records with the golden annotation list.

    Connectivity (decoding_order / frontier_order pairs) must match exactly; x / y of the
    keypoints and of the decoding_order xyv copies within XY_ULPS; v and joint scales within
    ATOL; score within SCORE_ATOL.  Returns a list of human-readable mismatch strings
    (empty = parity); `stats` (a dict, optional) receives the largest deviations seen.
    """
    errs = []
    n = len(g['ann_score'])
    if stats is None:
        stats = {}
    stats.update(xy_ulps=0, v=0.0, scale=0.0, score=0.0)
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
        gdat = g['ann_data'][i]
        ok, u = xy_close(r['data'][:k, :2], gdat[:, :2])
        stats['xy_ulps'] = max(stats['xy_ulps'], u)
        if not ok:
            errs.append('ann %d x/y differ by %d ulp' % (i, u))
        dv = float(np.abs(r['data'][:k, 2] - gdat[:, 2]).max(initial=0))
        stats['v'] = max(stats['v'], dv)
        if not dv <= ATOL:
            errs.append('ann %d v max|d|=%g' % (i, dv))
        gs = g['ann_joint_scales'][i]
        ds = float(np.abs(r['joint_scales'][:k] - gs).max(initial=0))
        stats['scale'] = max(stats['scale'], ds)
        if not (np.abs(r['joint_scales'][:k] - gs) <= ATOL + SCALE_RTOL * np.abs(gs)).all():
            errs.append('ann %d joint_scales max|d|=%g' % (i, ds))
        if nd:
            gx = g['ann_decoding_xyv'][i][:nd].reshape(nd, 2, 3)
            rx = r['decoding_xyv'][:nd].reshape(nd, 2, 3)
            ok, u = xy_close(rx[:, :, :2], gx[:, :, :2])
            stats['xy_ulps'] = max(stats['xy_ulps'], u)
            if not ok or not np.abs(rx[:, :, 2] - gx[:, :, 2]).max() <= ATOL:
                errs.append('ann %d decoding_order xyv differ (%d ulp)' % (i, u))
        dsc = abs(float(r['score']) - float(g['ann_score'][i]))
        stats['score'] = max(stats['score'], dsc)
        if not dsc <= SCORE_ATOL:
            errs.append('ann %d score %r != %r' % (i, r['score'], g['ann_score'][i]))
    return errs


DENSE = constants.DENSE_DECODE_SKELETON


def load_api(name):
    """api_initial_<mode>.npz / api_stages.npz (gen_golden.gen_api)."""
    with np.load(os.path.join(GOLDEN, 'api_%s.npz' % name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def api_initial_inputs(g):
    """(cif, caf) of an api_initial fixture and its initial annotations as pp_ann records."""
    from openpifpaf_amd._abi import ANN_DTYPE
    cif, caf = synthetic.planted(40, 40, n_people=8, seed=5)
    assert sha(cif, caf) == str(g['input_sha']), 'synthetic generator drifted from the fixture'
    n = len(g['init_score'])
    recs = np.zeros(n, ANN_DTYPE)
    recs['data'][:, :17] = g['init_data']
    recs['joint_scales'][:, :17] = g['init_joint_scales']
    recs['n_keypoints'] = 17
    recs['n_decoding'] = g['init_n_decoding']
    recs['n_frontier'] = g['init_n_frontier']
    for i in range(n):
        nd, nf = int(g['init_n_decoding'][i]), int(g['init_n_frontier'][i])
        recs['decoding_pairs'][i, :nd] = g['init_decoding_pairs'][i, :nd]
        recs['decoding_xyv'][i, :nd] = g['init_decoding_xyv'][i, :nd]
        recs['frontier_pairs'][i, :nf] = g['init_frontier_pairs'][i, :nf]
    return cif, caf, recs


def api_initial_annotations(g):
    """The fixture's initial annotations as openpifpaf_amd Annotation objects."""
    from openpifpaf_amd.annotation import Annotation
    out = []
    for i in range(len(g['init_score'])):
        a = Annotation(constants.COCO_KEYPOINTS, constants.COCO_PERSON_SKELETON)
        a.data = g['init_data'][i].copy()
        a.joint_scales = g['init_joint_scales'][i].copy()
        nd, nf = int(g['init_n_decoding'][i]), int(g['init_n_frontier'][i])
        a.decoding_order = [(int(p[0]), int(p[1]), x[:3].copy(), x[3:].copy())
                            for p, x in zip(g['init_decoding_pairs'][i, :nd],
                                            g['init_decoding_xyv'][i, :nd])]
        a.frontier_order = [(int(p[0]), int(p[1])) for p in g['init_frontier_pairs'][i, :nf]]
        out.append(a)
    return out


def api_stage_heads(g):
    """The four heads of api_stages.npz: (cif8, caf8), then three stride-16 (cif, caf)."""
    heads = synthetic.planted_multi(321, 321, [8, 16, 16, 16], n_people=5, seed=21)
    assert sha(*[f for hd in heads for f in hd]) == str(g['input_sha'])
    return heads
