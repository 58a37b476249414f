"""HIP path vs the reference (golden fixtures) and vs the oracle, on an MI355X.

Bit-exact: CifHr maps, seed lists, CafScored column sets, every functional primitive, and
(round 6) the decoded annotations against the reference's own outputs too: golden_util's
tolerances are zero since the decoder restates np.exp and the scalar `sigma**2` as NumPy
computes them (tests/test_np_exp.py).  Against the oracle the device decode matches byte
for byte.
"""
import os

import numpy as np
import pytest

import golden_util as gu
import oracle

pytestmark = pytest.mark.gpu

CASES = gu.case_names()


@pytest.fixture(scope='module')
def F():
    from openpifpaf_amd import functional
    return functional


@pytest.fixture(scope='module')
def dec():
    from openpifpaf_amd import decoder
    return decoder


@pytest.fixture(scope='module')
def prim():
    return gu.load_primitives()


def _pts(p, key):
    return [np.ascontiguousarray(r) for r in p[key]]


# ---- functional primitives -------------------------------------------------------------

@pytest.mark.parametrize('t', range(4))
def test_add_gauss_with_max(F, prim, t):
    field = prim['sqg_max_%d_in' % t].copy()
    trunc, maxv = prim['sqg_max_%d_args' % t]
    F.scalar_square_add_gauss_with_max(field, *_pts(prim, 'sqg_max_%d_pts' % t),
                                       truncate=trunc, max_value=maxv)
    assert np.array_equal(field, prim['sqg_max_%d_out' % t])


def test_add_gauss_with_max_strided_and_empty(F, prim):
    big = prim['sqg_max_strided_in'].copy()
    F.scalar_square_add_gauss_with_max(big[::2, 1::2], *_pts(prim, 'sqg_max_strided_pts'),
                                       truncate=1.0)
    assert np.array_equal(big, prim['sqg_max_strided_out'])
    field = prim['sqg_max_empty_in'].copy()
    e = np.zeros(0, np.float32)
    F.scalar_square_add_gauss_with_max(field, e, e, e, e)
    assert np.array_equal(field, prim['sqg_max_empty_out'])


@pytest.mark.parametrize('t', range(2))
def test_add_gauss(F, prim, t):
    field = prim['sqg_%d_in' % t].copy()
    F.scalar_square_add_gauss(field, *_pts(prim, 'sqg_%d_pts' % t),
                              truncate=prim['sqg_%d_args' % t][0])
    assert np.array_equal(field, prim['sqg_%d_out' % t])


@pytest.mark.parametrize('t', range(2))
def test_max_gauss(F, prim, t):
    field = prim['sqmax_%d_in' % t].copy()
    F.scalar_square_max_gauss(field, *_pts(prim, 'sqmax_%d_pts' % t),
                              truncate=prim['sqmax_%d_args' % t][0])
    assert np.array_equal(field, prim['sqmax_%d_out' % t])


def test_add_constant(F, prim):
    field = prim['sqc_in'].copy()
    F.scalar_square_add_constant(field, *_pts(prim, 'sqc_pts'))
    assert np.array_equal(field, prim['sqc_out'])


def test_cumulative_average(F, prim):
    cuma, cumw = [a.copy() for a in prim['cuma_in']]
    F.cumulative_average(cuma, cumw, *_pts(prim, 'cuma_pts'))
    assert np.array_equal(np.stack([cuma, cumw]), prim['cuma_out'])


@pytest.mark.parametrize('t', range(3))
def test_weiszfeld(F, prim, t):
    y = prim['weisz_%d_y0' % t].copy()
    _, denom = F.weiszfeld_nd(prim['weisz_%d_x' % t].copy(), y, weights=prim['weisz_%d_w' % t].copy())
    assert np.array_equal(y, prim['weisz_%d_y' % t])
    assert np.array_equal(denom, prim['weisz_%d_denom' % t])


def test_lookups(F, prim):
    f = prim['lookup_field'].copy()
    px, py = [a.copy() for a in prim['lookup_pts']]
    assert np.array_equal(F.scalar_values(f, px, py), prim['scalar_values'])
    assert np.array_equal(F.scalar_values(f, px, py, default=0.0), prim['scalar_values_d0'])
    got = np.array([F.scalar_value(f, a, b) for a, b in zip(px, py)], np.float32)
    assert np.array_equal(got, prim['scalar_value'])
    got = np.array([F.scalar_value_clipped(f, a, b) for a, b in zip(px, py)], np.float32)
    assert np.array_equal(got, prim['scalar_value_clipped'])
    occ = prim['lookup_occ'].copy()
    got = np.array([F.scalar_nonzero(occ, a, b) for a, b in zip(px, py)], np.uint8)
    assert np.array_equal(got, prim['scalar_nonzero'])
    got = np.array([F.scalar_nonzero_clipped(occ, a, b) for a, b in zip(px, py)], np.uint8)
    assert np.array_equal(got, prim['scalar_nonzero_clipped'])
    got = np.array([F.scalar_nonzero_clipped_with_reduction(occ, 2 * a, 2 * b, 2.0)
                    for a, b in zip(px, py)], np.uint8)
    assert np.array_equal(got, prim['scalar_nonzero_red'])


def test_center_filters(F, prim):
    caf = prim['center_field'].copy()
    for t, (qx, qy, qs) in enumerate(prim['center_queries']):
        assert np.array_equal(F.caf_center_s(caf, qx, qy, qs), prim['caf_center_s_%d' % t])
        p7 = np.ascontiguousarray(caf[:7])
        assert np.array_equal(F.paf_center(p7, qx, qy, qs), prim['paf_center_%d' % t])
        assert np.array_equal(F.paf_center_b(p7, qx, qy, sigma=qs / 3), prim['paf_center_b_%d' % t])
        assert np.array_equal(F.paf_mask_center(p7, qx, qy, sigma=qs / 3),
                              prim['paf_mask_center_%d' % t])


def test_grow_connection_blend_matches_oracle_decode(F):
    """Every grow_connection on a real column set: device == oracle restatement."""
    g = gu.load_case('p40_s0_eval')
    cif, caf, skeleton = gu.case_inputs(g)
    cfg = gu.case_config(g)
    hr = oracle.cifhr(cif, cfg)
    fwd, _ = oracle.caf_scored(caf, hr, skeleton, 0.1, cfg)
    rng = np.random.default_rng(0)
    checked = 0
    for cols in fwd:
        if cols.shape[1] == 0:
            continue
        for _ in range(10):
            i = rng.integers(cols.shape[1])
            x = np.float32(cols[1, i] + rng.normal(0, 3))
            y = np.float32(cols[2, i] + rng.normal(0, 3))
            s = np.float32(rng.uniform(1, 12))
            got = F.grow_connection_blend(cols.copy(), x, y, s)
            want = _oracle_grow_connection(cols, x, y, s)
            assert np.array_equal(np.asarray(got, np.float32), want), (got, want)
            checked += 1
    assert checked > 50


def _oracle_grow_connection(cols, x, y, s):
    """Direct restatement of cifcaf.py:124-192 in numpy float32 (small n), with NumPy's own
    scalar power and exp."""
    sb = np.float32(2.0) * s
    m = ~((cols[1] < x - sb) | (cols[1] > x + sb) | (cols[2] < y - sb) | (cols[2] > y + sb))
    c = cols[:, m]
    if c.shape[1] == 0:
        return np.zeros(4, np.float32)
    dx = x - c[1]
    dy = y - c[2]
    d = np.sqrt(dx * dx + dy * dy)
    sig = np.float32(0.5) * s
    # as the reference evaluates `np.exp(-0.5 * d**2 / sigma**2)`: sigma**2 of a float32
    # scalar is libm powf, np.exp of a float32 array NumPy's SIMD routine
    q = (np.float32(-0.5) * (d * d)) / (sig ** 2)
    scores = np.exp(q) * c[0]
    order = np.argsort(scores, kind='stable')
    t = c[5:]
    if len(scores) == 1:
        return np.array([t[0, 0], t[1, 0], t[3, 0], scores[0] * np.float32(0.5)], np.float32)
    i1, i2 = order[-1], order[-2]
    s1, s2 = scores[i1], scores[i2]
    if s2 < np.float32(0.01) or s2 < np.float32(0.5) * s1:
        return np.array([t[0, i1], t[1, i1], t[3, i1], s1 * np.float32(0.5)], np.float32)
    ex = t[0, i1] - t[0, i2]
    ey = t[1, i1] - t[1, i2]
    if np.sqrt(ex * ex + ey * ey) > t[3, i1] / np.float32(2.0):
        return np.array([t[0, i1], t[1, i1], t[3, i1], s1 * np.float32(0.5)], np.float32)
    ss = s1 + s2
    return np.array([(s1 * t[0, i1] + s2 * t[0, i2]) / ss, (s1 * t[1, i1] + s2 * t[1, i2]) / ss,
                     (s1 * t[3, i1] + s2 * t[3, i2]) / ss, np.float32(0.5) * (s1 + s2)],
                    np.float32)


# ---- decoder stages (single image, reference API) --------------------------------------

def _configure(dec, g):
    gu.configure_decoder(dec, g)


@pytest.mark.parametrize('name', CASES)
def test_stages_bit_exact(dec, name):
    g = gu.load_case(name)
    cif, caf, skeleton = gu.case_inputs(g)
    _configure(dec, g)
    fc = dec.FieldConfig()
    hr = dec.CifHr(fc).fill([cif, caf]).accumulated
    assert gu.sha(hr) == str(g['cifhr_sha'])
    seeds = dec.CifSeeds(hr, fc).fill([cif, caf]).get()
    rows = np.array([tuple(float(t) for t in s) for s in seeds], np.float32).reshape(-1, 5)
    assert np.array_equal(rows, g['seeds'])
    for tag, th in (('a', None), ('b', 0.0001)):
        cs = dec.CafScored(hr, fc, skeleton, score_th=th).fill([cif, caf])
        assert [f.shape[1] for f in cs.forward] == list(g['caf_%s_fwd_counts' % tag])
        assert [gu.sha(f) for f in cs.forward] == [str(s) for s in g['caf_%s_fwd_sha' % tag]]
        assert [gu.sha(b) for b in cs.backward] == [str(s) for s in g['caf_%s_bwd_sha' % tag]]


@pytest.mark.parametrize('name', CASES)
def test_cifcaf_vs_reference(dec, name):
    from openpifpaf_amd import constants
    g = gu.load_case(name)
    cif, caf, skeleton = gu.case_inputs(g)
    _configure(dec, g)
    cc = dec.CifCaf(dec.FieldConfig(), keypoints=constants.COCO_KEYPOINTS, skeleton=skeleton,
                    out_skeleton=constants.COCO_PERSON_SKELETON)
    recs, _, _ = cc.decode_records(cif[None], caf[None])
    stats = {}
    errs = gu.compare_annotations(g, recs, stats=stats)
    print('max deviation vs reference:', stats)
    assert not errs, errs[:10]
    anns = cc([cif, caf])
    assert len(anns) == len(g['ann_score'])
    for a, s in zip(anns, g['ann_score']):
        assert abs(a.score() - s) <= gu.SCORE_ATOL


@pytest.mark.parametrize('name', CASES)
def test_cifcaf_vs_oracle_exact(dec, name):
    """The device decode and the oracle round np.exp and `sigma**2` alike: identical."""
    from openpifpaf_amd import constants
    g = gu.load_case(name)
    cif, caf, skeleton = gu.case_inputs(g)
    _configure(dec, g)
    cc = dec.CifCaf(dec.FieldConfig(), keypoints=constants.COCO_KEYPOINTS, skeleton=skeleton)
    recs, _, _ = cc.decode_records(cif[None], caf[None])
    ref = oracle.decode(cif, caf, skeleton, gu.case_config(g))
    assert len(recs) == len(ref)
    for r, o in zip(recs, ref):
        for key in ('data', 'joint_scales', 'score', 'n_decoding', 'decoding_pairs',
                    'decoding_xyv', 'n_frontier', 'frontier_pairs'):
            assert np.array_equal(r[key], o[key]), key


# ---- batches at the BASELINE sizes ---------------------------------------------------------

def _batch_vs_oracle(dec, kind, n, h, n_check, mode='eval'):
    from openpifpaf_amd import constants, synthetic
    from openpifpaf_amd._abi import EVAL_CONFIG, PREDICT_CONFIG, make_config
    g = {'mode': np.array(mode), 'greedy': 0, 'connection_method': np.array('blend')}
    _configure(dec, g)
    cif, caf = synthetic.batch(kind, n, h, h)
    cc = dec.CifCaf(dec.FieldConfig(), keypoints=constants.COCO_KEYPOINTS,
                    skeleton=constants.COCO_PERSON_SKELETON)
    recs, offsets, _ = cc.decode_records(cif, caf)
    cfg = make_config(**(EVAL_CONFIG if mode == 'eval' else PREDICT_CONFIG))
    step = max(1, n // n_check)
    for i in range(0, n, step):
        ref = oracle.decode(cif[i], caf[i], constants.COCO_PERSON_SKELETON, cfg)
        got = recs[offsets[i]:offsets[i + 1]]
        assert len(got) == len(ref), i
        for r, o in zip(got, ref):
            assert np.array_equal(r['data'], o['data']), i
            assert np.array_equal(r['decoding_pairs'], o['decoding_pairs']), i
            assert r['score'] == o['score'], i
    return offsets


def test_batch256_planted_eval(dec):
    offsets = _batch_vs_oracle(dec, 'planted', 256, 80, 32)
    assert offsets[-1] > 256 * 6  # ~8 people per image


def test_batch_uniform_eval(dec):
    _batch_vs_oracle(dec, 'uniform', 16, 80, 4)


def test_batch_predict(dec):
    _batch_vs_oracle(dec, 'planted', 64, 80, 16, mode='predict')


@pytest.mark.parametrize('kind', ['planted', 'uniform'])
def test_batch160_dense_vs_oracle(dec, kind):
    """BASELINE configs[4] shapes: 160x160 fields with the 44-edge dense skeleton, a batch of
    4 images per generator in one device decode (workspace, capacities and the dense CAF set
    at ~1.4k annotations per uniform image), every image against the oracle byte for byte."""
    from openpifpaf_amd import constants, synthetic
    from openpifpaf_amd._abi import EVAL_CONFIG, make_config
    g = {'mode': np.array('eval'), 'greedy': 0, 'connection_method': np.array('blend')}
    _configure(dec, g)
    sk = constants.DENSE_DECODE_SKELETON
    kw = {'n_caf': len(sk)} if kind == 'uniform' else {'skeleton': sk, 'n_people': 16}
    cif, caf = synthetic.batch(kind, 4, 160, 160, first_seed=60, **kw)
    cc = dec.CifCaf(dec.FieldConfig(), keypoints=constants.COCO_KEYPOINTS, skeleton=sk,
                    out_skeleton=constants.COCO_PERSON_SKELETON)
    recs, offsets, _ = cc.decode_records(cif, caf)
    cfg = make_config(**EVAL_CONFIG)
    for i in range(4):
        ref = oracle.decode(cif[i], caf[i], sk, cfg)
        got = recs[offsets[i]:offsets[i + 1]]
        assert len(got) == len(ref), (i, len(got), len(ref))
        for r, o in zip(got, ref):
            for key in ('data', 'joint_scales', 'score', 'decoding_pairs', 'decoding_xyv',
                        'frontier_pairs'):
                assert np.array_equal(r[key], o[key]), (i, key)
    assert offsets[-1] > (4 * 12 if kind == 'planted' else 4 * 1000)


def test_cifhr_batch_bit_exact():
    """CifHr over a 256-image batch: every image equals the oracle bit for bit."""
    import torch
    from openpifpaf_amd import synthetic
    from openpifpaf_amd._abi import make_config
    from openpifpaf_amd.decoder.cif_hr import cifhr_device
    cif, _ = synthetic.batch('planted', 256, 80, 80)
    hr = cifhr_device(torch.from_numpy(cif).cuda(), 8, 0.1, 16)
    ww = 633
    host = hr[:, :, :, :ww].cpu().numpy()
    assert not hr[:, :, :, ww:].any().item()  # pitch padding written as zeros
    cfg = make_config()
    for i in range(0, 256, 16):
        assert np.array_equal(host[i], oracle.cifhr(cif[i], cfg)), i
    ucif, _ = synthetic.batch('uniform', 8, 80, 80)
    uh = cifhr_device(torch.from_numpy(ucif).cuda(), 8, 0.1, 16)[:, :, :, :ww].cpu().numpy()
    for i in range(8):
        assert np.array_equal(uh[i], oracle.cifhr(ucif[i], cfg)), i


def test_cifhr_sparse_bit_exact():
    """The decoder's block-sparse CifHr (pp_cifhr_sparse) expands to the oracle's map bit for
    bit: planted (short LDS lists), uniform (lists beyond LDS, tiles over 128 candidates)
    and wide splats (sigma up to 40 px: every tile needs several candidate passes)."""
    import torch
    from openpifpaf_amd import synthetic
    from openpifpaf_amd._abi import make_config
    from openpifpaf_amd.decoder.cif_hr import cifhr_sparse_device, sparse_to_dense
    cfg = make_config()
    pcif, _ = synthetic.batch('planted', 64, 80, 80)
    ucif, _ = synthetic.batch('uniform', 4, 80, 80)
    rng = np.random.default_rng(5)
    wcif = ucif[:2].copy()
    wcif[:, :, 4] = rng.uniform(0.5, 10.0, wcif[:, :, 4].shape).astype(np.float32)
    wcif[:, :, 0, 30:50, 30:50] = 0.9  # a dense patch of wide splats
    for cif, n_check in ((pcif, 16), (ucif, 4), (wcif, 2)):
        hmap, masks = cifhr_sparse_device(torch.from_numpy(cif).cuda(), 8, 0.1, 16)
        hmap, masks = hmap.cpu().numpy(), masks.cpu().numpy()
        step = len(cif) // n_check
        for i in range(0, len(cif), step):
            dense = sparse_to_dense(hmap[i], masks[i], 633, 633)
            assert np.array_equal(dense, oracle.cifhr(cif[i], cfg)), i
    # planted maps are sparse: most blocks never written
    on = np.unpackbits(masks.view(np.uint8)).mean()
    assert 0.0 < on <= 1.0


# 17*144 seeds sort in registers (4 per thread), 17*400 in the 8-per-thread network (ties
# re-sorted through global scratch), 17*576 in the global network
@pytest.mark.parametrize('hw', [12, 20, 24])
def test_seed_ties(dec, hw):
    """Saturated CifHr gives equal v within a field: the sort must fall back to the full
    tuple order (x, y, s descending, then emission order), cif_seeds.py:54."""
    g = {'mode': np.array('eval'), 'greedy': 0, 'connection_method': np.array('blend')}
    _configure(dec, g)
    rng = np.random.default_rng(3)
    yy, xx = np.mgrid[0:hw, 0:hw].astype(np.float32)
    cif = np.zeros((17, 5, hw, hw), np.float32)
    cif[:, 0] = 0.9
    cif[:, 1] = np.floor(xx / 2) * 2   # duplicate positions -> ties on (x, y)
    cif[:, 2] = np.floor(yy / 2) * 2
    cif[:, 3] = 0.5
    cif[:, 4] = rng.choice(np.array([1.0, 2.0], np.float32), (17, hw, hw))  # ties on s too
    cif[5, 0, 3:6, 3:6] = 0.35  # a few distinct v
    caf = np.zeros((19, 9, hw, hw), np.float32)
    fc = dec.FieldConfig()
    hr = dec.CifHr(fc).fill([cif, caf]).accumulated
    assert np.array_equal(hr, oracle.cifhr(cif))
    seeds = dec.CifSeeds(hr, fc).fill([cif, caf]).get()
    got = np.array([tuple(float(t) for t in sd) for sd in seeds], np.float32).reshape(-1, 5)
    ref = oracle.seeds(cif, hr)
    exp = np.stack([ref['v'], ref['field'].astype(np.float32), ref['x'], ref['y'], ref['s']], 1)
    assert len(got) == len(exp) > 17 * hw * hw // 2
    assert np.array_equal(got, exp)
    assert (np.diff(exp[:, 0]) == 0).sum() > len(exp) // 2  # the case really has ties


# 17*324 seeds, no (v, field) ties: sorted with 8 keys per thread, output from registers;
# 17*441 (6958 seeds, three ties where 0.9 + 0.1 * conf rounds equal): the same network,
# then the ties re-sorted with the full comparator through global scratch
@pytest.mark.parametrize('hw', [18, 21])
def test_seeds_8k_network(dec, hw):
    """Seed sets of 4096 < n <= 8192 (stages.hip seeds_sort_kernel), against the oracle."""
    g = {'mode': np.array('eval'), 'greedy': 0, 'connection_method': np.array('blend')}
    _configure(dec, g)
    rng = np.random.default_rng(11)
    yy, xx = np.mgrid[0:hw, 0:hw].astype(np.float32)
    cif = np.zeros((17, 5, hw, hw), np.float32)
    cif[:, 0] = rng.uniform(0.8, 1.0, (17, hw, hw)).astype(np.float32)  # distinct: no ties
    cif[:, 1] = np.floor(xx / 2) * 2  # shared positions: CifHr saturates, every cell seeds
    cif[:, 2] = np.floor(yy / 2) * 2
    cif[:, 3] = 0.5
    cif[:, 4] = rng.uniform(0.5, 1.5, (17, hw, hw)).astype(np.float32)
    caf = np.zeros((19, 9, hw, hw), np.float32)
    fc = dec.FieldConfig()
    hr = dec.CifHr(fc).fill([cif, caf]).accumulated
    seeds = dec.CifSeeds(hr, fc).fill([cif, caf]).get()
    got = np.array([tuple(float(t) for t in sd) for sd in seeds], np.float32).reshape(-1, 5)
    ref = oracle.seeds(cif, hr)
    exp = np.stack([ref['v'], ref['field'].astype(np.float32), ref['x'], ref['y'], ref['s']], 1)
    assert 4096 < len(exp) <= 8192, len(exp)
    assert np.array_equal(got, exp)


def _tie_fields(hw, distinct):
    rng = np.random.default_rng(3 if not distinct else 11)
    yy, xx = np.mgrid[0:hw, 0:hw].astype(np.float32)
    cif = np.zeros((17, 5, hw, hw), np.float32)
    cif[:, 0] = rng.uniform(0.8, 1.0, (17, hw, hw)).astype(np.float32) if distinct else 0.9
    cif[:, 1] = np.floor(xx / 2) * 2
    cif[:, 2] = np.floor(yy / 2) * 2
    cif[:, 3] = 0.5
    cif[:, 4] = rng.choice(np.array([1.0, 2.0], np.float32), (17, hw, hw))
    return cif


# the DEVICE order of the seeds (the seed loop's order; the API's get() re-sorts on the
# host), one image and a batch of 17: seeds_sort_kernel's bitonic network up to 256 seeds
# (3: 153), the radix sort up to 4096 (4: 272, 10: 1700, 12: all tied, 15: 3825; ties
# re-sorted in LDS), 8 keys per thread up to 8192 (ties through global scratch), the
# global network beyond
@pytest.mark.parametrize('n_img', [1, 17])
@pytest.mark.parametrize('hw,distinct', [(3, True), (4, True), (10, True), (12, False),
                                         (15, True), (18, True), (20, False), (24, False)])
def test_seeds_device_order(dec, n_img, hw, distinct, seed_mask=None):
    import torch
    from openpifpaf_amd import _device
    from openpifpaf_amd._abi import SEED_DTYPE, make_config, scale_list
    from openpifpaf_amd._lib import call
    from openpifpaf_amd.decoder._fields import cfg_ptr, pitched_hr, with_geometry
    cfg = make_config(seed_mask=seed_mask)
    cif = _tie_fields(hw, distinct)
    hr = oracle.cifhr(cif)
    ref = oracle.seeds(cif, hr, cfg)
    c = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(cif, (n_img,) + cif.shape))).cuda()
    h1 = pitched_hr(hr)
    hrb = h1.expand(n_img, -1, -1, -1).contiguous()
    k = 17
    cap = k * hw * hw
    arr = with_geometry(scale_list([(c.data_ptr(), hw, hw)], [], [8], [], [0.0]), hr.shape)
    out = torch.empty(n_img * cap * SEED_DTYPE.itemsize, dtype=torch.uint8, device='cuda')
    count = torch.zeros(n_img, dtype=torch.int32, device='cuda')
    call('pp_seeds_multi', arr, len(arr), _device.ptr(hrb), n_img, k, cfg_ptr(cfg),
         _device.ptr(out), cap, _device.ptr(count), _device.stream())
    recs = np.frombuffer(out.cpu().numpy().tobytes(), dtype=SEED_DTYPE).reshape(n_img, cap)
    counts = count.cpu().numpy()
    for i in range(n_img):
        got = recs[i, :counts[i]]
        assert len(got) == len(ref), (i, len(got), len(ref))
        for name in ('v', 'field', 'x', 'y', 's'):
            assert np.array_equal(got[name], ref[name]), (i, name)


@pytest.mark.parametrize('n_img', [1, 3])
def test_seeds_crowded_bucket_falls_back(dec, n_img):
    """seeds_sort_kernel's bucket pass ranks a key by scanning its bucket, so a
    bucket of b keys costs b^2 LDS reads.  9 seeding fields of 17 x 17 cells, every cell of
    a field at one v: 289 keys per bucket, above kBucketMax, so the sort falls back to the
    radix passes (2601 keys <= 4096); the device order equals the oracle's."""
    test_seeds_device_order(dec, n_img, 17, False, seed_mask=[f % 2 == 0 for f in range(17)])


# the decoder's own seeds at a batch whose fields get one workgroup each (64 images x 17
# fields >= 1024): emitted by the CifHr kernel itself (cifhr_fused_kernel<true>), then
# sorted; and at 2 images, whose fields split over several workgroups (the list kernel
# writes the seed candidates, the fold's last workgroup per field finishes them);
# saturated and tied confidences, the full decode against the oracle
@pytest.mark.parametrize('n', [64, 2])
@pytest.mark.parametrize('hw,distinct', [(12, False), (18, True), (20, False)])
def test_fused_seeds_decode_ties(dec, hw, distinct, n):
    import torch
    from openpifpaf_amd import constants
    from openpifpaf_amd._abi import make_config
    from openpifpaf_amd.engine import DecodeEngine
    cfg = make_config(seed_threshold=0.2, force_complete=False)
    cif = _tie_fields(hw, distinct)
    caf = np.zeros((19, 9, hw, hw), np.float32)
    skel = constants.COCO_PERSON_SKELETON
    ref = oracle.decode(cif, caf, skel, cfg)
    c = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(cif, (n,) + cif.shape))).cuda()
    f = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(caf, (n,) + caf.shape))).cuda()
    recs, offs, _ = DecodeEngine().decode(c, f, skel, cfg)
    for i in sorted({0, 1, n // 2 - 1, n - 1}):
        got = recs[offs[i]:offs[i + 1]]
        assert len(got) == len(ref) > 0, (i, len(got), len(ref))
        for name in ('data', 'joint_scales', 'decoding_pairs'):
            assert got[name].tobytes() == ref[name].tobytes(), (i, name)


def test_stage_calls_equal_full_decode(dec):
    """pp_decode_stages called stage by stage, or with several stages per call, gives the
    same records as pp_decode_batch (the stage contract of include/pifpaf_amd.h)."""
    import torch
    from openpifpaf_amd import constants, engine, synthetic
    from openpifpaf_amd._abi import EVAL_CONFIG, make_config
    cif, caf = synthetic.batch('planted', 32, 80, 80, first_seed=900)
    c, f = torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda()
    cfg = make_config(**EVAL_CONFIG)
    sk = constants.COCO_PERSON_SKELETON
    eng = engine.DecodeEngine()
    ref, ref_off = eng.fetch(eng.launch(c, f, sk, cfg))
    ref = ref.copy()
    # 16: force-complete sets built early (with stage 4, or before the CifHr map with
    # stage 1); 32 / 64: stage 8 split into the seed loop and the rest (same output slot)
    for groups in ((1, 2, 4, 8), (1, 14), (15,), (1, 2 | 4 | 16, 8 | 16),
                   (1, 2 | 4 | 16, 8 | 16 | 32, 8 | 16 | 64), (1 | 16, 2 | 4, 8 | 16 | 32, 8 | 16 | 64)):
        for bits in groups:
            b = eng.launch(c, f, sk, cfg, stages=bits)
        got, off = eng.fetch(b)
        assert np.array_equal(off, ref_off), groups
        assert got.tobytes() == ref.tobytes(), groups


def test_workspace_left_clean(dec):
    """The occupancy workspace is zero again after a decode (workspace contract)."""
    from openpifpaf_amd import constants, engine, synthetic
    g = {'mode': np.array('eval'), 'greedy': 0, 'connection_method': np.array('blend')}
    _configure(dec, g)
    cif, caf = synthetic.batch('uniform', 4, 40, 40)
    cc = dec.CifCaf(dec.FieldConfig(), keypoints=constants.COCO_KEYPOINTS,
                    skeleton=constants.COCO_PERSON_SKELETON)
    _, _, b = cc.decode_records(cif, caf)
    from openpifpaf_amd._lib import load
    import ctypes
    cfg = cc.config()
    zoff = load().pp_decode_workspace_zero_offset(4, 17, 19, 40, 40, ctypes.byref(cfg), b.cap)
    # H' = 313 -> 156 rows; rows padded to 16 bytes: 17 planes of (156 + 64) x 224
    occ_bytes = b.ws[zoff:zoff + 4 * 17 * (156 + 64) * 224]
    assert int(occ_bytes.sum().item()) == 0
    assert engine.engine() is not None


# ---- standalone nms.Keypoints (nms.py:17-57) ------------------------------------------------

def _nms_anns(data, scales):
    from openpifpaf_amd import constants
    from openpifpaf_amd.annotation import Annotation
    anns = []
    for d, sc in zip(data, scales):
        a = Annotation(constants.COCO_KEYPOINTS, constants.COCO_PERSON_SKELETON)
        a.data = d.copy()
        a.joint_scales = sc.copy()
        anns.append(a)
    return anns


@pytest.mark.parametrize('name', ['eval', 'predict', 'supp', 'dense', 'zeros'])
def test_nms_keypoints_vs_reference(dec, name):
    """Device NMS over host Annotation lists: the reference's order, in-place edits, scores."""
    g = np.load(os.path.join(gu.GOLDEN, 'nms.npz'))
    kt, it, sup = (float(t) for t in g[name + '_cfg'])
    anns = _nms_anns(g[name + '_data_in'], g[name + '_scales'])
    k = dec.nms.Keypoints()
    k.keypoint_threshold, k.instance_threshold, k.suppression = kt, it, sup
    res = k.annotations(list(anns))
    ids = {id(a): i for i, a in enumerate(anns)}
    assert [ids[id(a)] for a in res] == g[name + '_order'].tolist()
    assert np.array_equal(np.stack([a.data for a in anns]), g[name + '_data_out'])
    assert np.array_equal(np.array([a.score() for a in res]), g[name + '_score'])


@pytest.mark.parametrize('name', ['mixed', 'fixed_ties'])
def test_nms_keypoints_scored_vs_reference(dec, name):
    """Annotations with fixed_score / suppress_score_index (annotation.py:60-71): the
    reference's filter, order and in-place edits (pp_nms_keypoints_scored)."""
    from openpifpaf_amd import constants
    from openpifpaf_amd.annotation import Annotation
    g = np.load(os.path.join(gu.GOLDEN, 'nms_scored.npz'))
    kt, it, sup = (float(t) for t in g[name + '_cfg'])
    anns = []
    for d, sc, fx, sp in zip(g[name + '_data_in'], g[name + '_scales'], g[name + '_fixed'],
                             g[name + '_supp']):
        a = Annotation(constants.COCO_KEYPOINTS, constants.COCO_PERSON_SKELETON,
                       suppress_score_index=None if sp == -999 else int(sp))
        a.data = d.copy()
        a.joint_scales = sc.copy()
        if not np.isnan(fx):
            a.fixed_score = float(fx)
        anns.append(a)
    k = dec.nms.Keypoints()
    k.keypoint_threshold, k.instance_threshold, k.suppression = kt, it, sup
    res = k.annotations(list(anns))
    ids = {id(a): i for i, a in enumerate(anns)}
    assert [ids[id(a)] for a in res] == g[name + '_order'].tolist()
    assert np.array_equal(np.stack([a.data for a in anns]), g[name + '_data_out'])
    assert np.array_equal(np.array([a.score() for a in res]), g[name + '_score'])


def test_nms_keypoints_many_vs_oracle(dec):
    """More kept annotations than the LDS box lists hold (global-memory path)."""
    rng = np.random.default_rng(7)
    n = 1500
    xy = rng.uniform(0.0, 2000.0, (n, 17, 2)).astype(np.float32)
    v = rng.uniform(0.05, 1.0, (n, 17)).astype(np.float32)
    data = np.concatenate([xy, v[:, :, None]], axis=2)
    scales = rng.uniform(0.5, 6.0, (n, 17)).astype(np.float32)
    order, recs = oracle.nms_keypoints(data, scales, 0.0, 0.0, 0.0)
    assert len(order) > 1100
    anns = _nms_anns(data, scales)
    res = dec.nms.Keypoints().annotations(list(anns))
    ids = {id(a): i for i, a in enumerate(anns)}
    assert [ids[id(a)] for a in res] == order.tolist()
    assert np.array_equal(np.stack([a.data for a in res]), recs['data'][:, :17])


# ---- head conv output -> decoder fields (network/heads.py) ------------------------------------

@pytest.mark.parametrize('quad', [0, 1, 2])
@pytest.mark.parametrize('kind,n_fields', [('cif', 17), ('caf', 19), ('cifdet', 3)])
def test_ingest_vs_reference(kind, n_fields, quad):
    import torch
    from openpifpaf_amd import heads
    g = np.load(os.path.join(gu.GOLDEN, 'heads.npz'))
    conv = g['q%d_%s_conv' % (quad, kind)]
    got = heads.fields_from_conv(torch.from_numpy(conv).cuda(), n_fields, kind, quad).cpu().numpy()
    exp = g['q%d_%s' % (quad, kind)]
    assert got.shape == exp.shape
    np.testing.assert_allclose(got, exp, rtol=1e-6, atol=1e-7)  # torch f32 sigmoid / exp
    ref = oracle.fields_from_conv(conv, n_fields, kind, quad)  # same f64-rounded math
    ulp = np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1


def test_ingest_large_batch():
    """An 8-image CIF head at quad 1 (h = w = 41 -> 81 x 81) against the restatement."""
    import torch
    from openpifpaf_amd import heads
    rng = np.random.default_rng(5)
    conv = rng.standard_normal((8, 17 * 5 * 4, 41, 41)).astype(np.float32)
    got = heads.fields_from_conv(torch.from_numpy(conv).cuda(), 17, 'cif', 1).cpu().numpy()
    ref = oracle.fields_from_conv(conv, 17, 'cif', 1)
    assert got.shape == (8, 17, 5, 81, 81)
    ulp = np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1


# ---- CifDet (decoder/generator/cifdet.py) -----------------------------------------------------

DET_NAMES = sorted(os.path.basename(p)[4:-4] for p in
                   __import__('glob').glob(os.path.join(gu.GOLDEN, 'det_*.npz'))
                   if not p.endswith('det_nms.npz'))


def _det_case(dec, name):
    from openpifpaf_amd import synthetic
    g = np.load(os.path.join(gu.GOLDEN, 'det_%s.npz' % name))
    det = synthetic.det_batch(str(g['gen']), 1, int(g['h']), int(g['w']), first_seed=int(g['seed']),
                              n_categories=int(g['n_categories']))[0]
    assert gu.sha(det) == str(g['input_sha'])
    dec.CifHr.v_threshold = 0.1
    dec.CifSeeds.threshold = float(g['seed_threshold'])
    return g, det


@pytest.mark.parametrize('name', DET_NAMES)
def test_cifdet_stages_vs_reference(dec, name):
    g, det = _det_case(dec, name)
    fc = dec.FieldConfig()
    hr = dec.CifDetHr(fc).fill([det]).accumulated
    assert gu.sha(hr) == str(g['cifhr_sha'])
    seeds = dec.CifDetSeeds(hr, fc).fill([det]).get()
    rows = np.array([[float(t) for t in sd] for sd in seeds], np.float32).reshape(-1, 6)
    assert np.array_equal(rows, g['seeds'])


@pytest.mark.parametrize('name', DET_NAMES)
def test_cifdet_vs_reference(dec, name):
    g, det = _det_case(dec, name)
    k = int(g['n_categories'])
    anns = dec.CifDet(dec.FieldConfig(), ['c%d' % i for i in range(k)])([det])
    assert [a.field_i for a in anns] == g['ann_field'].tolist()
    assert np.array_equal(np.array([a.score for a in anns], np.float32), g['ann_score'])
    assert np.array_equal(np.array([a.bbox for a in anns], np.float32).reshape(-1, 4),
                          g['ann_bbox'])


@pytest.mark.parametrize('kind', ['planted', 'uniform'])
def test_cifdet_batch_vs_oracle(dec, kind):
    from openpifpaf_amd import synthetic
    from openpifpaf_amd._abi import make_config
    dec.CifHr.v_threshold = 0.1
    dec.CifSeeds.threshold = 0.3 if kind == 'planted' else 0.1
    det = synthetic.det_batch(kind, 24, 48, 40, first_seed=50, n_categories=4)
    cd = dec.CifDet(dec.FieldConfig(), ['a', 'b', 'c', 'd'])
    recs, offsets = cd.decode_records(det)
    cfg = make_config(seed_threshold=dec.CifSeeds.threshold)
    for i in range(len(det)):
        ref = oracle.cifdet_decode(det[i], cfg)
        got = recs[offsets[i]:offsets[i + 1]]
        assert len(got) == len(ref), i
        assert np.array_equal(got['field'], ref['field']), i
        assert np.array_equal(got['score'], ref['score']), i
        assert np.array_equal(got['bbox'], ref['bbox']), i


DETM_NAMES = sorted(os.path.basename(p)[5:-4] for p in
                    __import__('glob').glob(os.path.join(gu.GOLDEN, 'detm_*.npz')))


def _detm_case(dec, name):
    """detm_<name>.npz: the reference CifDet over several heads / min scales
    (gen_golden.DET_MULTI_CASES); (fixture, FieldConfig, per-head fields, categories)."""
    from openpifpaf_amd import synthetic
    g = np.load(os.path.join(gu.GOLDEN, 'detm_%s.npz' % name))
    k = int(g['n_categories'])
    heads = [tuple(r) for r in g['heads']]
    fields = [synthetic.det_batch(str(g['gen']), 1, int(h), int(w), first_seed=int(seed),
                                  n_categories=k)[0] for h, w, _, _, seed in heads]
    assert [gu.sha(f) for f in fields] == [str(x) for x in g['input_sha']]
    fc = dec.FieldConfig(cif_indices=list(range(len(heads))),
                         cif_strides=[int(st) for _, _, st, _, _ in heads],
                         cif_min_scales=[float(ms) for _, _, _, ms, _ in heads])
    dec.CifHr.v_threshold = 0.1
    dec.CifSeeds.threshold = float(g['seed_threshold'])
    return g, fc, fields, ['c%d' % i for i in range(k)]


@pytest.mark.parametrize('name', DETM_NAMES)
def test_cifdet_multi_stages_vs_reference(dec, name):
    """CifDetHr / CifDetSeeds over several heads and min scales (cif_hr.py:67-90,
    cif_seeds.py:56-90): map digest and the full seed list."""
    g, fc, fields, _ = _detm_case(dec, name)
    hr = dec.CifDetHr(fc).fill(fields).accumulated
    assert gu.sha(hr) == str(g['cifhr_sha'])
    seeds = dec.CifDetSeeds(hr, fc).fill(fields).get()
    rows = np.array([[float(t) for t in sd] for sd in seeds], np.float32).reshape(-1, 6)
    assert np.array_equal(rows, g['seeds'])


@pytest.mark.parametrize('name', DETM_NAMES)
def test_cifdet_multi_vs_reference(dec, name):
    """CifDet.__call__ over several heads / min scales (pp_cifdet_decode_multi)."""
    g, fc, fields, cats = _detm_case(dec, name)
    anns = dec.CifDet(fc, cats)(fields)
    assert [a.field_i for a in anns] == g['ann_field'].tolist()
    assert np.array_equal(np.array([a.score for a in anns], np.float32), g['ann_score'])
    assert np.array_equal(np.array([a.bbox for a in anns], np.float32).reshape(-1, 4),
                          g['ann_bbox'])


def test_cifdet_multi_batch_matches_single_images(dec):
    """decode_batch over a batch of two-head fields (one pp_cifdet_decode_multi launch) equals
    each image's own decode, record for record (but the image index); a one-head FieldConfig
    with a zero min scale
    through the multi entry point equals pp_cifdet_decode."""
    import torch
    from openpifpaf_amd import synthetic
    dec.CifHr.v_threshold = 0.1
    dec.CifSeeds.threshold = 0.3
    h0 = synthetic.det_batch('planted', 6, 40, 48, first_seed=70, n_categories=3)
    h1 = synthetic.det_batch('planted', 6, 20, 24, first_seed=170, n_categories=3)
    fc = dec.FieldConfig(cif_indices=[0, 1], cif_strides=[8, 16], cif_min_scales=[0.0, 48.0])
    cd = dec.CifDet(fc, ['a', 'b', 'c'])
    recs, offsets = cd.decode_records([torch.from_numpy(h0).cuda(), torch.from_numpy(h1).cuda()])
    for i in range(6):
        one, off1 = cd.decode_records([torch.from_numpy(h0[i:i + 1]).cuda(),
                                       torch.from_numpy(h1[i:i + 1]).cuda()])
        got = recs[offsets[i]:offsets[i + 1]]
        assert (got['image'] == i).all() and (one['image'] == 0).all(), i
        for key in ('field', 'score', 'bbox'):
            assert got[key].tobytes() == one[key].tobytes(), (i, key)
    # the multi entry point with one plain head is the single-head decode
    from openpifpaf_amd import _device
    from openpifpaf_amd._abi import scale_list
    from openpifpaf_amd._lib import call, load
    import ctypes
    single = dec.CifDet(dec.FieldConfig(), ['a', 'b', 'c'])
    ref, ref_off = single.decode_records(h0)
    cfg = single.config()
    z = __import__('openpifpaf_amd.decoder.generator.cifdet', fromlist=['x']).det_nms_config()
    t = torch.from_numpy(h0).cuda()
    arr = scale_list([(t.data_ptr(), 40, 48)], [], [8], [], [0.0])
    cap = 40 * 48
    ws = torch.empty(int(load().pp_cifdet_multi_workspace_size(arr, 1, 0, 6, 3, cap)),
                     dtype=torch.uint8, device='cuda')
    out = torch.empty((6, cap, 32), dtype=torch.uint8, device='cuda')
    counts = torch.empty(6, dtype=torch.int32, device='cuda')
    status = torch.empty(6, dtype=torch.int32, device='cuda')
    call('pp_cifdet_decode_multi', arr, 1, 0, 6, 3, ctypes.byref(cfg), ctypes.byref(z),
         _device.ptr(None), _device.ptr(out), cap, _device.ptr(counts), _device.ptr(status),
         _device.ptr(ws), ctypes.c_size_t(ws.numel()), _device.stream())
    host, n = out.cpu().numpy(), counts.cpu().numpy()
    assert not status.cpu().numpy().any()
    got = np.concatenate([host[i, :n[i]].reshape(-1) for i in range(6)]).tobytes()
    assert got == ref.tobytes()


@pytest.mark.parametrize('name', ['few', 'many', 'ties'])
def test_nms_detection_vs_reference(dec, name):
    from openpifpaf_amd.annotation import AnnotationDet
    g = np.load(os.path.join(gu.GOLDEN, 'det_nms.npz'))
    anns = [AnnotationDet(['a', 'b', 'c']).set(int(f), np.float32(s), b)
            for f, s, b in zip(g[name + '_field'], g[name + '_score_in'], g[name + '_bbox'])]
    ids = {id(a): i for i, a in enumerate(anns)}
    res = dec.nms.Detection().annotations(list(anns))
    assert [ids[id(a)] for a in res] == g[name + '_order'].tolist()
    assert np.array_equal(np.array([a.score for a in anns], np.float32), g[name + '_score_out'])



# ---- Preprocess.annotations_inverse + json_data (transforms/preprocess.py, annotation.py) ----

@pytest.mark.parametrize('name', ['shift', 'flip', 'rot'])
def test_annotations_inverse_vs_reference(name):
    import json
    from test_oracle_golden import inverse_metas
    from openpifpaf_amd import constants, eval_coco, transforms
    from openpifpaf_amd.annotation import Annotation, AnnotationDet
    g = np.load(os.path.join(gu.GOLDEN, 'inverse.npz'))
    meta = inverse_metas()[name]
    anns = []
    for i in range(len(g['pose_data'])):
        a = Annotation(constants.COCO_KEYPOINTS, constants.COCO_PERSON_SKELETON)
        a.data = g['pose_data'][i].copy()
        a.joint_scales = g['pose_scales'][i].copy()
        a.decoding_order = [(int(j1), int(j2), g['pose_dxyv'][i, t, :3].copy(),
                             g['pose_dxyv'][i, t, 3:].copy())
                            for t, (j1, j2) in enumerate(g['pose_dpairs'][i][:g['pose_nd'][i]])]
        anns.append(a)
    inv = transforms.Preprocess.annotations_inverse(anns, meta)
    assert np.array_equal(np.stack([a.data for a in inv]), g[name + '_pose_data'])
    assert np.array_equal(np.stack([a.joint_scales for a in inv]), g[name + '_pose_scales'])
    o = np.zeros_like(g['pose_dxyv'])
    for i, a in enumerate(inv):
        for t, (_, __, c1, c2) in enumerate(a.decoding_order):
            o[i, t, :3], o[i, t, 3:] = c1[:3], c2[:3]
    assert np.array_equal(o, g[name + '_pose_dxyv'])
    assert json.dumps([a.json_data() for a in inv]) == str(g[name + '_pose_json'])
    assert np.array_equal(np.stack([a.data for a in anns]), g['pose_data'])  # inputs untouched
    dets = [AnnotationDet(['c0', 'c1', 'c2']).set(int(f), np.float32(sc), b)
            for f, sc, b in zip(g['det_field'], g['det_score'], g['det_bbox'])]
    dinv = transforms.Preprocess.annotations_inverse(dets, meta)
    assert np.array_equal(np.stack([a.bbox for a in dinv]), g[name + '_det_bbox'])
    assert json.dumps([a.json_data() for a in dinv]) == str(g[name + '_det_json'])
    recs = eval_coco.coco_predictions(anns, meta)
    assert [r['image_id'] for r in recs] == [7] * len(anns)


# ---- multi-scale FieldConfig (cif_hr.py:59-73, cif_seeds.py:56-64, caf_scored.py:88-98) ----

MULTI_NAMES = [(c, m) for c in ('ms2', 'ms10') for m in ('eval', 'predict')]
REC_KEYS = ('data', 'joint_scales', 'score', 'n_keypoints', 'n_decoding', 'decoding_pairs',
            'decoding_xyv', 'n_frontier', 'frontier_pairs')


def _same_records(got, ref):
    assert len(got) == len(ref)
    for r, o in zip(got, ref):
        for key in REC_KEYS:
            assert np.array_equal(r[key], o[key]), key


def _multi_case(dec, name, mode):
    from openpifpaf_amd import synthetic
    g = np.load(os.path.join(gu.GOLDEN, 'multi_%s_%s.npz' % (name, mode)))
    fields, kw = synthetic.multi_case(name)
    assert gu.sha(*fields) == str(g['input_sha'])
    _configure(dec, g)
    return g, fields, kw


@pytest.mark.parametrize('name,mode', MULTI_NAMES)
def test_multi_stages_vs_reference(dec, name, mode):
    """CifHr (pairs / maxima), seeds and both CafScored sets of a multi-scale FieldConfig
    through the reference API, bit-exact against the reference's fixtures."""
    from openpifpaf_amd import constants
    g, fields, kw = _multi_case(dec, name, mode)
    fc = dec.FieldConfig(**kw)
    hr = dec.CifHr(fc).fill(fields).accumulated
    assert list(hr.shape) == list(g['cifhr_shape'])
    assert gu.sha(hr) == str(g['cifhr_sha'])
    seeds = dec.CifSeeds(hr, fc).fill(fields).get()
    rows = np.array([tuple(float(t) for t in s) for s in seeds], np.float32).reshape(-1, 5)
    assert np.array_equal(rows, g['seeds'])
    skel = constants.COCO_PERSON_SKELETON
    for tag, th in (('a', None), ('b', 0.0001)):
        cs = dec.CafScored(hr, fc, skel, score_th=th).fill(fields)
        assert [f.shape[1] for f in cs.forward] == list(g['caf_%s_fwd_counts' % tag])
        assert [gu.sha(f) for f in cs.forward] == [str(s) for s in g['caf_%s_fwd_sha' % tag]]
        assert [gu.sha(b) for b in cs.backward] == [str(s) for s in g['caf_%s_bwd_sha' % tag]]


@pytest.mark.parametrize('name,mode', MULTI_NAMES)
def test_multi_cifcaf_vs_reference(dec, name, mode):
    from openpifpaf_amd import constants
    g, fields, kw = _multi_case(dec, name, mode)
    cc = dec.CifCaf(dec.FieldConfig(**kw), keypoints=constants.COCO_KEYPOINTS,
                    skeleton=constants.COCO_PERSON_SKELETON)
    recs, _, _ = cc.decode_fields_records([f[None] for f in fields])
    stats = {}
    errs = gu.compare_annotations(g, recs, stats=stats)
    print('max deviation vs reference:', stats)
    assert not errs, errs[:10]
    oracle_recs = oracle.decode_multi(oracle.Members(fields, **kw),
                                      constants.COCO_PERSON_SKELETON, gu.case_config(g))
    _same_records(recs, oracle_recs)
    anns = cc(fields)
    assert len(anns) == len(g['ann_score'])
    for a, s in zip(anns, g['ann_score']):
        assert abs(a.score() - s) <= gu.SCORE_ATOL


def _multi_batch(name, n, first_seed=100, n_people=4):
    from openpifpaf_amd import synthetic
    per = [synthetic.multi_case(name, seed=first_seed + i, n_people=n_people) for i in range(n)]
    kw = per[0][1]
    fields = [np.stack([p[0][j] for p in per]) for j in range(len(per[0][0]))]
    return fields, kw


@pytest.mark.parametrize('name', ['ms2', 'ms10'])
def test_multi_batch_vs_oracle(dec, name):
    """A batch of multi-scale images in one pp_decode_multi call equals the oracle per image
    (records compared byte for byte)."""
    from openpifpaf_amd import constants
    from openpifpaf_amd._abi import EVAL_CONFIG, make_config
    g = {'mode': np.array('eval'), 'greedy': 0, 'connection_method': np.array('blend')}
    _configure(dec, g)
    fields, kw = _multi_batch(name, 12, n_people=6)
    cc = dec.CifCaf(dec.FieldConfig(**kw), keypoints=constants.COCO_KEYPOINTS,
                    skeleton=constants.COCO_PERSON_SKELETON)
    recs, offsets, _ = cc.decode_fields_records(fields)
    cfg = make_config(**EVAL_CONFIG)
    for i in range(len(offsets) - 1):
        ref = oracle.decode_multi(oracle.Members([f[i] for f in fields], **kw),
                                  constants.COCO_PERSON_SKELETON, cfg)
        _same_records(recs[offsets[i]:offsets[i + 1]], ref)
    assert offsets[-1] > 12 * 3


def test_multi_unequal_heads_vs_oracle(dec):
    """Two CIF heads and one CAF head at another stride (FieldConfig lists of different
    lengths): the CIF / CAF head lists are independent."""
    from openpifpaf_amd import constants, synthetic
    from openpifpaf_amd._abi import EVAL_CONFIG, make_config
    g = {'mode': np.array('eval'), 'greedy': 0, 'connection_method': np.array('blend')}
    _configure(dec, g)
    heads = synthetic.planted_multi(321, 321, [8, 16], n_people=5, seed=7)
    fields = [heads[0][0], heads[1][0], heads[1][1]]  # cif s8, cif s16, caf s16
    kw = dict(cif_indices=[0, 1], caf_indices=[2], cif_strides=[8, 16], caf_strides=[16],
              cif_min_scales=[0.0, 8.0], caf_min_distances=[12.0], caf_max_distances=[None])
    cc = dec.CifCaf(dec.FieldConfig(**kw), keypoints=constants.COCO_KEYPOINTS,
                    skeleton=constants.COCO_PERSON_SKELETON)
    recs, _, _ = cc.decode_fields_records([f[None] for f in fields])
    ref = oracle.decode_multi(oracle.Members(fields, **kw), constants.COCO_PERSON_SKELETON,
                              make_config(**EVAL_CONFIG))
    assert len(ref) > 2
    _same_records(recs, ref)


def test_multi_stage_calls_equal_full_decode(dec):
    """pp_decode_multi stage by stage == one call (stage contract)."""
    import torch
    from openpifpaf_amd import constants, engine
    from openpifpaf_amd._abi import EVAL_CONFIG, make_config
    fields, kw = _multi_batch('ms10', 4)
    heads = engine.HeadSet([torch.from_numpy(f).cuda() for f in fields], dec.FieldConfig(**kw))
    cfg = make_config(**EVAL_CONFIG)
    sk = constants.COCO_PERSON_SKELETON
    eng = engine.DecodeEngine()
    ref, ref_off = eng.fetch(eng.launch_multi(heads, sk, cfg))
    ref = ref.copy()
    for bits in (1, 2, 4, 8):
        b = eng.launch_multi(heads, sk, cfg, stages=bits)
    got, off = eng.fetch(b)
    assert np.array_equal(off, ref_off)
    assert got.tobytes() == ref.tobytes()


def test_pack_records_zero_copy():
    """pp_pack_records (engine.fetch, one synchronisation, pinned host destination) returns
    exactly the records and offsets of the gather path; a too-small destination gets only
    its first records but every count; the overflow fallback and a pageable (unpinned)
    host destination, which the library must refuse."""
    import ctypes
    import torch
    from openpifpaf_amd import _device, constants, engine, synthetic
    from openpifpaf_amd._abi import ANN_DTYPE, EVAL_CONFIG, make_config
    from openpifpaf_amd._lib import PPError, call
    cfg = make_config(**EVAL_CONFIG)
    sk = constants.COCO_PERSON_SKELETON
    eng = engine.DecodeEngine()
    for kind, n in (('planted', 24), ('uniform', 3)):
        cif, caf = synthetic.batch(kind, n, 48, 48, first_seed=31)
        b = eng.launch(torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda(), sk, cfg)
        ref, ref_off = eng.fetch_gather(b)
        ref = ref.copy()
        got, off = eng.fetch(b)  # uniform: > 16 records per image -> re-packed into a larger block
        assert np.array_equal(off, ref_off) and got.tobytes() == ref.tobytes(), kind
        got, off = eng.fetch(b)  # the grown block: zero-copy again
        assert getattr(b, 'pack_cap', 0) == 0 or b.pack_cap >= len(ref)
        assert np.array_equal(off, ref_off) and got.tobytes() == ref.tobytes(), kind
    # device destination smaller than the batch: first records, complete counts
    cut = max(1, len(ref) // 3)
    out = torch.zeros(cut * ANN_DTYPE.itemsize, dtype=torch.uint8, device='cuda')
    cnt = torch.full((b.n,), -1, dtype=torch.int32, device='cuda')
    call('pp_pack_records', _device.ptr(b.anns), _device.ptr(b.counts), b.n, b.cap,
         _device.ptr(out), cut, _device.ptr(cnt), _device.stream())
    torch.cuda.synchronize()
    assert np.array_equal(np.diff(ref_off), cnt.cpu().numpy())
    assert out.cpu().numpy().tobytes() == ref[:cut].tobytes()
    pageable = np.zeros(cut * ANN_DTYPE.itemsize, np.uint8)
    with pytest.raises(PPError):
        call('pp_pack_records', _device.ptr(b.anns), _device.ptr(b.counts), b.n, b.cap,
             ctypes.c_void_p(pageable.ctypes.data), cut, _device.ptr(cnt), _device.stream())


def test_cifhr_sparse_poisoned_buffers():
    """Block-sparse CifHr on map / mask / workspace buffers poisoned with NaN and junk, after
    launches that leave wide-splat candidates in LDS: every tile with block 31 live once also
    marked blocks 32-63 (a sign-extended live mask) and folded a stale candidate into them.
    Bit-exact against the oracle, and no block marked that no splat box touches."""
    import ctypes
    import torch
    from openpifpaf_amd import _device, synthetic
    from openpifpaf_amd._abi import make_config
    from openpifpaf_amd._lib import call, load
    from openpifpaf_amd.decoder.cif_hr import sparse_to_dense
    lib = load()
    cfg = make_config()
    pcif, _ = synthetic.batch('planted', 8, 80, 80)
    ucif, _ = synthetic.batch('uniform', 2, 80, 80)
    rng = np.random.default_rng(5)
    wide = ucif.copy()
    wide[:, :, 4] = rng.uniform(0.5, 30.0, wide[:, :, 4].shape).astype(np.float32)
    wide[:, :, 0, 20:60, 20:60] = 0.9
    for name, cif in (('wide', wide), ('planted', pcif), ('uniform', ucif)):
        n, k, _, h, w = cif.shape
        t = int(lib.pp_cifhr_sparse_tiles(h, w, 8))
        hmap = torch.full((n, k, t, 64, 64), float('nan'), device='cuda')
        masks = torch.full((n, k, t), 0x5A5A5A5A, dtype=torch.int64, device='cuda')
        ws = torch.full((max(1, lib.pp_cifhr_sparse_workspace_size(n, k, h, w)),), 0x7F,
                        dtype=torch.uint8, device='cuda')
        dcif = torch.from_numpy(cif).cuda()
        call('pp_cifhr_sparse', _device.ptr(dcif), n, k, h, w, ctypes.byref(cfg),
             _device.ptr(hmap), _device.ptr(masks), _device.ptr(ws), ctypes.c_size_t(ws.numel()),
             _device.stream())
        hm, mk = hmap.cpu().numpy(), masks.cpu().numpy()
        assert not (mk.view(np.uint64) == 0x5A5A5A5A).any(), name  # every tile's mask written
        for i in range(n):
            ref = oracle.cifhr(cif[i], cfg)
            dense = sparse_to_dense(hm[i], mk[i], 633, 633)
            assert np.array_equal(dense, ref), (name, i)
            # marked blocks lie inside some splat box: a block no box touches is unmarked
            bits = np.unpackbits(mk[i].view(np.uint8), bitorder='little').reshape(k, t, 64)
            covered = np.zeros((k, t, 64), bool)
            keep = cif[i, :, 0] > np.float32(0.1)
            for f in range(k):
                cx = cif[i, f, 1][keep[f]] * np.float32(8)
                cy = cif[i, f, 2][keep[f]] * np.float32(8)
                sg = np.fmax(np.float32(1), (np.float32(0.5) * cif[i, f, 4][keep[f]]) * np.float32(8))
                x0 = np.clip(cx - sg, 0, 632).astype(int)
                x1 = np.clip(cx + sg + 1, x0 + 1, 633).astype(int)
                y0 = np.clip(cy - sg, 0, 632).astype(int)
                y1 = np.clip(cy + sg + 1, y0 + 1, 633).astype(int)
                for a0, a1, b0, b1 in zip(x0, x1, y0, y1):
                    for by in range(b0 // 8, (b1 - 1) // 8 + 1):
                        bx = np.arange(a0 // 8, (a1 - 1) // 8 + 1)
                        covered[f, (by // 8) * 10 + bx // 8, (by % 8) * 8 + bx % 8] = True
            assert not (bits.astype(bool) & ~covered).any(), (name, i)


def test_fetch_async_two_deep():
    """Decode i + 1 launched before decode i's records are fetched (the bench's two-deep
    pipeline): each PendingRecords returns exactly its own decode's records, including the
    re-pack when the pinned block is too small (uniform: > 16 records per image)."""
    import torch
    from openpifpaf_amd import constants, engine, synthetic
    from openpifpaf_amd._abi import EVAL_CONFIG, make_config
    cfg = make_config(**EVAL_CONFIG)
    sk = constants.COCO_PERSON_SKELETON
    batches = [synthetic.batch('planted', 6, 48, 48, first_seed=s) for s in (0, 50)]
    batches += [synthetic.batch('uniform', 6, 48, 48, first_seed=s) for s in (3, 9)]
    dev = [(torch.from_numpy(c).cuda(), torch.from_numpy(f).cuda()) for c, f in batches]
    ref = []
    for c, f in dev:
        r, off = engine.DecodeEngine().decode(c, f, sk, cfg)[:2]
        ref.append((r.copy(), off))
    eng = engine.DecodeEngine()
    for order in ((0, 1, 0, 1), (2, 3, 2, 3)):
        pending = None
        for i in order:
            b = eng.launch(*dev[i], sk, cfg)
            p = (i, eng.fetch_async(b))
            if pending is not None:
                j, q = pending
                got, off = q.result()
                assert np.array_equal(off, ref[j][1]) and got.tobytes() == ref[j][0].tobytes(), j
            pending = p
        j, q = pending
        got, off = q.result()
        assert np.array_equal(off, ref[j][1]) and got.tobytes() == ref[j][0].tobytes(), j


# ---- compact records (pp_pack_compact) -----------------------------------------------------

def _compact_vs_full(recs_full, recs_c, k=17):
    from openpifpaf_amd import constants
    from openpifpaf_amd.annotation import Annotation
    from openpifpaf_amd._abi import PP_PACK_REFETCH
    assert len(recs_full) == len(recs_c)
    assert not (recs_c['n_decoding'] & PP_PACK_REFETCH).any()
    kps, sk = constants.COCO_KEYPOINTS[:k], constants.COCO_PERSON_SKELETON
    for rf, rc in zip(recs_full, recs_c):
        a, b = Annotation.from_record(rf, kps, sk), Annotation.from_packed(rc, kps, sk)
        assert a.data.tobytes() == b.data.tobytes()
        assert a.joint_scales.tobytes() == b.joint_scales.tobytes()
        assert rf['score'] == rc['score'] and rf['image'] == rc['image']
        assert a.frontier_order == b.frontier_order
        assert len(a.decoding_order) == len(b.decoding_order)
        for (j1, k1, x1, y1), (j2, k2, x2, y2) in zip(a.decoding_order, b.decoding_order):
            assert (j1, k1) == (j2, k2)
            assert x1.tobytes() == x2.tobytes() and y1.tobytes() == y2.tobytes()


@pytest.mark.parametrize('name', CASES)
def test_compact_records_equal_full(dec, name):
    """Compact records (PP_PACK_DECODING | PP_PACK_FRONTIER) rebuild exactly the
    Annotation of the full pp_ann record, with no record flagged for a refetch."""
    from openpifpaf_amd import constants
    from openpifpaf_amd._abi import PACK_ALL
    g = gu.load_case(name)
    cif, caf, skeleton = gu.case_inputs(g)
    _configure(dec, g)
    cc = dec.CifCaf(dec.FieldConfig(), keypoints=constants.COCO_KEYPOINTS, skeleton=skeleton)
    full, off_f, _ = cc.decode_records(cif[None], caf[None])
    full = full.copy()
    comp, off_c, _ = cc.decode_records(cif[None], caf[None], compact=PACK_ALL)
    assert np.array_equal(off_f, off_c)
    assert comp.dtype.itemsize <= (0.49 if len(skeleton) == 19 else 0.63) * full.dtype.itemsize
    _compact_vs_full(full, comp)


def test_compact_records_batch_and_device_out():
    """256-image planted + 32-image uniform batches: compact records into pinned host memory
    and into device memory (the multi-GPU send buffer) equal the full records; flag subsets."""
    import torch
    from openpifpaf_amd import constants, engine, synthetic
    from openpifpaf_amd._abi import (EVAL_CONFIG, PACK_ALL, PP_PACK_DECODING, make_config,
                                     packed_dtype)
    cfg = make_config(**EVAL_CONFIG)
    sk = constants.COCO_PERSON_SKELETON
    for kind, n in (('planted', 256), ('uniform', 32)):
        cif, caf = synthetic.batch(kind, n, 80, 80, first_seed=300)
        eng = engine.DecodeEngine()
        b = eng.launch(torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda(), sk, cfg)
        full, off = eng.fetch_gather(b)
        full = full.copy()
        for flags in (PACK_ALL, PP_PACK_DECODING, 0):
            p = eng.fetch_async(b, (17, 19, flags), capacity=len(full))
            got, got_off = p.result()
            assert got.dtype == packed_dtype(17, 19, flags)
            assert np.array_equal(off, got_off)
            assert np.array_equal(got['data'], full['data'][:, :17])
            assert np.array_equal(got['score'], full['score'])
            if flags == PACK_ALL:
                _compact_vs_full(full, got)
        p = eng.fetch_async(b, (17, 19, PACK_ALL), device_out=True, capacity=len(full))
        counts = p.wait()
        assert np.array_equal(np.concatenate([[0], np.cumsum(counts)]), off)
        got = p.device_records[:len(full) * p.dtype.itemsize].cpu().numpy().view(p.dtype)
        _compact_vs_full(full, got)


def test_compact_refetch_flag():
    """A record whose decoding_order x / y differ from its data rows (or whose order is too
    long) is flagged PP_PACK_REFETCH, and PendingRecords.result() then returns the full
    records."""
    import ctypes
    import torch
    from openpifpaf_amd import _device, constants, engine, synthetic
    from openpifpaf_amd._abi import (ANN_DTYPE, EVAL_CONFIG, PACK_ALL, PP_PACK_REFETCH,
                                     make_config, packed_dtype)
    from openpifpaf_amd._lib import call
    cfg = make_config(**EVAL_CONFIG)
    sk = constants.COCO_PERSON_SKELETON
    cif, caf = synthetic.batch('planted', 4, 48, 48, first_seed=3)
    eng = engine.DecodeEngine()
    b = eng.launch(torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda(), sk, cfg)
    full, off = eng.fetch_gather(b)
    full = full.copy()
    assert off[1] >= 2
    rows = b.anns.view(b.n * b.cap, ANN_DTYPE.itemsize)
    tampered = full[:2].copy()
    tampered[0]['decoding_xyv'][0, 0] += np.float32(1.0)
    tampered[1]['n_frontier'] = 200  # > 4 * 19
    rows[:2] = torch.from_numpy(tampered.view(np.uint8).reshape(2, -1)).cuda()
    dt = packed_dtype(17, 19, PACK_ALL)
    out = torch.zeros(int(off[-1]) * dt.itemsize, dtype=torch.uint8, device='cuda')
    cnt = torch.zeros(b.n, dtype=torch.int32, device='cuda')
    flg = torch.full((b.n,), -1, dtype=torch.int32, device='cuda')
    call('pp_pack_compact', _device.ptr(b.anns), _device.ptr(b.counts), b.n, b.cap, 17, 19,
         ctypes.c_uint32(PACK_ALL), _device.ptr(out), int(off[-1]), _device.ptr(cnt),
         _device.ptr(flg), _device.stream())
    got = out.cpu().numpy().view(dt)
    flagged = (got['n_decoding'] & PP_PACK_REFETCH) != 0
    assert flagged[:2].all() and not flagged[2:].any()
    # per-image flags: image 0 holds the two tampered records
    assert flg.cpu().tolist() == [1] + [0] * (b.n - 1)
    recs, _ = eng.fetch_async(b, (17, 19, PACK_ALL)).result()
    assert recs.dtype == ANN_DTYPE and recs.tobytes() == b''.join(
        [tampered.tobytes(), full[2:].tobytes()])


def test_expand_compact_matches_full_records():
    """distributed.expand_compact (rank 0's merge when another rank sent full records)
    rebuilds every live field of the device's full pp_ann records from the compact ones."""
    import torch
    from openpifpaf_amd import constants, engine, synthetic
    from openpifpaf_amd._abi import EVAL_CONFIG, PACK_ALL, make_config
    from openpifpaf_amd.distributed import expand_compact
    cfg = make_config(**EVAL_CONFIG)
    sk = constants.COCO_PERSON_SKELETON
    cif, caf = synthetic.batch('uniform', 3, 40, 40, first_seed=11)
    eng = engine.DecodeEngine()
    b = eng.launch(torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda(), sk, cfg)
    full, _ = eng.fetch_gather(b)
    full = full.copy()
    comp, _ = eng.fetch_async(b, (17, 19, PACK_ALL)).result()
    assert len(full) > 20 and len(comp) == len(full)
    got = expand_compact(comp, 17, 19)
    for name in ('score', 'image', 'n_decoding', 'n_frontier'):
        assert np.array_equal(got[name], full[name]), name
    assert np.array_equal(got['data'][:, :17], full['data'][:, :17])
    assert np.array_equal(got['joint_scales'][:, :17], full['joint_scales'][:, :17])
    for g, f in zip(got, full):
        nd, nf = int(f['n_decoding']), int(f['n_frontier'])
        assert np.array_equal(g['decoding_pairs'][:nd], f['decoding_pairs'][:nd])
        assert g['decoding_xyv'][:nd].tobytes() == f['decoding_xyv'][:nd].tobytes()
        assert np.array_equal(g['frontier_pairs'][:nf], f['frontier_pairs'][:nf])


def test_occupancy_device_grid():
    """decoder.Occupancy on the device (pp_occupancy_set + pp_scalar_lookup) against the
    reference's set / get (occupancy.py:36-47, utils.py:61-66) restated on a NumPy grid,
    including the u8 wrap and marks on planes past the grid."""
    from openpifpaf_amd.decoder import Occupancy
    from openpifpaf_amd.functional import scalar_nonzero_clipped_with_reduction
    rng = np.random.default_rng(3)
    occ = Occupancy((5, 37, 29), 2, min_scale=4)
    ref = np.zeros((5, 18, 14), np.uint8)

    def ref_set(f, x, y, sigma):
        if f >= len(ref):
            return
        xi, yi = round(x / 2), round(y / 2)
        si = round(max(2.0, sigma / 2))
        minx, miny = max(0, int(xi - si)), max(0, int(yi - si))
        maxx = max(minx + 1, min(ref.shape[2], int(xi + si) + 1))
        maxy = max(miny + 1, min(ref.shape[1], int(yi + si) + 1))
        ref[f][miny:maxy, minx:maxx] += np.uint8(1)

    marks = [(int(rng.integers(0, 6)), np.float32(rng.uniform(-5, 40)),
              np.float32(rng.uniform(-5, 45)), np.float32(rng.uniform(0, 12)))
             for _ in range(200)]
    marks += [(1, np.float32(9.0), np.float32(11.0), np.float32(1.0))] * 260  # wraps past 255
    # Python floats divide in f64 (9.000000000000002 / 2 rounds to 5; in f32 it would be
    # 4.5 -> 4) and negative planes count from the end, as self.occupancy[f] does
    marks[:0] = [(2, 9.000000000000002, 7.0, 1.0), (-1, 20.0, 30.0, 5.0),
                 (-5, np.float32(3.0), np.float32(4.0), np.float32(9.0))]
    for m in marks[:30]:
        occ.set(*m)
        ref_set(*m)
    rest = [m for m in marks[30:] if m[0] >= 0]
    occ.mark([m[0] for m in rest], [m[1] for m in rest], [m[2] for m in rest],
             [m[3] for m in rest])
    for m in rest:
        ref_set(*m)
    assert np.array_equal(occ.occupancy.cpu().numpy(), ref)
    for _ in range(50):
        f, x, y = int(rng.integers(0, 6)), float(rng.uniform(-4, 40)), float(rng.uniform(-4, 40))
        want = 1.0 if f >= 5 else scalar_nonzero_clipped_with_reduction(ref[f], x, y, 2)
        assert occ.get(f, x, y) == want
    assert occ.get(-2, 9.0, 9.0) == scalar_nonzero_clipped_with_reduction(ref[-2], 9.0, 9.0, 2)
