"""The drop-in API surface beyond the default decode, on the device, against the
reference's own outputs (tests/golden/api_*.npz, gen_golden.gen_api) and the oracle:

  * CifCaf.__call__(fields, initial_annotations) (cifcaf.py:67-71, 95-98) through
    pp_decode_initial: the returned list holds the caller's initial Annotation objects,
    mutated, in the reference's output positions;
  * CifHr.fill_cif(min_scale) / fill_multiple over three heads and into an existing map
    (cif_hr.py:23-57), CifSeeds.fill_cif(min_scale, seed_mask) and two heads
    (cif_seeds.py:23-54), CafScored.fill_caf(min_distance, max_distance) and two calls
    (caf_scored.py:32-86) -- pp_cifhr_multi / pp_seeds_multi / pp_caf_scored_multi with a
    PP_ROLE_HRMAP geometry entry.
"""
import numpy as np
import pytest

import golden_util as gu
import oracle

pytestmark = pytest.mark.gpu

SKEL = gu.constants.COCO_PERSON_SKELETON


@pytest.fixture(scope='module')
def dec():
    from openpifpaf_amd import decoder
    return decoder


def _mode_fixture(mode):
    return {'mode': mode, 'connection_method': 'blend', 'greedy': 0}


@pytest.mark.parametrize('mode', ['eval', 'predict'])
def test_initial_annotations_vs_reference(dec, mode):
    g = gu.load_api('initial_' + mode)
    cif, caf, init_recs = gu.api_initial_inputs(g)
    gu.configure_decoder(dec, _mode_fixture(mode))
    init = gu.api_initial_annotations(g)
    cc = dec.CifCaf(dec.FieldConfig(), keypoints=gu.constants.COCO_KEYPOINTS, skeleton=SKEL)
    anns = cc([cif, caf], initial_annotations=init)
    errs = gu.compare_annotations(g, gu.annotations_as_records(anns))
    assert not errs, errs[:10]
    # the reference returns the initial objects themselves at these positions
    ident = [next((i for i, a0 in enumerate(init) if a0 is a), -1) for a in anns]
    assert ident == g['init_index'].tolist()
    # every initial object as the reference leaves it, also those NMS dropped (edited in
    # place before the filter, nms.py:20-53; the fixture's fourth one in predict mode)
    final = {'ann_' + k[6:]: v for k, v in g.items() if k.startswith('final_')}
    errs = gu.compare_annotations(final, gu.annotations_as_records(init))
    assert not errs, errs[:10]
    if mode == 'predict':
        assert len({i for i in ident if i >= 0}) < len(init)  # some were dropped
    # and bit-exact against the oracle (same exp), positions included
    ref, idx = oracle.decode_initial(cif, caf, SKEL, init_recs, gu.case_config(_mode_fixture(mode)))
    got = gu.annotations_as_records(anns)
    for name in ('data', 'joint_scales', 'n_decoding', 'n_frontier', 'decoding_pairs',
                 'decoding_xyv', 'frontier_pairs'):
        assert got[name].tobytes() == ref[name].tobytes(), name
    assert np.array_equal(np.where(idx < len(init), idx, -1), ident)


def test_initial_annotations_batch_vs_oracle():
    """A batch of 6 images (planted and uniform), each with its own initial annotations
    (0-5, from another image's decode, shifted), through engine.decode: every image's
    records and pre-NMS positions byte-equal to the oracle's."""
    from openpifpaf_amd import synthetic
    cp, ap = synthetic.batch('planted', 4, 48, 48, first_seed=30)
    cu, au = synthetic.batch('uniform', 2, 24, 24, first_seed=31)
    _initial_batch_check(((cp, ap), (cu, au)), range(6))


def test_initial_annotations_one_cu_seed_loop():
    """The same check on a batch of more than CUs / 2 images, which runs the one-CU
    seed_loop_kernel (no external helper workgroups, seed_ext_per_image = 0) instead of
    seed_loop_ext_kernel; every 9th image has initial annotations."""
    from openpifpaf_amd import synthetic
    cif, caf = synthetic.batch('planted', 136, 40, 40, first_seed=50)
    _initial_batch_check(((cif, caf),), range(0, 136, 9))


def _initial_batch_check(batches, with_init):
    import torch
    from openpifpaf_amd._abi import ANN_DTYPE, EVAL_CONFIG, make_config
    from openpifpaf_amd.engine import DecodeEngine, InitialAnnotations
    cfg = make_config(**EVAL_CONFIG)
    rng = np.random.default_rng(4)
    for cif, caf in batches:
        per_image = []
        for i in range(len(cif)):
            if i not in with_init:
                per_image.append(np.zeros(0, ANN_DTYPE))
                continue
            prev = oracle.decode(cif[(i + 1) % len(cif)], caf[(i + 1) % len(cif)], SKEL, cfg)
            take = prev[:int(rng.integers(0, min(6, len(prev)) + 1))].copy()
            take['data'][:, :, 0] += np.where(take['data'][:, :, 2] > 0, np.float32(2.5), 0)
            take['data'][:, 9:, :] = 0.0  # keep joints 0-8: the grow has work to do
            take['joint_scales'][:, 9:] = 0.0
            keep = (take['decoding_pairs'][:, :, 0] < 9) & (take['decoding_pairs'][:, :, 1] < 9)
            for r, k in zip(take, keep):
                nd = int(r['n_decoding'])
                sel = np.nonzero(k[:nd])[0]
                pairs, xyv = r['decoding_pairs'][sel].copy(), r['decoding_xyv'][sel].copy()
                r['decoding_pairs'][:] = 0
                r['decoding_xyv'][:] = 0
                r['decoding_pairs'][:len(sel)] = pairs
                r['decoding_xyv'][:len(sel)] = xyv
                r['n_decoding'] = len(sel)
            per_image.append(take)
        init = InitialAnnotations(per_image, torch.device('cuda'))
        recs, offs, b = DecodeEngine().decode(torch.from_numpy(cif).cuda(),
                                              torch.from_numpy(caf).cuda(), SKEL, cfg,
                                              initial=init)
        index = b.out_index.cpu().numpy().reshape(len(cif), -1)
        for i in range(len(cif)):
            ref, idx = oracle.decode_initial(cif[i], caf[i], SKEL, per_image[i], cfg)
            got = recs[offs[i]:offs[i + 1]]
            assert len(got) == len(ref), i
            for name in ('data', 'joint_scales', 'n_decoding', 'decoding_pairs', 'decoding_xyv',
                         'n_frontier', 'frontier_pairs'):
                assert got[name].tobytes() == ref[name].tobytes(), (i, name)
            assert np.array_equal(index[i, :len(ref)], idx), i


def _hr_check(g, tag, hr):
    hr = hr.cpu().numpy() if hasattr(hr, 'cpu') else np.asarray(hr)
    hr = np.ascontiguousarray(hr)
    assert list(hr.shape) == g[tag + '_shape'].tolist(), tag
    assert gu.sha(hr) == str(g[tag + '_sha']), tag


@pytest.mark.parametrize('where', ['host', 'device'])
def test_stage_api_vs_reference(dec, where):
    import torch
    g = gu.load_api('stages')
    heads = gu.api_stage_heads(g)
    if where == 'device':
        heads = [tuple(torch.from_numpy(f).cuda() for f in hd) for hd in heads]
    (cif, caf), (c16a, a16), (c16b, _), (c16c, _) = heads
    gu.configure_decoder(dec, _mode_fixture('eval'))
    fc = dec.FieldConfig()
    hr = dec.CifHr(fc).fill_cif(cif, 8).accumulated
    _hr_check(g, 'hr_base', hr)
    _hr_check(g, 'hr_minscale', dec.CifHr(fc).fill_cif(cif, 8, min_scale=12.0).accumulated)
    h2 = dec.CifHr(fc).fill_cif(cif, 8)
    h2.fill_multiple([c16a, c16b, c16c], 16, min_scale=10.0)
    _hr_check(g, 'hr_into', h2.accumulated)
    _hr_check(g, 'hr_three', dec.CifHr(fc).fill_multiple([c16a, c16b, c16c], 16).accumulated)

    def rows(seeds):
        return np.array([[float(t) for t in s] for s in seeds], np.float32).reshape(-1, 5)

    mask = g['seed_mask'].tolist()
    got = rows(dec.CifSeeds(hr, fc).fill_cif(cif, 8, min_scale=10.0, seed_mask=mask).get())
    assert np.array_equal(got, g['seeds_masked'])
    sd = dec.CifSeeds(hr, fc).fill_cif(cif, 8)
    sd.fill_cif(c16a, 16, min_scale=12.0)
    assert np.array_equal(rows(sd.get()), g['seeds_two'])

    def check_caf(tag, cs):
        fw = [np.ascontiguousarray(f.cpu().numpy() if hasattr(f, 'cpu') else f)
              for f in cs.forward]
        bw = [np.ascontiguousarray(b.cpu().numpy() if hasattr(b, 'cpu') else b)
              for b in cs.backward]
        assert [f.shape[1] for f in fw] == g[tag + '_fwd_counts'].tolist(), tag
        assert [gu.sha(f) for f in fw] == g[tag + '_fwd_sha'].tolist(), tag
        assert [gu.sha(b) for b in bw] == g[tag + '_bwd_sha'].tolist(), tag

    check_caf('caf_dist', dec.CafScored(hr, fc, SKEL).fill_caf(caf, 8, min_distance=24.0,
                                                               max_distance=80.0))
    cs = dec.CafScored(hr, fc, SKEL).fill_caf(caf, 8)
    cs.fill_caf(a16, 16, min_distance=20.0)
    check_caf('caf_two', cs)
    check_caf('caf_b_two', dec.CafScored(hr, fc, SKEL, score_th=0.0001).fill_caf(caf, 8).fill_caf(
        a16, 16, max_distance=200.0))


def test_fill_multiple_pairs_match_fill(dec):
    """CifHr.fill over the 10-head hflip layout equals fill_multiple pair by pair into one
    map (cif_hr.py:59-68), and a FieldConfig fill into an existing map takes that path."""
    from openpifpaf_amd import synthetic
    fields, kw = synthetic.multi_case('ms10', seed=2)
    fc = dec.FieldConfig(**kw)
    dec.CifHr.v_threshold = 0.1
    one = dec.CifHr(fc).fill(fields).accumulated
    step = dec.CifHr(fc)
    for i1, i2, stride, ms in zip(fc.cif_indices[:5], fc.cif_indices[5:], fc.cif_strides[:5],
                                  fc.cif_min_scales[:5]):
        step.fill_multiple([fields[i1], fields[i2]], stride, min_scale=ms)
    assert np.asarray(one).tobytes() == np.asarray(step.accumulated).tobytes()
    ref = oracle.cifhr_multi(oracle.Members(fields, **kw))
    assert np.asarray(one).tobytes() == ref.tobytes()


@pytest.mark.parametrize('mode', ['eval', 'predict'])
def test_seed_mask_decode_vs_reference(dec, mode):
    """CifCaf with FieldConfig(seed_mask=...) (cif_seeds.py:28-29, 63): masked fields seed
    nothing (pp_config.seed_skip_mask), through the whole device decode."""
    g = gu.load_api('seedmask_' + mode)
    cif, caf = gu.synthetic.planted(40, 40, n_people=8, seed=5)
    gu.configure_decoder(dec, _mode_fixture(mode))
    cc = dec.CifCaf(dec.FieldConfig(seed_mask=g['seed_mask'].tolist()),
                    keypoints=gu.constants.COCO_KEYPOINTS, skeleton=SKEL)
    anns = cc([cif, caf])
    errs = gu.compare_annotations(g, gu.annotations_as_records(anns))
    assert not errs, errs[:10]


@pytest.mark.parametrize('name', gu.CONFSCALE_NAMES)
def test_confidence_scales_decode_vs_reference(dec, name):
    """CifCaf(confidence_scales=...) (cifcaf.py:259-260, 282-284): the per-CAF weights on
    the frontier priorities of every _grow (seed loop and force-complete), through the
    whole device decode, against the reference (tests/golden/api_confscales_*.npz) and
    bit-exact against the oracle."""
    g = gu.load_api('confscales_' + name)
    cif, caf, skeleton = gu.case_inputs(g)
    gu.configure_decoder(dec, g)
    cc = dec.CifCaf(dec.FieldConfig(), keypoints=gu.constants.COCO_KEYPOINTS,
                    skeleton=skeleton, out_skeleton=SKEL,
                    confidence_scales=[float(v) for v in g['confidence_scales']])
    got = gu.annotations_as_records(cc([cif, caf]))
    errs = gu.compare_annotations(g, got)
    assert not errs, errs[:10]
    ref = oracle.decode(cif, caf, skeleton, gu.confscale_config(g))
    for field in ('data', 'joint_scales', 'decoding_pairs', 'decoding_xyv', 'frontier_pairs'):
        assert got[field].tobytes() == ref[field].tobytes(), field


@pytest.mark.parametrize('n_img', [6, 136])
def test_confidence_scales_batch_vs_oracle(n_img):
    """The weights on a batch: 6 images (seed_loop_ext_kernel) and 136 (the one-CU
    seed_loop_kernel), every image's records byte-equal to the oracle's."""
    import torch
    from openpifpaf_amd import synthetic
    from openpifpaf_amd._abi import EVAL_CONFIG, make_config
    from openpifpaf_amd.engine import DecodeEngine
    scales = [0.5 + 0.37 * (i % 5) for i in range(len(SKEL))]
    cfg = make_config(**dict(EVAL_CONFIG, confidence_scales=scales))
    cif, caf = synthetic.batch('planted', n_img, 40, 40, first_seed=70)
    recs, offs, _ = DecodeEngine().decode(torch.from_numpy(cif).cuda(),
                                          torch.from_numpy(caf).cuda(), SKEL, cfg)
    for i in range(n_img):
        ref = oracle.decode(cif[i], caf[i], SKEL, cfg)
        got = recs[offs[i]:offs[i + 1]]
        assert len(got) == len(ref), i
        for field in ('data', 'joint_scales', 'n_decoding', 'decoding_pairs', 'decoding_xyv',
                      'n_frontier', 'frontier_pairs'):
            assert got[field].tobytes() == ref[field].tobytes(), (i, field)


def test_custom_nms_runs_on_host(dec):
    """An NMS object other than nms.Keypoints (cifcaf.py:117-118): the device decodes
    without suppression and the object's annotations() gets each image's list; the result
    equals the nms=None decode passed through the same object, and nms=None matches the
    oracle with apply_nms off."""
    from openpifpaf_amd._abi import EVAL_CONFIG, make_config

    class KeepStrong:
        def __init__(self):
            self.calls = 0

        def annotations(self, anns):
            self.calls += 1
            return [a for a in anns if a.score() > 0.2][::-1]

    cif, caf = gu.synthetic.planted(40, 40, n_people=8, seed=5)
    gu.configure_decoder(dec, _mode_fixture('eval'))
    kw = dict(keypoints=gu.constants.COCO_KEYPOINTS, skeleton=SKEL)
    nms = KeepStrong()
    got = dec.CifCaf(dec.FieldConfig(), nms=nms, **kw)([cif, caf])
    assert nms.calls == 1
    plain = dec.CifCaf(dec.FieldConfig(), nms=None, **kw)([cif, caf])
    ref = oracle.decode(cif, caf, SKEL, make_config(**dict(EVAL_CONFIG, apply_nms=False)))
    mine = gu.annotations_as_records(plain)
    assert len(mine) == len(ref)
    for field in ('data', 'joint_scales', 'decoding_pairs', 'decoding_xyv', 'frontier_pairs'):
        assert mine[field].tobytes() == ref[field].tobytes(), field
    want = KeepStrong().annotations(plain)
    assert 0 < len(got) < len(plain)
    assert gu.annotations_as_records(got).tobytes() == gu.annotations_as_records(want).tobytes()


@pytest.mark.parametrize('extra', [{'connection_method': 'max'}, {'greedy': True},
                                   {'force_complete': False}])
def test_confidence_scales_variants_vs_oracle(extra):
    """confidence_scales with the max connection method, greedy growth (the reference
    returns a greedy entry before weighting it, cifcaf.py:280-284) and without
    force-complete: every image's records byte-equal to the oracle's (the oracle is pinned
    to the reference's api_confscales fixtures)."""
    import torch
    from openpifpaf_amd import synthetic
    from openpifpaf_amd._abi import EVAL_CONFIG, make_config
    from openpifpaf_amd.engine import DecodeEngine
    scales = [0.01 if i % 4 == 1 else 0.4 + 0.3 * (i % 3) for i in range(len(SKEL))]
    cfg = make_config(**dict(EVAL_CONFIG, confidence_scales=scales, **extra))
    cif, caf = synthetic.batch('planted', 5, 48, 48, first_seed=80)
    recs, offs, _ = DecodeEngine().decode(torch.from_numpy(cif).cuda(),
                                          torch.from_numpy(caf).cuda(), SKEL, cfg)
    for i in range(len(cif)):
        ref = oracle.decode(cif[i], caf[i], SKEL, cfg)
        got = recs[offs[i]:offs[i + 1]]
        assert len(got) == len(ref), i
        for field in ('data', 'joint_scales', 'n_decoding', 'decoding_pairs', 'decoding_xyv',
                      'n_frontier', 'frontier_pairs'):
            assert got[field].tobytes() == ref[field].tobytes(), (i, field)
