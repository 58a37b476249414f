"""Host twins of the front stages (openpifpaf_amd.stages_cpu / pp_*_cpu in
csrc/stages_cpu.hip) against the reference's own fixtures (tests/golden/decode_*.npz, made by
the reference decoder: CifHr.accumulated, CifSeeds.get(), CafScored sets at 0.1 and 1e-4),
and against each other on a batch.  CPU only."""
import numpy as np
import pytest

import golden_util as gu

CASES = gu.case_names()


@pytest.fixture(scope='module')
def sc():
    from openpifpaf_amd import stages_cpu
    return stages_cpu


@pytest.mark.parametrize('name', CASES)
def test_stages_cpu_vs_reference(sc, name):
    g = gu.load_case(name)
    cif, caf, skeleton = gu.case_inputs(g)
    cfg = gu.case_config(g)
    hh, ww = (cif.shape[2] - 1) * cfg.stride + 1, (cif.shape[3] - 1) * cfg.stride + 1
    hr = sc.cifhr(cif[None], cfg)
    assert not hr[..., ww:].any()
    assert gu.sha(hr[0, :, :hh, :ww]) == str(g['cifhr_sha'])
    seeds = sc.seeds(cif[None], hr, cfg)[0]
    rows = np.stack([seeds['v'], seeds['field'].astype(np.float32), seeds['x'], seeds['y'],
                     seeds['s']], axis=1) if len(seeds) else np.zeros((0, 5), np.float32)
    assert np.array_equal(rows, g['seeds'].reshape(-1, 5))
    for tag, th in (('a', cfg.caf_threshold), ('b', 0.0001)):
        fwd, bwd = sc.caf_scored(caf[None], hr, skeleton, th, cfg)[0]
        assert [f.shape[1] for f in fwd] == list(g['caf_%s_fwd_counts' % tag])
        assert [gu.sha(f) for f in fwd] == [str(s) for s in g['caf_%s_fwd_sha' % tag]]
        assert [gu.sha(b) for b in bwd] == [str(s) for s in g['caf_%s_bwd_sha' % tag]]


def test_stages_cpu_batch_equals_single_images(sc):
    """A batch decodes each image as a batch of one would (no state across images)."""
    from openpifpaf_amd import constants, synthetic
    from openpifpaf_amd._abi import make_config
    cfg = make_config()
    cif, caf = synthetic.batch('planted', 3, 24, 24)
    hr = sc.cifhr(cif, cfg)
    seeds = sc.seeds(cif, hr, cfg)
    sets = sc.caf_scored(caf, hr, constants.COCO_PERSON_SKELETON, 0.1, cfg)
    for i in range(3):
        h1 = sc.cifhr(cif[i:i + 1], cfg)
        assert np.array_equal(h1[0], hr[i])
        assert np.array_equal(sc.seeds(cif[i:i + 1], h1, cfg)[0], seeds[i])
        f1, b1 = sc.caf_scored(caf[i:i + 1], h1, constants.COCO_PERSON_SKELETON, 0.1, cfg)[0]
        for a, b in zip(f1 + b1, sets[i][0] + sets[i][1]):
            assert np.array_equal(a, b)
    assert sum(len(s) for s in seeds) > 0


def test_stages_cpu_errors(sc):
    from openpifpaf_amd._abi import make_config
    from openpifpaf_amd._lib import PPError
    cfg = make_config()
    with pytest.raises(ValueError):
        sc.cifhr(np.zeros((17, 5, 4, 4), np.float32), cfg)
    cif = np.zeros((1, 17, 5, 4, 4), np.float32)
    with pytest.raises(ValueError):
        sc.seeds(cif, np.zeros((1, 17, 25, 25), np.float32), cfg)
    with pytest.raises(ValueError):
        sc.caf_scored(np.zeros((1, 2, 9, 4, 4), np.float32), sc.cifhr(cif, cfg), [(1, 2)], 0.1, cfg)
    with pytest.raises(PPError, match='1-based'):
        sc.caf_scored(np.zeros((1, 1, 9, 4, 4), np.float32), sc.cifhr(cif, cfg), [(0, 2)], 0.1, cfg)


@pytest.mark.parametrize('name', ['eval', 'predict', 'supp', 'dense', 'zeros'])
def test_nms_keypoints_cpu_vs_reference(sc, name):
    """pp_nms_keypoints_cpu against nms.Keypoints runs of the reference (tests/golden/nms.npz):
    survivor order, in-place edits of every annotation, scores."""
    import os
    from openpifpaf_amd._abi import make_config
    g = np.load(os.path.join(gu.GOLDEN, 'nms.npz'))
    kt, it, sup = (float(t) for t in g[name + '_cfg'])
    cfg = make_config(nms_keypoint_threshold=kt, nms_instance_threshold=it, nms_suppression=sup)
    data = g[name + '_data_in'].astype(np.float32).copy()
    order, scores = sc.nms_keypoints(data, g[name + '_scales'].astype(np.float32), cfg)
    assert order == g[name + '_order'].tolist()
    assert np.array_equal(data, g[name + '_data_out'])
    assert np.array_equal(scores, g[name + '_score'])


@pytest.mark.parametrize('name', ['mixed', 'fixed_ties'])
def test_nms_keypoints_scored_cpu_vs_reference(sc, name):
    """pp_nms_keypoints_scored_cpu with fixed_score / suppress_score_index annotations
    against the reference's runs (tests/golden/nms_scored.npz)."""
    import os
    from openpifpaf_amd import constants
    from openpifpaf_amd._abi import make_config
    from openpifpaf_amd.annotation import Annotation
    from openpifpaf_amd.decoder.nms import _score_spec
    g = np.load(os.path.join(gu.GOLDEN, 'nms_scored.npz'))
    kt, it, sup = (float(t) for t in g[name + '_cfg'])
    anns = []
    for d, scl, fx, sp in zip(g[name + '_data_in'], g[name + '_scales'], g[name + '_fixed'],
                              g[name + '_supp']):
        a = Annotation(constants.COCO_KEYPOINTS, constants.COCO_PERSON_SKELETON,
                       suppress_score_index=None if sp == -999 else int(sp))
        if not np.isnan(fx):
            a.fixed_score = float(fx)
        anns.append(a)
    spec = _score_spec(anns, 17)
    assert spec is not None
    cfg = make_config(nms_keypoint_threshold=kt, nms_instance_threshold=it, nms_suppression=sup)
    data = g[name + '_data_in'].astype(np.float32).copy()
    order, scores = sc.nms_keypoints(data, g[name + '_scales'].astype(np.float32), cfg,
                                     score_spec=spec, instance_threshold=it)
    assert order == g[name + '_order'].tolist()
    assert np.array_equal(data, g[name + '_data_out'])
    assert np.array_equal(scores, g[name + '_score'])
