"""The host twin of the whole decode (pp_decode_batch_cpu, csrc/decode_cpu.hip;
openpifpaf_amd.stages_cpu.decode_batch): CifCaf.__call__ (cifcaf.py:67-122) with the seed
loop, _grow (cifcaf.py:247-307), complete_annotations / _flood_fill (cifcaf.py:309-351) and
nms.Keypoints (nms.py:17-57) on host threads.

Against the reference's own outputs (every decode fixture, bit for bit: golden_util's
tolerances are zero), CifCaf(confidence_scales=...) fixtures, and against the oracle on
synthetic batches (planted and uniform, eval and predict), byte for byte, with one thread
and with several."""
import numpy as np
import pytest

import golden_util as gu
import oracle
from openpifpaf_amd import constants, stages_cpu, synthetic
from openpifpaf_amd._abi import ANN_DTYPE, EVAL_CONFIG, PREDICT_CONFIG, make_config

KEYS = ('data', 'joint_scales', 'score', 'n_decoding', 'decoding_pairs', 'decoding_xyv',
        'n_frontier', 'frontier_pairs')


@pytest.mark.parametrize('name', gu.case_names())
def test_twin_vs_reference(name):
    g = gu.load_case(name)
    cif, caf, skeleton = gu.case_inputs(g)
    recs, offsets = stages_cpu.decode_batch(cif[None], caf[None], skeleton, gu.case_config(g),
                                            n_threads=1)
    assert recs.dtype == ANN_DTYPE and offsets.tolist() == [0, len(recs)]
    stats = {}
    errs = gu.compare_annotations(g, recs, stats=stats)
    assert not errs, errs[:10]


@pytest.mark.parametrize('name', gu.CONFSCALE_NAMES)
def test_twin_confidence_scales(name):
    g = gu.load_api('confscales_' + name)
    cif, caf, skeleton = gu.case_inputs(g)
    recs, _ = stages_cpu.decode_batch(cif[None], caf[None], skeleton, gu.confscale_config(g))
    assert not gu.compare_annotations(g, recs)


def _same(got, want):
    assert len(got) == len(want)
    for key in KEYS:
        assert np.array_equal(got[key], want[key]), key


@pytest.mark.parametrize('kind,mode', [('planted', 'eval'), ('uniform', 'eval'),
                                       ('planted', 'predict'), ('uniform', 'predict')])
def test_twin_vs_oracle_batch(kind, mode):
    """A 6-image 80x80 batch on 3 threads and on 1: byte-identical to each other and to
    oracle.decode of every image."""
    skel = constants.COCO_PERSON_SKELETON
    cfg = make_config(**(EVAL_CONFIG if mode == 'eval' else PREDICT_CONFIG))
    kw = {'n_caf': len(skel)} if kind == 'uniform' else {'skeleton': skel, 'n_people': 8}
    cif, caf = synthetic.batch(kind, 6, 80, 80, first_seed=40, **kw)
    recs, offsets = stages_cpu.decode_batch(cif, caf, skel, cfg, n_threads=3)
    one, off1 = stages_cpu.decode_batch(cif, caf, skel, cfg, n_threads=1)
    assert np.array_equal(offsets, off1) and recs.tobytes() == one.tobytes()
    for i in range(6):
        _same(recs[offsets[i]:offsets[i + 1]], oracle.decode(cif[i], caf[i], skel, cfg))


def test_twin_dense_skeleton_and_capacity_retry():
    """The 44-edge dense skeleton at 160x160, starting from a capacity of 4 annotations per
    image (the decode retries with doubled capacities, as the device decode does)."""
    skel = constants.DENSE_DECODE_SKELETON
    cfg = make_config(**EVAL_CONFIG)
    cif, caf = synthetic.batch('planted', 2, 160, 160, skeleton=skel, n_people=16, first_seed=7)
    recs, offsets = stages_cpu.decode_batch(cif, caf, skel, cfg, cap=4)
    assert offsets[-1] > 8
    for i in range(2):
        _same(recs[offsets[i]:offsets[i + 1]], oracle.decode(cif[i], caf[i], skel, cfg))


def test_twin_rejects_bad_arguments():
    cfg = make_config()
    cif = np.zeros((1, 17, 5, 8, 8), np.float32)
    caf = np.zeros((1, 19, 9, 8, 8), np.float32)
    with pytest.raises(ValueError):
        stages_cpu.decode_batch(cif, caf[:, :18], constants.COCO_PERSON_SKELETON, cfg)
    recs, offsets = stages_cpu.decode_batch(cif, caf, constants.COCO_PERSON_SKELETON, cfg)
    assert len(recs) == 0 and offsets.tolist() == [0, 0]
    from openpifpaf_amd._lib import PPError
    bad = np.array(constants.COCO_PERSON_SKELETON) * 0
    with pytest.raises(PPError):
        stages_cpu.decode_batch(cif, caf, bad, cfg)
