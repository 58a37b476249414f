"""The reference's construction path on the device: factory_decode (decoder/factory.py:
122-213) for single-scale, dense-connection, multi-scale (hflip and not) and detection
heads, decoding through Generator.batch (generator.py:84-101) with a stub model whose
head outputs are resident device tensors; results against the reference's fixtures or
the oracle."""
import os

import numpy as np
import pytest

import factory_util as fu
import golden_util as gu
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dec():
    from openpifpaf_amd import decoder
    return decoder


class StubModel:
    """model(image_batch) -> the head outputs (each (B, ...)), as a network would return."""

    def __init__(self, outputs):
        self.outputs = outputs
        self.calls = 0

    def __call__(self, image_batch):
        self.calls += 1
        return self.outputs


def _dev(arrays):
    import torch
    return [None if a is None else torch.from_numpy(np.ascontiguousarray(a)).cuda()
            for a in arrays]


@pytest.mark.parametrize('name', ['p80_s0_eval', 'u20_s0_eval', 'p40_s0_predict',
                                  'p40_s3_max', 'p160_s0_dense_eval', 'u160_s0_dense_eval'])
def test_factory_batch_vs_reference(dec, name):
    import torch
    g = gu.load_case(name)
    cif, caf, skeleton = gu.case_inputs(g)
    gu.configure_decoder(dec, g)
    dense = len(skeleton) == 44
    heads = [fu.cif_head(), fu.caf_head()] + ([fu.caf25_head()] if dense else [])
    cc = dec.factory_decode(heads, basenet_stride=16, dense_connections=dense)
    assert list(map(tuple, cc.skeleton)) == [tuple(e) for e in skeleton]
    # the collector concatenates caf + caf25 into one CAF head (heads.py:65-88)
    model = StubModel(_dev([np.stack([cif] * 3), np.stack([caf] * 3)]))
    result = cc.batch(model, torch.zeros(3, 3, 16, 16))
    assert model.calls == 1 and len(result) == 3 and cc.last_decoder_time > 0
    for anns in result:
        stats = {}
        errs = gu.compare_annotations(g, gu.annotations_as_records(anns), stats=stats)
        assert not errs, errs[:10]
    print('max deviation vs reference:', stats)


def _multi_fields(fields, n_scales, per=3):
    """[cif_0, caf_0, cif_1, ...] -> the reference model layout of `per` heads per scale."""
    out = [None] * (per * n_scales)
    for i in range(n_scales):
        out[per * i], out[per * i + 1] = fields[2 * i], fields[2 * i + 1]
    return out


@pytest.mark.parametrize('mode', ['eval', 'predict'])
def test_factory_multi_scale_hflip_vs_reference(dec, mode):
    import torch
    from openpifpaf_amd import synthetic
    g = np.load(os.path.join(gu.GOLDEN, 'multi_ms10_%s.npz' % mode))
    fields, kw = synthetic.multi_case('ms10')
    assert gu.sha(*fields) == str(g['input_sha'])
    gu.configure_decoder(dec, g)
    cc = dec.factory_decode(fu.multi_heads(kw['cif_strides']), basenet_stride=16,
                            multi_scale=True, multi_scale_hflip=True)
    fc = cc.field_config
    for key in ('cif_strides', 'caf_strides', 'cif_min_scales', 'caf_min_distances',
                'caf_max_distances'):
        assert list(getattr(fc, key)) == list(kw[key]), key
    outputs = _dev([None if f is None else f[None] for f in _multi_fields(fields, 10)])
    result = cc.batch(StubModel(outputs), torch.zeros(1, 3, 8, 8))
    errs = gu.compare_annotations(g, gu.annotations_as_records(result[0]))
    assert not errs, errs[:10]


def test_factory_multi_scale_no_hflip_vs_oracle(dec):
    import torch
    from openpifpaf_amd import constants, synthetic
    from openpifpaf_amd._abi import EVAL_CONFIG, make_config
    gu.configure_decoder(dec, {'mode': np.array('eval'), 'greedy': 0,
                               'connection_method': np.array('blend')})
    strides = [8, 16, 8, 16, 8]
    imgs = [synthetic.planted_multi(321, 321, strides, n_people=5, seed=40 + s) for s in range(3)]
    per_image = [[a for pair in heads for a in pair] for heads in imgs]  # cif_0, caf_0, ...
    cc = dec.factory_decode(fu.multi_heads(strides), basenet_stride=16, multi_scale=True,
                            multi_scale_hflip=False)
    stacked = [np.stack([p[j] for p in per_image]) for j in range(10)]
    outputs = _dev(_multi_fields(stacked, 5))
    result = cc.batch(StubModel(outputs), torch.zeros(3, 3, 8, 8))
    fc = cc.field_config
    kw = dict(cif_indices=[2 * i for i in range(5)], caf_indices=[2 * i + 1 for i in range(5)],
              cif_strides=fc.cif_strides, caf_strides=fc.caf_strides,
              cif_min_scales=fc.cif_min_scales, caf_min_distances=fc.caf_min_distances,
              caf_max_distances=fc.caf_max_distances)
    total = 0
    for i, anns in enumerate(result):
        ref = oracle.decode_multi(oracle.Members(per_image[i], **kw),
                                  constants.COCO_PERSON_SKELETON, make_config(**EVAL_CONFIG))
        got = gu.annotations_as_records(anns)
        assert len(got) == len(ref)
        for r, o in zip(got, ref):
            for key in ('data', 'joint_scales', 'score', 'decoding_pairs', 'decoding_xyv',
                        'frontier_pairs'):
                assert np.array_equal(r[key][:17] if key in ('data', 'joint_scales') else r[key],
                                      o[key][:17] if key in ('data', 'joint_scales') else o[key]), key
        total += len(got)
    assert total > 6


@pytest.mark.parametrize('name', ['dp40_s0', 'du20_s0'])
def test_factory_cifdet_batch_vs_reference(dec, name):
    import torch
    from openpifpaf_amd import synthetic
    g = np.load(os.path.join(gu.GOLDEN, 'det_%s.npz' % name))
    det = synthetic.det_batch(str(g['gen']), 1, int(g['h']), int(g['w']),
                              first_seed=int(g['seed']), n_categories=int(g['n_categories']))[0]
    assert gu.sha(det) == str(g['input_sha'])
    dec.CifHr.v_threshold = 0.1
    dec.CifSeeds.threshold = float(g['seed_threshold'])
    k = int(g['n_categories'])
    cd = dec.factory_decode([fu.det_head(['c%d' % i for i in range(k)])], basenet_stride=16)
    result = cd.batch(StubModel(_dev([np.stack([det, det])])), torch.zeros(2, 3, 8, 8))
    for anns in result:
        assert [a.field_i for a in anns] == g['ann_field'].tolist()
        assert np.array_equal(np.array([a.score for a in anns], np.float32), g['ann_score'])
        assert np.array_equal(np.array([a.bbox for a in anns], np.float32).reshape(-1, 4),
                              g['ann_bbox'])
