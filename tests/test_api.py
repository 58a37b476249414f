"""Host-side API behaviour that needs no GPU: boundary errors (the reference's Cython
messages), configuration plumbing, synthetic generators."""
import argparse

import numpy as np
import pytest

import golden_util as gu
from openpifpaf_amd import functional as F
from openpifpaf_amd import synthetic
from openpifpaf_amd._abi import make_config


def test_error_messages_match_reference():
    errs = gu.load_errors()
    p = np.zeros(2, np.float32)
    with pytest.raises(ValueError) as e:
        F.scalar_square_add_gauss_with_max(np.zeros((4, 4)), p, p, p, p)
    assert [type(e.value).__name__, str(e.value)] == errs['dtype']
    ro = np.zeros((4, 4), np.float32)
    ro.setflags(write=False)
    with pytest.raises(ValueError) as e:
        F.scalar_values(ro, p, p)
    assert [type(e.value).__name__, str(e.value)] == errs['readonly']
    with pytest.raises(ValueError) as e:
        F.scalar_values(np.zeros((2, 4, 4), np.float32), p, p)
    assert [type(e.value).__name__, str(e.value)] == errs['ndim']
    with pytest.raises(ValueError) as e:
        F.weiszfeld_nd(np.zeros((3, 2), np.float32), np.zeros(2, np.float32))
    assert [type(e.value).__name__, str(e.value)] == errs['weiszfeld_none']
    with pytest.raises(ValueError) as e:
        F.scalar_values(np.zeros((4, 4), np.float32), np.zeros((2, 2), np.float32), p)
    assert [type(e.value).__name__, str(e.value)] == errs['ndim_points']


def test_no_cpu_fallback():
    """Without a HIP device the product path raises instead of computing on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip('a GPU is visible')
    from openpifpaf_amd._lib import PPError
    f = np.zeros((8, 8), np.float32)
    p = np.ones(1, np.float32)
    with pytest.raises(PPError):
        F.scalar_square_add_gauss_with_max(f, p, p, p, p)


def test_configure_writes_class_attributes():
    from openpifpaf_amd import decoder
    parser = argparse.ArgumentParser()
    decoder.cli(parser, force_complete_pose=False, instance_threshold=0.1, seed_threshold=0.5)
    args = parser.parse_args([])
    args.debug = False
    decoder.configure(args)
    assert decoder.CifSeeds.threshold == 0.5
    assert decoder.CifCaf.force_complete is False
    assert decoder.CifCaf.keypoint_threshold == 0.001
    assert decoder.nms.Keypoints.instance_threshold == 0.1
    cc = decoder.CifCaf(decoder.FieldConfig(), keypoints=list('abcdefghijklmnopq'),
                        skeleton=[(1, 2), (2, 3)])
    cfg = cc.config()
    assert cfg.seed_threshold == pytest.approx(0.5)
    assert cfg.force_complete == 0
    assert cfg.apply_nms == 1
    args = parser.parse_args(['--force-complete-pose', '--seed-threshold', '0.2',
                              '--instance-threshold', '0.0', '--keypoint-threshold', '0.0'])
    args.debug = False
    decoder.configure(args)
    assert decoder.CifCaf.force_complete is True


def test_by_source_tables_follow_dict_order():
    from openpifpaf_amd import constants, decoder
    cc = decoder.CifCaf(decoder.FieldConfig(), keypoints=constants.COCO_KEYPOINTS,
                        skeleton=constants.COCO_PERSON_SKELETON)
    # joint 5 (left shoulder, 0-based) appears in edges (6,12), (6,7), (6,8), (4,6)
    assert list(cc.by_source[5].keys()) == [11, 6, 7, 3]


def test_unsupported_configurations_raise():
    from openpifpaf_amd import decoder
    fc = decoder.FieldConfig(cif_indices=[0, 3], caf_indices=[1, 4], cif_strides=[8, 16],
                             caf_strides=[8, 16], cif_min_scales=[0.0, 12.0],
                             caf_min_distances=[0.0, 36.0], caf_max_distances=[None, None])
    with pytest.raises(NotImplementedError):
        fc.single_scale()
    with pytest.raises(IndexError):  # one weight per CAF (cifcaf.py:260, 284)
        decoder.CifCaf(decoder.FieldConfig(), keypoints=['a', 'b'], skeleton=[(1, 2), (2, 1)],
                       confidence_scales=[1.0])
    cc = decoder.CifCaf(decoder.FieldConfig(), keypoints=['a', 'b'], skeleton=[(1, 2)],
                        confidence_scales=[0.1])
    assert cc.confidence_scales == [0.1]
    cfg = make_config(confidence_scales=cc.confidence_scales)
    assert cfg.confidence_scales[0] == np.float32(0.1)
    assert not make_config().confidence_scales
    with pytest.raises(TypeError):  # cifcaf.py:117-118 calls nms.annotations
        decoder.CifCaf(decoder.FieldConfig(), keypoints=['a'], skeleton=[(1, 1)], nms=object())


def test_nms_objects_choose_device_or_host():
    """nms.Keypoints runs inside the device decode (pp_config.apply_nms); another object
    with annotations() runs on the host over the unsuppressed device list."""
    from openpifpaf_amd import decoder

    class Top2:
        def annotations(self, anns):
            return sorted(anns, key=lambda a: -a.score())[:2]

    class Sub(decoder.nms.Keypoints):
        instance_threshold = 0.25

    class Own(decoder.nms.Keypoints):
        def annotations(self, anns):
            return anns[:1]

    kw = dict(keypoints=['a', 'b'], skeleton=[(1, 2)])
    old = decoder.CifSeeds.threshold
    decoder.CifSeeds.threshold = 0.2
    try:
        dev = decoder.CifCaf(decoder.FieldConfig(), **kw)
        assert dev._device_nms() and dev.config().apply_nms == 1
        sub = decoder.CifCaf(decoder.FieldConfig(), nms=Sub(), **kw)
        assert sub._device_nms() and sub.config().nms_instance_threshold == np.float32(0.25)
        for nms in (Top2(), Own()):
            host = decoder.CifCaf(decoder.FieldConfig(), nms=nms, **kw)
            assert not host._device_nms() and host.config().apply_nms == 0
            stubs = [argparse.Namespace(score=lambda v=v: v) for v in (0.3, 0.9, 0.5)]
            assert host._host_nms(stubs) == nms.annotations(stubs)
        off = decoder.CifCaf(decoder.FieldConfig(), nms=None, **kw)
        assert off.config().apply_nms == 0 and off._host_nms([3, 1]) == [3, 1]
    finally:
        decoder.CifSeeds.threshold = old


def test_generators_deterministic():
    a = synthetic.planted(40, 40, seed=3)
    b = synthetic.planted(40, 40, seed=3)
    assert synthetic.digest(*a) == synthetic.digest(*b)
    c, f = synthetic.uniform(16, 21, seed=0)
    assert c.shape == (17, 5, 16, 21) and f.shape == (19, 9, 16, 21)
    cb, fb = synthetic.batch('uniform', 3, 10, 10, first_seed=5)
    assert np.array_equal(cb[1], synthetic.uniform(10, 10, seed=6)[0])


def test_make_config_rejects_unknown_method():
    with pytest.raises(Exception):
        make_config(connection_method='nearest')


# ---- decoder factory (decoder/factory.py:100-213), construction only -----------------------

def _args(extra=()):
    from openpifpaf_amd import decoder
    parser = argparse.ArgumentParser()
    decoder.cli(parser)
    args = parser.parse_args(list(extra))
    args.debug = False
    return args


def test_configure_detection_threshold_and_workers():
    from openpifpaf_amd import decoder
    args = _args(['--instance-threshold', '0.25', '--no-force-complete-pose'])
    args.batch_size = 8
    decoder.configure(args)
    assert decoder.nms.Detection.instance_threshold == 0.25
    assert decoder.nms.Keypoints.instance_threshold == 0.25
    assert args.decoder_workers == 8  # factory.py:93-98
    args = _args()
    args.batch_size = 1
    decoder.configure(args)
    assert args.decoder_workers is None


def test_factory_decode_variants():
    import factory_util as fu
    from openpifpaf_amd import constants, decoder
    cc = decoder.factory_decode([fu.cif_head(), fu.caf_head()], basenet_stride=16)
    assert isinstance(cc, decoder.CifCaf) and cc.field_config.is_single_scale()
    assert cc.skeleton == constants.COCO_PERSON_SKELETON
    # dense connections: skeleton extended in place with the 25 denser edges (factory.py:182-188)
    heads = [fu.cif_head(), fu.caf_head(), fu.caf25_head()]
    cc = decoder.factory_decode(heads, basenet_stride=16, dense_connections=True,
                                dense_coupling=0.01)
    assert len(cc.skeleton) == 44 and cc.skeleton == constants.DENSE_DECODE_SKELETON
    assert cc.field_config.confidence_scales == [1.0] * 19 + [0.01] * 25
    # multi-scale, no hflip: 5 scales of (cif, caf, caf25)
    strides = [8, 16, 8, 16, 8]
    cc = decoder.factory_decode(fu.multi_heads(strides), basenet_stride=16, multi_scale=True,
                                multi_scale_hflip=False)
    fc = cc.field_config
    assert fc.cif_indices == [0, 3, 6, 9, 12] and fc.caf_indices == [1, 4, 7, 10, 13]
    assert fc.cif_strides == strides and fc.caf_strides == strides
    assert fc.cif_min_scales == [0.0, 12.0, 16.0, 24.0, 40.0]
    assert fc.caf_min_distances == [0.0, 36.0, 48.0, 72.0, 120.0]
    assert fc.caf_max_distances == [160.0, 240.0, 320.0, 480.0, None]
    # multi-scale with hflip: 10 heads, lists repeated (factory.py:169-180)
    cc = decoder.factory_decode(fu.multi_heads(strides * 2), basenet_stride=16, multi_scale=True)
    fc = cc.field_config
    assert fc.cif_indices == [3 * v for v in range(10)]
    assert fc.cif_min_scales == [0.0, 12.0, 16.0, 24.0, 40.0] * 2
    assert fc.caf_max_distances == [160.0, 240.0, 320.0, 480.0, None] * 2
    # detection heads -> CifDet
    cd = decoder.factory_decode([fu.det_head(['a', 'b'])], basenet_stride=16)
    assert isinstance(cd, decoder.CifDet) and cd.categories == ['a', 'b']
    with pytest.raises(Exception):
        decoder.factory_decode([fu.caf_head()], basenet_stride=16)


def test_factory_from_args_profile_decoder(tmp_path):
    import types
    import factory_util as fu
    from openpifpaf_amd import decoder
    from openpifpaf_amd.decoder.profiler import Profiler, ProfilerAutograd
    args = _args(['--profile-decoder', str(tmp_path / 'dec.prof')])
    model = types.SimpleNamespace(head_nets=[fu.cif_head(), fu.caf_head()],
                                  base_net=types.SimpleNamespace(stride=16))
    cls_call = decoder.CifCaf.__call__
    try:
        dec = decoder.factory_from_args(args, model)
        assert isinstance(type(dec).__call__, Profiler)
        assert isinstance(dec.fields_batch, ProfilerAutograd)
        out = Profiler(lambda x: x + 1, out_name=str(tmp_path / 'p.prof'))(1)
        assert out == 2 and (tmp_path / 'p.prof').exists()
    finally:
        decoder.CifCaf.__call__ = cls_call


def test_fields_batch_indexes_by_image():
    """Generator.fields_batch (generator.py:43-78): one entry per image, each the model's
    nested head list indexed by that image (None kept); the reference's .cpu().numpy() copy
    is skipped, so the entries are views of the model's outputs."""
    import torch
    from openpifpaf_amd.decoder.generator.generator import Generator

    heads = [torch.arange(3 * 4.0).reshape(3, 4), None,
             (torch.zeros(3, 2, 5), [torch.ones(4, 1)])]

    def model(image_batch):
        assert image_batch.shape[0] == 3
        return heads

    out = Generator.fields_batch(model, torch.zeros(3, 3, 8, 8))
    assert len(out) == 3  # the shortest batch dimension (the reference stops there)
    for i, f in enumerate(out):
        assert torch.equal(f[0], heads[0][i]) and f[1] is None
        assert f[2][0].shape == (2, 5) and torch.equal(f[2][1][0], heads[2][1][0][i])
        assert f[0].data_ptr() == heads[0][i].data_ptr()  # a view, not a copy


def test_short_seed_mask_raises_index_error():
    """The reference reads seed_mask[field_i] for every field (cif_seeds.py:28-29): a mask
    shorter than K raises IndexError on every path."""
    from openpifpaf_amd import constants, decoder
    from openpifpaf_amd._abi import check_seed_mask
    decoder.CifSeeds.threshold = 0.2
    cc = decoder.CifCaf(decoder.FieldConfig(seed_mask=[1] * 5),
                        keypoints=constants.COCO_KEYPOINTS,
                        skeleton=constants.COCO_PERSON_SKELETON)
    with pytest.raises(IndexError):
        cc.config()
    check_seed_mask([1] * 17, 17)
    check_seed_mask(None, 17)
    with pytest.raises(IndexError):
        check_seed_mask([0] * 16, 17)


def test_nms_score_spec_host_logic():
    """nms.Keypoints' per-annotation score() inputs for pp_nms_keypoints_scored."""
    from openpifpaf_amd import constants
    from openpifpaf_amd.annotation import Annotation
    from openpifpaf_amd.decoder.nms import _score_spec

    def ann(**kw):
        return Annotation(constants.COCO_KEYPOINTS, constants.COCO_PERSON_SKELETON, **kw)

    assert _score_spec([ann(), ann()], 17) is None  # default score(): the plain entry
    a_fixed, a_last, a_zero = ann(), ann(suppress_score_index=-1), ann(suppress_score_index=0)
    a_fixed.fixed_score = 0.25
    spec, sw, fixed = _score_spec([ann(), a_fixed, a_last, a_zero], 17)
    assert spec.tolist() == [-1, -2, 16, 0]
    assert fixed[1] == 0.25
    assert sw[2, 16] == 0.0 and sw[3, 16] > 0.0  # `if suppress_score_index:` (annotation.py:25)
    assert np.array_equal(sw[0], ann().score_weights)
    with pytest.raises(IndexError):
        _score_spec([ann(suppress_score_index=17)], 17)
