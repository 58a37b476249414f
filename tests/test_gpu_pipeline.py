"""engine.DecodePipeline (consecutive batches overlapped on two streams, two workspaces):
every batch's records are byte-identical to a one-stream DecodeEngine.decode of it."""
import numpy as np
import pytest

from openpifpaf_amd import constants, synthetic
from openpifpaf_amd._abi import EVAL_CONFIG, PACK_ALL, make_config, packed_dtype


@pytest.mark.gpu
@pytest.mark.parametrize('split', [True, False])
@pytest.mark.parametrize('b_first', [None, False, True, 'lazy'])
def test_pipeline_matches_engine_decode(b_first, split, monkeypatch):
    """Every placement of the force-complete sets (None: the density rule, which switches
    between lazy and first across these batches), the tail in one call or two."""
    import torch
    from openpifpaf_amd import engine
    from openpifpaf_amd.engine import DecodeEngine, DecodePipeline
    monkeypatch.setattr(engine, '_B_FIRST', b_first)
    monkeypatch.setattr(engine, '_SPLIT_TAIL', split)
    skel = constants.COCO_PERSON_SKELETON
    cfg = make_config(**EVAL_CONFIG)
    compact = (17, len(skel), PACK_ALL)
    batches = []
    for i, kind in enumerate(('planted', 'uniform', 'planted', 'planted', 'uniform')):
        kw = {'n_caf': len(skel)} if kind == 'uniform' else {'skeleton': skel, 'n_people': 8}
        cif, caf = synthetic.batch(kind, 8, 40, 40, first_seed=100 * i, **kw)
        batches.append((torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda()))
    eng = DecodeEngine()
    want = []
    for cif, caf in batches:
        recs, offsets, _ = eng.decode(cif, caf, skel, cfg, cap=1024, compact=PACK_ALL)
        want.append((recs.tobytes(), offsets.copy()))
    pipe = DecodePipeline()
    pend = [pipe.submit(cif, caf, skel, cfg, cap=1024, compact=compact)[1]
            for cif, caf in batches]  # all five in flight before any result is read
    for (w_bytes, w_off), p in zip(want, pend):
        recs, offsets = p.result()
        np.testing.assert_array_equal(offsets, w_off)
        assert recs.tobytes() == w_bytes


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['ms2', 'ms10'])
def test_pipeline_multi_scale_matches_engine_decode(name):
    """The pipeline over multi-scale HeadSets (pp_decode_multi, stage by stage on three
    streams) gives the one-stream records byte for byte."""
    import torch
    from openpifpaf_amd.decoder import FieldConfig
    from openpifpaf_amd.engine import DecodeEngine, DecodePipeline, HeadSet
    skel = constants.COCO_PERSON_SKELETON
    cfg = make_config(**EVAL_CONFIG)
    sets = []
    for rep in range(3):
        per = [synthetic.multi_case(name, seed=10 * rep + i, h_px=161, w_px=161, n_people=4)
               for i in range(4)]
        fields = [torch.from_numpy(np.stack([p[0][j] for p in per])).cuda()
                  for j in range(len(per[0][0]))]
        sets.append(HeadSet(fields, FieldConfig(**per[0][1])))
    eng = DecodeEngine()
    want = []
    for heads in sets:
        recs, offsets, _ = eng.decode(None, None, skel, cfg, cap=512, heads=heads,
                                      compact=PACK_ALL)
        want.append((recs.tobytes(), offsets.copy()))
    pipe = DecodePipeline()
    pend = [pipe.submit(None, None, skel, cfg, cap=512, heads=heads,
                        compact=(heads.k, len(skel), PACK_ALL))[1] for heads in sets]
    for (w_bytes, w_off), p in zip(want, pend):
        recs, offsets = p.result()
        np.testing.assert_array_equal(offsets, w_off)
        assert recs.tobytes() == w_bytes


@pytest.mark.gpu
@pytest.mark.parametrize('n_img', [8, 136])
def test_pipeline_wide_nms_matches_engine_decode(n_img):
    """Dense batches in the pipeline take the 8-wave NMS (PP_STAGE_NMS_WIDE) when the batch
    runs the one-CU seed loop (136 images; 8 images keep the 4-wave form): records byte for
    byte as the one-stream decode with the default 4-wave NMS."""
    import torch
    from openpifpaf_amd.engine import DecodeEngine, DecodePipeline
    skel = constants.COCO_PERSON_SKELETON
    cfg = make_config(**EVAL_CONFIG)
    cif, caf = synthetic.batch('uniform', n_img, 40, 40, first_seed=7, n_caf=len(skel))
    cif, caf = torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda()
    recs0, off0, _ = DecodeEngine().decode(cif, caf, skel, cfg, cap=1024, compact=PACK_ALL)
    assert off0[-1] / n_img >= 32  # dense: the pipeline's rule picks the wide NMS
    pipe = DecodePipeline()
    pipe.density = float(off0[-1]) / n_img
    pend = [pipe.submit(cif, caf, skel, cfg, cap=1024, compact=(17, len(skel), PACK_ALL))[1]
            for _ in range(3)]
    for p in pend:
        recs, offsets = p.result()
        np.testing.assert_array_equal(offsets, off0)
        assert recs.tobytes() == recs0.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize('kind', ['planted', 'uniform', 'far'])
def test_nms_bitmap_matches_box_lists(kind):
    """PP_STAGE_NMS_BITMAP (the occupancy planes as LDS bitmaps, one wave per (image, plane),
    nms_planes_kernel) gives the single-launch NMS's records byte for byte; 'far' moves CAF
    targets far right so force-complete puts joints beyond the bitmap's grid, which those
    planes decide with the box lists instead."""
    import torch
    from openpifpaf_amd.engine import STAGE_ALL, STAGE_NMS_BITMAP, DecodeEngine
    skel = constants.COCO_PERSON_SKELETON
    cfg = make_config(**EVAL_CONFIG)
    kw = {'n_caf': len(skel)} if kind == 'uniform' else {'skeleton': skel, 'n_people': 8}
    cif, caf = synthetic.batch('uniform' if kind == 'uniform' else 'planted', 6, 40, 40,
                               first_seed=31, **kw)
    if kind == 'far':
        caf[:, 3:6, 5, :, 20:] += 120.0  # x2 of three limbs, right half of the field
    cif, caf = torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda()
    recs = []
    for stages in (STAGE_ALL, STAGE_ALL | STAGE_NMS_BITMAP):
        eng = DecodeEngine()
        b = eng.launch(cif, caf, skel, cfg, cap=1024, stages=stages)
        r, off = DecodeEngine.fetch(b, (17, len(skel), PACK_ALL))
        recs.append((r.tobytes(), off.copy(), b.status.cpu().numpy().copy()))
    assert not recs[0][2].any()
    np.testing.assert_array_equal(recs[0][1], recs[1][1])
    assert recs[0][0] == recs[1][0]
    if kind == 'far':
        r = np.frombuffer(recs[0][0], dtype=packed_dtype(17, len(skel), PACK_ALL))
        assert (r['data'][:, :, 0] > 400).any()  # joints beyond the nominal 160-px map


@pytest.mark.gpu
def test_seed_loop_only_twice_then_decode():
    """The workspace contract after a split stage 8: two PP_STAGE_SEED_LOOP_ONLY
    calls on one workspace with external helper workgroups (8 images: n_ext 3), with no
    force-complete or NMS call between or after them, then a whole decode of another batch
    on the same workspace: its records equal a fresh engine's byte for byte, so the
    external-helper hand-off words the seed loops left (SeedExt) were zero again.  Nothing
    is skipped in the checked decode."""
    import torch
    from openpifpaf_amd.engine import (STAGE_CAF, STAGE_CIFHR, STAGE_GROW, STAGE_SEEDS,
                                       STAGE_SEED_LOOP_ONLY, DecodeEngine)
    skel = constants.COCO_PERSON_SKELETON
    cfg = make_config(**EVAL_CONFIG)
    fields = []
    for i, kind in enumerate(('planted', 'uniform', 'planted')):
        kw = {'n_caf': len(skel)} if kind == 'uniform' else {'skeleton': skel, 'n_people': 8}
        cif, caf = synthetic.batch(kind, 8, 80, 80, first_seed=300 + 10 * i, **kw)
        fields.append((torch.from_numpy(cif).cuda(), torch.from_numpy(caf).cuda()))
    eng = DecodeEngine()
    for cif, caf in fields[:2]:
        eng.launch(cif, caf, skel, cfg, cap=1024, stages=STAGE_CIFHR | STAGE_SEEDS | STAGE_CAF)
        eng.launch(cif, caf, skel, cfg, cap=1024, stages=STAGE_GROW | STAGE_SEED_LOOP_ONLY)
    torch.cuda.synchronize()
    got, got_off, _ = eng.decode(*fields[2], skel, cfg, cap=1024, compact=PACK_ALL)
    want, want_off, _ = DecodeEngine().decode(*fields[2], skel, cfg, cap=1024, compact=PACK_ALL)
    np.testing.assert_array_equal(got_off, want_off)
    assert got.tobytes() == want.tobytes()
    # and the first batch again, whole, on the same workspace
    got1, off1, _ = eng.decode(*fields[0], skel, cfg, cap=1024, compact=PACK_ALL)
    want1, woff1, _ = DecodeEngine().decode(*fields[0], skel, cfg, cap=1024, compact=PACK_ALL)
    np.testing.assert_array_equal(off1, woff1)
    assert got1.tobytes() == want1.tobytes()
