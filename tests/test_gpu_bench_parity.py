"""The bench's own decode paths against the oracle, at the bench's batch sizes.

bench.py decodes its workloads through engine.DecodePipeline, whose kernel choices depend
on the batch: 256 images take the one-CU seed loop (seed_loop_kernel), dense batches (the
pipeline's density hint >= 32 annotations per image) build the force-complete sets first
and run the 8-wave NMS; 64-image cfg5 batches take the seed loop with external helper
workgroups (seed_loop_ext_kernel) and the 4-wave NMS.  These tests run exactly those
batches (synthetic.batch with the bench's arguments and seeds) through the pipeline and
compare sampled images with oracle.decode byte for byte (data, joint scales, score,
decoding / frontier order).  Reference: decoder/generator/cifcaf.py:67-122,333-351,
decoder/nms.py:17-57 (the oracle restates them, pinned by tests/test_oracle_golden.py).
"""
import concurrent.futures
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

KEYS = ('data', 'joint_scales', 'score', 'n_decoding', 'decoding_pairs', 'decoding_xyv',
        'n_frontier', 'frontier_pairs')


def _pipeline_decode(cif_h, caf_h, skel, density, repeats=2):
    """Decode one resident batch `repeats` times through a DecodePipeline whose density
    hint is `density` (what the bench's warmup steps leave it at); returns the records of
    the last submission (expanded to pp_ann) and per-image offsets, after checking that
    every submission gave the same bytes."""
    import torch
    from openpifpaf_amd._abi import ANN_DTYPE, EVAL_CONFIG, PACK_ALL, make_config
    from openpifpaf_amd.distributed import expand_compact
    from openpifpaf_amd.engine import DecodePipeline
    cif, caf = torch.from_numpy(cif_h).cuda(), torch.from_numpy(caf_h).cuda()
    cfg = make_config(**EVAL_CONFIG)
    pipe = DecodePipeline()
    pipe.density = density
    pend = [pipe.submit(cif, caf, skel, cfg, compact=(cif.shape[1], len(skel), PACK_ALL))[1]
            for _ in range(repeats)]
    results = []
    for p in pend:
        pipe_density = pipe.density
        recs, offsets = p.result()
        pipe.density = pipe_density  # keep the hint for the submissions already queued
        # raw bytes: ndarray.copy() of a dtype with padding leaves the holes uninitialised
        results.append((recs.tobytes(), recs.dtype, offsets.copy()))
    raw, dtype, offsets = results[-1]
    for r, _, o in results[:-1]:
        np.testing.assert_array_equal(o, offsets)
        assert r == raw
    recs = np.frombuffer(raw, dtype=dtype)
    if recs.dtype != ANN_DTYPE:
        recs = expand_compact(recs)
    return recs, offsets


def _check_images(cif_h, caf_h, skel, recs, offsets, images):
    """oracle.decode of each listed image (on host threads: ctypes drops the GIL) against
    the device records, byte for byte."""
    from openpifpaf_amd._abi import EVAL_CONFIG, make_config
    cfg = make_config(**EVAL_CONFIG)
    oracle.lib()
    threads = max(1, min(8, len(images), (os.cpu_count() or 1)))
    with concurrent.futures.ThreadPoolExecutor(threads) as ex:
        refs = list(ex.map(lambda i: oracle.decode(cif_h[i], caf_h[i], skel, cfg), images))
    for i, ref in zip(images, refs):
        got = recs[offsets[i]:offsets[i + 1]]
        assert len(got) == len(ref), (i, len(got), len(ref))
        for r, o in zip(got, ref):
            for key in KEYS:
                assert np.array_equal(r[key], o[key]), (i, key)
    return sum(len(r) for r in refs)


def test_cfg3_uniform_bench_batch():
    """bench.py's uniform cfg3 line: 256 x 80x80 uniform images (synthetic.batch('uniform',
    256, 80, 80), ~400 annotations per image) through the pipeline with the dense hint: the
    one-CU seed loop, force-complete sets first, the 8-wave NMS.  8 spread images checked."""
    from openpifpaf_amd import constants, synthetic
    skel = constants.COCO_PERSON_SKELETON
    cif_h, caf_h = synthetic.batch('uniform', 256, 80, 80, n_caf=len(skel))
    recs, offsets = _pipeline_decode(cif_h, caf_h, skel, density=400.0)
    assert offsets[-1] / 256 >= 32  # dense: the rule that picks sets-first and the wide NMS
    n = _check_images(cif_h, caf_h, skel, recs, offsets, list(range(0, 256, 32))[::-1][:8])
    assert n > 8 * 300


def test_cfg3_planted_bench_batch():
    """The headline batch (256 x 80x80 planted, eval) through the pipeline with the sparse
    hint (lazy force-complete sets, 4-wave NMS): 32 spread images against the oracle."""
    from openpifpaf_amd import constants, synthetic
    skel = constants.COCO_PERSON_SKELETON
    cif_h, caf_h = synthetic.batch('planted', 256, 80, 80, skeleton=skel, n_people=8)
    recs, offsets = _pipeline_decode(cif_h, caf_h, skel, density=8.0, repeats=3)
    _check_images(cif_h, caf_h, skel, recs, offsets, list(range(3, 256, 8)))


def test_cfg5_planted_bench_batch():
    """bench.py's cfg5 planted line: 64 x 160x160 images, dense 44-edge skeleton, 16 people
    (seed_loop_ext_kernel: 64 images leave CUs for helper workgroups): all 64 images."""
    from openpifpaf_amd import constants, synthetic
    skel = constants.DENSE_DECODE_SKELETON
    cif_h, caf_h = synthetic.batch('planted', 64, 160, 160, skeleton=skel, n_people=16)
    recs, offsets = _pipeline_decode(cif_h, caf_h, skel, density=16.0)
    n = _check_images(cif_h, caf_h, skel, recs, offsets, list(range(64)))
    assert n > 64 * 12


def test_cfg5_uniform_bench_batch():
    """bench.py's cfg5 uniform line: 64 x 160x160 uniform images with 44 CAFs (~1.4k
    annotations per image) in one pipeline decode with the dense hint: 4 sampled images."""
    from openpifpaf_amd import constants, synthetic
    skel = constants.DENSE_DECODE_SKELETON
    cif_h, caf_h = synthetic.batch('uniform', 64, 160, 160, n_caf=len(skel))
    recs, offsets = _pipeline_decode(cif_h, caf_h, skel, density=1400.0, repeats=1)
    n = _check_images(cif_h, caf_h, skel, recs, offsets, [0, 21, 42, 63])
    assert n > 4 * 1000
