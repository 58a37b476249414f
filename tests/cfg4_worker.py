"""One rank of tests/test_gpu_multirank.py::test_cfg4_eight_ranks (not collected by pytest):
BASELINE.json configs[3] (cfg4) at full size on one GPU -- a 2048-image planted 80x80 batch
split over 8 gloo ranks, 256 images per rank, rank r's images made by
synthetic.batch('planted', 256, 80, 80, first_seed=256 r) as bench.py --workload cfg4 makes
them.  Every rank decodes its shard through CifCaf.decode_batch(group=, local=True) (the
reference's worker_pool.starmap over the batch, generator.py:84-101); rank 0 receives the
annotations of all 2048 images (compact records, every sender's digest checked), then
regenerates each shard, decodes it in this one process without a group and compares
annotation bytes, and checks 4 images per shard against oracle.decode byte for byte.
Environment: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT."""
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'oracle'))
from openpifpaf_amd import constants, decoder, synthetic  # noqa: E402

PER_RANK = 256
# Annotation.to_record() leaves the score field 0 (score() computes it), so the score is
# compared through score()
KEYS = ('data', 'joint_scales', 'n_decoding', 'decoding_pairs', 'decoding_xyv', 'n_frontier',
        'frontier_pairs')


def _fields(rank):
    cif, caf = synthetic.batch('planted', PER_RANK, 80, 80, first_seed=rank * PER_RANK,
                               skeleton=constants.COCO_PERSON_SKELETON, n_people=8)
    return cif, caf


def _bytes(lists):
    return [[a.to_record().tobytes() for a in anns] for anns in lists]


def main():
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    t0 = time.perf_counter()
    dist.init_process_group('gloo')
    torch.cuda.set_device(0)
    decoder.CifSeeds.threshold = 0.2  # eval defaults (factory.py, --decoder-... unset)
    decoder.CifCaf.force_complete = True
    skel = constants.COCO_PERSON_SKELETON
    cc = decoder.CifCaf(decoder.FieldConfig(), keypoints=constants.COCO_KEYPOINTS,
                        skeleton=skel)
    cif_h, caf_h = _fields(rank)
    cif, caf = torch.from_numpy(cif_h).cuda(), torch.from_numpy(caf_h).cuda()
    got = cc.decode_batch(cif, caf, group=dist.group.WORLD, local=True)
    if rank != 0:
        assert got is None
        dist.barrier()
        dist.destroy_process_group()
        return
    rep = cc.last_gather
    assert rep['ranks_seen'] == world and rep['ranks_verified'] == world, rep
    assert len(got) == world * PER_RANK, len(got)
    print('cfg4 gathered {} images, {} annotations, ranks_seen {}, ranks_verified {} '
          '({:.1f} s)'.format(len(got), sum(len(a) for a in got), rep['ranks_seen'],
                              rep['ranks_verified'], time.perf_counter() - t0), flush=True)
    import oracle  # the checker (tests only)
    oracle.lib()
    cfg = cc.config()
    n_oracle = 0
    for r in range(world):
        c_h, a_h = (cif_h, caf_h) if r == 0 else _fields(r)
        one = cc.decode_batch(torch.from_numpy(c_h).cuda(), torch.from_numpy(a_h).cuda())
        mine = got[r * PER_RANK:(r + 1) * PER_RANK]
        assert _bytes(mine) == _bytes(one), 'shard {} differs from its one-process decode'.format(r)
        for i in (r % 7, 64 + r, 150 + 3 * r, PER_RANK - 1 - r):
            ref = oracle.decode(c_h[i], a_h[i], skel, cfg)
            anns = mine[i]
            assert len(anns) == len(ref), (r, i, len(anns), len(ref))
            for a, o in zip(anns, ref):
                rec = a.to_record()
                for key in KEYS:
                    assert np.array_equal(rec[key], o[key]), (r, i, key)
                assert abs(a.score() - float(o['score'])) <= 1e-6, (r, i, a.score(), o['score'])
            n_oracle += len(ref)
        print('shard {} ok: {} annotations byte-identical to the one-process decode'.format(
            r, sum(len(a) for a in mine)), flush=True)
    dist.barrier()
    print('cfg4 ok: world {}, {} images, {} oracle-checked annotations, {:.1f} s'.format(
        world, len(got), n_oracle, time.perf_counter() - t0), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
