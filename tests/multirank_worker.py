"""One rank of tests/test_gpu_multirank.py (not collected by pytest): decodes its shard()
of a 32-image planted + uniform batch on cuda:0, packs compact records (rank 0 into pinned
host memory, the others into device memory), and gathers them to rank 0 over gloo; rank 0
compares the gathered records byte for byte with a one-process decode of the whole batch.
Environment: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd import constants, synthetic  # noqa: E402
from openpifpaf_amd._abi import EVAL_CONFIG, PACK_ALL, make_config  # noqa: E402
from openpifpaf_amd.distributed import gather_packed, max_shard, shard  # noqa: E402
from openpifpaf_amd.engine import DecodeEngine  # noqa: E402

N = 32


def _ann_bytes(lists):
    return [[a.to_record().tobytes() for a in anns] for anns in lists]


def api_main(rank, world, cif, caf):
    """The library's sharded API: CifCaf.decode_batch(group=) and Generator.batch(group=)
    (the model stand-in maps image indices to their fields), checked on rank 0 against a
    one-process decode of the whole batch, annotation record by record."""
    from openpifpaf_amd import decoder
    decoder.CifSeeds.threshold = 0.2
    decoder.CifCaf.force_complete = True
    cc = decoder.CifCaf(decoder.FieldConfig(), keypoints=constants.COCO_KEYPOINTS,
                        skeleton=constants.COCO_PERSON_SKELETON)
    got = cc.decode_batch(cif, caf, group=dist.group.WORLD)
    got_b = cc.batch(lambda idx: [cif[idx], caf[idx]], torch.arange(N), device='cuda',
                     group=dist.group.WORLD)
    if rank == 0:
        assert cc.last_gather['ranks_verified'] == world, cc.last_gather
        ref = cc.decode_batch(cif, caf)
        assert len(got) == len(got_b) == len(ref) == N
        assert _ann_bytes(got) == _ann_bytes(ref), 'decode_batch(group=) differs'
        assert _ann_bytes(got_b) == _ann_bytes(ref), 'batch(group=) differs'
        print('multirank ok: api, {} annotations, world {}'.format(
            sum(len(a) for a in ref), world), flush=True)
    else:
        assert got is None and got_b is None
    dist.destroy_process_group()


def det_main(rank, world):
    """CifDet.decode_batch(group=) with the real device decode (ref generator.py:84-101,
    cifdet.py): each rank decodes its shard of a 24-image planted detection batch on cuda:0,
    rank 0 gathers pp_det records (K = -1 headers, digests checked) and compares every
    image's detections byte for byte with a one-process decode_batch."""
    from openpifpaf_amd import decoder
    decoder.CifHr.v_threshold = 0.1
    decoder.CifSeeds.threshold = 0.3
    det = torch.from_numpy(synthetic.det_batch('planted', 24, 48, 40, first_seed=50,
                                               n_categories=4)).cuda()
    cd = decoder.CifDet(decoder.FieldConfig(), ['a', 'b', 'c', 'd'])
    got = cd.decode_batch(det, group=dist.group.WORLD)
    if rank == 0:
        assert cd.last_gather['ranks_seen'] == world, cd.last_gather
        assert cd.last_gather['ranks_verified'] == world, cd.last_gather
        ref = cd.decode_batch(det)
        assert len(got) == len(ref) == 24

        def key(lists):
            return [[(a.field_i, np.float32(a.score).tobytes(),
                      np.asarray(a.bbox, np.float32).tobytes()) for a in anns] for anns in lists]
        assert key(got) == key(ref), 'gathered detections differ'
        print('multirank ok: det, {} detections, world {}'.format(
            sum(len(a) for a in ref), world), flush=True)
    else:
        assert got is None
    dist.destroy_process_group()


def main():
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    dist.init_process_group('gloo')
    torch.cuda.set_device(0)
    if len(sys.argv) > 1 and sys.argv[1] == 'det':
        det_main(rank, world)
        return
    skel = constants.COCO_PERSON_SKELETON
    cfg = make_config(**EVAL_CONFIG)
    cp, ap = synthetic.batch('planted', N // 2, 80, 80)
    cu, au = synthetic.batch('uniform', N // 2, 80, 80, first_seed=N // 2)
    cif = torch.from_numpy(np.concatenate([cp, cu])).cuda()
    caf = torch.from_numpy(np.concatenate([ap, au])).cuda()
    if len(sys.argv) > 1 and sys.argv[1] == 'api':
        api_main(rank, world, cif, caf)
        return
    a, b = shard(N, rank, world)
    eng = DecodeEngine()
    buf = eng.launch(cif[a:b].contiguous(), caf[a:b].contiguous(), skel, cfg)
    pend = eng.fetch_async(buf, (17, len(skel), PACK_ALL), device_out=rank != 0,
                           capacity=1024 * (b - a))
    counts = pend.wait()
    nbytes = int(counts.sum()) * pend.dtype.itemsize
    src = (pend.device_records if rank != 0 else pend.host_records())[:nbytes].cpu()
    assert not pend.refetch
    report = {}
    recs, offs = gather_packed(src, counts, dist, n_max=max_shard(N, world), dtype=pend.dtype,
                               device=torch.device('cpu'), report=report)
    if rank == 0:
        assert report['ranks_seen'] == world and report['ranks_verified'] == world, report
        ref, ref_offs, _ = DecodeEngine().decode(cif, caf, skel, cfg, compact=PACK_ALL)
        assert ref.dtype == recs.dtype, 'one-process decode fell back to full records'
        assert np.array_equal(offs, ref_offs), (offs[:8], ref_offs[:8])
        assert recs.tobytes() == ref.tobytes(), 'gathered records differ'
        print('multirank ok: {} records, {} images, world {}'.format(len(recs), N, world),
              flush=True)
    else:
        assert recs is None
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
