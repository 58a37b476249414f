"""The RCCL leg of the record gather (distributed.gather_records / gather_packed with
device payloads), run when two GPUs are visible: two ranks on backend 'nccl' (RCCL over
xGMI), a subgroup, the records of each rank in device memory, collected on dst = 0 or 1.
Skipped on a one-GPU box (the gloo rehearsal of the same code is tests/test_distributed.py).
Reference: generator.py:84-101 (Generator.batch's per-image lists from all workers)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from openpifpaf_amd.distributed import gather_records

from test_distributed import _compact_records

pytestmark = [
    pytest.mark.gpu,
    pytest.mark.skipif(torch.cuda.device_count() < 2, reason='needs two GPUs (RCCL)'),
]


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _nccl_worker(rank, world, port, dst, n_imgs):
    os.environ.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    torch.cuda.set_device(rank)
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:{}'.format(port),
                            rank=rank, world_size=world)
    try:
        group = dist.new_group(list(range(world)))
        recs, offs = _compact_records(rank, n_imgs[rank])
        report = {}
        got, got_offs = gather_records(recs, offs, dist, torch.device('cuda', rank), dst=dst,
                                       report=report, group=group)
        if rank != dst:
            assert got is None and got_offs is None
            return
        assert report['ranks_seen'] == world and report['ranks_verified'] == world
        exp, base = [], 0
        for r in range(world):
            e, _ = _compact_records(r, n_imgs[r])
            e['image'] += base
            base += n_imgs[r]
            exp.append(e)
        assert got.tobytes() == b''.join(e.tobytes() for e in exp)
        assert got_offs[-1] == sum(len(e) for e in exp)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('dst', [0, 1])
@pytest.mark.parametrize('n_imgs', [(4, 4), (3, 0)])
def test_gather_records_nccl(dst, n_imgs):
    mp.spawn(_nccl_worker, args=(2, _free_port(), dst, n_imgs), nprocs=2, join=True)
