"""Multi-rank path on CPU (gloo, world size 2): image sharding and the record all-gather
that bench.py runs over RCCL on the box."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpifpaf_amd._abi import ANN_DTYPE, PACK_ALL, packed_dtype  # noqa: E402
from openpifpaf_amd.distributed import gather_records, shard  # noqa: E402


def test_shard_covers_batch():
    for n in (0, 1, 7, 256, 257):
        for world in (1, 2, 3, 8):
            parts = [shard(n, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            for (a0, a1), (b0, _) in zip(parts, parts[1:]):
                assert a1 == b0
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard(4, 2, 2)


DTYPES = {'full': ANN_DTYPE, 'compact': packed_dtype(17, 19, PACK_ALL)}


def _rank_records(rank, n_img, dtype):
    """Deterministic fake decode output of one rank: image i has (rank + i) % 3 records."""
    rng = np.random.default_rng(100 + rank)
    counts = [(rank + i) % 3 for i in range(n_img)]
    recs = np.zeros(sum(counts), dtype)
    recs['image'] = np.repeat(np.arange(n_img), counts)
    recs['data'] = rng.random(recs['data'].shape, dtype=np.float32)
    recs['score'] = rng.random(len(recs))
    return recs, np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)


def _worker(rank, world, port, n_imgs, kind):
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:{}'.format(port),
                            rank=rank, world_size=world)
    dtype = DTYPES[kind]
    try:
        recs, offs = _rank_records(rank, n_imgs[rank], dtype)
        got, got_offs = gather_records(recs, offs, dist, torch.device('cpu'))
        if rank != 0:  # records are collected on rank 0 only
            assert got is None and got_offs is None
            return
        exp = [_rank_records(r, n_imgs[r], dtype) for r in range(world)]
        assert got.dtype == dtype
        # image indices rebased to the global batch (rank r's images follow rank r - 1's)
        bases = np.concatenate([[0], np.cumsum(n_imgs)[:-1]])
        for (r_recs, _), b in zip(exp, bases):
            r_recs['image'] += b
        # bytes of each rank's array, padding included (np.concatenate would not copy the
        # gaps of a structured dtype)
        assert got.tobytes() == b''.join(e[0].tobytes() for e in exp)
        # offsets: images of rank 0 first, then rank 1, each shifted by the records before
        exp_offs, base = [0], 0
        for r_recs, r_offs in exp:
            exp_offs.extend((base + r_offs[1:]).tolist())
            base += len(r_recs)
        assert got_offs.tolist() == exp_offs
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.parametrize('kind', sorted(DTYPES))
@pytest.mark.parametrize('n_imgs', [(4, 4), (3, 5), (0, 2), (2, 0), (3, 3, 2, 0)])
def test_gather_records(n_imgs, kind):
    world = len(n_imgs)
    mp.spawn(_worker, args=(world, _free_port(), n_imgs, kind), nprocs=world, join=True)
