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
from openpifpaf_amd.distributed import (GatherMismatch, decode_sharded,  # noqa: E402
                                        digest, expand_compact, gather_packed,
                                        gather_records, shard)


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


def _compact_records(rank, n_img):
    """Fake compact records that expand_compact accepts: valid joint indices in the
    decoding pairs, counts within K / F."""
    dtype = DTYPES['compact']
    recs, offs = _rank_records(rank, n_img, dtype)
    rng = np.random.default_rng(7 + rank)
    recs['n_decoding'] = rng.integers(0, 17, len(recs))
    recs['n_frontier'] = rng.integers(0, 4 * 19, len(recs))
    recs['decoding_pairs'] = rng.integers(0, 17, recs['decoding_pairs'].shape)
    recs['decoding_xy'] = rng.random(recs['decoding_xy'].shape, dtype=np.float32)
    recs['decoding_v'] = rng.random(recs['decoding_v'].shape, dtype=np.float32)
    recs['frontier_pairs'] = rng.integers(0, 17, recs['frontier_pairs'].shape)
    return recs, offs


def _worker(rank, world, port, n_imgs, kind):
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:{}'.format(port),
                            rank=rank, world_size=world)
    try:
        if kind == 'mixed':
            _mixed_worker(rank, world, n_imgs)
            return
        if kind == 'records_mixed':
            _records_mixed_worker(rank, world, n_imgs)
            return
        if kind.startswith('sharded'):
            _sharded_worker(rank, world, n_imgs, kind)
            return
        dtype = DTYPES[kind]
        recs, offs = _rank_records(rank, n_imgs[rank], dtype)
        report = {}
        got, got_offs = gather_records(recs, offs, dist, torch.device('cpu'), report=report)
        if rank != 0:  # records are collected on rank 0 only
            assert got is None and got_offs is None and not report
            return
        # every rank's metadata arrived and every sender's digest matched on rank 0
        assert report['ranks_seen'] == world and report['ranks_verified'] == world
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


def _mixed_worker(rank, world, n_imgs):
    """Rank 1 had a PP_PACK_REFETCH and sends full records; the others send compact ones,
    which rank 0 expands so the gathered array has one dtype."""
    recs, offs = _compact_records(rank, n_imgs[rank])
    full = rank == 1
    if full:
        recs = expand_compact(recs, 17, 19)
    data = torch.from_numpy(recs.view(np.uint8).reshape(-1))
    report = {}
    got, got_offs = gather_packed(data, np.diff(offs), dist, n_max=max(n_imgs),
                                  dtype=DTYPES['compact'], device=torch.device('cpu'),
                                  full=full, k=17, c=19, report=report)
    if rank != 0:
        assert got is None
        return
    assert report['full_records'] and report['ranks_verified'] == world
    exp, base = [], 0
    for r in range(world):
        e = expand_compact(_compact_records(r, n_imgs[r])[0], 17, 19)
        e['image'] += base
        base += n_imgs[r]
        exp.append(e)
    assert got.dtype == ANN_DTYPE
    assert got.tobytes() == b''.join(e.tobytes() for e in exp)
    assert got_offs[-1] == len(got)


def _records_mixed_worker(rank, world, n_imgs):
    """gather_records with per-rank formats: rank 0 holds full records (its
    pack was refetched), the others compact ones; rank 0 learns each rank's layout from
    the metadata and expands the compact ones."""
    recs, offs = _compact_records(rank, n_imgs[rank])
    if rank == 0:
        recs = expand_compact(recs)
    report = {}
    got, got_offs = gather_records(recs, offs, dist, torch.device('cpu'), report=report)
    if rank != 0:
        assert got is None
        return
    assert report['full_records'] and report['ranks_verified'] == world
    exp, base = [], 0
    for r in range(world):
        e = expand_compact(_compact_records(r, n_imgs[r])[0], 17, 19)
        e['image'] += base
        base += n_imgs[r]
        exp.append(e)
    assert got.dtype == ANN_DTYPE
    assert got.tobytes() == b''.join(e.tobytes() for e in exp)
    assert got_offs.tolist() == np.concatenate(
        [[0], np.cumsum([c for r in range(world) for c in np.diff(_compact_records(r, n_imgs[r])[1])])]).tolist()


class _FakePending:
    """The PendingRecords surface decode_sharded reads: a finished compact pack in host
    memory (what a gloo rank holds)."""

    def __init__(self, recs, offs, refetch=False):
        self.dtype = recs.dtype
        self.device_records = None
        self._host = torch.from_numpy(recs.view(np.uint8).reshape(-1).copy())
        self._counts = np.diff(offs).astype(np.int64)
        self.refetch = refetch
        self._full = expand_compact(recs) if refetch else None

    def wait(self):
        return self._counts

    def fits(self, total):
        return True

    def host_records(self):
        return self._host

    def full_device_records(self):
        return torch.from_numpy(self._full.view(np.uint8).reshape(-1).copy())


def _sharded_worker(rank, world, n_imgs, kind):
    """decode_sharded with a stand-in for the device decode: rank r 'decodes' its shard of
    a global batch into the compact records _compact_records(r, ...) would hold; rank 0
    gets every rank's records, image indices rebased, and the digests checked."""
    n_total = sum(n_imgs)
    a, b = shard(n_total, rank, world)
    recs, offs = _compact_records(rank, b - a)
    refetch = kind == 'sharded_refetch' and rank == world - 1
    calls = []

    def decode_local(device_out):
        calls.append(device_out)
        return _FakePending(recs, offs, refetch)

    report = {}
    got, got_offs = decode_sharded(decode_local, b - a, dist, report=report)
    assert calls == ([False] if b > a else [])  # gloo: records stay in host memory
    if rank != 0:
        assert got is None and got_offs is None
        return
    assert report['ranks_seen'] == world and report['ranks_verified'] == world
    # one rank's full records turn the result into full records (if it had any)
    la, lb = shard(n_total, world - 1, world)
    any_full = kind == 'sharded_refetch' and len(_compact_records(world - 1, lb - la)[0]) > 0
    exp, base, counts = [], 0, []
    for r in range(world):
        ra, rb = shard(n_total, r, world)
        e, eo = _compact_records(r, rb - ra)
        if any_full:
            e = expand_compact(e)
        e['image'] += base
        base += rb - ra
        exp.append(e)
        counts.extend(np.diff(eo).tolist())
    assert got.dtype == exp[0].dtype
    assert got.tobytes() == b''.join(e.tobytes() for e in exp)
    assert got_offs.tolist() == np.concatenate([[0], np.cumsum(counts)]).astype(int).tolist()


def _corrupt_worker(rank, world, port):
    """A sender whose digest does not match its bytes: rank 0 raises GatherMismatch."""
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:{}'.format(port),
                            rank=rank, world_size=world)
    try:
        recs, offs = _compact_records(rank, 3)
        import openpifpaf_amd.distributed as D
        if rank == 1:
            real = D.digest
            D.digest = lambda t: real(t) + 1
        try:
            decode_sharded(lambda _: _FakePending(recs, offs), 3, dist)
        except GatherMismatch:
            assert rank == 0
            return
        assert rank != 0, 'rank 0 accepted a corrupted transfer'
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('n_imgs', [(4, 4), (3, 4), (1, 0), (3, 3, 3)])
@pytest.mark.parametrize('kind', ['sharded', 'sharded_refetch'])
def test_decode_sharded_gloo(n_imgs, kind):
    world = len(n_imgs)
    mp.spawn(_worker, args=(world, _free_port(), n_imgs, kind), nprocs=world, join=True)


def test_decode_sharded_digest_mismatch():
    mp.spawn(_corrupt_worker, args=(2, _free_port()), nprocs=2, join=True)


@pytest.mark.parametrize('n_imgs', [(3, 4), (2, 0, 3)])
def test_gather_records_mixed_formats(n_imgs):
    world = len(n_imgs)
    mp.spawn(_worker, args=(world, _free_port(), n_imgs, 'records_mixed'), nprocs=world,
             join=True)


def test_digest_detects_changes():
    rng = np.random.default_rng(0)
    a = torch.from_numpy(rng.integers(0, 256, 4096, dtype=np.uint8))
    d0 = digest(a)
    assert torch.equal(d0, digest(a.clone()))
    for pos in (0, 1, 2047, 4095):
        b = a.clone()
        b[pos] ^= 1
        assert not torch.equal(d0, digest(b))
    # swapping two words changes it too (position-weighted)
    b = a.clone()
    b[0:4], b[4:8] = a[4:8].clone(), a[0:4].clone()
    assert torch.equal(a[0:4], a[4:8]) or not torch.equal(d0, digest(b))
    assert digest(a[:0]).tolist() == [0, 0]


def test_expand_compact_roundtrip_fields():
    recs, _ = _compact_records(0, 6)
    full = expand_compact(recs, 17, 19)
    for i, r in enumerate(recs):
        f = full[i]
        nd = int(r['n_decoding'])
        assert f['n_decoding'] == nd and f['n_frontier'] == r['n_frontier']
        assert np.array_equal(f['data'][:17], r['data'])
        for t in range(nd):
            js, jt = r['decoding_pairs'][t]
            assert np.array_equal(f['decoding_xyv'][t][:2], r['decoding_xy'][js])
            assert f['decoding_xyv'][t][2] == r['decoding_v'][t][0]
            assert np.array_equal(f['decoding_xyv'][t][3:5], r['decoding_xy'][jt])
            assert f['decoding_xyv'][t][5] == r['decoding_v'][t][1]
        assert not f['decoding_xyv'][nd:].any() and not f['decoding_pairs'][nd:].any()
    flagged = recs.copy()
    flagged['n_decoding'][0] |= 0x8000
    with pytest.raises(ValueError):
        expand_compact(flagged, 17, 19)


@pytest.mark.parametrize('n_imgs', [(3, 4), (2, 3, 0)])
def test_gather_mixed_full_and_compact(n_imgs):
    world = len(n_imgs)
    mp.spawn(_worker, args=(world, _free_port(), n_imgs, 'mixed'), nprocs=world, join=True)


def _fake_det_records(det_batch):
    """Stand-in for CifDet.decode_records (the device decode): image i of the batch holds
    int(det[i, 0, 0, 0, 0]) detections whose values are read from its fields."""
    from openpifpaf_amd._abi import DET_DTYPE
    det = np.asarray(det_batch)
    counts = det[:, 0, 0, 0, 0].astype(np.int64)
    recs = np.zeros(int(counts.sum()), DET_DTYPE)
    o = 0
    for i, c in enumerate(counts):
        for r in range(c):
            recs[o] = (r % det.shape[1], det[i, 0, 1, 0, r], det[i, 0, 2, 0, r:r + 4], i, 0)
            o += 1
    return recs, np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)


def _det_batch(n):
    rng = np.random.default_rng(5)
    det = rng.random((n, 3, 7, 2, 8), dtype=np.float32)
    det[:, 0, 0, 0, 0] = rng.integers(0, 4, n)  # 0-3 detections per image
    return torch.from_numpy(det)


class _DetModel(torch.nn.Module):
    """Generator.batch's model: the 'images' are the CifDet fields themselves; counts the
    images it sees (a rank runs the model on its shard only)."""
    seen = 0

    def forward(self, x):
        _DetModel.seen += len(x)
        return [x]


def _det_worker(rank, world, port, n_img):
    """CifDet.decode_batch / Generator.batch with group=: each rank decodes its shard, rank 0
    returns every image's detections, in order, digests checked (ref generator.py:84-101)."""
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:{}'.format(port),
                            rank=rank, world_size=world)
    try:
        from openpifpaf_amd import constants
        from openpifpaf_amd.decoder import FieldConfig
        from openpifpaf_amd.decoder.generator.cifdet import CifDet
        det = _det_batch(n_img)
        dec = CifDet(FieldConfig(), ['a', 'b', 'c'])
        dec.decode_records = _fake_det_records
        want = dec.annotations_from_records(*_fake_det_records(det))

        def key(lists):
            return [[(a.field_i, float(a.score), tuple(np.asarray(a.bbox).tolist()))
                     for a in anns] for anns in lists]
        for run in ('decode_batch', 'batch'):
            if run == 'decode_batch':
                got = dec.decode_batch(det, group=dist.group.WORLD)
            else:
                _DetModel.seen = 0
                got = dec.batch(_DetModel(), det, group=dist.group.WORLD)
                a, b = shard(n_img, rank, world)
                assert _DetModel.seen == b - a
            if rank != 0:
                assert got is None
                continue
            assert dec.last_gather['ranks_seen'] == world
            assert dec.last_gather['ranks_verified'] == world
            assert key(got) == key(want)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world,n_img', [(2, 7), (2, 1), (3, 5)])
def test_cifdet_sharded_gloo(world, n_img):
    mp.spawn(_det_worker, args=(world, _free_port(), n_img), nprocs=world, join=True)


def test_batch_refuses_unsharded_generator_before_model():
    """A generator without sharding support raises before the model runs."""
    from openpifpaf_amd.decoder.generator.generator import Generator
    _DetModel.seen = 0
    with pytest.raises(NotImplementedError):
        Generator().batch(_DetModel(), _det_batch(4), group=object())
    assert _DetModel.seen == 0


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.parametrize('kind', sorted(DTYPES))
@pytest.mark.parametrize('n_imgs', [(4, 4), (3, 5), (0, 2), (2, 0), (3, 3, 2, 0)])
def test_gather_records(n_imgs, kind):
    world = len(n_imgs)
    mp.spawn(_worker, args=(world, _free_port(), n_imgs, kind), nprocs=world, join=True)
