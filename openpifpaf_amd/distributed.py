"""Image-sharded multi-GPU decoding.

Images are independent through the whole decoder (cifcaf.py:67-118 touches one image's
fields only), so N ranks split a batch by image with no data-path collective; the only
exchange is collecting every rank's finished annotation records on rank 0 — the
replacement of the reference's `worker_pool.starmap` result list (generator.py:96-97).
One process per GPU; `nccl` (RCCL over xGMI) on the box, `gloo` in the CPU tests.

The gather moves compact records (pp_pack_compact) straight from the device buffer they
were packed into: one small all-gather of (images, records, record format, per-image
counts), then one batch of point-to-point ops to rank 0 with exact sizes (no padding, no
host round trip on the sending ranks).  Every sender also sends a digest of its record
bytes, computed where the bytes are, and rank 0 recomputes it over what arrived (`report`),
so a run proves its own transfers.  Both sides post their point-to-point ops through
`dist.batch_isend_irecv`: RCCL then runs them on the group's communicator on both ends (a
plain `dist.send` would use a separate two-rank communicator that rank 0's batched receives
never meet).  With gloo the records travel from host memory.
"""
import contextlib

import numpy as np
import torch

from ._abi import (ANN_DTYPE, DET_DTYPE, PACK_ALL, PP_MAX_FRONTIER, PP_MAX_KP,
                   PP_PACK_DECODING, PP_PACK_FRONTIER, packed_dtype)

# digest of a record block: two sums of ((word + 1) * w_i mod p) over its 32-bit words, with
# per-position weights w_i < p < 2**31 (products < 2**63, sums of < 2**32 terms fit int64)
_DIGEST_P = (2147483647, 2147483629)
_DIGEST_A = (40503, 65599)
_weights = {}


def shard(n_images, rank, world):
    """[start, stop) of the images rank `rank` decodes: contiguous, sizes differ by <= 1."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError('bad rank {} of {}'.format(rank, world))
    base, extra = divmod(n_images, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def max_shard(n_images, world):
    return -(-n_images // world)


def digest(data):
    """(2,) int64 tensor on data's device: position-weighted checksum of a uint8 tensor whose
    length is a multiple of 4 (records are 16-byte multiples).  The same arithmetic on any
    device, so a digest computed on a sender's GPU checks bytes received on rank 0."""
    words = data.reshape(-1).view(torch.int32).to(torch.int64) & 0xffffffff
    n = words.numel()
    out = torch.zeros(2, dtype=torch.int64, device=data.device)
    if n == 0:
        return out
    key = data.device
    have = _weights.get(key)
    if have is None or have[0].numel() < n:
        i = torch.arange(max(n, 1 << 16), dtype=torch.int64, device=data.device)
        have = tuple((i * a + 1) % p for a, p in zip(_DIGEST_A, _DIGEST_P))
        _weights[key] = have
    for j, (w, p) in enumerate(zip(have, _DIGEST_P)):
        out[j] = (((words + 1) * w[:n]) % p).sum()
    return out


def compact_spec(dtype):
    """(K, frontier length, pack flags) of a compact record dtype (_abi.packed_dtype)."""
    names = dtype.names
    k = dtype['data'].shape[0]
    f = dtype['frontier_pairs'].shape[0] if 'frontier_pairs' in names else 0
    flags = ((PP_PACK_DECODING if 'decoding_pairs' in names else 0) |
             (PP_PACK_FRONTIER if 'frontier_pairs' in names else 0))
    return k, f, flags


def compact_dtype(k, f, flags):
    """The compact record dtype of compact_spec's (K, frontier length, flags)."""
    # packed_dtype takes the skeleton size C and stores min(PP_MAX_FRONTIER, 4 C) pairs
    return packed_dtype(k, -(-f // 4) if f < PP_MAX_FRONTIER else PP_MAX_FRONTIER, flags)


def expand_compact(recs, k=None, c=None):
    """Compact records (pp_pack_compact, not flagged PP_PACK_REFETCH) -> full ANN_DTYPE
    records holding the same annotation (data, scales, score, decoding / frontier order);
    used when another rank of the same gather had to send full records.  K and the
    frontier length come from the record dtype (`k` / `c` are accepted for callers that
    pass them)."""
    k = recs.dtype['data'].shape[0] if k is None else k
    out = np.zeros(len(recs), ANN_DTYPE)
    if not len(recs):
        return out
    if (recs['n_decoding'] & 0x8000).any():
        raise ValueError('compact record flagged PP_PACK_REFETCH')
    out['score'] = recs['score']
    out['image'] = recs['image']
    out['n_keypoints'] = k
    out['data'][:, :k] = recs['data']
    out['joint_scales'][:, :k] = recs['joint_scales']
    names = recs.dtype.names
    if 'decoding_pairs' in names:
        nd = recs['n_decoding'].astype(np.int64)
        out['n_decoding'] = nd
        pairs = recs['decoding_pairs']
        out['decoding_pairs'][:, :k] = pairs
        live = np.arange(k)[None, :] < nd[:, None]
        rows = np.arange(len(recs))[:, None]
        xyv = np.zeros((len(recs), k, 6), np.float32)
        xyv[:, :, 0:2] = recs['decoding_xy'][rows, pairs[:, :, 0].astype(np.int64) % k]
        xyv[:, :, 2] = recs['decoding_v'][:, :, 0]
        xyv[:, :, 3:5] = recs['decoding_xy'][rows, pairs[:, :, 1].astype(np.int64) % k]
        xyv[:, :, 5] = recs['decoding_v'][:, :, 1]
        out['decoding_xyv'][:, :k] = np.where(live[:, :, None], xyv, np.float32(0))
        out['decoding_pairs'][:, :k] *= live[:, :, None].astype(np.uint8)
    if 'frontier_pairs' in names:
        f = recs.dtype['frontier_pairs'].shape[0]  # min(PP_MAX_FRONTIER, 4 * c)
        out['n_frontier'] = recs['n_frontier']
        out['frontier_pairs'][:, :f] = recs['frontier_pairs']
    assert k <= PP_MAX_KP
    return out


_META = 6  # per-rank header: images, records, full?, then the compact dtype's K, F, flags
_META_DET = -1  # K slot of a rank sending pp_det records (CifDet, _abi.DET_DTYPE)


def _meta_format(dtype, full):
    """The header's (K, F, flags) for a rank's record format (zeros: full pp_ann)."""
    if full or dtype is None or dtype == ANN_DTYPE:
        return (0, 0, 0)
    if dtype == DET_DTYPE:
        return (_META_DET, 0, 0)
    return compact_spec(dtype)


def _meta_dtype(m):
    """A rank's record dtype from its header row (inverse of _meta_format)."""
    if m[2] or not m[5] and not m[3]:
        return ANN_DTYPE
    if m[3] == _META_DET:
        return DET_DTYPE
    return compact_dtype(*m[3:6])


def _ranks(dist, group):
    """(this rank, world size, global rank of group rank r) of `group` (None: default)."""
    if group is None:
        return dist.get_rank(), dist.get_world_size(), lambda r: r
    return (dist.get_rank(group), dist.get_world_size(group),
            lambda r: dist.get_global_rank(group, r))


def gather_packed(records, counts, dist, *, n_max, dtype, device, dst=0, stream=None,
                  full=False, k=None, c=None, report=None, group=None):
    """Collect every rank's packed records on rank `dst` (a rank of `group`).

    `records`: this rank's records as a uint8 tensor (device memory for nccl, host for
    gloo; at least sum(counts) * itemsize bytes): compact `dtype` records, or with `full`
    full ANN_DTYPE records (a rank whose pack flagged PP_PACK_REFETCH).  `counts`: its
    per-image record counts, `n_max` >= every rank's image count.  Each rank's record
    format travels in the all-gathered metadata, so ranks may differ: on `dst` the result
    is (records of all ranks in rank order with `image` rebased to the global image index,
    per-image offsets over all images) in the common compact dtype, or ANN_DTYPE when any
    rank sent full records (compact ones are then expanded with expand_compact); elsewhere
    (None, None).  Compact records of different layouts cannot be merged (ValueError).
    `k` / `c` are accepted for older callers and not needed.  With `stream`, the exchange
    is ordered on it (it must already wait for the pack), not behind later work on the
    current stream.  `report` (a dict, optional) receives on `dst`: ranks_seen (ranks
    whose metadata arrived), ranks_verified (ranks whose received bytes match the digest
    they sent; `dst` itself counts as verified), bytes received, and whether full records
    were involved."""
    rank, world, glob = _ranks(dist, group)
    width = (ANN_DTYPE if full or dtype is None else dtype).itemsize
    counts = np.asarray(counts, dtype=np.int64)
    ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
    with ctx:
        # metadata: (images, records, full?, K, F, flags, counts[n_max]) of every rank
        meta = np.zeros(n_max + _META, np.int64)
        meta[0], meta[1], meta[2] = len(counts), int(counts.sum()), int(full)
        meta[3:6] = _meta_format(dtype, full)
        meta[_META:_META + len(counts)] = counts
        t = torch.from_numpy(meta)
        if device.type == 'cuda':
            t = t.pin_memory().to(device, non_blocking=True)
        gathered = torch.empty(world * (n_max + _META), dtype=torch.int64, device=device)
        dist.all_gather_into_tensor(gathered, t, group=group)
        if rank != dst:
            # the sender needs nothing back: no host synchronisation here
            n = int(counts.sum()) * width
            if n:
                payload = records[:n]
                ops = [dist.P2POp(dist.isend, payload, glob(dst), group),
                       dist.P2POp(dist.isend, digest(payload), glob(dst), group)]
                for req in dist.batch_isend_irecv(ops):
                    req.wait()
            return None, None
        metas = gathered.cpu().numpy().reshape(world, n_max + _META)
        # each rank's record dtype: full records, or the compact layout it announced
        dtypes = [_meta_dtype(m) for m in metas]
        widths = np.array([d.itemsize for d in dtypes], np.int64)
        totals = metas[:, 1]
        bufs, sums, ops = {}, {}, []
        for r in range(world):
            n = int(totals[r]) * int(widths[r])
            if r == dst or n == 0:
                continue
            bufs[r] = torch.empty(n, dtype=torch.uint8, device=device)
            sums[r] = torch.empty(2, dtype=torch.int64, device=device)
            ops += [dist.P2POp(dist.irecv, bufs[r], glob(r), group),
                    dist.P2POp(dist.irecv, sums[r], glob(r), group)]
        for req in (dist.batch_isend_irecv(ops) if ops else []):
            req.wait()
        # rank dst recomputes each sender's digest over the bytes that arrived
        check = (torch.stack([torch.cat([digest(bufs[r]), sums[r]]) for r in sorted(bufs)])
                 if bufs else None)
        pinned = device.type == 'cuda'
        host = torch.empty(int((totals * widths).sum()), dtype=torch.uint8, pin_memory=pinned)
        o = 0
        for r in range(world):
            n = int(totals[r]) * int(widths[r])
            if n:
                host[o:o + n].copy_(records[:n] if r == dst else bufs[r], non_blocking=pinned)
            o += n
        check_h = check.to('cpu', non_blocking=pinned) if check is not None else None
        if pinned:
            torch.cuda.current_stream(device).synchronize()
    # ranks with records decide the output format (an empty rank's format does not matter)
    live = [r for r in range(world) if totals[r]]
    any_det = any(dtypes[r] == DET_DTYPE for r in live)
    if any_det and any(dtypes[r] != DET_DTYPE for r in live):
        raise ValueError('ranks sent detection and keypoint records to one gather')
    any_full = any(dtypes[r] == ANN_DTYPE for r in live)
    out_dtype = ANN_DTYPE if any_full else (dtypes[live[0]] if live else
                                            (dtype if dtype is not None else ANN_DTYPE))
    if not any_full and any(dtypes[r] != out_dtype for r in live):
        raise ValueError('ranks sent compact records of different layouts')
    parts, o = [], 0
    for r in range(world):
        n = int(totals[r]) * int(widths[r])
        part = host[o:o + n].numpy().view(dtypes[r]) if n else np.zeros(0, out_dtype)
        if any_full and n and dtypes[r] != ANN_DTYPE:
            part = expand_compact(part)
        parts.append(part)
        o += n
    recs = (np.concatenate(parts) if any_full else
            host.numpy().view(out_dtype) if len(host) else np.zeros(0, out_dtype))
    # a record's image is its index in its rank's batch: rebase to the global image index
    # (rank r's images follow those of ranks < r, as shard() assigns them)
    n_imgs = metas[:, 0]
    img_base = np.repeat(np.concatenate([[0], np.cumsum(n_imgs)[:-1]]), totals)
    if len(recs) and img_base.any():
        recs['image'] += img_base.astype(recs['image'].dtype)
    per_image = np.concatenate([metas[r, _META:_META + metas[r, 0]] for r in range(world)])
    if report is not None:
        ok = 1 + sum(1 for r in range(world) if r != dst and totals[r] == 0)
        if check_h is not None:
            cv = check_h.numpy()
            ok += int((cv[:, :2] == cv[:, 2:]).all(axis=1).sum())
        report.update(ranks_seen=int(len(metas)), ranks_verified=int(ok),
                      bytes=int(len(host)), full_records=any_full)
    return recs, np.concatenate([[0], np.cumsum(per_image)]).astype(np.int64)


def gather_records(recs, offsets, dist, device, dst=0, report=None, group=None):
    """Host records (full ANN_DTYPE or compact, may differ between ranks) + per-image
    offsets of this rank -> all ranks' (records, offsets) on `dst` (None, None elsewhere);
    the host-side form of gather_packed for callers that already hold their records on
    the host."""
    recs = np.ascontiguousarray(recs)
    counts = np.diff(np.asarray(offsets, dtype=np.int64))
    n_max_t = torch.tensor([len(counts)], dtype=torch.int64, device=device)
    dist.all_reduce(n_max_t, op=dist.ReduceOp.MAX, group=group)
    data = torch.from_numpy(recs.view(np.uint8).reshape(-1))
    if device.type == 'cuda':
        data = data.to(device)
    return gather_packed(data, counts, dist, n_max=int(n_max_t.item()), dtype=recs.dtype,
                         device=device, dst=dst, full=recs.dtype == ANN_DTYPE, report=report,
                         group=group)


def pending_payload(pending, counts, device):
    """A waited PendingRecords (DecodeEngine.fetch_async) -> (uint8 tensor on `device`
    (None: where they are) holding this rank's records, full?): the compact block as packed, full records after a
    PP_PACK_REFETCH flag, or the re-packed records when the batch outgrew the block."""
    total = int(counts.sum())
    if pending.refetch:
        src, full = pending.full_device_records(), True
    elif not pending.fits(total):
        recs, _ = pending.result()
        full = recs.dtype == ANN_DTYPE
        src = torch.from_numpy(np.ascontiguousarray(recs).view(np.uint8).reshape(-1))
    else:
        src = (pending.device_records if pending.device_records is not None
               else pending.host_records())
        full = False
    width = (ANN_DTYPE if full else pending.dtype).itemsize
    src = src[:total * width]
    if device is not None and src.device != device:
        src = src.to(device)
    return src, full


class GatherMismatch(RuntimeError):
    """Rank dst received records whose digest differs from the one their sender computed."""


def decode_sharded(decode_local, n_local, dist, *, group=None, dst=0, report=None):
    """Image-sharded decode (the reference's worker_pool.starmap over the
    batch, generator.py:96-97): this rank decodes its own `n_local` images through
    `decode_local(device_out)` -> (PendingRecords, or None for no images), and rank `dst`
    collects every rank's records (gather_packed over `group`'s backend: RCCL device
    buffers for nccl, host memory for gloo).  On `dst` returns (records, offsets) over the
    images of all ranks in rank order; None, None elsewhere.  Raises GatherMismatch on
    `dst` when a sender's digest does not match the bytes that arrived."""
    rank, world, _ = _ranks(dist, group)
    nccl = dist.get_backend(group) == 'nccl'
    device = (torch.device('cuda', torch.cuda.current_device()) if nccl
              else torch.device('cpu'))
    n_max_t = torch.tensor([n_local], dtype=torch.int64, device=device)
    dist.all_reduce(n_max_t, op=dist.ReduceOp.MAX, group=group)
    n_max = int(n_max_t.item())
    pending = decode_local(nccl and rank != dst) if n_local else None
    if pending is None:
        payload, full, counts = torch.zeros(0, dtype=torch.uint8, device=device), False, \
            np.zeros(n_local, np.int64)
        dtype = None
    else:
        counts = pending.wait()
        # rank dst copies its own records into the host result from wherever they are
        payload, full = pending_payload(pending, counts, device if rank != dst else None)
        dtype = pending.dtype
    rep = {} if report is None else report
    recs, offsets = gather_packed(payload, counts, dist, n_max=n_max, dtype=dtype,
                                  device=device, dst=dst, full=full, report=rep, group=group)
    if rank == dst and rep['ranks_verified'] != world:
        raise GatherMismatch('gathered records of {} of {} ranks do not match their digests'
                             .format(world - rep['ranks_verified'], world))
    return recs, offsets
