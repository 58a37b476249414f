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

from ._abi import ANN_DTYPE, PP_MAX_FRONTIER, PP_MAX_KP

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


def expand_compact(recs, k, c):
    """Compact records (pp_pack_compact, not flagged PP_PACK_REFETCH) -> full ANN_DTYPE
    records holding the same annotation (data, scales, score, decoding / frontier order);
    used when another rank of the same gather had to send full records."""
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
        f = min(PP_MAX_FRONTIER, 4 * c)
        out['n_frontier'] = recs['n_frontier']
        out['frontier_pairs'][:, :f] = recs['frontier_pairs']
    assert k <= PP_MAX_KP
    return out


def gather_packed(records, counts, dist, *, n_max, dtype, device, dst=0, stream=None,
                  full=False, k=None, c=None, report=None):
    """Collect every rank's packed records on rank `dst`.

    `records`: this rank's records as a uint8 tensor (device memory for nccl, host for
    gloo; at least sum(counts) * itemsize bytes): compact `dtype` records, or with `full`
    full ANN_DTYPE records (a rank whose pack flagged PP_PACK_REFETCH).  `counts`: its
    per-image record counts, `n_max` >= every rank's image count.  On `dst` returns (records
    of all ranks in rank order with `image` rebased to the global image index, per-image
    offsets over all images): `dtype` records, or ANN_DTYPE when any rank sent full records
    (compact ones are then expanded with expand_compact; `k` / `c` = keypoints / skeleton
    edges); elsewhere (None, None).  With `stream`, the exchange is ordered on it (it must
    already wait for the pack), not behind later work on the current stream.
    `report` (a dict, optional) receives on `dst`: ranks_seen (ranks whose metadata
    arrived), ranks_verified (ranks whose received bytes match the digest they sent; `dst`
    itself counts as verified), bytes received, and whether full records were involved."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    width = (ANN_DTYPE if full else dtype).itemsize
    counts = np.asarray(counts, dtype=np.int64)
    ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
    with ctx:
        # metadata: (images, records, full?, counts[n_max]) of every rank
        meta = np.zeros(n_max + 3, np.int64)
        meta[0], meta[1], meta[2] = len(counts), int(counts.sum()), int(full)
        meta[3:3 + len(counts)] = counts
        t = torch.from_numpy(meta)
        if device.type == 'cuda':
            t = t.pin_memory().to(device, non_blocking=True)
        gathered = torch.empty(world * (n_max + 3), dtype=torch.int64, device=device)
        dist.all_gather_into_tensor(gathered, t)
        if rank != dst:
            # the sender needs nothing back: no host synchronisation here
            n = int(counts.sum()) * width
            if n:
                payload = records[:n]
                ops = [dist.P2POp(dist.isend, payload, dst),
                       dist.P2POp(dist.isend, digest(payload), dst)]
                for req in dist.batch_isend_irecv(ops):
                    req.wait()
            return None, None
        metas = gathered.cpu().numpy().reshape(world, n_max + 3)
        widths = np.where(metas[:, 2] != 0, ANN_DTYPE.itemsize, dtype.itemsize)
        totals = metas[:, 1]
        bufs, sums, ops = {}, {}, []
        for r in range(world):
            n = int(totals[r]) * int(widths[r])
            if r == dst or n == 0:
                continue
            bufs[r] = torch.empty(n, dtype=torch.uint8, device=device)
            sums[r] = torch.empty(2, dtype=torch.int64, device=device)
            ops += [dist.P2POp(dist.irecv, bufs[r], r), dist.P2POp(dist.irecv, sums[r], r)]
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
    any_full = bool(metas[:, 2].any())
    parts, o = [], 0
    for r in range(world):
        n = int(totals[r]) * int(widths[r])
        part = host[o:o + n].numpy().view(ANN_DTYPE if metas[r, 2] else dtype) if n else \
            np.zeros(0, ANN_DTYPE if metas[r, 2] else dtype)
        if any_full and not metas[r, 2]:
            part = expand_compact(part, k, c)
        parts.append(part)
        o += n
    recs = (np.concatenate(parts) if any_full else
            host.numpy().view(dtype) if len(host) else np.zeros(0, dtype))
    # a record's image is its index in its rank's batch: rebase to the global image index
    # (rank r's images follow those of ranks < r, as shard() assigns them)
    n_imgs = metas[:, 0]
    img_base = np.repeat(np.concatenate([[0], np.cumsum(n_imgs)[:-1]]), totals)
    if len(recs) and img_base.any():
        recs['image'] += img_base.astype(recs['image'].dtype)
    per_image = np.concatenate([metas[r, 3:3 + metas[r, 0]] for r in range(world)])
    if report is not None:
        ok = 1 + sum(1 for r in range(world) if r != dst and totals[r] == 0)
        if check_h is not None:
            cv = check_h.numpy()
            ok += int((cv[:, :2] == cv[:, 2:]).all(axis=1).sum())
        report.update(ranks_seen=int(len(metas)), ranks_verified=int(ok),
                      bytes=int(len(host)), full_records=any_full)
    return recs, np.concatenate([[0], np.cumsum(per_image)]).astype(np.int64)


def gather_records(recs, offsets, dist, device, dst=0, report=None):
    """Host records (any record dtype) + per-image offsets of this rank -> all ranks'
    (records, offsets) on `dst` (None, None elsewhere); the host-side form of
    gather_packed for callers that already hold their records on the host."""
    recs = np.ascontiguousarray(recs)
    counts = np.diff(np.asarray(offsets, dtype=np.int64))
    n_max_t = torch.tensor([len(counts)], dtype=torch.int64, device=device)
    dist.all_reduce(n_max_t, op=dist.ReduceOp.MAX)
    data = torch.from_numpy(recs.view(np.uint8).reshape(-1))
    if device.type == 'cuda':
        data = data.to(device)
    return gather_packed(data, counts, dist, n_max=int(n_max_t.item()), dtype=recs.dtype,
                         device=device, dst=dst, full=recs.dtype == ANN_DTYPE, report=report)
