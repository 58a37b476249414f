"""Image-sharded multi-GPU decoding.

Images are independent through the whole decoder (cifcaf.py:67-118 touches one image's
fields only), so N ranks split a batch by image with no data-path collective; the only
exchange is collecting every rank's finished annotation records on rank 0 — the
replacement of the reference's `worker_pool.starmap` result list (generator.py:96-97).
One process per GPU; `nccl` (RCCL over xGMI) on the box, `gloo` in the CPU tests.

The gather moves compact records (pp_pack_compact) straight from the device buffer they
were packed into: one small all-gather of (images, records, per-image counts), then a
batch of point-to-point sends to rank 0 with exact sizes (no padding, no host round trip
on the sending ranks).  With gloo the records travel from host memory.
"""
import contextlib

import numpy as np
import torch


def shard(n_images, rank, world):
    """[start, stop) of the images rank `rank` decodes: contiguous, sizes differ by <= 1."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError('bad rank {} of {}'.format(rank, world))
    base, extra = divmod(n_images, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def max_shard(n_images, world):
    return -(-n_images // world)


def _meta_gather(dist, counts, n_max, device):
    """All ranks' (n_images, records, counts[n_max]) as an int64 (world, n_max + 2) array."""
    world = dist.get_world_size()
    meta = np.zeros(n_max + 2, np.int64)
    meta[0], meta[1] = len(counts), int(np.sum(counts))
    meta[2:2 + len(counts)] = counts
    t = torch.from_numpy(meta).to(device)
    out = torch.empty(world * (n_max + 2), dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(out, t)
    return out.cpu().numpy().reshape(world, n_max + 2)


def gather_packed(records, counts, dist, *, n_max, dtype, device, dst=0, stream=None):
    """Collect every rank's packed records on rank `dst`.

    `records`: this rank's records as a uint8 tensor (device memory for nccl, host for
    gloo; at least sum(counts) * dtype.itemsize bytes), `counts`: its per-image record
    counts, `n_max` >= every rank's image count.  On `dst` returns (records of all ranks in
    rank order as a `dtype` array with `image` rebased to the global image index, per-image
    offsets over all images); elsewhere
    (None, None).  With `stream`, the exchange is ordered on it (it must already wait for
    the pack), not behind later work on the current stream."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    width = dtype.itemsize
    counts = np.asarray(counts, dtype=np.int64)
    ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
    with ctx:
        metas = _meta_gather(dist, counts, n_max, device)
        totals = metas[:, 1]
        if rank != dst:
            n = int(totals[rank]) * width
            if n:
                dist.send(records[:n].contiguous(), dst)
            return None, None
        bufs, ops = {}, []
        for r in range(world):
            n = int(totals[r]) * width
            if r == dst or n == 0:
                continue
            bufs[r] = torch.empty(n, dtype=torch.uint8, device=device)
            ops.append(dist.P2POp(dist.irecv, bufs[r], r))
        for req in (dist.batch_isend_irecv(ops) if ops else []):
            req.wait()
        host = torch.empty(int(totals.sum()) * width, dtype=torch.uint8,
                           pin_memory=device.type == 'cuda')
        o = 0
        for r in range(world):
            n = int(totals[r]) * width
            if n:
                host[o:o + n].copy_(records[:n] if r == dst else bufs[r],
                                    non_blocking=device.type == 'cuda')
            o += n
        if device.type == 'cuda':
            torch.cuda.current_stream(device).synchronize()
    recs = host.numpy().view(dtype) if len(host) else np.zeros(0, dtype)
    # a record's image is its index in its rank's batch: rebase to the global image index
    # (rank r's images follow those of ranks < r, as shard() assigns them)
    n_imgs = metas[:, 0]
    img_base = np.repeat(np.concatenate([[0], np.cumsum(n_imgs)[:-1]]), totals)
    if len(recs) and img_base.any():
        recs['image'] += img_base.astype(recs['image'].dtype)
    per_image = np.concatenate([metas[r, 2:2 + metas[r, 0]] for r in range(world)])
    return recs, np.concatenate([[0], np.cumsum(per_image)]).astype(np.int64)


def gather_records(recs, offsets, dist, device, dst=0):
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
                         device=device, dst=dst)
