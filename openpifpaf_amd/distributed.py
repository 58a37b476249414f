"""Image-sharded multi-GPU decoding.

Images are independent through the whole decoder (cifcaf.py:67-118 touches one image's
fields only), so N ranks split a batch by image with no data-path collective; the only
exchange is collecting every rank's finished annotation records on rank 0.  One process
per GPU; `nccl` (RCCL over xGMI) on the box, `gloo` in the CPU tests.
"""
import numpy as np
import torch

from ._abi import ANN_DTYPE


def shard(n_images, rank, world):
    """[start, stop) of the images rank `rank` decodes: contiguous, sizes differ by <= 1."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError('bad rank {} of {}'.format(rank, world))
    base, extra = divmod(n_images, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_records(recs, offsets, dist, device):
    """All-gather every rank's packed pp_ann records and per-image offsets.

    `recs` is this rank's ANN_DTYPE array, `offsets` its per-image offsets (len n + 1).
    Returns (records, offsets) of all ranks in rank order (images of rank 0 first), on every
    rank.  Records and offsets travel as one padded uint8 tensor per rank (one all-gather
    after the (count, images) exchange).
    """
    world = dist.get_world_size()
    width = ANN_DTYPE.itemsize
    n_img = len(offsets) - 1
    meta = torch.tensor([len(recs), n_img], dtype=torch.int64, device=device)
    metas = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta)
    counts = [int(m[0].item()) for m in metas]
    n_imgs = [int(m[1].item()) for m in metas]
    # one padded uint8 buffer per rank: the records, then the offsets (int64) in the rows
    # after them, so the data travels in a single all-gather
    cap = max(counts)
    off_rows = -(-8 * (max(n_imgs) + 1) // width)
    buf = torch.zeros((cap + off_rows, width), dtype=torch.uint8, device=device)
    if len(recs):
        buf[:len(recs)] = torch.from_numpy(
            np.ascontiguousarray(recs).view(np.uint8).reshape(-1, width)).to(device)
    offs = np.zeros(off_rows * width // 8, dtype=np.int64)
    offs[:n_img + 1] = np.asarray(offsets, dtype=np.int64)
    buf[cap:] = torch.from_numpy(offs.view(np.uint8).reshape(off_rows, width)).to(device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)

    out_recs, out_offs, base = [], [0], 0
    for r in range(world):
        host = parts[r].cpu().numpy()
        out_recs.append(host[:counts[r]].reshape(-1).view(ANN_DTYPE) if counts[r] else
                        np.zeros(0, ANN_DTYPE))
        o = np.ascontiguousarray(host[cap:]).reshape(-1).view(np.int64)[:n_imgs[r] + 1]
        out_offs.extend((base + o[1:]).tolist())
        base += counts[r]
    return np.concatenate(out_recs), np.asarray(out_offs, dtype=np.int64)
