"""Batch driver (decoder/generator/generator.py:14-107).

The reference moves every field batch to the host (`.cpu().numpy()`, generator.py:65) and
maps images over a multiprocessing.Pool.  Here the fields stay in HBM and the whole batch
is decoded by one device launch sequence; `worker_pool` is accepted for API compatibility
and ignored.
"""
import logging
import time

import torch

from ...distributed import shard

LOG = logging.getLogger(__name__)


def _apply(f, items):
    """generator.py:48-54: f on every item that is not a list or tuple, nested."""
    if items is None:
        return None
    if isinstance(items, (list, tuple)):
        return [_apply(f, i) for i in items]
    return f(items)


def per_image(heads):
    """Batch-major head outputs -> one nested head list per image (generator.py:66-74:
    the reference zips iterators over the batch dimension until the first runs out)."""
    lens = []
    _apply(lambda t: lens.append(len(t)), heads)
    n = min(lens) if lens else 0
    return [_apply(lambda t, i=i: t[i], heads) for i in range(n)]


class DummyPool():
    @staticmethod
    def starmap(f, iterable):
        return [f(*i) for i in iterable]


class Generator:
    # decode_heads(heads, group=, dst=, local=) is implemented (checked by batch() before
    # the model runs on a rank's share)
    supports_sharding = False

    def __init__(self, worker_pool=None):
        self.worker_pool = DummyPool() if not worker_pool else worker_pool
        self.last_decoder_time = 0.0
        self.last_nn_time = 0.0

    def __getstate__(self):
        return {k: v for k, v in self.__dict__.items() if k not in ('worker_pool',)}

    @staticmethod
    def _heads(model, image_batch, *, device=None):
        """Network forward: the model's head outputs, batch-major tensors on the device."""
        start = time.time()
        with torch.no_grad():
            if device is not None:
                image_batch = image_batch.to(device, non_blocking=True)
            with torch.autograd.profiler.record_function('model'):
                heads = model(image_batch)
        LOG.debug('nn processing time: %.3fs', time.time() - start)
        return heads

    @staticmethod
    def fields_batch(model, image_batch, *, device=None):
        """From image batch to field batch (generator.py:43-78): one entry per image, each
        the model's (nested) head list indexed by that image, as the reference returns it.
        The per-image fields are views of the device outputs (the reference's
        `.cpu().numpy()` copy is skipped)."""
        heads = Generator._heads(model, image_batch, device=device)
        return per_image(heads)

    def __call__(self, fields, *, initial_annotations=None):
        raise NotImplementedError()

    def decode_heads(self, heads):
        """Every head output of a batch (the model's list, each (B, ...)) -> one list of
        annotations per image; the subclass reads the heads its FieldConfig names."""
        raise NotImplementedError()

    def batch(self, model, image_batch, *, device=None, group=None, dst=0):
        """From image batch straight to annotations batch (generator.py:84-101): the head
        list of any FieldConfig (single-scale, dense connections, multi-scale) is decoded
        as one device batch instead of per image over a worker pool.

        With a torch.distributed process `group` (one rank per GPU), every rank passes the
        same image batch, runs the model on its `distributed.shard` of the images only and
        decodes them, and rank `dst` returns the annotation lists of the whole batch
        (CifCaf.decode_batch); the other ranks return None."""
        if group is not None:
            if not self.supports_sharding:
                raise NotImplementedError('image-sharded decoding is not implemented for '
                                          + type(self).__name__)
            import torch.distributed as dist  # pylint: disable=import-outside-toplevel
            a, b = shard(len(image_batch), dist.get_rank(group), dist.get_world_size(group))
            image_batch = image_batch[a:b]
        start_nn = time.perf_counter()
        heads = (self._heads(model, image_batch, device=device)
                 if group is None or len(image_batch) else None)
        self.last_nn_time = time.perf_counter() - start_nn
        start = time.perf_counter()
        result = (self.decode_heads(heads) if group is None else
                  self.decode_heads(heads, group=group, dst=dst, local=True))
        self.last_decoder_time = time.perf_counter() - start
        LOG.debug('time: nn = %.3fs, dec = %.3fs', self.last_nn_time, self.last_decoder_time)
        return result
