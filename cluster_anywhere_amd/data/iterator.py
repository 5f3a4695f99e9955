"""DataIterator and streaming_split (reference: python/ray/data/iterator.py,
_internal/iterator/stream_split_iterator.py).

``iter_torch_batches`` stages each batch host→HBM on a side HIP stream from
pinned host memory, one batch ahead of the consumer (so the copy overlaps the
previous step's compute). ``streaming_split(n)`` runs ONE execution of the
dataset inside a coordinator actor and hands its blocks out to ``n`` consumers
(e.g. the ranks of a TorchTrainer) as they ask, epoch by epoch.
"""
from __future__ import annotations

import collections
import threading
from typing import Any, Callable, Dict, Iterator, List, Optional

import numpy as np

from . import block as B


def _batcher(blocks: Iterator[B.Block], batch_size, drop_last, shuffle_buffer, seed):
    rng = np.random.default_rng(seed)
    buf: List[B.Block] = []
    buffered = 0
    for b in blocks:
        if not b or B.num_rows(b) == 0:
            continue
        buf.append(b)
        buffered += B.num_rows(b)
        threshold = max(batch_size or 0, shuffle_buffer or 0)
        while batch_size is not None and buffered >= threshold and buffered >= batch_size:
            merged = B.concat(buf)
            if shuffle_buffer:
                merged = B.take_indices(merged, rng.permutation(B.num_rows(merged)))
            out = B.slice_block(merged, 0, batch_size)
            rest = B.slice_block(merged, batch_size, B.num_rows(merged))
            buf = [rest] if B.num_rows(rest) else []
            buffered = B.num_rows(rest)
            yield out
        if batch_size is None:
            yield B.concat(buf)
            buf, buffered = [], 0
    if buf:
        merged = B.concat(buf)
        if shuffle_buffer:
            merged = B.take_indices(merged, rng.permutation(B.num_rows(merged)))
        n = B.num_rows(merged)
        s = 0
        while batch_size is not None and n - s >= batch_size:
            yield B.slice_block(merged, s, s + batch_size)
            s += batch_size
        if n - s > 0 and not drop_last:
            yield B.slice_block(merged, s, n)


def _prefetched(it: Iterator, depth: int) -> Iterator:
    """Run ``it`` in a background thread ``depth`` items ahead."""
    if depth <= 0:
        yield from it
        return
    q: "collections.deque" = collections.deque()
    cv = threading.Condition()
    done = [False]
    err = [None]

    def run():
        try:
            for x in it:
                with cv:
                    while len(q) >= depth and not done[0]:
                        cv.wait()
                    q.append(x)
                    cv.notify_all()
        except BaseException as e:  # noqa
            err[0] = e
        finally:
            with cv:
                done[0] = True
                cv.notify_all()

    th = threading.Thread(target=run, daemon=True)
    th.start()
    while True:
        with cv:
            while not q and not done[0]:
                cv.wait()
            if q:
                x = q.popleft()
                cv.notify_all()
            elif err[0] is not None:
                raise err[0]
            else:
                return
        yield x


class DataIterator:
    def __init__(self, block_ref_source: Callable[[], Iterator]):
        self._source = block_ref_source

    def _blocks(self):
        from ..core.api import get

        for ref, meta in self._source():
            yield get(ref)

    def iter_batches(self, *, batch_size: Optional[int] = 256, batch_format: Optional[str] = "default",
                     drop_last: bool = False, prefetch_batches: int = 1,
                     local_shuffle_buffer_size: Optional[int] = None, local_shuffle_seed=None, **kw):
        it = _batcher(_prefetched(self._blocks(), prefetch_batches), batch_size, drop_last,
                      local_shuffle_buffer_size, local_shuffle_seed)
        for b in it:
            yield B.to_batch(b, batch_format)

    def iter_rows(self):
        for b in self._blocks():
            yield from B.iter_rows(b)

    def iter_torch_batches(self, *, batch_size: Optional[int] = 256, dtypes=None, device="auto",
                           collate_fn=None, drop_last: bool = False, prefetch_batches: int = 1,
                           local_shuffle_buffer_size=None, local_shuffle_seed=None, **kw):
        import torch

        if device == "auto":
            try:
                from ..train.torch import get_device

                device = get_device()
            except Exception:
                device = torch.device("cpu")
        device = torch.device(device) if isinstance(device, str) else device
        gpu = device.type == "cuda"

        registered = False
        if gpu:
            # batches whose numpy buffer lies in the HIP-registered object-store arena
            # are copied straight from shared memory (no pin_memory() staging copy);
            # the arena is registered in the background, batches take the staging
            # copy until it is
            from ..core import hip_pinning

            registered = True
            hip_pinning.pin_object_store_async()

        def to_host(batch):
            if collate_fn is not None:
                return collate_fn(batch)
            from ..core.hip_pinning import arena_contains

            out = {}
            for k, v in batch.items():
                if v.dtype == object:
                    out[k] = v
                    continue
                dt = dtypes.get(k) if isinstance(dtypes, dict) else dtypes
                direct = registered and v.flags["C_CONTIGUOUS"] and arena_contains(v)
                if direct:
                    import warnings

                    with warnings.catch_warnings():  # read-only shm view; only ever read
                        warnings.simplefilter("ignore", UserWarning)
                        t = torch.from_numpy(v)
                    if dt is not None and t.dtype != dt:
                        t = t.to(dt)  # the conversion makes an ordinary host tensor
                        direct = False
                else:
                    t = torch.from_numpy(np.ascontiguousarray(v))
                    if dt is not None:
                        t = t.to(dt)
                if gpu and not direct:
                    t = t.pin_memory()
                out[k] = t
            return out

        host_batches = _prefetched(
            (to_host(b) for b in self.iter_batches(batch_size=batch_size, batch_format="numpy",
                                                   drop_last=drop_last, prefetch_batches=prefetch_batches,
                                                   local_shuffle_buffer_size=local_shuffle_buffer_size,
                                                   local_shuffle_seed=local_shuffle_seed)),
            max(1, prefetch_batches))
        if not gpu:
            yield from host_batches
            return
        # copies run one batch ahead on a side stream; hand_over() makes the compute
        # stream wait for them and record_stream()s every device tensor, so a dropped
        # batch's HBM is not reused by the next copy while compute still reads it
        from ..util.device_transfer import SideStreamMover

        mover = SideStreamMover(device)
        try:
            nxt = None
            for hb in host_batches:
                # hand the staged batch over BEFORE enqueuing the next copy, so the
                # compute stream waits for that batch's copy only
                ready = mover.hand_over(nxt) if nxt is not None else None
                nxt = mover.stage(hb)
                if ready is not None:
                    yield ready
            if nxt is not None:
                yield mover.hand_over(nxt)
        finally:
            mover.close()

    def materialize(self):
        from .dataset import Dataset

        refs = list(self._source())
        ds = Dataset(("refs", refs))
        ds._materialized = refs
        return ds

    def stats(self):
        return ""


class _SplitCoordinator:
    """Actor: executes the dataset once per epoch, deals blocks to n consumers
    round-robin as they ask (fast consumers are not held back by slow ones
    beyond one block)."""

    def __init__(self, ds, n, equal):
        self.ds = ds
        self.n = n
        self.equal = equal
        self.epoch = -1
        self.it = None
        self.queues = None
        self.lock = threading.Lock()
        self.done = True
        self.next_split = 0
        self.started = set()

    def _start(self):
        self.epoch += 1
        self.it = iter(self.ds._execute())
        self.queues = [collections.deque() for _ in range(self.n)]
        self.done = False
        self.next_split = 0

    def get(self, split, epoch):
        with self.lock:
            if epoch > self.epoch:
                if not self.done and self.epoch >= 0:
                    # a consumer moved on: drain the previous epoch first
                    for _ in self.it:
                        pass
                self._start()
            q = self.queues[split]
            while not q and not self.done:
                try:
                    item = next(self.it)
                except StopIteration:
                    self.done = True
                    break
                self.queues[self.next_split].append(item)
                self.next_split = (self.next_split + 1) % self.n
            if q:
                return q.popleft()
            return None


class _SplitIterator(DataIterator):
    def __init__(self, coord, idx):
        self._coord = coord
        self._idx = idx
        self._epoch = 0
        super().__init__(self._gen)

    def _gen(self):
        from ..core.api import get

        ep = self._epoch
        self._epoch += 1
        while True:
            item = get(self._coord.get.remote(self._idx, ep))
            if item is None:
                return
            yield item

    def __reduce__(self):
        return (_rebuild_split, (self._coord, self._idx, self._epoch))


def _rebuild_split(coord, idx, epoch):
    s = _SplitIterator(coord, idx)
    s._epoch = epoch
    return s


def make_streaming_split(ds, n, equal) -> List[DataIterator]:
    from ..core.api import remote

    coord = remote(num_cpus=0, max_concurrency=max(4, 2 * n))(_SplitCoordinator).remote(ds, n, equal)
    return [_SplitIterator(coord, i) for i in range(n)]
