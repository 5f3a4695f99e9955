"""Host -> HBM batch staging on a side HIP stream, safe against allocator reuse.

Used by ``Dataset.iter_torch_batches`` (data/iterator.py) and the Train device
loader (train/torch/__init__.py ``prepare_data_loader``). Reference role:
python/ray/train/torch/train_loop_utils.py:688-703 (the reference's
``_WrappedDataLoader`` waits on its copy stream and calls ``record_stream`` on
every moved tensor before handing the batch to the compute stream).

Two lifetimes matter when a copy runs on a side stream while the consumer runs
on the compute stream:

* The DEVICE tensor is allocated on the side stream. When the consumer drops it,
  torch's caching allocator returns the block to the side stream's pool at once,
  so the next prefetch copy may overwrite it while compute kernels queued on the
  compute stream still read it. ``record_stream(compute)`` makes the allocator wait
  for the compute stream's work queued at free time.
* The HOST source must stay alive until its copy has executed. torch's pinned
  host allocator tracks its own blocks by event; a block that lies in the HIP-
  registered object-store arena (core/hip_pinning.py, copied without a staging
  ``pin_memory()``) is not torch's, so the mover keeps such host batches
  referenced until an event recorded behind their copy has completed.
"""
from __future__ import annotations

import collections
import os
from typing import Any

_NO_RECORD = os.environ.get("CAAMD_XFER_NO_RECORD_STREAM", "0") == "1"


def _map(obj, fn):
    import torch

    if isinstance(obj, torch.Tensor):
        return fn(obj)
    if isinstance(obj, dict):
        return {k: _map(v, fn) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_map(v, fn) for v in obj)
    return obj


class SideStreamMover:
    """Copies nested batches (tensors / dicts / lists) to ``device`` on a side stream.

    ``stage(host)`` enqueues the copies and returns the device batch; ``hand_over``
    makes the current (compute) stream wait for them and records every device tensor
    on it, so the batch may be dropped by the consumer at any time."""

    def __init__(self, device):
        import torch

        self.device = device
        self.stream = torch.cuda.Stream(device)
        self._hold: "collections.deque" = collections.deque()  # (event, host batch)

    def _release_done(self):
        while self._hold and self._hold[0][0].query():
            self._hold.popleft()

    def stage(self, host: Any, keep_host_alive: bool = True) -> Any:
        import torch

        self._release_done()
        with torch.cuda.stream(self.stream):
            out = _map(host, lambda t: t.to(self.device, non_blocking=True))
            if keep_host_alive:
                ev = torch.cuda.Event()
                ev.record(self.stream)
                self._hold.append((ev, host))
        return out

    def hand_over(self, dev_batch: Any) -> Any:
        import torch

        cur = torch.cuda.current_stream(self.device)
        cur.wait_stream(self.stream)
        if _NO_RECORD:  # negative control for tests/test_device_transfer_gpu.py only
            return dev_batch

        def rec(t):
            if t.device.type == "cuda":
                t.record_stream(cur)
            return t

        return _map(dev_batch, rec)

    def close(self):
        # the host batches must outlive their copies even if the consumer stops early
        if self._hold:
            self.stream.synchronize()
            self._hold.clear()
