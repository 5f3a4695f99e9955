"""Random access by key over a Dataset (reference: data/random_access_dataset.py).
The dataset is sorted by ``key`` and range-partitioned over ``num_workers``
actors; each holds its sorted partition and answers lookups by binary search.
The driver keeps only the partition boundaries."""
from __future__ import annotations

import bisect
from typing import Any, List

import numpy as np

from . import block as B


class _Server:
    def __init__(self, block, key):
        self.key = key
        block = B.to_numpy(block) if block else block
        self.keys = np.asarray(block[key]) if block else np.zeros(0)
        self.block = block

    def get(self, k):
        i = int(np.searchsorted(self.keys, k))
        if i < len(self.keys) and self.keys[i] == k:
            return {c: B._scalar(v[i]) for c, v in B.to_numpy(self.block).items()}
        return None

    def multiget(self, ks):
        return [self.get(k) for k in ks]


class RandomAccessDataset:
    def __init__(self, ds, key: str, num_workers: int):
        from ..core.api import get, remote

        blk = B.concat([get(r) for r, _ in ds.sort(key)._execute()])
        n = B.num_rows(blk)
        bounds = np.linspace(0, n, num_workers + 1).astype(int)
        Server = remote(num_cpus=0)(_Server)
        self.key = key
        self.workers, self.lows = [], []
        for i in range(num_workers):
            part = B.slice_block(blk, int(bounds[i]), int(bounds[i + 1]))
            if B.num_rows(part) == 0:
                continue
            self.workers.append(Server.remote(part, key))
            self.lows.append(part[key][0])

    def _worker(self, k):
        return self.workers[max(0, bisect.bisect_right(self.lows, k) - 1)]

    def get_async(self, k):
        return self._worker(k).get.remote(k)

    def multiget(self, keys: List[Any]):
        from ..core.api import get

        return get([self.get_async(k) for k in keys])

    def stats(self) -> str:
        return f"RandomAccessDataset(key={self.key!r}, workers={len(self.workers)})"
