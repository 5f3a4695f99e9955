"""Distributed FIFO queue backed by an async actor (reference: python/ray/util/queue.py:21)."""
from __future__ import annotations

import asyncio
import queue as _q
from typing import Any, List, Optional


class Empty(_q.Empty):
    pass


class Full(_q.Full):
    pass


class _QueueActor:
    def __init__(self, maxsize):
        self.maxsize = maxsize
        self.queue = asyncio.Queue(maxsize)

    def qsize(self):
        return self.queue.qsize()

    def empty(self):
        return self.queue.empty()

    def full(self):
        return self.queue.full()

    async def put(self, item, timeout=None):
        try:
            await asyncio.wait_for(self.queue.put(item), timeout)
        except asyncio.TimeoutError:
            raise Full

    async def put_batch(self, items, timeout=None):
        for item in items:
            try:
                await asyncio.wait_for(self.queue.put(item), timeout)
            except asyncio.TimeoutError:
                raise Full

    async def get(self, timeout=None):
        try:
            return await asyncio.wait_for(self.queue.get(), timeout)
        except asyncio.TimeoutError:
            raise Empty

    def put_nowait(self, item):
        self.queue.put_nowait(item)

    def put_nowait_batch(self, items):
        if self.maxsize > 0 and len(items) + self.qsize() > self.maxsize:
            raise Full(f"Cannot add {len(items)} items to queue of size {self.qsize()} "
                       f"and maxsize {self.maxsize}.")
        for item in items:
            self.queue.put_nowait(item)

    def get_nowait(self):
        return self.queue.get_nowait()

    def get_nowait_batch(self, num_items):
        if num_items > self.qsize():
            raise Empty(f"Cannot get {num_items} items from queue of size {self.qsize()}.")
        return [self.queue.get_nowait() for _ in range(num_items)]


class Queue:
    def __init__(self, maxsize: int = 0, actor_options: Optional[dict] = None):
        from ..core.api import remote

        self.maxsize = maxsize
        self.actor = remote(**(actor_options or {}))(_QueueActor).remote(maxsize)

    def __len__(self):
        return self.size()

    def size(self) -> int:
        from ..core.api import get

        return get(self.actor.qsize.remote())

    def qsize(self):
        return self.size()

    def empty(self) -> bool:
        from ..core.api import get

        return get(self.actor.empty.remote())

    def full(self) -> bool:
        from ..core.api import get

        return get(self.actor.full.remote())

    def put(self, item: Any, block: bool = True, timeout: Optional[float] = None) -> None:
        from ..core.api import get

        if self.maxsize <= 0:
            self.actor.put_nowait.remote(item)
        elif not block:
            try:
                get(self.actor.put_nowait.remote(item))
            except _q.Full:
                raise Full
        else:
            if timeout is not None and timeout < 0:
                raise ValueError("'timeout' must be a non-negative number")
            try:
                get(self.actor.put.remote(item, timeout))
            except Full:
                raise
            except _q.Full:
                raise Full

    def put_nowait(self, item):
        return self.put(item, block=False)

    def put_nowait_batch(self, items):
        from ..core.api import get

        try:
            get(self.actor.put_nowait_batch.remote(list(items)))
        except _q.Full as e:
            raise Full(str(e))

    def get(self, block: bool = True, timeout: Optional[float] = None) -> Any:
        from ..core.api import get

        if not block:
            try:
                return get(self.actor.get_nowait.remote())
            except (asyncio.QueueEmpty, _q.Empty):
                raise Empty
        if timeout is not None and timeout < 0:
            raise ValueError("'timeout' must be a non-negative number")
        try:
            return get(self.actor.get.remote(timeout))
        except _q.Empty:
            raise Empty

    def get_nowait(self):
        return self.get(block=False)

    def get_nowait_batch(self, num_items: int) -> List[Any]:
        from ..core.api import get

        try:
            return get(self.actor.get_nowait_batch.remote(num_items))
        except _q.Empty as e:
            raise Empty(str(e))

    def shutdown(self, force: bool = False, grace_period_s: int = 5):
        from ..core.api import kill

        if self.actor is not None:
            kill(self.actor)
            self.actor = None
