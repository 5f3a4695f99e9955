"""Distributed FIFO queue (API of the reference's python/ray/util/queue.py:21).

Design: the items live in ONE threaded actor (``_QueueState``): a deque guarded
by a ``threading.Condition``. Every actor method returns a ``(status, payload)``
pair instead of raising through the actor boundary, and the client turns the
status into ``Empty``/``Full``. Blocking ``put``/``get`` wait inside the actor
(one of its ``max_concurrency`` threads parks on the condition), so a blocked
consumer costs no polling round trips; batch operations are all-or-nothing.
"""
from __future__ import annotations

import collections
import queue as _stdq
import threading
import time
from typing import Any, Iterable, List, Optional

OK, EMPTY, FULL = 0, 1, 2


class Empty(_stdq.Empty):
    pass


class Full(_stdq.Full):
    pass


class _QueueState:
    def __init__(self, maxsize: int):
        self._cap = maxsize if maxsize > 0 else None
        self._items = collections.deque()
        self._cv = threading.Condition()

    def _room(self, n: int = 1) -> bool:
        return self._cap is None or len(self._items) + n <= self._cap

    def stat(self):
        with self._cv:
            n = len(self._items)
        return n, (self._cap is not None and n >= self._cap)

    def push(self, items: list, wait_s: Optional[float], all_or_nothing: bool):
        """Append ``items``. wait_s None = block forever, 0 = never block."""
        deadline = None if wait_s is None else time.monotonic() + wait_s
        with self._cv:
            if self._cap is not None and all_or_nothing and len(items) > self._cap:
                return FULL, f"batch of {len(items)} exceeds the queue capacity {self._cap}"
            while not self._room(len(items)):
                left = None if deadline is None else deadline - time.monotonic()
                if left is not None and left <= 0:
                    return FULL, f"queue is full ({len(self._items)}/{self._cap})"
                self._cv.wait(left)
            self._items.extend(items)
            self._cv.notify_all()
        return OK, None

    def pop(self, n: int, wait_s: Optional[float], all_or_nothing: bool):
        deadline = None if wait_s is None else time.monotonic() + wait_s
        with self._cv:
            need = n if all_or_nothing else 1
            while len(self._items) < need:
                left = None if deadline is None else deadline - time.monotonic()
                if left is not None and left <= 0:
                    return EMPTY, f"{len(self._items)} item(s) available, {need} requested"
                self._cv.wait(left)
            out = [self._items.popleft() for _ in range(min(n, len(self._items)))]
            self._cv.notify_all()
        return OK, out


def _check_timeout(timeout):
    if timeout is not None and timeout < 0:
        raise ValueError("timeout must be None or >= 0")


class Queue:
    """FIFO queue usable from any driver, task or actor that holds the handle."""

    def __init__(self, maxsize: int = 0, actor_options: Optional[dict] = None):
        from ..core.api import remote

        self.maxsize = maxsize
        opts = dict(actor_options or {})
        opts.setdefault("max_concurrency", 64)  # parked blocking calls each hold one thread
        opts.setdefault("num_cpus", 0)
        self.actor = remote(**opts)(_QueueState).remote(maxsize)

    # -- introspection
    def _stat(self):
        from ..core.api import get

        return get(self.actor.stat.remote())

    def __len__(self) -> int:
        return self._stat()[0]

    def size(self) -> int:
        return self._stat()[0]

    qsize = size

    def empty(self) -> bool:
        return self._stat()[0] == 0

    def full(self) -> bool:
        return self._stat()[1]

    # -- put
    def _push(self, items, wait_s, batch):
        from ..core.api import get

        status, msg = get(self.actor.push.remote(items, wait_s, batch))
        if status == FULL:
            raise Full(msg)

    def put(self, item: Any, block: bool = True, timeout: Optional[float] = None) -> None:
        _check_timeout(timeout)
        self._push([item], timeout if block else 0, False)

    def put_nowait(self, item: Any) -> None:
        self._push([item], 0, False)

    def put_nowait_batch(self, items: Iterable[Any]) -> None:
        self._push(list(items), 0, True)

    async def put_async(self, item: Any, block: bool = True, timeout: Optional[float] = None) -> None:
        _check_timeout(timeout)
        status, msg = await self.actor.push.remote([item], timeout if block else 0, False)
        if status == FULL:
            raise Full(msg)

    # -- get
    def _pop(self, n, wait_s, batch):
        from ..core.api import get

        status, payload = get(self.actor.pop.remote(n, wait_s, batch))
        if status == EMPTY:
            raise Empty(payload)
        return payload

    def get(self, block: bool = True, timeout: Optional[float] = None) -> Any:
        _check_timeout(timeout)
        return self._pop(1, timeout if block else 0, False)[0]

    def get_nowait(self) -> Any:
        return self._pop(1, 0, False)[0]

    def get_nowait_batch(self, num_items: int) -> List[Any]:
        if num_items < 0:
            raise ValueError("num_items must be >= 0")
        return self._pop(num_items, 0, True)

    async def get_async(self, block: bool = True, timeout: Optional[float] = None) -> Any:
        _check_timeout(timeout)
        status, payload = await self.actor.pop.remote(1, timeout if block else 0, False)
        if status == EMPTY:
            raise Empty(payload)
        return payload[0]

    def shutdown(self, force: bool = False, grace_period_s: int = 5) -> None:
        from ..core.api import kill

        if self.actor is not None:
            kill(self.actor)
            self.actor = None
