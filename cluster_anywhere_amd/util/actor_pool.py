"""ActorPool: schedule work items over a fixed set of actors
(API of the reference's python/ray/util/actor_pool.py:13).

Design: every submitted value gets a sequence number. A value runs as soon as an
actor is idle (otherwise it waits in a FIFO backlog); its in-flight record maps
the returned ObjectRef back to (sequence number, actor). A finished task frees
its actor immediately (the next backlog item starts on it) and its result is
parked until consumed. Results are consumed in submission order (``get_next``)
or completion order (``get_next_unordered``); the two may be mixed — the ordered
cursor skips sequence numbers that were already consumed out of order.
"""
from __future__ import annotations

import collections
from typing import Any, Callable, Deque, Dict, Iterable, List, Optional, Tuple

from ..core import api as core


class ActorPool:
    def __init__(self, actors: List):
        self._idle: Deque = collections.deque(actors)
        self._members = list(actors)
        self._backlog: Deque[Tuple[int, Callable, Any]] = collections.deque()
        self._running: Dict[int, Tuple[Any, Any]] = {}  # seq -> (actor, ref)
        self._done: Dict[int, Any] = {}                 # seq -> ref of a finished task
        self._abandoned: Dict[int, Any] = {}            # timed-out seqs given up on: seq -> actor
        self._seq = 0
        self._cursor = 0
        self._taken = set()  # seqs >= _cursor consumed out of order

    # ------------------------------------------------------------------ submit
    def submit(self, fn: Callable, value: Any) -> None:
        """Run ``fn(actor, value)`` (returning an ObjectRef) on an idle actor, or
        queue it until one frees up."""
        seq = self._seq
        self._seq += 1
        if self._idle:
            self._launch(seq, fn, value, self._idle.popleft())
        else:
            self._backlog.append((seq, fn, value))

    def _launch(self, seq, fn, value, actor):
        self._running[seq] = (actor, fn(actor, value))

    def _free(self, actor):
        if self._backlog:
            self._launch(*self._backlog.popleft(), actor)
        else:
            self._idle.append(actor)

    def _reap(self, timeout: Optional[float]) -> bool:
        """Move finished tasks (at least one, waiting up to ``timeout``) to _done."""
        refs = {ref: seq for seq, (_, ref) in self._running.items()}
        if not refs:
            return False
        ready, _ = core.wait(list(refs), num_returns=1, timeout=timeout)
        if not ready:
            return False
        more, _ = core.wait(list(refs), num_returns=len(refs), timeout=0)
        for r in set(ready) | set(more):
            seq = refs[r]
            actor, ref = self._running.pop(seq)
            if seq in self._abandoned:
                self._abandoned.pop(seq)
            else:
                self._done[seq] = ref
            self._free(actor)
        return True

    # ------------------------------------------------------------------ results
    def has_next(self) -> bool:
        live = len(self._running) - len(self._abandoned)
        return live > 0 or bool(self._backlog) or bool(self._done)

    def get_next(self, timeout: Optional[float] = None, ignore_if_timedout: bool = False):
        """Next result in submission order."""
        while self._cursor in self._taken:
            self._taken.discard(self._cursor)
            self._cursor += 1
        if not self.has_next():
            raise StopIteration("ActorPool has no pending results")
        seq = self._cursor
        while seq not in self._done:
            if not self._reap(timeout):
                if ignore_if_timedout:
                    self._give_up(seq)
                raise TimeoutError(f"result #{seq} not ready within {timeout}s")
        self._cursor += 1
        return core.get(self._done.pop(seq))

    def get_next_unordered(self, timeout: Optional[float] = None, ignore_if_timedout: bool = False):
        """Any finished result (completion order)."""
        if not self.has_next():
            raise StopIteration("ActorPool has no pending results")
        if not self._done and not self._reap(timeout):
            raise TimeoutError(f"no result ready within {timeout}s")
        seq = min(self._done)
        if seq == self._cursor:
            self._cursor += 1
        else:
            self._taken.add(seq)
        return core.get(self._done.pop(seq))

    def _give_up(self, seq):
        self._cursor = seq + 1
        if seq in self._running:
            self._abandoned[seq] = self._running[seq][0]
        else:  # still queued: drop it from the backlog
            self._backlog = collections.deque(b for b in self._backlog if b[0] != seq)

    # ------------------------------------------------------------------ map
    def map(self, fn: Callable, values: Iterable) -> Iterable:
        self._discard_pending()
        for v in values:
            self.submit(fn, v)
        return self._iter(self.get_next)

    def map_unordered(self, fn: Callable, values: Iterable) -> Iterable:
        self._discard_pending()
        for v in values:
            self.submit(fn, v)
        return self._iter(self.get_next_unordered)

    def _discard_pending(self):
        # a new map() starts from a quiet pool: finish and drop unconsumed results
        while self._running or self._backlog:
            self._reap(None)
        self._done.clear()
        self._cursor = self._seq
        self._taken.clear()

    def _iter(self, getter):
        while self.has_next():
            yield getter()

    # ------------------------------------------------------------------ membership
    def has_free(self) -> bool:
        if self._abandoned:
            self._reap(0)
        return bool(self._idle) and not self._backlog

    def pop_idle(self):
        if not self.has_free():
            return None
        a = self._idle.popleft()
        self._members = [m for m in self._members if m is not a]
        return a

    def push(self, actor) -> None:
        if any(m is actor for m in self._members):
            raise ValueError("this actor is already a member of the pool")
        self._members.append(actor)
        self._free(actor)
