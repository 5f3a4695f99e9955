"""ObjectRef / ObjectRefGenerator (reference: python/ray/includes/object_ref.pxi,
python/ray/_raylet.pyx ObjectRefGenerator). Process-local reference counting:
the first ObjectRef of an id in a process registers a borrow with the head, the
last one to die releases it (batched, ordered on the control connection)."""
from __future__ import annotations

import asyncio
import concurrent.futures
from typing import Optional

from . import context


class ObjectRef:
    __slots__ = ("_id", "__weakref__")

    def __init__(self, id_bytes: bytes, _owned: bool = False):
        self._id = id_bytes
        w = context.worker
        if w is not None:
            w.refs.add(id_bytes, announce=not _owned)

    def __del__(self):
        w = context.worker
        if w is not None:
            try:
                w.refs.remove(self._id, blocking=False)
            except Exception:
                pass

    def binary(self) -> bytes:
        return self._id

    def hex(self) -> str:
        return self._id.hex()

    def task_id(self):
        from .ids import TaskID

        return TaskID(self._id[:16])

    def is_nil(self):
        return self._id == b"\xff" * 24

    def __hash__(self):
        return hash(self._id)

    def __eq__(self, other):
        return isinstance(other, ObjectRef) and other._id == self._id

    def __repr__(self):
        return f"ObjectRef({self._id.hex()})"

    def __reduce__(self):
        w = context.worker
        if w is not None and (w.refs.local_only or w.refs.direct_pending):
            w._escape((self._id,))  # the ref leaves this process: the head must know it
        return (_rebuild_ref, (self._id,))

    # -- futures / asyncio -------------------------------------------------------
    def future(self) -> concurrent.futures.Future:
        return context.worker.get_future(self)

    def __await__(self):
        return asyncio.wrap_future(self.future()).__await__()

    def as_future(self):
        return asyncio.wrap_future(self.future())


def _rebuild_ref(id_bytes):
    return ObjectRef(id_bytes)


_END = object()  # end-of-stream sentinel of ObjectRefGenerator.__anext__


class ObjectRefGenerator:
    """Iterator over the ObjectRefs a ``num_returns="streaming"`` task yields,
    in order, as soon as each is produced (reference: _raylet.pyx:ObjectRefGenerator)."""

    def __init__(self, task_id: bytes, first_ref: Optional[ObjectRef] = None):
        self._task_id = task_id
        self._index = 0
        self._done = False
        self._keep = first_ref

    def __iter__(self):
        return self

    def __next__(self) -> ObjectRef:
        if self._done:
            raise StopIteration
        kind, val = context.worker.gen_next(self._task_id, self._index)
        if kind == "end":
            self._done = True
            raise StopIteration
        if kind == "error":
            self._done = True
            from .serialization import deserialize

            err = deserialize(val)
            raise err.as_instanceof_cause() if hasattr(err, "as_instanceof_cause") else err
        self._index += 1
        return ObjectRef(val, _owned=True)

    def __aiter__(self):
        return self

    def _next_or_end(self):
        # StopIteration cannot cross a Future (asyncio turns it into a TypeError):
        # the end of the stream comes back as a sentinel instead
        try:
            return self.__next__()
        except StopIteration:
            return _END

    async def __anext__(self):
        loop = asyncio.get_running_loop()
        item = await loop.run_in_executor(None, self._next_or_end)
        if item is _END:
            raise StopAsyncIteration
        return item

    def completed(self) -> ObjectRef:
        return self._keep

    def __del__(self):
        # a dropped generator never holds a backpressured producer back again
        if not self._done:
            try:
                w = context.worker
                if w is not None and getattr(w, "alive", False):
                    # never send from a finalizer (it may run inside a send's critical
                    # section): the flush thread delivers it
                    w.gen_drops.append(self._task_id)
            except Exception:
                pass

    def __reduce__(self):
        return (ObjectRefGenerator, (self._task_id, None))


class DynamicObjectRefGenerator:
    """Value of a ``num_returns="dynamic"`` task: an iterable of ObjectRefs."""

    def __init__(self, refs):
        self._refs = list(refs)

    def __iter__(self):
        return iter(self._refs)

    def __len__(self):
        return len(self._refs)
