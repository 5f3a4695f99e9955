"""Shared-memory channels (reference: python/ray/experimental/channel/
shared_memory_channel.py, common.py; the C++ side is
src/ray/core_worker/experimental_mutable_object_manager.cc).

A :class:`Channel` is one writer → N readers, backed by the native lock-free ring
in ``csrc/runtime/channel.cc`` (a /dev/shm file of ``num_slots`` fixed-size
slots). Every reader receives every value, in order; the writer blocks when the
slowest reader is ``num_slots`` values behind (that is the compiled graph's
``max_inflight_executions``). Values are pickled (protocol 5); a value larger
than a slot is put in the object store and only its reference goes through the
ring. The handle pickles by name, so passing it to an actor attaches that
process to the same ring.
"""
from __future__ import annotations

import os
import pickle
from typing import Any, Optional

_REF_FLAG = 1
DEFAULT_SLOT_BYTES = 1 << 20
DEFAULT_SLOTS = 8


class ChannelClosedError(EOFError):
    pass


def _native():
    from .. import _native  # noqa: WPS433

    return _native


def _t(timeout: Optional[float]) -> float:
    return -1.0 if timeout is None else float(timeout)


class Channel:
    def __init__(self, num_readers: int = 1, num_slots: int = DEFAULT_SLOTS,
                 slot_bytes: int = DEFAULT_SLOT_BYTES, name: Optional[str] = None,
                 _create: bool = True):
        self.name = name or f"caamd-chan-{os.getpid()}-{os.urandom(6).hex()}"
        self._owner = _create
        self._c = _native().Channel(self.name, _create, num_readers, num_slots, slot_bytes)

    # -- pickling: attach by name in the receiving process ----------------------
    def __reduce__(self):
        return (_attach, (self.name,))

    @property
    def num_readers(self) -> int:
        return self._c.num_readers

    @property
    def num_slots(self) -> int:
        return self._c.num_slots

    def write(self, value: Any, timeout: Optional[float] = None) -> None:
        data = pickle.dumps(value, protocol=5)
        flags = 0
        if len(data) > self._c.slot_bytes:
            from ..core import api

            data = pickle.dumps(api.put(value), protocol=5)
            flags = _REF_FLAG
        try:
            self._c.write(data, flags, _t(timeout))
        except ValueError:
            raise TimeoutError(f"channel {self.name}: write timed out") from None
        except StopIteration:
            raise ChannelClosedError(self.name) from None

    def read(self, reader: int = 0, timeout: Optional[float] = None) -> Any:
        try:
            data, flags = self._c.read(reader, _t(timeout))
        except ValueError:
            raise TimeoutError(f"channel {self.name}: read timed out") from None
        except StopIteration:
            raise ChannelClosedError(self.name) from None
        v = pickle.loads(data)
        if flags & _REF_FLAG:
            from ..core import api

            v = api.get(v)
        return v

    def close(self) -> None:
        """Wake every blocked reader/writer with :class:`ChannelClosedError`."""
        self._c.close()

    def destroy(self) -> None:
        self._c.close()
        self._c.unlink()

    @property
    def closed(self) -> bool:
        return self._c.closed


def _attach(name: str) -> Channel:
    ch = Channel.__new__(Channel)
    ch.name = name
    ch._owner = False
    ch._c = _native().Channel(name, False)
    return ch


__all__ = ["Channel", "ChannelClosedError"]
