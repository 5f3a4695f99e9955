"""Binary IDs (reference: src/ray/common/id.h). All IDs are random bytes with a
``hex()`` form; object IDs are 24 bytes = the object-store key width."""
from __future__ import annotations

import os
import threading

_counter_lock = threading.Lock()
_counter = 0


def _rand(n: int) -> bytes:
    return os.urandom(n)


class BaseID:
    SIZE = 16
    __slots__ = ("_b",)

    def __init__(self, b: bytes):
        if len(b) != self.SIZE:
            raise ValueError(f"{type(self).__name__} needs {self.SIZE} bytes, got {len(b)}")
        self._b = bytes(b)

    @classmethod
    def from_random(cls):
        return cls(_rand(cls.SIZE))

    @classmethod
    def from_hex(cls, h: str):
        return cls(bytes.fromhex(h))

    @classmethod
    def nil(cls):
        return cls(b"\xff" * cls.SIZE)

    def is_nil(self):
        return self._b == b"\xff" * self.SIZE

    def binary(self) -> bytes:
        return self._b

    def hex(self) -> str:
        return self._b.hex()

    def __hash__(self):
        return hash(self._b)

    def __eq__(self, other):
        return type(self) is type(other) and self._b == other._b

    def __repr__(self):
        return f"{type(self).__name__}({self.hex()})"

    def __reduce__(self):
        return (type(self), (self._b,))


class JobID(BaseID):
    SIZE = 4


class NodeID(BaseID):
    SIZE = 16


class WorkerID(BaseID):
    SIZE = 16


class ActorID(BaseID):
    SIZE = 16


class TaskID(BaseID):
    SIZE = 16


class PlacementGroupID(BaseID):
    SIZE = 16


class FunctionID(BaseID):
    SIZE = 16


class ObjectID(BaseID):
    """24 bytes: 16-byte task id + 8-byte return/put index."""

    SIZE = 24

    @staticmethod
    def for_task_return(task_id: bytes, index: int) -> bytes:
        return task_id + (index + 1).to_bytes(8, "little")

    @staticmethod
    def for_put(worker_prefix: bytes) -> bytes:
        global _counter
        with _counter_lock:
            _counter += 1
            c = _counter
        return worker_prefix[:8] + _rand(8) + (c | (1 << 63)).to_bytes(8, "little")


UniqueID = BaseID
