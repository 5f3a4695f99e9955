"""Object serialization (reference: python/ray/_private/serialization.py).

Pickle protocol 5 with OUT-OF-BAND buffers: numpy arrays, torch CPU tensors and
bytes-like payloads are not copied into the pickle stream; they are laid out
64-byte aligned after it, so a reader deserialises straight from the shared-memory
arena with zero copies (the arrays it gets back are views of the arena).

Wire/arena format::

    [u32 magic][u32 nbuf][u64 pickle_len][u64 len_i ...][pad->64][pickle][pad->64][buf0][pad->64][buf1]...

``ObjectRef`` / ``ActorHandle`` values found while pickling are recorded as
contained references (the object store keeps them alive while the outer object
lives).  torch GPU tensors are copied to host on serialisation and restored onto
the same device index when the reader has a GPU; with ``tensor_transport="ipc"``
they travel as HIP IPC handles instead (same-node GPU->GPU zero-copy hand-off,
:mod:`cluster_anywhere_amd.experimental.gpu_objects`).
"""
from __future__ import annotations

import io
import pickle
import types
import struct
import sys
import threading
from typing import Any, List, Tuple

import cloudpickle

MAGIC = 0xCA5E0001
ALIGN = 64
_HDR = struct.Struct("<IIQ")
_tls = threading.local()  # .transport: None (host copy) | "ipc" (see experimental/gpu_objects.py)


def _gpu_reduce(t):
    if t.is_cuda and getattr(_tls, "transport", None) == "ipc":
        from ..experimental.gpu_objects import reduce_ipc

        return reduce_ipc(t)
    return _reduce_torch(t)


def _pad(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


class SerializedObject:
    __slots__ = ("pickled", "buffers", "contained_refs", "_size", "_lens")

    def __init__(self, pickled: bytes, buffers, contained_refs):
        self.pickled = pickled
        self.buffers = [b.raw() for b in buffers]
        self.contained_refs = contained_refs
        self._lens = [b.nbytes for b in self.buffers]
        head = _HDR.size + 8 * len(self.buffers)
        size = _pad(head) + _pad(len(pickled))
        for n in self._lens:
            size += _pad(n)
        self._size = size

    @property
    def total_bytes(self) -> int:
        return self._size

    def write_into(self, mv: memoryview, big_copy=None) -> None:
        """``big_copy(offset, buffer)``, if given, copies buffers >= 8 MiB (the
        native multi-threaded arena copy)."""
        nb = len(self.buffers)
        _HDR.pack_into(mv, 0, MAGIC, nb, len(self.pickled))
        off = _HDR.size
        for n in self._lens:
            struct.pack_into("<Q", mv, off, n)
            off += 8
        off = _pad(off)
        mv[off : off + len(self.pickled)] = self.pickled
        off += _pad(len(self.pickled))
        for b, n in zip(self.buffers, self._lens):
            if n:
                src = b.cast("B") if b.format != "B" or b.ndim != 1 else b
                if big_copy is not None and n >= (8 << 20):
                    big_copy(off, src)
                else:
                    mv[off : off + n] = src
            off += _pad(n)

    def to_bytes(self) -> bytes:
        buf = bytearray(self._size)
        self.write_into(memoryview(buf))
        return bytes(buf)


# -- reducers ---------------------------------------------------------------------

def _rebuild_torch(arr, dtype_name, shape, device_index):
    import torch

    import warnings

    with warnings.catch_warnings():  # read-only arena views: torch warns, the data is never written
        warnings.simplefilter("ignore", UserWarning)
        t = torch.from_numpy(arr)
    dt = getattr(torch, dtype_name)
    if dt in (torch.bfloat16,) or t.dtype != dt:
        t = t.view(dt)
    t = t.reshape(shape)
    if device_index is not None and torch.cuda.is_available():
        t = t.to(f"cuda:{min(device_index, torch.cuda.device_count() - 1)}", non_blocking=False)
    return t


def _reduce_torch(t):
    import numpy as np
    import torch

    dev = t.device.index if t.is_cuda else None
    src = t.detach()
    if src.is_cuda:
        src = src.cpu()
    src = src.contiguous()
    dtype_name = str(src.dtype).replace("torch.", "")
    if src.dtype == torch.bfloat16:
        arr = src.view(torch.int16).numpy()
    elif src.dtype == torch.bool:
        arr = src.numpy()
    else:
        try:
            arr = src.numpy()
        except TypeError:
            arr = src.view(torch.uint8).numpy()
    return _rebuild_torch, (arr, dtype_name, tuple(src.shape), dev)


# user-registered serializers (util.register_serializer; reference:
# util/serialization.py): type -> (serializer, deserializer)
_CUSTOM: dict = {}


def _custom_rebuild(deserializer, payload):
    return deserializer(payload)


def _custom_reduce(obj):
    ent = _CUSTOM.get(type(obj))
    if ent is None:
        return None
    ser, de = ent
    return (_custom_rebuild, (de, ser(obj)))


class _Pickler(pickle.Pickler):
    def __init__(self, file, buffer_callback, refs):
        super().__init__(file, protocol=5, buffer_callback=buffer_callback)
        self._refs = refs

    def reducer_override(self, obj):
        from .object_ref import ObjectRef

        if isinstance(obj, ObjectRef):
            self._refs.append(obj.binary())
            return obj.__reduce__()
        if _CUSTOM and type(obj) in _CUSTOM:
            raise pickle.PicklingError("custom serializer")  # by-value path below
        if isinstance(obj, (type, types.FunctionType)) and getattr(obj, "__module__", None) in (
                "__main__", "__mp_main__"):
            # by-reference pickling of a driver-script class/function cannot be
            # resolved in a worker: fall back to cloudpickle (by value)
            raise pickle.PicklingError("__main__ object")
        mod = type(obj).__module__
        if mod == "torch" and "torch" in sys.modules:
            import torch

            if isinstance(obj, torch.Tensor) and not isinstance(obj, torch.nn.Parameter):
                return _gpu_reduce(obj)
        if type(obj).__name__ == "State" and mod == "starlette.datastructures":
            return (type(obj), (dict(obj._state),))
        return NotImplemented


class _CloudPickler(cloudpickle.CloudPickler):
    def __init__(self, file, buffer_callback, refs):
        super().__init__(file, protocol=5, buffer_callback=buffer_callback)
        self._refs = refs

    def reducer_override(self, obj):
        from .object_ref import ObjectRef

        if isinstance(obj, ObjectRef):
            self._refs.append(obj.binary())
            return obj.__reduce__()
        if _CUSTOM:
            red = _custom_reduce(obj)
            if red is not None:
                return red
        if type(obj).__module__ == "torch" and "torch" in sys.modules:
            import torch

            if isinstance(obj, torch.Tensor) and not isinstance(obj, torch.nn.Parameter):
                return _gpu_reduce(obj)
        if type(obj).__name__ == "State" and type(obj).__module__ == "starlette.datastructures":
            # starlette's State.__getattr__ recurses when unpickled attribute-by-attribute
            return (type(obj), (dict(obj._state),))
        if type(obj).__name__ == "MockValSer" and type(obj).__module__ == "pydantic._internal._mock_val_ser":
            # same __getattr__ recursion for pydantic's lazy validator placeholders (FastAPI apps)
            kind = "validator" if obj._val_or_ser.__name__ == "SchemaValidator" else "serializer"
            return (_rebuild_mock_val_ser, (obj._error_message, obj._code, kind, obj._attempt_rebuild))
        return super().reducer_override(obj)


def _rebuild_mock_val_ser(msg, code, kind, attempt):
    from pydantic._internal._mock_val_ser import MockValSer

    return MockValSer(msg, code=code, val_or_ser=kind, attempt_rebuild=attempt)


def serialize(value: Any, tensor_transport: Any = None) -> SerializedObject:
    """``tensor_transport="ipc"``: GPU tensors travel as HIP IPC handles (zero
    copy for readers on the same node) instead of host copies."""
    buffers: List[pickle.PickleBuffer] = []
    refs: List[bytes] = []
    f = io.BytesIO()
    prev = getattr(_tls, "transport", None)
    _tls.transport = tensor_transport
    try:
        try:
            _Pickler(f, buffers.append, refs).dump(value)
        except Exception:
            buffers.clear()
            refs.clear()
            f = io.BytesIO()
            _CloudPickler(f, buffers.append, refs).dump(value)
    finally:
        _tls.transport = prev
    return SerializedObject(f.getvalue(), buffers, refs)


def deserialize(mv) -> Any:
    mv = memoryview(mv)
    magic, nb, plen = _HDR.unpack_from(mv, 0)
    if magic != MAGIC:
        raise ValueError("corrupt object (bad magic)")
    off = _HDR.size
    lens = []
    for _ in range(nb):
        lens.append(struct.unpack_from("<Q", mv, off)[0])
        off += 8
    off = _pad(off)
    pk = mv[off : off + plen]
    off += _pad(plen)
    bufs = []
    for n in lens:
        bufs.append(mv[off : off + n])
        off += _pad(n)
    return pickle.loads(pk, buffers=bufs)


def dumps_function(fn) -> bytes:
    return cloudpickle.dumps(fn, protocol=5)


def loads_function(b: bytes):
    return pickle.loads(b)
