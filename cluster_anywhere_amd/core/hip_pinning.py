"""Page-lock (hipHostRegister) this node's shared-memory object-store arena in a
GPU worker process, so host→HBM copies of object-store blocks (Data batches,
sample batches, tensors) DMA straight out of the shm arena — no staging copy
into a separate pinned buffer (reference role: the Plasma store's CUDA host
registration; BASELINE north star: "Plasma object store backed by HIP-pinned
shared memory").

The HIP runtime used is the one torch already loaded (same libamdhip64.so, so
the registration is visible to torch's copies). Registration is per process
and idempotent; :func:`arena_contains` tells a caller whether an array's buffer
lies inside the registered range.
"""
from __future__ import annotations

import bisect
import ctypes
import os
import threading
from typing import List, Optional, Tuple

_lock = threading.Lock()
_range: Optional[Tuple[int, int]] = None  # the whole arena once every chunk is registered
_chunks: List[Tuple[int, int]] = []  # registered [start, end) chunks, ascending
_starts: List[int] = []
_tried = False
# Registering the arena costs ~0.12 s/GB, during which the process's other HIP calls
# (copies, launches) wait (measured: 0.55-0.64 s for a 4.9 GB arena). CAAMD_PIN_CHUNK_MB
# > 0 registers it in chunks of that size instead (a copy may then not span two
# chunks, see arena_contains); 0 = one registration (default: it spreads the same
# stall, measured no gain, and a chunked arena loses the DMA path for blocks
# straddling a chunk boundary).
CHUNK = int(os.environ.get("CAAMD_PIN_CHUNK_MB", "0")) << 20


def _hip():
    import torch  # noqa: F401  (ensures torch's HIP runtime is loaded first)

    for path in open("/proc/self/maps").read().split("\n"):
        if "libamdhip64.so" in path:
            return ctypes.CDLL(path.split()[-1])
    return ctypes.CDLL("libamdhip64.so")


def pin_object_store(max_bytes: Optional[int] = None) -> bool:
    """Register the arena with HIP (once, chunk by chunk). False if there is no GPU,
    no arena, or the registration failed (callers then fall back to staging copies
    for what is not registered)."""
    global _range, _tried
    with _lock:
        if _range is not None:
            return True
        if _tried:
            return False
        _tried = True
        if os.environ.get("CAAMD_PIN_OBJECT_STORE", "1") == "0":
            return False
        import torch

        if not torch.cuda.is_available():
            return False
        from . import context

        w = context.worker
        store = getattr(w, "store", None) if w is not None else None
        if store is None:
            return False
        base, size = int(store.address(0)), int(store.map_size)
        if max_bytes is not None:
            size = min(size, max_bytes)
        hip = _hip()
        hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
        hip.hipHostRegister.restype = ctypes.c_int
        page = 1 << 21
        step = max(page, (CHUNK // page) * page) if CHUNK > 0 else size
        off = 0
        while off < size:
            n = min(step, size - off)
            if hip.hipHostRegister(ctypes.c_void_p(base + off), ctypes.c_size_t(n), 0) != 0:
                return bool(_chunks)
            _chunks.append((base + off, base + off + n))
            _starts.append(base + off)
            off += n
        _range = (base, base + size)
        return True


_async_started = False


def pin_object_store_async() -> None:
    """Start :func:`pin_object_store` once, on a background thread (callers take the
    staging copy until :func:`arena_contains` says the arena is registered)."""
    global _async_started
    with _lock:
        if _async_started or _tried:
            return
        _async_started = True
    threading.Thread(target=pin_object_store, name="caamd-pin-arena", daemon=True).start()


def arena_contains(arr) -> bool:
    """True if ``arr``'s buffer lies inside ONE registered chunk (a copy must not
    span two registrations)."""
    if not _chunks:
        return False
    try:
        ptr = arr.__array_interface__["data"][0]
    except Exception:
        return False
    i = bisect.bisect_right(_starts, ptr) - 1
    if i < 0 or i >= len(_chunks):
        return False
    lo, hi = _chunks[i]
    return lo <= ptr and ptr + arr.nbytes <= hi
