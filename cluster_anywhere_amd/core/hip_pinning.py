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

import ctypes
import os
import threading
from typing import Optional, Tuple

_lock = threading.Lock()
_range: Optional[Tuple[int, int]] = None
_tried = False


def _hip():
    import torch  # noqa: F401  (ensures torch's HIP runtime is loaded first)

    for path in open("/proc/self/maps").read().split("\n"):
        if "libamdhip64.so" in path:
            return ctypes.CDLL(path.split()[-1])
    return ctypes.CDLL("libamdhip64.so")


def pin_object_store(max_bytes: Optional[int] = None) -> bool:
    """Register the arena with HIP (once). False if there is no GPU, no arena,
    or the registration failed (callers then fall back to staging copies)."""
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
        rc = hip.hipHostRegister(ctypes.c_void_p(base), ctypes.c_size_t(size), 0)
        if rc != 0:
            return False
        _range = (base, base + size)
        return True


def arena_contains(arr) -> bool:
    if _range is None:
        return False
    try:
        ptr = arr.__array_interface__["data"][0]
    except Exception:
        return False
    return _range[0] <= ptr and ptr + arr.nbytes <= _range[1]
