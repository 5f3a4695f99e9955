"""Compiled-graph defaults (reference role: python/ray/dag/context.py DAGContext):
``experimental_compile()`` takes its ring depth and slot size from here unless
passed explicitly; environment overrides use the reference's variable names."""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass

_lock = threading.Lock()
_current = None


def _env(name, default, cast):
    v = os.environ.get(f"RAY_CGRAPH_{name}")
    return cast(v) if v is not None else default


@dataclass
class DAGContext:
    submit_timeout: int = _env("submit_timeout", 10, int)
    get_timeout: int = _env("get_timeout", 10, int)
    teardown_timeout: int = _env("teardown_timeout", 30, int)
    read_iteration_timeout: float = _env("read_iteration_timeout_s", 0.1, float)
    buffer_size_bytes: int = _env("buffer_size_bytes", 0, int)  # 0: the channel default slot size
    max_inflight_executions: int = _env("max_inflight_executions", 8, int)
    overlap_gpu_communication: bool = _env("overlap_gpu_communication", False, lambda v: v == "1")

    def __post_init__(self):
        if self.read_iteration_timeout > self.get_timeout:
            raise ValueError(f"read_iteration_timeout ({self.read_iteration_timeout}) must be <= "
                             f"get_timeout ({self.get_timeout})")

    @staticmethod
    def get_current() -> "DAGContext":
        global _current
        with _lock:
            if _current is None:
                _current = DAGContext()
            return _current
