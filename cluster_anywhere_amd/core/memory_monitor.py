"""Node memory monitor + OOM worker killer (reference: src/ray/common/memory_monitor.cc,
src/ray/raylet/worker_killing_policy_group_by_owner.cc,
python/ray/_private/memory_monitor.py).

The head samples node memory every ``refresh_ms`` (default 250 ms; env
``CAAMD_MEMORY_MONITOR_REFRESH_MS`` or ``RAY_memory_monitor_refresh_ms``, 0
disables). When used/total exceeds ``threshold`` (default 0.95; env
``CAAMD_MEMORY_USAGE_THRESHOLD`` / ``RAY_memory_usage_threshold``) it kills ONE
worker, then waits for the memory to be released before it may kill again.

Victim choice (the reference's group-by-owner policy, simplified to one node):
workers running *retriable* work (tasks with retries left, actors with restarts
left) go first; within a class the most recently started one goes first — it
has made the least progress. A killed task is retried if it has retries left,
otherwise it fails with ``OutOfMemoryError``; a killed actor restarts if
``max_restarts`` allows, else dies with ``ActorDiedError``.

Usage is read from the cgroup (v2 ``memory.current``/``memory.max``, v1
``memory.usage_in_bytes``/``limit_in_bytes``) when the process is limited, else
from ``/proc/meminfo`` (total - available). ``CAAMD_MEMORY_MONITOR_TEST_FILE``
names a file whose content (a float) overrides the usage fraction — the tests
use it to drive the killer deterministically.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple


def _read_int(path: str) -> Optional[int]:
    try:
        with open(path) as f:
            s = f.read().strip()
        return None if s in ("max", "") else int(s)
    except (OSError, ValueError):
        return None


def _meminfo() -> Tuple[int, int]:
    vals = {}
    with open("/proc/meminfo") as f:
        for line in f:
            k, v = line.split(":", 1)
            vals[k] = int(v.split()[0]) * 1024
    total = vals.get("MemTotal", 0)
    avail = vals.get("MemAvailable", vals.get("MemFree", 0))
    return total - avail, total


def node_memory() -> Tuple[int, int]:
    """(used_bytes, total_bytes) for this node / container."""
    used, total = _meminfo()
    cur, lim = _read_int("/sys/fs/cgroup/memory.current"), _read_int("/sys/fs/cgroup/memory.max")
    if cur is None:
        cur = _read_int("/sys/fs/cgroup/memory/memory.usage_in_bytes")
        lim = _read_int("/sys/fs/cgroup/memory/memory.limit_in_bytes")
    if cur is not None and lim is not None and 0 < lim < total:
        return cur, lim
    return used, total


def _env(names, default):
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            return float(v)
    return default


class MemoryMonitor:
    def __init__(self, threshold: Optional[float] = None, refresh_ms: Optional[float] = None):
        self.threshold = threshold if threshold is not None else _env(
            ("CAAMD_MEMORY_USAGE_THRESHOLD", "RAY_memory_usage_threshold"), 0.95)
        ms = refresh_ms if refresh_ms is not None else _env(
            ("CAAMD_MEMORY_MONITOR_REFRESH_MS", "RAY_memory_monitor_refresh_ms"), 250.0)
        self.refresh_s = ms / 1000.0
        self.enabled = ms > 0
        self.test_file = os.environ.get("CAAMD_MEMORY_MONITOR_TEST_FILE")
        self.kills = 0

    def usage_fraction(self) -> Optional[float]:
        if self.test_file:
            try:
                with open(self.test_file) as f:
                    return float(f.read().strip() or 0.0)
            except (OSError, ValueError):
                return 0.0
        try:
            used, total = node_memory()
        except OSError:
            return None
        return used / total if total else None

    def over_threshold(self) -> Optional[float]:
        f = self.usage_fraction()
        if f is not None and f >= self.threshold:
            return f
        return None


def pick_victim(candidates):
    """``candidates``: iterable of (worker, retriable: bool, start_time: float).
    Retriable before non-retriable; newest first within a class."""
    best, key = None, None
    for w, retriable, start in candidates:
        k = (0 if retriable else 1, -(start or 0.0))
        if key is None or k < key:
            best, key = w, k
    return best
