"""MetricsLogger (reference role: rllib/utils/metrics/metrics_logger.py).

Components (env runners, learners, callbacks) log scalar values under (possibly
nested) keys with a reduction; ``reduce()`` returns a plain nested dict and
resets the window for keys logged with ``clear_on_reduce``. Results from
several loggers (one per env runner) are combined with ``merge_reduced``:
means are averaged weighted by sample count, sums are added, min/max taken.
"""
from __future__ import annotations

from collections import deque
from typing import Any, Dict, Iterable, List, Optional, Tuple, Union

import numpy as np

Key = Union[str, Tuple[str, ...]]


def _path(key: Key) -> Tuple[str, ...]:
    return tuple(key) if isinstance(key, (tuple, list)) else (key,)


class _Stat:
    __slots__ = ("reduce", "window", "values", "clear", "count")

    def __init__(self, reduce: str, window: Optional[int], clear: bool):
        if reduce not in ("mean", "sum", "min", "max", None):
            raise ValueError(f"unknown reduce {reduce!r}")
        self.reduce = reduce
        self.window = window
        self.clear = clear
        self.values: deque = deque(maxlen=window if reduce != "sum" or window else None)
        self.count = 0

    def push(self, v):
        if self.reduce == "sum" and not self.window and self.values:
            self.values[0] = self.values[0] + v  # running sum, O(1) memory
        else:
            self.values.append(v)
        self.count += 1

    def value(self):
        if not self.values:
            return float("nan")
        if self.reduce is None:
            return list(self.values)
        a = np.asarray(list(self.values), dtype=np.float64)
        return float({"mean": np.mean, "sum": np.sum, "min": np.min, "max": np.max}[self.reduce](a))


class MetricsLogger:
    def __init__(self):
        self._stats: Dict[Tuple[str, ...], _Stat] = {}

    def log_value(self, key: Key, value: Any, reduce: Optional[str] = "mean", window: Optional[int] = None,
                  clear_on_reduce: bool = False):
        p = _path(key)
        s = self._stats.get(p)
        if s is None:
            s = self._stats[p] = _Stat(reduce, window, clear_on_reduce)
        s.push(float(value) if isinstance(value, (int, float, np.floating, np.integer)) else value)

    def log_dict(self, d: Dict[str, Any], *, key: Optional[Key] = None, reduce: Optional[str] = "mean",
                 window: Optional[int] = None, clear_on_reduce: bool = False):
        base = _path(key) if key is not None else ()
        for k, v in d.items():
            if isinstance(v, dict):
                self.log_dict(v, key=base + (k,), reduce=reduce, window=window, clear_on_reduce=clear_on_reduce)
            else:
                self.log_value(base + (k,), v, reduce, window, clear_on_reduce)

    def peek(self, key: Key, default=None):
        s = self._stats.get(_path(key))
        return default if s is None else s.value()

    def __contains__(self, key: Key) -> bool:
        return _path(key) in self._stats

    def reset(self):
        self._stats.clear()

    def reduce(self) -> Dict[str, Any]:
        """Nested dict of reduced values; ``__count`` keeps sample counts for merging."""
        out: Dict[str, Any] = {}
        for p, s in list(self._stats.items()):
            d = out
            for k in p[:-1]:
                d = d.setdefault(k, {})
            d[p[-1]] = s.value()
            d.setdefault("__meta", {})[p[-1]] = (s.reduce, s.count)
            if s.clear:
                del self._stats[p]
        return out


def merge_reduced(results: Iterable[Dict[str, Any]]) -> Dict[str, Any]:
    """Combine ``MetricsLogger.reduce()`` outputs of several components."""
    results = [r for r in results if r]
    if not results:
        return {}
    out: Dict[str, Any] = {}
    keys: List[str] = []
    for r in results:
        keys += [k for k in r if k != "__meta" and k not in keys]
    for k in keys:
        vals = [(r[k], r.get("__meta", {}).get(k, ("mean", 1))) for r in results if k in r]
        if isinstance(vals[0][0], dict):
            out[k] = merge_reduced([v for v, _ in vals])
            continue
        red = vals[0][1][0]
        xs = [(v, m[1]) for v, m in vals if not (isinstance(v, float) and np.isnan(v))]
        if not xs:
            out[k] = float("nan")
        elif red == "sum":
            out[k] = float(sum(v for v, _ in xs))
        elif red == "min":
            out[k] = float(min(v for v, _ in xs))
        elif red == "max":
            out[k] = float(max(v for v, _ in xs))
        elif red is None:
            out[k] = [x for v, _ in xs for x in v]
        else:
            w = sum(c for _, c in xs)
            out[k] = float(sum(v * c for v, c in xs) / max(w, 1))
    return out


def strip_meta(d: Dict[str, Any]) -> Dict[str, Any]:
    return {k: strip_meta(v) if isinstance(v, dict) else v for k, v in d.items() if k != "__meta"}
