"""Application metrics: Counter / Gauge / Histogram (reference:
python/ray/util/metrics.py). Records are sent fire-and-forget to the head,
aggregated per (name, tags) and exported in Prometheus text format by the
dashboard's ``/metrics`` endpoint (``dashboard.render_prometheus``)."""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple


class Metric:
    kind = "gauge"

    def __init__(self, name: str, description: str = "", tag_keys: Optional[Sequence[str]] = None):
        if not name or not all(ch.isalnum() or ch in "_:" for ch in name):
            raise ValueError(f"invalid metric name {name!r}")
        self._name = name
        self._description = description
        self._tag_keys: Tuple[str, ...] = tuple(tag_keys or ())
        self._default_tags: Dict[str, str] = {}

    @property
    def info(self):
        return {"name": self._name, "description": self._description, "tag_keys": self._tag_keys,
                "default_tags": dict(self._default_tags)}

    def set_default_tags(self, tags: Dict[str, str]):
        for k in tags:
            if k not in self._tag_keys:
                raise ValueError(f"unknown tag key {k!r}")
        self._default_tags = dict(tags)
        return self

    def _tags(self, tags: Optional[Dict[str, str]]):
        t = dict(self._default_tags)
        t.update(tags or {})
        missing = [k for k in self._tag_keys if k not in t]
        if missing:
            raise ValueError(f"missing tag values for {missing}")
        extra = [k for k in t if k not in self._tag_keys]
        if extra:
            raise ValueError(f"unknown tag keys {extra}")
        return tuple(str(t[k]) for k in self._tag_keys)

    def _record(self, value: float, tags, boundaries=None):
        from ..core import context

        w = context.worker
        if w is None:
            return
        try:
            w.send(("metric", self._name, self.kind, self._description, self._tag_keys, self._tags(tags),
                    float(value), boundaries))
        except Exception:
            pass


class Counter(Metric):
    kind = "counter"

    def inc(self, value: float = 1.0, tags: Optional[Dict[str, str]] = None):
        if value < 0:
            raise ValueError("Counter.inc() needs a non-negative value")
        self._record(value, tags)


class Gauge(Metric):
    kind = "gauge"

    def set(self, value: float, tags: Optional[Dict[str, str]] = None):
        self._record(value, tags)


class Histogram(Metric):
    kind = "histogram"

    def __init__(self, name: str, description: str = "", boundaries: Optional[List[float]] = None,
                 tag_keys: Optional[Sequence[str]] = None):
        super().__init__(name, description, tag_keys)
        if not boundaries or any(b <= 0 for b in boundaries) or sorted(boundaries) != list(boundaries):
            raise ValueError("Histogram needs increasing positive boundaries")
        self.boundaries = list(boundaries)

    def observe(self, value: float, tags: Optional[Dict[str, str]] = None):
        self._record(value, tags, self.boundaries)
