"""Progress bars usable inside tasks and actors (reference:
experimental/tqdm_ray.py). Workers' stderr is forwarded to the driver, so each
bar emits a throttled single-line state record that the driver prints; in the
driver itself it renders in place."""
from __future__ import annotations

import json
import os
import sys
import time
import uuid
from typing import Iterable, Optional

_PREFIX = "__caamd_tqdm__"


class tqdm:
    def __init__(self, iterable: Optional[Iterable] = None, desc: Optional[str] = None,
                 total: Optional[int] = None, position: Optional[int] = None, flush_interval_s: float = 1.0,
                 unit: str = "it", **_kw):
        self._iterable = iterable
        if total is None and iterable is not None:
            try:
                total = len(iterable)  # type: ignore[arg-type]
            except TypeError:
                total = None
        self.total, self.desc, self.unit = total, desc or "", unit
        self.n = 0
        self.position = position
        self._uuid = uuid.uuid4().hex[:12]
        self._interval = flush_interval_s
        self._last = 0.0
        self._start = time.time()
        self._closed = False

    def __iter__(self):
        for x in self._iterable or ():
            yield x
            self.update(1)
        self.close()

    def update(self, n: int = 1) -> None:
        self.n += n
        now = time.time()
        if now - self._last >= self._interval:
            self._emit(False)
            self._last = now

    def set_description(self, desc: str) -> None:
        self.desc = desc

    def refresh(self) -> None:
        self._emit(False)

    def close(self) -> None:
        if not self._closed:
            self._closed = True
            self._emit(True)

    def _emit(self, closed: bool):
        rate = self.n / max(time.time() - self._start, 1e-9)
        rec = {"uuid": self._uuid, "desc": self.desc, "x": self.n, "total": self.total,
               "pid": os.getpid(), "closed": closed, "rate": round(rate, 2), "unit": self.unit}
        from ..core import context

        w = context.worker
        if w is not None and getattr(w, "kind", "driver") == "worker":
            print(_PREFIX + json.dumps(rec), file=sys.stderr, flush=True)
        else:
            tot = f"/{self.total}" if self.total is not None else ""
            end = "\n" if closed else "\r"
            print(f"{self.desc}: {self.n}{tot} [{rate:.1f}{self.unit}/s]", end=end, file=sys.stderr, flush=True)


def safe_print(*args, **kwargs):
    print(*args, **kwargs)
