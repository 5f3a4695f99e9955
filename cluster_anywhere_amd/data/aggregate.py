"""Aggregations (reference: python/ray/data/aggregate.py)."""
from __future__ import annotations

import math
from typing import Any, Callable, Optional

import numpy as np


class AggregateFn:
    def __init__(self, init: Callable, accumulate_block: Callable, merge: Callable,
                 finalize: Optional[Callable] = None, name: Optional[str] = None):
        self.init = init
        self.accumulate_block = accumulate_block
        self.merge = merge
        self.finalize = finalize or (lambda a: a)
        self.name = name


def _col(on):
    return on


class Count(AggregateFn):
    def __init__(self, on: Optional[str] = None, alias_name: Optional[str] = None, ignore_nulls=True):
        super().__init__(lambda k: 0, lambda a, b: a + (len(next(iter(b.values()))) if b else 0),
                         lambda a, b: a + b, name=alias_name or "count()")


class Sum(AggregateFn):
    def __init__(self, on: str, alias_name: Optional[str] = None, ignore_nulls=True):
        super().__init__(lambda k: 0, lambda a, b: a + (b[on].sum() if len(b[on]) else 0),
                         lambda a, b: a + b, name=alias_name or f"sum({on})")


class Min(AggregateFn):
    def __init__(self, on: str, alias_name: Optional[str] = None, ignore_nulls=True):
        super().__init__(lambda k: math.inf, lambda a, b: min(a, b[on].min()) if len(b[on]) else a,
                         min, name=alias_name or f"min({on})")


class Max(AggregateFn):
    def __init__(self, on: str, alias_name: Optional[str] = None, ignore_nulls=True):
        super().__init__(lambda k: -math.inf, lambda a, b: max(a, b[on].max()) if len(b[on]) else a,
                         max, name=alias_name or f"max({on})")


class Mean(AggregateFn):
    def __init__(self, on: str, alias_name: Optional[str] = None, ignore_nulls=True):
        super().__init__(lambda k: (0.0, 0), lambda a, b: (a[0] + float(b[on].sum()), a[1] + len(b[on])),
                         lambda a, b: (a[0] + b[0], a[1] + b[1]),
                         lambda a: a[0] / a[1] if a[1] else None, name=alias_name or f"mean({on})")


class Std(AggregateFn):
    """Chan et al. parallel variance (count, mean, M2)."""

    def __init__(self, on: str, ddof: int = 1, alias_name: Optional[str] = None, ignore_nulls=True):
        def acc(a, b):
            x = b[on].astype(np.float64)
            if not len(x):
                return a
            return _merge(a, (len(x), float(x.mean()), float(((x - x.mean()) ** 2).sum())))

        def _merge(a, b):
            n1, m1, s1 = a
            n2, m2, s2 = b
            if n1 == 0:
                return b
            if n2 == 0:
                return a
            n = n1 + n2
            d = m2 - m1
            return (n, m1 + d * n2 / n, s1 + s2 + d * d * n1 * n2 / n)

        super().__init__(lambda k: (0, 0.0, 0.0), acc, _merge,
                         lambda a: math.sqrt(a[2] / (a[0] - ddof)) if a[0] > ddof else None,
                         name=alias_name or f"std({on})")


class AbsMax(AggregateFn):
    def __init__(self, on: str, alias_name: Optional[str] = None, ignore_nulls=True):
        super().__init__(lambda k: 0, lambda a, b: max(a, np.abs(b[on]).max()) if len(b[on]) else a,
                         max, name=alias_name or f"abs_max({on})")
