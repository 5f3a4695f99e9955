"""Stoppers (reference: python/ray/tune/stopper/)."""
from __future__ import annotations

import collections
import time
from typing import Callable, Dict, Optional


class Stopper:
    def __call__(self, trial_id: str, result: Dict) -> bool:
        return False

    def stop_all(self) -> bool:
        return False


class MaximumIterationStopper(Stopper):
    def __init__(self, max_iter: int):
        self.max_iter = max_iter

    def __call__(self, trial_id, result):
        return result.get("training_iteration", 0) >= self.max_iter


class TimeoutStopper(Stopper):
    def __init__(self, timeout):
        self.timeout = timeout.total_seconds() if hasattr(timeout, "total_seconds") else float(timeout)
        self.start = time.time()

    def stop_all(self):
        return time.time() - self.start > self.timeout


class FunctionStopper(Stopper):
    def __init__(self, fn: Callable[[str, Dict], bool]):
        self.fn = fn

    def __call__(self, trial_id, result):
        return bool(self.fn(trial_id, result))


class TrialPlateauStopper(Stopper):
    def __init__(self, metric: str, std: float = 0.01, num_results: int = 4, grace_period: int = 4,
                 metric_threshold: Optional[float] = None, mode: Optional[str] = None):
        self.metric, self.std, self.n, self.grace = metric, std, num_results, grace_period
        self.hist = collections.defaultdict(lambda: collections.deque(maxlen=num_results))
        self.count = collections.Counter()

    def __call__(self, trial_id, result):
        v = result.get(self.metric)
        if v is None:
            return False
        self.count[trial_id] += 1
        h = self.hist[trial_id]
        h.append(v)
        if self.count[trial_id] < self.grace or len(h) < self.n:
            return False
        mean = sum(h) / len(h)
        sd = (sum((x - mean) ** 2 for x in h) / len(h)) ** 0.5
        return sd <= self.std


class ExperimentPlateauStopper(Stopper):
    def __init__(self, metric: str, std: float = 0.001, top: int = 10, mode: str = "min", patience: int = 0):
        self.metric, self.std, self.top, self.mode, self.patience = metric, std, top, mode, patience
        self.values = []
        self.iters = 0

    def __call__(self, trial_id, result):
        v = result.get(self.metric)
        if v is not None:
            self.values.append(v)
        return False

    def stop_all(self):
        if len(self.values) < self.top:
            return False
        best = sorted(self.values, reverse=self.mode == "max")[: self.top]
        m = sum(best) / len(best)
        sd = (sum((x - m) ** 2 for x in best) / len(best)) ** 0.5
        if sd <= self.std:
            self.iters += 1
        else:
            self.iters = 0
        return self.iters > self.patience


class CombinedStopper(Stopper):
    def __init__(self, *stoppers: Stopper):
        self.stoppers = stoppers

    def __call__(self, trial_id, result):
        return any(s(trial_id, result) for s in self.stoppers)

    def stop_all(self):
        return any(s.stop_all() for s in self.stoppers)


class _DictStopper(Stopper):
    def __init__(self, crit: Dict):
        self.crit = crit

    def __call__(self, trial_id, result):
        return any(k in result and result[k] >= v for k, v in self.crit.items())


def make_stopper(stop) -> Optional[Stopper]:
    if stop is None:
        return None
    if isinstance(stop, Stopper):
        return stop
    if isinstance(stop, dict):
        return _DictStopper(stop)
    if callable(stop):
        return FunctionStopper(stop)
    raise ValueError(f"invalid stop criteria {stop!r}")
