"""Trial schedulers (reference: python/ray/tune/schedulers/: trial_scheduler.py,
async_hyperband.py:19 (ASHA), hyperband.py, median_stopping_rule.py,
pbt.py:221 (PopulationBasedTraining))."""
from __future__ import annotations

import collections
import copy
import math
import random
from typing import Any, Callable, Dict, List, Optional


class TrialScheduler:
    CONTINUE = "CONTINUE"
    PAUSE = "PAUSE"
    STOP = "STOP"
    NOOP = "NOOP"

    def __init__(self, metric: Optional[str] = None, mode: Optional[str] = None):
        self.metric, self.mode = metric, mode

    def set_search_properties(self, metric, mode, **spec):
        self.metric = self.metric or metric
        self.mode = self.mode or mode
        return True

    def _score(self, result):
        v = result.get(self.metric)
        if v is None:
            return None
        return v if self.mode == "max" else -v

    def on_trial_add(self, trial):
        pass

    def on_trial_result(self, trial, result) -> str:
        return self.CONTINUE

    def on_trial_complete(self, trial, result):
        pass

    def on_trial_error(self, trial):
        pass


class FIFOScheduler(TrialScheduler):
    pass


class AsyncHyperBandScheduler(TrialScheduler):
    """ASHA: a trial reaching rung r (grace_period * rf^k of time_attr) continues
    only if it is in the top 1/rf of all results recorded at that rung."""

    def __init__(self, time_attr: str = "training_iteration", metric=None, mode=None,
                 max_t: int = 100, grace_period: int = 1, reduction_factor: float = 4,
                 brackets: int = 1, stop_last_trials: bool = True):
        super().__init__(metric, mode)
        self.time_attr, self.max_t, self.grace, self.rf = time_attr, max_t, grace_period, reduction_factor
        self.rungs = []
        r = grace_period
        while r < max_t:
            self.rungs.append(r)
            r = int(math.ceil(r * reduction_factor))
        self.recorded = collections.defaultdict(dict)  # rung -> {trial_id: score}

    def on_trial_result(self, trial, result):
        t = result.get(self.time_attr, 0)
        if t >= self.max_t:
            return self.STOP
        s = self._score(result)
        if s is None:
            return self.CONTINUE
        for rung in reversed(self.rungs):
            if t >= rung and trial.trial_id not in self.recorded[rung]:
                self.recorded[rung][trial.trial_id] = s
                scores = sorted(self.recorded[rung].values(), reverse=True)
                k = max(1, int(len(scores) / self.rf))
                cutoff = scores[k - 1] if len(scores) >= self.rf else None
                if cutoff is not None and s < cutoff:
                    return self.STOP
                break
        return self.CONTINUE


ASHAScheduler = AsyncHyperBandScheduler


class HyperBandScheduler(AsyncHyperBandScheduler):
    """Synchronous HyperBand approximated by its asynchronous successive-halving
    form (the reference's HyperBandScheduler pauses whole brackets; ASHA has the
    same promotion rule without the synchronisation barrier)."""

    def __init__(self, time_attr="training_iteration", metric=None, mode=None, max_t=81,
                 reduction_factor=3, stop_last_trials=True):
        super().__init__(time_attr, metric, mode, max_t, 1, reduction_factor)


class MedianStoppingRule(TrialScheduler):
    def __init__(self, time_attr: str = "time_total_s", metric=None, mode=None,
                 grace_period: float = 60.0, min_samples_required: int = 3,
                 min_time_slice: int = 0, hard_stop: bool = True):
        super().__init__(metric, mode)
        self.time_attr, self.grace, self.min_samples = time_attr, grace_period, min_samples_required
        self.hist = collections.defaultdict(list)  # trial -> [(t, score)]
        self.completed = {}

    def _running_mean(self, tid, t):
        xs = [s for (tt, s) in self.hist[tid] if tt <= t]
        return sum(xs) / len(xs) if xs else None

    def on_trial_result(self, trial, result):
        t = result.get(self.time_attr, 0)
        s = self._score(result)
        if s is None:
            return self.CONTINUE
        self.hist[trial.trial_id].append((t, s))
        if t < self.grace:
            return self.CONTINUE
        others = [self._running_mean(o, t) for o in self.hist if o != trial.trial_id]
        others = [o for o in others if o is not None]
        if len(others) < self.min_samples:
            return self.CONTINUE
        med = sorted(others)[len(others) // 2]
        best = max(s2 for _, s2 in self.hist[trial.trial_id])
        return self.STOP if best < med else self.CONTINUE


class PopulationBasedTraining(TrialScheduler):
    """Every ``perturbation_interval`` a trial in the bottom quantile clones the
    checkpoint + config of a top-quantile trial and perturbs the config
    (resample with ``resample_probability``, else multiply by 0.8 / 1.2)."""

    def __init__(self, time_attr: str = "training_iteration", metric=None, mode=None,
                 perturbation_interval: float = 60.0, burn_in_period: float = 0,
                 hyperparam_mutations: Optional[Dict] = None, quantile_fraction: float = 0.25,
                 resample_probability: float = 0.25, perturbation_factors=(1.2, 0.8),
                 custom_explore_fn: Optional[Callable] = None, seed=None, synch: bool = False):
        super().__init__(metric, mode)
        self.time_attr, self.interval, self.burn = time_attr, perturbation_interval, burn_in_period
        self.mutations = hyperparam_mutations or {}
        self.q, self.resample_p, self.factors = quantile_fraction, resample_probability, perturbation_factors
        self.explore_fn = custom_explore_fn
        self.rng = random.Random(seed)
        self.last_perturb = {}
        self.latest = {}  # trial_id -> (score, trial)
        self.num_perturbations = 0

    def _explore(self, config):
        new = copy.deepcopy(config)
        for k, spec in self.mutations.items():
            if isinstance(spec, dict):
                continue
            if self.rng.random() < self.resample_p or k not in new:
                if isinstance(spec, list):
                    new[k] = self.rng.choice(spec)
                elif callable(spec):
                    new[k] = spec()
                elif hasattr(spec, "sample"):
                    new[k] = spec.sample(None, self.rng)
            else:
                if isinstance(spec, list) and new[k] in spec:
                    i = spec.index(new[k]) + self.rng.choice([-1, 1])
                    new[k] = spec[max(0, min(len(spec) - 1, i))]
                elif isinstance(new[k], (int, float)):
                    f = self.rng.choice(self.factors)
                    new[k] = type(new[k])(new[k] * f)
        if self.explore_fn:
            new = self.explore_fn(new)
        return new

    def on_trial_result(self, trial, result):
        t = result.get(self.time_attr, 0)
        s = self._score(result)
        if s is None:
            return self.CONTINUE
        self.latest[trial.trial_id] = (s, trial)
        if t < self.burn or t - self.last_perturb.get(trial.trial_id, 0) < self.interval:
            return self.CONTINUE
        self.last_perturb[trial.trial_id] = t
        ranked = sorted(self.latest.values(), key=lambda x: x[0])
        n = len(ranked)
        k = max(1, int(math.ceil(n * self.q)))
        if n < 2:
            return self.CONTINUE
        bottom = [x[1].trial_id for x in ranked[:k]]
        top = [x[1] for x in ranked[-k:]]
        if trial.trial_id in bottom and trial not in top:
            donor = self.rng.choice(top)
            if donor.latest_checkpoint is not None:
                trial.pending_exploit = (donor.latest_checkpoint, self._explore(donor.config))
                self.num_perturbations += 1
                return self.PAUSE
        return self.CONTINUE


__all__ = ["TrialScheduler", "FIFOScheduler", "AsyncHyperBandScheduler", "ASHAScheduler",
           "HyperBandScheduler", "MedianStoppingRule", "PopulationBasedTraining"]
