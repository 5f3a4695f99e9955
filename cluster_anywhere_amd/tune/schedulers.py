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

    # -- which waiting trial runs next (synchronous schedulers gate resumption) --
    def choose_trial_to_run(self, candidates):
        """Among PENDING / PAUSED trials without an actor, the one to launch next (None:
        keep waiting). Reference: trial_scheduler.py ``choose_trial_to_run``."""
        return candidates[0] if candidates else None

    def pop_stopped_trials(self) -> List[str]:
        """Trial ids of PAUSED trials the scheduler has decided to terminate."""
        return []


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


class _Bracket:
    """One HyperBand bracket: n trials, first milestone r, successive halving by eta."""

    def __init__(self, s: int, n: int, r: float, eta: float, max_t: int):
        self.s, self.n, self.eta, self.max_t = s, n, eta, max_t
        self.milestone = min(max_t, max(1, int(round(r))))
        self.trials: List[str] = []          # members still alive in this bracket
        self.scores: Dict[str, float] = {}   # trial -> score at the current milestone
        self.promoted = set()                # may resume past the current milestone
        self.stopped = set()

    def full(self):
        return len(self.trials) + len(self.stopped) >= self.n


class HyperBandScheduler(TrialScheduler):
    """Synchronous HyperBand (reference: python/ray/tune/schedulers/hyperband.py:42;
    Li et al. 2018). Trials are dealt into brackets s = s_max..0 of
    n_s = ceil((s_max+1)/(s+1) * eta^s) trials whose first milestone is
    max_t * eta^-s. A trial PAUSES when it reaches its bracket's milestone; once every
    live member of the bracket is there, the top 1/eta are promoted (milestone x eta,
    resumed from their checkpoints) and the rest are stopped."""

    def __init__(self, time_attr: str = "training_iteration", metric=None, mode=None,
                 max_t: int = 81, reduction_factor: float = 3, stop_last_trials: bool = True):
        super().__init__(metric, mode)
        self.time_attr, self.max_t, self.eta = time_attr, max_t, reduction_factor
        self.s_max = int(math.floor(math.log(max_t) / math.log(reduction_factor) + 1e-9))
        self.brackets: List[_Bracket] = []
        self.of: Dict[str, _Bracket] = {}
        self._next_s = self.s_max
        self._to_stop: List[str] = []
        self._at_milestone = set()

    def _new_bracket(self):
        s = self._next_s
        self._next_s = self._next_s - 1 if self._next_s > 0 else self.s_max
        n = int(math.ceil((self.s_max + 1) / (s + 1) * self.eta ** s))
        b = _Bracket(s, n, self.max_t * self.eta ** (-s), self.eta, self.max_t)
        self.brackets.append(b)
        return b

    def on_trial_add(self, trial):
        b = self.brackets[-1] if self.brackets and not self.brackets[-1].full() else self._new_bracket()
        b.trials.append(trial.trial_id)
        self.of[trial.trial_id] = b

    def on_trial_result(self, trial, result):
        b = self.of.get(trial.trial_id)
        t = result.get(self.time_attr, 0)
        if t >= self.max_t:
            return self.STOP
        if b is None:
            return self.CONTINUE
        s = self._score(result)
        if t < b.milestone or s is None:
            return self.CONTINUE
        b.scores[trial.trial_id] = s
        self._at_milestone.add(trial.trial_id)
        b.promoted.discard(trial.trial_id)
        decision = self._maybe_cut(b)
        if trial.trial_id in self._to_stop:
            self._to_stop.remove(trial.trial_id)
            return self.STOP
        return decision if decision is not None else self.PAUSE

    def _maybe_cut(self, b: _Bracket):
        live = [tid for tid in b.trials if tid not in b.stopped]
        if not b.full() or any(tid not in b.scores for tid in live):
            return None  # wait for the whole bracket to reach the milestone
        ranked = sorted(live, key=lambda tid: b.scores[tid], reverse=True)
        keep = max(1, int(len(ranked) / b.eta))
        for tid in ranked[keep:]:
            b.stopped.add(tid)
            self._to_stop.append(tid)
        b.milestone = min(self.max_t, int(math.ceil(b.milestone * b.eta)))
        b.scores = {}
        for tid in ranked[:keep]:
            b.promoted.add(tid)
            self._at_milestone.discard(tid)
        return None

    def on_trial_complete(self, trial, result):
        b = self.of.get(trial.trial_id)
        if b is not None and trial.trial_id in b.trials:
            b.trials.remove(trial.trial_id)
            b.scores.pop(trial.trial_id, None)
            self._maybe_cut(b)

    on_trial_error = lambda self, trial: self.on_trial_complete(trial, None)  # noqa: E731

    def choose_trial_to_run(self, candidates):
        for t in candidates:
            if getattr(t, "status", None) == "PENDING" and t.trial_id not in self._at_milestone:
                return t
        for t in candidates:
            b = self.of.get(t.trial_id)
            if b is not None and t.trial_id in b.promoted:
                return t
        return None

    def pop_stopped_trials(self):
        out, self._to_stop = self._to_stop, []
        return out


class HyperBandForBOHB(HyperBandScheduler):
    """HyperBand whose successive-halving decisions feed the BOHB searcher
    (reference: python/ray/tune/schedulers/hb_bohb.py:16): every milestone result
    is reported to ``TuneBOHB`` so its density models are trained per budget."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.searcher = None

    def on_trial_result(self, trial, result):
        d = super().on_trial_result(trial, result)
        if self.searcher is not None and d in (self.PAUSE, self.STOP) and hasattr(self.searcher, "on_budget_result"):
            b = self.of.get(trial.trial_id)
            self.searcher.on_budget_result(trial.trial_id, result, b.milestone if b else None)
        return d


class ResourceChangingScheduler(TrialScheduler):
    """Wraps a scheduler and re-sizes running trials (reference:
    python/ray/tune/schedulers/resource_changing_scheduler.py:592). After each
    result the allocation function proposes resources for the trial; if they
    differ, the trial is paused and relaunched from its latest checkpoint with the
    new resources (a Trainable sees them via ``tune.get_trial_resources()``)."""

    def __init__(self, base_scheduler: Optional[TrialScheduler] = None,
                 resources_allocation_function: Optional[Callable] = None):
        super().__init__()
        self.base = base_scheduler or FIFOScheduler()
        self.alloc = resources_allocation_function or DistributeResources()
        self.controller = None

    def set_search_properties(self, metric, mode, **spec):
        super().set_search_properties(metric, mode, **spec)
        return self.base.set_search_properties(metric, mode, **spec)

    def on_trial_add(self, trial):
        self.base.on_trial_add(trial)

    def on_trial_result(self, trial, result):
        d = self.base.on_trial_result(trial, result)
        if d != self.CONTINUE:
            return d
        new = self.alloc(self.controller, trial, result, self)
        if new and dict(new) != dict(trial.resources) and trial.latest_checkpoint is not None:
            trial.resources = dict(new)
            return self.PAUSE
        return d

    def on_trial_complete(self, trial, result):
        self.base.on_trial_complete(trial, result)

    def on_trial_error(self, trial):
        self.base.on_trial_error(trial)

    def choose_trial_to_run(self, candidates):
        return self.base.choose_trial_to_run(candidates)

    def pop_stopped_trials(self):
        return self.base.pop_stopped_trials()


class DistributeResources:
    """Default allocation: spread the cluster's CPUs (and GPUs) evenly over the
    running trials, never below the trial's base request."""

    def __init__(self, add_bundles: bool = False, increase_by: Optional[Dict] = None,
                 increase_by_times: int = -1, reserve_resources: Optional[Dict] = None):
        self.reserve = reserve_resources or {}

    def __call__(self, controller, trial, result, scheduler):
        from ..core import api as core

        if controller is None:
            return None
        running = [t for t in controller.trials if t.status == "RUNNING"] or [trial]
        total = core.cluster_resources()
        out = dict(trial.resources)
        base = getattr(trial, "base_resources", None) or dict(trial.resources)
        trial.base_resources = base
        for key in ("CPU", "GPU"):
            avail = float(total.get(key, 0)) - float(self.reserve.get(key, 0))
            if avail <= 0 or key not in base:
                continue
            share = max(float(base[key]), math.floor(avail / len(running)))
            out[key] = share
        return out


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
                 custom_explore_fn: Optional[Callable] = None, seed=None, synch: bool = False,
                 log_config: bool = True):
        super().__init__(metric, mode)
        self.log_config = log_config
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
                new_cfg = self._explore(donor.config)
                if self.log_config:
                    self._log_policy(trial, donor, t, new_cfg)
                trial.pending_exploit = (donor.latest_checkpoint, new_cfg)
                self.num_perturbations += 1
                return self.PAUSE
        return self.CONTINUE

    def _log_policy(self, trial, donor, step, new_cfg):
        """``<experiment>/pbt_policy_<trial_id>.txt``: the donor's schedule, then one
        JSON row [donor_id, trial_id, donor_step, step, donor_config, new_config]
        -- the file :class:`PopulationBasedTrainingReplay` replays."""
        import json
        import os

        exp = os.path.dirname(trial.local_path)
        src = os.path.join(exp, f"pbt_policy_{donor.trial_id}.txt")
        prior = open(src).read() if os.path.exists(src) else ""
        row = [donor.trial_id, trial.trial_id, donor.last_result.get(self.time_attr, 0), step,
               _jsonable(donor.config), _jsonable(new_cfg)]
        os.makedirs(exp, exist_ok=True)
        with open(os.path.join(exp, f"pbt_policy_{trial.trial_id}.txt"), "w") as f:
            f.write(prior + json.dumps(row) + "\n")


def _jsonable(cfg):
    import json

    out = {}
    for k, v in cfg.items():
        try:
            json.dumps(v)
            out[k] = v
        except TypeError:
            out[k] = repr(v)
    return out


class PopulationBasedTrainingReplay(TrialScheduler):
    """Replay the hyperparameter schedule one PBT trial ended up with (reference
    role: pbt.py:1012): reads ``pbt_policy_<trial_id>.txt`` (written by PBT with
    ``log_config=True``), starts the single trial with the schedule's initial
    config and, when the trial reaches each recorded step, restarts it from its
    own latest checkpoint with the next config."""

    def __init__(self, policy_file: str):
        import json
        import os

        path = os.path.expanduser(policy_file)
        if not os.path.exists(path):
            raise ValueError(f"Policy file not found: {path}")
        rows = []
        with open(path) as f:
            for ln in f:
                if ln.strip():
                    try:
                        rows.append(json.loads(ln))
                    except json.JSONDecodeError:
                        raise ValueError(f"Could not read PBT policy file: {path}") from None
        # walk back from the last change while the chain of trial ids is unbroken
        schedule, expect, initial = [], None, None
        for old_tag, new_tag, _old_step, new_step, old_conf, new_conf in reversed(rows):
            if expect is not None and new_tag != expect:
                break
            expect = old_tag
            initial = old_conf
            schedule.append((new_step, new_conf))
        super().__init__()
        self.policy_file = path
        self.config = initial
        self.schedule = list(reversed(schedule))
        self._trial = None
        self.num_perturbations = 0
        self.time_attr = "training_iteration"

    def on_trial_add(self, trial):
        if self._trial is not None:
            raise ValueError("PopulationBasedTrainingReplay trains one trial (num_samples=1)")
        self._trial = trial
        if self.config is not None:
            trial.config = dict(trial.config or {}, **self.config)
        elif not trial.config:
            raise ValueError("the replay policy is empty and the trial has no config")

    def on_trial_result(self, trial, result):
        if not self.schedule:
            return self.CONTINUE
        step, cfg = self.schedule[0]
        if result.get(self.time_attr, 0) < step or trial.latest_checkpoint is None:
            return self.CONTINUE
        self.schedule.pop(0)
        trial.pending_exploit = (trial.latest_checkpoint, dict(trial.config, **cfg))
        self.num_perturbations += 1
        return self.PAUSE


class PB2(PopulationBasedTraining):
    """Population Based Bandits (reference: python/ray/tune/schedulers/pb2.py:256;
    Parker-Holder et al. 2020): PBT's exploit step, but the explore step picks the
    new hyperparameters with a GP-UCB bandit fitted on (time, hyperparameters) ->
    reward change observed across the population, inside ``hyperparam_bounds``."""

    def __init__(self, time_attr: str = "training_iteration", metric=None, mode=None,
                 perturbation_interval: float = 60.0, hyperparam_bounds: Optional[Dict] = None,
                 quantile_fraction: float = 0.25, log_config: bool = True, seed=None,
                 custom_explore_fn: Optional[Callable] = None, synch: bool = False):
        self.bounds = dict(hyperparam_bounds or {})
        if not self.bounds:
            raise ValueError("PB2 needs hyperparam_bounds={name: [low, high]}")
        super().__init__(time_attr, metric, mode, perturbation_interval,
                         hyperparam_mutations={k: list(v) for k, v in self.bounds.items()},
                         quantile_fraction=quantile_fraction, custom_explore_fn=custom_explore_fn,
                         seed=seed, synch=synch)
        self.data: List[tuple] = []  # (t, x-normalised..., reward delta)
        self._last = {}              # trial_id -> (t, score)
        self._np_rng = None

    def _norm(self, cfg):
        out = []
        for k, (lo, hi) in self.bounds.items():
            v = float(cfg.get(k, lo))
            out.append((v - lo) / (hi - lo) if hi > lo else 0.0)
        return out

    def on_trial_result(self, trial, result):
        t = result.get(self.time_attr, 0)
        s = self._score(result)
        if s is not None:
            prev = self._last.get(trial.trial_id)
            if prev is not None and t > prev[0]:
                self.data.append((t, *self._norm(trial.config), (s - prev[1]) / (t - prev[0])))
            self._last[trial.trial_id] = (t, s)
        return super().on_trial_result(trial, result)

    def _explore(self, config):
        import numpy as np

        if self._np_rng is None:
            self._np_rng = np.random.default_rng(self.rng.randrange(1 << 30))
        new = copy.deepcopy(config)
        keys = list(self.bounds)
        cands = self._np_rng.random((256, len(keys)))
        if len(self.data) >= 3:
            from sklearn.gaussian_process import GaussianProcessRegressor
            from sklearn.gaussian_process.kernels import RBF, WhiteKernel

            D = np.asarray(self.data[-500:], dtype=np.float64)
            X, y = D[:, :-1], D[:, -1]
            tmax = max(1.0, X[:, 0].max())
            X = X.copy()
            X[:, 0] /= tmax
            y = (y - y.mean()) / (y.std() + 1e-9)
            gp = GaussianProcessRegressor(kernel=RBF(length_scale=0.5) + WhiteKernel(1e-2), normalize_y=False,
                                          random_state=0)
            gp.fit(X, y)
            tcol = np.full((len(cands), 1), 1.0)  # predict at the latest time
            mu, sd = gp.predict(np.hstack([tcol, cands]), return_std=True)
            beta = 2.0
            best = cands[int(np.argmax(mu + beta * sd))]
        else:
            best = cands[0]
        for k, x in zip(keys, best):
            lo, hi = self.bounds[k]
            v = lo + float(x) * (hi - lo)
            new[k] = type(config[k])(v) if isinstance(config.get(k), int) else v
        if self.explore_fn:
            new = self.explore_fn(new)
        return new


__all__ = ["TrialScheduler", "FIFOScheduler", "AsyncHyperBandScheduler", "ASHAScheduler",
           "HyperBandScheduler", "HyperBandForBOHB", "MedianStoppingRule", "PopulationBasedTraining",
           "PB2", "ResourceChangingScheduler", "DistributeResources"]
