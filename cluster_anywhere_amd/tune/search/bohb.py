"""BOHB's model-based searcher (reference: python/ray/tune/search/bohb/bohb_search.py,
Falkner et al. 2018), implemented without hpbandster / ConfigSpace: a TPE-style
pair of kernel density estimates over the numeric hyperparameters (categoricals
by smoothed frequencies), fitted on the largest HyperBand budget that has enough
observations; new configurations maximise l(x) / g(x) among samples drawn from
the "good" density. Use it with ``HyperBandForBOHB``, which reports every
milestone result through ``on_budget_result``."""
from __future__ import annotations

import math
import random
from typing import Dict, List, Optional

from . import Searcher
from .sample import Categorical, Domain, Float, Integer


class TuneBOHB(Searcher):
    def __init__(self, space: Optional[Dict] = None, metric: Optional[str] = None,
                 mode: Optional[str] = None, min_points_in_model: Optional[int] = None,
                 top_n_percent: int = 15, num_samples: int = 64, random_fraction: float = 1 / 3,
                 bandwidth_factor: float = 3.0, min_bandwidth: float = 1e-3, seed: Optional[int] = None,
                 max_concurrent: int = 0):
        super().__init__(metric, mode)
        self.space = dict(space or {})
        self.min_points = min_points_in_model
        self.gamma = top_n_percent / 100.0
        self.n_samples = num_samples
        self.random_fraction = random_fraction
        self.bw_factor, self.min_bw = bandwidth_factor, min_bandwidth
        self.rng = random.Random(seed)
        self.configs: Dict[str, Dict] = {}
        self.obs: Dict[float, List[tuple]] = {}  # budget -> [(vector, score)]

    def set_search_properties(self, metric, mode, config, **spec):
        super().set_search_properties(metric, mode, config, **spec)
        self.max_trials = spec.get("num_samples")
        if not self.space:
            self.space = {k: v for k, v in (config or {}).items() if isinstance(v, Domain)}
        return True

    # -- encoding: every hyperparameter -> [0, 1]
    def _encode(self, cfg):
        out = []
        for k, d in self.space.items():
            v = cfg[k]
            if isinstance(d, Categorical):
                out.append((d.categories.index(v) + 0.5) / len(d.categories))
            elif getattr(d, "log", False):
                lo, hi = math.log(d.lower), math.log(d.upper)
                out.append((math.log(v) - lo) / (hi - lo))
            else:
                out.append((v - d.lower) / (d.upper - d.lower))
        return out

    def _decode(self, vec):
        cfg = {}
        for (k, d), x in zip(self.space.items(), vec):
            x = min(max(x, 0.0), 1.0)
            if isinstance(d, Categorical):
                cfg[k] = d.categories[min(len(d.categories) - 1, int(x * len(d.categories)))]
            elif getattr(d, "log", False):
                lo, hi = math.log(d.lower), math.log(d.upper)
                v = math.exp(lo + x * (hi - lo))
                cfg[k] = int(round(v)) if isinstance(d, Integer) else v
            else:
                v = d.lower + x * (d.upper - d.lower)
                cfg[k] = int(round(min(v, d.upper - 1))) if isinstance(d, Integer) else v
        return cfg

    def _model_budget(self):
        need = self.min_points or (len(self.space) + 1)
        for b in sorted(self.obs, reverse=True):
            if len(self.obs[b]) >= need + 2:
                return b
        return None

    def suggest(self, trial_id):
        if getattr(self, "max_trials", None) and len(self.configs) >= self.max_trials:
            return Searcher.FINISHED
        b = self._model_budget()
        if b is None or self.rng.random() < self.random_fraction:
            cfg = {k: d.sample(None, self.rng) for k, d in self.space.items()}
        else:
            cfg = self._decode(self._propose(self.obs[b]))
        self.configs[trial_id] = cfg
        return dict(cfg)

    def _propose(self, data):
        import numpy as np
        from scipy.stats import gaussian_kde

        data = sorted(data, key=lambda x: x[1], reverse=True)
        n_good = max(len(self.space) + 1, int(math.ceil(self.gamma * len(data))))
        good = np.asarray([d[0] for d in data[:n_good]]).T
        bad = np.asarray([d[0] for d in data[n_good:]] or [d[0] for d in data[-2:]]).T
        jitter = lambda a: a + 1e-6 * np.random.default_rng(0).standard_normal(a.shape)  # noqa: E731
        try:
            lk = gaussian_kde(jitter(good), bw_method=max(self.min_bw, 0.3 * self.bw_factor / 3))
            gk = gaussian_kde(jitter(bad), bw_method=max(self.min_bw, 0.3 * self.bw_factor / 3))
        except (np.linalg.LinAlgError, ValueError):
            return [self.rng.random() for _ in self.space]
        cands = np.clip(lk.resample(self.n_samples, seed=self.rng.randrange(1 << 30)), 0.0, 1.0)
        score = lk(cands) / np.maximum(gk(cands), 1e-32)
        return list(cands[:, int(np.argmax(score))])

    def on_budget_result(self, trial_id, result, budget):
        cfg = self.configs.get(trial_id)
        v = result.get(self.metric)
        if cfg is None or v is None or budget is None:
            return
        s = v if self.mode == "max" else -v
        self.obs.setdefault(float(budget), []).append((self._encode(cfg), s))

    def on_trial_complete(self, trial_id, result=None, error=False):
        if result and not error:
            b = result.get("training_iteration")
            self.on_budget_result(trial_id, result, b)
