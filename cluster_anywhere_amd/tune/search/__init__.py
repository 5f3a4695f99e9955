"""Search algorithms (reference: python/ray/tune/search/: basic_variant.py:189,
searcher.py, concurrency_limiter.py, repeater.py)."""
from __future__ import annotations

import random
from typing import Any, Dict, List, Optional

from .sample import (Categorical, Domain, Float, Function, Integer, choice, generate_variants,
                     grid_search, lograndint, loguniform, qlograndint, qloguniform, qrandint, qrandn,
                     quniform, randint, randn, sample_from, uniform)


class Searcher:
    FINISHED = "FINISHED"

    def __init__(self, metric: Optional[str] = None, mode: Optional[str] = None):
        self.metric, self.mode = metric, mode

    def set_search_properties(self, metric, mode, config, **spec) -> bool:
        self.metric = self.metric or metric
        self.mode = self.mode or mode
        return True

    def suggest(self, trial_id: str) -> Optional[Dict]:
        raise NotImplementedError

    def on_trial_result(self, trial_id: str, result: Dict):
        pass

    def on_trial_complete(self, trial_id: str, result: Optional[Dict] = None, error: bool = False):
        pass

    def save(self, path):
        import cloudpickle

        with open(path, "wb") as f:
            cloudpickle.dump(self, f)

    @staticmethod
    def load(path) -> "Searcher":
        import cloudpickle

        # written by Searcher.save() of this same experiment
        with open(path, "rb") as f:
            return cloudpickle.load(f)


class BasicVariantGenerator(Searcher):
    """Grid search x random sampling (the default)."""

    def __init__(self, points_to_evaluate: Optional[List[Dict]] = None, max_concurrent: int = 0,
                 random_state=None, constant_grid_search: bool = False):
        super().__init__()
        self.points = list(points_to_evaluate or [])
        self.seed = random_state
        self._it = None
        self.space = None
        self.num_samples = 1

    def set_search_properties(self, metric, mode, config, num_samples=1, **spec):
        super().set_search_properties(metric, mode, config)
        self.space = config
        self.num_samples = num_samples
        if self.seed is None:
            self.seed = random.randrange(2 ** 31)
        self._consumed = 0
        self._it = generate_variants(config, num_samples, self.seed)
        return True

    def suggest(self, trial_id):
        if self.points:
            p = self.points.pop(0)
            cfg = dict(self.space)
            cfg.update(p)
            return next(generate_variants(cfg, 1, self.seed))
        try:
            cfg = next(self._it)
        except StopIteration:
            return Searcher.FINISHED
        self._consumed += 1
        return cfg

    def __getstate__(self):
        d = dict(self.__dict__)
        d["_it"] = None
        return d

    def __setstate__(self, d):
        self.__dict__.update(d)
        if self.space is not None:
            # deterministic given the seed: replay and skip what was handed out
            self._it = generate_variants(self.space, self.num_samples, self.seed)
            for _ in range(self._consumed):
                next(self._it, None)


class RandomLocalSearch(Searcher):
    """Model-free sequential search: after ``n_initial`` random trials, sample
    around the incumbent (Gaussian perturbation of numeric domains, occasional
    categorical flips). A dependency-free stand-in for BayesOpt/HyperOpt."""

    def __init__(self, metric=None, mode=None, n_initial: int = 5, scale: float = 0.2, seed=None):
        super().__init__(metric, mode)
        self.n_initial, self.scale = n_initial, scale
        self.rng = random.Random(seed)
        self.results = []
        self.space = None
        self.count = 0
        self.limit = None

    def set_search_properties(self, metric, mode, config, num_samples=1, **spec):
        super().set_search_properties(metric, mode, config)
        self.space = config
        self.limit = num_samples
        return True

    def suggest(self, trial_id):
        if self.limit is not None and self.count >= self.limit:
            return Searcher.FINISHED
        self.count += 1
        base = next(generate_variants(self.space, 1, self.rng.random()))
        if len(self.results) < self.n_initial:
            return base
        sign = 1 if self.mode == "max" else -1
        best = max(self.results, key=lambda r: sign * r[1])[0]
        cfg = dict(best)
        for k, d in self.space.items():
            if isinstance(d, Float) and d.normal is None and isinstance(cfg.get(k), float):
                span = (d.upper - d.lower)
                v = cfg[k] + self.rng.gauss(0, self.scale * span)
                cfg[k] = min(d.upper, max(d.lower, v))
            elif isinstance(d, Integer):
                v = int(round(cfg[k] + self.rng.gauss(0, self.scale * (d.upper - d.lower))))
                cfg[k] = min(d.upper - 1, max(d.lower, v))
            elif isinstance(d, Categorical) and self.rng.random() < self.scale:
                cfg[k] = self.rng.choice(d.categories)
        return cfg

    def on_trial_complete(self, trial_id, result=None, error=False):
        if result and not error and self.metric in result:
            self.results.append((result.get("config", {}), result[self.metric]))


class ConcurrencyLimiter(Searcher):
    def __init__(self, searcher: Searcher, max_concurrent: int, batch: bool = False):
        super().__init__(searcher.metric, searcher.mode)
        self.searcher = searcher
        self.max_concurrent = max_concurrent
        self.live = set()

    def set_search_properties(self, metric, mode, config, **spec):
        return self.searcher.set_search_properties(metric, mode, config, **spec)

    def suggest(self, trial_id):
        if len(self.live) >= self.max_concurrent:
            return None
        cfg = self.searcher.suggest(trial_id)
        if cfg is not None and cfg != Searcher.FINISHED:
            self.live.add(trial_id)
        return cfg

    def on_trial_result(self, trial_id, result):
        self.searcher.on_trial_result(trial_id, result)

    def on_trial_complete(self, trial_id, result=None, error=False):
        self.live.discard(trial_id)
        self.searcher.on_trial_complete(trial_id, result, error)


class Repeater(Searcher):
    def __init__(self, searcher: Searcher, repeat: int = 1, set_index: bool = True):
        super().__init__(searcher.metric, searcher.mode)
        self.searcher, self.repeat, self.set_index = searcher, repeat, set_index
        self.pending = []

    def set_search_properties(self, metric, mode, config, **spec):
        return self.searcher.set_search_properties(metric, mode, config, **spec)

    def suggest(self, trial_id):
        if not self.pending:
            cfg = self.searcher.suggest(trial_id)
            if cfg is None or cfg == Searcher.FINISHED:
                return cfg
            self.pending = [dict(cfg, __trial_index__=i) if self.set_index else dict(cfg)
                            for i in range(self.repeat)]
        return self.pending.pop(0)

    def on_trial_complete(self, trial_id, result=None, error=False):
        self.searcher.on_trial_complete(trial_id, result, error)


__all__ = ["Searcher", "BasicVariantGenerator", "RandomLocalSearch", "ConcurrencyLimiter", "Repeater",
           "uniform", "quniform", "loguniform", "qloguniform", "randn", "qrandn", "randint", "qrandint",
           "lograndint", "qlograndint", "choice", "sample_from", "grid_search", "generate_variants"]
