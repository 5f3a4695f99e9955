"""Named trainables / envs, Experiment specs, scheduler & searcher factories
(reference: tune/registry.py, tune/experiment/experiment.py,
tune/schedulers/__init__.py create_scheduler, tune/search/__init__.py create_searcher)."""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional

_TRAINABLES: Dict[str, Any] = {}


def register_trainable(name: str, trainable, warn: bool = True):
    _TRAINABLES[name] = trainable


def register_env(name: str, env_creator: Callable):
    from ..rllib.env import register_env as _reg

    _reg(name, env_creator)


def get_trainable_cls(name: str):
    if name in _TRAINABLES:
        return _TRAINABLES[name]
    try:
        from ..rllib.algorithms import get_algorithm_class

        return get_algorithm_class(name)
    except KeyError:
        raise ValueError(f"unknown trainable {name!r}; register it with tune.register_trainable") from None


def resolve(trainable):
    return get_trainable_cls(trainable) if isinstance(trainable, str) else trainable


class ResumeConfig:
    """Which trials to resume/restart (reference: tune/tune.py ResumeConfig)."""

    def __init__(self, finished: str = "skip", unfinished: str = "resume", errored: str = "skip"):
        for v in (finished, unfinished, errored):
            if v not in ("skip", "resume", "restart"):
                raise ValueError("ResumeConfig values are 'skip', 'resume' or 'restart'")
        self.finished, self.unfinished, self.errored = finished, unfinished, errored


class Experiment:
    def __init__(self, name: str, run, *, stop=None, config: Optional[Dict] = None,
                 resources_per_trial=None, num_samples: int = 1, storage_path: Optional[str] = None,
                 checkpoint_config=None, max_failures: int = 0, **kw):
        self.name, self.run_identifier = name, run
        self.spec = dict(stop=stop, config=config or {}, resources_per_trial=resources_per_trial,
                         num_samples=num_samples, storage_path=storage_path, max_failures=max_failures, **kw)

    @classmethod
    def from_json(cls, name: str, spec: Dict[str, Any]) -> "Experiment":
        spec = dict(spec)
        return cls(name, spec.pop("run"), **spec)


def run_experiments(experiments, scheduler=None, verbose: int = 1, callbacks=None, **kw) -> List[Any]:
    from .tuner import run

    if isinstance(experiments, Experiment):
        experiments = [experiments]
    elif isinstance(experiments, dict):
        experiments = [Experiment.from_json(n, s) for n, s in experiments.items()]
    out = []
    for e in experiments:
        spec = {k: v for k, v in e.spec.items() if v is not None}
        out.append(run(resolve(e.run_identifier), name=e.name, scheduler=scheduler, verbose=verbose,
                       callbacks=callbacks, **spec))
    return out


def create_scheduler(scheduler: str, **kwargs):
    from . import schedulers as S

    table = {"fifo": S.FIFOScheduler, "async_hyperband": S.AsyncHyperBandScheduler, "asynchyperband":
             S.AsyncHyperBandScheduler, "asha": S.ASHAScheduler, "hyperband": S.HyperBandScheduler,
             "median_stopping_rule": S.MedianStoppingRule, "medianstopping": S.MedianStoppingRule,
             "pbt": S.PopulationBasedTraining, "pb2": S.PB2, "hb_bohb": S.HyperBandForBOHB,
             "resource_changing": S.ResourceChangingScheduler}
    if scheduler not in table:
        raise ValueError(f"unknown scheduler {scheduler!r}; available: {sorted(table)}")
    return table[scheduler](**kwargs)


def create_searcher(search_alg: str, **kwargs):
    from . import search as S

    from .search.bohb import TuneBOHB
    from .search.model_based import BayesOptSearch, HyperOptSearch, OptunaSearch

    table = {"variant_generator": S.BasicVariantGenerator, "random": S.BasicVariantGenerator,
             "random_local": S.RandomLocalSearch, "bohb": TuneBOHB, "optuna": OptunaSearch,
             "hyperopt": HyperOptSearch, "bayesopt": BayesOptSearch}
    if search_alg not in table:
        raise ValueError(f"unknown searcher {search_alg!r}; available here: {sorted(table)} "
                         "(external optimisation libraries are not installed in this image)")
    return table[search_alg](**kwargs)
