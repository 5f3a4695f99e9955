"""Trainable APIs (reference: python/ray/tune/trainable/trainable.py (class API),
function_trainable.py (function API), util.py:with_parameters,
tune/execution/placement_groups.py:PlacementGroupFactory)."""
from __future__ import annotations

import functools
import inspect
import os
import time
from typing import Any, Callable, Dict, List, Optional, Union


class Trainable:
    """Class-based trainable: override ``setup``, ``step``, ``save_checkpoint``,
    ``load_checkpoint`` (and optionally ``reset_config`` / ``cleanup``)."""

    def __init__(self, config: Optional[Dict] = None, trial_dir: str = "", trial_id: str = ""):
        self.config = dict(config or {})
        self._iteration = 0
        self._time_total = 0.0
        self._trial_dir = trial_dir
        self._trial_id = trial_id
        self.setup(self.config)

    # -- user hooks
    def setup(self, config: Dict):
        pass

    def step(self) -> Dict:
        raise NotImplementedError

    def save_checkpoint(self, checkpoint_dir: str) -> Optional[Dict]:
        return None

    def load_checkpoint(self, checkpoint: Union[Dict, str]):
        pass

    def reset_config(self, new_config: Dict) -> bool:
        return False

    def cleanup(self):
        pass

    # -- driver-facing
    @property
    def iteration(self):
        return self._iteration

    @property
    def training_iteration(self):
        return self._iteration

    @property
    def trial_id(self):
        return self._trial_id

    @property
    def logdir(self):
        return self._trial_dir

    def train(self) -> Dict:
        t0 = time.time()
        r = self.step()
        if not isinstance(r, dict):
            raise TypeError("Trainable.step() must return a dict")
        dt = time.time() - t0
        self._iteration += 1
        self._time_total += dt
        r = dict(r)
        r.setdefault("training_iteration", self._iteration)
        r.setdefault("time_this_iter_s", dt)
        r.setdefault("time_total_s", self._time_total)
        return r

    def save(self, checkpoint_dir: str) -> str:
        import json
        import pickle

        os.makedirs(checkpoint_dir, exist_ok=True)
        state = self.save_checkpoint(checkpoint_dir)
        if isinstance(state, dict):
            with open(os.path.join(checkpoint_dir, "_trainable_state.pkl"), "wb") as f:
                pickle.dump(state, f)
        with open(os.path.join(checkpoint_dir, "_trainable_meta.json"), "w") as f:
            json.dump({"iteration": self._iteration, "time_total": self._time_total}, f)
        return checkpoint_dir

    def restore(self, checkpoint_dir: str):
        import json
        import pickle

        meta = os.path.join(checkpoint_dir, "_trainable_meta.json")
        if os.path.exists(meta):
            with open(meta) as f:
                m = json.load(f)
            self._iteration, self._time_total = m["iteration"], m["time_total"]
        st = os.path.join(checkpoint_dir, "_trainable_state.pkl")
        if os.path.exists(st):
            # written by Trainable.save() of this same experiment
            with open(st, "rb") as f:
                self.load_checkpoint(pickle.load(f))
        else:
            self.load_checkpoint(checkpoint_dir)

    def stop(self):
        self.cleanup()


class PlacementGroupFactory:
    """Resource request of one trial as a list of bundles (bundle 0 = the trial
    actor itself)."""

    def __init__(self, bundles: List[Dict[str, float]], strategy: str = "PACK"):
        self.bundles = [dict(b) for b in bundles]
        self.strategy = strategy

    @property
    def head_bundle(self):
        return self.bundles[0] if self.bundles else {}

    def required_resources(self):
        out: Dict[str, float] = {}
        for b in self.bundles:
            for k, v in b.items():
                out[k] = out.get(k, 0) + v
        return out


def _normalize_resources(res) -> Dict[str, float]:
    if res is None:
        return {"CPU": 1}
    if isinstance(res, PlacementGroupFactory):
        return {k.upper() if k.lower() in ("cpu", "gpu") else k: v for k, v in res.head_bundle.items()}
    out = {}
    for k, v in dict(res).items():
        if k.lower() == "cpu":
            out["CPU"] = v
        elif k.lower() == "gpu":
            out["GPU"] = v
        else:
            out[k] = v
    out.setdefault("CPU", 1 if not out.get("GPU") else 1)
    return out


def with_resources(trainable, resources):
    """Attach a per-trial resource request (dict, PlacementGroupFactory or a
    callable config -> request)."""
    if inspect.isclass(trainable):
        cls = type(trainable.__name__, (trainable,), {})
        cls._tune_resources = resources
        return cls

    @functools.wraps(trainable)
    def wrapped(*a, **k):
        return trainable(*a, **k)

    wrapped._tune_resources = resources
    return wrapped


def with_parameters(trainable, **kwargs):
    """Store large objects in the object store once; each trial fetches them
    by reference instead of re-serialising them with the trainable."""
    from ..core import api as core

    refs = {k: core.put(v) for k, v in kwargs.items()}
    if inspect.isclass(trainable):
        base = trainable

        class _WithParams(base):
            def setup(self, config):
                params = {k: core.get(r) for k, r in refs.items()}
                return base.setup(self, config, **params)

        _WithParams.__name__ = base.__name__
        return _WithParams

    @functools.wraps(trainable)
    def fn(config):
        params = {k: core.get(r) for k, r in refs.items()}
        return trainable(config, **params)

    fn._tune_param_refs = refs
    if hasattr(trainable, "_tune_resources"):
        fn._tune_resources = trainable._tune_resources
    return fn


def trainable_resources(trainable, config=None) -> Dict[str, float]:
    from ..train.trainer import DataParallelTrainer

    if isinstance(trainable, DataParallelTrainer):
        return {"CPU": 0}
    res = getattr(trainable, "_tune_resources", None)
    if callable(res) and not isinstance(res, (dict, PlacementGroupFactory)):
        res = res(config or {})
    return _normalize_resources(res)
