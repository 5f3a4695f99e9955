"""Tuner / TuneConfig / ResultGrid / tune.run (reference: python/ray/tune/tuner.py:44,
tune_config.py, result_grid.py, tune.py:run, analysis/experiment_analysis.py)."""
from __future__ import annotations

import json
import math
import os
import time
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional

from ..core import api as core
from ..train.checkpoint import Checkpoint
from ..train.config import CheckpointConfig, FailureConfig, RunConfig
from ..train.trainer import Result
from .controller import Trial, TuneController
from .schedulers import TrialScheduler
from .search import Searcher


@dataclass
class TuneConfig:
    metric: Optional[str] = None
    mode: Optional[str] = None
    search_alg: Optional[Searcher] = None
    scheduler: Optional[TrialScheduler] = None
    num_samples: int = 1
    max_concurrent_trials: Optional[int] = None
    time_budget_s: Any = None
    reuse_actors: bool = False
    trial_name_creator: Optional[Callable] = None
    trial_dirname_creator: Optional[Callable] = None

    def __post_init__(self):
        if self.mode not in (None, "min", "max"):
            raise ValueError("mode must be 'min' or 'max'")


def _trial_result(t: Trial) -> Result:
    return Result(metrics=dict(t.last_result), checkpoint=t.checkpoint, error=t.error,
                  path=t.local_path, metrics_history=list(t.history))


class ResultGrid:
    def __init__(self, trials: List[Trial], experiment_path: str, metric=None, mode=None):
        self._trials = trials
        self._results = [_trial_result(t) for t in trials]
        self.experiment_path = experiment_path
        self._metric, self._mode = metric, mode

    def __len__(self):
        return len(self._results)

    def __getitem__(self, i) -> Result:
        return self._results[i]

    def __iter__(self):
        return iter(self._results)

    @property
    def errors(self):
        return [r.error for r in self._results if r.error is not None]

    @property
    def num_errors(self):
        return len(self.errors)

    @property
    def num_terminated(self):
        return sum(1 for t in self._trials if t.status == Trial.TERMINATED)

    def get_best_result(self, metric: Optional[str] = None, mode: Optional[str] = None,
                        scope: str = "last", filter_nan_and_inf: bool = True) -> Result:
        metric = metric or self._metric
        mode = mode or self._mode
        if not metric or not mode:
            raise ValueError("get_best_result needs metric and mode (pass them or set TuneConfig)")
        best, best_v = None, None
        for r in self._results:
            v = _scope_value(r._history, metric, mode, scope)
            if v is None or (filter_nan_and_inf and (math.isnan(v) or math.isinf(v))):
                continue
            if best_v is None or (v > best_v if mode == "max" else v < best_v):
                best, best_v = r, v
        if best is None:
            raise RuntimeError(f"no trial reported metric {metric!r}")
        return best

    def get_dataframe(self, filter_metric: Optional[str] = None, filter_mode: Optional[str] = None):
        import pandas as pd

        rows = []
        for r in self._results:
            if filter_metric and filter_mode:
                vals = [h[filter_metric] for h in r._history if filter_metric in h]
                if not vals:
                    continue
                pick = max if filter_mode == "max" else min
                target = pick(vals)
                row = next(h for h in r._history if h.get(filter_metric) == target)
            else:
                row = r.metrics
            flat = {}
            for k, v in row.items():
                if k == "config" and isinstance(v, dict):
                    for ck, cv in v.items():
                        flat[f"config/{ck}"] = cv
                else:
                    flat[k] = v
            flat["logdir"] = r.path
            rows.append(flat)
        return pd.DataFrame(rows)

    def __repr__(self):
        return f"ResultGrid<{len(self)} results, {self.num_errors} errors>"


def _scope_value(history, metric, mode, scope):
    vals = [h[metric] for h in history if metric in h and isinstance(h[metric], (int, float))]
    if not vals:
        return None
    if scope == "last":
        return vals[-1]
    if scope == "all":
        return max(vals) if mode == "max" else min(vals)
    if scope == "avg":
        return sum(vals) / len(vals)
    if scope.startswith("last-") and scope.endswith("-avg"):
        n = int(scope.split("-")[1])
        tail = vals[-n:]
        return sum(tail) / len(tail)
    raise ValueError(f"unknown scope {scope!r}")


class Tuner:
    """``Tuner(trainable, param_space=..., tune_config=..., run_config=...).fit()``.
    ``trainable`` may be a function, a ``Trainable`` subclass or a Train trainer
    (``DataParallelTrainer``/``TorchTrainer``) whose ``train_loop_config`` is
    tuned."""

    def __init__(self, trainable=None, *, param_space: Optional[Dict] = None,
                 tune_config: Optional[TuneConfig] = None, run_config: Optional[RunConfig] = None,
                 _restored_trials: Optional[List[Trial]] = None, _exp_dir: Optional[str] = None):
        from .registry import resolve

        self.trainable = resolve(trainable)
        self.param_space = param_space or {}
        self.tune_config = tune_config or TuneConfig()
        if run_config is None:
            run_config = getattr(trainable, "run_config", None) or RunConfig()
        self.run_config = run_config
        self._restored = _restored_trials
        self._exp_dir = _exp_dir

    def _experiment_dir(self):
        if self._exp_dir:
            return self._exp_dir
        name = self.run_config.name or f"{getattr(self.trainable, '__name__', type(self.trainable).__name__)}" \
                                       f"_{time.strftime('%Y-%m-%d_%H-%M-%S')}"
        self.run_config.name = name
        self._storage = _remote_storage(self.run_config)
        if self._storage is not None:
            # remote storage (URI / storage_filesystem): the experiment is staged in a
            # local directory of the driver and mirrored to the storage filesystem
            d = os.path.join(_fresh_staging_dir(), name)
        else:
            d = os.path.join(self.run_config.storage_path, name)
        os.makedirs(d, exist_ok=True)
        self._exp_dir = d
        return d

    def fit(self) -> ResultGrid:
        core._ensure_init()
        exp_dir = self._experiment_dir()
        self._save_tuner(exp_dir)
        st = getattr(self, "_storage", None)
        syncer = None
        if st is not None:
            st.create_experiment_dir()
            period = float(getattr(self.run_config.sync_config, "sync_period", 60) or 60)
            syncer = _Syncer(exp_dir, st, period)
        ctl = TuneController(self.trainable, self.param_space, self.tune_config, self.run_config,
                             exp_dir, self._restored, syncer=syncer)
        trials = ctl.run()
        self._restored = trials
        grid = ResultGrid(trials, exp_dir, self.tune_config.metric, self.tune_config.mode)
        if st is not None:
            grid.storage_filesystem, grid.storage_path = st.storage_filesystem, st.experiment_fs_path
        return grid

    def get_results(self) -> ResultGrid:
        if self._restored is None:
            raise RuntimeError("fit() has not been called")
        return ResultGrid(self._restored, self._exp_dir, self.tune_config.metric, self.tune_config.mode)

    def _save_tuner(self, exp_dir):
        from ..core.serialization import dumps_function

        try:
            blob = dumps_function({"param_space": self.param_space, "tune_config": self.tune_config,
                                   "run_config": self.run_config})
            with open(os.path.join(exp_dir, "tuner.pkl"), "wb") as f:
                f.write(blob)
        except Exception:
            pass

    @classmethod
    def can_restore(cls, path: str, storage_filesystem=None) -> bool:
        if storage_filesystem is not None or "://" in path:
            from ..train.storage import get_fs_and_path
            import pyarrow.fs as pafs

            fs, p = get_fs_and_path(path, storage_filesystem)
            return fs.get_file_info(p.rstrip("/") + "/experiment_state.json").type == pafs.FileType.File
        return os.path.exists(os.path.join(path, "experiment_state.json"))

    @classmethod
    def restore(cls, path: str, trainable, *, resume_unfinished: bool = True, resume_errored: bool = False,
                restart_errored: bool = False, param_space: Optional[Dict] = None, **kw) -> "Tuner":
        """Resume an interrupted experiment: finished trials are kept, unfinished
        ones relaunch from their latest checkpoint (errored ones on request).
        ``path`` may be a URI or a path inside ``storage_filesystem``: the
        experiment is downloaded into the local staging directory first."""
        import cloudpickle

        storage_filesystem = kw.get("storage_filesystem")
        remote = storage_filesystem is not None or "://" in path
        if remote:
            from ..train.storage import download_dir, get_fs_and_path

            fs, fs_path = get_fs_and_path(path, storage_filesystem)
            fs_path = fs_path.rstrip("/")
            local = os.path.join(_fresh_staging_dir(), os.path.basename(fs_path))
            download_dir(fs, fs_path, local)
            remote_root = (path.rstrip("/").rsplit("/", 1)[0] if "://" in path
                           else os.path.dirname(fs_path) if storage_filesystem is None else fs_path.rsplit("/", 1)[0])
            path = local

        with open(os.path.join(path, "experiment_state.json")) as f:
            st = json.load(f)
        tc, rc, ps = TuneConfig(), RunConfig(), param_space or {}
        tp = os.path.join(path, "tuner.pkl")
        if os.path.exists(tp):
            # written by Tuner._save_tuner of this experiment (our own file)
            with open(tp, "rb") as f:
                saved = cloudpickle.loads(f.read())
            tc, rc = saved["tune_config"], saved["run_config"]
            ps = param_space or saved["param_space"]
        tc._searcher_finished = st.get("searcher_finished", False)
        if remote:  # keep mirroring to where it came from
            rc.storage_path, rc.storage_filesystem = remote_root, storage_filesystem
        else:
            rc.storage_path = os.path.dirname(os.path.abspath(path))
        rc.name = os.path.basename(os.path.abspath(path))
        trials = []
        for ts in st["trials"]:
            t = Trial(ts["trial_id"], ts["config"] or {}, path, ts["name"], ts.get("resources") or {"CPU": 1})
            t.status = ts["status"]
            t.last_result = ts.get("last_result") or {}
            t.latest_checkpoint = ts.get("latest_checkpoint")
            t.num_failures = ts.get("num_failures", 0)
            t.iteration = ts.get("iteration", 0)
            t.ckpt_index = ts.get("ckpt_index", 0)
            t.error_msg = ts.get("error_msg")
            rp = os.path.join(t.local_path, "result.json")
            if os.path.exists(rp):
                with open(rp) as f:
                    t.history = [json.loads(l) for l in f if l.strip()]
            if t.status in (Trial.RUNNING, Trial.PAUSED, Trial.PENDING):
                t.status = Trial.PENDING if resume_unfinished else Trial.TERMINATED
            elif t.status == Trial.ERROR:
                if restart_errored:
                    t.status, t.latest_checkpoint, t.num_failures = Trial.PENDING, None, 0
                    t.iteration, t.history = 0, []
                elif resume_errored:
                    t.status, t.num_failures = Trial.PENDING, 0
                else:
                    t.error = RuntimeError(t.error_msg or "trial errored")
            trials.append(t)
        return cls(trainable, param_space=ps, tune_config=tc, run_config=rc, _restored_trials=trials,
                   _exp_dir=os.path.abspath(path))


class ExperimentAnalysis(ResultGrid):
    """Return type of the legacy ``tune.run``."""

    @property
    def trials(self):
        return self._trials

    @property
    def best_result(self):
        return self.get_best_result().metrics

    @property
    def best_config(self):
        return self.get_best_result().metrics.get("config")

    def get_best_config(self, metric=None, mode=None, scope="last"):
        return self.get_best_result(metric, mode, scope).metrics.get("config")

    @property
    def best_checkpoint(self):
        return self.get_best_result().checkpoint

    @property
    def best_trial(self):
        best = self.get_best_result()
        return next(t for t in self._trials if t.local_path == best.path)

    @property
    def results_df(self):
        return self.get_dataframe()

    @property
    def dataframe(self):
        return self.get_dataframe()


def run(run_or_experiment, *, config: Optional[Dict] = None, name: Optional[str] = None,
        metric: Optional[str] = None, mode: Optional[str] = None, stop=None, num_samples: int = 1,
        storage_path: Optional[str] = None, search_alg=None, scheduler=None,
        resources_per_trial=None, max_concurrent_trials: Optional[int] = None, time_budget_s=None,
        max_failures: int = 0, checkpoint_freq: int = 0, checkpoint_at_end: bool = False,
        callbacks=None, verbose: int = 1, fail_fast: bool = False, **_ignored) -> ExperimentAnalysis:
    from .trainable import with_resources

    from .registry import resolve

    trainable = resolve(run_or_experiment)
    if resources_per_trial is not None:
        trainable = with_resources(trainable, resources_per_trial)
    rc = RunConfig(name=name, storage_path=storage_path, stop=stop, callbacks=callbacks,
                   failure_config=FailureConfig(max_failures=max_failures, fail_fast=fail_fast),
                   checkpoint_config=CheckpointConfig(checkpoint_frequency=checkpoint_freq,
                                                      checkpoint_at_end=checkpoint_at_end))
    tc = TuneConfig(metric=metric, mode=mode, search_alg=search_alg, scheduler=scheduler,
                    num_samples=num_samples, max_concurrent_trials=max_concurrent_trials,
                    time_budget_s=time_budget_s)
    tuner = Tuner(trainable, param_space=config or {}, tune_config=tc, run_config=rc)
    grid = tuner.fit()
    return ExperimentAnalysis(grid._trials, grid.experiment_path, metric, mode)


def _staging_root() -> str:
    import tempfile

    return os.environ.get("CAAMD_TUNE_STAGING_DIR") or os.path.join(tempfile.gettempdir(), "caamd_tune_staging")


_staged_dirs: List[str] = []


def _fresh_staging_dir() -> str:
    """A new local staging directory per fit / restore: a reused one would mirror a
    previous run's (or a concurrent tuner's) trial dirs to the new remote experiment
    and merge a restore's download into stale files. Removed at exit
    (the results of the run live in the storage filesystem)."""
    import atexit
    import shutil
    import tempfile

    root = _staging_root()
    os.makedirs(root, exist_ok=True)
    d = tempfile.mkdtemp(prefix="run_", dir=root)
    if not _staged_dirs:
        atexit.register(lambda: [shutil.rmtree(x, ignore_errors=True) for x in _staged_dirs])
    _staged_dirs.append(d)
    return d


def _remote_storage(run_config):
    """A StorageContext when the run's storage is not a plain local path."""
    sp, fs = run_config.storage_path, getattr(run_config, "storage_filesystem", None)
    if fs is None and not (isinstance(sp, str) and "://" in sp):
        return None
    from ..train.storage import StorageContext

    st = StorageContext(sp, run_config.name, fs)
    return None if st.local and fs is None and not sp.startswith("file://") else st


class _Syncer:
    """Mirror of the local experiment staging directory to the storage filesystem
    (reference role: tune/syncer.py): at most every ``period_s`` seconds, and on
    ``sync(force=True)`` (end of the experiment)."""

    def __init__(self, local_dir: str, storage, period_s: float = 60.0):
        self.local_dir, self.storage, self.period_s = local_dir, storage, period_s
        self.last = 0.0

    def sync(self, force: bool = False):
        now = time.time()
        if not force and now - self.last < self.period_s:
            return
        self.last = now
        from ..train.storage import upload_dir

        upload_dir(self.local_dir, self.storage.storage_filesystem, self.storage.experiment_fs_path)
