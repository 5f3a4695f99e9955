"""Trial execution (reference: python/ray/tune/execution/tune_controller.py:68,
experiment/trial.py, trainable/function_trainable.py).

Each trial runs in its own ``_TrialRunner`` actor (resources = the trial's
request; 0 CPU for Trainer trainables, whose workers reserve their own
placement group). The controller loop on the driver:

  launch  : ask the searcher for configs while concurrency allows
  poll    : one batched ``poll`` call per running trial (reports + done/error)
  decide  : stopper -> scheduler (CONTINUE / PAUSE / STOP) -> searcher hooks
  persist : per-trial result.json / progress.csv / params.json and an
            experiment_state.json snapshot used by ``Tuner.restore``
"""
from __future__ import annotations

import csv
import inspect
import json
import math
import os
import shutil
import threading
import time
import traceback
import uuid
from typing import Any, Dict, List, Optional

from ..core import api as core
from .schedulers import FIFOScheduler, PopulationBasedTraining, TrialScheduler
from .search import BasicVariantGenerator, Searcher
from .session import StopTrial, TuneSession, set_session
from .stopper import make_stopper
from .trainable import Trainable, trainable_resources


def _jsonable(v):
    try:
        json.dumps(v)
        return True
    except (TypeError, ValueError):
        return False


def _flatten(d, prefix=""):
    out = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            out.update(_flatten(v, key + "/"))
        else:
            out[key] = v
    return out


class Trial:
    PENDING, RUNNING, PAUSED, TERMINATED, ERROR = "PENDING", "RUNNING", "PAUSED", "TERMINATED", "ERROR"

    def __init__(self, trial_id: str, config: Dict, exp_dir: str, name: str, resources: Dict):
        self.trial_id = trial_id
        self.config = config
        self.trial_name = name
        self.local_path = os.path.join(exp_dir, name)
        self.status = Trial.PENDING
        self.last_result: Dict[str, Any] = {}
        self.history: List[Dict] = []
        self.latest_checkpoint: Optional[str] = None
        self.error: Optional[BaseException] = None
        self.error_msg: Optional[str] = None
        self.num_failures = 0
        self.resources = resources
        self.actor = None
        self.pending_exploit = None
        self.iteration = 0
        self.ckpt_index = 0
        self.start_time = None
        self._csv_keys = None

    @property
    def path(self):
        return self.local_path

    @property
    def checkpoint(self):
        from ..train.checkpoint import Checkpoint

        return Checkpoint(self.latest_checkpoint) if self.latest_checkpoint else None

    def __repr__(self):
        return f"Trial({self.trial_name}, {self.status})"

    def to_state(self):
        return {"trial_id": self.trial_id, "config": self.config if _jsonable(self.config) else None,
                "name": self.trial_name, "status": self.status, "last_result": self.last_result,
                "latest_checkpoint": self.latest_checkpoint, "num_failures": self.num_failures,
                "iteration": self.iteration, "ckpt_index": self.ckpt_index,
                "error_msg": self.error_msg, "resources": self.resources}


class _TrainerForwarder:
    """RunConfig callback that forwards a nested Trainer's reports to the trial."""

    def __init__(self, session: TuneSession):
        self.session = session

    def on_report_with_checkpoint(self, metrics, path):
        s = self.session
        s.iteration += 1
        m = dict(metrics)
        m["training_iteration"] = s.iteration
        s.reports.put((m, path))


class _TrialRunner:
    """Actor hosting one trial's training thread."""

    def __init__(self):
        self.session = None
        self.thread = None
        self.done = False
        self.error = None

    def start(self, trainable, config, info, ckpt_path, checkpoint_freq, checkpoint_at_end):
        from ..train.checkpoint import Checkpoint
        from ..train.trainer import DataParallelTrainer

        os.makedirs(info["trial_dir"], exist_ok=True)
        ckpt = Checkpoint(ckpt_path) if ckpt_path else None
        s = TuneSession(info["trial_id"], info["trial_name"], info["trial_dir"], info["experiment_name"],
                        ckpt, info["iteration"], info["ckpt_index"], info["storage_path"], info["resources"])
        self.session = s
        set_session(s, global_=True)

        def run_function():
            if len(inspect.signature(trainable).parameters) == 0:
                trainable()
            else:
                trainable(config)

        def run_class():
            obj = trainable(config, info["trial_dir"], info["trial_id"])
            if ckpt_path:
                obj.restore(ckpt_path)
            try:
                while not s.stop_requested:
                    r = obj.train()
                    s.iteration = r["training_iteration"]
                    path = None
                    done = bool(r.get("done"))
                    if (checkpoint_freq and r["training_iteration"] % checkpoint_freq == 0) or \
                            (done and checkpoint_at_end):
                        path = obj.save(os.path.join(info["trial_dir"], f"checkpoint_{s.ckpt_index:06d}"))
                        s.ckpt_index += 1
                    s.reports.put((r, path))
                    if done:
                        break
            finally:
                obj.stop()

        def run_trainer():
            import copy

            tr = copy.copy(trainable)
            base = dict(tr.train_loop_config or {})
            cfg = dict(config)
            base.update(cfg.pop("train_loop_config", {}) or {})
            base.update({k: v for k, v in cfg.items() if k not in ("scaling_config", "datasets")})
            tr.train_loop_config = base
            if "scaling_config" in cfg:
                tr.scaling_config = cfg["scaling_config"]
            rc = copy.copy(tr.run_config)
            rc.name = info["trial_name"]
            rc.storage_path = os.path.dirname(info["trial_dir"])
            rc.callbacks = list(rc.callbacks or []) + [_TrainerForwarder(s)]
            tr.run_config = rc
            if ckpt is not None:
                tr.resume_from_checkpoint = ckpt
            tr.fit()

        if isinstance(trainable, DataParallelTrainer):
            body = run_trainer
        elif inspect.isclass(trainable) and issubclass(trainable, Trainable):
            body = run_class
        else:
            body = run_function

        def target():
            try:
                body()
            except StopTrial:
                pass
            except BaseException as e:  # noqa
                from ..exceptions import RayTaskError

                self.error = RayTaskError.from_exception(info["trial_name"], e)
            finally:
                self.done = True

        self.thread = threading.Thread(target=target, name="tune-trial", daemon=True)
        self.thread.start()
        return True

    def poll(self, timeout=0.2):
        deadline = time.time() + timeout
        while self.session is None:  # poll may overtake start on a threaded actor
            if time.time() >= deadline:
                return [], False, None
            time.sleep(0.01)
        s = self.session
        out = []
        while True:
            try:
                out.append(s.reports.get(timeout=max(0.0, min(0.05, deadline - time.time()))))
                while True:
                    out.append(s.reports.get_nowait())
            except Exception:
                pass
            if out or self.done or time.time() >= deadline:
                break
        if out:
            s.consumed.set()
        return out, self.done and s.reports.empty(), self.error

    def stop(self):
        if self.session is not None:
            self.session.stop_requested = True
        return True


class TuneController:
    def __init__(self, trainable, param_space: Dict, tune_config, run_config, exp_dir: str,
                 trials: Optional[List[Trial]] = None, syncer=None):
        self.syncer = syncer  # mirror of exp_dir to remote storage (tuner._Syncer) or None
        self.trainable = trainable
        self.param_space = param_space or {}
        self.tc = tune_config
        self.rc = run_config
        self.exp_dir = exp_dir
        self.exp_name = os.path.basename(exp_dir)
        self.metric, self.mode = tune_config.metric, tune_config.mode
        self.searcher: Searcher = tune_config.search_alg or BasicVariantGenerator()
        self.scheduler: TrialScheduler = tune_config.scheduler or FIFOScheduler()
        self.scheduler.set_search_properties(self.metric, self.mode)
        self.stopper = make_stopper(run_config.stop)
        self.callbacks = list(run_config.callbacks or [])
        self.trials: List[Trial] = list(trials or [])
        self.searcher_finished = False
        self._counter = len(self.trials)
        self._last_save = 0.0
        self.start = time.time()
        cc = run_config.checkpoint_config
        self.ckpt_freq = getattr(cc, "checkpoint_frequency", 0) or 0
        self.ckpt_at_end = bool(getattr(cc, "checkpoint_at_end", False))
        from .schedulers import HyperBandForBOHB, HyperBandScheduler, ResourceChangingScheduler

        if isinstance(self.scheduler, (PopulationBasedTraining, HyperBandScheduler, ResourceChangingScheduler)) \
                and not self.ckpt_freq:
            self.ckpt_freq = 1  # pausing schedulers resume trials from checkpoints
        if isinstance(self.scheduler, ResourceChangingScheduler):
            self.scheduler.controller = self
        if isinstance(self.scheduler, HyperBandForBOHB):
            self.scheduler.searcher = self.searcher
        sp = os.path.join(exp_dir, "searcher_state.pkl")
        if trials is not None and os.path.exists(sp):
            self.searcher = Searcher.load(sp)
            self.searcher_finished = bool(getattr(tune_config, "_searcher_finished", False))
        elif not trials:
            self.searcher.set_search_properties(self.metric, self.mode, self.param_space,
                                                num_samples=tune_config.num_samples)
        else:
            self.searcher_finished = True
        self.max_concurrent = self._max_concurrent()

    # -------------------------------------------------------------- resources
    def _trial_request(self, config) -> Dict[str, float]:
        from ..train.trainer import DataParallelTrainer

        if isinstance(self.trainable, DataParallelTrainer):
            sc = (config or {}).get("scaling_config") or self.trainable.scaling_config
            return dict(sc.total_resources)  # workers + the coordinator's trainer_resources
        return trainable_resources(self.trainable, config)

    def _max_concurrent(self):
        limit = self.tc.max_concurrent_trials or 10 ** 9
        total = core.cluster_resources()
        req = self._trial_request(None)
        fit = 10 ** 9
        for k, v in req.items():
            if v > 0:
                fit = min(fit, int(math.floor(total.get(k, 0) / v + 1e-9)))
        return max(1, min(limit, fit))

    # ------------------------------------------------------------------ launch
    def _new_trial(self, config, tid=None):
        tid = tid or uuid.uuid4().hex[:8]
        base = getattr(self.trainable, "__name__", type(self.trainable).__name__)
        if self.tc.trial_name_creator:
            name = self.tc.trial_name_creator(_TrialInfo(tid, config))
        else:
            name = f"{base}_{tid}_{self._counter:05d}"
        self._counter += 1
        t = Trial(tid, config, self.exp_dir, name, trainable_resources(self.trainable, config))
        self.trials.append(t)
        self.scheduler.on_trial_add(t)
        return t

    def _launch(self, t: Trial):
        from .. import exceptions  # noqa
        from ..core.actor import ActorClass

        os.makedirs(t.local_path, exist_ok=True)
        with open(os.path.join(t.local_path, "params.json"), "w") as f:
            json.dump({k: v for k, v in t.config.items() if _jsonable(v)}, f, indent=1)
        res = t.resources
        Runner = ActorClass(_TrialRunner, {})
        env = {"CAAMD_NOSET_ROCR_VISIBLE_DEVICES": "1"} if not res.get("GPU") else {}
        t.actor = Runner.options(num_cpus=res.get("CPU", 1), num_gpus=res.get("GPU", 0),
                                 resources={k: v for k, v in res.items() if k not in ("CPU", "GPU")},
                                 runtime_env={"env_vars": env} if env else None,
                                 max_concurrency=4).remote()
        info = {"trial_id": t.trial_id, "trial_name": t.trial_name, "trial_dir": t.local_path,
                "experiment_name": self.exp_name, "iteration": t.iteration, "ckpt_index": t.ckpt_index,
                "storage_path": os.path.dirname(self.exp_dir), "resources": res}
        t._start_ref = t.actor.start.remote(self.trainable, t.config, info, t.latest_checkpoint,
                                            self.ckpt_freq, self.ckpt_at_end)
        t.status = Trial.RUNNING
        t.start_time = t.start_time or time.time()
        t._poll_ref = None
        for cb in self.callbacks:
            if hasattr(cb, "on_trial_start"):
                cb.on_trial_start(iteration=0, trials=self.trials, trial=t)

    def _fill(self):
        by_id = {t.trial_id: t for t in self.trials}
        for tid in self.scheduler.pop_stopped_trials():
            t = by_id.get(tid)
            if t is not None and t.status in (Trial.PAUSED, Trial.PENDING):
                self._complete(t)
        running = [t for t in self.trials if t.status == Trial.RUNNING]
        slots = self.max_concurrent - len(running)
        # resume paused / pending (restored or exploited) trials first, in the order
        # the scheduler allows (synchronous HyperBand gates paused trials)
        waiting = [t for t in self.trials if t.status in (Trial.PENDING, Trial.PAUSED) and t.actor is None]
        while slots > 0 and waiting:
            t = self.scheduler.choose_trial_to_run(waiting)
            if t is None:
                break
            waiting.remove(t)
            self._launch(t)
            slots -= 1
        if slots <= 0:
            return
        while slots > 0 and not self.searcher_finished:
            tid = uuid.uuid4().hex[:8]
            cfg = self.searcher.suggest(tid)
            if cfg is None:
                return
            if cfg == Searcher.FINISHED:
                self.searcher_finished = True
                return
            t = self._new_trial(cfg, tid)
            self._launch(t)
            slots -= 1

    # ---------------------------------------------------------------- results
    def _stop_actor(self, t: Trial):
        if t.actor is not None:
            try:
                core.kill(t.actor)
            except Exception:
                pass
            t.actor = None

    def _record(self, t: Trial, m: Dict, path: Optional[str]):
        m = dict(m)
        m.setdefault("trial_id", t.trial_id)
        m["config"] = t.config
        m.setdefault("timestamp", int(time.time()))
        m.setdefault("date", time.strftime("%Y-%m-%d_%H-%M-%S"))
        m.setdefault("done", False)
        m.setdefault("experiment_tag", t.trial_name)
        t.iteration = m.get("training_iteration", t.iteration)
        if path:
            t.latest_checkpoint = path
            t.ckpt_index = max(t.ckpt_index, int(os.path.basename(path).split("_")[-1]) + 1) \
                if os.path.basename(path).split("_")[-1].isdigit() else t.ckpt_index + 1
            m["checkpoint_dir_name"] = os.path.basename(path)
        t.last_result = m
        t.history.append(m)
        try:
            with open(os.path.join(t.local_path, "result.json"), "a") as f:
                f.write(json.dumps({k: v for k, v in m.items() if _jsonable(v)}) + "\n")
            flat = {k: v for k, v in _flatten(m).items() if _jsonable(v) and not isinstance(v, (list, dict))}
            newfile = t._csv_keys is None
            if newfile:
                t._csv_keys = list(flat.keys())
            with open(os.path.join(t.local_path, "progress.csv"), "a", newline="") as f:
                w = csv.DictWriter(f, fieldnames=t._csv_keys, extrasaction="ignore")
                if newfile:
                    w.writeheader()
                w.writerow(flat)
        except OSError:
            pass
        return m

    def _on_result(self, t: Trial, m: Dict) -> str:
        for cb in self.callbacks:
            if hasattr(cb, "on_trial_result"):
                cb.on_trial_result(iteration=t.iteration, trials=self.trials, trial=t, result=m)
        self.searcher.on_trial_result(t.trial_id, m)
        if self.stopper is not None and self.stopper(t.trial_id, m):
            return TrialScheduler.STOP
        if m.get("done"):
            return TrialScheduler.STOP
        return self.scheduler.on_trial_result(t, m)

    def _complete(self, t: Trial):
        self._stop_actor(t)
        t.status = Trial.TERMINATED
        self.scheduler.on_trial_complete(t, t.last_result)
        self.searcher.on_trial_complete(t.trial_id, dict(t.last_result, config=t.config))
        for cb in self.callbacks:
            if hasattr(cb, "on_trial_complete"):
                cb.on_trial_complete(iteration=t.iteration, trials=self.trials, trial=t)

    def _fail(self, t: Trial, err):
        self._stop_actor(t)
        t.num_failures += 1
        maxf = self.rc.failure_config.max_failures
        if maxf < 0 or t.num_failures <= maxf:
            t.status = Trial.PENDING  # relaunched from its latest checkpoint
            return
        t.status = Trial.ERROR
        t.error = err
        t.error_msg = str(err)
        try:
            with open(os.path.join(t.local_path, "error.txt"), "w") as f:
                f.write(str(err))
        except OSError:
            pass
        self.scheduler.on_trial_error(t)
        self.searcher.on_trial_complete(t.trial_id, None, error=True)
        for cb in self.callbacks:
            if hasattr(cb, "on_trial_error"):
                cb.on_trial_error(iteration=t.iteration, trials=self.trials, trial=t)
        if self.rc.failure_config.fail_fast:
            raise err

    def _step(self):
        from ..exceptions import RayActorError

        running = [t for t in self.trials if t.status == Trial.RUNNING]
        if not running:
            time.sleep(0.05)
            return
        for t in running:
            if t._poll_ref is None:
                t._poll_ref = t.actor.poll.remote(0.2)
        refs = [t._poll_ref for t in running]
        ready, _ = core.wait(refs, num_returns=1, timeout=1.0)
        ready_set = set(ready)
        for t in running:
            if t._poll_ref not in ready_set:
                continue
            ref, t._poll_ref = t._poll_ref, None
            try:
                reports, done, err = core.get(ref)
            except RayActorError as e:
                self._fail(t, e)
                continue
            except Exception as e:  # noqa
                self._fail(t, e)
                continue
            decision = TrialScheduler.CONTINUE
            for m, path in reports:
                m = self._record(t, m, path)
                decision = self._on_result(t, m)
                if decision != TrialScheduler.CONTINUE:
                    break
            if decision == TrialScheduler.STOP:
                self._complete(t)
            elif decision == TrialScheduler.PAUSE:
                self._stop_actor(t)
                if t.pending_exploit is not None:
                    src, new_cfg = t.pending_exploit
                    t.pending_exploit = None
                    dst = os.path.join(t.local_path, f"checkpoint_{t.ckpt_index:06d}")
                    shutil.copytree(src, dst, dirs_exist_ok=True)
                    t.latest_checkpoint = dst
                    t.ckpt_index += 1
                    t.config = new_cfg
                    t.status = Trial.PENDING
                else:
                    t.status = Trial.PAUSED
            elif err is not None:
                self._fail(t, err)
            elif done:
                if t.last_result:
                    t.last_result["done"] = True
                self._complete(t)

    def save_state(self, force=False):
        now = time.time()
        if not force and now - self._last_save < 2.0:
            return
        self._last_save = now
        st = {"trials": [t.to_state() for t in self.trials], "searcher_finished": self.searcher_finished,
              "time": now, "metric": self.metric, "mode": self.mode}
        tmp = os.path.join(self.exp_dir, ".experiment_state.json.tmp")
        with open(tmp, "w") as f:
            json.dump(st, f, default=str)
        os.replace(tmp, os.path.join(self.exp_dir, "experiment_state.json"))
        try:
            self.searcher.save(os.path.join(self.exp_dir, "searcher_state.pkl"))
        except Exception:
            pass
        if self.syncer is not None:
            try:
                self.syncer.sync(force=force)
            except Exception as e:  # storage hiccup: keep running, retry at the next save
                print(f"tune: syncing the experiment to storage failed: {e}", flush=True)

    def run(self):
        budget = self.tc.time_budget_s
        try:
            while True:
                self._fill()
                live = [t for t in self.trials if t.status in (Trial.RUNNING, Trial.PENDING)]
                if not live and self.searcher_finished:
                    break
                if not live and not self.searcher_finished:
                    # searcher returned None with no running trial: avoid a busy loop
                    time.sleep(0.05)
                self._step()
                self.save_state()
                stop_all = self.stopper is not None and self.stopper.stop_all()
                over = budget is not None and time.time() - self.start > _seconds(budget)
                if stop_all or over:
                    for t in self.trials:
                        if t.status in (Trial.RUNNING, Trial.PENDING, Trial.PAUSED):
                            self._complete(t)
                    break
        finally:
            for t in self.trials:
                if t.actor is not None:
                    self._stop_actor(t)
                    if t.status == Trial.RUNNING:
                        t.status = Trial.PAUSED
            self.save_state(force=True)
            for cb in self.callbacks:
                if hasattr(cb, "on_experiment_end"):
                    cb.on_experiment_end(trials=self.trials)
        return self.trials


def _seconds(x):
    return x.total_seconds() if hasattr(x, "total_seconds") else float(x)


class _TrialInfo:
    def __init__(self, trial_id, config):
        self.trial_id = trial_id
        self.config = config

    def __str__(self):
        return self.trial_id
