"""Function-trainable session used by Tune trials (reference:
python/ray/tune/trainable/function_trainable.py, train/_internal/session.py):
``tune.report`` / ``train.report`` inside a trial lands here."""
from __future__ import annotations

import os
import queue
import threading
import time
from typing import Any, Dict, Optional

_tls = threading.local()
_global = None


class StopTrial(BaseException):
    """Raised inside a trial's training thread when the controller stopped it."""


def get():
    return getattr(_tls, "session", None) or _global


def set_session(s, global_=False):
    global _global
    _tls.session = s
    if global_:
        _global = s


class TuneSession:
    def __init__(self, trial_id: str, trial_name: str, trial_dir: str, experiment_name: str,
                 checkpoint=None, iteration_start: int = 0, ckpt_index_start: int = 0,
                 storage_path: str = "", resources=None):
        from ..train.session import TrainContext

        self.trial_id = trial_id
        self.trial_dir = trial_dir
        self.checkpoint = checkpoint
        self.reports: "queue.Queue" = queue.Queue()
        # report() parks the trial until the controller has taken the result (the
        # reference's function trainable does the same: a trial never runs ahead of
        # its scheduler's decisions; function_trainable.py continue semaphore)
        self.consumed = threading.Event()
        self.iteration = iteration_start
        self.ckpt_index = ckpt_index_start
        self.start = time.time()
        self.last = self.start
        self.stop_requested = False
        self.resources = resources or {}
        self.context = TrainContext(1, 0, 0, 1, 0, experiment_name, trial_name, trial_id,
                                    storage_path, {}, trial_dir)

    def report(self, metrics: Dict[str, Any], checkpoint=None):
        if self.stop_requested:
            raise StopTrial()
        if not isinstance(metrics, dict):
            raise TypeError("report() expects a dict of metrics")
        from ..train.checkpoint import persist

        self.iteration += 1
        path = None
        if checkpoint is not None:
            dest = os.path.join(self.trial_dir, f"checkpoint_{self.ckpt_index:06d}")
            path = persist(checkpoint, dest).path
            self.ckpt_index += 1
        now = time.time()
        m = dict(metrics)
        m.setdefault("training_iteration", self.iteration)
        m.setdefault("time_this_iter_s", now - self.last)
        m.setdefault("time_total_s", now - self.start)
        self.last = now
        self.consumed.clear()
        self.reports.put((m, path))
        while not self.consumed.wait(0.5):
            if self.stop_requested:
                break
        if self.stop_requested:
            raise StopTrial()

    def get_checkpoint(self):
        return self.checkpoint


def report(metrics: Dict[str, Any], *, checkpoint=None):
    s = get()
    if s is None:
        from ..train import session as train_session

        return train_session.report(metrics, checkpoint=checkpoint)
    s.report(metrics, checkpoint)


def get_checkpoint():
    s = get()
    if s is None:
        from ..train import session as train_session

        return train_session.get_checkpoint()
    return s.checkpoint


def get_context():
    s = get()
    if s is None:
        from ..train import session as train_session

        return train_session.get_context()
    return s.context


def get_trial_id():
    return get_context().get_trial_id()


def get_trial_dir():
    return get_context().get_trial_dir()


def get_trial_resources():
    s = get()
    return s.resources if s is not None else {}
