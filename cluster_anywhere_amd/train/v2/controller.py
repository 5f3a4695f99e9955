"""The v2 training controller: an explicit state machine over run attempts
(reference: python/ray/train/v2/_internal/execution/controller/controller.py:91,
controller/state.py). See the package docstring for the states."""
from __future__ import annotations

import enum
import logging
import os
import time
import uuid
from typing import Dict, List, Optional

from ..checkpoint import Checkpoint
from ..trainer import Result, TrainingFailedError, _WorkerGroup
from .failure_policy import DefaultFailurePolicy, FailureDecision, FailurePolicy
from .scaling_policy import NoopDecision, ResizeDecision, ScalingDecision, ScalingPolicy, create_scaling_policy

logger = logging.getLogger(__name__)


class TrainControllerStateType(enum.Enum):
    # (name, terminal, starts a new run attempt); the name keeps the values distinct
    # (equal enum values would alias the members)
    INITIALIZING = ("INITIALIZING", False, True)
    SCHEDULING = ("SCHEDULING", False, False)
    RESCHEDULING = ("RESCHEDULING", False, False)
    RUNNING = ("RUNNING", False, False)
    RESTARTING = ("RESTARTING", False, True)
    RESIZING = ("RESIZING", False, True)
    ERRORED = ("ERRORED", True, False)
    FINISHED = ("FINISHED", True, False)

    @property
    def is_terminal(self):
        return self.value[1]

    @property
    def needs_new_run_attempt(self):
        return self.value[2]


class TrainControllerState:
    def __init__(self, type_: TrainControllerStateType, scaling_decision: Optional[ScalingDecision] = None,
                 error: Optional[BaseException] = None):
        self.type = type_
        self.scaling_decision = scaling_decision
        self.error = error

    def is_terminal(self):
        return self.type.is_terminal

    def needs_new_run_attempt(self):
        return self.type.needs_new_run_attempt

    def __repr__(self):
        return f"TrainControllerState({self.type.name})"


class ControllerCallback:
    """Hooks on the control loop (reference: v2 ``ControllerCallback``)."""

    def after_controller_start(self):
        pass

    def after_controller_state_update(self, previous: TrainControllerState, current: TrainControllerState):
        pass

    def before_controller_execute_scaling_decision(self, decision: ScalingDecision):
        pass

    def before_controller_execute_failure_decision(self, decision: FailureDecision, errors: Dict[int, BaseException]):
        pass

    def before_controller_shutdown(self):
        pass


class TrainController:
    """Runs a ``DataParallelTrainer`` (or any subclass: TorchTrainer, ...) as a
    sequence of run attempts driven by the scaling and failure policies."""

    def __init__(self, trainer, scaling_policy: Optional[ScalingPolicy] = None,
                 failure_policy: Optional[FailurePolicy] = None, callbacks: Optional[List] = None,
                 health_check_interval_s: Optional[float] = None, max_reschedules: int = 60):
        self.trainer = trainer
        self.scaling_policy = scaling_policy or create_scaling_policy(trainer.scaling_config)
        self.failure_policy = failure_policy or DefaultFailurePolicy(trainer.run_config.failure_config)
        self.callbacks = [c for c in (callbacks or []) if isinstance(c, ControllerCallback)]
        self.health_check_interval_s = float(health_check_interval_s if health_check_interval_s is not None
                                             else os.environ.get("RAY_TRAIN_HEALTH_CHECK_INTERVAL_S", "0.1"))
        self.max_reschedules = max_reschedules
        self.state = TrainControllerState(TrainControllerStateType.INITIALIZING)
        self.state_history: List[str] = [self.state.type.name]
        self.run_attempt_id: Optional[str] = None
        self.worker_group: Optional[_WorkerGroup] = None
        self.num_workers = 0
        self.run_dir = None
        self.history: List[dict] = []
        self.kept: List[tuple] = []
        self.latest_ckpt: Optional[Checkpoint] = trainer.resume_from_checkpoint
        self.ckpt_index = 0
        self.error: Optional[BaseException] = None
        self._reschedules = 0
        self._last_poll = float("-inf")

    # ------------------------------------------------------------- bookkeeping
    def get_state(self) -> TrainControllerState:
        return self.state

    def _set_state(self, nxt: TrainControllerState):
        prev, self.state = self.state, nxt
        self.state_history.append(nxt.type.name)
        for cb in [self.scaling_policy] + self.callbacks:
            if hasattr(cb, "after_controller_state_update"):
                cb.after_controller_state_update(prev, nxt)

    def _harvest(self):
        """Fold the worker group's reports / checkpoints into the run's record."""
        wg = self.worker_group
        if wg is None:
            return
        self.history.extend(wg.history)
        for m, p in wg.ckpts:
            self.latest_ckpt = self.trainer._ckpt(p)
            self.kept = self.trainer._track_checkpoint(self.kept, m, p)
        self.ckpt_index = wg.ckpt_index
        wg.history, wg.ckpts = [], []

    def _shutdown_worker_group(self):
        if self.worker_group is not None:
            self._harvest()
            self.worker_group.shutdown()
            self.worker_group = None

    # ------------------------------------------------------------------- steps
    def _start_worker_group(self, decision: ResizeDecision) -> bool:
        wg = _WorkerGroup(self.trainer, self.run_dir, self.latest_ckpt, self.ckpt_index, decision.num_workers)
        self.worker_group = wg
        try:
            wg.start()
        except Exception as e:  # noqa: BLE001 - startup failures are retried (RESCHEDULING)
            logger.warning("worker group startup failed (%s); rescheduling", e)
            self._shutdown_worker_group()
            return False
        self.num_workers = decision.num_workers
        return True

    def _execute_scaling_decision(self, decision: ScalingDecision) -> TrainControllerState:
        for cb in self.callbacks:
            cb.before_controller_execute_scaling_decision(decision)
        if isinstance(decision, ResizeDecision):
            self._shutdown_worker_group()
            if self._start_worker_group(decision):
                self._reschedules = 0
                return TrainControllerState(TrainControllerStateType.RUNNING)
            self._reschedules += 1
            if self._reschedules > self.max_reschedules:
                return TrainControllerState(TrainControllerStateType.ERRORED,
                                            error=TrainingFailedError("could not schedule the worker group"))
            return TrainControllerState(TrainControllerStateType.RESCHEDULING)
        return TrainControllerState(TrainControllerStateType.RUNNING)

    def _poll(self):
        wait = self.health_check_interval_s - (time.monotonic() - self._last_poll)
        if wait > 0:
            time.sleep(wait)
        from ...exceptions import RayActorError

        try:
            finished, err = self.worker_group.poll(timeout=0.5)
        except RayActorError as e:  # a worker died outright
            finished, err = False, e
        self._last_poll = time.monotonic()
        return finished, ({0: err} if err is not None else {})

    def _execute_failure_decision(self, decision: FailureDecision, errors) -> TrainControllerState:
        for cb in self.callbacks:
            cb.before_controller_execute_failure_decision(decision, errors)
        first = next(iter(errors.values()))
        if decision == FailureDecision.RESTART:
            logger.warning("restarting the worker group after: %s", first)
            return TrainControllerState(TrainControllerStateType.RESTARTING, error=first)
        if decision == FailureDecision.RAISE:
            n = getattr(self.failure_policy, "total_failures", 1)
            err = TrainingFailedError(f"Training failed after {n} attempt(s): {first}")
            err.__cause__ = first if isinstance(first, BaseException) else None
            return TrainControllerState(TrainControllerStateType.ERRORED, error=err)
        return TrainControllerState(TrainControllerStateType.RUNNING)

    def _step(self) -> TrainControllerState:
        s, T = self.state, TrainControllerStateType
        if s.type in (T.INITIALIZING, T.RESCHEDULING, T.RESTARTING):
            if s.type == T.RESCHEDULING:
                time.sleep(min(5.0, 0.2 * self._reschedules))
            return TrainControllerState(T.SCHEDULING, self.scaling_policy.make_decision_for_non_running_worker_group())
        if s.type == T.SCHEDULING:
            return self._execute_scaling_decision(s.scaling_decision)
        if s.type == T.RESIZING:
            return TrainControllerState(T.SCHEDULING, s.scaling_decision)
        if s.type == T.RUNNING:
            finished, errors = self._poll()
            if errors:
                return self._execute_failure_decision(self.failure_policy.make_decision(errors), errors)
            if finished:
                self.worker_group.finish()
                return TrainControllerState(T.FINISHED)
            d = self.scaling_policy.make_decision_for_running_worker_group(self.num_workers)
            if isinstance(d, ResizeDecision):
                return TrainControllerState(T.RESIZING, d)
            return TrainControllerState(T.RUNNING)
        raise ValueError(f"unexpected controller state {s}")

    # -------------------------------------------------------------------- run
    def run(self) -> Result:
        from ...core import api as core

        core._ensure_init()
        self.run_dir = self.trainer._run_dir()
        for cb in self.callbacks:
            cb.after_controller_start()
        try:
            while not self.state.is_terminal():
                if self.state.needs_new_run_attempt():
                    self.run_attempt_id = uuid.uuid4().hex
                self._set_state(self._step())
        finally:
            self._shutdown_worker_group()
            for cb in self.callbacks:
                cb.before_controller_shutdown()
            self.trainer._write_history(self.run_dir, self.history)
        return self.get_result()

    def get_result(self) -> Result:
        last = self.history[-1] if self.history else {}
        err = self.state.error if self.state.type == TrainControllerStateType.ERRORED else None
        res = self.trainer._result(last, self.latest_ckpt, err, self.run_dir, self.history,
                                   [(self.trainer._ckpt(p), m) for m, p in self.kept])
        if err is not None:
            raise err
        return res

    def get_training_failed_error(self) -> Optional[BaseException]:
        return self.state.error if self.state.type == TrainControllerStateType.ERRORED else None
