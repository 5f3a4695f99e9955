"""Per-worker training session: ``report`` / ``get_checkpoint`` / ``get_context`` /
``get_dataset_shard`` (reference: python/ray/train/_internal/session.py:112,
report :672, get_checkpoint :786, get_context, get_dataset_shard :1114)."""
from __future__ import annotations

import os
import queue
import threading
import time
from typing import Any, Dict, Optional

from .checkpoint import Checkpoint


class TrainContext:
    def __init__(self, world_size=1, world_rank=0, local_rank=0, local_world_size=1, node_rank=0,
                 experiment_name="", trial_name="", trial_id="", storage_path="", metadata=None,
                 trial_dir=""):
        self.world_size = world_size
        self.world_rank = world_rank
        self.local_rank = local_rank
        self.local_world_size = local_world_size
        self.node_rank = node_rank
        self.experiment_name = experiment_name
        self.trial_name = trial_name
        self.trial_id = trial_id
        self.storage_path = storage_path
        self.metadata = metadata or {}
        self.trial_dir = trial_dir

    def get_world_size(self):
        return self.world_size

    def get_world_rank(self):
        return self.world_rank

    def get_local_rank(self):
        return self.local_rank

    def get_local_world_size(self):
        return self.local_world_size

    def get_node_rank(self):
        return self.node_rank

    def get_experiment_name(self):
        return self.experiment_name

    def get_trial_name(self):
        return self.trial_name

    def get_trial_id(self):
        return self.trial_id

    def get_trial_dir(self):
        return self.trial_dir

    def get_metadata(self):
        return dict(self.metadata)

    def get_storage(self):
        return self.storage_path


class _Session:
    def __init__(self, ctx: TrainContext, checkpoint: Optional[Checkpoint], dataset_shards=None,
                 storage=None, ckpt_index_start: int = 0):
        self.ctx = ctx
        self.loaded_checkpoint = checkpoint
        self.dataset_shards = dataset_shards or {}
        # train/storage.py StorageContext (None: checkpoints stay where they are); a
        # plain directory string is accepted as a local storage root
        if isinstance(storage, str):
            from .storage import StorageContext

            storage = StorageContext(os.path.dirname(storage), os.path.basename(storage)) if storage else None
        self.storage = storage
        self.run_dir = storage.experiment_fs_path if storage is not None else ""
        self.reports: "queue.Queue" = queue.Queue()
        self.ckpt_index = ckpt_index_start
        self.iteration = 0
        self.start = time.time()
        self.stop_requested = False

    def report(self, metrics: Dict[str, Any], checkpoint: Optional[Checkpoint] = None,
               checkpoint_dir_name: Optional[str] = None):
        if not isinstance(metrics, dict):
            raise TypeError("report() expects a dict of metrics")
        self.iteration += 1
        persisted = None
        if checkpoint is not None:
            name = checkpoint_dir_name or f"checkpoint_{self.ckpt_index:06d}"
            if self.storage is not None:
                # upload from THIS worker's process: its directory may be node-local
                # (reference: StorageContext.persist_current_checkpoint)
                with checkpoint.as_directory() as local:
                    persisted = self.storage.persist_checkpoint(local, name)
            else:
                persisted = checkpoint.path
            self.ckpt_index += 1
        m = dict(metrics)
        m.setdefault("training_iteration", self.iteration)
        m.setdefault("time_total_s", time.time() - self.start)
        self.reports.put((self.ctx.world_rank, m, persisted))


_session: Optional[_Session] = None
_lock = threading.Lock()


def init_session(s: _Session):
    global _session
    _session = s


def get_session() -> Optional[_Session]:
    return _session


def shutdown_session():
    global _session
    _session = None


def report(metrics: Dict[str, Any], *, checkpoint: Optional[Checkpoint] = None,
           checkpoint_dir_name: Optional[str] = None) -> None:
    s = _session
    if s is None:
        # outside a trainer: also used by Tune function trainables
        from ..tune import session as tune_session

        if tune_session.get() is not None:
            return tune_session.get().report(metrics, checkpoint=checkpoint)
        raise RuntimeError("train.report() called outside of a training worker")
    s.report(metrics, checkpoint, checkpoint_dir_name)


def get_checkpoint() -> Optional[Checkpoint]:
    s = _session
    if s is None:
        from ..tune import session as tune_session

        ts = tune_session.get()
        return ts.checkpoint if ts is not None else None
    return s.loaded_checkpoint


def get_context() -> TrainContext:
    s = _session
    if s is None:
        from ..tune import session as tune_session

        ts = tune_session.get()
        if ts is not None:
            return ts.context
        return TrainContext()
    return s.ctx


def get_dataset_shard(dataset_name: Optional[str] = None):
    s = _session
    if s is None:
        return None
    if dataset_name is None:
        if len(s.dataset_shards) != 1:
            raise ValueError("specify dataset_name: the trainer has several datasets")
        return next(iter(s.dataset_shards.values()))
    return s.dataset_shards.get(dataset_name)
