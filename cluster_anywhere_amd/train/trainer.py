"""Trainers and the training worker group (reference: python/ray/train/
base_trainer.py, data_parallel_trainer.py:26, _internal/backend_executor.py:69,
_internal/worker_group.py:102).

``DataParallelTrainer.fit()``:
  1. reserves one placement-group bundle per worker (PACK by default, so a
     node's GPUs are used together and RCCL rings stay on xGMI),
  2. starts one ``_TrainWorker`` actor per bundle; GPU workers see every GPU
     of their node (device = their assigned id) so RCCL can use peer xGMI links,
  3. runs the backend's process-group setup (torch: ``init_process_group``
     over RCCL on GPUs / gloo on CPUs, 127.0.0.1 / node address rendezvous),
  4. runs ``train_loop_per_worker`` in every worker, streaming ``report()``ed
     metrics + persisted checkpoints back to the driver,
  5. on worker failure restarts the whole group from the latest checkpoint up
     to ``FailureConfig.max_failures`` times.

When the process is already one rank of a torch.distributed job
(``torchrun``/``python -m torch.distributed.run`` sets WORLD_SIZE / RANK), ``fit()``
runs the loop in-process on that rank ("SPMD mode") — same session, report and
checkpoint semantics, no actors.
"""
from __future__ import annotations

import json
import os
import shutil
import socket
import threading
import time
import traceback
import uuid
from typing import Any, Callable, Dict, List, Optional

from ..core import api as core
from .checkpoint import Checkpoint
from .config import CheckpointConfig, DataConfig, FailureConfig, RunConfig, ScalingConfig
from .session import TrainContext, _Session, init_session, shutdown_session


class TrainingFailedError(RuntimeError):
    pass


class Result:
    def __init__(self, metrics=None, checkpoint=None, error=None, path=None, metrics_history=None,
                 best_checkpoints=None):
        self.metrics = metrics or {}
        self.checkpoint = checkpoint
        self.error = error
        self.path = path
        self._history = metrics_history or []
        self.best_checkpoints = best_checkpoints or []
        self.filesystem = None

    @property
    def metrics_dataframe(self):
        import pandas as pd

        return pd.DataFrame(self._history)

    @property
    def config(self):
        return self.metrics.get("config")

    def __repr__(self):
        return f"Result(metrics={self.metrics}, path={self.path}, checkpoint={self.checkpoint}, error={self.error!r})"

    @classmethod
    def from_path(cls, path: str, storage_filesystem=None) -> "Result":
        """A finished run's result from its experiment directory (a local path, a
        URI, or a path inside ``storage_filesystem``)."""
        from .storage import StorageContext

        st = StorageContext(os.path.dirname(path.rstrip("/")) if not "://" in path else path.rstrip("/").rsplit("/", 1)[0],
                            os.path.basename(path.rstrip("/")), storage_filesystem)
        hist = []
        try:
            if st.local:
                with open(os.path.join(st.experiment_fs_path, "result.json")) as f:
                    text = f.read()
            else:
                with st.storage_filesystem.open_input_stream(st._join("result.json")) as f:
                    text = f.read().decode()
            hist = [json.loads(l) for l in text.splitlines() if l.strip()]
        except (OSError, FileNotFoundError):
            pass
        ckpts = st.list_checkpoints()
        fs = None if st.local else st.storage_filesystem
        ck = Checkpoint(st.checkpoint_fs_path(ckpts[-1]), filesystem=fs) if ckpts else None
        r = cls(hist[-1] if hist else {}, ck, None, st.experiment_fs_path, hist)
        r.filesystem = fs
        return r


class Backend:
    """Process-group hooks run inside every worker (reference: train/backend.py)."""

    def on_start(self, rank, world_size, master_addr, master_port, device_id):
        pass

    def on_shutdown(self):
        pass


def _free_port(host: str = "") -> int:
    s = socket.socket()
    s.bind((host, 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _TrainWorker:
    def __init__(self):
        self.thread = None
        self.session = None
        self.error = None
        self.done = False
        self.backend = None

    def node_info(self):
        gpus = [int(g) for g in os.environ.get("CAAMD_GPU_IDS", "").split(",") if g]
        # the rendezvous runs on rank 0's node: its address as the other nodes reach
        # it (reference: python/ray/train/torch/config.py:66 uses the rank-0 worker's
        # node IP as MASTER_ADDR)
        from ..util import get_node_ip_address

        return {"node_id": os.environ.get("CAAMD_NODE_ID", "local"), "gpu_ids": gpus,
                "port": _free_port(), "addr": get_node_ip_address(), "pid": os.getpid()}

    def setup(self, backend, rank, world_size, local_rank, local_world_size, node_rank,
              master_addr, master_port, device_id):
        os.environ.update({
            "RANK": str(rank), "WORLD_SIZE": str(world_size), "LOCAL_RANK": str(local_rank),
            "LOCAL_WORLD_SIZE": str(local_world_size), "NODE_RANK": str(node_rank),
            "MASTER_ADDR": master_addr, "MASTER_PORT": str(master_port),
            "HSA_ENABLE_IPC_MODE_LEGACY": "0",
        })
        self.backend = backend
        backend.on_start(rank, world_size, master_addr, master_port, device_id)
        return True

    def run(self, fn, config, ckpt_path, shards, ctx_kwargs, storage, ckpt_index, ckpt_fs=None):
        ckpt = Checkpoint(ckpt_path, filesystem=ckpt_fs) if ckpt_path else None
        self.session = _Session(TrainContext(**ctx_kwargs), ckpt, shards, storage, ckpt_index)
        init_session(self.session)

        def target():
            try:
                import inspect

                if len(inspect.signature(fn).parameters) == 0:
                    fn()
                else:
                    fn(config if config is not None else {})
            except BaseException as e:  # noqa
                from ..exceptions import RayTaskError

                self.error = RayTaskError.from_exception("train_loop_per_worker", e)
            finally:
                self.done = True

        self.thread = threading.Thread(target=target, name="train-loop", daemon=True)
        self.thread.start()
        return True

    def poll(self, timeout=0.5):
        out = []
        s = self.session
        deadline = time.time() + timeout
        while True:
            try:
                out.append(s.reports.get(timeout=max(0.0, min(0.05, deadline - time.time()))))
                while True:
                    out.append(s.reports.get_nowait())
            except Exception:
                pass
            if out or self.done or time.time() >= deadline:
                break
        done = self.done and s.reports.empty()
        return out, done, self.error

    def shutdown(self):
        try:
            if self.backend is not None:
                self.backend.on_shutdown()
        finally:
            shutdown_session()
        return True


class DataParallelTrainer:
    _default_backend = Backend

    def __init__(self, train_loop_per_worker: Callable, *, train_loop_config: Optional[Dict] = None,
                 backend_config: Optional[Backend] = None, scaling_config: Optional[ScalingConfig] = None,
                 run_config: Optional[RunConfig] = None, datasets: Optional[Dict[str, Any]] = None,
                 dataset_config: Optional[DataConfig] = None,
                 resume_from_checkpoint: Optional[Checkpoint] = None,
                 metadata: Optional[Dict[str, Any]] = None):
        self.train_loop_per_worker = train_loop_per_worker
        self.train_loop_config = train_loop_config
        self.backend = backend_config or self._default_backend()
        self.scaling_config = scaling_config or ScalingConfig(num_workers=1)
        self.run_config = run_config or RunConfig()
        self.datasets = datasets or {}
        self.dataset_config = dataset_config or DataConfig()
        self.resume_from_checkpoint = resume_from_checkpoint
        self.metadata = metadata or {}

    # ------------------------------------------------------------------ helpers
    def _run_dir(self):
        """Create the experiment directory on the run's storage (RunConfig
        storage_path / storage_filesystem, train/storage.py); returns its path there."""
        from .storage import StorageContext

        name = self.run_config.name or f"{type(self).__name__}_{time.strftime('%Y-%m-%d_%H-%M-%S')}"
        self.run_config.name = name
        self._storage = StorageContext(self.run_config.storage_path, name, self.run_config.storage_filesystem)
        return self._storage.create_experiment_dir()

    def _ckpt(self, path) -> Checkpoint:
        """A checkpoint persisted on the run's storage."""
        st = getattr(self, "_storage", None)
        return Checkpoint(path, filesystem=None if st is None or st.local else st.storage_filesystem)

    def _split_datasets(self, n):
        shards = [dict() for _ in range(n)]
        split = self.dataset_config.datasets_to_split
        for name, ds in self.datasets.items():
            if split == "all" or (isinstance(split, list) and name in split):
                parts = ds.streaming_split(n, equal=True) if hasattr(ds, "streaming_split") else [ds] * n
            else:
                parts = [ds] * n
            for i in range(n):
                shards[i][name] = parts[i]
        return shards

    @staticmethod
    def _spmd_env() -> bool:
        return "WORLD_SIZE" in os.environ and "RANK" in os.environ and not os.environ.get("CAAMD_WORKER_ID")

    # ---------------------------------------------------------------- SPMD mode
    def _fit_spmd(self) -> Result:
        rank = int(os.environ["RANK"])
        world = int(os.environ["WORLD_SIZE"])
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        run_dir = self._run_dir()
        ctx = TrainContext(world, rank, local_rank, int(os.environ.get("LOCAL_WORLD_SIZE", world)),
                           int(os.environ.get("GROUP_RANK", "0")), self.run_config.name,
                           self.run_config.name, "spmd", self.run_config.storage_path, self.metadata, run_dir)
        shards = self._split_datasets(world)[rank] if self.datasets else {}
        s = _Session(ctx, self.resume_from_checkpoint, shards, self._storage if rank == 0 else None, 0)
        init_session(s)
        history, last, ckpt = [], {}, None
        error = None
        try:
            import inspect

            fn = self.train_loop_per_worker
            if len(inspect.signature(fn).parameters) == 0:
                fn()
            else:
                fn(self.train_loop_config or {})
        except BaseException as e:  # noqa
            error = e
        finally:
            shutdown_session()
        while not s.reports.empty():
            _, m, p = s.reports.get()
            history.append(m)
            last = m
            if p:
                ckpt = self._ckpt(p)
        if error is not None:
            raise error
        return self._result(last, ckpt, None, run_dir, history)

    # ------------------------------------------------------------ actor mode
    def fit(self) -> Result:
        if self._spmd_env():
            return self._fit_spmd()
        if os.environ.get("RAY_TRAIN_V2_ENABLED", "0") == "1" or isinstance(self.scaling_config.num_workers,
                                                                            (tuple, list)):
            from .v2 import TrainController

            return TrainController(self).run()
        core._ensure_init()
        run_dir = self._run_dir()
        fc: FailureConfig = self.run_config.failure_config
        failures = 0
        latest_ckpt = self.resume_from_checkpoint
        history: List[dict] = []
        kept: List[tuple] = []
        ckpt_index = 0
        last_metrics: Dict[str, Any] = {}
        while True:
            try:
                res = self._run_attempt(run_dir, latest_ckpt, ckpt_index)
            except _AttemptFailed as af:
                history.extend(af.history)
                if af.history:
                    last_metrics = af.history[-1]
                for m, p in af.ckpts:
                    latest_ckpt = self._ckpt(p)
                    kept = self._track_checkpoint(kept, m, p)
                ckpt_index = af.ckpt_index
                failures += 1
                if fc.max_failures >= 0 and failures > fc.max_failures:
                    err = TrainingFailedError(f"Training failed after {failures} attempt(s): {af.error}")
                    err.__cause__ = af.error if isinstance(af.error, BaseException) else None
                    result = self._result(last_metrics, latest_ckpt, err, run_dir, history,
                                          [(self._ckpt(p), m) for m, p in kept])
                    self._write_history(run_dir, history)
                    raise err
                continue
            hist, ckpts, ckpt_index = res
            history.extend(hist)
            for m, p in ckpts:
                latest_ckpt = self._ckpt(p)
                kept = self._track_checkpoint(kept, m, p)
            if hist:
                last_metrics = hist[-1]
            break
        self._write_history(run_dir, history)
        return self._result(last_metrics, latest_ckpt, None, run_dir, history,
                            [(self._ckpt(p), m) for m, p in kept])

    def _result(self, *a) -> Result:
        r = Result(*a)
        st = getattr(self, "_storage", None)
        r.filesystem = None if st is None or st.local else st.storage_filesystem
        return r

    def _write_history(self, run_dir, history):
        text = "".join(json.dumps({k: v for k, v in m.items() if _jsonable(v)}) + "\n" for m in history)
        try:
            st = getattr(self, "_storage", None)
            if st is not None:
                st.write_text("result.json", text)
            else:
                with open(os.path.join(run_dir, "result.json"), "w") as f:
                    f.write(text)
        except OSError:
            pass

    def _track_checkpoint(self, kept, metrics, path):
        cc: CheckpointConfig = self.run_config.checkpoint_config
        kept = [k for k in kept if k[1] != path] + [(metrics, path)]
        if cc.num_to_keep is not None and len(kept) > cc.num_to_keep:
            attr = cc.checkpoint_score_attribute
            if attr:
                rev = cc.checkpoint_score_order == "max"
                order = sorted(kept, key=lambda x: x[0].get(attr, float("-inf") if rev else float("inf")),
                               reverse=rev)
            else:
                order = list(reversed(kept))
            keep, drop = order[: cc.num_to_keep], order[cc.num_to_keep:]
            latest = kept[-1]
            if latest not in keep:  # never delete the newest (needed for restore)
                drop = [d for d in drop if d is not latest]
                keep.append(latest)
            for m, p in drop:
                st = getattr(self, "_storage", None)
                if st is not None:
                    st.delete(p)
                else:
                    shutil.rmtree(p, ignore_errors=True)
            kept = [k for k in kept if k in keep]
        return kept

    def _run_attempt(self, run_dir, ckpt, ckpt_index):
        wg = _WorkerGroup(self, run_dir, ckpt, ckpt_index)
        try:
            wg.start()
            while True:
                finished, err = wg.poll()
                if err is not None:
                    raise _AttemptFailed(err, wg.history, wg.ckpts, wg.ckpt_index)
                if finished:
                    break
            wg.finish()
            return wg.history, wg.ckpts, wg.ckpt_index
        except _AttemptFailed:
            raise
        except Exception as e:
            from ..exceptions import RayActorError

            if isinstance(e, RayActorError):
                raise _AttemptFailed(e, wg.history, wg.ckpts, wg.ckpt_index)
            raise
        finally:
            wg.shutdown()


class _WorkerGroup:
    """One run attempt's worker group: placement group + one ``_TrainWorker`` actor
    per bundle, backend setup, the training function started on every rank, and a
    non-blocking ``poll()`` that streams reports / checkpoints back (used by the
    v1 ``fit()`` loop and by the v2 ``TrainController`` state machine)."""

    def __init__(self, trainer: "DataParallelTrainer", run_dir: str, ckpt, ckpt_index: int,
                 num_workers: Optional[int] = None):
        self.trainer = trainer
        self.run_dir, self.ckpt, self.ckpt_index = run_dir, ckpt, ckpt_index
        self.n = num_workers or trainer.scaling_config.total_workers
        self.workers: List[Any] = []
        self.pg = None
        self.history: List[dict] = []
        self.ckpts: List[tuple] = []
        self.done: List[bool] = []
        self.started_at = None

    def start(self):
        from ..core.actor import ActorClass
        from ..util.placement_group import placement_group, remove_placement_group
        from ..util.scheduling_strategies import PlacementGroupSchedulingStrategy

        sc = self.trainer.scaling_config
        n = self.n
        res = sc._resources_per_worker_not_none
        # bundle 0 reserves trainer_resources for the coordinator when it asks for any
        # (reference: air/config.py:156-161, as_placement_group_factory); the workers
        # take the bundles after it
        coord = sc._trainer_resources_not_none
        off = 1 if coord else 0
        bundles = ([dict(coord)] if coord else []) + [dict(res) for _ in range(n)]
        self.pg = pg = placement_group(bundles, strategy=sc.placement_strategy)
        ready, _ = core.wait([pg.ready()], timeout=float(os.environ.get("CAAMD_TRAIN_PG_TIMEOUT", "600")))
        if not ready:
            remove_placement_group(pg)
            self.pg = None
            raise RuntimeError(f"could not reserve {n} training workers with {res} each "
                               f"(cluster: {core.available_resources()})")
        Worker = ActorClass(_TrainWorker, {})
        for i in range(n):
            opts = dict(num_cpus=res.get("CPU", 1), num_gpus=res.get("GPU", 0),
                        resources={k: v for k, v in res.items() if k not in ("CPU", "GPU")},
                        scheduling_strategy=PlacementGroupSchedulingStrategy(pg, i + off),
                        runtime_env={"env_vars": {"CAAMD_NOSET_ROCR_VISIBLE_DEVICES": "1",
                                                  "HSA_ENABLE_IPC_MODE_LEGACY": "0"}})
            self.workers.append(Worker.options(**opts).remote())
        workers, tr = self.workers, self.trainer
        infos = core.get([w.node_info.remote() for w in workers], timeout=600)
        # ranks: group workers by node (node_rank order of first appearance)
        nodes = []
        for inf in infos:
            if inf["node_id"] not in nodes:
                nodes.append(inf["node_id"])
        local_counts = {nd: 0 for nd in nodes}
        local_world = {nd: sum(1 for x in infos if x["node_id"] == nd) for nd in nodes}
        master = infos[0]
        setups = []
        ranks = []
        for rank, (w, inf) in enumerate(zip(workers, infos)):
            nd = inf["node_id"]
            lr = local_counts[nd]
            local_counts[nd] += 1
            dev = inf["gpu_ids"][0] if inf["gpu_ids"] else None
            ranks.append((rank, lr, local_world[nd], nodes.index(nd)))
            setups.append(w.setup.remote(tr.backend, rank, n, lr, local_world[nd], nodes.index(nd),
                                         master["addr"], master["port"], dev))
        core.get(setups, timeout=900)
        shards = tr._split_datasets(n)
        runs = []
        for (rank, lr, lw, nr), w in zip(ranks, workers):
            ctx = dict(world_size=n, world_rank=rank, local_rank=lr, local_world_size=lw,
                       node_rank=nr, experiment_name=tr.run_config.name,
                       trial_name=tr.run_config.name, trial_id=uuid.uuid4().hex[:8],
                       storage_path=tr.run_config.storage_path, metadata=tr.metadata,
                       trial_dir=self.run_dir)
            runs.append(w.run.remote(tr.train_loop_per_worker, tr.train_loop_config,
                                     self.ckpt.path if self.ckpt else None, shards[rank], ctx,
                                     getattr(tr, "_storage", None), self.ckpt_index,
                                     getattr(self.ckpt, "filesystem", None) if self.ckpt else None))
        core.get(runs, timeout=600)
        self.done = [False] * n
        self.started_at = time.time()

    def poll(self, timeout: float = 0.5):
        """One poll round over every rank: (all finished, first error or None)."""
        polls = core.get([w.poll.remote(timeout) for w in self.workers])
        err = None
        round_reports = {}
        for i, (reports, d, e) in enumerate(polls):
            self.done[i] = d
            if e is not None and err is None:
                err = e
            for (rank, m, p) in reports:
                round_reports.setdefault(rank, []).append((m, p))
        # rank 0 metrics define the result; a checkpoint reported by any rank counts
        all_paths = {}
        for rank, items in round_reports.items():
            for k, (m, p) in enumerate(items):
                if p:
                    all_paths.setdefault(k, p)
        callbacks = self.trainer.run_config.callbacks or []
        for k, (m, p) in enumerate(round_reports.get(0, [])):
            path = p or all_paths.get(k)
            self.history.append(m)
            if path:
                self.ckpts.append((m, path))
                self.ckpt_index += 1
            for cb in callbacks:
                if hasattr(cb, "on_report_with_checkpoint"):
                    cb.on_report_with_checkpoint(m, path)
                elif hasattr(cb, "on_report"):
                    cb.on_report(m)
        return all(self.done), err

    def finish(self):
        core.get([w.shutdown.remote() for w in self.workers], timeout=60)

    def shutdown(self):
        from ..util.placement_group import remove_placement_group

        for w in self.workers:
            try:
                core.kill(w)
            except Exception:
                pass
        self.workers = []
        if self.pg is not None:
            remove_placement_group(self.pg)
            self.pg = None
        time.sleep(0.05)


class _AttemptFailed(Exception):
    def __init__(self, error, history, ckpts, ckpt_index):
        super().__init__(str(error))
        self.error = error
        self.history = history
        self.ckpts = ckpts
        self.ckpt_index = ckpt_index


def _jsonable(v):
    try:
        json.dumps(v)
        return True
    except TypeError:
        return False
