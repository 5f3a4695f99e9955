"""``get_runtime_context()`` (reference: python/ray/runtime_context.py:16)."""
from __future__ import annotations

import os
from typing import Dict, List, Optional

from .core import context


class RuntimeContext:
    def __init__(self, worker):
        self._worker = worker

    def get_job_id(self) -> str:
        return self._worker.job_id.hex() if self._worker else ""

    @property
    def job_id(self):
        from .core.ids import JobID

        return JobID(self._worker.job_id)

    def get_node_id(self) -> str:
        return self._worker.node_hex if self._worker else ""

    @property
    def node_id(self):
        from .core.ids import NodeID

        return NodeID(bytes.fromhex(self.get_node_id()))

    def get_worker_id(self) -> str:
        return self._worker.worker_id.hex() if self._worker else ""

    def get_task_id(self) -> Optional[str]:
        ctx = context.current_task()
        return ctx.task_id.hex() if ctx else None

    def get_actor_id(self) -> Optional[str]:
        w = self._worker
        if w is not None and w.actor_id is not None:
            return w.actor_id.hex()
        return None

    def get_actor_name(self) -> Optional[str]:
        w = self._worker
        if w is not None and w.actor_id is not None:
            return (w.actor_opts or {}).get("name")
        return None

    @property
    def current_actor(self):
        from .core.actor import ActorHandle

        w = self._worker
        if w is None or w.actor_id is None:
            raise RuntimeError("This method is only available in an actor.")
        return ActorHandle(w.actor_id, (w.actor_opts or {}).get("handle_meta", {}))

    @property
    def namespace(self) -> str:
        return self._worker.namespace if self._worker else "default"

    def get_namespace(self) -> str:
        return self.namespace

    def get_placement_group_id(self) -> Optional[str]:
        ctx = context.current_task()
        if ctx is not None and ctx.pg:
            return ctx.pg[1].hex()
        return None

    @property
    def should_capture_child_tasks_in_placement_group(self) -> bool:
        ctx = context.current_task()
        return bool(ctx and ctx.pg and len(ctx.pg) > 3 and ctx.pg[3])

    def get_assigned_resources(self) -> Dict[str, float]:
        ctx = context.current_task()
        return dict(ctx.resources or {}) if ctx else {}

    def get_accelerator_ids(self) -> Dict[str, List[str]]:
        env = os.environ.get("CAAMD_GPU_IDS", "")
        return {"GPU": [x for x in env.split(",") if x]}

    def get_runtime_env_string(self) -> str:
        return os.environ.get("CAAMD_RUNTIME_ENV", "{}")

    @property
    def was_current_actor_reconstructed(self) -> bool:
        return False

    @property
    def gcs_address(self):
        return self._worker.address if self._worker else None

    def get(self):
        return {"job_id": self.get_job_id(), "node_id": self.get_node_id(),
                "task_id": self.get_task_id(), "actor_id": self.get_actor_id(),
                "namespace": self.namespace}


def get_runtime_context() -> RuntimeContext:
    from .core.api import _ensure_init

    _ensure_init()
    return RuntimeContext(context.worker)
