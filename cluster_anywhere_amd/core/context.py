"""Process-global runtime state: the connected CoreWorker (driver or worker) and
the task-execution context used by ``get_runtime_context()``."""
from __future__ import annotations

import threading

worker = None  # CoreWorker of this process, or None when not initialised
local_mode = False

_tls = threading.local()


class TaskContext:
    __slots__ = ("task_id", "actor_id", "fn_name", "attempt", "gpu_ids", "resources", "pg",
                 "actor_name", "cancelled")

    def __init__(self, **kw):
        for s in self.__slots__:
            setattr(self, s, kw.get(s))


def current_task() -> "TaskContext":
    return getattr(_tls, "ctx", None)


def set_current_task(ctx):
    _tls.ctx = ctx


# the placement-group strategy tuple of this process's actor (set at actor creation):
# its method calls -- including ones running on thread pools or event loops, which
# have no task context of their own -- belong to the actor's placement group
actor_pg = None


def current_pg():
    """``("pg", pg_id, bundle, capture)`` of the running task, else of this actor."""
    ctx = getattr(_tls, "ctx", None)
    if ctx is not None and getattr(ctx, "pg", None):
        return ctx.pg
    return actor_pg
