"""Replica / request context (reference: python/ray/serve/context.py)."""
from __future__ import annotations

import contextvars
from dataclasses import dataclass
from typing import Any, Optional


@dataclass
class ReplicaContext:
    app_name: str
    deployment: str
    replica_tag: str
    servable_object: Any = None

    @property
    def replica_id(self):
        return self.replica_tag


@dataclass
class RequestContext:
    route: str = ""
    request_id: str = ""
    app_name: str = ""
    multiplexed_model_id: str = ""


_replica_context: Optional[ReplicaContext] = None
_request_context: contextvars.ContextVar = contextvars.ContextVar("serve_request_context",
                                                                  default=RequestContext())


def _set_replica_context(ctx: ReplicaContext):
    global _replica_context
    _replica_context = ctx


def get_replica_context() -> ReplicaContext:
    if _replica_context is None:
        raise RuntimeError("get_replica_context() called outside a Serve replica")
    return _replica_context


def get_multiplexed_model_id() -> str:
    return _request_context.get().multiplexed_model_id
