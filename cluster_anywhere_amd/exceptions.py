"""Exception hierarchy (reference: python/ray/exceptions.py)."""
from __future__ import annotations

import traceback
from typing import Optional


class RayError(Exception):
    """Base of every framework error."""


class RaySystemError(RayError):
    pass


class TaskCancelledError(RayError):
    def __init__(self, task_id=None, error_message: Optional[str] = None):
        self.task_id = task_id
        self.error_message = error_message
        super().__init__(error_message or f"Task {task_id} was cancelled")


class RayTaskError(RayError):
    """Wraps an exception raised inside a remote task/actor method.

    ``ray.get`` re-raises it as an instance that is BOTH a RayTaskError and the
    original exception class (``except ValueError`` still works), exactly like
    the reference (exceptions.py:97 ``as_instanceof_cause``).
    """

    def __init__(self, function_name, traceback_str, cause=None, proctitle=None, pid=None, ip=None):
        self.function_name = function_name
        self.traceback_str = traceback_str
        self.cause = cause
        self.pid = pid
        self.ip = ip
        super().__init__(f"{function_name} failed:\n{traceback_str}")

    def __str__(self):
        return f"{type(self.cause).__name__ if self.cause else 'Error'} in {self.function_name}:\n{self.traceback_str}"

    def __reduce__(self):
        return (RayTaskError, (self.function_name, self.traceback_str, self.cause))

    def as_instanceof_cause(self):
        cause = self.cause
        if cause is None or isinstance(cause, RayTaskError):
            return self
        cause_cls = type(cause)
        try:
            name = f"RayTaskError({cause_cls.__name__})"
            cls = type(name, (RayTaskError, cause_cls), {})

            def __init__(s, fn, tb, c):
                RayTaskError.__init__(s, fn, tb, c)

            cls.__init__ = __init__
            cls.__reduce__ = lambda s: (RayTaskError, (s.function_name, s.traceback_str, s.cause))
            inst = cls(self.function_name, self.traceback_str, cause)
            inst.args = getattr(cause, "args", ())
            return inst
        except TypeError:
            return self

    @staticmethod
    def from_exception(fn_name: str, exc: BaseException) -> "RayTaskError":
        tb = "".join(traceback.format_exception(type(exc), exc, exc.__traceback__))
        try:
            import pickle

            pickle.dumps(exc)
            cause = exc
        except Exception:
            cause = RayError(f"{type(exc).__name__}: {exc}")
        return RayTaskError(fn_name, tb, cause)


class WorkerCrashedError(RayError):
    def __init__(self, msg="The worker died unexpectedly while executing this task."):
        super().__init__(msg)


class LocalRayletDiedError(RayError):
    pass


class RayActorError(RayError):
    def __init__(self, msg="The actor died unexpectedly before finishing this task.", actor_id=None):
        self.actor_id = actor_id
        super().__init__(msg)


class ActorDiedError(RayActorError):
    pass


class ActorUnavailableError(RayActorError):
    pass


class ActorUnschedulableError(RayError):
    pass


class TaskUnschedulableError(RayError):
    pass


class ObjectStoreFullError(RayError):
    pass


class OutOfMemoryError(RayError):
    pass


class OutOfDiskError(RayError):
    pass


class NodeDiedError(RayError):
    pass


class ObjectLostError(RayError):
    def __init__(self, object_ref_hex="", msg=None):
        self.object_ref_hex = object_ref_hex
        super().__init__(msg or f"Object {object_ref_hex} is lost")


class ObjectFreedError(ObjectLostError):
    pass


class OwnerDiedError(ObjectLostError):
    pass


class ObjectReconstructionFailedError(ObjectLostError):
    pass


class GetTimeoutError(RayError, TimeoutError):
    pass


class RuntimeEnvSetupError(RayError):
    pass


class TaskPlacementGroupRemoved(RayError):
    pass


class ActorPlacementGroupRemoved(RayError):
    pass


class PendingCallsLimitExceeded(RayError):
    pass


class AsyncioActorExit(RayError):
    pass


class ObjectRefStreamEndOfStreamError(RayError):
    pass


class RayChannelError(RaySystemError):
    pass


class RayChannelTimeoutError(RayChannelError, TimeoutError):
    pass


class CrossLanguageError(RayError):
    pass
