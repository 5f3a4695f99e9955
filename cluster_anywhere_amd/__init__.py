"""cluster_anywhere_amd — an MI355X-native distributed AI runtime with Ray's
capabilities (tasks / actors / objects, Train, Data, Tune, Serve, RLlib), built
on PyTorch-ROCm, hand-written gfx950 HIP kernels and RCCL over xGMI.

``import cluster_anywhere_amd as ray`` gives the familiar API surface
(reference: python/ray/__init__.py:176 ``__all__``). Importing the package does
NOT import torch, so CPU worker processes start in milliseconds; the GPU
subsystems (ops / models / parallel / train) import it lazily.
"""
import importlib as _importlib

__version__ = "0.1.0"

from . import exceptions  # noqa: E402
from .core.actor import ActorClass, ActorHandle, exit_actor, method  # noqa: E402
from .core.api import (  # noqa: E402
    LOCAL_MODE,
    SCRIPT_MODE,
    WORKER_MODE,
    available_resources,
    cancel,
    cluster_resources,
    free,
    get,
    get_actor,
    get_gpu_ids,
    init,
    is_initialized,
    kill,
    nodes,
    put,
    remote,
    show_in_dashboard,
    shutdown,
    timeline,
    wait,
)
from .core.ids import (  # noqa: E402
    ActorID,
    FunctionID,
    JobID,
    NodeID,
    ObjectID,
    PlacementGroupID,
    TaskID,
    UniqueID,
    WorkerID,
)
from .core.object_ref import DynamicObjectRefGenerator, ObjectRef, ObjectRefGenerator  # noqa: E402
from .runtime_context import get_runtime_context  # noqa: E402

_LAZY = {"train", "data", "tune", "serve", "rllib", "dag", "ops", "models", "parallel", "util",
         "air", "autoscaler", "dashboard", "job_submission", "workflow", "experimental", "llm",
         "cluster_utils", "scripts", "runtime_env", "job_config", "client_builder"}


def __getattr__(name):
    if name in _LAZY:
        mod = _importlib.import_module(f".{name}", __name__)
        globals()[name] = mod
        return mod
    if name == "JobConfig":
        from .job_config import JobConfig

        return JobConfig
    if name == "client":
        from .client_builder import client

        return client
    if name == "ClientBuilder":
        from .client_builder import ClientBuilder

        return ClientBuilder
    if name in ("Language", "LoggingConfig", "cpp_function", "java_function", "java_actor_class"):
        from . import _compat

        return getattr(_compat, name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


__all__ = [
    "__version__", "init", "shutdown", "is_initialized", "get", "put", "wait", "remote",
    "get_actor", "kill", "cancel", "free", "nodes", "cluster_resources", "available_resources",
    "get_gpu_ids", "timeline", "show_in_dashboard", "method", "exit_actor", "get_runtime_context",
    "ObjectRef", "ObjectRefGenerator", "DynamicObjectRefGenerator", "ActorClass", "ActorHandle",
    "ActorID", "JobID", "NodeID", "ObjectID", "TaskID", "WorkerID", "FunctionID",
    "PlacementGroupID", "UniqueID", "LOCAL_MODE", "SCRIPT_MODE", "WORKER_MODE", "exceptions",
]
