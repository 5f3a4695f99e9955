"""``@remote`` functions (reference: python/ray/remote_function.py:41)."""
from __future__ import annotations

import inspect
from typing import Any, Dict

from . import context, options as opt_utils, serialization
from .head import NORMAL


class RemoteFunction:
    def __init__(self, fn, opts: Dict[str, Any]):
        if inspect.isclass(fn):
            raise TypeError("use ActorClass for classes")
        self._function = fn
        self._function_name = f"{fn.__module__}.{fn.__qualname__}"
        if "num_returns" not in opts and (inspect.isgeneratorfunction(fn)):
            opts = dict(opts, num_returns="streaming")
        self._options = opt_utils.validate(opts, opt_utils.TASK_DEFAULTS, "remote function")
        from .worker import function_id

        self._fn_id = function_id(fn)
        self._blob = None
        self.__doc__ = fn.__doc__
        self.__name__ = getattr(fn, "__name__", "remote_function")
        self.__wrapped__ = fn

    def __call__(self, *args, **kwargs):
        raise TypeError(
            f"Remote functions cannot be called directly. Instead of running "
            f"'{self.__name__}()', try '{self.__name__}.remote()'."
        )

    def options(self, **kw) -> "RemoteFunction":
        rf = RemoteFunction.__new__(RemoteFunction)
        rf.__dict__.update(self.__dict__)
        wf = kw.pop("_workflow_options", None)  # workflow.options(...) (workflow/api.py)
        if wf is not None:
            rf._workflow_opts = dict(getattr(self, "_workflow_opts", {}) or {}, **wf)
        merged = dict(self._options)
        merged.update(kw)
        rf._options = opt_utils.validate(merged, opt_utils.TASK_DEFAULTS, "remote function")
        return rf

    def _blob_fn(self):
        if self._blob is None:
            self._blob = serialization.dumps_function(self._function)
        return self._blob

    def remote(self, *args, **kwargs):
        from .api import _ensure_init

        _ensure_init()
        o = self._options
        if context.local_mode:
            from .local_mode import run_local_task

            return run_local_task(self._function, args, kwargs, o["num_returns"])
        w = context.worker
        w.register_function(self._fn_id, self._blob_fn)
        refs = w.submit(
            NORMAL, self._fn_id, o.get("name") or self._function_name, args, kwargs,
            num_returns=o["num_returns"], resources=opt_utils.resource_demand(o),
            strategy=opt_utils.strategy_tuple(o), max_retries=o["max_retries"],
            retry_exceptions=o["retry_exceptions"], runtime_env=o.get("runtime_env"),
            gen_bp=o.get("_generator_backpressure_num_objects"),
        )
        nr = o["num_returns"]
        if nr == "streaming":
            return refs
        if nr == "dynamic" or nr == 1:
            return refs[0]
        return refs

    def bind(self, *args, **kwargs):
        from ..dag import FunctionNode

        return FunctionNode(self, args, kwargs, dict(self._options))
