"""Remaining top-level names of the reference API (python/ray/__init__.py):
``Language``, ``LoggingConfig`` and the cross-language entry points. Workers
here are Python-only, so Java/C++ functions raise a clear error."""
from __future__ import annotations

import enum
import logging
from typing import Optional


class Language(enum.IntEnum):
    PYTHON = 0
    JAVA = 1
    CPP = 2


class LoggingConfig:
    """Worker/driver log format (reference: _private/ray_logging/logging_config.py)."""

    def __init__(self, encoding: str = "TEXT", log_level: str = "INFO",
                 additional_log_standard_attrs: Optional[list] = None):
        if encoding not in ("TEXT", "JSON"):
            raise ValueError("encoding must be 'TEXT' or 'JSON'")
        self.encoding, self.log_level = encoding, log_level
        self.additional_log_standard_attrs = list(additional_log_standard_attrs or [])

    def _apply(self):
        """Root logger level, and with ``encoding="JSON"`` a JSON-lines formatter
        on every root handler (a stderr handler is added when there is none)."""
        root = logging.getLogger()
        root.setLevel(self.log_level)
        if self.encoding != "JSON":
            return
        if not root.handlers:
            root.addHandler(logging.StreamHandler())
        fmt = _JsonFormatter(self.additional_log_standard_attrs)
        for h in root.handlers:
            h.setFormatter(fmt)

    def _to_env(self) -> str:
        import json

        return json.dumps({"encoding": self.encoding, "log_level": self.log_level,
                           "additional_log_standard_attrs": self.additional_log_standard_attrs})

    @staticmethod
    def _from_env(text: str) -> "LoggingConfig":
        import json

        return LoggingConfig(**json.loads(text))


class _JsonFormatter(logging.Formatter):
    """One JSON object per record: time, level, message, source location, the
    job / node / worker / actor / task ids of the process (reference:
    _private/ray_logging/formatters.py JSONFormatter) and any extra standard
    LogRecord attributes asked for."""

    def __init__(self, extra_attrs=()):
        super().__init__()
        self.extra_attrs = list(extra_attrs)

    def format(self, record: logging.LogRecord) -> str:
        import json

        out = {"asctime": self.formatTime(record), "levelname": record.levelname, "message": record.getMessage(),
               "filename": record.filename, "lineno": record.lineno, "name": record.name}
        try:
            from .runtime_context import get_runtime_context

            ctx = get_runtime_context()
            for key, fn in (("job_id", ctx.get_job_id), ("node_id", ctx.get_node_id),
                            ("worker_id", ctx.get_worker_id), ("actor_id", ctx.get_actor_id),
                            ("task_id", ctx.get_task_id)):
                try:
                    v = fn()
                except Exception:  # noqa: BLE001 - not in a task / not initialised
                    v = None
                if v:
                    out[key] = v
        except Exception:  # noqa: BLE001
            pass
        for a in self.extra_attrs:
            if hasattr(record, a):
                out[a] = getattr(record, a)
        if record.exc_info:
            out["exc_text"] = self.formatException(record.exc_info)
        return json.dumps(out, default=str)


def _cross_language(kind):
    def fn(*a, **k):
        raise NotImplementedError(f"{kind}: cross-language workers are not supported; "
                                  "this runtime's workers are Python processes")
    return fn


cpp_function = _cross_language("cpp_function")
java_function = _cross_language("java_function")
java_actor_class = _cross_language("java_actor_class")
