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
        logging.getLogger().setLevel(self.log_level)


def _cross_language(kind):
    def fn(*a, **k):
        raise NotImplementedError(f"{kind}: cross-language workers are not supported; "
                                  "this runtime's workers are Python processes")
    return fn


cpp_function = _cross_language("cpp_function")
java_function = _cross_language("java_function")
java_actor_class = _cross_language("java_actor_class")
