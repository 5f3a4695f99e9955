"""log_once helpers (reference: python/ray/util/debug.py)."""
from __future__ import annotations

import time

_logged = set()
_disabled = False
_periodic_interval = None
_last_periodic = 0.0


def log_once(key: str) -> bool:
    """True the first time ``key`` is seen (or every interval with periodic logging)."""
    global _last_periodic
    if _disabled:
        return False
    if key not in _logged:
        _logged.add(key)
        return True
    if _periodic_interval is not None and time.time() - _last_periodic > _periodic_interval:
        _last_periodic = time.time()
        _logged.clear()
        _logged.add(key)
        return True
    return False


def disable_log_once_globally():
    global _disabled
    _disabled = True


def enable_periodic_logging(interval_s: float = 60.0):
    global _periodic_interval
    _periodic_interval = interval_s
