"""Function-trainable session used by Tune trials (reference:
python/ray/tune/trainable/function_trainable.py): ``train.report`` inside a
trial lands here."""
from __future__ import annotations

import threading

_tls = threading.local()
_global = None


def get():
    return getattr(_tls, "session", None) or _global


def set_session(s, global_=False):
    global _global
    _tls.session = s
    if global_:
        _global = s
