"""Custom serializers (reference: python/ray/util/serialization.py)."""
from __future__ import annotations

from typing import Any, Callable

from ..core import serialization as _ser


def register_serializer(cls: type, *, serializer: Callable[[Any], Any], deserializer: Callable[[Any], Any]):
    """Objects of exactly ``cls`` are pickled as ``deserializer(serializer(obj))``
    (the deserializer travels with the value, so workers need no registration)."""
    if not isinstance(cls, type):
        raise TypeError("register_serializer expects a class")
    _ser._CUSTOM[cls] = (serializer, deserializer)


def deregister_serializer(cls: type):
    _ser._CUSTOM.pop(cls, None)
