"""Experimental APIs (reference: python/ray/experimental/): the internal KV
table and zero-copy GPU tensor hand-off between processes of one node
(``tensor_transport="ipc"``, see :mod:`.gpu_objects`)."""
from . import internal_kv  # noqa: F401
from .locations import get_local_object_locations, get_object_locations

__all__ = ["internal_kv", "get_object_locations", "get_local_object_locations"]
