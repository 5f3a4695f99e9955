"""Object locations (reference role: python/ray/experimental/locations.py)."""
from __future__ import annotations

from typing import Any, Dict, List


def _entry(ref, st, local_only) -> Dict[str, Any]:
    oid = ref.binary() if hasattr(ref, "binary") else bytes(ref)
    if oid in local_only:  # an inline result kept by its owner (this process)
        return {"node_ids": [], "object_size": local_only[oid][1], "did_spill": False}
    if st is None:
        return None
    return {"node_ids": list(st["node_ids"]), "object_size": st["size"], "did_spill": st["spilled"]}


def get_object_locations(obj_refs: List[Any], timeout_ms: int = -1) -> Dict[Any, Dict[str, Any]]:
    """{ref: {"node_ids", "object_size", "did_spill"}} for objects the cluster
    knows; inline (small) objects have no node. Refs whose lookup fails are left
    out."""
    from ..core import context
    from ..core.api import _state

    if context.worker is None:
        raise RuntimeError("get_object_locations() needs init()")
    local_only = getattr(context.worker.refs, "local_only", {})
    oids = [r.binary() for r in obj_refs]
    states = _state("object_locations", [o for o in oids if o not in local_only]) or {}
    out = {}
    for r, o in zip(obj_refs, oids):
        e = _entry(r, states.get(o), local_only)
        if e is not None:
            out[r] = e
    return out


def get_local_object_locations(obj_refs: List[Any]) -> Dict[Any, Dict[str, Any]]:
    """Like :func:`get_object_locations`; this process's view (its owner-local
    results plus what its node holds)."""
    from ..core import context

    out = get_object_locations(obj_refs)
    node = getattr(context.worker, "node_hex", None)
    return {r: (dict(e, node_ids=[n for n in e["node_ids"] if n == node]) if e["node_ids"] else e)
            for r, e in out.items()}
