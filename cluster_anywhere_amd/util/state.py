"""State API (reference: python/ray/util/state/api.py): list / get / summarize
cluster entities from the head's tables."""
from __future__ import annotations

import collections
from typing import Any, Dict, List, Optional


def _state(what, arg=None):
    from ..core.api import _state as s

    return s(what, arg)


def _filter(rows, filters):
    if not filters:
        return rows
    out = []
    for r in rows:
        ok = True
        for (k, op, v) in filters:
            val = r.get(k)
            if op == "=" and str(val) != str(v):
                ok = False
            elif op == "!=" and str(val) == str(v):
                ok = False
        if ok:
            out.append(r)
    return out


def list_actors(filters=None, limit: int = 10000, detail: bool = False, **kw) -> List[Dict]:
    return _filter(_state("actors"), filters)[:limit]


def list_tasks(filters=None, limit: int = 10000, detail: bool = False, **kw) -> List[Dict]:
    return _filter(_state("tasks"), filters)[:limit]


def list_objects(filters=None, limit: int = 10000, detail: bool = False, **kw) -> List[Dict]:
    return _filter(_state("objects"), filters)[:limit]


def list_nodes(filters=None, limit: int = 10000, detail: bool = False, **kw) -> List[Dict]:
    rows = [{"node_id": n["NodeID"], "state": "ALIVE" if n["Alive"] else "DEAD",
             "node_ip": n["NodeManagerAddress"], "resources_total": n["Resources"],
             "is_head_node": n.get("local", False)} for n in _state("nodes")]
    return _filter(rows, filters)[:limit]


def list_workers(filters=None, limit: int = 10000, detail: bool = False, **kw) -> List[Dict]:
    return _filter(_state("workers"), filters)[:limit]


def list_placement_groups(filters=None, limit: int = 10000, detail: bool = False, **kw) -> List[Dict]:
    return _filter(_state("placement_groups"), filters)[:limit]


def list_jobs(filters=None, limit: int = 10000, detail: bool = False, **kw) -> List[Dict]:
    return _filter(_state("jobs"), filters)[:limit]


def get_actor(id: str) -> Optional[Dict]:
    for a in list_actors():
        if a["actor_id"] == id:
            return a
    return None


def summarize_tasks() -> Dict[str, Any]:
    c = collections.Counter((t["name"], t["state"]) for t in list_tasks())
    out: Dict[str, Dict[str, int]] = collections.defaultdict(dict)
    for (name, st), n in c.items():
        out[name][st] = n
    return {"cluster": {"summary": dict(out), "total_tasks": sum(c.values())}}


def summarize_actors() -> Dict[str, Any]:
    c = collections.Counter((a["class_name"], a["state"]) for a in list_actors())
    out: Dict[str, Dict[str, int]] = collections.defaultdict(dict)
    for (name, st), n in c.items():
        out[name][st] = n
    return {"cluster": {"summary": dict(out), "total_actors": sum(c.values())}}


def summarize_objects() -> Dict[str, Any]:
    objs = list_objects()
    return {"cluster": {"total_objects": len(objs),
                        "total_size_bytes": sum(o["size"] for o in objs),
                        "spilled": sum(1 for o in objs if o["spilled"])}}


def object_store_stats() -> Dict[str, int]:
    return _state("store")


def subscribe(channel: str, callback):
    """Subscribe to the head's state-change publisher (reference:
    src/ray/pubsub/publisher.h): ``channel`` "actor" delivers ``callback(actor_id,
    {"state", "name", "namespace", "class_name", "pid", "node", "death_cause"})`` on
    every actor state change, "node" delivers ``callback(node_id, {"state", ...})``
    when nodes join or die. Callbacks run on the driver's reader thread."""
    from ..core import context

    if context.worker is None:
        raise RuntimeError("subscribe() needs init()")
    context.worker.subscribe(channel, callback)


def unsubscribe(channel: str, callback):
    from ..core import context

    if context.worker is not None:
        context.worker.unsubscribe(channel, callback)
