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


def _get_one(rows: List[Dict], key: str, id: str) -> Optional[Dict]:
    for r in rows:
        if r.get(key) == id:
            return r
    return None


def get_actor(id: str, **kw) -> Optional[Dict]:
    return _get_one(list_actors(), "actor_id", id)


def get_task(id: str, **kw) -> Optional[Dict]:
    """The task's record (latest attempt); None if the head no longer tracks it."""
    rows = [t for t in list_tasks() if t["task_id"] == id]
    return max(rows, key=lambda t: t.get("attempt", 0)) if rows else None


def get_node(id: str, **kw) -> Optional[Dict]:
    return _get_one(list_nodes(), "node_id", id)


def get_worker(id: str, **kw) -> Optional[Dict]:
    return _get_one(list_workers(), "worker_id", id)


def get_job(id: str, **kw) -> Optional[Dict]:
    return _get_one(list_jobs(), "job_id", id)


def get_placement_group(id: str, **kw) -> Optional[Dict]:
    return _get_one(list_placement_groups(), "placement_group_id", id)


def get_objects(id: str, **kw) -> List[Dict]:
    """Every record of object ``id`` (a list, as in the reference: one per copy)."""
    return [o for o in list_objects() if o["object_id"] == id]


def list_runtime_envs(filters=None, limit: int = 10000, detail: bool = False, **kw) -> List[Dict]:
    """Runtime envs the cluster has set up (or failed to): key, the env, nodes,
    workers running in it, success / error."""
    return _filter(_state("runtime_envs"), filters)[:limit]


def list_cluster_events(filters=None, limit: int = 10000, detail: bool = False, **kw) -> List[Dict]:
    """Node joins / deaths, actor deaths and restarts, job starts, worker crashes,
    OOM kills and infeasible tasks, oldest first (``time`` is epoch seconds)."""
    return _filter(_state("cluster_events"), filters)[:limit]


def _session_dir() -> Optional[str]:
    from ..core import context

    w = context.worker
    return getattr(w, "session_dir", None) if w is not None else None


def list_logs(node_id: Optional[str] = None, node_ip: Optional[str] = None, glob_filter: str = "*",
              **kw) -> Dict[str, List[str]]:
    """Log files of the session, grouped like the reference (``worker_out`` for
    task / actor worker logs, ``jobs``, ``head`` ...). This node's session
    directory is listed; logs of other nodes stay on those nodes."""
    import fnmatch
    import os

    d = _session_dir()
    out: Dict[str, List[str]] = collections.defaultdict(list)
    if not d or not os.path.isdir(d):
        return {}
    for root, _dirs, names in os.walk(d):
        for n in sorted(names):
            rel = os.path.relpath(os.path.join(root, n), d)
            if not n.endswith((".log", ".out", ".err")) or not fnmatch.fnmatch(rel, glob_filter):
                continue
            group = ("worker_out" if n.startswith("worker-") else
                     "jobs" if rel.startswith("jobs" + os.sep) else
                     "head" if "head" in n else "other")
            out[group].append(rel)
    return dict(out)


def get_log(filename: Optional[str] = None, *, actor_id: Optional[str] = None, task_id: Optional[str] = None,
            pid: Optional[int] = None, worker_id: Optional[str] = None, node_id: Optional[str] = None,
            tail: int = 1000, follow: bool = False, **kw):
    """Lines of one log file, as a generator: by ``filename`` (relative to the
    session directory), or the worker log of ``actor_id`` / ``task_id`` / ``pid``
    / ``worker_id``. ``tail`` = last N lines (-1: all); ``follow`` keeps yielding
    appended lines until the generator is closed."""
    import os
    import time as _time

    d = _session_dir()
    if not d:
        raise RuntimeError("get_log() needs init()")
    if filename is None:
        wid = worker_id
        if wid is None:
            if actor_id is not None:
                a = get_actor(actor_id)
                pid = a["pid"] if a else None
            elif task_id is not None:
                t = get_task(task_id)
                ev = [e for e in _state("events") if len(e) > 4 and e[0] == "start"
                      and getattr(e[1], "hex", lambda: e[1])() == task_id]
                pid = ev[-1][4] if ev else None
                if t is None and pid is None:
                    raise ValueError(f"unknown task {task_id}")
            if pid is None:
                raise ValueError("give filename, actor_id, task_id, pid or worker_id")
            w = next((w for w in list_workers() if w.get("pid") == pid), None)
            if w is None:
                raise ValueError(f"no worker with pid {pid}")
            wid = w["worker_id"]
        filename = f"worker-{wid[:8]}.log"
    path = os.path.realpath(os.path.join(d, filename))
    if not path.startswith(os.path.realpath(d) + os.sep) or not os.path.isfile(path):
        raise ValueError(f"no log file {filename!r} in the session directory")

    def gen():
        with open(path, errors="replace") as f:
            lines = f.readlines()
            for ln in (lines if tail is None or tail < 0 else lines[-tail:]):
                yield ln.rstrip("\n")
            while follow:
                ln = f.readline()
                if ln:
                    yield ln.rstrip("\n")
                else:
                    _time.sleep(0.2)

    return gen()


class StateApiClient:
    """Object form of the state API (reference: util/state/api.py:110): the same
    list / get / summarize calls as methods. ``address`` is accepted for parity;
    the client talks to the cluster this process is connected to."""

    def __init__(self, address: Optional[str] = None, cookies=None, headers=None):
        self.address = address

    def list(self, resource: str, options=None, raise_on_missing_output: bool = True, **kw) -> List[Dict]:
        fns = {"actors": list_actors, "tasks": list_tasks, "objects": list_objects, "nodes": list_nodes,
               "workers": list_workers, "placement_groups": list_placement_groups, "jobs": list_jobs,
               "runtime_envs": list_runtime_envs, "cluster_events": list_cluster_events}
        key = str(getattr(resource, "value", resource)).lower()
        if key not in fns:
            raise ValueError(f"unknown state resource {resource!r}; one of {sorted(fns)}")
        o = dict(options or {})
        o.update(kw)
        return fns[key](filters=o.get("filters"), limit=o.get("limit", 10000), detail=o.get("detail", False))

    def get(self, resource: str, id: str, options=None, **kw):
        fns = {"actors": get_actor, "tasks": get_task, "objects": get_objects, "nodes": get_node,
               "workers": get_worker, "placement_groups": get_placement_group, "jobs": get_job}
        key = str(getattr(resource, "value", resource)).lower()
        if key not in fns:
            raise ValueError(f"unknown state resource {resource!r}; one of {sorted(fns)}")
        return fns[key](id)

    def summary(self, resource: str, options=None, **kw) -> Dict[str, Any]:
        fns = {"tasks": summarize_tasks, "actors": summarize_actors, "objects": summarize_objects}
        key = str(getattr(resource, "value", resource)).lower()
        return fns[key]()

    def list_logs(self, node_id: Optional[str] = None, **kw):
        return list_logs(node_id=node_id, **kw)

    def get_log(self, **kw):
        return get_log(**kw)


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
