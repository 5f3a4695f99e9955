"""Resource-demand autoscaler (reference: python/ray/autoscaler/_private/
autoscaler.py ``StandardAutoscaler``, resource_demand_scheduler.py,
monitor.py; config schema: ray-schema.json ``available_node_types``).

Every ``update()``:

1. reads the head's view (``state("autoscaler")``): resource shapes of queued
   and infeasible tasks/actors, bundles of pending placement groups, and each
   node's total / available resources and busy-worker count; plus the standing
   ``request_resources()`` bundles (internal KV);
2. bin-packs the demand onto the free capacity of live nodes and of nodes
   already launched but not yet joined; what does not fit is packed onto NEW
   nodes, choosing for each leftover shape the smallest configured node type
   that fits it (first-fit decreasing), within per-type and global
   ``max_workers`` and ``upscaling_speed``;
3. keeps every type at ``min_workers``;
4. terminates worker nodes idle (no busy worker, all resources free) for
   ``idle_timeout_minutes`` when no demand is pending, never below
   ``min_workers``.

Config (dict or YAML file)::

    {"max_workers": 8, "idle_timeout_minutes": 5, "upscaling_speed": 1.0,
     "available_node_types": {
        "cpu": {"resources": {"CPU": 16}, "min_workers": 0, "max_workers": 8},
        "mi355x": {"resources": {"CPU": 32, "GPU": 8}, "min_workers": 0, "max_workers": 4}}}
"""
from __future__ import annotations

import threading
import time
from typing import Dict, List, Optional, Tuple

from .node_provider import TAG_NODE_KIND, TAG_NODE_TYPE, NodeProvider

_IGNORE = ("memory", "object_store_memory")
KV_NS = "autoscaler"
KV_REQUEST = "request_resources"


def _fits(d: Dict[str, float], avail: Dict[str, float]) -> bool:
    return all(avail.get(k, 0.0) + 1e-9 >= v for k, v in d.items() if v > 0 and k not in _IGNORE)


def _take(avail: Dict[str, float], d: Dict[str, float]) -> None:
    for k, v in d.items():
        if k not in _IGNORE:
            avail[k] = avail.get(k, 0.0) - v


def _size(d: Dict[str, float]) -> Tuple[float, float]:
    return (d.get("GPU", 0.0), sum(v for k, v in d.items() if k not in _IGNORE))


def load_config(cfg) -> dict:
    if isinstance(cfg, str):
        import yaml

        with open(cfg) as f:
            cfg = yaml.safe_load(f)
    cfg = dict(cfg)
    cfg.setdefault("max_workers", 8)
    cfg.setdefault("idle_timeout_minutes", 5.0)
    cfg.setdefault("upscaling_speed", 1.0)
    types = cfg.get("available_node_types") or {}
    if not types:
        raise ValueError("autoscaler config needs available_node_types")
    for name, t in types.items():
        t.setdefault("min_workers", 0)
        t.setdefault("max_workers", cfg["max_workers"])
        if "resources" not in t:
            raise ValueError(f"node type {name!r} needs resources")
    return cfg


class StandardAutoscaler:
    def __init__(self, config, provider: NodeProvider, state_fn=None, kv_get=None):
        self.config = load_config(config)
        self.provider = provider
        self._state_fn = state_fn
        self._kv_get = kv_get
        self.idle_since: Dict[str, float] = {}
        self.last: dict = {}
        self.num_launched = 0
        self.num_terminated = 0

    # -- inputs ------------------------------------------------------------------
    def _state(self) -> dict:
        if self._state_fn is not None:
            return self._state_fn()
        from ..core.api import _state

        return _state("autoscaler")

    def _requested(self) -> List[Dict[str, float]]:
        if self._kv_get is not None:
            return self._kv_get() or []
        import json

        from ..experimental import internal_kv as kv

        v = kv._internal_kv_get(KV_REQUEST, namespace=KV_NS)
        return json.loads(v) if v else []

    # -- one reconcile round -----------------------------------------------------
    def update(self) -> dict:
        now = time.time()
        types = self.config["available_node_types"]
        st = self._state()
        nodes = st.get("nodes", {})
        demand = [dict(d) for d in st.get("demand", [])]
        for pg in st.get("pending_placement_groups", []):
            bundles = [dict(b) for b in pg["bundles"]]
            if pg.get("strategy") == "STRICT_PACK":
                merged: Dict[str, float] = {}
                for b in bundles:
                    for k, v in b.items():
                        merged[k] = merged.get(k, 0.0) + v
                demand.append(merged)
            else:
                demand.extend(bundles)

        workers = self.provider.non_terminated_nodes({TAG_NODE_KIND: "worker"})
        by_type: Dict[str, List[str]] = {t: [] for t in types}
        for n in workers:
            by_type.setdefault(self.provider.node_tags(n).get(TAG_NODE_TYPE, "?"), []).append(n)

        # free capacity: live nodes + launched-but-not-joined nodes (full type capacity)
        free: List[Dict[str, float]] = []
        totals: List[Dict[str, float]] = []
        for hexid, info in nodes.items():
            if info.get("alive"):
                free.append(dict(info.get("available", {})))
                totals.append(dict(info.get("total", {})))
        for n in workers:
            hid = self.provider.head_node_id(n)
            if hid not in nodes or not nodes[hid].get("alive"):
                r = dict(types.get(self.provider.node_tags(n).get(TAG_NODE_TYPE), {}).get("resources", {}))
                free.append(dict(r))
                totals.append(dict(r))

        leftover: List[Dict[str, float]] = []
        for d in sorted(demand, key=_size, reverse=True):
            for f in free:
                if _fits(d, f):
                    _take(f, d)
                    break
            else:
                leftover.append(d)
        # request_resources(): the cluster's TOTAL capacity must hold these bundles
        for d in sorted(self._requested(), key=_size, reverse=True):
            for t in totals:
                if _fits(d, t):
                    _take(t, d)
                    break
            else:
                leftover.append(d)

        # plan new nodes for the leftover shapes
        plan: Dict[str, int] = {t: 0 for t in types}
        planned: List[Tuple[str, Dict[str, float]]] = []
        infeasible: List[Dict[str, float]] = []
        total_workers = len(workers)
        for d in sorted(leftover, key=_size, reverse=True):
            for _, cap in planned:
                if _fits(d, cap):
                    _take(cap, d)
                    break
            else:
                cands = [(t, c) for t, c in types.items() if _fits(d, c["resources"])]
                cands.sort(key=lambda tc: _size(tc[1]["resources"]))
                chosen = None
                for t, c in cands:
                    if len(by_type.get(t, [])) + plan[t] < c["max_workers"] and \
                            total_workers + sum(plan.values()) < self.config["max_workers"]:
                        chosen = t
                        break
                if chosen is None:
                    infeasible.append(d)
                    continue
                plan[chosen] += 1
                cap = dict(types[chosen]["resources"])
                _take(cap, d)
                planned.append((chosen, cap))
        # min_workers
        for t, c in types.items():
            short = c["min_workers"] - len(by_type.get(t, [])) - plan[t]
            if short > 0:
                plan[t] += short
        launched: Dict[str, int] = {}
        for t, n in plan.items():
            if n <= 0:
                continue
            cur = len(by_type.get(t, []))
            limit = max(1, int(self.config["upscaling_speed"] * max(cur, 1))) if cur else n
            n = min(n, max(limit, types[t]["min_workers"] - cur))
            ids = self.provider.create_node(types[t], {TAG_NODE_KIND: "worker", TAG_NODE_TYPE: t}, n)
            launched[t] = len(ids)
            self.num_launched += len(ids)
            for i in ids:
                by_type.setdefault(t, []).append(i)

        # idle termination (only when nothing is waiting)
        terminated = []
        idle_s = float(self.config["idle_timeout_minutes"]) * 60.0
        for t, ids in by_type.items():
            for n in list(ids):
                info = nodes.get(self.provider.head_node_id(n))
                if not info or not info.get("alive"):
                    self.idle_since.pop(n, None)
                    continue
                tot, av = info.get("total", {}), info.get("available", {})
                idle = info.get("busy_workers", 0) == 0 and all(
                    av.get(k, 0.0) + 1e-9 >= v for k, v in tot.items() if k not in _IGNORE)
                if not idle:
                    self.idle_since.pop(n, None)
                    continue
                since = self.idle_since.setdefault(n, now)
                keep = types.get(t, {}).get("min_workers", 0)
                if (now - since >= idle_s and not leftover and not demand
                        and len(ids) > keep):
                    self.provider.terminate_node(n)
                    ids.remove(n)
                    terminated.append(n)
                    self.idle_since.pop(n, None)
                    self.num_terminated += 1
        self.last = {"time": now, "demand": demand, "leftover": leftover, "infeasible": infeasible,
                     "launched": launched, "terminated": terminated,
                     "workers": {t: len(v) for t, v in by_type.items()}}
        return self.last

    def summary(self) -> str:
        s = self.last or {}
        lines = ["======== Autoscaler status ========", "Node types:"]
        for t, n in (s.get("workers") or {}).items():
            lines.append(f"  {t}: {n} worker node(s)")
        lines.append(f"Pending demand: {len(s.get('demand', []))} shape(s), "
                     f"infeasible: {s.get('infeasible', [])}")
        lines.append(f"Launched total: {self.num_launched}, terminated total: {self.num_terminated}")
        return "\n".join(lines)


class Monitor:
    """Runs ``autoscaler.update()`` every ``interval_s`` on a daemon thread
    (reference: autoscaler/_private/monitor.py)."""

    def __init__(self, autoscaler: StandardAutoscaler, interval_s: float = 1.0):
        self.autoscaler = autoscaler
        self.interval_s = interval_s
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.errors: List[str] = []

    def start(self):
        self._thread = threading.Thread(target=self._run, name="caamd-autoscaler", daemon=True)
        self._thread.start()
        return self

    def _run(self):
        while not self._stop.is_set():
            try:
                self.autoscaler.update()
            except Exception as e:  # keep monitoring; surface the last errors
                self.errors = (self.errors + [repr(e)])[-10:]
            self._stop.wait(self.interval_s)

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=10)
