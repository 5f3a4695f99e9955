"""Task / actor option handling (reference: python/ray/_private/ray_option_utils.py)."""
from __future__ import annotations

from typing import Any, Dict

TASK_DEFAULTS = {
    "num_cpus": 1,
    "num_gpus": 0,
    "resources": None,
    "memory": None,
    "accelerator_type": None,
    "max_retries": 3,
    "retry_exceptions": False,
    "num_returns": 1,
    "scheduling_strategy": None,
    "placement_group": None,
    "placement_group_bundle_index": -1,
    "placement_group_capture_child_tasks": None,
    "runtime_env": None,
    "name": None,
    "max_calls": 0,
    "label_selector": None,
    "_metadata": None,
    # streaming generators: pause the producer once this many yielded items are
    # unconsumed (reference: remote_function.py:396)
    "_generator_backpressure_num_objects": None,
}

ACTOR_DEFAULTS = {
    "num_cpus": None,
    "num_gpus": 0,
    "resources": None,
    "memory": None,
    "accelerator_type": None,
    "max_restarts": 0,
    "max_task_retries": 0,
    "max_concurrency": None,
    "max_pending_calls": -1,
    "name": None,
    "namespace": None,
    "lifetime": None,
    "get_if_exists": False,
    "scheduling_strategy": None,
    "placement_group": None,
    "placement_group_bundle_index": -1,
    "placement_group_capture_child_tasks": None,
    "runtime_env": None,
    "concurrency_groups": None,
    "label_selector": None,
    "_metadata": None,
}


def validate(opts: Dict[str, Any], defaults: Dict[str, Any], what: str) -> Dict[str, Any]:
    for k in opts:
        if k not in defaults:
            raise ValueError(f"Invalid option keyword {k!r} for {what}")
    out = dict(defaults)
    out.update(opts)
    for k in ("num_cpus", "num_gpus", "memory"):
        v = out.get(k)
        if v is not None and (not isinstance(v, (int, float)) or v < 0):
            raise ValueError(f"{k} must be a non-negative number, got {v!r}")
    if out.get("runtime_env"):
        from .api import _check_runtime_env

        _check_runtime_env(out["runtime_env"])
    nr = out.get("num_returns")
    if nr is not None and not (nr in ("streaming", "dynamic") or (isinstance(nr, int) and nr >= 0)):
        raise ValueError(f"num_returns must be a non-negative int, 'streaming' or 'dynamic', got {nr!r}")
    return out


def resource_demand(o: Dict[str, Any], actor: bool = False) -> Dict[str, float]:
    d: Dict[str, float] = {}
    cpus = o.get("num_cpus")
    if cpus is None:
        cpus = 0 if actor else 1
    if cpus:
        d["CPU"] = float(cpus)
    if o.get("num_gpus"):
        d["GPU"] = float(o["num_gpus"])
    if o.get("memory"):
        d["memory"] = float(o["memory"])
    for k, v in (o.get("resources") or {}).items():
        if k in ("CPU", "GPU"):
            raise ValueError("Use num_cpus / num_gpus instead of resources={'CPU'/'GPU': ...}")
        d[k] = float(v)
    if o.get("accelerator_type"):
        d[f"accelerator_type:{o['accelerator_type']}"] = 0.001
    return d


def label_conditions(spec: Dict[str, Any]):
    """{key: In(..)|NotIn(..)|Exists()|DoesNotExist()|"v"|"!v"|"in(a,b)"|"!in(a,b)"}
    -> [(key, op, values)] with op 0 in, 1 not-in, 2 exists, 3 does-not-exist."""
    from ..util.scheduling_strategies import DoesNotExist, Exists, In, NotIn

    out = []
    for k, v in (spec or {}).items():
        if isinstance(v, In):
            out.append((k, 0, [str(x) for x in v.values]))
        elif isinstance(v, NotIn):
            out.append((k, 1, [str(x) for x in v.values]))
        elif isinstance(v, Exists) or v is Exists:
            out.append((k, 2, []))
        elif isinstance(v, DoesNotExist) or v is DoesNotExist:
            out.append((k, 3, []))
        elif isinstance(v, str):
            neg = v.startswith("!")
            body = v[1:] if neg else v
            if body.startswith("in(") and body.endswith(")"):
                vals = [x.strip() for x in body[3:-1].split(",") if x.strip()]
            else:
                vals = [body]
            out.append((k, 1 if neg else 0, vals))
        elif isinstance(v, (list, tuple, set)):
            out.append((k, 0, [str(x) for x in v]))
        else:
            raise ValueError(f"unsupported label condition {k}={v!r}")
    # hashable: the strategy tuple is part of the head's ready-queue key
    return tuple((k, op, tuple(vals)) for (k, op, vals) in out)


def strategy_tuple(o: Dict[str, Any]):
    st = _strategy_tuple(o)
    sel = o.get("label_selector")
    if sel:
        conds = label_conditions(sel)
        if st is None:
            return ("label", conds, ())
        if st[0] == "label":
            return ("label", tuple(st[1]) + conds, st[2])
        raise ValueError("label_selector cannot be combined with a placement-group / node-affinity strategy")
    return st


def _strategy_tuple(o: Dict[str, Any]):
    from ..util.scheduling_strategies import (NodeAffinitySchedulingStrategy,
                                              NodeLabelSchedulingStrategy,
                                              PlacementGroupSchedulingStrategy)
    from . import context

    st = o.get("scheduling_strategy")
    pg = o.get("placement_group")
    if pg is not None and pg != "default" and st is None:
        st = PlacementGroupSchedulingStrategy(pg, o.get("placement_group_bundle_index", -1),
                                              o.get("placement_group_capture_child_tasks"))
    if st is None or st == "DEFAULT":
        cur = context.current_pg()
        if cur is not None and len(cur) > 3 and cur[3]:
            return ("pg", cur[1], -1, True)
        return None
    if st == "SPREAD":
        return ("spread",)
    if isinstance(st, PlacementGroupSchedulingStrategy):
        if st.placement_group is None:
            return None
        bi = st.placement_group_bundle_index
        return ("pg", st.placement_group.id.binary(), None if bi is None or bi < 0 else bi,
                bool(st.placement_group_capture_child_tasks))
    if isinstance(st, NodeAffinitySchedulingStrategy):
        nid = st.node_id if isinstance(st.node_id, str) else st.node_id.hex()
        return ("node", nid, st.soft)
    if isinstance(st, NodeLabelSchedulingStrategy):
        return ("label", label_conditions(st.hard), label_conditions(st.soft))
    raise ValueError(f"unsupported scheduling strategy {st!r}")
