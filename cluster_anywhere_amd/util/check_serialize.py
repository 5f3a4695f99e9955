"""Find what makes an object unpicklable (reference: util/check_serialize.py
``inspect_serializability``): walks closures, referenced globals and attributes
down to the leaves that fail, and reports them."""
from __future__ import annotations

import inspect
from typing import Any, Optional, Set, Tuple

import cloudpickle


class FailureTuple:
    def __init__(self, obj: Any, name: str, parent: Any):
        self.obj, self.name, self.parent = obj, name, parent

    def __repr__(self):
        return f"FailTuple({self.name} [obj={self.obj!r}, parent={self.parent!r}])"


def _ok(obj) -> bool:
    try:
        cloudpickle.dumps(obj)
        return True
    except Exception:
        return False


def _members(obj):
    if inspect.isfunction(obj):
        cv = inspect.getclosurevars(obj)
        yield from cv.nonlocals.items()
        yield from cv.globals.items()
        return
    d = getattr(obj, "__dict__", None)
    if isinstance(d, dict):
        yield from d.items()
    if isinstance(obj, dict):
        yield from ((repr(k), v) for k, v in obj.items())
    elif isinstance(obj, (list, tuple, set, frozenset)):
        yield from ((f"[{i}]", v) for i, v in enumerate(obj))


def inspect_serializability(base_obj: Any, name: Optional[str] = None, depth: int = 3,
                            print_file=None) -> Tuple[bool, Set[FailureTuple]]:
    failures: Set[FailureTuple] = set()
    seen = set()

    def walk(obj, nm, parent, d):
        if id(obj) in seen:
            return
        seen.add(id(obj))
        if _ok(obj):
            return
        found = False
        if d > 0:
            for mn, mv in _members(obj):
                if not _ok(mv):
                    found = True
                    walk(mv, mn, obj, d - 1)
        if not found:
            failures.add(FailureTuple(obj, nm, parent))

    walk(base_obj, name or repr(base_obj)[:60], None, depth)
    if print_file is not None:
        for f in failures:
            print(f"Serialization failure: {f}", file=print_file)
    return not failures, failures
