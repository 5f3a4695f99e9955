"""``init(local_mode=True)``: run every task / actor method inline in the driver
(reference: LOCAL_MODE in python/ray/_private/worker.py), for debugging."""
from __future__ import annotations

import os

from .object_ref import ObjectRef

_values = {}
_actors = {}


class _LocalRef(ObjectRef):
    __slots__ = ()

    def __init__(self, id_bytes):
        self._id = id_bytes

    def __del__(self):
        pass


def reset_local():
    _values.clear()
    _actors.clear()


def _new(value, is_err=False):
    r = _LocalRef(os.urandom(24))
    _values[r.binary()] = (value, is_err)
    return r


def local_put(value):
    return _new(value)


def _resolve(a):
    if isinstance(a, ObjectRef):
        return local_get(a)
    return a


def local_get(refs):
    single = isinstance(refs, ObjectRef)
    out = []
    for r in ([refs] if single else refs):
        v, is_err = _values[r.binary()]
        if is_err:
            raise v
        out.append(v)
    return out[0] if single else out


def _call(fn, args, kwargs, num_returns):
    from ..exceptions import RayTaskError

    try:
        res = fn(*[_resolve(a) for a in args], **{k: _resolve(v) for k, v in kwargs.items()})
    except Exception as e:  # noqa
        err = RayTaskError.from_exception(getattr(fn, "__name__", "task"), e).as_instanceof_cause()
        n = 1 if num_returns in ("streaming", "dynamic") else num_returns
        refs = [_new(err, True) for _ in range(max(n, 1))]
        return refs[0] if n == 1 else refs
    if num_returns == "streaming":
        return iter([_new(x) for x in res])
    if num_returns == "dynamic":
        from .object_ref import DynamicObjectRefGenerator

        return _new(DynamicObjectRefGenerator([_new(x) for x in res]))
    if num_returns == 1:
        return _new(res)
    return [_new(x) for x in res]


def run_local_task(fn, args, kwargs, num_returns):
    return _call(fn, args, kwargs, num_returns)


def create_local_actor(cls, args, kwargs, meta):
    from .actor import ActorHandle

    aid = os.urandom(16)
    _actors[aid] = cls(*[_resolve(a) for a in args], **{k: _resolve(v) for k, v in kwargs.items()})
    return ActorHandle(aid, meta)


def run_local_method(actor_id, name, args, kwargs, num_returns):
    inst = _actors[actor_id]
    if name == "__ray_ready__":
        return _new(True)
    return _call(getattr(inst, name), args, kwargs, num_returns)
