"""Cluster-wide key/value store kept by the head (reference:
python/ray/experimental/internal_kv.py — ``_internal_kv_put/_get/_del/_exists/_list``;
the GCS ``InternalKV`` table). Keys and values are bytes (str is utf-8 encoded);
namespaces isolate users (collective groups, the autoscaler, jobs). In
``local_mode`` the table is a process-local dict."""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple, Union

_LOCAL: Dict[Tuple[bytes, bytes], bytes] = {}


def _b(x) -> bytes:
    if x is None:
        return b""
    return x.encode() if isinstance(x, str) else bytes(x)


def _local() -> bool:
    from ..core import context

    return context.local_mode


def _req(op: str, key, value=None, overwrite: bool = True, namespace=None):
    from ..core.api import _w

    w = _w()
    ns, k = _b(namespace), _b(key)
    v = None if value is None else _b(value)
    return w.request(lambda r: ("kv", r, op, ns, k, v, overwrite))


def _internal_kv_initialized() -> bool:
    from ..core.api import is_initialized

    return is_initialized()


def _internal_kv_put(key: Union[str, bytes], value: Union[str, bytes], overwrite: bool = True, *,
                     namespace: Optional[Union[str, bytes]] = None) -> bool:
    """Store ``value``; returns True if the key already existed."""
    if _local():
        k = (_b(namespace), _b(key))
        existed = k in _LOCAL
        if overwrite or not existed:
            _LOCAL[k] = _b(value)
        return existed
    return not _req("put", key, value, overwrite, namespace)


def _internal_kv_get(key: Union[str, bytes], *, namespace=None) -> Optional[bytes]:
    if _local():
        return _LOCAL.get((_b(namespace), _b(key)))
    return _req("get", key, namespace=namespace)


def _internal_kv_exists(key: Union[str, bytes], *, namespace=None) -> bool:
    if _local():
        return (_b(namespace), _b(key)) in _LOCAL
    return bool(_req("exists", key, namespace=namespace))


def _internal_kv_del(key: Union[str, bytes], *, del_by_prefix: bool = False, namespace=None) -> int:
    if _local():
        ns, k = _b(namespace), _b(key)
        gone = [kk for kk in _LOCAL if kk[0] == ns and (kk[1].startswith(k) if del_by_prefix else kk[1] == k)]
        for kk in gone:
            del _LOCAL[kk]
        return len(gone)
    k = _b(key) + (b"*" if del_by_prefix else b"")
    return int(_req("del", k, namespace=namespace) or 0)


def _internal_kv_list(prefix: Union[str, bytes], *, namespace=None) -> List[bytes]:
    if _local():
        ns, p = _b(namespace), _b(prefix)
        return [kk[1] for kk in _LOCAL if kk[0] == ns and kk[1].startswith(p)]
    return list(_req("keys", prefix, namespace=namespace) or [])
