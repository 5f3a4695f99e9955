"""Durable GCS tables for head fault tolerance.

Reference behaviour: with GCS fault tolerance on, the GCS writes its tables
(internal KV, function table, actor table, placement groups, jobs) through a
store client (``src/ray/gcs/store_client/redis_store_client.h:107``,
``gcs_table_storage.h``) so that a restarted GCS reloads them
(``gcs_server.cc`` ``GcsServer::Start`` -> ``GcsInitData::AsyncLoad``), and
detached actors / placement groups outlive their creators.

Here the head writes the same tables through the native append-only log store
(``csrc/runtime/gcs_store.cc``, exposed as ``_native.GcsStore``). A head started
with the same ``gcs_storage`` path restores:

* the internal KV (all namespaces) and the exported function table;
* job history;
* detached placement groups (re-reserved with their ids and names);
* detached actors: re-created from their creation specs with their actor ids,
  names and namespaces, so ``get_actor(name)`` resolves to the same actor id.
  Their worker processes died with the old head, so, as after any actor
  restart, in-memory actor state starts over from ``__init__``.

Creation specs that reference object-store arguments (``ObjectRef`` args) are
not persisted: those objects do not survive the head, so such detached actors
are not restorable (logged once at registration).
"""
from __future__ import annotations

import logging
import pickle
from typing import Any, Dict, Optional

log = logging.getLogger(__name__)

_SPEC_RUNTIME_FIELDS = ("node", "worker", "gpu_ids", "state", "submit_time", "start_time", "acquired",
                        "cancelled", "owner", "blocked", "pinned_refs")


class GcsPersistence:
    def __init__(self, path: str, fsync_each: bool = False):
        from .. import _native

        self.path = path
        self.store = _native.GcsStore(path, fsync_each)

    # ---------------------------------------------------------------- writes
    def kv_put(self, ns: str, key: bytes, value: bytes):
        self.store.put("kv", _kv_key(ns, key), value)

    def kv_del(self, ns: str, key: bytes):
        self.store.delete("kv", _kv_key(ns, key))

    def fn_put(self, fn_id: bytes, blob: bytes):
        self.store.put("fn", fn_id, blob)

    def job_put(self, job_id: bytes, info: dict):
        try:
            self.store.put("job", job_id or b"", pickle.dumps(info))
        except Exception:  # noqa: BLE001 - job info is best effort
            pass

    def actor_put(self, spec) -> bool:
        if spec.arg_refs:
            log.warning("detached actor %s takes ObjectRef arguments: not restorable after a head restart",
                        spec.fn_name)
            return False
        fields = {s: getattr(spec, s) for s in spec.__slots__ if s not in _SPEC_RUNTIME_FIELDS}
        try:
            self.store.put("actor", spec.actor_id, pickle.dumps(fields))
        except Exception as e:  # noqa: BLE001
            log.warning("detached actor %s not persisted: %s", spec.fn_name, e)
            return False
        return True

    def actor_del(self, actor_id: bytes):
        self.store.delete("actor", actor_id)

    def pg_put(self, pg_id: bytes, bundles, strategy: str, name: Optional[str], lifetime):
        self.store.put("pg", pg_id, pickle.dumps({"bundles": bundles, "strategy": strategy, "name": name,
                                                   "lifetime": lifetime}))

    def pg_del(self, pg_id: bytes):
        self.store.delete("pg", pg_id)

    def sync(self):
        self.store.sync()

    # ---------------------------------------------------------------- reads
    def load(self) -> Dict[str, Any]:
        kv = {}
        for k, v in self.store.items("kv"):
            n = int.from_bytes(k[1:5], "little")
            ns = k[5:5 + n]
            kv[({b"n": None, b"b": ns, b"s": None}[k[:1]] if k[:1] != b"s" else ns.decode(), k[5 + n:])] = v
        out = {"kv": kv, "fn": dict(self.store.items("fn")), "job": {}, "pg": {}, "actor": {}}
        for table in ("job", "pg", "actor"):
            for k, v in self.store.items(table):
                try:
                    out[table][k] = pickle.loads(v)  # records this module wrote itself
                except Exception as e:  # noqa: BLE001
                    log.warning("GCS %s record %s unreadable: %s", table, k.hex(), e)
        return out


def _kv_key(ns, key: bytes) -> bytes:
    """Namespace type tag (None / bytes / str) + length-prefixed namespace + key."""
    if ns is None:
        tag, raw = b"n", b""
    elif isinstance(ns, bytes):
        tag, raw = b"b", ns
    else:
        tag, raw = b"s", str(ns).encode()
    return tag + len(raw).to_bytes(4, "little") + raw + key
