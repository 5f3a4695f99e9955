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
* the head's session identity (session dir, node id, object-store arena name and
  size, control port): a standalone head restarted on the same storage while the
  arena still exists re-attaches to it and listens on the same addresses, so the
  node's workers, actors and drivers RECONNECT instead of dying (reference: raylets
  and core workers survive a GCS restart and re-register, gcs_server.cc:182
  DoStart(GcsInitData));
* every actor's creation record (not only detached ones): a re-registering actor
  worker is matched to its record and keeps running with its in-memory state;
  detached actors whose worker does not come back within the re-attach grace are
  re-created from their specs (same ids and names, state from ``__init__``), other
  actors are declared dead.

Creation specs that reference object-store arguments (``ObjectRef`` args) cannot
be re-created (those objects may not survive); such actors are persisted for
re-attachment only.
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

    def actor_put(self, spec, owner=None, lifetime=None) -> bool:
        restorable = not spec.arg_refs
        if not restorable and lifetime == "detached":
            log.warning("detached actor %s takes ObjectRef arguments: re-attachable after a head restart "
                        "but not re-creatable", spec.fn_name)
        fields = {s: getattr(spec, s) for s in spec.__slots__ if s not in _SPEC_RUNTIME_FIELDS}
        try:
            self.store.put("actor", spec.actor_id, pickle.dumps({"fields": fields, "owner": owner,
                                                                 "lifetime": lifetime,
                                                                 "restorable": restorable}))
        except Exception as e:  # noqa: BLE001
            log.warning("actor %s not persisted: %s", spec.fn_name, e)
            return False
        return True

    def session_put(self, info: dict):
        self.store.put("session", b"head", pickle.dumps(info))

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
        for k, rec in list(out["actor"].items()):
            if "fields" not in rec:  # pre-round-3 record: a detached actor's spec fields
                out["actor"][k] = {"fields": rec, "owner": None, "lifetime": "detached", "restorable": True}
        return out


def peek_session(path: str) -> Optional[dict]:
    """The session record a previous head wrote to ``path`` (None if none). Opens
    the log, reads and closes it, so the head can open it afterwards."""
    import os

    from .. import _native

    if not os.path.exists(path):
        return None
    st = _native.GcsStore(path)
    try:
        v = st.get("session", b"head")
        return pickle.loads(v) if v else None  # a record this module wrote itself
    finally:
        del st


def _kv_key(ns, key: bytes) -> bytes:
    """Namespace type tag (None / bytes / str) + length-prefixed namespace + key."""
    if ns is None:
        tag, raw = b"n", b""
    elif isinstance(ns, bytes):
        tag, raw = b"b", ns
    else:
        tag, raw = b"s", str(ns).encode()
    return tag + len(raw).to_bytes(4, "little") + raw + key
