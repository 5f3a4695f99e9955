"""Client mode: ``init("ray://host:port")`` (reference: python/ray/client_builder.py,
python/ray/util/client/).

The reference runs a separate gRPC "client server" that hosts a proxy driver
per client. Here the head's TCP control endpoint already speaks the full driver
protocol, so a client is simply a driver that has **no local object store**: it
never maps the cluster's ``/dev/shm`` arenas (it may run on another machine).

* ``put`` ships the serialized value inline over the control connection (the
  head keeps it, like the reference's client-server copy);
* ``get`` of an object living in a node's store is pulled over TCP from that
  node's object server (the same path node agents use for node-to-node pulls);
* tasks, actors, placement groups, named actors, cancel/kill, wait — unchanged.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

from .core import context
from .core.worker import CoreWorker

PREFIX = "ray://"


class _NoStore:
    """Stands in for the shm arena on a client: nothing is ever local."""

    name = ""
    capacity = 0
    used = 0

    def get_pinned(self, oid):
        return None

    def create(self, *a):
        return -2

    def contains(self, oid):
        return False


class ClientCoreWorker(CoreWorker):
    def __init__(self, address: str, job_id: bytes):
        super().__init__(address, "driver", os.urandom(16),
                         node_hex="client:" + os.urandom(6).hex(), job_id=job_id,
                         extra={"client": True})
        self.is_client = True

    def _attach_store(self, store_name):
        return _NoStore()

    def _store(self, oid, so):
        return so.to_bytes(), so.total_bytes, None


def parse_address(address: str) -> str:
    if not address.startswith(PREFIX):
        raise ValueError(f"client addresses start with {PREFIX!r}, got {address!r}")
    hp = address[len(PREFIX):].rstrip("/")
    if ":" not in hp:
        hp += ":10001"
    return hp


def connect(address: str, namespace: Optional[str] = None, runtime_env: Optional[dict] = None) -> Dict[str, Any]:
    from .core import api

    hp = parse_address(address)
    job_id = os.urandom(4)
    cw = ClientCoreWorker(hp, job_id)
    if namespace:
        cw.namespace = namespace
    context.worker = cw
    info = {"address": address, "node_id": cw.node_hex, "session_dir": cw.session_dir,
            "namespace": cw.namespace, "job_id": job_id.hex(), "object_store_address": "",
            "webui_url": None, "gcs_address": hp, "client_mode": True}
    if runtime_env:
        info["runtime_env"] = runtime_env
    api._session.clear()
    api._session.update(info)
    return info


class ClientContext:
    def __init__(self, info: Dict[str, Any]):
        self._info = info
        self.dashboard_url = info.get("webui_url")
        self.python_version = "%d.%d.%d" % tuple(__import__("sys").version_info[:3])
        from . import __version__

        self.ray_version = __version__
        self.ray_commit = "n/a"
        self.protocol_version = "caamd-1"

    def __getitem__(self, k):
        return self._info[k]

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.disconnect()

    def disconnect(self):
        from .core.api import shutdown

        shutdown()


class ClientBuilder:
    """``client("ray://host:port").namespace(..).env(..).connect()``."""

    def __init__(self, address: Optional[str]):
        self.address = address or os.environ.get("RAY_ADDRESS") or ""
        if not self.address.startswith(PREFIX):
            self.address = PREFIX + self.address
        self._namespace = None
        self._env = None

    def namespace(self, namespace: str) -> "ClientBuilder":
        self._namespace = namespace
        return self

    def env(self, env: Dict[str, Any]) -> "ClientBuilder":
        self._env = env
        return self

    def connect(self) -> ClientContext:
        from .core.api import init

        return ClientContext(dict(init(self.address, namespace=self._namespace, runtime_env=self._env)))


def client(address: Optional[str] = None) -> ClientBuilder:
    return ClientBuilder(address)
