"""Node providers (reference: python/ray/autoscaler/node_provider.py — the
``NodeProvider`` interface — and _private/fake_multi_node/node_provider.py).

A provider creates/terminates machines; the autoscaler only talks to this
interface. :class:`LocalNodeProvider` launches node agents (``core.node_agent``,
exactly what ``start --address`` runs on a real machine) as local processes —
the fake multi-node provider used for tests and single-host elasticity.
Cloud / Kubernetes providers implement the same five methods.
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile
import threading
from typing import Dict, List, Optional

TAG_NODE_TYPE = "caamd-node-type"
TAG_NODE_KIND = "caamd-node-kind"
TAG_STATUS = "caamd-node-status"


class NodeProvider:
    """Interface: node ids are opaque strings; tags are str -> str."""

    def non_terminated_nodes(self, tag_filters: Dict[str, str]) -> List[str]:
        raise NotImplementedError

    def is_running(self, node_id: str) -> bool:
        raise NotImplementedError

    def node_tags(self, node_id: str) -> Dict[str, str]:
        raise NotImplementedError

    def create_node(self, node_config: dict, tags: Dict[str, str], count: int) -> List[str]:
        raise NotImplementedError

    def terminate_node(self, node_id: str) -> None:
        raise NotImplementedError

    def terminate_nodes(self, node_ids: List[str]) -> None:
        for n in node_ids:
            self.terminate_node(n)

    def head_node_id(self, node_id: str) -> str:
        """The id the head's node table uses for this provider node."""
        return node_id


class LocalNodeProvider(NodeProvider):
    """Launches ``core.node_agent`` processes on this host that join ``address``.
    The provider node id IS the cluster node id (passed as ``--node-id``)."""

    def __init__(self, address: str, log_dir: Optional[str] = None):
        self.address = address
        self.log_dir = log_dir or tempfile.mkdtemp(prefix="caamd-autoscaler-")
        self._procs: Dict[str, subprocess.Popen] = {}
        self._tags: Dict[str, Dict[str, str]] = {}
        self._lock = threading.Lock()

    def _env(self):
        from ..cluster_utils import _env

        return _env()

    def non_terminated_nodes(self, tag_filters: Dict[str, str]) -> List[str]:
        with self._lock:
            out = []
            for nid, p in self._procs.items():
                if p.poll() is not None:
                    continue
                tags = self._tags[nid]
                if all(tags.get(k) == v for k, v in tag_filters.items()):
                    out.append(nid)
            return out

    def is_running(self, node_id: str) -> bool:
        p = self._procs.get(node_id)
        return p is not None and p.poll() is None

    def node_tags(self, node_id: str) -> Dict[str, str]:
        return dict(self._tags.get(node_id, {}))

    def create_node(self, node_config: dict, tags: Dict[str, str], count: int) -> List[str]:
        res = dict(node_config.get("resources", {}))
        ids = []
        for _ in range(count):
            nid = os.urandom(16).hex()
            argv = [sys.executable, "-m", "cluster_anywhere_amd.core.node_agent", "--address", self.address,
                    "--node-id", nid, "--num-cpus", str(res.get("CPU", 1)),
                    "--num-gpus", str(int(res.get("GPU", 0))),
                    "--object-store-memory", str(int(node_config.get("object_store_memory", 128 << 20)))]
            custom = {k: v for k, v in res.items() if k not in ("CPU", "GPU", "memory")}
            if custom:
                import json

                argv += ["--resources", json.dumps(custom)]
            log = open(os.path.join(self.log_dir, f"node-{nid[:8]}.out"), "ab")
            p = subprocess.Popen(argv, env=self._env(), stdout=log, stderr=subprocess.STDOUT,
                                 stdin=subprocess.DEVNULL, start_new_session=True)
            log.close()
            with self._lock:
                self._procs[nid] = p
                self._tags[nid] = dict(tags)
            ids.append(nid)
        return ids

    def terminate_node(self, node_id: str) -> None:
        p = self._procs.get(node_id)
        if p is None or p.poll() is not None:
            return
        p.terminate()
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()

    def shutdown(self):
        for nid in list(self._procs):
            self.terminate_node(nid)
