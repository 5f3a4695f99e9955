"""Multi-node clusters on one machine for tests and development (reference:
python/ray/cluster_utils.py — ``Cluster`` :135, ``add_node`` :217,
``remove_node`` :260, ``wait_for_nodes`` :320).

The head is a standalone ``core.head_main`` process listening on TCP (its own
object store + object server); every ``add_node`` after the first starts a
``core.node_agent`` process (own shared-memory store, own worker pool) that
joins it — exactly the processes ``python -m cluster_anywhere_amd start
--head/--address`` launches on real nodes. ``connect()`` attaches this process
as a driver.
"""
from __future__ import annotations

import atexit
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class ClusterNode:
    def __init__(self, proc: subprocess.Popen, node_id: str, head: bool, log_path: str):
        self.proc = proc
        self.node_id = node_id
        self.head = head
        self.log_path = log_path

    @property
    def unique_id(self) -> str:
        return self.node_id

    def alive(self) -> bool:
        return self.proc.poll() is None

    def __repr__(self):
        return f"ClusterNode({'head' if self.head else 'worker'}, {self.node_id[:8]}, pid={self.proc.pid})"


def _env():
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return e


class Cluster:
    def __init__(self, initialize_head: bool = False, connect: bool = False,
                 head_node_args: Optional[dict] = None, shutdown_at_exit: bool = True):
        self._temp = tempfile.mkdtemp(prefix="caamd-cluster-")
        self.head_node: Optional[ClusterNode] = None
        self.worker_nodes: Dict[str, ClusterNode] = {}
        self.address: Optional[str] = None
        self.connected = False
        if shutdown_at_exit:
            atexit.register(self.shutdown)
        if initialize_head:
            self.add_node(**(head_node_args or {}))
            if connect:
                self.connect()

    @property
    def gcs_address(self) -> Optional[str]:
        return self.address

    def _node_args(self, num_cpus=None, num_gpus=None, resources=None, object_store_memory=None,
                   labels=None):
        argv = []
        if labels:
            argv += ["--labels", json.dumps(labels)]
        if num_cpus is not None:
            argv += ["--num-cpus", str(num_cpus)]
        argv += ["--num-gpus", str(0 if num_gpus is None else num_gpus)]
        if resources:
            argv += ["--resources", json.dumps(resources)]
        argv += ["--object-store-memory", str(object_store_memory or (256 << 20))]
        return argv

    def add_node(self, wait: bool = True, num_cpus=None, num_gpus=None, resources=None,
                 object_store_memory=None, labels=None, node_ip_address: str = None,
                 **_ignored) -> ClusterNode:
        args = self._node_args(num_cpus, num_gpus, resources, object_store_memory, labels)
        if node_ip_address and self.head_node is not None:
            args = [*args, "--node-ip-address", node_ip_address]
        if self.head_node is None:
            log = os.path.join(self._temp, "head.out")
            argv = [sys.executable, "-m", "cluster_anywhere_amd.core.head_main", "--port", "0",
                    "--host", "127.0.0.1", "--include-dashboard", "false", "--temp-dir", self._temp, *args]
            with open(log, "ab") as f:
                p = subprocess.Popen(argv, env=_env(), stdout=f, stderr=subprocess.STDOUT,
                                     stdin=subprocess.DEVNULL, start_new_session=True)
            info_path = os.path.join(self._temp, "head.json")
            deadline = time.time() + 120
            while time.time() < deadline:
                if os.path.exists(info_path):
                    try:
                        with open(info_path) as f:
                            info = json.load(f)
                        if info.get("pid") == p.pid:
                            break
                    except (OSError, ValueError):
                        pass
                if p.poll() is not None:
                    raise RuntimeError(f"head failed to start; see {log}")
                time.sleep(0.05)
            else:
                raise TimeoutError("head did not come up")
            self.address = info["address"]
            self.head_node = ClusterNode(p, info["node_id"], True, log)
            return self.head_node
        node_id = os.urandom(16).hex()
        log = os.path.join(self._temp, f"node-{node_id[:8]}.out")
        argv = [sys.executable, "-m", "cluster_anywhere_amd.core.node_agent", "--address", self.address,
                "--node-id", node_id, *args]
        with open(log, "ab") as f:
            p = subprocess.Popen(argv, env=_env(), stdout=f, stderr=subprocess.STDOUT,
                                 stdin=subprocess.DEVNULL, start_new_session=True)
        node = ClusterNode(p, node_id, False, log)
        self.worker_nodes[node_id] = node
        if wait:
            self._wait_joined(node)
        return node

    def _wait_joined(self, node: ClusterNode, timeout: float = 120.0):
        deadline = time.time() + timeout
        while time.time() < deadline:
            try:
                with open(node.log_path) as f:
                    if f"node {node.node_id} joined" in f.read():
                        return
            except OSError:
                pass
            if node.proc.poll() is not None:
                raise RuntimeError(f"node agent exited; see {node.log_path}")
            time.sleep(0.05)
        raise TimeoutError(f"node {node.node_id} did not join")

    def remove_node(self, node: ClusterNode, allow_graceful: bool = True):
        if node.alive():
            node.proc.terminate() if allow_graceful else node.proc.kill()
            try:
                node.proc.wait(timeout=10)
            except subprocess.TimeoutExpired:
                node.proc.kill()
                node.proc.wait()
        if node.head:
            self.head_node = None
        else:
            self.worker_nodes.pop(node.node_id, None)

    def list_all_nodes(self) -> List[ClusterNode]:
        return ([self.head_node] if self.head_node else []) + list(self.worker_nodes.values())

    def connect(self, namespace: Optional[str] = None):
        from .core import api

        ctx = api.init(address=self.address, namespace=namespace)
        self.connected = True
        return ctx

    def wait_for_nodes(self, timeout: float = 30.0):
        from .core import api

        want = len(self.list_all_nodes())
        deadline = time.time() + timeout
        while time.time() < deadline:
            if sum(1 for n in api.nodes() if n["Alive"]) >= want:
                return
            time.sleep(0.1)
        raise TimeoutError(f"timed out waiting for {want} nodes")

    def shutdown(self):
        if self.connected:
            from .core import api

            try:
                api.shutdown()
            except Exception:
                pass
            self.connected = False
        for n in list(self.worker_nodes.values()):
            self.remove_node(n)
        if self.head_node is not None:
            self.remove_node(self.head_node)
        shutil.rmtree(self._temp, ignore_errors=True)
