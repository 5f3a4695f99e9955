"""Multi-node cluster on one machine (reference: python/ray/cluster_utils.py
Cluster + tests/test_multi_node*.py): a head with a TCP control endpoint plus
a separate node agent process with its own object store; tasks/actors placed
by resources, objects pulled node-to-node, node death detected."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import cluster_anywhere_amd as ray

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def two_nodes():
    ctx = ray.init(num_cpus=2, _listen_tcp="127.0.0.1:0")
    addr = ctx["gcs_address"]
    env = dict(os.environ, PYTHONPATH=ROOT)
    agent = subprocess.Popen([sys.executable, "-m", "cluster_anywhere_amd.core.node_agent", "--address", addr,
                              "--num-cpus", "2", "--num-gpus", "0", "--resources", '{"remote": 4}',
                              "--object-store-memory", str(256 << 20)], env=env)
    deadline = time.time() + 60
    while time.time() < deadline and sum(n["Alive"] for n in ray.nodes()) < 2:
        time.sleep(0.1)
    assert sum(n["Alive"] for n in ray.nodes()) == 2
    yield agent
    agent.kill()
    agent.wait()
    ray.shutdown()


@ray.remote(resources={"remote": 1})
def where(x=None):
    import numpy as np

    from cluster_anywhere_amd import get_runtime_context

    s = float(np.asarray(x).sum()) if x is not None else None
    return get_runtime_context().get_node_id(), s


@ray.remote(resources={"remote": 1})
def make_big(n):
    import numpy as np

    return np.arange(n, dtype=np.float64)


@ray.remote(resources={"remote": 1})
class Counter:
    def __init__(self):
        self.n = 0

    def add(self, arr):
        self.n += int(arr.sum())
        return self.n

    def node(self):
        from cluster_anywhere_amd import get_runtime_context

        return get_runtime_context().get_node_id()


def test_remote_node_tasks_and_objects(two_nodes):
    me = ray.get_runtime_context().get_node_id()
    nid, _ = ray.get(where.remote())
    assert nid != me
    assert ray.cluster_resources()["remote"] == 4
    big = np.ones(2_000_000)  # 16 MB: lives in the head node's store, pulled by the remote node
    ref = ray.put(big)
    nid, s = ray.get(where.remote(ref))
    assert nid != me and s == 2_000_000
    # object created on the remote node, pulled by the driver
    out = ray.get(make_big.remote(3_000_000))
    assert out.shape == (3_000_000,) and out[-1] == 2_999_999
    # remote -> remote (same node) and chained refs
    nid, s = ray.get(where.remote(make_big.remote(1000)))
    assert s == sum(range(1000))
    c = Counter.remote()
    assert ray.get(c.node.remote()) != me
    assert ray.get(c.add.remote(np.ones(500_000))) == 500_000


def test_node_death_detected(two_nodes):
    assert ray.get(where.remote())[0] != ray.get_runtime_context().get_node_id()
    two_nodes.kill()
    two_nodes.wait()
    deadline = time.time() + 30
    while time.time() < deadline and sum(n["Alive"] for n in ray.nodes()) > 1:
        time.sleep(0.1)
    assert sum(n["Alive"] for n in ray.nodes()) == 1
    # work that needs the dead node's resources cannot be placed any more
    r = where.remote()
    ready, _ = ray.wait([r], timeout=1.0)
    assert not ready


def _start_agent(addr):
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.Popen([sys.executable, "-m", "cluster_anywhere_amd.core.node_agent", "--address", addr,
                             "--num-cpus", "2", "--num-gpus", "0", "--resources", '{"remote": 4}',
                             "--object-store-memory", str(256 << 20)], env=env)


@ray.remote(resources={"remote": 1})
def plus_one(arr):
    return arr + 1


def test_lineage_reconstruction_after_node_death(two_nodes):
    """Objects whose only copy lived on a dead node are re-created by re-executing
    their lineage, including a lost intermediate argument whose own ref was dropped
    (reference: object_recovery_manager.cc, test_reconstruction*.py)."""
    me = ray.get_runtime_context().get_node_id()
    a = make_big.remote(1_000_000)            # 8 MB, lives in the remote node's store
    b = plus_one.remote(a)
    c = make_big.options(max_retries=0).remote(1_000_000)  # not recoverable
    ray.wait([b, c], num_returns=2, timeout=60)
    del a                                      # only b's lineage references a now
    assert ray.get(where.remote())[0] != me
    two_nodes.kill()
    two_nodes.wait()
    deadline = time.time() + 30
    while time.time() < deadline and sum(n["Alive"] for n in ray.nodes()) > 1:
        time.sleep(0.1)
    agent2 = _start_agent(ray.get_runtime_context().gcs_address)
    try:
        out = ray.get(b, timeout=90)
        assert out.shape == (1_000_000,) and out[0] == 1 and out[-1] == 1_000_000
        with pytest.raises(ray.exceptions.ObjectLostError):
            ray.get(c, timeout=30)
    finally:
        agent2.kill()
        agent2.wait()
