"""Node-label scheduling (reference: python/ray/util/scheduling_strategies.py:135,
tests/test_node_label_scheduling_strategy.py): hard / soft conditions of
NodeLabelSchedulingStrategy and the ``label_selector`` option, enforced by the
native ClusterScheduler across a 3-node cluster."""
import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd.cluster_utils import Cluster
from cluster_anywhere_amd.util.scheduling_strategies import (DoesNotExist, Exists, In,
                                                             NodeLabelSchedulingStrategy, NotIn)


@pytest.fixture(scope="module")
def cluster():
    c = Cluster()
    c.add_node(num_cpus=2, labels={"zone": "a"})
    c.add_node(num_cpus=2, labels={"zone": "b", "gpu-kind": "mi355x"})
    c.add_node(num_cpus=2, labels={"zone": "c"})
    ray.init(address=c.address)
    c.wait_for_nodes()
    yield c
    ray.shutdown()
    c.shutdown()


@ray.remote(num_cpus=1)
def where():
    return ray.get_runtime_context().get_node_id()


def _zone_of(cluster):
    return {n["NodeID"]: n.get("Labels", {}).get("zone") for n in ray.nodes()}


def test_labels_visible(cluster):
    zones = sorted(z for z in _zone_of(cluster).values() if z)
    assert zones == ["a", "b", "c"]
    assert all("ray.io/node-id" in n["Labels"] for n in ray.nodes())


def test_hard_in_notin_exists(cluster):
    zone = _zone_of(cluster)
    st = NodeLabelSchedulingStrategy(hard={"zone": In("b")})
    assert {zone[n] for n in ray.get([where.options(scheduling_strategy=st).remote() for _ in range(6)])} == {"b"}
    st = NodeLabelSchedulingStrategy(hard={"zone": NotIn("a", "b")})
    assert {zone[n] for n in ray.get([where.options(scheduling_strategy=st).remote() for _ in range(6)])} == {"c"}
    st = NodeLabelSchedulingStrategy(hard={"gpu-kind": Exists()})
    assert {zone[n] for n in ray.get([where.options(scheduling_strategy=st).remote() for _ in range(4)])} == {"b"}
    st = NodeLabelSchedulingStrategy(hard={"gpu-kind": DoesNotExist(), "zone": In("a", "b", "c")})
    assert {zone[n] for n in ray.get([where.options(scheduling_strategy=st).remote() for _ in range(6)])} <= {"a", "c"}


def test_soft_preference_and_label_selector(cluster):
    zone = _zone_of(cluster)
    st = NodeLabelSchedulingStrategy(hard={"zone": In("a", "c")}, soft={"zone": In("c")})
    assert zone[ray.get(where.options(scheduling_strategy=st).remote())] == "c"
    assert zone[ray.get(where.options(label_selector={"zone": "a"}).remote())] == "a"
    assert zone[ray.get(where.options(label_selector={"zone": "!in(a,b)"}).remote())] == "c"


def test_unsatisfiable_is_infeasible(cluster):
    st = NodeLabelSchedulingStrategy(hard={"zone": In("nowhere")})
    r = where.options(scheduling_strategy=st).remote()
    ready, _ = ray.wait([r], timeout=1.0)
    assert not ready  # parked as infeasible, never runs on a non-matching node
    ray.cancel(r)


def test_actor_label_placement(cluster):
    zone = _zone_of(cluster)

    @ray.remote(num_cpus=1)
    class A:
        def node(self):
            return ray.get_runtime_context().get_node_id()

    a = A.options(scheduling_strategy=NodeLabelSchedulingStrategy(hard={"zone": In("b")})).remote()
    assert zone[ray.get(a.node.remote())] == "b"
