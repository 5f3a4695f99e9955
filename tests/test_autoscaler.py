"""Autoscaler (reference: python/ray/tests/test_autoscaler.py with mock providers,
test_autoscaler_fake_multinode.py with real node processes)."""
import time

import pytest

from cluster_anywhere_amd.autoscaler import NodeProvider, StandardAutoscaler, load_config
from cluster_anywhere_amd.autoscaler.node_provider import TAG_NODE_KIND, TAG_NODE_TYPE


class MockProvider(NodeProvider):
    def __init__(self):
        self.nodes = {}
        self.n = 0

    def non_terminated_nodes(self, tag_filters):
        return [k for k, v in self.nodes.items() if all(v.get(a) == b for a, b in tag_filters.items())]

    def is_running(self, node_id):
        return node_id in self.nodes

    def node_tags(self, node_id):
        return dict(self.nodes[node_id])

    def create_node(self, node_config, tags, count):
        ids = []
        for _ in range(count):
            self.n += 1
            nid = f"n{self.n}"
            self.nodes[nid] = dict(tags)
            ids.append(nid)
        return ids

    def terminate_node(self, node_id):
        self.nodes.pop(node_id, None)


CFG = {"max_workers": 5, "idle_timeout_minutes": 0.0,
       "available_node_types": {
           "small": {"resources": {"CPU": 2}, "max_workers": 3},
           "gpu": {"resources": {"CPU": 8, "GPU": 8}, "max_workers": 2}}}


def _scaler(state, requested=None, cfg=CFG):
    p = MockProvider()
    a = StandardAutoscaler(cfg, p, state_fn=lambda: state, kv_get=lambda: requested or [])
    return a, p


def test_config_validation():
    with pytest.raises(ValueError):
        load_config({"available_node_types": {}})
    c = load_config(CFG)
    assert c["available_node_types"]["small"]["min_workers"] == 0


def test_scale_up_picks_smallest_fitting_type_and_packs():
    head = {"h": {"alive": True, "total": {"CPU": 0}, "available": {"CPU": 0}, "busy_workers": 0}}
    state = {"demand": [{"CPU": 1}] * 3 + [{"GPU": 1, "CPU": 1}], "pending_placement_groups": [], "nodes": head}
    a, p = _scaler(state)
    r = a.update()
    # first-fit decreasing: the GPU task opens a gpu node, the 1-CPU tasks fill its CPUs
    assert r["launched"] == {"gpu": 1}
    # nodes launched but not joined count as capacity: no double launch
    assert a.update()["launched"] == {}
    a2, _ = _scaler({"demand": [{"CPU": 1}] * 3, "pending_placement_groups": [], "nodes": head})
    assert a2.update()["launched"] == {"small": 2}  # smallest type that fits, packed


def test_max_workers_and_infeasible():
    state = {"demand": [{"CPU": 2}] * 10 + [{"TPU": 1}], "pending_placement_groups": [], "nodes": {}}
    a, p = _scaler(state)
    r = a.update()
    assert sum(r["launched"].values()) <= 5
    assert r["launched"]["small"] == 3  # per-type cap
    assert {"TPU": 1} in r["infeasible"]


def test_placement_group_bundles_and_request_resources():
    state = {"demand": [], "nodes": {},
             "pending_placement_groups": [{"strategy": "STRICT_PACK", "bundles": [{"CPU": 4}, {"CPU": 3}]}]}
    a, p = _scaler(state)
    assert a.update()["launched"] == {"gpu": 1}  # 7 CPUs on one node: only the 8-CPU type fits
    a2, _ = _scaler({"demand": [], "nodes": {}, "pending_placement_groups": []}, requested=[{"CPU": 2}] * 2)
    assert a2.update()["launched"] == {"small": 2}


def test_idle_termination_respects_min_workers():
    cfg = dict(CFG)
    cfg["available_node_types"] = {"small": {"resources": {"CPU": 2}, "min_workers": 1, "max_workers": 3}}
    p = MockProvider()
    ids = p.create_node({}, {TAG_NODE_KIND: "worker", TAG_NODE_TYPE: "small"}, 3)
    nodes = {i: {"alive": True, "total": {"CPU": 2}, "available": {"CPU": 2}, "busy_workers": 0} for i in ids}
    nodes[ids[0]]["busy_workers"] = 1
    a = StandardAutoscaler(cfg, p, state_fn=lambda: {"demand": [], "pending_placement_groups": [],
                                                     "nodes": nodes}, kv_get=lambda: [])
    a.update()
    # two idle nodes, min_workers 1: both idle ones go (the busy one stays)
    assert p.non_terminated_nodes({}) == [ids[0]]


def test_local_provider_end_to_end(tmp_path):
    """Real node-agent processes: a head with no CPUs, tasks trigger scale-up,
    then the idle nodes are terminated."""
    import cluster_anywhere_amd as ray
    from cluster_anywhere_amd.autoscaler import LocalNodeProvider, Monitor
    from cluster_anywhere_amd.cluster_utils import Cluster

    cluster = Cluster(initialize_head=True, head_node_args={"num_cpus": 0})
    try:
        cluster.connect()
        prov = LocalNodeProvider(cluster.address, log_dir=str(tmp_path))
        cfg = {"max_workers": 2, "idle_timeout_minutes": 2.0 / 60,
               "available_node_types": {"w": {"resources": {"CPU": 2}, "max_workers": 2}}}
        mon = Monitor(StandardAutoscaler(cfg, prov), interval_s=0.5).start()

        @ray.remote(num_cpus=1)
        def f(i):
            time.sleep(0.5)
            return i

        assert sorted(ray.get([f.remote(i) for i in range(4)], timeout=120)) == [0, 1, 2, 3]
        assert mon.autoscaler.num_launched >= 1
        deadline = time.time() + 60
        while prov.non_terminated_nodes({}) and time.time() < deadline:
            time.sleep(0.5)
        assert prov.non_terminated_nodes({}) == []
        assert not mon.errors, mon.errors
        mon.stop()
    finally:
        cluster.shutdown()
