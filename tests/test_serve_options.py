"""Serve deployment options that change scheduling and admission (reference:
serve/_private/router.py:125-136 max_queued_requests -> BackPressureError,
proxy.py:143-147 / 1026-1053 request_timeout_s -> 408 and backpressure -> 503,
deployment_scheduler.py:143-176 per-replica placement groups and
max_replicas_per_node, api.py:438-454 _local_testing_mode; tests modelled on
serve/tests/test_backpressure.py, test_request_timeout.py,
test_replica_placement_group.py, test_max_replicas_per_node.py,
test_local_testing_mode.py)."""
import asyncio
import threading
import time
import urllib.error
import urllib.request

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import serve
from cluster_anywhere_amd.serve.exceptions import BackPressureError


def _get(port, path, timeout=30):
    try:
        with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=timeout) as r:
            return r.status, r.read()
    except urllib.error.HTTPError as e:
        return e.code, e.read()


@pytest.fixture
def one_node():
    ray.init(num_cpus=8)
    yield
    serve.shutdown()
    ray.shutdown()


def test_config_validation():
    with pytest.raises(ValueError, match="max_replicas_per_node is not allowed"):
        serve.deployment(max_replicas_per_node=1, placement_group_bundles=[{"CPU": 1}])(lambda r: r)
    with pytest.raises(ValueError):
        serve.deployment(max_replicas_per_node=0)(lambda r: r)
    with pytest.raises(ValueError):
        serve.deployment(max_queued_requests=0)(lambda r: r)
    with pytest.raises(ValueError):
        serve.deployment(placement_group_bundles=[{"CPU": 1}], placement_group_strategy="BOGUS")(lambda r: r)


@serve.deployment(max_ongoing_requests=1, max_queued_requests=2)
class Gate:
    """Each request waits until the test opens the gate (a named signal actor)."""

    def __init__(self):
        self.calls = 0

    async def __call__(self, request=None):
        self.calls += 1
        sig = ray.get_actor("gate_signal")
        while not await sig.is_open.remote():
            await asyncio.sleep(0.02)
        return "ok"


@ray.remote(num_cpus=0)
class Signal:
    def __init__(self):
        self.open = False

    def set(self, v):
        self.open = v

    def is_open(self):
        return self.open


def test_max_queued_requests_backpressure_handle_and_http(one_node):
    sig = Signal.options(name="gate_signal").remote()
    serve.start(http_options={"port": 0})
    h = serve.run(Gate.bind(), name="gate", route_prefix="/gate")
    port = serve.http_port()
    # handle side: 1 running (max_ongoing_requests=1) + 2 queued; the 4th is rejected
    first = h.remote()
    deadline = time.time() + 10
    from cluster_anywhere_amd.serve.handle import _router

    r = _router("gate", "Gate")
    queued = [h.remote(), h.remote()]
    assert r.num_queued() == 2
    with pytest.raises(BackPressureError) as ei:
        h.remote()
    assert ei.value.max_queued_requests == 2 and "backpressure" in str(ei.value)
    # HTTP side: the proxy has its own router; fill its slot and queue, the next is a 503
    results = {}

    def call(i):
        results[i] = _get(port, "/gate")

    ts = [threading.Thread(target=call, args=(i,)) for i in range(3)]
    for t in ts:
        t.start()
        time.sleep(0.3)  # 1 running + 2 queued at the proxy router
    code, body = _get(port, "/gate")
    assert code == 503 and b"backpressure" in body
    ray.get(sig.set.remote(True))
    for t in ts:
        t.join(30)
    assert all(results[i] == (200, b"ok") for i in range(3)), results
    assert first.result(timeout_s=30) == "ok"
    assert [q.result(timeout_s=30) for q in queued] == ["ok", "ok"]
    assert time.time() < deadline + 60


@serve.deployment(max_ongoing_requests=1)
class Slow:
    def __init__(self):
        self.started = 0
        self.finished = 0

    async def __call__(self, request):
        self.started += 1
        await asyncio.sleep(float(request.query_params.get("s", "0")))
        self.finished += 1
        return "done"

    def counts(self):
        return self.started, self.finished


def test_http_request_timeout_408_and_cancel(one_node):
    serve.start(http_options={"port": 0, "request_timeout_s": 0.5})
    h = serve.run(Slow.bind(), name="slow", route_prefix="/slow")
    port = serve.http_port()
    assert _get(port, "/slow?s=0") == (200, b"done")
    t0 = time.time()
    code, body = _get(port, "/slow?s=5")
    assert code == 408 and b"timed out after 0.5s" in body
    assert time.time() - t0 < 4
    # the replica call was cancelled: it never finishes its 5 s sleep
    time.sleep(1.0)
    started, finished = h.counts.remote().result(timeout_s=30)
    assert started == 2 and finished == 1
    # the proxy router's slot came back: a fast request still gets through
    assert _get(port, "/slow?s=0") == (200, b"done")


@serve.deployment(placement_group_bundles=[{"CPU": 1}, {"CPU": 2}], placement_group_strategy="PACK",
                  ray_actor_options={"num_cpus": 1}, num_replicas=2)
class Ganged:
    def __call__(self):
        from cluster_anywhere_amd.util import get_current_placement_group

        pg = get_current_placement_group()
        return pg.id.hex() if pg is not None else None

    def child_in_pg(self):
        @ray.remote(num_cpus=2)
        def where():
            from cluster_anywhere_amd.util import get_current_placement_group

            pg = get_current_placement_group()
            return pg.id.hex() if pg is not None else None

        return ray.get(where.remote())


def test_replica_placement_group(one_node):
    from cluster_anywhere_amd.util.state import list_placement_groups

    h = serve.run(Ganged.bind(), name="gang", route_prefix=None)
    pgs = {h.remote().result(timeout_s=30) for _ in range(20)}
    assert len(pgs) == 2 and None not in pgs  # one gang per replica
    rows = [p for p in list_placement_groups() if p.get("name", "").startswith("SERVE_REPLICA_PG::")]
    live = [p for p in rows if p.get("state") != "REMOVED"]
    assert len(live) == 2
    assert all(len(p.get("bundles", [])) == 2 for p in live), live
    # the replica's own tasks land in its gang (capture_child_tasks) -- bundle 1 holds 2 CPUs
    assert h.child_in_pg.remote().result(timeout_s=30) in pgs
    # 2 gangs x 3 CPUs reserved
    assert ray.available_resources().get("CPU", 0) <= 8 - 6 + 1e-6
    serve.delete("gang")
    deadline = time.time() + 20
    while time.time() < deadline:
        live = [p for p in list_placement_groups() if p.get("name", "").startswith("SERVE_REPLICA_PG::")
                and p.get("state") != "REMOVED"]
        if not live:
            break
        time.sleep(0.2)
    assert not live


@serve.deployment(num_replicas=4, max_replicas_per_node=2, ray_actor_options={"num_cpus": 0})
class Spread:
    def __call__(self):
        return ray.get_runtime_context().get_node_id()


def test_max_replicas_per_node_two_nodes():
    from cluster_anywhere_amd.cluster_utils import Cluster

    c = Cluster(initialize_head=True, head_node_args={"num_cpus": 4})
    try:
        c.add_node(num_cpus=4)
        c.connect()
        c.wait_for_nodes()
        h = serve.run(Spread.bind(), name="spread", route_prefix=None)
        st = serve.status().applications["spread"].deployments["Spread"]
        assert st.running_replicas == 4
        nodes = {}
        deadline = time.time() + 30
        while time.time() < deadline and len(nodes) < 2:
            for _ in range(40):
                n = h.remote().result(timeout_s=30)
                nodes[n] = nodes.get(n, 0) + 1
        assert len(nodes) == 2
        from cluster_anywhere_amd.util.state import list_actors

        per_node = {}
        for a in list_actors():
            if a["name"].startswith("SERVE_REPLICA::spread#Spread") and a["state"] == "ALIVE":
                per_node[a["node_id"]] = per_node.get(a["node_id"], 0) + 1
        assert sorted(per_node.values()) == [2, 2], per_node
        # a fifth replica has nowhere to go: it stays pending, with the reason in the status
        with pytest.raises(TimeoutError):
            serve.run(Spread.options(num_replicas=5, version="v1").bind(), name="spread2", route_prefix=None,
                      timeout_s=6)
        d = serve.status().applications["spread2"].deployments["Spread"]
        assert d.running_replicas == 0 or "max_replicas_per_node" in d.message
        serve.shutdown()
    finally:
        ray.shutdown()
        c.shutdown()


@serve.deployment
class Doubler:
    def __call__(self, x):
        return 2 * x


@serve.deployment(user_config={"offset": 1})
class Ingress:
    def __init__(self, child):
        self.child = child
        self.offset = 0

    def reconfigure(self, cfg):
        self.offset = cfg["offset"]

    async def __call__(self, x):
        return await self.child.remote(x) + self.offset

    def stream(self, n):
        for i in range(n):
            yield i


def test_local_testing_mode_needs_no_cluster():
    assert not ray.is_initialized()
    h = serve.run(Ingress.bind(Doubler.bind()), _local_testing_mode=True)
    assert h.remote(5).result() == 11
    assert list(h.options(method_name="stream", stream=True).remote(3)) == [0, 1, 2]
    assert h.remote(h.remote(1)).result() == 7  # responses passed as arguments are resolved
    with pytest.raises(RuntimeError, match="local testing mode"):
        h.remote(1)._to_object_ref()

    async def main():
        return await h.remote(2)

    assert asyncio.run(main()) == 5
    assert not ray.is_initialized()
