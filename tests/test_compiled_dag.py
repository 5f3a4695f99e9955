"""Compiled graphs over native shared-memory channels (reference:
python/ray/dag/tests/experimental/test_accelerated_dag.py,
python/ray/experimental/channel/tests)."""
import threading
import time

import numpy as np
import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd.dag import InputNode, MultiOutputNode
from cluster_anywhere_amd.experimental.channel import Channel, ChannelClosedError


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4, object_store_memory=256 << 20)
    yield
    ray.shutdown()


def test_channel_broadcast_and_backpressure():
    ch = Channel(num_readers=2, num_slots=2, slot_bytes=4096)
    got = {0: [], 1: []}

    def reader(r):
        while True:
            try:
                got[r].append(ch.read(r, timeout=10))
            except ChannelClosedError:
                return

    ths = [threading.Thread(target=reader, args=(r,)) for r in (0, 1)]
    for t in ths:
        t.start()
    for i in range(50):
        ch.write({"i": i, "a": np.arange(i)})
    deadline = time.time() + 10
    while (len(got[0]) < 50 or len(got[1]) < 50) and time.time() < deadline:
        time.sleep(0.01)
    ch.close()
    for t in ths:
        t.join(10)
    for r in (0, 1):
        assert [g["i"] for g in got[r]] == list(range(50))
        assert np.array_equal(got[r][7]["a"], np.arange(7))
    ch.destroy()


def test_channel_full_timeout_and_attach():
    import pickle

    ch = Channel(num_readers=1, num_slots=1, slot_bytes=256)
    ch.write(1)
    with pytest.raises(TimeoutError):
        ch.write(2, timeout=0.05)
    other = pickle.loads(pickle.dumps(ch))  # attach by name
    assert other.read(0, timeout=1) == 1
    ch.write(3, timeout=1)
    assert other.read(0, timeout=1) == 3
    with pytest.raises(TimeoutError):
        other.read(0, timeout=0.05)
    ch.destroy()


def test_channel_large_value_via_object_store(cluster):
    ch = Channel(num_readers=1, num_slots=2, slot_bytes=1024)
    big = np.ones(1 << 16, dtype=np.float32)
    ch.write(big)
    assert np.array_equal(ch.read(0, timeout=5), big)
    ch.destroy()


@ray.remote
class Stage:
    def __init__(self, k):
        self.k = k
        self.calls = 0

    def fwd(self, x):
        self.calls += 1
        if isinstance(x, int) and x < 0:
            raise ValueError("negative input")
        return x * self.k

    def add(self, a, b):
        return a + b

    def ncalls(self):
        return self.calls


def test_compiled_pipeline_chain_and_multi_output(cluster):
    a, b, c = Stage.remote(2), Stage.remote(3), Stage.remote(10)
    with InputNode() as inp:
        x = a.fwd.bind(inp)
        y = b.fwd.bind(x)
        z = c.add.bind(x, y)
        dag = MultiOutputNode([y, z])
    cdag = dag.experimental_compile(_max_inflight_executions=4)
    assert ray.get(cdag.execute(1)) == [6, 8]
    # pipelined: more executions in flight than the ring depth
    refs = [cdag.execute(i) for i in range(20)]
    assert [ray.get(r) for r in refs] == [[6 * i, 8 * i] for i in range(20)]
    # out-of-order get
    r1, r2 = cdag.execute(5), cdag.execute(7)
    assert ray.get(r2) == [42, 56] and ray.get(r1) == [30, 40]
    # an exception inside a stage surfaces at get() and the graph keeps running
    with pytest.raises(ValueError, match="negative input"):
        ray.get(cdag.execute(-1))
    assert ray.get(cdag.execute(2)) == [12, 16]
    cdag.teardown()
    # the actors still serve ordinary calls after teardown
    assert ray.get(a.ncalls.remote()) == 25


def test_compiled_same_actor_and_input_attributes(cluster):
    s = Stage.remote(4)
    with InputNode() as inp:
        u = s.fwd.bind(inp[0])
        dag = s.add.bind(u, inp.y)
    cdag = dag.experimental_compile()
    assert ray.get(cdag.execute(3, y=5)) == 17
    assert ray.get(cdag.execute(1, y=0)) == 4
    cdag.teardown()


@ray.remote
class TensorStage:
    def make(self, n):
        import torch

        return torch.arange(n, dtype=torch.float32)

    def double(self, t):
        return (t * 2, int(t.numel()))

    def total(self, pair):
        t, n = pair
        return float(t.sum()), n


def test_compiled_tensor_transport_gloo(cluster):
    p, q, r = TensorStage.remote(), TensorStage.remote(), TensorStage.remote()
    with InputNode() as inp:
        t = p.make.bind(inp).with_tensor_transport("gloo")
        d = q.double.bind(t).with_tensor_transport("gloo")
        dag = r.total.bind(d)
    cdag = dag.experimental_compile()
    for n in (4, 100, 1000):
        assert ray.get(cdag.execute(n), timeout=60) == (float(n * (n - 1)), n)
    cdag.teardown()


def test_compiled_replay_with_task_nodes(cluster):
    @ray.remote
    def inc(x):
        return x + 1

    s = Stage.remote(3)
    with InputNode() as inp:
        dag = s.fwd.bind(inc.bind(inp))
    cdag = dag.experimental_compile()
    assert ray.get(cdag.execute(1)) == 6


def test_compiled_asyncio_pipelines_eight_in_flight(cluster):
    """experimental_compile(enable_asyncio=True) + await dag.execute_async()
    (reference: compiled_dag_node.py:798,2417-2434; dag/tests/experimental/
    test_accelerated_dag.py::test_asyncio): 8 executions in flight at once from one
    event loop, more submissions than the ring depth, results in order, errors
    re-raised at await, sync execute() refused."""
    import asyncio

    a, b = Stage.remote(2), Stage.remote(5)
    with InputNode() as inp:
        dag = b.fwd.bind(a.fwd.bind(inp))
    cdag = dag.experimental_compile(enable_asyncio=True, _max_inflight_executions=8)
    with pytest.raises(RuntimeError, match="execute_async"):
        cdag.execute(1)

    async def main():
        futs = [await cdag.execute_async(i) for i in range(8)]  # fills the ring, no await of results
        first = await asyncio.gather(*futs)
        # 24 more from concurrent producers: submissions beyond the depth wait for slots
        async def one(i):
            fut = await cdag.execute_async(i)
            return await fut

        more = await asyncio.gather(*[one(i) for i in range(8, 32)])
        with pytest.raises(ValueError, match="negative input"):
            await (await cdag.execute_async(-1))
        after = await (await cdag.execute_async(3))
        return first, more, after

    first, more, after = asyncio.run(main())
    assert first == [10 * i for i in range(8)]
    assert more == [10 * i for i in range(8, 32)]
    assert after == 30
    cdag.teardown()


def test_compiled_overlap_flag_cpu_is_equivalent(cluster):
    """overlap_gpu_communication on CPU actors (gloo edges) changes nothing but the
    schedule: same results (the comm stream and the writer thread exist only on GPU
    actors; a CPU actor runs the synchronous loop)."""
    from cluster_anywhere_amd.dag.context import DAGContext

    p, q, r = TensorStage.remote(), TensorStage.remote(), TensorStage.remote()
    with InputNode() as inp:
        t = p.make.bind(inp).with_tensor_transport("gloo")
        d = q.double.bind(t).with_tensor_transport("gloo")
        dag = r.total.bind(d)
    ctx = DAGContext.get_current()
    ctx.overlap_gpu_communication = True
    try:
        cdag = dag.experimental_compile()
    finally:
        ctx.overlap_gpu_communication = False
    assert cdag._overlap
    for n in (4, 100, 1000):
        assert ray.get(cdag.execute(n), timeout=60) == (float(n * (n - 1)), n)
    cdag.teardown()
