"""Collective nodes in compiled graphs (reference: python/ray/dag/collective_node.py,
python/ray/dag/tests/experimental/test_collective_dag.py) over gloo on CPU."""
import pytest
import torch

import cluster_anywhere_amd as ray
from cluster_anywhere_amd.dag import InputNode, MultiOutputNode
from cluster_anywhere_amd.experimental.collective import ReduceOp, allgather, allreduce, reducescatter


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


@ray.remote
class Worker:
    def __init__(self, rank):
        self.rank = rank

    def grad(self, x):
        return torch.full((4,), float(self.rank + 1)) * x

    def apply(self, g):
        return (self.rank, g.tolist() if isinstance(g, torch.Tensor) else [t.tolist() for t in g])


def test_allreduce_sum_and_max(cluster):
    ws = [Worker.remote(r) for r in range(3)]
    with InputNode() as inp:
        gs = [w.grad.bind(inp) for w in ws]
        red = allreduce.bind(gs)
        dag = MultiOutputNode([w.apply.bind(g) for w, g in zip(ws, red)])
    cdag = dag.experimental_compile()
    try:
        for x in (1.0, 2.0, 0.5):
            out = ray.get(cdag.execute(x))
            assert [o[0] for o in out] == [0, 1, 2]
            for _, v in out:
                assert v == [6.0 * x] * 4
    finally:
        cdag.teardown()
    ws2 = [Worker.remote(r) for r in range(2)]
    with InputNode() as inp:
        mx = allreduce.bind([w.grad.bind(inp) for w in ws2], op=ReduceOp.MAX)
        dag = MultiOutputNode([w.apply.bind(g) for w, g in zip(ws2, mx)])
    cdag = dag.experimental_compile()
    try:
        assert [v for _, v in ray.get(cdag.execute(3.0))] == [[6.0] * 4, [6.0] * 4]
    finally:
        cdag.teardown()


def test_allgather_and_reducescatter(cluster):
    ws = [Worker.remote(r) for r in range(2)]
    with InputNode() as inp:
        gs = [w.grad.bind(inp) for w in ws]
        gathered = allgather.bind(gs)
        dag = MultiOutputNode([w.apply.bind(g) for w, g in zip(ws, gathered)])
    cdag = dag.experimental_compile()
    try:
        out = ray.get(cdag.execute(1.0))
        for _, v in out:
            assert v == [[1.0] * 4, [2.0] * 4]
    finally:
        cdag.teardown()
    with InputNode() as inp:
        rs = reducescatter.bind([w.grad.bind(inp) for w in ws])
        dag = MultiOutputNode([w.apply.bind(g) for w, g in zip(ws, rs)])
    cdag = dag.experimental_compile()
    try:
        out = ray.get(cdag.execute(2.0))
        assert [v for _, v in out] == [[6.0, 6.0], [6.0, 6.0]]
    finally:
        cdag.teardown()


def test_collective_validation(cluster):
    w = Worker.remote(0)
    with InputNode() as inp:
        a = w.grad.bind(inp)
        with pytest.raises(ValueError, match="different actor"):
            allreduce.bind([a, w.grad.bind(inp)])
        with pytest.raises(ValueError, match="at least two"):
            allreduce.bind([a])
