"""Collective ops as compiled-graph nodes (reference:
python/ray/experimental/collective/ + python/ray/dag/collective_node.py)::

    from cluster_anywhere_amd.experimental.collective import allreduce
    with InputNode() as inp:
        grads = [w.backward.bind(inp) for w in workers]
        reduced = allreduce.bind(grads)            # one output node per worker
        dag = MultiOutputNode([w.apply.bind(g) for w, g in zip(workers, reduced)])
    cdag = dag.experimental_compile()

Each output node runs on the actor that produced its input; the participants
form one collective group (RCCL over xGMI for GPU tensors, gloo for CPU) set up
once when the graph is compiled, and execute the op together every iteration.
``transport="auto"`` picks RCCL in actors that were given GPUs, gloo otherwise.
"""
from __future__ import annotations

import itertools
from typing import List

from ..util.collective.types import ReduceOp

_ids = itertools.count()


class _CollectiveOp:
    def __init__(self, kind: str):
        self.kind = kind

    def bind(self, input_nodes: List, op=ReduceOp.SUM, transport: str = "auto"):
        from ..dag import ClassMethodNode, CollectiveOutputNode

        nodes = list(input_nodes)
        if len(nodes) < 2:
            raise ValueError("a collective needs at least two participant nodes")
        for n in nodes:
            if not isinstance(n, ClassMethodNode):
                raise ValueError("collective inputs must be actor method nodes")
        if len({id(n._target) for n in nodes}) != len(nodes):
            raise ValueError("each participant of a collective must be a different actor")
        if transport not in ("auto", "nccl", "rccl", "gloo"):
            raise ValueError(f"unknown collective transport {transport!r}")
        coll = {"id": next(_ids), "kind": self.kind, "op": op, "transport": transport}
        outs = [CollectiveOutputNode(n, coll, r) for r, n in enumerate(nodes)]
        coll["outputs"] = outs
        return outs


allreduce = _CollectiveOp("allreduce")
allgather = _CollectiveOp("allgather")
reducescatter = _CollectiveOp("reducescatter")

__all__ = ["allreduce", "allgather", "reducescatter", "ReduceOp"]
