"""Lazy task DAGs (reference: python/ray/dag/): ``f.bind(...)``, ``Cls.bind(...)``,
``actor.method.bind(...)``, ``InputNode``, ``MultiOutputNode``; ``dag.execute(x)``
submits the graph as ordinary tasks (ObjectRefs flow between nodes, so the
scheduler overlaps independent branches); ``dag.experimental_compile()`` builds a
:class:`~cluster_anywhere_amd.dag.compiled.CompiledDAG`: resident per-actor
execution loops connected by native shared-memory channels (and RCCL for
tensor-transport edges)."""
from __future__ import annotations

from typing import Any, Dict, List


class DAGNode:
    def __init__(self, args, kwargs):
        self._args = tuple(args)
        self._kwargs = dict(kwargs)

    def _children(self):
        out = [a for a in self._args if isinstance(a, DAGNode)]
        out += [v for v in self._kwargs.values() if isinstance(v, DAGNode)]
        return out

    def _resolve_args(self, cache, inp):
        a = [x._exec(cache, inp) if isinstance(x, DAGNode) else x for x in self._args]
        k = {n: (v._exec(cache, inp) if isinstance(v, DAGNode) else v) for n, v in self._kwargs.items()}
        return a, k

    def _exec(self, cache, inp):
        key = id(self)
        if key not in cache:
            cache[key] = self._run(cache, inp)
        return cache[key]

    def _run(self, cache, inp):  # pragma: no cover
        raise NotImplementedError

    def execute(self, *args, **kwargs):
        inp = InputValue(args, kwargs)
        return self._exec({}, inp)

    def with_tensor_transport(self, transport: str = "auto", **_kw):
        """Mark this node's output for out-of-band tensor transfer in a compiled
        graph: ``"nccl"``/``"rccl"`` (GPU→GPU over xGMI), ``"ipc"`` (same-node GPU
        actors through shared HBM buffers, HIP IPC) or ``"gloo"`` (CPU)."""
        self._transport = transport
        return self

    def experimental_compile(self, **kw):
        from .compiled import CompiledDAG

        ctx = DAGContext.get_current()
        kw.setdefault("_max_inflight_executions", ctx.max_inflight_executions)
        if ctx.buffer_size_bytes:
            kw.setdefault("_buffer_size_bytes", ctx.buffer_size_bytes)
        return CompiledDAG(self, **kw)

    def _label(self) -> str:
        kind = type(self).__name__
        name = (getattr(self, "_method", None) or getattr(getattr(self, "_fn", None), "__name__", None)
                or getattr(getattr(self, "_ac", None), "__name__", None) or "")
        return f"{kind}\\n{name}" if name else kind

    def visualize(self, filename: str = "compiled_graph", format: str = "dot", view: bool = False,
                  return_dot: bool = False, **kwargs):
        """Graphviz DOT text of the graph (graphviz itself is not in the image):
        written to ``filename`` + ``.dot`` and returned with ``return_dot``."""
        dot = to_dot(self)
        path = filename if filename.endswith(".dot") else f"{filename}.dot"
        with open(path, "w") as f:
            f.write(dot)
        return dot if return_dot else path


class InputValue:
    def __init__(self, args, kwargs):
        self.args, self.kwargs = args, kwargs


class InputNode(DAGNode):
    def __init__(self):
        super().__init__((), {})

    def __enter__(self):
        return self

    def __exit__(self, *e):
        return False

    def _run(self, cache, inp):
        if len(inp.args) == 1 and not inp.kwargs:
            return inp.args[0]
        return inp.args if inp.args else inp.kwargs

    def __getitem__(self, key):
        return InputAttributeNode(self, key)

    def __getattr__(self, key):
        if key.startswith("_"):
            raise AttributeError(key)
        return InputAttributeNode(self, key)


class InputAttributeNode(DAGNode):
    def __init__(self, parent, key):
        super().__init__((), {})
        self._parent, self._key = parent, key

    def _run(self, cache, inp):
        if isinstance(self._key, int):
            return inp.args[self._key]
        return inp.kwargs[self._key] if self._key in inp.kwargs else getattr(inp.args[0], self._key)


class FunctionNode(DAGNode):
    def __init__(self, rf, args, kwargs, options):
        super().__init__(args, kwargs)
        self._rf = rf
        self._options = options

    def _run(self, cache, inp):
        a, k = self._resolve_args(cache, inp)
        return self._rf.remote(*a, **k)


class ClassNode(DAGNode):
    def __init__(self, ac, args, kwargs):
        super().__init__(args, kwargs)
        self._ac = ac
        self._handle = None

    def _run(self, cache, inp):
        if self._handle is None:
            a, k = self._resolve_args(cache, inp)
            self._handle = self._ac.remote(*a, **k)
        return self._handle

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        node = self

        class _M:
            def bind(_, *args, **kwargs):
                return ClassMethodNode(node, name, args, kwargs, 1)

        return _M()


class ClassMethodNode(DAGNode):
    def __init__(self, target, method, args, kwargs, num_returns):
        super().__init__(args, kwargs)
        self._target = target
        self._method = method
        self._num_returns = num_returns

    def _run(self, cache, inp):
        h = self._target._exec(cache, inp) if isinstance(self._target, DAGNode) else self._target
        a, k = self._resolve_args(cache, inp)
        return getattr(h, self._method).remote(*a, **k)


class CollectiveOutputNode(ClassMethodNode):
    """One participant's output of a collective op across several actors' node
    outputs (reference: python/ray/dag/collective_node.py): it runs on the
    actor that produced its input; all participants execute the op together
    inside a compiled graph (``experimental.collective.allreduce.bind``)."""

    METHOD = "__caamd_collective__"

    def __init__(self, inp: ClassMethodNode, coll: dict, rank: int):
        super().__init__(inp._target, self.METHOD, (inp,), {}, 1)
        self._coll = coll
        self._rank = rank

    def _run(self, cache, inp):
        raise ValueError("collective nodes run only inside a compiled graph (dag.experimental_compile())")


class MultiOutputNode(DAGNode):
    def __init__(self, outputs: List[DAGNode]):
        super().__init__(tuple(outputs), {})

    def _run(self, cache, inp):
        return [x._exec(cache, inp) if isinstance(x, DAGNode) else x for x in self._args]


def to_dot(root: DAGNode) -> str:
    """DOT digraph of the nodes reachable from ``root`` (edges: argument -> consumer)."""
    ids: Dict[int, str] = {}
    lines = ["digraph DAG {", "  rankdir=LR;"]
    stack, seen = [root], set()
    edges = []
    while stack:
        n = stack.pop()
        if id(n) in seen:
            continue
        seen.add(id(n))
        ids[id(n)] = f"n{len(ids)}"
        deps = list(n._children())
        tgt = getattr(n, "_target", None)
        if isinstance(tgt, DAGNode):
            deps.append(tgt)
        for d in deps:
            edges.append((d, n))
            stack.append(d)
    nodes = {}
    stack, seen = [root], set()
    while stack:
        n = stack.pop()
        if id(n) in seen:
            continue
        seen.add(id(n))
        nodes[id(n)] = n
        stack.extend(n._children())
        tgt = getattr(n, "_target", None)
        if isinstance(tgt, DAGNode):
            stack.append(tgt)
    for k, n in nodes.items():
        lines.append(f'  {ids[k]} [label="{n._label()}"];')
    for a, b in edges:
        lines.append(f"  {ids[id(a)]} -> {ids[id(b)]};")
    lines.append("}")
    return "\n".join(lines) + "\n"


def plot(dag: DAGNode, to_file=None) -> str:
    """Reference: ray.dag.plot (pydot): here the DOT text, also written to ``to_file``."""
    dot = to_dot(dag)
    if to_file:
        with open(str(to_file), "w") as f:
            f.write(dot)
    return dot


from .context import DAGContext  # noqa: E402

# node-metadata keys of the reference's DAG serialization (python/ray/dag/constants.py)
PARENT_CLASS_NODE_KEY = "parent_class_node"
PREV_CLASS_METHOD_CALL_KEY = "prev_class_method_call"
BIND_INDEX_KEY = "bind_index"
IS_CLASS_METHOD_OUTPUT_KEY = "is_class_method_output"
COLLECTIVE_OPERATION_KEY = "collective_operation"
DAGNODE_TYPE_KEY = "__dag_node_type__"

__all__ = ["DAGNode", "InputNode", "FunctionNode", "ClassNode", "ClassMethodNode", "MultiOutputNode",
           "CollectiveOutputNode", "DAGContext", "plot", "PARENT_CLASS_NODE_KEY", "PREV_CLASS_METHOD_CALL_KEY",
           "BIND_INDEX_KEY", "IS_CLASS_METHOD_OUTPUT_KEY", "COLLECTIVE_OPERATION_KEY", "DAGNODE_TYPE_KEY"]
