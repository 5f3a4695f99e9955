"""Compiled graphs (reference: python/ray/dag/compiled_dag_node.py,
python/ray/experimental/channel/{shared_memory_channel,torch_tensor_nccl_channel}.py).

``dag.experimental_compile()`` turns a DAG of actor-method nodes into a
standing pipeline:

* every participating actor runs ONE resident execution loop (a thread started
  through ``__ray_call__``) over its slice of the graph in topological order —
  no task submission, scheduling or object-store round trip per call;
* edges are native shared-memory rings (:mod:`experimental.channel`,
  ``csrc/runtime/channel.cc``): the driver writes the input into one ring,
  every producer writes its result into one ring that all its consumers read,
  and results consumed on the same actor are passed in-process;
* an edge marked ``node.with_tensor_transport("nccl")`` (alias ``"rccl"``;
  ``"gloo"`` for CPU) sends only tensor metadata through the ring and the tensor
  payload point-to-point over an RCCL communicator spanning the graph's actors
  — on MI355X that is a direct xGMI GPU→GPU copy, never a host bounce;
* ``with_tensor_transport("ipc")`` keeps GPU tensors on the GPU between actors
  of one node: the producer copies each output tensor into one of ``depth + 1``
  HBM buffers it shares once by HIP IPC handle, the ring carries only metadata,
  and the consumer maps the buffers once and copies out of them on its GPU;
* collective nodes (``experimental.collective.allreduce/allgather/reducescatter``,
  reference: dag/collective_node.py) run an op across several actors' outputs
  over a collective group set up at compile time;
* up to ``_max_inflight_executions`` executions are pipelined (the ring depth);
  ``execute()`` returns a :class:`CompiledDAGRef`; ``ray.get`` on it reads the
  outputs in submission order. An exception inside a node is forwarded through
  the graph and re-raised by ``get`` as a ``RayTaskError``.

Graphs that contain plain task nodes (``f.bind``) fall back to a pre-planned
replay through ordinary task submission (:class:`_ReplayDAG`).
"""
from __future__ import annotations

import asyncio
import inspect
import os
import threading
import time
import traceback
from typing import Any, Dict, List, Optional

from ..experimental.channel import DEFAULT_SLOT_BYTES, Channel, ChannelClosedError

COLLECTIVE_TRANSPORTS = ("nccl", "rccl", "gloo")


class _Stop:
    """Teardown sentinel flowing through the graph."""


class _DagError:
    def __init__(self, err):
        self.err = err


class _TensorSlot:
    """Placeholder for a tensor sent out-of-band over the collective group."""

    def __init__(self, i, shape, dtype):
        self.i, self.shape, self.dtype = i, tuple(shape), dtype


class _IpcSlot(_TensorSlot):
    """Placeholder for a tensor left in shared HBM buffer ``buf`` (``handle`` is
    sent with a buffer's first use / reallocation)."""

    def __init__(self, i, shape, dtype, buf, handle):
        super().__init__(i, shape, dtype)
        self.buf, self.handle = buf, handle


# --------------------------------------------------------------------- refs
class CompiledDAGRef:
    def __init__(self, dag, seq, multi):
        self._dag, self._seq, self._multi = dag, seq, multi
        self._refs = None  # replay mode
        self._done = False

    def get(self, timeout=None):
        if self._done:
            raise ValueError("a CompiledDAGRef can be fetched only once")
        self._done = True
        if self._refs is not None:
            from ..core.api import get

            vals = get(self._refs, timeout=timeout)
            return vals if self._multi else vals[0]
        return self._dag._fetch(self._seq, timeout)

    def __repr__(self):
        return f"CompiledDAGRef(seq={self._seq})"


class CompiledDAGFuture:
    """``await dag.execute_async(...)`` returns this; ``await fut`` gives the result
    (reference: compiled_dag_node.py:2417-2434, compiled_dag_ref.py CompiledDAGFuture)."""

    def __init__(self, fut, multi):
        self._fut, self._multi = fut, multi
        self._done = False

    def __await__(self):
        if self._done:
            raise ValueError("a CompiledDAGFuture can be awaited only once")
        self._done = True
        vals = yield from self._fut.__await__()
        return _unpack(vals, self._multi)

    def __repr__(self):
        return f"CompiledDAGFuture(done={self._fut.done()})"


def _unpack(vals, multi):
    for v in vals:
        if isinstance(v, _DagError):
            e = v.err
            raise e.as_instanceof_cause() if hasattr(e, "as_instanceof_cause") else e
    return vals if multi else vals[0]


# --------------------------------------------------------------------- actor side
def _split_tensors(value):
    """Replace torch tensors at the top level of value (or in a list/tuple/dict)
    by _TensorSlot placeholders; returns (skeleton, tensors)."""
    import torch

    tensors = []

    def sub(v):
        if isinstance(v, torch.Tensor):
            tensors.append(v.contiguous())
            return _TensorSlot(len(tensors) - 1, v.shape, v.dtype)
        return v

    if isinstance(value, (list, tuple)):
        sk = type(value)(sub(v) for v in value)
    elif isinstance(value, dict):
        sk = {k: sub(v) for k, v in value.items()}
    else:
        sk = sub(value)
    return sk, tensors


def _fill_tensors(skel, tensors):
    def sub(v):
        return tensors[v.i] if isinstance(v, _TensorSlot) else v

    if isinstance(skel, (list, tuple)):
        return type(skel)(sub(v) for v in skel)
    if isinstance(skel, dict):
        return {k: sub(v) for k, v in skel.items()}
    return sub(skel)


def _slots(skel):
    vals = list(skel) if isinstance(skel, (list, tuple)) else (
        list(skel.values()) if isinstance(skel, dict) else [skel])
    return [v for v in vals if isinstance(v, _TensorSlot)]


class _ActorLoop:
    """One actor's resident execution loop.

    With ``overlap_gpu_communication`` (reference: compiled_dag_node.py:192-226, 540)
    a GPU actor moves its edge transfers onto a communication stream of its own,
    ordered against compute by events, so the host loop never waits for them:
      * RCCL sends are enqueued on the comm stream behind an event recorded after the
        producing compute and are not waited for (NCCL records the tensors on its
        stream, so dropping them is safe); RCCL recvs run on the comm stream and the
        compute stream waits on them GPU-side;
      * an IPC producer copies into the shared HBM buffer on the comm stream, and a
        writer thread publishes the ring message once that copy's event completed
        (FIFO with every other write, so ring order is unchanged) while the loop
        goes on to the next compute;
      * an IPC consumer copies out on the comm stream and waits for that copy only
        before its NEXT read of the same edge (the producer reuses a buffer only
        after that read).
    """

    def __init__(self, instance, plan):
        self.inst = instance
        self.plan = plan
        self.group = None
        self.cgroups = {}
        self.ipc_out = {}   # (out key, tensor index) -> [buffers]
        self.ipc_seq = {}   # out key -> executions written
        self.ipc_maps = {}  # (channel name, tensor index, buffer) -> mapped uint8 tensor
        self.overlap = bool(plan.get("overlap"))
        self.comm = None         # comm stream (overlap mode, GPU actors)
        self.writer = None       # writer thread + its FIFO (overlap mode)
        self.pending_read = {}   # channel name -> event of the last copy-out from it
        self.pending_sends = []  # (works, tensors) of un-waited RCCL sends

    def _comm_stream(self):
        import torch

        if not self.overlap or not torch.cuda.is_available():
            return None
        if self.comm is None:
            self.comm = torch.cuda.Stream()
        return self.comm

    def _start_writer(self):
        import queue

        self.wq = queue.Queue()
        self.writer_err = None

        def run():
            while True:
                item = self.wq.get()
                if item is None:
                    return
                ev, ch, msg = item
                try:
                    if ev is not None:
                        ev.synchronize()
                    ch.write(msg)
                except Exception as e:  # noqa: BLE001 (channel closed at teardown)
                    self.writer_err = e
                    return

        self.writer = threading.Thread(target=run, name="caamd-cdag-writer", daemon=True)
        self.writer.start()

    def _post(self, ch, msg, ev=None):
        """Write a ring message: in order through the writer thread in overlap mode."""
        if self.writer is None:
            if ev is not None:
                ev.synchronize()
            ch.write(msg)
            return
        if self.writer_err is not None:
            raise ChannelClosedError(str(self.writer_err))
        self.wq.put((ev, ch, msg))

    def _setup_group(self):
        from ..util.collective import collective as col

        for cg in self.plan.get("cgroups", []):
            backend = cg["backend"]
            if backend == "auto":
                backend = "nccl" if os.environ.get("CAAMD_GPU_IDS") else "gloo"
            col.init_collective_group(cg["world"], cg["rank"], backend=backend, group_name=cg["name"])
            self.cgroups[cg["name"]] = backend
        g = self.plan.get("group")
        if not g:
            return
        from ..util.collective import collective as col

        col.init_collective_group(g["world"], g["rank"], backend=g["backend"], group_name=g["name"])
        self.group = col._check_and_get_group(g["name"])
        import torch

        self.device = (torch.device("cuda", torch.cuda.current_device()) if g["backend"] != "gloo"
                       else torch.device("cpu"))

    def _read(self, ch, reader, producer_rank):
        ev = self.pending_read.pop(ch.name, None)
        if ev is not None:
            ev.synchronize()  # the previous copy-out of this edge is done: its buffer may be reused
        v = ch.read(reader)
        if producer_rank == "ipc" and not isinstance(v, (_Stop, _DagError)):
            return self._read_ipc(ch, v)
        if producer_rank is not None and not isinstance(v, (_Stop, _DagError)):
            import torch

            slots = _slots(v)
            comm = self._comm_stream() if self.device.type == "cuda" else None
            if comm is None:
                bufs = [torch.empty(s.shape, dtype=s.dtype, device=self.device) for s in slots]
                works = [self.group.pg.recv([b], producer_rank, 0) for b in bufs]
                for w in works:
                    w.wait()
            else:
                cur = torch.cuda.current_stream()
                with torch.cuda.stream(comm):
                    bufs = [torch.empty(s.shape, dtype=s.dtype, device=self.device) for s in slots]
                    works = [self.group.pg.recv([b], producer_rank, 0) for b in bufs]
                    for w in works:
                        w.wait()  # NCCL: the comm stream waits, not the host
                cur.wait_stream(comm)
                for b in bufs:
                    b.record_stream(cur)
            v = _fill_tensors(v, {s.i: b for s, b in zip(slots, bufs)})
        return v

    # -- HIP IPC edges: shared HBM buffer ring (depth + 1 buffers per tensor) ----
    def _write_ipc(self, out, value):
        import torch

        from ..experimental.gpu_objects import reduce_ipc

        key = id(out)
        seq = self.ipc_seq.get(key, 0)
        self.ipc_seq[key] = seq + 1
        nbuf = out["ipc_depth"] + 1
        j = seq % nbuf

        comm = self._comm_stream()
        if comm is not None:
            comm.wait_stream(torch.cuda.current_stream())  # the producing compute first

        def sub_all(skel, tensors):
            def sub(v):
                if not isinstance(v, _TensorSlot):
                    return v
                t = tensors[v.i]
                if not t.is_cuda:
                    return t  # CPU tensors travel in the ring itself
                nbytes = t.numel() * t.element_size()
                bufs = self.ipc_out.setdefault((key, v.i), [None] * nbuf)
                handle = None
                if bufs[j] is None or bufs[j].numel() < nbytes or bufs[j].device != t.device:
                    bufs[j] = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=t.device)
                    handle = reduce_ipc(bufs[j])
                if comm is not None:
                    with torch.cuda.stream(comm):
                        bufs[j][:nbytes].copy_(t.reshape(-1).view(torch.uint8))
                    t.record_stream(comm)
                else:
                    bufs[j][:nbytes].copy_(t.reshape(-1).view(torch.uint8))
                return _IpcSlot(v.i, t.shape, t.dtype, j, handle)

            if isinstance(skel, (list, tuple)):
                return type(skel)(sub(x) for x in skel)
            if isinstance(skel, dict):
                return {k: sub(x) for k, x in skel.items()}
            return sub(skel)

        skel, tensors = _split_tensors(value)
        msg = sub_all(skel, tensors)
        ev = None
        if any(t.is_cuda for t in tensors):
            # data in HBM before the consumer sees the slot: the writer thread waits for
            # the copy's event in overlap mode, the loop itself otherwise
            ev = torch.cuda.Event()
            ev.record(comm if comm is not None else torch.cuda.current_stream())
        self._post(out["chan"], msg, ev)

    def _read_ipc(self, ch, v):
        import torch

        def sub(x):
            if not isinstance(x, _IpcSlot):
                return x
            k = (ch.name, x.i, x.buf)
            if x.handle is not None:
                fn, args = x.handle
                self.ipc_maps[k] = fn(*args)
            src = self.ipc_maps[k]
            n = 1
            for d in x.shape:
                n *= d
            nbytes = n * torch.empty((), dtype=x.dtype).element_size()
            if comm is not None:
                with torch.cuda.stream(comm):
                    t = src[:nbytes].view(x.dtype).view(x.shape).clone()
                t.record_stream(cur)
                return t
            return src[:nbytes].view(x.dtype).view(x.shape).clone()

        comm = self._comm_stream()
        cur = torch.cuda.current_stream() if comm is not None else None
        if comm is not None:
            comm.wait_stream(cur)  # earlier compute may still read this actor's last copies
        if isinstance(v, (list, tuple)):
            out = type(v)(sub(x) for x in v)
        elif isinstance(v, dict):
            out = {k: sub(x) for k, x in v.items()}
        else:
            out = sub(v)
        if torch.cuda.is_available() and self.ipc_maps:
            if comm is not None:
                # compute waits GPU-side; the host waits for the copy only before the
                # next read of this edge (the producer reuses the buffer after it)
                ev = torch.cuda.Event()
                ev.record(comm)
                cur.wait_event(ev)
                self.pending_read[ch.name] = ev
            else:
                # copies done before the next read lets the producer reuse the buffer
                torch.cuda.current_stream().synchronize()
        return out

    def _collective(self, spec, x):
        import torch

        from ..util.collective import collective as col

        name, kind, op = spec["group"], spec["kind"], spec["op"]
        if not isinstance(x, torch.Tensor):
            raise TypeError(f"collective {kind} needs a torch.Tensor input, got {type(x).__name__}")
        world = spec["world"]
        if kind == "allreduce":
            t = x.clone()
            col.allreduce(t, name, op)
            return t
        if kind == "allgather":
            outs = [torch.empty_like(x) for _ in range(world)]
            col.allgather(outs, x.contiguous(), name)
            return outs
        if kind == "reducescatter":
            if x.shape[0] % world:
                raise ValueError(f"reducescatter: dim 0 ({x.shape[0]}) must divide by {world}")
            chunks = [c.contiguous() for c in x.chunk(world, 0)]
            t = torch.empty_like(chunks[0])
            col.reducescatter(t, chunks, name, op)
            return t
        raise ValueError(kind)

    def _write(self, out, value):
        if out.get("ipc") and not isinstance(value, (_Stop, _DagError)):
            return self._write_ipc(out, value)
        ch, dst_ranks = out["chan"], out.get("dst_ranks")
        if dst_ranks and not isinstance(value, (_Stop, _DagError)):
            skel, tensors = _split_tensors(value)
            self._post(ch, skel)
            comm = self._comm_stream() if self.device.type == "cuda" else None
            if comm is None:
                works = [self.group.pg.send([t], r, 0) for r in dst_ranks for t in tensors]
                for w in works:
                    w.wait()
                return
            import torch

            comm.wait_stream(torch.cuda.current_stream())  # behind the producing compute
            with torch.cuda.stream(comm):
                works = [self.group.pg.send([t], r, 0) for r in dst_ranks for t in tensors]
            self.pending_sends.append((works, tensors))
            while len(self.pending_sends) > int(self.plan.get("depth", 8)):
                old_works, _ = self.pending_sends.pop(0)
                with torch.cuda.stream(comm):
                    for w in old_works:
                        w.wait()
        else:
            self._post(ch, value)

    def _drain(self):
        """Overlap mode: every queued ring write and comm-stream transfer completes."""
        if self.pending_sends:
            import torch

            with torch.cuda.stream(self.comm):
                for works, _ in self.pending_sends:
                    for w in works:
                        w.wait()
            self.pending_sends = []
        if self.comm is not None:
            self.comm.synchronize()
        if self.writer is not None:
            self.wq.put(None)
            self.writer.join(30)
            self.writer = None

    def _call(self, method, a, k):
        fn = getattr(self.inst, method)
        r = fn(*a, **k)
        if inspect.iscoroutine(r):
            from ..core import context

            loop = getattr(context.worker, "async_loop", None) if context.worker else None
            if loop is not None and loop.is_running():
                r = asyncio.run_coroutine_threadsafe(r, loop).result()
            else:
                r = asyncio.run(r)
        return r

    def run(self):
        try:
            self._run()
        finally:
            try:
                self._drain()
            except Exception:
                pass

    def _run(self):
        from ..exceptions import RayTaskError

        try:
            if self.overlap and self._comm_stream() is not None:
                self._start_writer()
            self._setup_group()
        except Exception:  # pragma: no cover - surfaced through the graph outputs
            err = _DagError(RayTaskError("compiled-graph setup", traceback.format_exc()))
            for t in self.plan["tasks"]:
                if t["out"]:
                    t["out"]["chan"].write(err)
            return
        tasks = self.plan["tasks"]
        while True:
            cache: Dict[Any, Any] = {}
            local: Dict[int, Any] = {}
            stop = False

            def resolve(spec):
                kind = spec[0]
                if kind == "const":
                    return spec[1]
                if kind == "loc":
                    return local[spec[1]]
                key = (spec[1].name, spec[2])
                if key not in cache:
                    cache[key] = self._read(spec[1], spec[2], spec[4] if len(spec) > 4 else None)
                v = cache[key]
                if kind == "in" and not isinstance(v, (_Stop, _DagError)):
                    return _input_select(v, spec[3])
                return v

            for t in tasks:
                try:
                    a = [resolve(s) for s in t["args"]]
                    k = {n: resolve(s) for n, s in t["kwargs"].items()}
                except ChannelClosedError:
                    return
                vals = a + list(k.values())
                if any(isinstance(v, _Stop) for v in vals):
                    stop = True
                    res = _Stop()
                else:
                    err = next((v for v in vals if isinstance(v, _DagError)), None)
                    if err is not None:
                        res = err
                    else:
                        try:
                            if t.get("coll") is not None:
                                res = self._collective(t["coll"], a[0])
                            else:
                                res = self._call(t["method"], a, k)
                        except Exception as e:
                            res = _DagError(RayTaskError(t["method"], traceback.format_exc(), e))
                local[t["idx"]] = res
                if t["out"] is not None:
                    try:
                        self._write(t["out"], res)
                    except ChannelClosedError:
                        return
            if stop:
                self._drain()  # in-flight transfers land before the groups go away
                from ..util import collective as col

                names = list(self.cgroups) + ([self.plan["group"]["name"]] if self.group is not None else [])
                for nm in names:
                    try:
                        col.destroy_collective_group(nm)
                    except Exception:
                        pass
                return


def _input_select(inp, key):
    args, kwargs = inp
    if key is None:
        if len(args) == 1 and not kwargs:
            return args[0]
        return args if args else kwargs
    if isinstance(key, int):
        return args[key]
    return kwargs[key] if key in kwargs else getattr(args[0], key)


def _start_loop(instance, plan):
    loop = _ActorLoop(instance, plan)
    th = threading.Thread(target=loop.run, name="caamd-compiled-dag", daemon=True)
    th.start()
    return os.getpid()


# --------------------------------------------------------------------- driver side
def _topo(root):
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
    return order


class CompiledDAG:
    def __new__(cls, root, **kw):
        from . import FunctionNode

        if any(isinstance(n, FunctionNode) for n in _topo(root)):
            return _ReplayDAG(root)
        return super().__new__(cls)

    def __init__(self, root, _max_inflight_executions: Optional[int] = None,
                 _buffer_size_bytes: Optional[int] = None, enable_asyncio: bool = False,
                 _overlap_gpu_communication: Optional[bool] = None, **_kw):
        from . import (ClassMethodNode, ClassNode, InputAttributeNode, InputNode,
                       MultiOutputNode)
        from ..core.api import get

        self._multi = isinstance(root, MultiOutputNode)
        self._slots = int(_max_inflight_executions or 8)
        slot_bytes = int(_buffer_size_bytes or DEFAULT_SLOT_BYTES)
        order = _topo(root)
        tasks = [n for n in order if isinstance(n, ClassMethodNode)]
        if not tasks:
            raise ValueError("a compiled graph needs at least one actor method node")
        outputs = list(root._args) if self._multi else [root]
        for o in outputs:
            if not isinstance(o, ClassMethodNode):
                raise ValueError("compiled graph outputs must be actor method nodes")
        # actor handle per task (ClassNode targets are instantiated once, here)
        handles = {}
        for t in tasks:
            tgt = t._target
            h = tgt._exec({}, None) if isinstance(tgt, ClassNode) else tgt
            handles[id(t)] = h
        actors: List[Any] = []
        for t in tasks:
            if handles[id(t)] not in actors:
                actors.append(handles[id(t)])
        akey = {id(t): actors.index(handles[id(t)]) for t in tasks}
        tidx = {id(t): i for i, t in enumerate(tasks)}

        def deps(n):
            return list(n._args) + list(n._kwargs.values())

        # consumers of each producer (other actors) and of the input
        input_readers: List[int] = []
        consumers: Dict[int, List[Any]] = {id(t): [] for t in tasks}
        for t in tasks:
            a = akey[id(t)]
            for d in deps(t):
                if isinstance(d, (InputNode, InputAttributeNode)):
                    if a not in input_readers:
                        input_readers.append(a)
                elif isinstance(d, ClassMethodNode):
                    if akey[id(d)] != a and a not in consumers[id(d)]:
                        consumers[id(d)].append(a)
                elif hasattr(d, "_children"):
                    raise ValueError(f"unsupported node in a compiled graph: {type(d).__name__}")
        for o in outputs:
            if "driver" not in consumers[id(o)]:
                consumers[id(o)].append("driver")
        if not input_readers:
            raise ValueError("a compiled graph must consume its InputNode")

        # collective group for tensor-transport edges (ranks = actor order); "ipc"
        # edges need no group (shared HBM buffers between same-node actors)
        transports = {getattr(t, "_transport", None) for t in tasks} - {None, "auto", "shm", "ipc"}
        bad = transports - set(COLLECTIVE_TRANSPORTS)
        if bad:
            raise ValueError(f"unknown tensor transport(s) {sorted(bad)}")
        if len(transports) > 1:
            raise ValueError("one compiled graph uses one collective transport")
        backend = None
        if transports:
            backend = transports.pop()
            backend = "nccl" if backend == "rccl" else backend
        self._group = f"cdag-{os.getpid()}-{os.urandom(4).hex()}" if backend else None

        self._input = Channel(len(input_readers), self._slots, slot_bytes)
        chans: Dict[int, Channel] = {}
        for t in tasks:
            if consumers[id(t)]:
                chans[id(t)] = Channel(len(consumers[id(t)]), self._slots, slot_bytes)
        self._channels = [self._input] + list(chans.values())
        self._out_specs = []  # (channel, reader) per output position
        for o in outputs:
            self._out_specs.append((chans[id(o)], consumers[id(o)].index("driver")))

        if _overlap_gpu_communication is None:
            from .context import DAGContext

            _overlap_gpu_communication = DAGContext.get_current().overlap_gpu_communication
        self._overlap = bool(_overlap_gpu_communication)
        plans = {a: {"tasks": [], "group": None, "cgroups": [], "overlap": self._overlap,
                     "depth": self._slots} for a in range(len(actors))}
        if backend:
            for a in plans:
                plans[a]["group"] = {"world": len(actors), "rank": a, "backend": backend,
                                     "name": self._group}
        # collective nodes: one group per collective op, ranks = participant order
        from . import CollectiveOutputNode

        colls: Dict[int, dict] = {}
        for t in tasks:
            if isinstance(t, CollectiveOutputNode) and t._coll["id"] not in colls:
                c = t._coll
                parts = [akey[id(o)] for o in c["outputs"]]
                if any(id(o) not in akey for o in c["outputs"]):
                    raise ValueError("every output of a collective must be part of the compiled graph")
                name = f"cdag-{os.getpid()}-{os.urandom(3).hex()}-c{c['id']}"
                colls[c["id"]] = {"group": name, "kind": c["kind"], "op": c["op"], "world": len(parts)}
                tr = {"rccl": "nccl"}.get(c["transport"], c["transport"])
                for r, a in enumerate(parts):
                    plans[a]["cgroups"].append({"name": name, "world": len(parts), "rank": r, "backend": tr})

        def spec(d, a):
            if isinstance(d, InputNode):
                return ("in", self._input, input_readers.index(a), None)
            if isinstance(d, InputAttributeNode):
                return ("in", self._input, input_readers.index(a), d._key)
            if isinstance(d, ClassMethodNode):
                if akey[id(d)] == a:
                    return ("loc", tidx[id(d)])
                tr = getattr(d, "_transport", None)
                if tr == "ipc":
                    return ("ch", chans[id(d)], consumers[id(d)].index(a), None, "ipc")
                tr = tr if backend else None
                src = akey[id(d)] if tr in COLLECTIVE_TRANSPORTS else None
                return ("ch", chans[id(d)], consumers[id(d)].index(a), None, src)
            return ("const", d)

        for t in tasks:
            a = akey[id(t)]
            out = None
            if id(t) in chans:
                out = {"chan": chans[id(t)]}
                tr = getattr(t, "_transport", None)
                if tr == "ipc":
                    if "driver" in consumers[id(t)]:
                        raise ValueError("an ipc tensor-transport node cannot be a graph output")
                    out["ipc"] = True
                    out["ipc_depth"] = self._slots
                if backend and tr in COLLECTIVE_TRANSPORTS:
                    if "driver" in consumers[id(t)]:
                        raise ValueError("a tensor-transport node cannot be a graph output "
                                         "(the driver is not in the collective group)")
                    out["dst_ranks"] = list(consumers[id(t)])
            plans[a]["tasks"].append({
                "idx": tidx[id(t)], "method": t._method, "out": out,
                "coll": colls[t._coll["id"]] if isinstance(t, CollectiveOutputNode) else None,
                "args": [spec(d, a) for d in t._args],
                "kwargs": {k: spec(d, a) for k, d in t._kwargs.items()},
            })
        self._actors = actors
        get([h.__ray_call__.remote(_start_loop, plans[i]) for i, h in enumerate(actors)])
        self._submitted = 0
        self._fetched = 0
        self._results: Dict[int, Any] = {}
        self._lock = threading.Lock()
        self._torn_down = False
        self._asyncio = bool(enable_asyncio)
        if self._asyncio:
            # results are read by one thread, in submission order, and handed to the
            # futures' event loops (reference: compiled_dag_node.py:798,849,2417-2434)
            self._afuts: Dict[int, Any] = {}
            self._acv = threading.Condition(self._lock)
            self._aspace: Dict[int, Any] = {}  # id(loop) -> asyncio.Event (a slot freed)
            self._alocks: Dict[int, Any] = {}
            self._reader = threading.Thread(target=self._async_reader, name="caamd-cdag-reader", daemon=True)
            self._reader.start()

    # -- asyncio execution -----------------------------------------------------------
    async def execute_async(self, *args, **kwargs) -> "CompiledDAGFuture":
        """Submit one execution without blocking the event loop; ``await`` the returned
        future for its result. At most ``_max_inflight_executions`` are in flight: a
        further submission waits (asynchronously) for the oldest to be read."""
        if not self._asyncio:
            raise RuntimeError("execute_async() needs experimental_compile(enable_asyncio=True)")
        if self._torn_down:
            raise RuntimeError("compiled graph was torn down")
        loop = asyncio.get_running_loop()
        lk = self._alocks.setdefault(id(loop), asyncio.Lock())
        async with lk:  # submission order = result order
            while True:
                with self._lock:
                    if self._submitted - self._fetched < self._slots:
                        fut = loop.create_future()
                        seq = self._submitted
                        self._afuts[seq] = (loop, fut)
                        self._input.write((args, kwargs))  # never blocks: the ring has a free slot
                        self._submitted += 1
                        self._acv.notify_all()
                        break
                    ev = self._aspace.setdefault(id(loop), (loop, asyncio.Event()))[1]
                    ev.clear()
                await ev.wait()
        return CompiledDAGFuture(fut, self._multi)

    def _async_reader(self):
        def deliver(fut, vals):
            if not fut.done():
                fut.set_result(vals)

        while True:
            with self._lock:
                while self._fetched >= self._submitted and not self._torn_down:
                    self._acv.wait(0.1)
                if self._torn_down:
                    return
            vals = []
            try:
                for ch, r in self._out_specs:
                    while True:
                        try:
                            vals.append(ch.read(r, 0.1))
                            break
                        except TimeoutError:
                            if self._torn_down:
                                return
            except ChannelClosedError:
                return
            with self._lock:
                seq = self._fetched
                self._fetched += 1
                loop, fut = self._afuts.pop(seq)
            loop.call_soon_threadsafe(deliver, fut, vals)
            for lp, ev in list(self._aspace.values()):  # a ring slot freed
                lp.call_soon_threadsafe(ev.set)

    # -- execution ---------------------------------------------------------------
    def execute(self, *args, **kwargs) -> CompiledDAGRef:
        if self._torn_down:
            raise RuntimeError("compiled graph was torn down")
        if self._asyncio:
            raise RuntimeError("this graph was compiled with enable_asyncio=True: use "
                               "`await dag.execute_async(...)`")
        with self._lock:
            # keep at most `slots` executions in flight: drain the oldest first
            while self._submitted - self._fetched >= self._slots:
                self._read_one(None)
            self._input.write((args, kwargs))
            seq = self._submitted
            self._submitted += 1
        return CompiledDAGRef(self, seq, self._multi)

    def _read_one(self, timeout):
        vals = [ch.read(r, timeout) for ch, r in self._out_specs]
        self._results[self._fetched] = vals
        self._fetched += 1

    def _fetch(self, seq, timeout):
        with self._lock:
            while seq not in self._results:
                if seq < self._fetched:
                    raise ValueError("result already fetched")
                self._read_one(timeout)
            vals = self._results.pop(seq)
        return _unpack(vals, self._multi)

    def teardown(self, timeout: float = 30.0):
        if self._torn_down:
            return
        if self._asyncio:
            # let the reader deliver what is in flight, then stop it
            deadline = time.time() + timeout
            while time.time() < deadline:
                with self._lock:
                    if self._fetched >= self._submitted:
                        break
                time.sleep(0.01)
        self._torn_down = True
        if self._asyncio:
            with self._lock:
                self._acv.notify_all()
            self._reader.join(timeout)
        try:
            self._input.write(_Stop(), timeout=timeout)
            # drain until every output ring delivered the stop sentinel
            for ch, r in self._out_specs:
                while True:
                    v = ch.read(r, timeout)
                    if isinstance(v, _Stop):
                        break
        except (TimeoutError, ChannelClosedError):
            pass
        finally:
            for c in self._channels:
                try:
                    c.destroy()
                except Exception:
                    pass

    def __del__(self):
        try:
            if not self._torn_down:
                for c in self._channels:
                    c.destroy()
        except Exception:
            pass


class _ReplayDAG:
    """Graphs with plain task nodes: actors are created once and the topological
    order is computed once; every ``execute()`` replays the submissions."""

    def __init__(self, root):
        from . import ClassNode, MultiOutputNode

        self._root = root
        self._multi = isinstance(root, MultiOutputNode)
        for n in _topo(root):
            if isinstance(n, ClassNode):
                n._exec({}, None)

    def execute(self, *args, **kwargs):
        from . import InputValue

        out = self._root._exec({}, InputValue(args, kwargs))
        ref = CompiledDAGRef(None, 0, self._multi)
        ref._refs = out if self._multi else [out]
        return ref

    def teardown(self):
        pass
