"""Streaming executor (reference: python/ray/data/_internal/execution/
streaming_executor.py:48, operators/task_pool_map_operator.py,
operators/actor_pool_map_operator.py, resource_manager.py:25).

The logical plan is a chain of operators. Consecutive task-based block
transforms are FUSED into the source read (one remote task per input block does
read → map → map ...). An actor-pool map (stateful UDF class, e.g. a model on a
GPU) becomes its own streaming stage fed by the upstream stage. All-to-all
operators (shuffle / sort / repartition / groupby) are barriers.

Backpressure: every stage keeps at most ``max_inflight`` tasks outstanding (by
default 2 x cluster CPUs for task stages, ``actor_max_tasks_in_flight`` per actor
for actor stages) so a fast producer cannot flood the object store; output order
is preserved (FIFO retirement).
"""
from __future__ import annotations

import collections
import itertools
import time
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple

from . import block as B
from .context import DataContext

import os as _os

_PROFILE = _os.environ.get("CAAMD_DATA_PROFILE") == "1"


# ------------------------------------------------------------------ remote work
def _apply_chain(block, chain):
    out = [block]
    for fn in chain:
        nxt = []
        for b in out:
            for r in fn(b):
                if r is not None:
                    nxt.append(r)
        out = nxt
    return out


def _task_body(src, chain):
    """src: a block (resolved ObjectRef) or a zero-arg read callable."""
    blocks = src() if callable(src) else [src]
    if isinstance(blocks, dict) or B.is_arrow(blocks):
        blocks = [blocks]
    out = []
    for b in blocks:
        out.extend(_apply_chain(b, chain))
    res = B.concat(out) if len(out) != 1 else out[0]
    return res, {"num_rows": B.num_rows(res), "size_bytes": B.size_bytes(res), "schema": B.schema_of(res)}


_remote_task = None


def _get_remote_task():
    global _remote_task
    if _remote_task is None:
        from ..core.api import remote

        _remote_task = remote(num_returns=2)(_task_body)
    return _remote_task


class _MapWorker:
    """Actor hosting a stateful UDF (constructed once; reused for every block)."""

    def __init__(self, ctor, ctor_args, ctor_kwargs, chain_before, chain_after, make_fn):
        self.udf = ctor(*ctor_args, **ctor_kwargs)
        self.chain_before = chain_before
        self.chain_after = chain_after
        self.fn = make_fn(self.udf)

    def process(self, block):
        if _PROFILE:
            return self._process_profiled(block)
        return self._process(block)

    def _process_profiled(self, block):
        import sys

        t0 = time.perf_counter()
        st = self.__dict__.setdefault("_st", {"gap": 0.0, "body": 0.0, "n": 0, "last": None})
        if st["last"] is not None:
            st["gap"] += t0 - st["last"]
        r = self._process(block)
        t1 = time.perf_counter()
        st["body"] += t1 - t0
        st["n"] += 1
        st["last"] = t1
        if st["n"] % 20 == 0:
            print(f"[MapWorker] {st['n']} blocks: {st['body'] / st['n'] * 1e3:.1f} ms in process, "
                  f"{st['gap'] / (st['n'] - 1) * 1e3:.1f} ms between calls", file=sys.stderr, flush=True)
        return r

    def _process(self, block):
        out = []
        for b in _apply_chain(block, self.chain_before):
            for r in self.fn(b):
                out.extend(_apply_chain(r, self.chain_after))
        res = B.concat(out) if len(out) != 1 else out[0]
        return res, {"num_rows": B.num_rows(res), "size_bytes": B.size_bytes(res), "schema": B.schema_of(res)}

    def ready(self):
        return True


# ------------------------------------------------------------------ stages
def _cluster_cpus() -> int:
    """CPUs an execution may use: the cluster's, minus ExecutionOptions'
    ``exclude_resources.cpu``, capped by its ``resource_limits.cpu``."""
    from ..core import context

    if context.local_mode:
        return 1
    ctx = DataContext.get_current()
    try:
        from ..core.api import cluster_resources

        n = float(cluster_resources().get("CPU", 1)) - ctx.excluded_cpus()
    except Exception:
        n = 4.0
    cpu_limit = ctx.resource_limits()[0]
    if cpu_limit is not None:
        n = min(n, float(cpu_limit))
    return max(1, int(n))


def _cpu_limited_inflight(default: int) -> int:
    """Tasks in flight per operator under ExecutionOptions' CPU limit."""
    cpu_limit = DataContext.get_current().resource_limits()[0]
    if cpu_limit is not None and cpu_limit != float("inf"):
        return max(1, min(default, int(cpu_limit)))
    return default


def _retire(inflight: collections.deque, preserve_order: bool, block: bool = True):
    """Pop one finished (ref, meta_ref, tag) entry: the oldest one (order kept) or,
    without order preservation, whichever finished first (``block=False``: only if
    one already has)."""
    from ..core.api import wait

    if preserve_order:
        if not block:
            ready, _ = wait([inflight[0][1]], num_returns=1, timeout=0)
            if not ready:
                return None
        return inflight.popleft()
    ready, _ = wait([e[1] for e in inflight], num_returns=1, timeout=None if block else 0)
    if not ready:
        return None
    r0 = ready[0]
    for i, e in enumerate(inflight):
        if e[1] is r0 or e[1] == r0:
            del inflight[i]
            return e
    return inflight.popleft()


def task_stage(inputs: Iterator, chain: List[Callable], resources: Dict[str, Any],
               max_inflight: Optional[int] = None, op=None) -> Iterator[Tuple[Any, dict]]:
    """inputs yield read callables or (block_ref, meta); yields (block_ref, meta).

    Submission stops at ``max_inflight`` tasks or when the operator's object-store
    budget (``op.can_submit``, see resource_manager.py) is used up."""
    from ..core.api import get

    ctx = DataContext.get_current()
    max_inflight = _cpu_limited_inflight(max_inflight or ctx.max_tasks_in_flight_per_op or max(2, 2 * _cluster_cpus()))
    keep_order = ctx.execution_preserve_order
    if op is not None:
        op.warmup_cap = max(2, min(max_inflight, _cluster_cpus()))
    task = _get_remote_task().options(**resources) if resources else _get_remote_task()
    inflight = collections.deque()

    def out(e):
        meta = get(e[1])
        if op is not None:
            op.on_output(meta)
            op.on_pulled(meta)
        return e[0], meta

    for item in inputs:
        src = item[0] if isinstance(item, tuple) else item
        while inflight and (len(inflight) >= max_inflight or (op is not None and not op.can_submit())):
            yield out(_retire(inflight, keep_order))
        ref, meta_ref = task.remote(src, chain)
        if op is not None:
            op.on_submit()
        inflight.append((ref, meta_ref, None))
    while inflight:
        yield out(_retire(inflight, keep_order))


def actor_stage(inputs: Iterator, spec: dict, op=None) -> Iterator[Tuple[Any, dict]]:
    """Actor-pool map with autoscaling between ``min_size`` and ``max_size`` actors
    (reference: actor_pool_map_operator.py + autoscaling_actor_pool.py).

    Starts ``initial`` actors; a new actor is started (one at a time) when every
    ready actor has ``per_actor`` tasks in flight and more input is waiting; work
    only goes to actors that are ready, so a slow-starting actor never holds up
    the first outputs. Once the input is exhausted, actors that have no work left
    are released immediately (scale-down) instead of at the end of the stage."""
    from ..core.api import get, kill, remote, wait

    ctx = DataContext.get_current()
    keep_order = ctx.execution_preserve_order
    max_size = max(1, int(spec.get("max_size") or spec["size"]))
    gpu_limit = ctx.resource_limits()[1]
    per_gpu = float(spec["resources"].get("num_gpus") or 0)
    if gpu_limit is not None and gpu_limit != float("inf") and per_gpu > 0:
        max_size = max(1, min(max_size, int(gpu_limit / per_gpu)))  # ExecutionOptions GPU limit
    min_size = max(1, min(max_size, int(spec.get("min_size") or spec["size"])))
    initial = max(min_size, min(max_size, int(spec.get("initial_size") or min_size)))
    per_actor = spec.get("max_tasks_in_flight") or ctx.actor_max_tasks_in_flight
    opts = {k: v for k, v in spec["resources"].items() if v}
    # a map actor that dies (OOM kill, node loss) is restarted, its UDF re-constructed,
    # and the batches it owed are run again, so every row is produced exactly once
    # (reference: actor_pool_map_operator.py:351-357); ray_remote_args may override
    opts.setdefault("max_restarts", -1)
    opts.setdefault("max_task_retries", -1)
    Actor = remote(**opts)(_MapWorker)

    actors: List[Any] = []        # ready actors
    load: List[int] = []
    starting: Dict[Any, Any] = {}  # ready-ref -> actor handle
    inflight = collections.deque()  # (ref, meta_ref, actor_handle)

    def start_actor():
        a = Actor.remote(spec["ctor"], spec["ctor_args"], spec["ctor_kwargs"], spec["before"],
                         spec["after"], spec["make_fn"])
        starting[a.ready.remote()] = a
        if op is not None:
            op.scale_ups += 1

    def poll_starting(block: bool):
        if not starting:
            return
        ready, _ = wait(list(starting), num_returns=1, timeout=None if block else 0)
        for r in ready:
            a = starting.pop(r)
            get(r)  # surfaces constructor errors
            actors.append(a)
            load.append(0)
        if op is not None:
            op.set_actors(len(actors))

    def retire(block=True):
        e = _retire(inflight, keep_order, block)
        if e is None:
            return None
        r, m, a = e
        meta = get(m)
        load[actors.index(a)] -= 1
        if op is not None:
            op.on_output(meta)
            op.on_pulled(meta)
        return r, meta

    for _ in range(initial):
        start_actor()
    try:
        for item in inputs:
            ref_in = item[0]
            while True:
                poll_starting(block=not actors and not inflight)
                free = [i for i in range(len(actors)) if load[i] < per_actor]
                if free and (op is None or op.can_submit() or not inflight):
                    break
                if not free and len(actors) + len(starting) < max_size and not starting:
                    start_actor()  # every ready actor is saturated: scale up
                # block until an output (the oldest one if order is kept) or a new actor is ready
                heads = ([inflight[0][1]] if keep_order else [e[1] for e in inflight]) if inflight else []
                wait(heads + list(starting), num_returns=1, timeout=None)
                if inflight:
                    out = retire(block=False)
                    if out is not None:
                        yield out
            ai = min(free, key=lambda i: load[i])
            r, m = actors[ai].process.options(num_returns=2).remote(ref_in)
            load[ai] += 1
            if op is not None:
                op.on_submit()
            inflight.append((r, m, actors[ai]))
        # input exhausted: drain, releasing actors as they go idle
        for a in starting.values():
            kill(a)
        starting.clear()
        while inflight:
            out = retire()
            yield out
            for i in range(len(actors) - 1, -1, -1):
                if load[i] == 0 and not any(e[2] is actors[i] for e in inflight):
                    kill(actors[i])
                    del actors[i]
                    del load[i]
                    if op is not None:
                        op.scale_downs += 1
                        op.set_actors(len(actors))
    finally:
        for a in list(actors) + list(starting.values()):
            try:
                kill(a)
            except Exception:
                pass


def limit_stage(inputs: Iterator, n: int) -> Iterator[Tuple[Any, dict]]:
    from ..core.api import put

    seen = 0
    if n <= 0:
        return
    for ref, meta in inputs:
        rows = meta["num_rows"]
        if seen + rows <= n:
            seen += rows
            yield ref, meta
        else:
            from ..core.api import get

            blk = B.slice_block(get(ref), 0, n - seen)
            seen = n
            yield put(blk), {"num_rows": B.num_rows(blk), "size_bytes": B.size_bytes(blk),
                             "schema": B.schema_of(blk)}
        if seen >= n:
            return
