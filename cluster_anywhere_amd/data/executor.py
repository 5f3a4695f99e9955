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
    if isinstance(blocks, dict):
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
    from ..core import context

    if context.local_mode:
        return 1
    try:
        from ..core.api import cluster_resources

        return max(1, int(cluster_resources().get("CPU", 1)))
    except Exception:
        return 4


def task_stage(inputs: Iterator, chain: List[Callable], resources: Dict[str, Any],
               max_inflight: Optional[int] = None) -> Iterator[Tuple[Any, dict]]:
    """inputs yield read callables or (block_ref, meta); yields (block_ref, meta)."""
    from ..core.api import get

    ctx = DataContext.get_current()
    max_inflight = max_inflight or ctx.max_tasks_in_flight_per_op or max(2, 2 * _cluster_cpus())
    task = _get_remote_task().options(**resources) if resources else _get_remote_task()
    inflight = collections.deque()
    for item in inputs:
        src = item[0] if isinstance(item, tuple) else item
        ref, meta_ref = task.remote(src, chain)
        inflight.append((ref, meta_ref))
        while len(inflight) >= max_inflight:
            r, m = inflight.popleft()
            yield r, get(m)
    while inflight:
        r, m = inflight.popleft()
        yield r, get(m)


def actor_stage(inputs: Iterator, spec: dict) -> Iterator[Tuple[Any, dict]]:
    from ..core.api import get, kill, remote, wait

    size = spec["size"]
    per_actor = spec.get("max_tasks_in_flight") or DataContext.get_current().actor_max_tasks_in_flight
    opts = {k: v for k, v in spec["resources"].items() if v}
    Actor = remote(**opts)(_MapWorker) if opts else remote(_MapWorker)
    actors = [Actor.remote(spec["ctor"], spec["ctor_args"], spec["ctor_kwargs"], spec["before"],
                           spec["after"], spec["make_fn"]) for _ in range(size)]
    load = [0] * size
    inflight = collections.deque()  # (ref, meta_ref, actor_idx)
    try:
        for item in inputs:
            ref_in = item[0]
            while min(load) >= per_actor:
                r, m, ai = inflight.popleft()
                meta = get(m)
                load[ai] -= 1
                yield r, meta
            ai = min(range(size), key=lambda i: load[i])
            r, m = actors[ai].process.options(num_returns=2).remote(ref_in)
            load[ai] += 1
            inflight.append((r, m, ai))
        while inflight:
            r, m, ai = inflight.popleft()
            yield r, get(m)
            load[ai] -= 1
    finally:
        for a in actors:
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
