"""Dataset (reference: python/ray/data/dataset.py).

Lazy: transformations append operators to a plan; consumption (iteration,
take, write, materialize, ...) runs the plan through the streaming executor
(:mod:`.executor`). Blocks are dict-of-numpy (:mod:`.block`) living in the
shared-memory object store.
"""
from __future__ import annotations

import asyncio
import builtins
import collections
import inspect
import itertools
import math
import os
import random as _random
import threading
import time
from typing import Any, Callable, Dict, Iterable, Iterator, List, Optional, Tuple, Union

import numpy as np

from . import block as B
from .aggregate import AggregateFn, Count, Max, Mean, Min, Std, Sum
from .context import DataContext
from .executor import actor_stage, limit_stage, task_stage
from .resource_manager import ResourceManager


class ActorPoolStrategy:
    """Fixed (``size``) or autoscaling (``min_size``..``max_size``) actor pool
    (reference: python/ray/data/_internal/compute.py ActorPoolStrategy)."""

    def __init__(self, size: Optional[int] = None, min_size: Optional[int] = None,
                 max_size: Optional[int] = None, initial_size: Optional[int] = None,
                 max_tasks_in_flight_per_actor: Optional[int] = None):
        if size is not None:
            min_size = max_size = size
        self.min_size = max(1, min_size or 1)
        self.max_size = max(self.min_size, max_size or self.min_size)
        self.initial_size = initial_size
        self.size = self.max_size
        self.max_tasks_in_flight_per_actor = max_tasks_in_flight_per_actor


class TaskPoolStrategy:
    def __init__(self, size: Optional[int] = None):
        self.size = size


class Schema:
    def __init__(self, types: Dict[str, str]):
        self._types = dict(types)

    @property
    def names(self) -> List[str]:
        return list(self._types)

    @property
    def types(self) -> List[str]:
        return list(self._types.values())

    def __repr__(self):
        return "Schema(" + ", ".join(f"{k}: {v}" for k, v in self._types.items()) + ")"

    def __eq__(self, other):
        return isinstance(other, Schema) and other._types == self._types


# ---------------------------------------------------------------- block fns
def _row_map(fn):
    def f(b):
        rows = [fn(r) for r in B.iter_rows(b)]
        yield B.from_rows(rows)
    return f


def _row_flat_map(fn):
    def f(b):
        rows = [x for r in B.iter_rows(b) for x in fn(r)]
        yield B.from_rows(rows)
    return f


def _row_filter(fn):
    def f(b):
        keep = np.array([bool(fn(r)) for r in B.iter_rows(b)], dtype=bool)
        yield B.take_indices(b, np.nonzero(keep)[0]) if len(keep) else b
    return f


def _batch_map(fn, batch_size, batch_format, fn_args, fn_kwargs, zero_copy_batch=False):
    def f(b):
        if not b:
            return
        for sub in B.batches(b, batch_size):
            batch = B.to_batch(sub, batch_format)
            if not zero_copy_batch and isinstance(batch, dict):
                batch = {k: np.array(v, copy=True) if not v.flags.writeable else v for k, v in batch.items()}
            out = fn(batch, *fn_args, **fn_kwargs)
            if inspect.isasyncgen(out):
                yield from _drain_async(out, batch_size)
            elif inspect.iscoroutine(out):
                yield B.from_batch(_loop().run_until_complete(out))
            elif inspect.isgenerator(out):
                for o in out:
                    yield B.from_batch(o)
            else:
                yield B.from_batch(out)
    return f


_tls = threading.local()


def _loop():
    """One event loop per executing thread, kept across batches so async UDF state
    (HTTP sessions, engine handles) survives between calls."""
    lp = getattr(_tls, "loop", None)
    if lp is None or lp.is_closed():
        lp = asyncio.new_event_loop()
        _tls.loop = lp
    return lp


def _drain_async(agen, batch_size):
    """Async-generator UDF (reference: the LLM batch stages stream rows one by one,
    llm/_internal/batch/stages/base.py:83): outputs are coalesced into blocks of
    ``batch_size`` rows (all of them when ``batch_size`` is None)."""
    lp = _loop()
    pending: List[Any] = []
    rows = 0

    def flush():
        blocks = [B.from_batch(o) for o in pending]
        pending.clear()
        return blocks[0] if len(blocks) == 1 else B.concat(blocks)

    while True:
        try:
            o = lp.run_until_complete(agen.__anext__())
        except StopAsyncIteration:
            break
        pending.append(o)
        rows += len(next(iter(o.values()))) if isinstance(o, dict) and o else 1
        if batch_size and rows >= batch_size:
            yield flush()
            rows = 0
    if pending:
        yield flush()


def _make_class_fn(batch_size, batch_format, fn_args, fn_kwargs, zero_copy_batch):
    def make(udf):
        return _batch_map(udf, batch_size, batch_format, fn_args, fn_kwargs, zero_copy_batch)
    return make


def _resources(num_cpus=None, num_gpus=None, resources=None, memory=None):
    r = {}
    if num_cpus is not None:
        r["num_cpus"] = num_cpus
    if num_gpus:
        r["num_gpus"] = num_gpus
    if resources:
        r["resources"] = resources
    if memory:
        r["memory"] = memory
    return r


def _meta(b):
    return {"num_rows": B.num_rows(b), "size_bytes": B.size_bytes(b), "schema": B.schema_of(b)}


# ---------------------------------------------------------------- remote helpers
def _rf(fn, **opts):
    from ..core.api import remote

    return remote(**opts)(fn) if opts else remote(fn)


def _shuffle_map(block, n, seed):
    rng = np.random.default_rng(seed)
    rows = B.num_rows(block)
    assign = rng.integers(0, n, size=rows) if rows else np.zeros(0, dtype=np.int64)
    return tuple(B.take_indices(block, np.nonzero(assign == i)[0]) for i in range(n)) if n > 1 else \
        B.take_indices(block, rng.permutation(rows))


def _shuffle_reduce(seed, *parts):
    b = B.concat([p for p in parts if p])
    rng = np.random.default_rng(seed)
    b = B.take_indices(b, rng.permutation(B.num_rows(b))) if b else b
    return b, _meta(b)


def _range_partition(block, key, bounds, descending):
    if not block:
        return tuple({} for _ in range(len(bounds) + 1)) if bounds else {}
    k = B.col(block, key)
    idx = np.searchsorted(np.asarray(bounds), k, side="right") if bounds else np.zeros(len(k), dtype=np.int64)
    n = len(bounds) + 1
    if descending:
        idx = (n - 1) - idx
    parts = tuple(B.take_indices(block, np.nonzero(idx == i)[0]) for i in range(n))
    return parts if n > 1 else parts[0]


def _sort_reduce(key, descending, *parts):
    b = B.concat([p for p in parts if p])
    if b:
        order = np.argsort(B.col(b, key), kind="stable")
        if descending:
            order = order[::-1]
        b = B.take_indices(b, order)
    return b, _meta(b)


def _hash_partition(block, keys, n):
    if not block:
        return tuple({} for _ in range(n)) if n > 1 else {}
    if isinstance(keys, str):
        keys = [keys]
    h = np.zeros(B.num_rows(block), dtype=np.uint64)
    for k in keys:
        col = B.col(block, k)
        hv = np.array([hash(x.item() if isinstance(x, np.generic) else x) for x in col], dtype=np.int64).view(np.uint64)
        h = h * np.uint64(1000003) ^ hv
    idx = (h % np.uint64(n)).astype(np.int64)
    parts = tuple(B.take_indices(block, np.nonzero(idx == i)[0]) for i in range(n))
    return parts if n > 1 else parts[0]


def _group_reduce(keys, aggs, map_fn, batch_format, *parts):
    b = B.concat([p for p in parts if p])
    if not b:
        return {}, _meta({})
    if isinstance(keys, str):
        keys = [keys]
    keycols = [B.col(b, k) for k in keys]
    tuples = list(zip(*[c.tolist() for c in keycols]))
    groups = collections.OrderedDict()
    for i, t in enumerate(tuples):
        groups.setdefault(t, []).append(i)
    ordered = sorted(groups.items(), key=lambda kv: kv[0])
    if map_fn is not None:
        outs = []
        for t, idx in ordered:
            g = B.take_indices(b, np.asarray(idx))
            outs.append(B.from_batch(map_fn(B.to_batch(g, batch_format))))
        out = B.concat(outs)
        return out, _meta(out)
    cols = {k: [] for k in keys}
    for a in aggs:
        cols[a.name] = []
    for t, idx in ordered:
        g = B.take_indices(b, np.asarray(idx))
        for k, v in zip(keys, t):
            cols[k].append(v)
        for a in aggs:
            cols[a.name].append(a.finalize(a.accumulate_block(a.init(t), B.to_numpy(g))))
    out = {k: B._to_array(v) for k, v in cols.items()}
    return out, _meta(out)


def _agg_block(block, aggs):
    block = B.to_numpy(block) if block else block
    return [a.accumulate_block(a.init(None), block) if block else a.init(None) for a in aggs]


def _slice_concat(specs):
    """specs: list of (block_ref, start, end) — nested refs, resolved here."""
    from ..core.api import get

    blocks = get([r for r, _, _ in specs]) if specs else []
    out = B.concat([B.slice_block(b, s, e) for b, (_, s, e) in zip(blocks, specs)])
    return out, _meta(out)


def _datasink_write_task(sink, idx, op_name, *blocks):
    """Remote write task of ``write_datasink``: (sink's return, rows, bytes)."""
    from .datasource import TaskContext

    blocks = [b for b in blocks]
    ret = sink.write(iter(blocks), TaskContext(task_idx=idx, op_name=f"Write({op_name})"))
    return ret, sum(B.num_rows(b) for b in blocks), sum(B.size_bytes(b) for b in blocks)


def _write_block(block, path, fmt, idx, kw):
    if path:
        os.makedirs(path, exist_ok=True)
    fn = os.path.join(path, f"{idx:06d}.{ 'npy' if fmt == 'numpy' else fmt}")
    if fmt == "parquet":
        import pyarrow as pa
        import pyarrow.parquet as pq

        pq.write_table(B.to_batch(block, "pyarrow"), fn, **kw)
    elif fmt == "csv":
        B.to_batch(block, "pandas").to_csv(fn, index=False, **kw)
    elif fmt == "json":
        B.to_batch(block, "pandas").to_json(fn, orient="records", lines=True, **kw)
    elif fmt == "numpy":
        col = kw.get("column") or B.columns(block)[0]
        np.save(fn, B.col(block, col))
    elif fmt in ("tfrecords", "webdataset"):
        from . import formats

        fn = fn[: -len(fmt)] + ("tfrecords" if fmt == "tfrecords" else "tar")
        if fmt == "tfrecords":
            formats.write_tfrecords(B.iter_rows(block), fn)
        else:
            formats.write_webdataset(B.iter_rows(block), fn, start_key=idx * 1_000_000)
    elif fmt == "images":
        from PIL import Image

        col, ext = kw["column"], kw.get("file_format", "png")
        fn = []
        for j, row in enumerate(B.iter_rows(block)):
            f = os.path.join(path, f"{idx:06d}_{j:06d}.{ext}")
            Image.fromarray(np.asarray(row[col])).save(f)
            fn.append(f)
    elif fmt == "sql":
        conn = kw["connection_factory"]()
        try:
            cur = conn.cursor()
            cur.executemany(kw["sql"], [tuple(B._scalar(v) for v in r.values()) for r in B.iter_rows(block)])
            conn.commit()
        finally:
            conn.close()
    return fn


class Dataset:
    def __init__(self, source, ops=None):
        self._source = source  # ("read", [callables]) | ("refs", [(ref, meta)])
        self._ops = ops or []
        self._materialized = None
        self._stats = {}

    def __getstate__(self):
        st = dict(self.__dict__)
        st.pop("_rm", None)  # per-execution accounting (holds a lock) stays local
        return st

    def __setstate__(self, st):
        self.__dict__.update(st)

    def _with(self, op) -> "Dataset":
        return Dataset(self._source if self._materialized is None else ("refs", self._materialized),
                       (self._ops if self._materialized is None else []) + [op])

    # ------------------------------------------------------------ execution
    def _execute(self) -> Iterator[Tuple[Any, dict]]:
        if self._materialized is not None:
            yield from iter(self._materialized)
            return
        t0 = time.time()
        kind, items = self._source
        stream = iter(items)
        is_refs = kind == "refs"
        chain: List[Callable] = []
        res = None
        rm = ResourceManager.for_execution()
        self._rm = rm

        def _name(fns, read):
            names = [getattr(f, "__caamd_name__", None) or getattr(f, "__name__", "map") for f in fns]
            return "->".join((["Read"] if read else []) + names) or "Read"

        def flush(stream, chain, res, is_refs):
            if chain or not is_refs:
                return task_stage(stream, list(chain), res or {}, op=rm.op(_name(chain, not is_refs))), True
            return stream, is_refs

        for op in self._ops:
            t = op[0]
            if t == "map":
                _, fn, r, conc = op
                if chain and (r or {}) != (res or {}):
                    stream, is_refs = flush(stream, chain, res, is_refs)
                    chain = []
                if conc:
                    stream, is_refs = flush(stream, chain, res, is_refs)
                    stream = task_stage(stream, [fn], r or {}, max_inflight=conc, op=rm.op(_name([fn], False)))
                    chain, res = [], None
                    continue
                chain.append(fn)
                res = r
            elif t == "actor":
                stream, is_refs = flush(stream, chain, res, is_refs)
                chain, res = [], None
                stream = actor_stage(stream, op[1], op=rm.op(
                    f"ActorPoolMap({getattr(op[1]['ctor'], '__name__', 'udf')})"))
            elif t == "all2all":
                stream, is_refs = flush(stream, chain, res, is_refs)
                chain, res = [], None
                stream = iter(op[1](list(stream)))
            elif t == "limit":
                stream, is_refs = flush(stream, chain, res, is_refs)
                chain, res = [], None
                stream = limit_stage(stream, op[1])
        stream, is_refs = flush(stream, chain, res, is_refs)
        n = 0
        rows = 0
        for ref, meta in stream:
            n += 1
            rows += meta["num_rows"]
            yield ref, meta
        self._stats = {"num_blocks": n, "num_rows": rows, "wall_time_s": time.time() - t0}

    def _blocks(self) -> Iterator[B.Block]:
        from ..core.api import get

        for ref, meta in self._execute():
            yield get(ref)

    def materialize(self) -> "MaterializedDataset":
        refs = list(self._execute())
        ds = MaterializedDataset(("refs", refs))
        ds._materialized = refs
        ds._stats = dict(self._stats)
        return ds

    # ------------------------------------------------------------ transforms
    def map(self, fn, *, compute=None, fn_args=(), fn_kwargs=None, fn_constructor_args=(),
            fn_constructor_kwargs=None, num_cpus=None, num_gpus=None, concurrency=None, **kw):
        if inspect.isclass(fn):
            return self._actor_map(fn, None, None, fn_args, fn_kwargs or {}, fn_constructor_args,
                                   fn_constructor_kwargs or {}, num_cpus, num_gpus, concurrency, compute,
                                   row_mode="map")
        return self._with(("map", _row_map(fn), _resources(num_cpus, num_gpus), concurrency))

    def flat_map(self, fn, *, num_cpus=None, num_gpus=None, concurrency=None, **kw):
        return self._with(("map", _row_flat_map(fn), _resources(num_cpus, num_gpus), concurrency))

    def filter(self, fn=None, *, expr=None, num_cpus=None, concurrency=None, **kw):
        return self._with(("map", _row_filter(fn), _resources(num_cpus), concurrency))

    def map_batches(self, fn, *, batch_size: Union[int, None, str] = "default", compute=None,
                    batch_format: Optional[str] = "default", zero_copy_batch: bool = False,
                    fn_args: Iterable[Any] = (), fn_kwargs: Optional[Dict] = None,
                    fn_constructor_args: Iterable[Any] = (), fn_constructor_kwargs: Optional[Dict] = None,
                    num_cpus=None, num_gpus=None, memory=None, concurrency=None, resources=None, **kw):
        if batch_size == "default":
            batch_size = 1024 if not num_gpus else None
        if inspect.isclass(fn) or isinstance(compute, ActorPoolStrategy):
            return self._actor_map(fn, batch_size, batch_format, fn_args, fn_kwargs or {},
                                   fn_constructor_args, fn_constructor_kwargs or {}, num_cpus, num_gpus,
                                   concurrency, compute, zero_copy_batch=zero_copy_batch, resources=resources)
        f = _batch_map(fn, batch_size, batch_format, tuple(fn_args), fn_kwargs or {}, zero_copy_batch)
        conc = concurrency if isinstance(concurrency, int) else None
        return self._with(("map", f, _resources(num_cpus, num_gpus, resources, memory), conc))

    def _actor_map(self, cls, batch_size, batch_format, fn_args, fn_kwargs, ctor_args, ctor_kwargs,
                   num_cpus, num_gpus, concurrency, compute, row_mode=None, zero_copy_batch=False,
                   resources=None):
        initial = None
        if isinstance(compute, ActorPoolStrategy):
            lo, hi, initial = compute.min_size, compute.max_size, compute.initial_size
        elif isinstance(concurrency, tuple):
            lo, hi = concurrency[0], concurrency[1]
            initial = concurrency[2] if len(concurrency) > 2 else None
        else:
            lo = hi = concurrency or 1
        size = hi
        if row_mode == "map":
            def make(udf):
                return _row_map(udf)
        else:
            make = _make_class_fn(batch_size, batch_format, tuple(fn_args), fn_kwargs, zero_copy_batch)
        spec = {"size": size, "min_size": lo, "max_size": hi, "initial_size": initial, "ctor": cls, "ctor_args": tuple(ctor_args), "ctor_kwargs": ctor_kwargs,
                "before": [], "after": [], "make_fn": make,
                "resources": {"num_cpus": num_cpus if num_cpus is not None else (0 if num_gpus else 1),
                              "num_gpus": num_gpus or 0, "resources": resources},
                "max_tasks_in_flight": getattr(compute, "max_tasks_in_flight_per_actor", None)}
        return self._with(("actor", spec))

    def add_column(self, col: str, fn: Callable, *, batch_format="pandas", **kw):
        def f(batch):
            out = dict(batch) if isinstance(batch, dict) else batch
            if isinstance(out, dict):
                out[col] = np.asarray(fn(batch))
            else:
                out[col] = fn(batch)
            return out
        return self.map_batches(f, batch_format=batch_format, batch_size=None)

    def drop_columns(self, cols: List[str], **kw):
        cols = [cols] if isinstance(cols, str) else cols
        return self.map_batches(lambda b: {k: v for k, v in b.items() if k not in cols}, batch_size=None,
                                zero_copy_batch=True)

    def select_columns(self, cols: List[str], **kw):
        cols = [cols] if isinstance(cols, str) else cols
        return self.map_batches(lambda b: {k: b[k] for k in cols}, batch_size=None, zero_copy_batch=True)

    def rename_columns(self, names: Dict[str, str], **kw):
        return self.map_batches(lambda b: {names.get(k, k): v for k, v in b.items()}, batch_size=None,
                                zero_copy_batch=True)

    def random_sample(self, fraction: float, *, seed: Optional[int] = None):
        def f(b):
            rng = np.random.default_rng(seed)
            keep = rng.random(B.num_rows(b)) < fraction
            return B.take_indices(b, np.nonzero(keep)[0])
        return self.map_batches(f, batch_size=None, zero_copy_batch=True)

    def limit(self, n: int) -> "Dataset":
        return self._with(("limit", n))

    # ------------------------------------------------------------ all-to-all
    def random_shuffle(self, *, seed: Optional[int] = None, num_blocks: Optional[int] = None, **kw):
        def run(inputs):
            from ..core.api import get

            if not inputs:
                return []
            n = num_blocks or len(inputs)
            base = seed if seed is not None else _random.randrange(1 << 30)
            m = _rf(_shuffle_map, num_returns=n)
            parts = [m.remote(ref, n, base + i) for i, (ref, _) in enumerate(inputs)]
            if n == 1:
                parts = [[p] for p in parts]
            red = _rf(_shuffle_reduce, num_returns=2)
            outs = [red.remote(base + 7919 * (j + 1), *[p[j] for p in parts]) for j in range(n)]
            return [(r, get(mm)) for r, mm in outs]
        return self._with(("all2all", run))

    def randomize_block_order(self, *, seed: Optional[int] = None):
        def run(inputs):
            rng = _random.Random(seed)
            inputs = list(inputs)
            rng.shuffle(inputs)
            return inputs
        return self._with(("all2all", run))

    def repartition(self, num_blocks: int, *, shuffle: bool = False, **kw):
        if shuffle:
            return self.random_shuffle(num_blocks=num_blocks)

        def run(inputs):
            from ..core.api import get

            total = sum(m["num_rows"] for _, m in inputs)
            if total == 0:
                return inputs[:1]
            per = [total // num_blocks + (1 if i < total % num_blocks else 0) for i in range(num_blocks)]
            out, bi, off = [], 0, 0
            task = _rf(_slice_concat, num_returns=2)
            for want in per:
                specs = []
                while want > 0 and bi < len(inputs):
                    ref, m = inputs[bi]
                    avail = m["num_rows"] - off
                    take = min(avail, want)
                    specs.append((ref, off, off + take))
                    want -= take
                    off += take
                    if off >= m["num_rows"]:
                        bi += 1
                        off = 0
                r, mm = task.remote(specs)
                out.append((r, mm))
            return [(r, get(mm)) for r, mm in out]
        return self._with(("all2all", run))

    def sort(self, key: Union[str, List[str]], descending: bool = False, **kw):
        key = key[0] if isinstance(key, list) else key

        def run(inputs):
            from ..core.api import get

            inputs = [x for x in inputs if x[1]["num_rows"] > 0]
            if not inputs:
                return []
            n = len(inputs)
            samples = np.concatenate([np.asarray(get(r)[key])[:: max(1, m["num_rows"] // 16)]
                                      for r, m in inputs])
            samples.sort()
            bounds = [samples[int(len(samples) * (i + 1) / n)] for i in range(n - 1)] if n > 1 else []
            part = _rf(_range_partition, num_returns=n)
            parts = [part.remote(r, key, bounds, descending) for r, _ in inputs]
            if n == 1:
                parts = [[p] for p in parts]
            red = _rf(_sort_reduce, num_returns=2)
            outs = [red.remote(key, descending, *[p[j] for p in parts]) for j in range(n)]
            return [(r, get(mm)) for r, mm in outs]
        return self._with(("all2all", run))

    def groupby(self, key: Union[str, List[str], None]) -> "GroupedData":
        return GroupedData(self, key)

    def unique(self, column: str) -> List[Any]:
        return [r[column] for r in self.groupby(column).count().take_all()]

    def union(self, *others: "Dataset") -> "Dataset":
        def gen():
            for ds in (self,) + others:
                yield from ds._execute()
        refs = list(gen())
        return Dataset(("refs", refs))

    def zip(self, other: "Dataset") -> "Dataset":
        a = self.materialize()
        bds = other.repartition(max(1, a.num_blocks())).materialize()
        from ..core.api import get

        left = list(a._execute())
        counts = [m["num_rows"] for _, m in left]
        right_rows = B.concat([get(r) for r, _ in bds._execute()])
        out, off = [], 0
        for (ref, m), c in zip(left, counts):
            lb = B.to_numpy(get(ref))
            rb = B.to_numpy(B.slice_block(right_rows, off, off + c))
            off += c
            merged = dict(lb)
            for k, v in rb.items():
                merged[k if k not in merged else f"{k}_1"] = v
            from ..core.api import put

            out.append((put(merged), _meta(merged)))
        return Dataset(("refs", out))

    # ------------------------------------------------------------ splitting
    def split(self, n: int, *, equal: bool = False, locality_hints=None) -> List["MaterializedDataset"]:
        mat = self.materialize()
        total = mat.count()
        if equal:
            per = [total // n] * n
        else:
            per = [total // n + (1 if i < total % n else 0) for i in range(n)]
        idx = list(itertools.accumulate(per))[:-1]
        return mat.split_at_indices(idx)[:n] if not equal else mat.split_at_indices(idx + [sum(per)])[:n]

    def split_at_indices(self, indices: List[int]) -> List["MaterializedDataset"]:
        from ..core.api import get, put

        blocks = [get(r) for r, _ in self._execute()]
        full = B.concat(blocks)
        total = B.num_rows(full)
        cuts = [0] + [min(i, total) for i in indices] + [total]
        out = []
        for s, e in zip(cuts[:-1], cuts[1:]):
            b = B.slice_block(full, s, e)
            ds = MaterializedDataset(("refs", [(put(b), _meta(b))]))
            ds._materialized = ds._source[1]
            out.append(ds)
        return out

    def split_proportionately(self, proportions: List[float]):
        total = self.count()
        idx, acc = [], 0.0
        for p in proportions:
            acc += p
            idx.append(int(total * acc))
        return self.split_at_indices(idx)

    def train_test_split(self, test_size: Union[int, float], *, shuffle: bool = False,
                         seed: Optional[int] = None):
        ds = self.random_shuffle(seed=seed) if shuffle else self
        total = ds.count()
        n_test = int(test_size * total) if isinstance(test_size, float) else int(test_size)
        a, b = ds.split_at_indices([total - n_test])
        return a, b

    def streaming_split(self, n: int, *, equal: bool = False, locality_hints=None) -> List["DataIterator"]:
        from .iterator import make_streaming_split

        return make_streaming_split(self, n, equal)

    # ------------------------------------------------------------ consumption
    def iterator(self) -> "DataIterator":
        from .iterator import DataIterator

        return DataIterator(lambda: self._execute())

    def iter_rows(self) -> Iterator[Dict[str, Any]]:
        for b in self._blocks():
            yield from B.iter_rows(b)

    def iter_batches(self, *, batch_size: Optional[int] = 256, batch_format: Optional[str] = "default",
                     drop_last: bool = False, prefetch_batches: int = 1,
                     local_shuffle_buffer_size: Optional[int] = None, local_shuffle_seed=None, **kw):
        return self.iterator().iter_batches(batch_size=batch_size, batch_format=batch_format,
                                            drop_last=drop_last, prefetch_batches=prefetch_batches,
                                            local_shuffle_buffer_size=local_shuffle_buffer_size,
                                            local_shuffle_seed=local_shuffle_seed)

    def iter_torch_batches(self, *, batch_size: Optional[int] = 256, dtypes=None, device="auto",
                           collate_fn=None, drop_last: bool = False, prefetch_batches: int = 1,
                           local_shuffle_buffer_size=None, local_shuffle_seed=None, **kw):
        return self.iterator().iter_torch_batches(batch_size=batch_size, dtypes=dtypes, device=device,
                                                  collate_fn=collate_fn, drop_last=drop_last,
                                                  prefetch_batches=prefetch_batches,
                                                  local_shuffle_buffer_size=local_shuffle_buffer_size,
                                                  local_shuffle_seed=local_shuffle_seed)

    def take(self, limit: int = 20) -> List[Dict[str, Any]]:
        out = []
        for r in self.limit(limit).iter_rows():
            out.append(r)
            if len(out) >= limit:
                break
        return out

    def take_all(self, limit: Optional[int] = None) -> List[Dict[str, Any]]:
        out = list(self.iter_rows())
        if limit is not None and len(out) > limit:
            raise ValueError(f"dataset has more than {limit} rows")
        return out

    def take_batch(self, batch_size: int = 20, *, batch_format: Optional[str] = "default"):
        for b in self.limit(batch_size).iter_batches(batch_size=batch_size, batch_format=batch_format):
            return b
        return B.to_batch({}, batch_format)

    def show(self, limit: int = 20) -> None:
        for r in self.take(limit):
            print(r)

    def count(self) -> int:
        return sum(m["num_rows"] for _, m in self._execute())

    def schema(self) -> Optional[Schema]:
        for _, m in self.limit(1)._execute() if self._materialized is None else self._execute():
            if m["schema"]:
                return Schema(m["schema"])
        return None

    def columns(self) -> List[str]:
        s = self.schema()
        return s.names if s else []

    def num_blocks(self) -> int:
        if self._materialized is not None:
            return len(self._materialized)
        kind, items = self._source
        return len(items)

    def size_bytes(self) -> int:
        return sum(m["size_bytes"] for _, m in self._execute())

    def input_files(self) -> List[str]:
        return list(getattr(self, "_input_files", []))

    def stats(self) -> str:
        s = self._stats
        head = (f"Dataset: {s.get('num_blocks', '?')} blocks, {s.get('num_rows', '?')} rows, "
                f"executed in {s.get('wall_time_s', 0):.3f}s")
        rm = getattr(self, "_rm", None)
        return head + ("\n" + rm.summary() if rm is not None and rm.ops else "")

    def to_pandas(self, limit: Optional[int] = None):
        import pandas as pd

        b = B.concat(list(self._blocks()))
        df = B.to_batch(b, "pandas") if b else pd.DataFrame()
        return df if limit is None else df.head(limit)

    def to_numpy_refs(self, *, column: Optional[str] = None):
        from ..core.api import get, put

        out = []
        for r, _ in self._execute():
            b = get(r)
            out.append(put(B.col(b, column) if column else B.to_numpy(b)))
        return out

    def to_arrow_refs(self):
        from ..core.api import get, put

        return [put(B.to_batch(get(r), "pyarrow")) for r, _ in self._execute()]

    def to_pandas_refs(self):
        from ..core.api import get, put

        return [put(B.to_batch(get(r), "pandas")) for r, _ in self._execute()]

    def get_internal_block_refs(self):
        return [r for r, _ in self._execute()]

    def to_torch(self, *, label_column=None, feature_columns=None, batch_size=1, **kw):
        import torch

        ds = self

        class _It(torch.utils.data.IterableDataset):
            def __iter__(self):
                for b in ds.iter_torch_batches(batch_size=batch_size, device="cpu"):
                    feats = [b[c] for c in (feature_columns or [k for k in b if k != label_column])]
                    x = torch.stack(feats, 1) if len(feats) > 1 else feats[0]
                    yield (x, b[label_column]) if label_column else x

        return _It()

    # ------------------------------------------------------------ aggregates
    def aggregate(self, *aggs: AggregateFn) -> Dict[str, Any]:
        from ..core.api import get

        task = _rf(_agg_block)
        parts = get([task.remote(r, list(aggs)) for r, _ in self._execute()])
        out = {}
        for i, a in enumerate(aggs):
            acc = a.init(None)
            for p in parts:
                acc = a.merge(acc, p[i])
            out[a.name] = a.finalize(acc)
        return out

    def _agg1(self, agg, on):
        if isinstance(on, list):
            return {a.name: v for a, v in zip([agg(c) for c in on],
                                               self.aggregate(*[agg(c) for c in on]).values())}
        return next(iter(self.aggregate(agg(on)).values()))

    def sum(self, on=None, ignore_nulls=True):
        return self._agg1(Sum, on)

    def min(self, on=None, ignore_nulls=True):
        return self._agg1(Min, on)

    def max(self, on=None, ignore_nulls=True):
        return self._agg1(Max, on)

    def mean(self, on=None, ignore_nulls=True):
        return self._agg1(Mean, on)

    def std(self, on=None, ddof: int = 1, ignore_nulls=True):
        return self._agg1(lambda c: Std(c, ddof=ddof), on)

    # ------------------------------------------------------------ writes
    def _write(self, path, fmt, **kw):
        from ..core.api import get

        task = _rf(_write_block)
        refs = [task.remote(r, path, fmt, i, kw) for i, (r, _) in enumerate(self._execute())]
        return get(refs)

    def write_parquet(self, path: str, **kw):
        self._write(path, "parquet", **kw)

    def write_csv(self, path: str, **kw):
        self._write(path, "csv", **kw)

    def write_json(self, path: str, **kw):
        self._write(path, "json", **kw)

    def write_numpy(self, path: str, *, column: Optional[str] = None, **kw):
        self._write(path, "numpy", column=column)

    def write_tfrecords(self, path: str, **kw):
        self._write(path, "tfrecords")

    def write_webdataset(self, path: str, **kw):
        self._write(path, "webdataset")

    def write_images(self, path: str, column: str, file_format: str = "png", **kw):
        self._write(path, "images", column=column, file_format=file_format)

    def write_sql(self, sql: str, connection_factory, **kw):
        """``INSERT ... VALUES (?, ...)`` per row through DB-API ``executemany``."""
        self._write("", "sql", sql=sql, connection_factory=connection_factory)

    # ------------------------------------------------ misc reference surface
    @property
    def context(self):
        from .context import DataContext

        return DataContext.get_current()

    def copy(self) -> "Dataset":
        ds = Dataset(self._source, list(self._ops))
        ds._materialized = self._materialized
        return ds

    def has_serializable_lineage(self) -> bool:
        return self._source[0] == "read"

    def serialize_lineage(self) -> bytes:
        """The logical plan (read tasks + ops), re-executable in another job."""
        if not self.has_serializable_lineage():
            raise ValueError("lineage of datasets created from in-memory refs cannot be serialized")
        import cloudpickle

        return cloudpickle.dumps((self._source, self._ops))

    @staticmethod
    def deserialize_lineage(serialized: bytes) -> "Dataset":
        import cloudpickle  # our own serialize_lineage() output

        src, ops = cloudpickle.loads(serialized)
        return Dataset(src, ops)

    def iter_internal_ref_bundles(self):
        for r, meta in self._execute():
            yield [(r, meta)]

    def to_random_access_dataset(self, key: str, num_workers: Optional[int] = None):
        from .random_access import RandomAccessDataset

        return RandomAccessDataset(self, key, num_workers or 2)

    def iter_tf_batches(self, *a, **k):
        raise ImportError("iter_tf_batches needs tensorflow, which is not installed in this image")

    to_tf = iter_tf_batches

    def to_dask(self, *a, **k):
        raise ImportError("to_dask needs dask, which is not installed in this image")

    def to_spark(self, *a, **k):
        raise ImportError("to_spark needs pyspark, which is not installed in this image")

    def to_modin(self, *a, **k):
        raise ImportError("to_modin needs modin, which is not installed in this image")

    def to_mars(self, *a, **k):
        raise ImportError("to_mars needs mars, which is not installed in this image")

    def write_datasink(self, datasink, *, ray_remote_args: Optional[Dict[str, Any]] = None,
                       concurrency: Optional[int] = None) -> None:
        """Write through a :class:`~.datasource.Datasink`: ``on_write_start`` here,
        ``write(blocks, ctx)`` in remote tasks as the blocks stream out of the
        executor (bundled to ``min_rows_per_write`` rows when the sink sets it; at
        most ``concurrency`` tasks in flight), then ``on_write_complete`` with the
        collected :class:`~.datasource.WriteResult` -- or ``on_write_failed`` and a
        raise. Reference: dataset.py:3991."""
        from ..core.api import get, wait
        from .datasource import WriteResult
        from .executor import _cluster_cpus

        opts = dict(ray_remote_args or {})
        if not datasink.supports_distributed_writes:
            from ..runtime_context import get_runtime_context
            from ..util.scheduling_strategies import NodeAffinitySchedulingStrategy

            opts["scheduling_strategy"] = NodeAffinitySchedulingStrategy(get_runtime_context().get_node_id(),
                                                                         soft=False)
        task = _rf(_datasink_write_task, **opts)
        limit = max(1, int(concurrency or 2 * _cluster_cpus()))
        min_rows = datasink.min_rows_per_write or 0
        name = datasink.get_name()
        datasink.on_write_start()
        refs: List[Any] = []
        try:
            bundle, rows = [], 0
            running: List[Any] = []

            def submit():
                nonlocal bundle, rows, running
                ref = task.remote(datasink, len(refs), name, *bundle)
                refs.append(ref)
                running.append(ref)
                bundle, rows = [], 0
                if len(running) >= limit:  # bounded in flight: wait for one to finish
                    _, running = wait(running, num_returns=1)

            for r, meta in self._execute():
                bundle.append(r)
                rows += int(meta.get("num_rows") or 0)
                if rows >= min_rows:
                    submit()
            if bundle:
                submit()
            outs = get(refs)
        except Exception as e:  # noqa: BLE001 - reported to the sink, then raised
            datasink.on_write_failed(e)
            raise
        result = WriteResult(num_rows=sum(o[1] for o in outs), size_bytes=sum(o[2] for o in outs),
                             write_returns=[o[0] for o in outs])
        datasink.on_write_complete(result)

    def write_mongo(self, uri: str, database: str, collection: str, *,
                    ray_remote_args: Optional[Dict[str, Any]] = None, concurrency: Optional[int] = None) -> None:
        """Insert every row as a document (pymongo ``insert_many`` per block, from
        the write tasks). Reference: dataset.py write_mongo."""
        from .connectors import MongoDatasink

        self.write_datasink(MongoDatasink(uri, database, collection), ray_remote_args=ray_remote_args,
                            concurrency=concurrency)

    def write_bigquery(self, project_id: str, dataset: str, max_retry_cnt: int = 10,
                       overwrite_table: Optional[bool] = True, *,
                       ray_remote_args: Optional[Dict[str, Any]] = None, concurrency: Optional[int] = None) -> None:
        """``dataset`` = ``"<dataset>.<table>"``: the table is (re)created with the
        Dataset's schema and filled through the BigQuery REST ``tabledata.insertAll``
        API from the write tasks (retrying 429 / 5xx up to ``max_retry_cnt`` times)."""
        from .connectors import BigQueryDatasink

        sch = self.schema()
        self.write_datasink(BigQueryDatasink(project_id, dataset, dict(zip(sch.names, sch.types)) if sch else None,
                                             max_retry_cnt=max_retry_cnt, overwrite_table=overwrite_table),
                            ray_remote_args=ray_remote_args, concurrency=concurrency)

    def __repr__(self):
        return f"Dataset(num_ops={len(self._ops)}, source={self._source[0]})"

    def __iter__(self):
        raise TypeError("Datasets are not directly iterable; use iter_rows() or iter_batches().")


class MaterializedDataset(Dataset):
    pass


class GroupedData:
    def __init__(self, ds: Dataset, key):
        self._ds = ds
        self._key = key

    def _run(self, aggs, map_fn=None, batch_format="default"):
        key = self._key
        ds = self._ds

        def run(inputs):
            from ..core.api import get

            inputs = [x for x in inputs if x[1]["num_rows"] > 0]
            if not inputs:
                return []
            n = max(1, min(len(inputs), 64))
            part = _rf(_hash_partition, num_returns=n)
            parts = [part.remote(r, key, n) for r, _ in inputs]
            if n == 1:
                parts = [[p] for p in parts]
            red = _rf(_group_reduce, num_returns=2)
            outs = [red.remote(key, aggs, map_fn, batch_format, *[p[j] for p in parts]) for j in range(n)]
            res = [(r, get(m)) for r, m in outs]
            return [x for x in res if x[1]["num_rows"] > 0]
        out = ds._with(("all2all", run))
        if map_fn is None and key is not None:
            return out.sort(key if isinstance(key, str) else key[0])
        return out

    def aggregate(self, *aggs: AggregateFn) -> Dataset:
        if self._key is None:
            r = self._ds.aggregate(*aggs)
            from .read_api import from_items

            return from_items([r])
        return self._run(list(aggs))

    def count(self) -> Dataset:
        return self.aggregate(Count())

    def sum(self, on: str = None, ignore_nulls=True) -> Dataset:
        return self.aggregate(*([Sum(c) for c in on] if isinstance(on, list) else [Sum(on)]))

    def min(self, on: str = None, ignore_nulls=True) -> Dataset:
        return self.aggregate(*([Min(c) for c in on] if isinstance(on, list) else [Min(on)]))

    def max(self, on: str = None, ignore_nulls=True) -> Dataset:
        return self.aggregate(*([Max(c) for c in on] if isinstance(on, list) else [Max(on)]))

    def mean(self, on: str = None, ignore_nulls=True) -> Dataset:
        return self.aggregate(*([Mean(c) for c in on] if isinstance(on, list) else [Mean(on)]))

    def std(self, on: str = None, ddof: int = 1, ignore_nulls=True) -> Dataset:
        return self.aggregate(*([Std(c, ddof) for c in on] if isinstance(on, list) else [Std(on, ddof)]))

    def map_groups(self, fn, *, batch_format: Optional[str] = "default", **kw) -> Dataset:
        return self._run(None, map_fn=fn, batch_format=batch_format)
