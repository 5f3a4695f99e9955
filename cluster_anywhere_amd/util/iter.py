"""Parallel iterators (reference: util/iter.py, deprecated upstream but still
exported): a ParallelIterator is a list of shards, each transformed lazily and
evaluated as one remote task per shard."""
from __future__ import annotations

import builtins
from typing import Any, Callable, Iterable, List


def _run_shard(items, fns):
    out = list(items)
    for kind, fn in fns:
        if kind == "map":
            out = [fn(x) for x in out]
        elif kind == "filter":
            out = [x for x in out if fn(x)]
        elif kind == "flatten":
            out = [y for x in out for y in x]
        elif kind == "batch":
            out = [out[i:i + fn] for i in builtins.range(0, len(out), fn)]
    return out


class LocalIterator:
    def __init__(self, gen: Iterable):
        self._it = iter(gen)

    def __iter__(self):
        return self._it

    def __next__(self):
        return next(self._it)

    def for_each(self, fn):
        return LocalIterator(fn(x) for x in self._it)

    def filter(self, fn):
        return LocalIterator(x for x in self._it if fn(x))

    def take(self, n: int) -> List[Any]:
        out = []
        for x in self._it:
            out.append(x)
            if len(out) >= n:
                break
        return out


class ParallelIterator:
    def __init__(self, shards: List[List[Any]], fns=(), name: str = "ParallelIterator"):
        self.shards, self.fns, self.name = shards, list(fns), name

    def _with(self, kind, fn, tag):
        return ParallelIterator(self.shards, self.fns + [(kind, fn)], f"{self.name}.{tag}()")

    def for_each(self, fn: Callable):
        return self._with("map", fn, "for_each")

    def filter(self, fn: Callable):
        return self._with("filter", fn, "filter")

    def flatten(self):
        return self._with("flatten", None, "flatten")

    def batch(self, n: int):
        return self._with("batch", n, "batch")

    def num_shards(self) -> int:
        return len(self.shards)

    def _refs(self):
        from ..core.api import remote

        task = remote(_run_shard)
        return [task.remote(s, self.fns) for s in self.shards]

    def gather_sync(self) -> LocalIterator:
        from ..core.api import get

        res = get(self._refs())
        return LocalIterator(x for i in builtins.range(max(map(len, res), default=0))
                             for r in res if i < len(r) for x in [r[i]])

    def gather_async(self) -> LocalIterator:
        from ..core.api import get, wait

        def gen():
            pending = self._refs()
            while pending:
                ready, pending = wait(pending, num_returns=1)
                yield from get(ready[0])
        return LocalIterator(gen())

    def take(self, n: int) -> List[Any]:
        return self.gather_sync().take(n)

    def __repr__(self):
        return f"ParallelIterator[{self.name}]"


def from_items(items: List[Any], num_shards: int = 2, repeat: bool = False) -> ParallelIterator:
    shards = [list(items[i::num_shards]) for i in builtins.range(num_shards)]
    return ParallelIterator(shards, name=f"from_items[{len(items)}, shards={num_shards}]")


def from_range(n: int, num_shards: int = 2, repeat: bool = False) -> ParallelIterator:
    return from_items(list(builtins.range(n)), num_shards)


def from_iterators(generators: List[Iterable], repeat: bool = False, name=None) -> ParallelIterator:
    return ParallelIterator([list(g) for g in generators], name=name or "from_iterators")
