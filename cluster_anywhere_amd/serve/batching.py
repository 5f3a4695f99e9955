"""``@serve.batch``: coalesce concurrent calls into one batched call
(reference: python/ray/serve/batching.py).

Each decorated method gets one queue per instance. A flusher task waits for the
first request, then gathers until ``max_batch_size`` items or
``batch_wait_timeout_s`` elapsed, calls the user function once with lists (one
list per positional argument) and scatters the returned list back to the
callers' futures."""
from __future__ import annotations

import asyncio
import functools
import inspect
from typing import Any, Callable, List, Optional


class _BatchQueue:
    def __init__(self, func, max_batch_size, timeout_s):
        self.func = func
        self.max_batch_size = max_batch_size
        self.timeout_s = timeout_s
        self.queue: "asyncio.Queue" = asyncio.Queue()
        self.task = asyncio.get_event_loop().create_task(self._loop())
        self.batch_sizes: List[int] = []

    async def _loop(self):
        while True:
            first = await self.queue.get()
            batch = [first]
            loop = asyncio.get_event_loop()
            deadline = loop.time() + self.timeout_s
            while len(batch) < self.max_batch_size:
                remaining = deadline - loop.time()
                if remaining <= 0:
                    while len(batch) < self.max_batch_size and not self.queue.empty():
                        batch.append(self.queue.get_nowait())
                    break
                try:
                    batch.append(await asyncio.wait_for(self.queue.get(), remaining))
                except asyncio.TimeoutError:
                    break
            self.batch_sizes.append(len(batch))
            await self._run(batch)

    async def _run(self, batch):
        self_obj = batch[0][0]
        nargs = len(batch[0][1])
        cols = [[b[1][i] for b in batch] for i in range(nargs)]
        kw = {}
        for k in batch[0][2]:
            kw[k] = [b[2][k] for b in batch]
        futs = [b[3] for b in batch]
        try:
            args = ([self_obj] if self_obj is not None else []) + cols
            out = self.func(*args, **kw)
            if inspect.isawaitable(out):
                out = await out
            out = list(out)
            if len(out) != len(batch):
                raise ValueError(f"batched function returned {len(out)} results for a batch of {len(batch)}")
            for f, r in zip(futs, out):
                if not f.done():
                    f.set_result(r)
        except BaseException as e:  # noqa
            for f in futs:
                if not f.done():
                    f.set_exception(e)


def batch(_func: Optional[Callable] = None, max_batch_size: int = 10, batch_wait_timeout_s: float = 0.01):
    if max_batch_size < 1:
        raise ValueError("max_batch_size must be >= 1")

    def deco(func):
        params = list(inspect.signature(func).parameters)
        is_method = bool(params) and params[0] == "self"
        attr = f"__serve_batch_queue_{func.__name__}"
        holder = {}

        @functools.wraps(func)
        async def wrapper(*args, **kwargs):
            if is_method:
                self_obj, rest = args[0], args[1:]
                q = self_obj.__dict__.get(attr)
                if q is None:
                    q = _BatchQueue(func, wrapper._max_batch_size, wrapper._timeout)
                    self_obj.__dict__[attr] = q
            else:
                self_obj, rest = None, args
                q = holder.get("q")
                if q is None:
                    q = holder["q"] = _BatchQueue(func, wrapper._max_batch_size, wrapper._timeout)
            q.max_batch_size, q.timeout_s = wrapper._max_batch_size, wrapper._timeout
            fut = asyncio.get_event_loop().create_future()
            q.queue.put_nowait((self_obj, rest, kwargs, fut))
            return await fut

        wrapper._max_batch_size = max_batch_size
        wrapper._timeout = batch_wait_timeout_s

        def set_max_batch_size(n):
            wrapper._max_batch_size = n

        def set_batch_wait_timeout_s(t):
            wrapper._timeout = t

        wrapper.set_max_batch_size = set_max_batch_size
        wrapper.set_batch_wait_timeout_s = set_batch_wait_timeout_s
        wrapper._serve_batch = True
        return wrapper

    if _func is not None and callable(_func):
        return deco(_func)
    return deco
