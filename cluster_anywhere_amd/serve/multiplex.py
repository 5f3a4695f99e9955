"""``@serve.multiplexed``: per-replica LRU of loaded models keyed by the
request's multiplexed model id (reference: python/ray/serve/multiplex.py,
api.py:566). Replicas report the ids they hold; handles route a request to a
replica that already has its model when one exists."""
from __future__ import annotations

import asyncio
import collections
import functools
import inspect
from typing import Callable, Optional

_LOADED_ATTR = "__serve_multiplexed_models"


def multiplexed(_func: Optional[Callable] = None, max_num_models_per_replica: int = 3):
    def deco(func):
        @functools.wraps(func)
        async def wrapper(self, model_id: str):
            cache = self.__dict__.setdefault(_LOADED_ATTR, collections.OrderedDict())
            locks = self.__dict__.setdefault(_LOADED_ATTR + "_locks", {})
            if model_id in cache:
                cache.move_to_end(model_id)
                return cache[model_id]
            lock = locks.setdefault(model_id, asyncio.Lock())
            async with lock:
                if model_id in cache:
                    return cache[model_id]
                while len(cache) >= max_num_models_per_replica:
                    _, old = cache.popitem(last=False)
                    unload = getattr(old, "__del__", None)
                    del old
                m = func(self, model_id)
                if inspect.isawaitable(m):
                    m = await m
                cache[model_id] = m
                return m

        wrapper._serve_multiplexed = True
        return wrapper

    if _func is not None and callable(_func):
        return deco(_func)
    return deco


def loaded_model_ids(obj) -> list:
    d = getattr(obj, "__dict__", {})
    return list(d.get(_LOADED_ATTR, {}).keys())
