"""Search-space domains (reference: python/ray/tune/search/sample.py)."""
from __future__ import annotations

import math
import random
from typing import Any, Callable, Dict, List, Sequence

import numpy as np


class Domain:
    def sample(self, spec=None, rng: random.Random = None):
        raise NotImplementedError

    def is_grid(self) -> bool:
        return False


class Float(Domain):
    def __init__(self, lower, upper, log=False, base=10, q=None, normal=None):
        self.lower, self.upper, self.log, self.base, self.q, self.normal = lower, upper, log, base, q, normal

    def sample(self, spec=None, rng=None):
        rng = rng or random
        if self.normal is not None:
            v = rng.gauss(*self.normal)
        elif self.log:
            lo, hi = math.log(self.lower, self.base), math.log(self.upper, self.base)
            v = self.base ** rng.uniform(lo, hi)
        else:
            v = rng.uniform(self.lower, self.upper)
        if self.q:
            v = round(v / self.q) * self.q
        return float(v)


class Integer(Domain):
    def __init__(self, lower, upper, log=False, base=10, q=None):
        self.lower, self.upper, self.log, self.base, self.q = lower, upper, log, base, q

    def sample(self, spec=None, rng=None):
        rng = rng or random
        if self.log:
            lo, hi = math.log(self.lower, self.base), math.log(self.upper, self.base)
            v = int(self.base ** rng.uniform(lo, hi))
        else:
            v = rng.randrange(self.lower, self.upper)
        if self.q:
            v = int(round(v / self.q) * self.q)
        return v


class Categorical(Domain):
    def __init__(self, categories: Sequence):
        self.categories = list(categories)

    def sample(self, spec=None, rng=None):
        return (rng or random).choice(self.categories)


class Function(Domain):
    def __init__(self, func: Callable):
        self.func = func

    def sample(self, spec=None, rng=None):
        try:
            return self.func(spec)
        except TypeError:
            return self.func()


class Grid(Domain):
    def __init__(self, values):
        self.values = list(values)

    def is_grid(self):
        return True


def uniform(lower, upper):
    return Float(lower, upper)


def quniform(lower, upper, q):
    return Float(lower, upper, q=q)


def loguniform(lower, upper, base=10):
    return Float(lower, upper, log=True, base=base)


def qloguniform(lower, upper, q, base=10):
    return Float(lower, upper, log=True, base=base, q=q)


def randn(mean=0.0, sd=1.0):
    return Float(None, None, normal=(mean, sd))


def qrandn(mean, sd, q):
    return Float(None, None, normal=(mean, sd), q=q)


def randint(lower, upper):
    return Integer(lower, upper)


def qrandint(lower, upper, q=1):
    return Integer(lower, upper + 1, q=q)


def lograndint(lower, upper, base=10):
    return Integer(lower, upper, log=True, base=base)


def qlograndint(lower, upper, q, base=10):
    return Integer(lower, upper, log=True, base=base, q=q)


def choice(categories):
    return Categorical(categories)


def sample_from(func):
    return Function(func)


def grid_search(values):
    return {"grid_search": list(values)}


# -------------------------------------------------------------- variant generation
def _walk(space, path=()):
    if isinstance(space, dict):
        if set(space.keys()) == {"grid_search"}:
            yield path, Grid(space["grid_search"])
            return
        for k, v in space.items():
            yield from _walk(v, path + (k,))
    elif isinstance(space, Domain):
        yield path, space


def _set(d, path, value):
    for k in path[:-1]:
        d = d[k]
    d[path[-1]] = value


def _copy(space):
    if isinstance(space, dict):
        if set(space.keys()) == {"grid_search"}:
            return space
        return {k: _copy(v) for k, v in space.items()}
    if isinstance(space, list):
        return [_copy(v) for v in space]
    return space


def generate_variants(space: Dict[str, Any], num_samples: int = 1, seed=None):
    """Grid axes are crossed; random domains re-sampled for every (grid point, sample)."""
    rng = random.Random(seed)
    leaves = list(_walk(space))
    grids = [(p, d) for p, d in leaves if d.is_grid()]
    rands = [(p, d) for p, d in leaves if not d.is_grid()]
    import itertools

    grid_points = list(itertools.product(*[d.values for _, d in grids])) if grids else [()]
    for _ in range(num_samples):
        for gp in grid_points:
            cfg = _copy(space)
            for (p, _), v in zip(grids, gp):
                _set(cfg, p, v)
            for p, d in rands:
                if isinstance(d, Function):
                    continue
                _set(cfg, p, d.sample(cfg, rng))
            for p, d in rands:
                if isinstance(d, Function):
                    _set(cfg, p, d.sample(_Spec(cfg), rng))
            yield cfg


class _Spec:
    def __init__(self, cfg):
        self.config = cfg

    def __getitem__(self, k):
        return self.config[k]
