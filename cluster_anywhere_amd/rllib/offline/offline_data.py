"""Offline input for BC / MARWIL / CQL: ``config.offline_data(input_=...)``.

Role of the reference's ``OfflineData`` + ``OfflinePreLearner``
(``rllib/offline/offline_data.py:23,118``, ``offline_prelearner.py:53``): experience
is read through a Data pipeline and STREAMED into the learners, so the driver never
holds the whole dataset.

* ``input_`` = Parquet path(s) / directory (``input_read_method`` names another
  ``data.read_*``) or a ``Dataset``: streaming. Each epoch runs
  ``ds.map_batches(prelearner, batch_size=None)`` -- one call per BLOCK, i.e. per
  recorded file, which holds whole episodes (``offline/io.py``) -- and iterates
  ``train_batch_size`` batches out of it with a local shuffle buffer. Only the blocks
  in flight and the shuffle buffer are resident.
* ``input_`` = a dict of columns or a list of such dicts (small in-memory data, the
  unit-test form): rows sampled uniformly with replacement, as before.

The pre-learner turns rows into learner batches: ``returns`` (discounted, per
episode; episodes are found by ``eps_id`` when present, else split at
``terminateds``/``truncateds``), float32 obs / next_obs, and the columns the
algorithm asked for.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Iterator, List, Optional, Sequence

import numpy as np


def discounted_returns(rew: np.ndarray, done: np.ndarray, gamma: float) -> np.ndarray:
    """Reward-to-go within each episode segment (``done`` marks a segment's last row)."""
    out = np.zeros(len(rew), dtype=np.float32)
    acc = 0.0
    for i in range(len(rew) - 1, -1, -1):
        if done[i]:
            acc = 0.0
        acc = float(rew[i]) + gamma * acc
        out[i] = acc
    return out


def episode_order(cols: Dict[str, np.ndarray]) -> np.ndarray:
    """Row order that makes every episode contiguous and time-ordered (by
    ``eps_id`` then ``t``), or the identity when the data carries no episode ids."""
    n = len(next(iter(cols.values())))
    if "eps_id" not in cols or "t" not in cols:
        return np.arange(n)
    eid = np.asarray(cols["eps_id"]).astype(str)
    return np.lexsort((np.asarray(cols["t"]), eid))


def episode_ends(cols: Dict[str, np.ndarray]) -> np.ndarray:
    """Boolean mask of each episode segment's last row (data in episode order)."""
    n = len(next(iter(cols.values())))
    done = np.zeros(n, dtype=bool)
    for k in ("terminateds", "truncateds"):
        if k in cols:
            done |= np.asarray(cols[k]).astype(bool)
    if "eps_id" in cols:
        eid = np.asarray(cols["eps_id"]).astype(str)
        done[:-1] |= eid[1:] != eid[:-1]
    if n:
        done[-1] = True  # a block ends every segment still open in it
    return done


class OfflinePreLearner:
    """``map_batches`` callable: one block of recorded rows -> learner-ready columns.

    ``columns``: the columns the algorithm trains on (missing derived ones --
    ``returns`` -- are computed here)."""

    def __init__(self, gamma: float = 0.99, columns: Optional[Sequence[str]] = None):
        self.gamma = float(gamma)
        self.columns = tuple(columns) if columns else None

    def __call__(self, batch: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
        cols = {k: np.asarray(v) for k, v in batch.items()}
        order = episode_order(cols)
        if not np.array_equal(order, np.arange(len(order))):
            cols = {k: v[order] for k, v in cols.items()}
        if "returns" not in cols and "rewards" in cols:
            cols["returns"] = discounted_returns(cols["rewards"].astype(np.float32), episode_ends(cols), self.gamma)
        for k in ("obs", "new_obs", "next_obs"):
            if k in cols:
                v = cols[k]
                if v.dtype == object:
                    v = np.stack(v)
                cols[k] = v.astype(np.float32, copy=False)
        if "new_obs" in cols and "next_obs" not in cols:
            cols["next_obs"] = cols["new_obs"]
        if self.columns is not None:
            missing = [k for k in self.columns if k not in cols]
            if missing:
                raise ValueError(f"offline data lacks columns {missing} (has {sorted(cols)})")
            cols = {k: cols[k] for k in self.columns}
        return cols


def _is_paths(inp) -> bool:
    return isinstance(inp, str) or (isinstance(inp, (list, tuple)) and inp and all(isinstance(x, str) for x in inp))


class OfflineData:
    """Sampler over offline experience (see module docstring).

    ``sample(n)`` -> dict of numpy columns with ``n`` rows (the last batch of an epoch
    may be shorter in streaming mode; epochs repeat forever)."""

    def __init__(self, input_, *, gamma: float = 0.99, columns: Optional[Sequence[str]] = None,
                 input_read_method: str = "read_parquet", input_read_method_kwargs: Optional[Dict] = None,
                 map_batches_kwargs: Optional[Dict] = None, iter_batches_kwargs: Optional[Dict] = None,
                 prelearner_class: Optional[Callable] = None, shuffle_buffer_rows: Optional[int] = None,
                 seed: Optional[int] = None):
        if input_ is None:
            raise ValueError("config.offline_data(input_=...) is required for offline algorithms")
        self.gamma = gamma
        self.columns = tuple(columns) if columns else None
        self.prelearner_class = prelearner_class or OfflinePreLearner
        self.rng = np.random.default_rng(seed)
        self.seed = seed
        self.epochs = 0
        self._it: Optional[Iterator] = None
        self._batch_rows = None
        self.map_batches_kwargs = dict(map_batches_kwargs or {})
        self.iter_batches_kwargs = dict(iter_batches_kwargs or {})
        self.shuffle_buffer_rows = shuffle_buffer_rows
        if isinstance(input_, dict) or (isinstance(input_, list) and input_ and isinstance(input_[0], dict)):
            parts = [input_] if isinstance(input_, dict) else list(input_)
            raw = {k: np.concatenate([np.asarray(p[k]) for p in parts]) for k in parts[0]}
            self._memory_full = self.prelearner_class(gamma, None)(raw)
            self.memory = (self._memory_full if self.columns is None
                           else self.prelearner_class(gamma, self.columns)(self._memory_full))
            self.n = len(next(iter(self.memory.values())))
            self.dataset = None
        else:
            self.memory = None
            if _is_paths(input_):
                from ... import data

                reader = getattr(data, input_read_method)
                input_ = reader(input_, **(input_read_method_kwargs or {}))
            if not hasattr(input_, "map_batches"):
                raise TypeError(f"offline input must be paths, a Dataset or column dicts, not {type(input_)}")
            self.dataset = input_

    @property
    def streaming(self) -> bool:
        return self.dataset is not None

    def _epoch(self, batch_rows: int) -> Iterator[Dict[str, np.ndarray]]:
        kw = dict(batch_size=None, batch_format="numpy")
        kw.update(self.map_batches_kwargs)
        pipe = self.dataset.map_batches(self.prelearner_class,
                                        fn_constructor_kwargs={"gamma": self.gamma, "columns": self.columns},
                                        concurrency=kw.pop("concurrency", 1), **kw)
        ikw = dict(batch_size=batch_rows, batch_format="numpy",
                   local_shuffle_buffer_size=self.shuffle_buffer_rows or 4 * batch_rows,
                   local_shuffle_seed=None if self.seed is None else self.seed + self.epochs)
        ikw.update(self.iter_batches_kwargs)
        for b in pipe.iter_batches(**ikw):
            yield b

    def sample(self, num_samples: int) -> Dict[str, np.ndarray]:
        if self.memory is not None:
            idx = self.rng.integers(0, self.n, size=min(num_samples, self.n))
            return {k: v[idx] for k, v in self.memory.items()}
        if self._it is None or self._batch_rows != num_samples:
            self._batch_rows = num_samples
            self._it = self._epoch(num_samples)
        for _ in range(2):
            try:
                return next(self._it)
            except StopIteration:
                self.epochs += 1
                self._it = self._epoch(num_samples)
        raise ValueError("offline dataset is empty")

    def iter_episodes(self, max_rows: Optional[int] = None) -> Iterator[Dict[str, np.ndarray]]:
        """Whole episodes (dict of columns each), in file order: what the off-policy
        estimators evaluate. ``max_rows`` bounds the rows read."""
        seen = 0
        if self.memory is not None:
            blocks = [self._memory_full]
        else:
            blocks = (self.prelearner_class(self.gamma, None)(b)
                      for b in self.dataset.iter_batches(batch_size=None, batch_format="numpy"))
        for cols in blocks:
            ends = np.nonzero(episode_ends(cols))[0]
            start = 0
            for e in ends:
                ep = {k: v[start:e + 1] for k, v in cols.items()}
                start = e + 1
                yield ep
                seen += len(ep["rewards"])
                if max_rows is not None and seen >= max_rows:
                    return
