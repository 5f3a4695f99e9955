"""Replay buffers (reference: rllib/utils/replay_buffers/replay_buffer.py,
prioritized_replay_buffer.py, utils/segment_tree.py).

Storage is a dict of pre-allocated numpy columns written circularly, so adding
a fragment and sampling a minibatch are single vectorised copies. The
prioritized buffer keeps a sum-tree (and a min-tree for importance weights) in
flat arrays; updates and prefix-sum searches are vectorised over the batch
(one pass per tree level)."""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np


class ReplayBuffer:
    def __init__(self, capacity: int = 100_000, seed: Optional[int] = None):
        self.capacity = int(capacity)
        self.cols: Dict[str, np.ndarray] = {}
        self.size = 0
        self.pos = 0
        self.rng = np.random.default_rng(seed)
        self.num_added = 0

    def __len__(self):
        return self.size

    def _alloc(self, batch):
        for k, v in batch.items():
            v = np.asarray(v)
            self.cols[k] = np.empty((self.capacity,) + v.shape[1:], dtype=v.dtype)

    def add(self, batch: Dict[str, np.ndarray]) -> np.ndarray:
        n = len(next(iter(batch.values())))
        if not self.cols:
            self._alloc(batch)
        idx = (self.pos + np.arange(n)) % self.capacity
        for k, v in batch.items():
            self.cols[k][idx] = v
        self.pos = (self.pos + n) % self.capacity
        self.size = min(self.capacity, self.size + n)
        self.num_added += n
        return idx

    def sample(self, n: int, **_) -> Dict[str, np.ndarray]:
        idx = self.rng.integers(0, self.size, size=n)
        out = {k: v[idx] for k, v in self.cols.items()}
        out["batch_indexes"] = idx
        out["weights"] = np.ones(n, dtype=np.float32)
        return out

    def update_priorities(self, idx, prio):
        pass

    def get_state(self):
        return {"cols": {k: v[: self.size] for k, v in self.cols.items()}, "pos": self.pos, "size": self.size}

    def set_state(self, st):
        self.cols = {}
        if st["cols"]:
            self._alloc({k: v[:1] for k, v in st["cols"].items()})
            for k, v in st["cols"].items():
                self.cols[k][: len(v)] = v
        self.pos, self.size = st["pos"], st["size"]


class _Tree:
    def __init__(self, capacity: int, op, neutral: float):
        cap = 1
        while cap < capacity:
            cap *= 2
        self.cap = cap
        self.op = op
        self.neutral = neutral
        self.t = np.full(2 * cap, neutral, dtype=np.float64)

    def set(self, idx: np.ndarray, vals: np.ndarray):
        i = np.asarray(idx) + self.cap
        self.t[i] = vals
        i = np.unique(i // 2)
        while i[0] >= 1:
            self.t[i] = self.op(self.t[2 * i], self.t[2 * i + 1])
            if i[0] == 1:
                break
            i = np.unique(i // 2)

    def total(self):
        return self.t[1]

    def find_prefix(self, mass: np.ndarray) -> np.ndarray:
        """Smallest leaf index with prefix-sum >= mass (vectorised descent)."""
        i = np.ones(len(mass), dtype=np.int64)
        mass = mass.astype(np.float64).copy()
        while i[0] < self.cap:
            left = 2 * i
            go_right = mass > self.t[left]
            mass = np.where(go_right, mass - self.t[left], mass)
            i = np.where(go_right, left + 1, left)
        return i - self.cap


class PrioritizedReplayBuffer(ReplayBuffer):
    def __init__(self, capacity: int = 100_000, alpha: float = 0.6, beta: float = 0.4, eps: float = 1e-6,
                 seed: Optional[int] = None):
        super().__init__(capacity, seed)
        self.alpha, self.beta, self.eps = alpha, beta, eps
        self.sum = _Tree(self.capacity, np.add, 0.0)
        self.min = _Tree(self.capacity, np.minimum, np.inf)
        self.max_prio = 1.0

    def add(self, batch, priorities: Optional[np.ndarray] = None):
        idx = super().add(batch)
        p = np.full(len(idx), self.max_prio) if priorities is None else np.asarray(priorities)
        pa = (p + self.eps) ** self.alpha
        self.sum.set(idx, pa)
        self.min.set(idx, pa)
        return idx

    def sample(self, n: int, beta: Optional[float] = None, **_):
        beta = self.beta if beta is None else beta
        total = self.sum.total()
        mass = (np.arange(n) + self.rng.random(n)) * (total / n)  # stratified
        idx = np.minimum(self.sum.find_prefix(mass), self.size - 1)
        probs = self.sum.t[idx + self.sum.cap] / total
        pmin = self.min.total() / total
        w = (probs * self.size) ** (-beta) / ((pmin * self.size) ** (-beta))
        out = {k: v[idx] for k, v in self.cols.items()}
        out["batch_indexes"] = idx
        out["weights"] = w.astype(np.float32)
        return out

    def update_priorities(self, idx, prio):
        prio = np.abs(np.asarray(prio, dtype=np.float64))
        self.max_prio = max(self.max_prio, float(prio.max()))
        pa = (prio + self.eps) ** self.alpha
        self.sum.set(idx, pa)
        self.min.set(idx, pa)


def fragments_to_transitions(frag: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Time-major fragment [T, N, ...] (with next_obs) -> flat transitions."""
    T, N = frag["rewards"].shape
    keep = frag["mask"].reshape(-1) if "mask" in frag else slice(None)  # multi-agent padding
    f = lambda x: x.reshape((T * N,) + x.shape[2:])[keep]
    return {"obs": f(frag["obs"]), "actions": f(frag["actions"]), "rewards": f(frag["rewards"]),
            "next_obs": f(frag["next_obs"]),
            "terminateds": f(frag["terminateds"] & ~frag["truncateds"]).astype(np.float32)}
