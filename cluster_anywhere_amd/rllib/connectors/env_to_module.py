"""env -> module connectors (reference role: rllib/connectors/env_to_module/:
flatten_observations.py, mean_std_filter.py, frame_stacking.py,
prev_actions_prev_rewards.py).

They see ``batch["obs"]`` as one numpy array ``[B, ...]`` for the B episodes
that act this step (``episodes[i]`` is the record of row i) and return the
module input. ``shared_data["peek"]`` is set when the runner only needs a
value estimate of an observation (truncation bootstrap): stateful connectors
must not update their statistics or history then.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import numpy as np

from ..env import Box, Discrete
from .connector_v2 import ConnectorV2


def _flat_size(space) -> int:
    if isinstance(space, Discrete):
        return space.n
    return int(np.prod(space.shape))


class FlattenObservations(ConnectorV2):
    """Flatten Box observations to 1-D and one-hot Discrete ones."""

    def recompute_output_observation_space(self, obs_space, act_space):
        if obs_space is None:
            return None
        n = _flat_size(obs_space)
        if isinstance(obs_space, Discrete):
            return Box(0.0, 1.0, (n,))
        return Box(np.asarray(obs_space.low, np.float32).reshape(-1), np.asarray(obs_space.high, np.float32).reshape(-1),
                   (n,))

    def __call__(self, *, batch, episodes=(), **kw):
        o = batch["obs"]
        if isinstance(self.input_observation_space, Discrete):
            oh = np.zeros((len(o), self.input_observation_space.n), np.float32)
            oh[np.arange(len(o)), np.asarray(o, np.int64).reshape(-1)] = 1.0
            batch["obs"] = oh
        else:
            batch["obs"] = np.asarray(o, np.float32).reshape(len(o), -1)
        return batch


class _Running:
    """Running count / mean / sum of squared deviations (Chan et al. parallel merge)."""

    @staticmethod
    def empty(shape):
        return [0.0, np.zeros(shape, np.float64), np.zeros(shape, np.float64)]

    @staticmethod
    def push(st, x: np.ndarray):
        n_b = x.shape[0]
        if n_b == 0:
            return st
        mean_b = x.mean(0)
        m2_b = ((x - mean_b) ** 2).sum(0)
        return _Running.combine(st, [float(n_b), mean_b, m2_b])

    @staticmethod
    def combine(a, b):
        n = a[0] + b[0]
        if n == 0:
            return [0.0, a[1].copy(), a[2].copy()]
        d = b[1] - a[1]
        mean = a[1] + d * (b[0] / n)
        m2 = a[2] + b[2] + d * d * (a[0] * b[0] / n)
        return [n, mean, m2]


class MeanStdFilter(ConnectorV2):
    """Normalise observations by running mean / std (``clip_by_value`` optional).

    The state is the global statistics last broadcast by the driver plus the
    local delta since then; ``merge_states`` folds every runner's delta into the
    global stats, so all runners normalise identically after each sync."""

    def __init__(self, input_observation_space=None, input_action_space=None, *,
                 clip_by_value: Optional[float] = 10.0, de_mean_observations: bool = True, **kw):
        super().__init__(input_observation_space, input_action_space)
        self.clip = clip_by_value
        self.de_mean = de_mean_observations
        self._global = None
        self._delta = None

    def _init(self, shape):
        if self._global is None:
            self._global = _Running.empty(shape)
            self._delta = _Running.empty(shape)

    def __call__(self, *, batch, shared_data=None, **kw):
        o = np.asarray(batch["obs"], np.float64)
        self._init(o.shape[1:])
        if not (shared_data or {}).get("peek"):
            self._delta = _Running.push(self._delta, o)
        n, mean, m2 = _Running.combine(self._global, self._delta)
        std = np.sqrt(m2 / max(n - 1, 1.0)) if n > 1 else np.ones_like(mean)
        x = (o - mean) if self.de_mean else o
        x = x / (std + 1e-8)
        if self.clip:
            x = np.clip(x, -self.clip, self.clip)
        batch["obs"] = x.astype(np.float32)
        return batch

    def get_state(self):
        if self._global is None:
            return {}
        return {"global": [self._global[0], self._global[1].copy(), self._global[2].copy()],
                "delta": [self._delta[0], self._delta[1].copy(), self._delta[2].copy()]}

    def set_state(self, state):
        if not state:
            return
        self._global = [state["global"][0], np.array(state["global"][1]), np.array(state["global"][2])]
        self._delta = _Running.empty(self._global[1].shape) if "delta" not in state or state.get("reset_delta") \
            else [state["delta"][0], np.array(state["delta"][1]), np.array(state["delta"][2])]

    @staticmethod
    def merge_states(states):
        states = [s for s in states if s]
        if not states:
            return {}
        g = states[0]["global"]
        g = [g[0], np.array(g[1]), np.array(g[2])]
        for s in states:
            g = _Running.combine(g, s["delta"])
        return {"global": g, "delta": _Running.empty(g[1].shape), "reset_delta": True}

    @property
    def count(self) -> float:
        return 0.0 if self._global is None else _Running.combine(self._global, self._delta)[0]


class FrameStackingEnvToModule(ConnectorV2):
    """Stack the last ``num_frames`` observations along the last axis (per
    episode; a new episode starts from copies of its first frame)."""

    def __init__(self, input_observation_space=None, input_action_space=None, *, num_frames: int = 4, **kw):
        super().__init__(input_observation_space, input_action_space)
        self.k = int(num_frames)
        self._hist: Dict[str, List[np.ndarray]] = {}

    def recompute_output_observation_space(self, obs_space, act_space):
        if obs_space is None:
            return None
        lo = np.asarray(obs_space.low)
        hi = np.asarray(obs_space.high)
        if len(obs_space.shape) <= 1:
            return Box(np.tile(lo.reshape(-1), self.k), np.tile(hi.reshape(-1), self.k),
                       (int(np.prod(obs_space.shape or (1,))) * self.k,), obs_space.dtype)
        return Box(np.concatenate([lo] * self.k, -1), np.concatenate([hi] * self.k, -1),
                   obs_space.shape[:-1] + (obs_space.shape[-1] * self.k,), obs_space.dtype)

    def __call__(self, *, batch, episodes=(), shared_data=None, **kw):
        o = batch["obs"]
        peek = (shared_data or {}).get("peek")
        vec = o.ndim <= 2
        out = []
        for i, ep in enumerate(episodes):
            key = ep.id_ if ep is not None else i
            frame = o[i].reshape(-1) if vec else o[i]
            h = self._hist.get(key)
            h = [frame] * self.k if h is None else h[1:] + [frame]
            if not peek:
                self._hist[key] = h
            out.append(np.concatenate(h, -1))
        if episodes:
            batch["obs"] = np.stack(out)
        # drop finished episodes' history
        for ep in episodes:
            if ep is not None and ep.is_done:
                self._hist.pop(ep.id_, None)
        return batch

    def reset_state(self):
        self._hist.clear()

    def episode_done(self, episode):
        self._hist.pop(episode.id_, None)


class PrevActionsPrevRewards(ConnectorV2):
    """Append the previous ``n_prev_actions`` actions (one-hot for Discrete) and
    ``n_prev_rewards`` rewards to flat observations."""

    def __init__(self, input_observation_space=None, input_action_space=None, *, n_prev_rewards: int = 1,
                 n_prev_actions: int = 1, **kw):
        super().__init__(input_observation_space, input_action_space)
        self.nr, self.na = int(n_prev_rewards), int(n_prev_actions)

    def _adim(self, act_space):
        return act_space.n if isinstance(act_space, Discrete) else int(np.prod(act_space.shape))

    def recompute_output_observation_space(self, obs_space, act_space):
        if obs_space is None or act_space is None:
            return obs_space
        d = int(np.prod(obs_space.shape)) + self.nr + self.na * self._adim(act_space)
        return Box(-np.inf, np.inf, (d,))

    def __call__(self, *, batch, episodes=(), **kw):
        o = np.asarray(batch["obs"], np.float32).reshape(len(batch["obs"]), -1)
        act_space = self.input_action_space
        ad = self._adim(act_space)
        extra = np.zeros((len(o), self.nr + self.na * ad), np.float32)
        for i, ep in enumerate(episodes):
            if ep is None:
                continue
            rs = ep.rewards[-self.nr:] if self.nr else []
            if rs:
                extra[i, self.nr - len(rs): self.nr] = rs
            acts = list(ep.get_actions())[-self.na:] if self.na else []
            for j, a in enumerate(acts):
                base = self.nr + (self.na - len(acts) + j) * ad
                if isinstance(act_space, Discrete):
                    extra[i, base + int(a)] = 1.0
                else:
                    extra[i, base: base + ad] = np.asarray(a, np.float32).reshape(-1)
        batch["obs"] = np.concatenate([o, extra], 1)
        return batch


__all__ = ["FlattenObservations", "MeanStdFilter", "FrameStackingEnvToModule", "PrevActionsPrevRewards"]
