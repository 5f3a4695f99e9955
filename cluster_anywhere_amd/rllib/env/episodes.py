"""Episode records handed to callbacks and connectors (reference roles:
rllib/env/single_agent_episode.py, rllib/env/multi_agent_episode.py).

The env runners keep the training data in preallocated time-major arrays, so an
episode here is a light record of one running episode: its id, length, rewards,
a bounded look-back of observations / actions / infos (for callbacks and
stateful connectors such as frame stacking) and a ``custom_data`` dict that
callbacks may use freely.
"""
from __future__ import annotations

import uuid
from collections import deque
from typing import Any, Dict, List, Optional

import numpy as np

LOOKBACK = 64


class SingleAgentEpisode:
    __slots__ = ("id_", "agent_id", "module_id", "t_started", "t", "rewards", "_obs", "_acts", "_infos",
                 "is_terminated", "is_truncated", "custom_data")

    def __init__(self, id_: Optional[str] = None, agent_id=None, module_id=None, lookback: int = LOOKBACK):
        self.id_ = id_ or uuid.uuid4().hex
        self.agent_id = agent_id
        self.module_id = module_id
        self.t_started = 0
        self.t = 0
        self.rewards: List[float] = []
        self._obs: deque = deque(maxlen=lookback)
        self._acts: deque = deque(maxlen=lookback)
        self._infos: deque = deque(maxlen=lookback)
        self.is_terminated = False
        self.is_truncated = False
        self.custom_data: Dict[str, Any] = {}

    # ---- recording (env runner side)
    def add_reset(self, obs, info=None):
        self._obs.append(obs)
        self._infos.append(info or {})

    def add_step(self, obs, action, reward: float, info=None, terminated=False, truncated=False):
        if obs is not None:  # turn-based agents get their next observation on a later env step
            self._obs.append(obs)
        self._acts.append(action)
        self._infos.append(info or {})
        self.rewards.append(float(reward))
        self.t += 1
        self.is_terminated = bool(terminated)
        self.is_truncated = bool(truncated)

    # ---- read API
    @property
    def is_done(self) -> bool:
        return self.is_terminated or self.is_truncated

    def __len__(self) -> int:
        return self.t

    def get_return(self) -> float:
        return float(sum(self.rewards))

    def get_duration_s(self) -> float:  # not tracked; kept for API shape
        return float("nan")

    @staticmethod
    def _pick(d: deque, indices):
        if indices is None:
            return list(d)
        if isinstance(indices, slice):
            return list(d)[indices]
        return d[indices]

    def get_observations(self, indices=None):
        return self._pick(self._obs, indices)

    def get_actions(self, indices=None):
        return self._pick(self._acts, indices)

    def get_infos(self, indices=None):
        return self._pick(self._infos, indices)

    def get_rewards(self, indices=None):
        if indices is None:
            return np.asarray(self.rewards, np.float32)
        r = self.rewards[indices]
        return np.asarray(r, np.float32) if isinstance(indices, slice) else r


class MultiAgentEpisode:
    """One multi-agent episode: per-agent ``SingleAgentEpisode`` records plus
    the agent -> module mapping chosen for this episode."""

    def __init__(self, id_: Optional[str] = None):
        self.id_ = id_ or uuid.uuid4().hex
        self.env_t = 0
        self.agent_episodes: Dict[Any, SingleAgentEpisode] = {}
        self.module_for_agent: Dict[Any, str] = {}
        self.is_terminated = False
        self.is_truncated = False
        self.custom_data: Dict[str, Any] = {}

    def agent(self, agent_id, module_id=None) -> SingleAgentEpisode:
        e = self.agent_episodes.get(agent_id)
        if e is None:
            e = self.agent_episodes[agent_id] = SingleAgentEpisode(f"{self.id_}:{agent_id}", agent_id, module_id)
        return e

    @property
    def agent_ids(self):
        return list(self.agent_episodes)

    @property
    def is_done(self) -> bool:
        return self.is_terminated or self.is_truncated

    def module_for(self, agent_id):
        return self.module_for_agent.get(agent_id)

    def __len__(self) -> int:
        return self.env_t

    def get_return(self) -> float:
        return float(sum(e.get_return() for e in self.agent_episodes.values()))

    def get_agent_returns(self) -> Dict[Any, float]:
        return {a: e.get_return() for a, e in self.agent_episodes.items()}
