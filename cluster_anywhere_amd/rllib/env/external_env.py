"""``ExternalEnv``: an environment driven from outside (a simulator or a service
calls in), reference role: rllib/env/external_env.py. Subclass and implement
``run()``, which uses ``start_episode`` / ``get_action`` / ``log_action`` /
``log_returns`` / ``end_episode``; the env runs ``run()`` on its own thread.
Actions come from the attached policy (``set_policy``); finished episodes are
collected as :class:`SampleBatch` es (``pop_batches``) for ``learn_on_batch``."""
from __future__ import annotations

import threading
import uuid
from typing import Any, Dict, List, Optional

import numpy as np

from ..policy.sample_batch import SampleBatch


class ExternalEnv(threading.Thread):
    def __init__(self, action_space, observation_space, max_concurrent: int = 100):
        super().__init__(daemon=True)
        self.action_space = action_space
        self.observation_space = observation_space
        self.max_concurrent = max_concurrent
        self._policy = None
        self._episodes: Dict[str, Dict[str, List[Any]]] = {}
        self._done: List[SampleBatch] = []
        self._lock = threading.Lock()

    def run(self):
        raise NotImplementedError("ExternalEnv subclasses implement run()")

    def set_policy(self, policy) -> None:
        self._policy = policy

    def start_episode(self, episode_id: Optional[str] = None, training_enabled: bool = True) -> str:
        eid = episode_id or uuid.uuid4().hex
        with self._lock:
            if eid in self._episodes:
                raise ValueError(f"episode {eid} already started")
            if len(self._episodes) >= self.max_concurrent:
                raise RuntimeError(f"too many concurrent episodes ({self.max_concurrent})")
            self._episodes[eid] = {k: [] for k in ("obs", "actions", "rewards")}
            self._episodes[eid]["training"] = training_enabled
        return eid

    def _ep(self, eid):
        ep = self._episodes.get(eid)
        if ep is None:
            raise ValueError(f"unknown episode {eid}")
        return ep

    def get_action(self, episode_id: str, observation):
        if self._policy is None:
            raise RuntimeError("no policy attached (set_policy)")
        action = self._policy.compute_single_action(observation)[0]
        self.log_action(episode_id, observation, action)
        return action

    def log_action(self, episode_id: str, observation, action) -> None:
        with self._lock:
            ep = self._ep(episode_id)
            if len(ep["rewards"]) < len(ep["actions"]):
                ep["rewards"].append(0.0)
            ep["obs"].append(np.asarray(observation))
            ep["actions"].append(action)

    def log_returns(self, episode_id: str, reward: float, info=None) -> None:
        with self._lock:
            ep = self._ep(episode_id)
            if len(ep["rewards"]) < len(ep["actions"]):
                ep["rewards"].append(float(reward))
            elif ep["rewards"]:
                ep["rewards"][-1] += float(reward)

    def end_episode(self, episode_id: str, observation) -> None:
        with self._lock:
            ep = self._episodes.pop(episode_id)
            n = len(ep["actions"])
            ep["rewards"] += [0.0] * (n - len(ep["rewards"]))
            if n and ep["training"]:
                term = np.zeros(n, bool)
                term[-1] = True
                self._done.append(SampleBatch({SampleBatch.OBS: np.stack(ep["obs"]),
                                               SampleBatch.ACTIONS: np.asarray(ep["actions"]),
                                               SampleBatch.REWARDS: np.asarray(ep["rewards"], np.float32),
                                               SampleBatch.TERMINATEDS: term,
                                               SampleBatch.EPS_ID: np.full(n, hash(episode_id) & 0x7fffffff)}))

    def pop_batches(self) -> List[SampleBatch]:
        with self._lock:
            out, self._done = self._done, []
        return out
