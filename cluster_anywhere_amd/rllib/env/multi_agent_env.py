"""Multi-agent environments (reference role: rllib/env/multi_agent_env.py:29).

A ``MultiAgentEnv`` exchanges dicts keyed by agent id: ``reset()`` returns
``(obs, infos)`` for the agents that must act first; ``step(action_dict)``
returns ``(obs, rewards, terminateds, truncateds, infos)`` where the two done
dicts carry the special ``"__all__"`` key that ends the episode. Agents may act
on different steps (turn-based games): only agents present in the returned
``obs`` act next.

``make_multi_agent(env)`` turns any single-agent env into an N-agent one
(independent copies; agent i drives copy i), which gives ``MultiAgentCartPole``
/ ``MultiAgentPendulum``. ``CooperativeMatchEnv`` is a small two-agent game
with one shared team reward and a different optimal mapping per agent.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Tuple

import numpy as np

from . import Box, Discrete, Space, make_env


class MultiAgentEnv:
    possible_agents: List[Any] = []
    agents: List[Any] = []
    observation_spaces: Dict[Any, Space] = {}
    action_spaces: Dict[Any, Space] = {}

    def reset(self, *, seed: Optional[int] = None, options=None) -> Tuple[Dict, Dict]:
        raise NotImplementedError

    def step(self, action_dict: Dict) -> Tuple[Dict, Dict, Dict, Dict, Dict]:
        raise NotImplementedError

    def get_observation_space(self, agent_id) -> Space:
        return self.observation_spaces[agent_id]

    def get_action_space(self, agent_id) -> Space:
        return self.action_spaces[agent_id]

    @property
    def num_agents(self) -> int:
        return len(self.agents)

    @property
    def max_num_agents(self) -> int:
        return len(self.possible_agents)

    def close(self):
        pass


def make_multi_agent(env_name_or_creator) -> type:
    """Class of an N-agent env made of independent single-agent copies
    (``config["num_agents"]``, default 2); agents are ``0 .. N-1``."""

    class _Multi(MultiAgentEnv):
        def __init__(self, config: Optional[Dict] = None):
            config = dict(config or {})
            n = int(config.pop("num_agents", 2))
            self.envs = [make_env(env_name_or_creator, config) for _ in range(n)]
            self.possible_agents = list(range(n))
            self.agents = list(self.possible_agents)
            self.observation_spaces = {i: e.observation_space for i, e in enumerate(self.envs)}
            self.action_spaces = {i: e.action_space for i, e in enumerate(self.envs)}
            self._done = set()

        def reset(self, *, seed=None, options=None):
            self._done = set()
            self.agents = list(self.possible_agents)
            obs, infos = {}, {}
            for i, e in enumerate(self.envs):
                o, inf = e.reset(seed=None if seed is None else seed + i)
                obs[i], infos[i] = o, inf
            return obs, infos

        def step(self, action_dict):
            obs, rew, te, tr, infos = {}, {}, {}, {}, {}
            for i, a in action_dict.items():
                o, r, t1, t2, inf = self.envs[i].step(a)
                obs[i], rew[i], te[i], tr[i], infos[i] = o, r, t1, t2, inf
                if t1 or t2:
                    self._done.add(i)
            self.agents = [i for i in self.possible_agents if i not in self._done]
            # the episode ends when every copy is done (terminated or truncated)
            all_done = len(self._done) == len(self.envs)
            te["__all__"] = all_done and not any(tr.values())
            tr["__all__"] = all_done and not te["__all__"]
            return obs, rew, te, tr, infos

    name = env_name_or_creator if isinstance(env_name_or_creator, str) else \
        getattr(env_name_or_creator, "__name__", "Env")
    _Multi.__name__ = _Multi.__qualname__ = f"MultiAgent{str(name).split('-')[0]}"
    return _Multi


MultiAgentCartPole = make_multi_agent("CartPole-v1")
MultiAgentPendulum = make_multi_agent("Pendulum-v1")


class CooperativeMatchEnv(MultiAgentEnv):
    """Two agents, one shared team reward. Each step both agents get a random
    bit (agent "a" sees its bit one-hot in obs slots 0..1, agent "b" in slots
    2..3); "a" scores a point by playing its bit, "b" by playing the OPPOSITE of
    its bit, and both receive the team's total. Each agent's credit is therefore
    noisy (the other agent's play is in its reward), and the two agents need
    different mappings. ``episode_len`` steps (default 10): random play returns
    10 per agent (team reward 1/step), optimal play 20."""

    def __init__(self, config: Optional[Dict] = None):
        config = config or {}
        self.episode_len = int(config.get("episode_len", 10))
        self.possible_agents = ["a", "b"]
        self.agents = list(self.possible_agents)
        sp = Box(0.0, 1.0, (4,))
        self.observation_spaces = {"a": sp, "b": sp}
        self.action_spaces = {"a": Discrete(2), "b": Discrete(2)}
        self.rng = np.random.default_rng(config.get("seed"))
        self.t = 0
        self.bits = np.zeros(2, np.int64)

    def _obs(self):
        oa = np.zeros(4, np.float32)
        ob = np.zeros(4, np.float32)
        oa[self.bits[0]] = 1.0
        ob[2 + self.bits[1]] = 1.0
        return {"a": oa, "b": ob}

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.t = 0
        self.bits = self.rng.integers(0, 2, size=2)
        return self._obs(), {"a": {}, "b": {}}

    def step(self, action_dict):
        r = float(int(action_dict["a"]) == self.bits[0]) + float(int(action_dict["b"]) == 1 - self.bits[1])
        self.t += 1
        done = self.t >= self.episode_len
        self.bits = self.rng.integers(0, 2, size=2)
        return (self._obs(), {"a": r, "b": r}, {"a": done, "b": done, "__all__": done},
                {"a": False, "b": False, "__all__": False}, {"a": {}, "b": {}})


__all__ = ["MultiAgentEnv", "make_multi_agent", "MultiAgentCartPole", "MultiAgentPendulum",
           "CooperativeMatchEnv"]
