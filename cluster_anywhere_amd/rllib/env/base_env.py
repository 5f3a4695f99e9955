"""``BaseEnv``: the old stack's asynchronous vectorized env interface (reference
role: rllib/env/base_env.py) — ``poll()`` returns per-env dicts of observations,
rewards, terminateds, truncateds and infos for envs that are ready;
``send_actions`` steps them; ``try_reset`` resets one. ``to_base_env`` adapts a
single env, a list of envs or a :class:`VectorEnv`. Env ids are ints, agent ids
``"agent0"`` for single-agent envs (``_DUMMY_AGENT_ID``)."""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

_DUMMY_AGENT_ID = "agent0"


class BaseEnv:
    def poll(self) -> Tuple[Dict, Dict, Dict, Dict, Dict, Dict]:
        raise NotImplementedError

    def send_actions(self, action_dict: Dict[int, Dict[Any, Any]]) -> None:
        raise NotImplementedError

    def try_reset(self, env_id: Optional[int] = None, *, seed=None, options=None):
        return None, None

    def get_sub_environments(self, as_dict: bool = False):
        return {} if as_dict else []

    @property
    def num_envs(self) -> int:
        return len(self.get_sub_environments())

    def stop(self) -> None:
        for e in self.get_sub_environments():
            if hasattr(e, "close"):
                e.close()

    @staticmethod
    def to_base_env(env, make_env=None, num_envs: int = 1, remote_envs: bool = False, **kwargs) -> "BaseEnv":
        if isinstance(env, BaseEnv):
            return env
        from . import VectorEnv

        if isinstance(env, VectorEnv):
            envs = list(env.envs)
        elif isinstance(env, (list, tuple)):
            envs = list(env)
        else:
            envs = [env] + [make_env(i) for i in range(1, num_envs)] if make_env else [env]
        return _EnvList(envs)


class _EnvList(BaseEnv):
    """Sub-environments stepped one by one; finished ones wait for ``try_reset``
    (or are reset on the next poll)."""

    def __init__(self, envs: List[Any]):
        self.envs = envs
        self.observation_space = envs[0].observation_space
        self.action_space = envs[0].action_space
        self._pending: Dict[int, Tuple] = {}
        for i, e in enumerate(envs):
            obs, info = e.reset()
            self._pending[i] = (obs, 0.0, False, False, info)

    def poll(self):
        obs, rew, term, trunc, infos = {}, {}, {}, {}, {}
        for i, (o, r, te, tr, inf) in self._pending.items():
            obs[i] = {_DUMMY_AGENT_ID: o}
            rew[i] = {_DUMMY_AGENT_ID: r}
            term[i] = {_DUMMY_AGENT_ID: te, "__all__": te}
            trunc[i] = {_DUMMY_AGENT_ID: tr, "__all__": tr}
            infos[i] = {_DUMMY_AGENT_ID: inf}
        self._pending = {}
        return obs, rew, term, trunc, infos, {}

    def send_actions(self, action_dict):
        for i, acts in action_dict.items():
            o, r, te, tr, inf = self.envs[i].step(acts[_DUMMY_AGENT_ID])
            self._pending[i] = (o, float(r), bool(te), bool(tr), inf)

    def try_reset(self, env_id=None, *, seed=None, options=None):
        o, inf = self.envs[env_id].reset(seed=seed, options=options)
        self._pending[env_id] = (o, 0.0, False, False, inf)
        return {env_id: {_DUMMY_AGENT_ID: o}}, {env_id: {_DUMMY_AGENT_ID: inf}}

    def get_sub_environments(self, as_dict: bool = False):
        return {i: e for i, e in enumerate(self.envs)} if as_dict else list(self.envs)
