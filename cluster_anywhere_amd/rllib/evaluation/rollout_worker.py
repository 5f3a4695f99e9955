"""Old-stack ``RolloutWorker`` (reference role: rllib/evaluation/rollout_worker.py):
steps a (vectorized) env with a :class:`~..policy.Policy` and returns
:class:`SampleBatch` es of ``rollout_fragment_length`` steps per env; also
``learn_on_batch``, weights and ``foreach_policy``. Usable locally or as an actor
(``ray.remote(RolloutWorker)``). New-stack algorithms sample with EnvRunners."""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional

import numpy as np

from ..policy.sample_batch import DEFAULT_POLICY_ID, SampleBatch


class RolloutWorker:
    def __init__(self, *, env_creator: Callable[[Dict], Any], default_policy_class=None, config=None,
                 worker_index: int = 0, num_workers: int = 0, policy_config: Optional[Dict] = None,
                 rollout_fragment_length: int = 200, num_envs: int = 1, seed: Optional[int] = None, **kwargs):
        from ..policy.policy import TorchPolicy

        cfg = dict(config or {}) if not hasattr(config, "to_dict") else config.to_dict()
        self.worker_index = worker_index
        self.env_config = dict(cfg.get("env_config", {}))
        self.envs = [env_creator(self.env_config) for _ in range(max(1, num_envs))]
        self.env = self.envs[0]
        self.fragment = int(cfg.get("rollout_fragment_length", rollout_fragment_length) or rollout_fragment_length)
        if not isinstance(self.fragment, int) or self.fragment <= 0:
            self.fragment = rollout_fragment_length
        cls = default_policy_class or TorchPolicy
        pc = dict(policy_config or cfg)
        self.policy_map = {DEFAULT_POLICY_ID: cls(self.env.observation_space, self.env.action_space, pc)}
        self._obs = []
        self._eps = []
        self._next_eps = worker_index * 1_000_000
        for i, e in enumerate(self.envs):
            o, _ = e.reset(seed=None if seed is None else seed + i)
            self._obs.append(o)
            self._eps.append(self._new_eps())
        self.episode_returns: List[float] = []
        self._ret = [0.0] * len(self.envs)

    def _new_eps(self) -> int:
        self._next_eps += 1
        return self._next_eps

    def get_policy(self, policy_id: str = DEFAULT_POLICY_ID):
        return self.policy_map.get(policy_id)

    def sample(self) -> SampleBatch:
        pol = self.policy_map[DEFAULT_POLICY_ID]
        cols: Dict[str, List[Any]] = {k: [] for k in (SampleBatch.OBS, SampleBatch.ACTIONS, SampleBatch.REWARDS,
                                                      SampleBatch.TERMINATEDS, SampleBatch.TRUNCATEDS,
                                                      SampleBatch.NEXT_OBS, SampleBatch.EPS_ID, SampleBatch.T)}
        extra: Dict[str, List[Any]] = {}
        per_env: List[Dict[str, List[Any]]] = [{k: [] for k in cols} for _ in self.envs]
        per_extra: List[Dict[str, List[Any]]] = [{} for _ in self.envs]
        t = [0] * len(self.envs)
        for _ in range(self.fragment):
            acts, _, ext = pol.compute_actions(np.stack(self._obs))
            for i, e in enumerate(self.envs):
                o2, r, te, tr, _ = e.step(acts[i])
                rec = per_env[i]
                rec[SampleBatch.OBS].append(self._obs[i])
                rec[SampleBatch.ACTIONS].append(acts[i])
                rec[SampleBatch.REWARDS].append(float(r))
                rec[SampleBatch.TERMINATEDS].append(bool(te))
                rec[SampleBatch.TRUNCATEDS].append(bool(tr))
                rec[SampleBatch.NEXT_OBS].append(o2)
                rec[SampleBatch.EPS_ID].append(self._eps[i])
                rec[SampleBatch.T].append(t[i])
                for k, v in ext.items():
                    per_extra[i].setdefault(k, []).append(v[i])
                t[i] += 1
                self._ret[i] += float(r)
                if te or tr:
                    self.episode_returns.append(self._ret[i])
                    self._ret[i] = 0.0
                    o2, _ = e.reset()
                    self._eps[i] = self._new_eps()
                    t[i] = 0
                self._obs[i] = o2
        batches = []
        for rec, ex in zip(per_env, per_extra):
            b = SampleBatch({k: np.asarray(v) for k, v in {**rec, **ex}.items()})
            batches.append(pol.postprocess_trajectory(b))
        return SampleBatch.concat_samples(batches)

    def learn_on_batch(self, samples: SampleBatch) -> Dict[str, Any]:
        return {DEFAULT_POLICY_ID: self.policy_map[DEFAULT_POLICY_ID].learn_on_batch(samples)}

    def sample_and_learn(self, *args, **kwargs):
        batch = self.sample()
        return batch, self.learn_on_batch(batch)

    def get_weights(self, policies: Optional[List[str]] = None) -> Dict[str, Any]:
        return {pid: p.get_weights() for pid, p in self.policy_map.items() if policies is None or pid in policies}

    def set_weights(self, weights: Dict[str, Any], global_vars: Optional[Dict] = None) -> None:
        for pid, w in weights.items():
            self.policy_map[pid].set_weights(w)
        if global_vars:
            for p in self.policy_map.values():
                p.on_global_var_update(global_vars)

    def foreach_policy(self, func: Callable) -> List[Any]:
        return [func(p, pid) for pid, p in self.policy_map.items()]

    def foreach_env(self, func: Callable) -> List[Any]:
        return [func(e) for e in self.envs]

    def get_metrics(self) -> Dict[str, Any]:
        out, self.episode_returns = self.episode_returns, []
        return {"episode_returns": out}

    def stop(self) -> None:
        for e in self.envs:
            if hasattr(e, "close"):
                e.close()
