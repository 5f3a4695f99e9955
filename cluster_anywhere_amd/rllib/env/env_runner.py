"""EnvRunners (reference: rllib/env/single_agent_env_runner.py,
env_runner_group.py).

Each runner owns a ``VectorEnv`` and a CPU copy of the RLModule, and returns
time-major numpy fragments ``[T, N, ...]`` (zero-copy through the shm object
store to the Learner). Truncated episodes are bootstrapped on the runner:
``rewards`` gets ``gamma * V(final_obs)`` added at truncation and the step is
then treated as terminal, so the learner-side GAE / V-trace only needs
``terminateds``."""
from __future__ import annotations

import time
from collections import deque
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from . import VectorEnv


class EnvRunner:
    def __init__(self, config: Dict[str, Any], worker_index: int = 0):
        self.cfg = config
        self.worker_index = worker_index
        seed = config.get("seed")
        torch.set_num_threads(1)
        if seed is not None:
            torch.manual_seed(seed + worker_index)
            np.random.seed(seed + worker_index)
        self.env = VectorEnv(config["env"], config.get("num_envs_per_env_runner", 1), config.get("env_config"),
                             None if seed is None else seed + 1000 * worker_index)
        self.module = config["module_factory"](self.env.observation_space, self.env.action_space)
        self.module.eval()
        self.obs = self.env.reset()
        self.ep_ret = np.zeros(self.env.num_envs)
        self.ep_len = np.zeros(self.env.num_envs, dtype=np.int64)
        self.done_returns: deque = deque(maxlen=config.get("metrics_num_episodes_for_smoothing", 100))
        self.done_lens: deque = deque(maxlen=config.get("metrics_num_episodes_for_smoothing", 100))
        self.new_episodes: List[float] = []
        self.total_steps = 0
        self.explore_extra: Dict[str, Any] = {}

    # ------------------------------------------------------------ weights
    def set_weights(self, state, extra: Optional[Dict] = None):
        self.module.set_state(state)
        if extra:
            self.explore_extra.update(extra)
        return True

    def get_weights(self):
        return self.module.get_state()

    def get_spaces(self):
        return self.env.observation_space, self.env.action_space

    # ------------------------------------------------------------ sampling
    @torch.no_grad()
    def sample(self, num_timesteps: Optional[int] = None, explore: bool = True) -> Dict[str, Any]:
        T = num_timesteps or self.cfg.get("rollout_fragment_length", 64)
        N = self.env.num_envs
        gamma = self.cfg.get("gamma", 0.99)
        need_next = self.cfg.get("need_next_obs", False)
        obs_buf = np.empty((T, N) + self.obs.shape[1:], dtype=self.obs.dtype)
        next_buf = np.empty_like(obs_buf) if need_next else None
        acts, logps, vfs, rews, raw, terms, truncs, dist = [], [], [], [], [], [], [], []
        t0 = time.time()
        for t in range(T):
            obs_buf[t] = self.obs
            batch = {"obs": torch.from_numpy(self.obs)}
            batch.update(self.explore_extra)
            out = self.module.forward_exploration(batch) if explore else self.module.forward_inference(batch)
            a = out["actions"].cpu().numpy()
            nobs, r, te, tr, final = self.env.step(a)
            r_aug = r.copy()
            if tr.any() and hasattr(self.module, "compute_values"):
                idx = np.nonzero(tr & ~te)[0]
                if len(idx):
                    v = self.module.compute_values({"obs": torch.from_numpy(final[idx])}).cpu().numpy()
                    r_aug[idx] += gamma * v
            if need_next:
                next_buf[t] = final
            acts.append(a)
            if "action_logp" in out:
                logps.append(out["action_logp"].cpu().numpy())
            if "vf_preds" in out:
                vfs.append(out["vf_preds"].cpu().numpy())
            if "action_dist_inputs" in out:
                dist.append(out["action_dist_inputs"].cpu().numpy())
            rews.append(r_aug)
            raw.append(r)
            terms.append(te | tr)
            truncs.append(tr)
            self.ep_ret += r
            self.ep_len += 1
            for i in np.nonzero(te | tr)[0]:
                self.done_returns.append(float(self.ep_ret[i]))
                self.done_lens.append(int(self.ep_len[i]))
                self.new_episodes.append(float(self.ep_ret[i]))
                self.ep_ret[i] = 0
                self.ep_len[i] = 0
            self.obs = nobs
        self.total_steps += T * N
        out = {"obs": obs_buf, "actions": np.stack(acts), "rewards": np.stack(rews).astype(np.float32),
               "terminateds": np.stack(terms), "truncateds": np.stack(truncs),
               "last_obs": self.obs.copy(), "env_steps": T * N, "sample_time_s": time.time() - t0}
        if logps:
            out["action_logp"] = np.stack(logps).astype(np.float32)
        if vfs:
            out["vf_preds"] = np.stack(vfs).astype(np.float32)
        if dist:
            out["action_dist_inputs"] = np.stack(dist).astype(np.float32)
        if need_next:
            out["next_obs"] = next_buf
        return out

    def get_metrics(self, reset_new: bool = True) -> Dict[str, Any]:
        m = {"num_episodes": len(self.new_episodes), "num_env_steps_sampled_lifetime": self.total_steps,
             "episode_returns": list(self.done_returns), "episode_lens": list(self.done_lens)}
        if reset_new:
            self.new_episodes = []
        return m

    def ping(self):
        return True


class EnvRunnerGroup:
    """A local runner (``num_env_runners == 0``) or N remote runner actors."""

    def __init__(self, config: Dict[str, Any], num_env_runners: int = 0, num_cpus_per_env_runner: float = 1):
        self.config = config
        self.local = None
        self.remote = []
        if num_env_runners == 0:
            self.local = EnvRunner(config, 0)
        else:
            from ...core import api as core
            from ...core.actor import ActorClass

            Remote = ActorClass(EnvRunner, {})
            self.remote = [Remote.options(num_cpus=num_cpus_per_env_runner).remote(config, i + 1)
                           for i in range(num_env_runners)]
            core.get([r.ping.remote() for r in self.remote])

    def spaces(self):
        from ...core import api as core

        if self.local is not None:
            return self.local.get_spaces()
        return core.get(self.remote[0].get_spaces.remote())

    def sync_weights(self, state, extra: Optional[Dict] = None):
        from ...core import api as core

        if self.local is not None:
            self.local.set_weights(state, extra)
            return
        ref = core.put(state)
        core.get([r.set_weights.remote(ref, extra) for r in self.remote])

    def sample(self, num_timesteps: Optional[int] = None, explore: bool = True) -> List[Dict]:
        from ...core import api as core

        if self.local is not None:
            return [self.local.sample(num_timesteps, explore)]
        return core.get([r.sample.remote(num_timesteps, explore) for r in self.remote])

    def sample_async(self, num_timesteps: Optional[int] = None):
        return [r.sample.remote(num_timesteps) for r in self.remote]

    def metrics(self) -> Dict[str, Any]:
        from ...core import api as core

        ms = [self.local.get_metrics()] if self.local is not None else \
            core.get([r.get_metrics.remote() for r in self.remote])
        rets = [x for m in ms for x in m["episode_returns"]]
        lens = [x for m in ms for x in m["episode_lens"]]
        return {"episode_return_mean": float(np.mean(rets)) if rets else float("nan"),
                "episode_return_max": float(np.max(rets)) if rets else float("nan"),
                "episode_return_min": float(np.min(rets)) if rets else float("nan"),
                "episode_len_mean": float(np.mean(lens)) if lens else float("nan"),
                "num_episodes": sum(m["num_episodes"] for m in ms),
                "num_env_steps_sampled_lifetime": sum(m["num_env_steps_sampled_lifetime"] for m in ms)}

    def stop(self):
        from ...core import api as core

        for r in self.remote:
            try:
                core.kill(r)
            except Exception:
                pass
        self.remote = []
