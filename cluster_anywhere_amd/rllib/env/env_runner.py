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
from .episodes import SingleAgentEpisode


def _runner_callbacks(config):
    from ..callbacks import RLlibCallback, make_callbacks

    cb = make_callbacks(config.get("callbacks_class"), config.get("callbacks_functions"))
    return cb, type(cb) is not RLlibCallback


class EnvRunner:
    def __init__(self, config: Dict[str, Any], worker_index: int = 0):
        from ..connectors import build_pipeline
        from ..utils.metrics import MetricsLogger

        self.cfg = config
        self.worker_index = worker_index
        seed = config.get("seed")
        torch.set_num_threads(1)
        if seed is not None:
            torch.manual_seed(seed + worker_index)
            np.random.seed(seed + worker_index)
        self.metrics = MetricsLogger()
        self.callbacks, self._has_cb = _runner_callbacks(config)
        self.env = VectorEnv(config["env"], config.get("num_envs_per_env_runner", 1), config.get("env_config"),
                             None if seed is None else seed + 1000 * worker_index)
        if self._has_cb:
            self.callbacks.on_environment_created(env_runner=self, metrics_logger=self.metrics, env=self.env,
                                                  env_context=dict(config.get("env_config") or {},
                                                                   worker_index=worker_index))
        env_obs, env_act = self.env.observation_space, self.env.action_space
        self.env_to_module = build_pipeline(config.get("env_to_module_connector"), self.env)
        self.env_to_module.set_input_spaces(env_obs, env_act)
        self.module_to_env = build_pipeline(config.get("module_to_env_connector"), self.env)
        self.module_to_env.set_input_spaces(env_obs, env_act)
        self.obs_space = self.env_to_module.recompute_output_observation_space(env_obs, env_act)
        self.act_space = env_act
        self.module = config["module_factory"](self.obs_space, self.act_space)
        self.module.eval()
        self.episodes: List[SingleAgentEpisode] = []
        raw = self.env.reset()
        for i in range(self.env.num_envs):
            self.episodes.append(self._new_episode(i, raw[i]))
        self.obs = self._to_module(raw, self.episodes)
        self.ep_ret = np.zeros(self.env.num_envs)
        self.ep_len = np.zeros(self.env.num_envs, dtype=np.int64)
        self.done_returns: deque = deque(maxlen=config.get("metrics_num_episodes_for_smoothing", 100))
        self.done_lens: deque = deque(maxlen=config.get("metrics_num_episodes_for_smoothing", 100))
        self.new_episodes: List[float] = []
        self.total_steps = 0
        self.explore_extra: Dict[str, Any] = {}

    # ------------------------------------------------------------ episodes / connectors
    def _new_episode(self, i: int, raw_obs) -> SingleAgentEpisode:
        ep = SingleAgentEpisode()
        ep.add_reset(raw_obs)
        if self._has_cb:
            kw = dict(episode=ep, env_runner=self, metrics_logger=self.metrics, env=self.env, env_index=i,
                      rl_module=getattr(self, "module", None))
            self.callbacks.on_episode_created(**kw)
            self.callbacks.on_episode_start(**kw)
        return ep

    def _to_module(self, raw: np.ndarray, episodes, peek: bool = False) -> np.ndarray:
        if not len(self.env_to_module):
            return raw
        b = self.env_to_module(rl_module=getattr(self, "module", None), batch={"obs": raw}, episodes=episodes,
                               shared_data={"peek": peek}, metrics=self.metrics)
        return b["obs"]

    def _to_env(self, out: Dict[str, Any], a: np.ndarray, explore: bool) -> np.ndarray:
        if not len(self.module_to_env):
            return a
        b = {k: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}
        b["actions"] = a
        b = self.module_to_env(rl_module=self.module, batch=b, episodes=self.episodes, explore=explore,
                               shared_data={}, metrics=self.metrics)
        return b.get("actions_for_env", b["actions"])

    def get_connector_state(self):
        return {"env_to_module": self.env_to_module.get_state(), "module_to_env": self.module_to_env.get_state()}

    def set_connector_state(self, state):
        self.env_to_module.set_state(state.get("env_to_module", {}))
        self.module_to_env.set_state(state.get("module_to_env", {}))
        return True

    # ------------------------------------------------------------ weights
    def set_weights(self, state, extra: Optional[Dict] = None):
        self.module.set_state(state)
        if extra:
            self.explore_extra.update(extra)
        return True

    def get_weights(self):
        return self.module.get_state()

    def get_spaces(self):
        return self.obs_space, self.act_space

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
        track = self._has_cb or len(self.env_to_module) or len(self.module_to_env)
        stateful = getattr(self.module, "is_stateful", lambda: False)()
        if stateful:
            if getattr(self, "state", None) is None:
                init = self.module.get_initial_state()
                self.state = {k: np.repeat(v.numpy()[None], N, 0) for k, v in init.items()}
            st_buf = {k: np.empty((T,) + v.shape, np.float32) for k, v in self.state.items()}
        t0 = time.time()
        for t in range(T):
            obs_buf[t] = self.obs
            batch = {"obs": torch.from_numpy(self.obs)}
            if stateful:
                for k, v in self.state.items():
                    st_buf[k][t] = v
                batch["state_in"] = {k: torch.from_numpy(v) for k, v in self.state.items()}
            batch.update(self.explore_extra)
            out = self.module.forward_exploration(batch) if explore else self.module.forward_inference(batch)
            new_state = {k: v.cpu().numpy() for k, v in out["state_out"].items()} if stateful else None
            a = out["actions"].cpu().numpy()
            nraw, r, te, tr, final = self.env.step(self._to_env(out, a, explore))
            done = te | tr
            if track:
                for i, ep in enumerate(self.episodes):
                    ep.add_step(final[i], a[i], r[i], terminated=te[i], truncated=tr[i])
            mfinal = final
            if need_next or tr.any():
                mfinal = self._to_module(final, self.episodes, peek=True) if track else final
            r_aug = r.copy()
            if tr.any() and hasattr(self.module, "compute_values"):
                idx = np.nonzero(tr & ~te)[0]
                if len(idx):
                    vb = {"obs": torch.from_numpy(mfinal[idx])}
                    if stateful:
                        vb["state_in"] = {k: torch.from_numpy(v[idx]) for k, v in new_state.items()}
                    v = self.module.compute_values(vb).cpu().numpy()
                    r_aug[idx] += gamma * v
            if need_next:
                next_buf[t] = mfinal
            acts.append(a)
            if "action_logp" in out:
                logps.append(out["action_logp"].cpu().numpy())
            if "vf_preds" in out:
                vfs.append(out["vf_preds"].cpu().numpy())
            if "action_dist_inputs" in out:
                dist.append(out["action_dist_inputs"].cpu().numpy())
            rews.append(r_aug)
            raw.append(r)
            terms.append(done)
            truncs.append(tr)
            self.ep_ret += r
            self.ep_len += 1
            for i in np.nonzero(done)[0]:
                self.done_returns.append(float(self.ep_ret[i]))
                self.done_lens.append(int(self.ep_len[i]))
                self.new_episodes.append(float(self.ep_ret[i]))
                self.ep_ret[i] = 0
                self.ep_len[i] = 0
                if track:
                    ep = self.episodes[i]
                    if self._has_cb:
                        self.callbacks.on_episode_end(episode=ep, env_runner=self, metrics_logger=self.metrics,
                                                      env=self.env, env_index=int(i), rl_module=self.module)
                    self.env_to_module.episode_done(ep)
                    self.episodes[i] = self._new_episode(int(i), nraw[i])
            if self._has_cb:
                for i in np.nonzero(~done)[0]:
                    self.callbacks.on_episode_step(episode=self.episodes[i], env_runner=self,
                                                   metrics_logger=self.metrics, env=self.env, env_index=int(i),
                                                   rl_module=self.module)
            self.obs = self._to_module(nraw, self.episodes) if track else nraw
            if stateful:  # episodes that ended start again from the initial state
                for k in new_state:
                    new_state[k][done] = 0.0
                self.state = new_state
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
        if stateful:  # recurrent state at every step (sequence starts) and after the fragment
            for k, v in st_buf.items():
                out[f"state_in_{k}"] = v
                out[f"last_state_{k}"] = self.state[k].copy()
        if self._has_cb:
            self.callbacks.on_sample_end(env_runner=self, metrics_logger=self.metrics, samples=out)
        return out

    def reset_envs(self, seed: Optional[int] = None):
        """Start fresh episodes in every env copy (evaluation: same seeds each time)."""
        if seed is not None:
            self.env.seed = seed
        raw = self.env.reset()
        self.state = None  # recurrent state restarts with the episodes
        for i in range(self.env.num_envs):
            self.env_to_module.episode_done(self.episodes[i])
            self.episodes[i] = self._new_episode(i, raw[i])
        self.obs = self._to_module(raw, self.episodes)
        self.ep_ret[:] = 0
        self.ep_len[:] = 0
        return True

    @torch.no_grad()
    def sample_episodes(self, num_episodes: int, explore: bool = False) -> List[float]:
        """Run until ``num_episodes`` episodes finished; returns their returns."""
        start = len(self.new_episodes)
        while len(self.new_episodes) - start < num_episodes:
            self.sample(1, explore)
        rets = self.new_episodes[start:start + num_episodes]
        return rets

    def get_metrics(self, reset_new: bool = True) -> Dict[str, Any]:
        m = {"num_episodes": len(self.new_episodes), "num_env_steps_sampled_lifetime": self.total_steps,
             "episode_returns": list(self.done_returns), "episode_lens": list(self.done_lens),
             "custom": self.metrics.reduce()}
        if reset_new:
            self.new_episodes = []
        return m

    def ping(self):
        return True


class EnvRunnerGroup:
    """A local runner (``num_env_runners == 0``) or N remote runner actors."""

    def __init__(self, config: Dict[str, Any], num_env_runners: int = 0, num_cpus_per_env_runner: float = 1,
                 runner_cls=None):
        self.config = config
        self.runner_cls = runner_cls or EnvRunner
        self.local = None
        self.remote = []
        if num_env_runners == 0:
            self.local = self.runner_cls(config, 0)
        else:
            from ...core import api as core
            from ...core.actor import ActorClass

            Remote = ActorClass(self.runner_cls, {})
            self.remote = [Remote.options(num_cpus=num_cpus_per_env_runner).remote(config, i + 1)
                           for i in range(num_env_runners)]
            core.get([r.ping.remote() for r in self.remote])
        self._merger = None

    def _all(self, method, *args):
        from ...core import api as core

        if self.local is not None:
            return [getattr(self.local, method)(*args)]
        return core.get([getattr(r, method).remote(*args) for r in self.remote])

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

    def sync_connector_states(self):
        """Merge the runners' connector statistics (e.g. MeanStdFilter deltas) and
        broadcast the merged state, so every runner normalises the same way."""
        from ..connectors import build_pipeline

        if not (self.config.get("env_to_module_connector") or self.config.get("module_to_env_connector")):
            return None
        states = self._all("get_connector_state")
        if self._merger is None:
            self._merger = {k: build_pipeline(self.config.get(f"{k}_connector"))
                            for k in ("env_to_module", "module_to_env")}
        merged = {k: p.merge_states([s[k] for s in states]) for k, p in self._merger.items()}
        self._all("set_connector_state", merged)
        return merged

    def sample(self, num_timesteps: Optional[int] = None, explore: bool = True) -> List[Dict]:
        from ...core import api as core

        if self.local is not None:
            return [self.local.sample(num_timesteps, explore)]
        return core.get([r.sample.remote(num_timesteps, explore) for r in self.remote])

    def sample_async(self, num_timesteps: Optional[int] = None):
        return [r.sample.remote(num_timesteps) for r in self.remote]

    def metrics(self) -> Dict[str, Any]:
        from ..utils.metrics import merge_reduced, strip_meta

        ms = self._all("get_metrics")
        rets = [x for m in ms for x in m["episode_returns"]]
        lens = [x for m in ms for x in m["episode_lens"]]
        out = {"episode_return_mean": float(np.mean(rets)) if rets else float("nan"),
               "episode_return_max": float(np.max(rets)) if rets else float("nan"),
               "episode_return_min": float(np.min(rets)) if rets else float("nan"),
               "episode_len_mean": float(np.mean(lens)) if lens else float("nan"),
               "num_episodes": sum(m["num_episodes"] for m in ms),
               "num_env_steps_sampled_lifetime": sum(m["num_env_steps_sampled_lifetime"] for m in ms)}
        for key in ("agent_episode_returns_mean", "module_episode_returns_mean"):
            per = {}
            for m in ms:
                for k, v in (m.get(key) or {}).items():
                    per.setdefault(k, []).extend(v)
            if per:
                out[key] = {k: float(np.mean(v)) for k, v in per.items()}
        custom = merge_reduced([m.get("custom") or {} for m in ms])
        if custom:
            out.update(strip_meta(custom))
        return out

    def stop(self):
        from ...core import api as core

        for r in self.remote:
            try:
                core.kill(r)
            except Exception:
                pass
        self.remote = []
