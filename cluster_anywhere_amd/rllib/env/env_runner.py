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
        # num_gpus_per_env_runner > 0: act on the runner's (fractional) GPU
        self.device = torch.device("cpu")
        if config.get("num_gpus_per_env_runner", 0) and torch.cuda.is_available():
            self.device = torch.device("cuda", 0)
            self.module.to(self.device)
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
        # config.offline_data(output=...): record every sampled step (whole episodes per file)
        self.recorder = None
        if config.get("output"):
            from ..offline.io import EpisodeRecorder

            self.recorder = EpisodeRecorder(config["output"], worker_index, self.env.num_envs,
                                            config.get("output_max_rows_per_file") or 10_000,
                                            config.get("output_write_episodes", True))

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
        rec = self.recorder
        need_next = self.cfg.get("need_next_obs", False) or rec is not None
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
            dev = self.device
            batch = {"obs": torch.from_numpy(self.obs).to(dev, non_blocking=True)}
            if stateful:
                for k, v in self.state.items():
                    st_buf[k][t] = v
                batch["state_in"] = {k: torch.from_numpy(v).to(dev) for k, v in self.state.items()}
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
                    vb = {"obs": torch.from_numpy(mfinal[idx]).to(self.device)}
                    if stateful:
                        vb["state_in"] = {k: torch.from_numpy(v[idx]).to(self.device) for k, v in new_state.items()}
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
            if rec is not None:
                lp = out["action_logp"].cpu().numpy() if "action_logp" in out else None
                vf = out["vf_preds"].cpu().numpy() if "vf_preds" in out else None
                for i in range(N):
                    rec.add_step(i, obs_buf[t][i], mfinal[i] if done[i] else self.obs[i], a[i], r[i], te[i], tr[i],
                                 None if lp is None else lp[i], None if vf is None else vf[i])
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

    def flush_output(self, include_open: bool = True) -> List[str]:
        """Write the recorded episodes (``config.offline_data(output=...)``) still
        buffered; with ``include_open`` unfinished episodes too (as truncated).
        Returns every file this runner has written."""
        if self.recorder is None:
            return []
        self.recorder.flush(include_open=include_open)
        return list(self.recorder.files_written)

    def stop(self):
        self.flush_output()
        return True


def _actor_failures():
    from ...exceptions import RayActorError, WorkerCrashedError

    return (RayActorError, WorkerCrashedError)


class EnvRunnerGroup:
    """A local runner (``num_env_runners == 0``) or N remote runner actors.

    Remote runners are fault tolerant (reference role: ``env_runner_group.py`` over
    ``FaultTolerantActorManager``): every fan-out call collects its results per
    runner, and a runner whose actor died is, by default
    (``restart_failed_env_runners``), replaced by a fresh runner at the same index
    that gets the last broadcast weights and connector state before it rejoins
    (``on_recreated`` fires with the indices). With restarts off,
    ``ignore_env_runner_failures`` keeps training on the healthy runners; otherwise
    the failure is raised. A fan-out never waits on a dead runner's result."""

    def __init__(self, config: Dict[str, Any], num_env_runners: int = 0, num_cpus_per_env_runner: float = 1,
                 runner_cls=None, *, num_gpus_per_env_runner: float = 0, restart_failed: bool = True,
                 ignore_failures: bool = False,
                 max_restarts: int = 1000, restart_delay_s: float = 0.0, on_recreated=None):
        self.config = config
        self.runner_cls = runner_cls or EnvRunner
        self.local = None
        self.remote = []
        self.restart_failed = restart_failed
        self.ignore_failures = ignore_failures
        self.max_restarts = max_restarts
        self.restart_delay_s = restart_delay_s
        self.on_recreated = on_recreated
        self.num_restarts = 0
        self._weights = None  # (object ref, extra) of the last broadcast
        self._connector_state = None
        if num_env_runners == 0:
            self.local = self.runner_cls(config, 0)
        else:
            from ...core import api as core
            from ...core.actor import ActorClass

            Remote = ActorClass(self.runner_cls, {})
            self._spawn = lambda i: Remote.options(num_cpus=num_cpus_per_env_runner,
                                                   num_gpus=num_gpus_per_env_runner).remote(config, i + 1)
            self.remote = [self._spawn(i) for i in range(num_env_runners)]
            self.healthy = [True] * num_env_runners
            core.get([r.ping.remote() for r in self.remote])
        self._merger = None

    # -------------------------------------------------------- fault tolerance
    def healthy_indices(self) -> List[int]:
        return [i for i, ok in enumerate(self.healthy) if ok] if self.remote else []

    def _fanout(self, method, *args, indices=None) -> Dict[int, Any]:
        """``method(*args)`` on the given (default: every healthy) remote runner;
        {index: result} of the runners that answered. Failed runners are handled
        (restored / dropped / raised) before this returns."""
        from ...core import api as core

        idx = self.healthy_indices() if indices is None else list(indices)
        calls = {i: getattr(self.remote[i], method).remote(*args) for i in idx}
        return self._gather(calls)

    def _gather(self, calls: Dict[int, Any]) -> Dict[int, Any]:
        from ...core import api as core

        out, failed = {}, []
        for i, ref in calls.items():
            try:
                out[i] = core.get(ref)
            except _actor_failures() as e:  # noqa: PERF203
                failed.append((i, e))
        if failed:
            self.handle_failures(failed)
        return out

    def handle_failures(self, failed) -> None:
        """[(index, error)] of runners whose actor died."""
        import logging

        for i, _ in failed:
            self.healthy[i] = False
        logging.getLogger(__name__).warning("env runner(s) %s failed: %s", [i for i, _ in failed], failed[0][1])
        if self.restart_failed:
            self.restore([i for i, _ in failed])
        elif not self.ignore_failures:
            raise failed[0][1]
        if not self.healthy_indices():
            raise RuntimeError("every env runner has failed and none could be restored") from failed[0][1]

    def restore(self, indices: List[int]) -> List[int]:
        """Replace the runners at ``indices`` by fresh actors brought up to date."""
        import time as _time

        from ...core import api as core

        todo = list(indices)
        for attempt in range(3):
            if not todo:
                break
            if self.num_restarts + len(todo) > self.max_restarts:
                raise RuntimeError(f"env runners {todo} failed after {self.num_restarts} restarts "
                                   f"(max_num_env_runner_restarts={self.max_restarts})")
            if self.restart_delay_s > 0:
                _time.sleep(self.restart_delay_s)
            for i in todo:
                try:
                    core.kill(self.remote[i])
                except Exception:  # noqa: BLE001 - already gone
                    pass
                self.remote[i] = self._spawn(i)
                self.num_restarts += 1
            try:
                self._catch_up(todo)
            except _actor_failures():
                continue  # a replacement died while starting: replace it again
            for i in todo:
                self.healthy[i] = True
            if self.on_recreated is not None:
                self.on_recreated(list(todo))
            return list(todo)
        raise RuntimeError(f"could not restore env runners {todo}")

    def _catch_up(self, idx: List[int]) -> None:
        from ...core import api as core

        core.get([self.remote[i].ping.remote() for i in idx])
        if self._weights is not None:
            core.get([self.remote[i].set_weights.remote(*self._weights) for i in idx])
        if self._connector_state is not None:
            core.get([self.remote[i].set_connector_state.remote(self._connector_state) for i in idx])

    # ----------------------------------------------------------------- calls
    def _all(self, method, *args):
        if self.local is not None:
            return [getattr(self.local, method)(*args)]
        res = self._fanout(method, *args)
        return [res[i] for i in sorted(res)]

    def spaces(self):
        if self.local is not None:
            return self.local.get_spaces()
        while True:
            res = self._fanout("get_spaces", indices=self.healthy_indices()[:1])
            if res:
                return next(iter(res.values()))

    def sync_weights(self, state, extra: Optional[Dict] = None, transport: Optional[str] = None):
        """``transport="ipc"``: ``state`` holds GPU tensors that same-node GPU runners
        map through HIP IPC handles and copy device-to-device (no host round trip)."""
        from ...core import api as core

        if self.local is not None:
            self.local.set_weights(state, extra)
            return
        self._weights = (core.put(state, _tensor_transport=transport), extra)
        # an "ipc" ref carries HIP IPC handles into THESE device tensors: keep them
        # alive while the ref is what restarted runners receive (_catch_up), so their
        # HBM is not handed to other tensors by the caching allocator in between
        self._weights_keep = state if transport == "ipc" else None
        self._fanout("set_weights", *self._weights)

    def sync_weights_to(self, state, indices: List[int], extra: Optional[Dict] = None):
        """Broadcast to some runners only (async samplers refresh the ones that
        just returned); the state also becomes what restored runners get."""
        from ...core import api as core

        self._weights = (core.put(state), extra)
        self._weights_keep = None  # a host-copy ref: nothing on the device to pin
        self._fanout("set_weights", *self._weights, indices=[i for i in indices if self.healthy[i]])

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
        self._connector_state = merged
        self._all("set_connector_state", merged)
        return merged

    def sample(self, num_timesteps: Optional[int] = None, explore: bool = True) -> List[Dict]:
        if self.local is not None:
            return [self.local.sample(num_timesteps, explore)]
        for _ in range(3):
            res = self._fanout("sample", num_timesteps, explore)
            if res:
                return [res[i] for i in sorted(res)]
        raise RuntimeError("no env runner returned a sample")

    def sample_async(self, num_timesteps: Optional[int] = None):
        return [self.remote[i].sample.remote(num_timesteps) for i in self.healthy_indices()]

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

    def flush_output(self) -> List[str]:
        """Flush every runner's recorded episodes; the files written so far."""
        if self.local is not None:
            return self.local.flush_output()
        out = []
        for v in self._fanout("flush_output").values():
            out.extend(v)
        return sorted(out)

    def stop(self):
        from ...core import api as core

        if self.local is not None and hasattr(self.local, "stop"):
            self.local.stop()
        elif self.remote:
            try:
                self.flush_output()
            except Exception:
                pass
        for r in self.remote:
            try:
                core.kill(r)
            except Exception:
                pass
        self.remote = []
