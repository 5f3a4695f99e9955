"""Multi-agent env runner (reference role: rllib/env/multi_agent_env_runner.py:61).

Steps ``num_envs_per_env_runner`` copies of a ``MultiAgentEnv``. Each env step:

1. the agents that received an observation act; they are grouped by the module
   their agent maps to (``policy_mapping_fn(agent_id, episode)``, fixed per
   episode) and every module runs ONE batched forward over its agents from all
   env copies (through that module's env->module / module->env connectors);
2. per-agent transitions are appended to the agent's open *segment* (one agent
   of one episode, within the current fragment).

A segment closes when its agent is done (terminal; truncation adds
``gamma * V(final_obs)`` to the last reward like the single-agent runner) or at
the fragment end (a cut: ``gamma * V(next obs)`` is added and the step is
marked terminal). The fragment for each module is time-major and padded:
``[T_m, S_m]`` with one column per segment and a ``mask`` of valid steps, so
the learner runs GAE over all columns at once (``rl_returns.hip``) and drops
the padding when flattening.

Off-policy mode (``need_next_obs``, DQN / SAC): segments carry ``next_obs`` and
true termination flags instead — a truncated or cut segment keeps its last
observation as ``next_obs`` with ``terminateds=False`` (the TD target
bootstraps from it), nothing is folded into the rewards.

Recurrent modules (``is_stateful()``): every agent carries its own recurrent
state (reset with its episode); each step's ``state_in_*`` is recorded, and the
fragment length is padded to a multiple of ``max_seq_len`` so the learner can
cut every column into whole sequences.
"""
from __future__ import annotations

import time
from collections import deque
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from . import make_env
from .episodes import MultiAgentEpisode, SingleAgentEpisode

_KEYS = ("action_logp", "vf_preds", "action_dist_inputs")


class _Segment:
    __slots__ = ("mid", "obs", "actions", "rewards", "extra", "closed", "final_obs", "terminated")

    def __init__(self, mid):
        self.mid = mid
        self.obs: List[np.ndarray] = []
        self.actions: List[Any] = []
        self.rewards: List[float] = []
        self.extra: Dict[str, List[np.ndarray]] = {}
        self.closed = False
        self.final_obs = None  # off-policy mode: module-space obs after the last step
        self.terminated = False


def _pad_stack(cols: List[List[np.ndarray]], T: int, fill_like) -> np.ndarray:
    z = np.zeros((T, len(cols)) + np.shape(fill_like), dtype=np.asarray(fill_like).dtype)
    for j, c in enumerate(cols):
        if c:
            z[:len(c), j] = np.stack(c)
    return z


def infer_module_spaces(env, mapping_fn, module_ids, explicit: Optional[Dict[str, tuple]] = None) -> Dict[str, tuple]:
    """module id -> (obs_space, act_space): explicit spaces first, else the
    spaces of an agent that maps to the module (several probe episodes, so a
    random mapping is covered), else the first agent's spaces."""
    out = dict(explicit or {})
    agents = list(getattr(env, "possible_agents", []) or getattr(env, "agents", []))
    for _ in range(8):
        if all(m in out for m in module_ids):
            break
        probe = MultiAgentEpisode()
        for a in agents:
            mid = mapping_fn(a, probe)
            if mid in module_ids and mid not in out:
                out[mid] = (env.get_observation_space(a), env.get_action_space(a))
    for m in module_ids:
        if m not in out and agents:
            out[m] = (env.get_observation_space(agents[0]), env.get_action_space(agents[0]))
    return out


class MultiAgentEnvRunner:
    def __init__(self, config: Dict[str, Any], worker_index: int = 0):
        from ..callbacks import RLlibCallback, make_callbacks
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
        self.callbacks = make_callbacks(config.get("callbacks_class"), config.get("callbacks_functions"))
        self._has_cb = type(self.callbacks) is not RLlibCallback
        n = config.get("num_envs_per_env_runner", 1)
        self.envs = [make_env(config["env"], config.get("env_config")) for _ in range(n)]
        if self._has_cb:
            for e in self.envs:
                self.callbacks.on_environment_created(env_runner=self, metrics_logger=self.metrics, env=e,
                                                      env_context=dict(config.get("env_config") or {},
                                                                       worker_index=worker_index))
        self.mapping_fn = config["policy_mapping_fn"]
        self.module_ids = list(config["policies"])
        env_spaces = infer_module_spaces(self.envs[0], self.mapping_fn, self.module_ids, config.get("policy_spaces"))
        self.e2m, self.m2e, self.spaces = {}, {}, {}
        for mid in self.module_ids:
            o, a = env_spaces[mid]
            self.e2m[mid] = build_pipeline(config.get("env_to_module_connector"), self.envs[0])
            self.e2m[mid].set_input_spaces(o, a)
            self.m2e[mid] = build_pipeline(config.get("module_to_env_connector"), self.envs[0])
            self.m2e[mid].set_input_spaces(o, a)
            self.spaces[mid] = (self.e2m[mid].recompute_output_observation_space(o, a), a)
        self.module = config["multi_module_factory"](self.spaces)
        self.module.eval()
        self.need_next = bool(config.get("need_next_obs", False))
        self.stateful = {mid: bool(getattr(self.module[mid], "is_stateful", lambda: False)())
                         for mid in self.module_ids}
        self.seq_len = int(config.get("max_seq_len") or 1) if any(self.stateful.values()) else 1
        self.rstate: List[Dict[Any, Dict[str, np.ndarray]]] = [{} for _ in range(n)]
        smooth = config.get("metrics_num_episodes_for_smoothing", 100)
        self.done_returns: deque = deque(maxlen=smooth)
        self.done_lens: deque = deque(maxlen=smooth)
        self.agent_returns: Dict[Any, deque] = {}
        self.module_returns: Dict[str, deque] = {}
        self.new_episodes: List[float] = []
        self.total_steps = 0
        self.total_agent_steps = 0
        self.explore_extra: Dict[str, Any] = {}
        base = None if seed is None else seed + 1000 * worker_index
        self.episodes: List[MultiAgentEpisode] = [None] * n  # type: ignore[list-item]
        self.pending: List[Dict[Any, np.ndarray]] = [{} for _ in range(n)]
        self.segments: List[Dict[Any, _Segment]] = [{} for _ in range(n)]
        for i, e in enumerate(self.envs):
            obs, infos = e.reset(seed=None if base is None else base + i)
            self._start_episode(i, obs, infos)

    # ------------------------------------------------------------ helpers
    def _module_for(self, ep: MultiAgentEpisode, agent) -> str:
        mid = ep.module_for_agent.get(agent)
        if mid is None:
            mid = self.mapping_fn(agent, ep)
            if mid not in self.spaces:
                raise KeyError(f"policy_mapping_fn returned unknown module {mid!r} for agent {agent!r}")
            ep.module_for_agent[agent] = mid
        return mid

    def _start_episode(self, i, obs, infos):
        ep = MultiAgentEpisode()
        self.episodes[i] = ep
        for a, o in obs.items():
            ep.agent(a, self._module_for(ep, a)).add_reset(o, (infos or {}).get(a))
        self.pending[i] = dict(obs)
        self.segments[i] = {}
        if hasattr(self, "rstate"):
            self.rstate[i] = {}  # recurrent state restarts with the episode
        if self._has_cb:
            kw = dict(episode=ep, env_runner=self, metrics_logger=self.metrics, env=self.envs[i], env_index=i,
                      rl_module=self.module)
            self.callbacks.on_episode_created(**kw)
            self.callbacks.on_episode_start(**kw)

    def _to_module(self, mid, raw: np.ndarray, eps, peek=False) -> np.ndarray:
        p = self.e2m[mid]
        if not len(p):
            return raw
        return p(rl_module=self.module[mid], batch={"obs": raw}, episodes=eps, shared_data={"peek": peek},
                 metrics=self.metrics)["obs"]

    def _state(self, i, a, mid) -> Dict[str, np.ndarray]:
        st = self.rstate[i].get(a)
        if st is None:
            st = {k: v.detach().cpu().numpy().astype(np.float32)
                  for k, v in self.module[mid].get_initial_state().items()}
            self.rstate[i][a] = st
        return st

    def _value(self, mid, ep: SingleAgentEpisode, raw_obs, state=None) -> float:
        m = self.module[mid]
        if not hasattr(m, "compute_values"):
            return 0.0
        o = self._to_module(mid, np.asarray(raw_obs)[None], [ep], peek=True)
        b = {"obs": torch.from_numpy(np.ascontiguousarray(o))}
        if state:
            b["state_in"] = {k: torch.from_numpy(v[None]) for k, v in state.items()}
        return float(m.compute_values(b)[0])

    def _final(self, seg: _Segment, ep: SingleAgentEpisode, raw_obs):
        """Off-policy mode: the module-space observation after the segment's last step."""
        if raw_obs is not None:
            seg.final_obs = self._to_module(seg.mid, np.asarray(raw_obs)[None], [ep], peek=True)[0]

    def _close(self, seg: _Segment, out: Dict[str, list]):
        if seg.obs and not seg.closed:
            seg.closed = True
            out.setdefault(seg.mid, []).append(seg)

    # ------------------------------------------------------------ weights / spaces
    def set_weights(self, state, extra: Optional[Dict] = None):
        self.module.set_state(state)
        if extra:
            self.explore_extra.update(extra)
        return True

    def get_weights(self):
        return self.module.get_state()

    def get_spaces(self):
        return self.spaces, None

    def get_connector_state(self):
        return {"env_to_module": {m: p.get_state() for m, p in self.e2m.items()},
                "module_to_env": {m: p.get_state() for m, p in self.m2e.items()}}

    def set_connector_state(self, state):
        for k, pipes in (("env_to_module", self.e2m), ("module_to_env", self.m2e)):
            for m, st in (state.get(k) or {}).items():
                if m in pipes:
                    pipes[m].set_state(st)
        return True

    # ------------------------------------------------------------ sampling
    @torch.no_grad()
    def sample(self, num_timesteps: Optional[int] = None, explore: bool = True) -> Dict[str, Any]:
        T = num_timesteps or self.cfg.get("rollout_fragment_length", 64)
        gamma = self.cfg.get("gamma", 0.99)
        done_segs: Dict[str, List[_Segment]] = {}
        agent_steps = 0
        t0 = time.time()
        for _ in range(T):
            # 1. group acting agents by module
            groups: Dict[str, List[Tuple[int, Any]]] = {}
            for i, ep in enumerate(self.episodes):
                for a in self.pending[i]:
                    groups.setdefault(self._module_for(ep, a), []).append((i, a))
            actions: List[Dict[Any, Any]] = [{} for _ in self.envs]
            step_rec: Dict[Tuple[int, Any], tuple] = {}
            for mid, rows in groups.items():
                eps = [self.episodes[i].agent(a) for i, a in rows]
                raw = np.stack([np.asarray(self.pending[i][a]) for i, a in rows])
                mobs = self._to_module(mid, raw, eps)
                b = {"obs": torch.from_numpy(np.ascontiguousarray(mobs))}
                b.update(self.explore_extra)
                m = self.module[mid]
                sts = None
                if self.stateful[mid]:
                    sts = [self._state(i, a, mid) for i, a in rows]
                    b["state_in"] = {k: torch.from_numpy(np.stack([st[k] for st in sts])) for k in sts[0]}
                out = m.forward_exploration(b) if explore else m.forward_inference(b)
                acts = out["actions"].cpu().numpy()
                extra = {k: out[k].cpu().numpy() for k in _KEYS if k in out}
                if sts is not None:
                    for k in sts[0]:
                        extra[f"state_in_{k}"] = np.stack([st[k] for st in sts])
                    new = {k: v.detach().cpu().numpy() for k, v in out["state_out"].items()}
                    for r, (i, a) in enumerate(rows):
                        self.rstate[i][a] = {k: new[k][r] for k in new}
                env_acts = acts
                if len(self.m2e[mid]):
                    mb = dict(extra, actions=acts)
                    env_acts = self.m2e[mid](rl_module=m, batch=mb, episodes=eps, explore=explore, shared_data={},
                                             metrics=self.metrics).get("actions_for_env", acts)
                for r, (i, a) in enumerate(rows):
                    actions[i][a] = env_acts[r]
                    step_rec[(i, a)] = (mid, mobs[r], acts[r], {k: v[r] for k, v in extra.items()})
            # 2. step every env copy
            for i, env in enumerate(self.envs):
                if not actions[i]:
                    continue
                ep = self.episodes[i]
                obs, rew, te, tr, infos = env.step(actions[i])
                ep.env_t += 1
                segs = self.segments[i]
                for a in actions[i]:
                    mid, mo, act, ex = step_rec[(i, a)]
                    seg = segs.get(a)
                    if seg is None or seg.closed:
                        seg = segs[a] = _Segment(mid)
                    seg.obs.append(mo)
                    seg.actions.append(act)
                    seg.rewards.append(float(rew.get(a, 0.0)))
                    for k, v in ex.items():
                        seg.extra.setdefault(k, []).append(v)
                    agent_steps += 1
                    ae = ep.agent(a, mid)
                    ae.add_step(obs.get(a), act, rew.get(a, 0.0), (infos or {}).get(a), te.get(a, False),
                                tr.get(a, False))
                for a, o in obs.items():  # observations of agents that did not act this step
                    if a not in actions[i]:
                        ep.agent(a, self._module_for(ep, a)).add_reset(o, (infos or {}).get(a))
                for a, r in rew.items():  # rewards for agents that did not act this step
                    if a not in actions[i] and a in segs and segs[a].rewards and not segs[a].closed:
                        segs[a].rewards[-1] += float(r)
                        ae = ep.agent(a)
                        if ae.rewards:
                            ae.rewards[-1] += float(r)
                all_done = te.get("__all__", False) or tr.get("__all__", False)
                for a in list(segs):
                    seg = segs[a]
                    if seg.closed:
                        continue
                    a_te, a_tr = te.get(a, False), tr.get(a, False)
                    if a_te or (all_done and not a_tr and te.get("__all__", False)):
                        seg.terminated = True
                        self._close(seg, done_segs)
                    elif a_tr or all_done:  # truncated: bootstrap from the final observation
                        fo = obs.get(a)
                        if self.need_next:
                            self._final(seg, ep.agent(a), fo)
                        elif fo is not None:
                            seg.rewards[-1] += gamma * self._value(seg.mid, ep.agent(a), fo,
                                                                   self.rstate[i].get(a))
                        self._close(seg, done_segs)
                    if a_te or a_tr:
                        self.rstate[i].pop(a, None)
                self.pending[i] = {a: o for a, o in obs.items() if not (te.get(a) or tr.get(a))}
                if all_done:
                    self._finish_episode(i)
                    o2, inf2 = env.reset()
                    self._start_episode(i, o2, inf2)
                elif self._has_cb:
                    self.callbacks.on_episode_step(episode=ep, env_runner=self, metrics_logger=self.metrics,
                                                   env=env, env_index=i, rl_module=self.module)
        # 3. fragment end: cut the open segments (bootstrap from the pending obs)
        for i, segs in enumerate(self.segments):
            ep = self.episodes[i]
            for a, seg in segs.items():
                if seg.closed or not seg.obs:
                    continue
                po = self.pending[i].get(a)
                if self.need_next:
                    self._final(seg, ep.agent(a), po)
                elif po is not None:
                    seg.rewards[-1] += gamma * self._value(seg.mid, ep.agent(a), po, self.rstate[i].get(a))
                self._close(seg, done_segs)
            self.segments[i] = {}
        self.total_steps += T * len(self.envs)
        self.total_agent_steps += agent_steps
        batches = {mid: self._pack(segs) for mid, segs in done_segs.items()}
        res = {"policy_batches": batches, "env_steps": T * len(self.envs), "agent_steps": agent_steps,
               "sample_time_s": time.time() - t0}
        if self._has_cb:
            self.callbacks.on_sample_end(env_runner=self, metrics_logger=self.metrics, samples=res)
        return res

    def reset_envs(self, seed: Optional[int] = None):
        for i, e in enumerate(self.envs):
            obs, infos = e.reset(seed=None if seed is None else seed + i)
            self._start_episode(i, obs, infos)
        return True

    @torch.no_grad()
    def sample_episodes(self, num_episodes: int, explore: bool = False) -> List[float]:
        """Run until ``num_episodes`` episodes finished; returns their (all-agent) returns."""
        start = len(self.new_episodes)
        while len(self.new_episodes) - start < num_episodes:
            self.sample(1, explore)
        return self.new_episodes[start:start + num_episodes]

    def _pack(self, segs: List[_Segment]) -> Dict[str, np.ndarray]:
        Tm = max(len(s.obs) for s in segs)
        L = self.seq_len
        Tm = ((Tm + L - 1) // L) * L  # recurrent: whole max_seq_len sequences per column
        S = len(segs)
        f = {"obs": _pad_stack([s.obs for s in segs], Tm, segs[0].obs[0]),
             "actions": _pad_stack([s.actions for s in segs], Tm, np.asarray(segs[0].actions[0])),
             "rewards": _pad_stack([[np.float32(r) for r in s.rewards] for s in segs], Tm, np.float32(0))}
        for k in segs[0].extra:
            f[k] = _pad_stack([s.extra.get(k, []) for s in segs], Tm, segs[0].extra[k][0]).astype(np.float32)
        mask = np.zeros((Tm, S), bool)
        term = np.zeros((Tm, S), bool)
        if self.need_next:  # transitions: next_obs within the segment, then its final obs
            nxt = np.zeros_like(f["obs"])
            for j, s in enumerate(segs):
                n = len(s.obs)
                mask[:n, j] = True
                if n > 1:
                    nxt[:n - 1, j] = np.stack(s.obs[1:])
                if s.final_obs is not None:
                    nxt[n - 1, j] = s.final_obs
                term[n - 1, j] = s.terminated or s.final_obs is None
            f["next_obs"] = nxt
        else:
            for j, s in enumerate(segs):
                mask[:len(s.obs), j] = True
                term[len(s.obs) - 1:, j] = True  # every column ends terminal (done or cut) and stays so
        f["mask"] = mask
        f["terminateds"] = term
        f["truncateds"] = np.zeros((Tm, S), bool)
        f["last_obs"] = f["obs"][-1].copy()
        return f

    def _finish_episode(self, i):
        ep = self.episodes[i]
        ep.is_terminated = True
        ret = ep.get_return()
        self.done_returns.append(ret)
        self.done_lens.append(ep.env_t)
        self.new_episodes.append(ret)
        per_mod: Dict[str, float] = {}
        for a, ae in ep.agent_episodes.items():
            self.agent_returns.setdefault(str(a), deque(maxlen=self.done_returns.maxlen)).append(ae.get_return())
            mid = ep.module_for_agent.get(a)
            if mid is not None:
                per_mod[mid] = per_mod.get(mid, 0.0) + ae.get_return()
            p = self.e2m.get(mid)
            if p is not None:
                p.episode_done(ae)
        for mid, r in per_mod.items():
            self.module_returns.setdefault(mid, deque(maxlen=self.done_returns.maxlen)).append(r)
        if self._has_cb:
            self.callbacks.on_episode_end(episode=ep, env_runner=self, metrics_logger=self.metrics,
                                          env=self.envs[i], env_index=i, rl_module=self.module)

    def get_metrics(self, reset_new: bool = True) -> Dict[str, Any]:
        m = {"num_episodes": len(self.new_episodes), "num_env_steps_sampled_lifetime": self.total_steps,
             "num_agent_steps_sampled_lifetime": self.total_agent_steps,
             "episode_returns": list(self.done_returns), "episode_lens": list(self.done_lens),
             "agent_episode_returns_mean": {a: list(v) for a, v in self.agent_returns.items()},
             "module_episode_returns_mean": {k: list(v) for k, v in self.module_returns.items()},
             "custom": self.metrics.reduce()}
        if reset_new:
            self.new_episodes = []
        return m

    def ping(self):
        return True


def concat_multi_agent(frags: List[Dict[str, Any]]) -> Dict[str, Dict[str, np.ndarray]]:
    """Merge several runners' ``policy_batches``: pad every module's columns to
    the longest T and concatenate along the column axis."""
    out: Dict[str, Dict[str, np.ndarray]] = {}
    mids = []
    for f in frags:
        mids += [m for m in f["policy_batches"] if m not in mids]
    for mid in mids:
        parts = [f["policy_batches"][mid] for f in frags if mid in f["policy_batches"]]
        Tm = max(p["rewards"].shape[0] for p in parts)
        merged = {}
        for k in parts[0]:
            if k == "last_obs":
                merged[k] = np.concatenate([p[k] for p in parts], 0)
                continue
            cols = []
            for p in parts:
                v = p[k]
                if v.shape[0] < Tm:
                    pad = np.zeros((Tm - v.shape[0],) + v.shape[1:], v.dtype)
                    if k == "terminateds":
                        pad[:] = True
                    v = np.concatenate([v, pad], 0)
                cols.append(v)
            merged[k] = np.concatenate(cols, 1)
        out[mid] = merged
    return out
