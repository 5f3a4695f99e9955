"""IMPALA and APPO (reference: rllib/algorithms/impala/impala.py,
impala_learner.py, torch/vtrace_torch_v2.py; rllib/algorithms/appo/appo.py,
appo_learner.py).

EnvRunners sample asynchronously: every runner always has one ``sample``
call in flight; each training step consumes the fragments that are ready,
refreshes only those runners' weights and re-launches them. Off-policy
correction is V-trace on the learner device (``rl_returns.hip`` kernel, one
thread per env column, reverse scan over T). APPO replaces the IMPALA policy
gradient by PPO's clipped surrogate on the V-trace advantages, with a target
network providing the KL anchor.

Multi-agent: every module learns from its own padded ``[T_m, S_m]`` fragment
(one column per agent segment, ``mask`` marks real steps; a segment's last
step is terminal or cut, so V-trace never crosses into the padding); the loss
averages over real steps only. Recurrent modules (``use_lstm`` / ``use_attention``),
single- or multi-agent, unroll each column as one T-step sequence from the state
the runner recorded at its first step (``state_in_*``), reset at episode starts.
"""
from __future__ import annotations

import copy
from typing import Any, Dict, List

import numpy as np
import torch

from ...ops.rl import vtrace
from ..core.learner import Learner, _to_tensor
from .algorithm import Algorithm, AlgorithmConfig, concat_fragments


class IMPALAConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or IMPALA)
        self.lr = 5e-4
        self.vtrace_clip_rho_threshold = 1.0
        self.vtrace_clip_pg_rho_threshold = 1.0
        self.vf_loss_coeff = 0.5
        self.entropy_coeff = 0.01
        self.rollout_fragment_length = 50
        self.train_batch_size = 500
        self.minibatch_size = None
        self.num_epochs = 1
        self.grad_clip = 40.0
        self.max_requests_in_flight_per_env_runner = 1
        # APPO
        self.clip_param = 0.4
        self.use_kl_loss = False
        self.kl_coeff = 1.0
        self.target_network_update_freq = 1


class IMPALALearner(Learner):
    appo = False

    def build(self):
        if self.appo:
            self.target = copy.deepcopy(self.module)
            for p in self.target.parameters():
                p.requires_grad_(False)
            self.updates_since_target = 0

    def compute_loss(self, b):
        c = self.config
        T, N = b["rewards"].shape
        flat = lambda x: x.reshape((T * N,) + tuple(x.shape[2:]))
        mask = b.get("mask")
        if mask is None:
            mean = lambda x: x.mean()
        else:
            msum = mask.sum().clamp(min=1.0)
            mean = lambda x: (x * mask.reshape(x.shape)).sum() / msum
        stateful = bool(getattr(self.module, "is_stateful", lambda: False)())
        if stateful:
            # recurrent module: each env / agent-segment column is ONE sequence of T
            # steps, unrolled from the state recorded at the fragment's first step
            # and reset where an episode starts inside it (reference role:
            # add_states_from_episodes_to_batch.py for IMPALA / APPO)
            train_in = self._seq_batch(b, T, N)
            out = self.module.forward_train(train_in)
            tm = lambda x: x.view((N, T) + tuple(x.shape[1:])).transpose(0, 1).reshape((T * N,) + tuple(x.shape[1:]))  # noqa: E731
            out = {k: tm(v) for k, v in out.items() if isinstance(v, torch.Tensor)}
        else:
            train_in = {"obs": flat(b["obs"])}
            out = self.module.forward_train(train_in)
        dist = self.module.dist_cls(out["action_dist_inputs"])
        logp = dist.logp(flat(b["actions"])).view(T, N)
        values = out["vf_preds"].view(T, N)
        with torch.no_grad():
            vb = {"obs": b["last_obs"]}
            last_st = {k[len("last_state_"):]: v for k, v in b.items() if k.startswith("last_state_")}
            if stateful and last_st:
                vb["state_in"] = last_st
            boot = self.module.compute_values(vb)
            disc = c["gamma"] * (1.0 - b["terminateds"].float())
            vs, pg_adv = vtrace(logp.detach() - b["action_logp"], disc, b["rewards"], values.detach(), boot,
                                c["vtrace_clip_rho_threshold"], c["vtrace_clip_pg_rho_threshold"])
        if self.appo:
            ratio = torch.exp(logp - b["action_logp"])
            mu = mean(pg_adv)
            adv = (pg_adv - mu) / (mean((pg_adv - mu) ** 2).sqrt() + 1e-8)
            cp = c["clip_param"]
            pi_loss = -mean(torch.min(ratio * adv, ratio.clamp(1 - cp, 1 + cp) * adv))
        else:
            pi_loss = -mean(logp * pg_adv)
        vf_loss = 0.5 * mean((values - vs) ** 2)
        ent = mean(dist.entropy().view(T, N))
        loss = pi_loss + c["vf_loss_coeff"] * vf_loss - c["entropy_coeff"] * ent
        stats = {"total_loss": loss.detach(), "policy_loss": pi_loss.detach(), "vf_loss": vf_loss.detach(),
                 "entropy": ent.detach()}
        if self.appo and c.get("use_kl_loss"):
            with torch.no_grad():
                old = self.target.forward_train(train_in)["action_dist_inputs"]
                if stateful:
                    old = tm(old)
            kl = mean(self.module.dist_cls(old).kl(dist).view(T, N))
            loss = loss + c["kl_coeff"] * kl
            stats["mean_kl_loss"] = kl.detach()
        return {"default": loss}, stats

    @staticmethod
    def _seq_batch(b, T, N):
        seq = lambda x: x.transpose(0, 1).contiguous()  # noqa: E731  [T, N, ...] -> [N, T, ...]
        prev_term = torch.zeros_like(b["terminateds"], dtype=torch.float32)
        prev_term[1:] = b["terminateds"][:-1].float()
        st = {k[len("state_in_"):]: v[0].float() for k, v in b.items() if k.startswith("state_in_")}
        out = {"obs": seq(b["obs"]), "resets": seq(prev_term)}
        if st:
            out["state_in"] = st
        return out

    def after_update(self):
        if self.appo:
            self.updates_since_target += 1
            if self.updates_since_target >= self.config.get("target_network_update_freq", 1):
                self.target.load_state_dict(self.module.state_dict())
                self.updates_since_target = 0

    def learn_fragments(self, frag: Dict[str, Any]):
        keys = ["obs", "actions", "rewards", "terminateds", "action_logp"]
        b = {k: _to_tensor(frag[k], self.device) for k in keys}
        b["rewards"] = b["rewards"].float()
        b["last_obs"] = _to_tensor(frag["last_obs"], self.device)
        for k in frag:  # recurrent modules: per-step states and the state after the last step
            if k.startswith(("state_in_", "last_state_")):
                b[k] = _to_tensor(frag[k], self.device)
        if "mask" in frag:
            b["mask"] = _to_tensor(frag["mask"], self.device).float()
        return {k: float(v) for k, v in self.update_once(b).items()}


class APPOLearner(IMPALALearner):
    appo = True


class IMPALA(Algorithm):
    config_class = IMPALAConfig
    learner_class = IMPALALearner
    supports_multi_agent = True
    supports_recurrent_multi_agent = True

    def setup_algo(self):
        self._inflight: Dict[int, Any] = {}

    def _collect(self) -> List[Dict]:
        g = self.env_runner_group
        if g.local is not None:
            return g.sample()
        from ...core import api as core

        frags = []
        while not frags:
            for i in g.healthy_indices():
                if i not in self._inflight:
                    self._inflight[i] = g.remote[i].sample.remote()
            ready, _ = core.wait(list(self._inflight.values()), num_returns=1)
            ready_set = set(ready)
            results = g._gather({i: ref for i, ref in self._inflight.items() if ref in ready_set})
            for i in [i for i, ref in self._inflight.items() if ref in ready_set]:
                del self._inflight[i]  # answered, or failed (then restored / dropped)
            frags = [results[i] for i in sorted(results)]
            done = sorted(results)
        # only the runners that returned get fresh weights (others keep sampling)
        g.sync_weights_to(self.learner_group.get_module_state(), done)
        for i in done:
            if g.healthy[i]:
                self._inflight[i] = g.remote[i].sample.remote()
        return frags

    def _sync_weights(self, extra=None):
        if self.env_runner_group.local is not None or not getattr(self, "_inflight", None):
            super()._sync_weights(extra)

    def training_step(self):
        c = self.algo_config
        frags = self._collect()
        if self.is_multi_agent:
            from ..env.multi_agent_env_runner import concat_multi_agent

            frag = concat_multi_agent(frags)
            steps = sum(f["env_steps"] for f in frags)
            self.agent_steps_sampled += sum(f["agent_steps"] for f in frags)
        else:
            frag = concat_fragments(frags)
            steps = int(frag["rewards"].size)
        self.env_steps_sampled += steps
        lg = self.learner_group
        stats = lg.local.learn_fragments(frag) if lg.local is not None else lg.call("learn_fragments", frag)
        self.env_steps_trained += steps
        if self.env_runner_group.local is not None:
            self._sync_weights()
        return stats


class APPOConfig(IMPALAConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or APPO)
        self.use_kl_loss = True
        self.kl_coeff = 0.1
        self.lr = 5e-4


class APPO(IMPALA):
    config_class = APPOConfig
    learner_class = APPOLearner
