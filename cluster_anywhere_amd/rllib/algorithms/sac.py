"""SAC (reference: rllib/algorithms/sac/sac.py, sac_learner.py,
torch/sac_torch_learner.py): tanh-squashed Gaussian policy, twin Q networks
with Polyak-averaged targets, automatic entropy temperature. Three parameter
groups (policy / twin-Q / log-alpha), each its own flat buffer + fused AdamW."""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn

from ..core.learner import Learner
from ..core.rl_module import RLModule, _act, mlp
from ..env import Box
from .algorithm import Algorithm, AlgorithmConfig, OffPolicyMixin


class SACModule(RLModule):
    def setup(self):
        mc = self.model_config
        assert isinstance(self.action_space, Box), "SAC (here) needs a continuous action space"
        d = int(np.prod(self.observation_space.shape))
        na = int(np.prod(self.action_space.shape))
        hp = list(mc.get("policy_hiddens", [256, 256]))
        hq = list(mc.get("q_hiddens", [256, 256]))
        act = _act(mc.get("fcnet_activation", "relu"))
        self.pi_net = mlp([d] + hp + [2 * na], act)
        self.q1 = mlp([d + na] + hq + [1], act)
        self.q2 = mlp([d + na] + hq + [1], act)
        self.log_alpha = nn.Parameter(torch.tensor(math.log(mc.get("initial_alpha", 1.0))))
        low = torch.as_tensor(self.action_space.low, dtype=torch.float32)
        high = torch.as_tensor(self.action_space.high, dtype=torch.float32)
        self.register_buffer("a_scale", (high - low) / 2)
        self.register_buffer("a_bias", (high + low) / 2)

    def policy(self, obs, deterministic=False):
        mean, log_std = self.pi_net(obs.reshape(obs.shape[0], -1).float()).chunk(2, -1)
        log_std = log_std.clamp(-20, 2)
        std = log_std.exp()
        u = mean if deterministic else mean + std * torch.randn_like(mean)
        a = torch.tanh(u)
        logp = (-0.5 * ((u - mean) / std) ** 2 - log_std - 0.5 * math.log(2 * math.pi)).sum(-1)
        logp = logp - (2 * (math.log(2) - u - nn.functional.softplus(-2 * u))).sum(-1)
        return a * self.a_scale + self.a_bias, logp

    def qs(self, obs, a):
        x = torch.cat([obs.reshape(obs.shape[0], -1).float(), (a - self.a_bias) / self.a_scale], -1)
        return self.q1(x).squeeze(-1), self.q2(x).squeeze(-1)

    @torch.no_grad()
    def forward_exploration(self, batch):
        a, _ = self.policy(batch["obs"])
        return {"actions": a}

    @torch.no_grad()
    def forward_inference(self, batch):
        a, _ = self.policy(batch["obs"], deterministic=True)
        return {"actions": a}


class _Group(nn.Module):
    def __init__(self, *mods):
        super().__init__()
        self.mods = nn.ModuleList(mods)


class _Param(nn.Module):
    def __init__(self, p):
        super().__init__()
        self.p = p


class SACConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or SAC)
        self.actor_lr = 3e-4
        self.critic_lr = 3e-4
        self.alpha_lr = 3e-4
        self.lr = None
        self.tau = 5e-3
        self.initial_alpha = 1.0
        self.target_entropy = "auto"
        self.train_batch_size = 256
        self.rollout_fragment_length = 1
        self.num_steps_sampled_before_learning_starts = 1000
        self.replay_buffer_config = {"type": "ReplayBuffer", "capacity": 100_000}
        self.training_intensity = None
        self.twin_q = True

    def default_module_class(self):
        return SACModule

    def algo_model_config(self):
        mc = dict(self.model_config)
        mc.setdefault("initial_alpha", self.initial_alpha)
        return mc

    def module_factory(self):
        mc = self.algo_model_config()
        cls = self.rl_module_class or SACModule
        return lambda o, a: cls(o, a, mc)

    def runner_config(self):
        d = super().runner_config()
        d["need_next_obs"] = True
        return d


class SACLearner(Learner):
    def build(self):
        import copy

        self.target_q = _Group(copy.deepcopy(self.module.q1), copy.deepcopy(self.module.q2))
        for p in self.target_q.parameters():
            p.requires_grad_(False)
        te = self.config.get("target_entropy", "auto")
        self.target_entropy = -float(np.prod(self.act_space.shape)) if te == "auto" else float(te)

    def param_groups(self):
        m = self.module
        return {"policy": m.pi_net, "qf": _Group(m.q1, m.q2), "alpha": _Param(m.log_alpha)}

    def lr_for(self, name):
        c = self.config
        return {"policy": c["actor_lr"], "qf": c["critic_lr"], "alpha": c["alpha_lr"]}[name]

    def compute_loss(self, batch):
        c = self.config
        m = self.module
        obs, act, nobs = batch["obs"], batch["actions"].float(), batch["next_obs"]
        alpha = m.log_alpha.exp()
        with torch.no_grad():
            na, nlogp = m.policy(nobs)
            x = torch.cat([nobs.reshape(nobs.shape[0], -1).float(), (na - m.a_bias) / m.a_scale], -1)
            tq = torch.min(self.target_q.mods[0](x), self.target_q.mods[1](x)).squeeze(-1)
            target = batch["rewards"] + c["gamma"] * (1 - batch["terminateds"]) * (tq - alpha.detach() * nlogp)
        q1, q2 = m.qs(obs, act)
        w = batch.get("weights", torch.ones_like(q1))
        qf_loss = 0.5 * (w * ((q1 - target) ** 2 + (q2 - target) ** 2)).mean()
        a, logp = m.policy(obs)
        q1p, q2p = m.qs(obs, a)
        pi_loss = (alpha.detach() * logp - torch.min(q1p, q2p)).mean()
        alpha_loss = -(m.log_alpha * (logp.detach() + self.target_entropy)).mean()
        self._td = (q1 - target).detach()
        return ({"qf": qf_loss, "policy": pi_loss, "alpha": alpha_loss},
                {"qf_loss": qf_loss.detach(), "policy_loss": pi_loss.detach(), "alpha_value": alpha.detach(),
                 "alpha_loss": alpha_loss.detach(), "qf_mean": q1.mean().detach()})

    def after_update(self):
        tau = self.config["tau"]
        with torch.no_grad():
            src = list(self.module.q1.parameters()) + list(self.module.q2.parameters())
            for pt, p in zip(self.target_q.parameters(), src):
                pt.mul_(1 - tau).add_(p, alpha=tau)

    def train_on(self, batch):
        stats = self.update(batch)
        return stats, self._td.abs().cpu().numpy()

    def get_state(self):
        st = super().get_state()
        st["target_q"] = {k: v.cpu() for k, v in self.target_q.state_dict().items()}
        return st

    def set_state(self, st):
        super().set_state(st)
        if "target_q" in st:
            self.target_q.load_state_dict(st["target_q"])
        return True


class SAC(OffPolicyMixin, Algorithm):
    config_class = SACConfig
    learner_class = SACLearner
    supports_multi_agent = True
    default_capacity = 100_000

    def setup_algo(self):
        self.setup_replay()

    def training_step(self):
        c = self.algo_config
        steps = self.sample_into_replay()
        stats = {}
        if self.replay_ready():
            n_updates = 1 if not c.training_intensity else max(1, int(round(
                c.training_intensity * steps / c.train_batch_size)))
            for _ in range(n_updates):
                stats = self.replay_update()
        self._sync_weights()
        return stats
