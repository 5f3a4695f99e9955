"""CQL — Conservative Q-Learning, offline (reference: rllib/algorithms/cql/cql.py,
torch/cql_torch_learner.py). SAC's actor / twin-Q / temperature on a static
dataset, plus the conservative regulariser that pushes Q down on actions the
data does not support:

    L_cql = w * ( T * logsumexp_a'(Q(s, a') / T) - Q(s, a_data) )

with a' drawn uniformly from the action box and from the current policy at s and
s' (importance-corrected by their log-densities). The first ``bc_iters`` updates
train the actor by behaviour cloning (log-likelihood of the data action).
Optional Lagrangian tuning of w keeps the CQL gap near ``lagrangian_thresh``."""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn

from .sac import SAC, SACConfig, SACLearner, _Param


class CQLConfig(SACConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or CQL)
        self.bc_iters = 200
        self.temperature = 1.0
        self.num_actions = 10
        self.lagrangian = False
        self.lagrangian_thresh = 5.0
        self.min_q_weight = 5.0
        self.updates_per_iteration = 1
        self.num_steps_sampled_before_learning_starts = 0


class CQLLearner(SACLearner):
    def build(self):
        super().build()
        self.n_updates = 0
        if self.config.get("lagrangian"):
            self.log_alpha_prime = nn.Parameter(torch.zeros((), device=self.module.log_alpha.device))

    def param_groups(self):
        g = super().param_groups()
        if self.config.get("lagrangian"):
            g["alpha_prime"] = _Param(self.log_alpha_prime)
        return g

    def lr_for(self, name):
        if name == "alpha_prime":
            return self.config["critic_lr"]
        return super().lr_for(name)

    def _data_logp(self, obs, act):
        """log pi(a_data | s) of the tanh-squashed Gaussian (for the BC phase)."""
        m = self.module
        mean, log_std = m.pi_net(obs.reshape(obs.shape[0], -1).float()).chunk(2, -1)
        log_std = log_std.clamp(-20, 2)
        y = ((act - m.a_bias) / m.a_scale).clamp(-1 + 1e-6, 1 - 1e-6)
        u = torch.atanh(y)
        logp = (-0.5 * ((u - mean) / log_std.exp()) ** 2 - log_std - 0.5 * math.log(2 * math.pi)).sum(-1)
        return logp - (2 * (math.log(2) - u - nn.functional.softplus(-2 * u))).sum(-1)

    def _repeat_q(self, obs, acts):
        """Q1, Q2 of ``acts`` [B, N, A] at ``obs`` [B, ...] -> two [B, N] tensors."""
        m = self.module
        B, N = acts.shape[:2]
        o = obs.reshape(B, -1).float().unsqueeze(1).expand(B, N, -1).reshape(B * N, -1)
        q1, q2 = m.qs(o, acts.reshape(B * N, -1))
        return q1.view(B, N), q2.view(B, N)

    def _policy_actions(self, obs, n):
        m = self.module
        B = obs.shape[0]
        o = obs.reshape(B, -1).float().unsqueeze(1).expand(B, n, -1).reshape(B * n, -1)
        a, logp = m.policy(o)
        return a.view(B, n, -1), logp.view(B, n)

    def compute_loss(self, batch):
        c = self.config
        m = self.module
        losses, stats = super().compute_loss(batch)
        obs, act, nobs = batch["obs"], batch["actions"].float(), batch["next_obs"]
        B, N, T = obs.shape[0], int(c["num_actions"]), float(c["temperature"])
        na = act.shape[-1]
        # conservative term on both Q heads
        u = torch.rand(B, N, na, device=act.device) * 2 - 1
        rand_a = u * m.a_scale + m.a_bias
        rand_logd = -float(na) * math.log(2.0) - torch.log(m.a_scale).sum()  # uniform density on the box
        with torch.no_grad():
            cur_a, cur_logp = self._policy_actions(obs, N)
            nxt_a, nxt_logp = self._policy_actions(nobs, N)
        qr1, qr2 = self._repeat_q(obs, rand_a)
        qc1, qc2 = self._repeat_q(obs, cur_a)
        qn1, qn2 = self._repeat_q(obs, nxt_a)
        q1, q2 = m.qs(obs, act)
        gaps = []
        for qr, qc, qn, qd in ((qr1, qc1, qn1, q1), (qr2, qc2, qn2, q2)):
            cat = torch.cat([qr - rand_logd, qn - nxt_logp, qc - cur_logp], 1)
            gaps.append(T * torch.logsumexp(cat / T, 1).mean() - qd.mean())
        w = float(c["min_q_weight"])
        if c.get("lagrangian"):
            ap = self.log_alpha_prime.exp().clamp(0.0, 1e6)
            cql = sum(ap.detach() * w * (g - c["lagrangian_thresh"]) for g in gaps)
            losses["alpha_prime"] = -0.5 * sum(ap * w * (g.detach() - c["lagrangian_thresh"]) for g in gaps)
            stats["alpha_prime_value"] = ap.detach()
        else:
            cql = w * (gaps[0] + gaps[1])
        losses["qf"] = losses["qf"] + cql
        # behaviour-cloning warm start of the actor
        if self.n_updates < int(c["bc_iters"]):
            alpha = m.log_alpha.exp().detach()
            a_pi, logp = m.policy(obs)
            losses["policy"] = (alpha * logp - self._data_logp(obs, act)).mean()
            stats["policy_loss"] = losses["policy"].detach()
        stats["cql_loss"] = cql.detach()
        stats["cql_gap_q1"] = gaps[0].detach()
        return losses, stats

    def after_update(self):
        super().after_update()
        self.n_updates += 1


class CQL(SAC):
    config_class = CQLConfig
    learner_class = CQLLearner
    supports_multi_agent = False  # offline: one static dataset

    def setup_algo(self):
        # (s, a, r, s', terminated) rows, streamed from paths / a Dataset or sampled
        # from in-memory columns; recorded episodes carry s' as `new_obs`
        self.offline_data = self.algo_config.build_offline_data(
            columns=("obs", "actions", "rewards", "next_obs", "terminateds"))

    def training_step(self):
        c = self.algo_config
        stats = {}
        for _ in range(c.updates_per_iteration):
            raw = self.offline_data.sample(c.train_batch_size)
            b = {k: np.asarray(v).astype(np.float32) for k, v in raw.items()}
            if b["actions"].ndim == 1:
                b["actions"] = b["actions"][:, None]
            idx = b["rewards"]
            if self.learner_group.local is not None:
                stats, _td = self.learner_group.local.train_on(b)
            else:
                stats, _td = self.learner_group.call("train_on", b)
            self.env_steps_trained += len(idx)
        self._sync_weights()
        return stats
