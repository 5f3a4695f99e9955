"""PPO (reference: rllib/algorithms/ppo/ppo.py, ppo_learner.py,
torch/ppo_torch_learner.py): clipped surrogate + clipped value loss + entropy
bonus + optional adaptive KL penalty; GAE on the learner's device with the
``rl_returns.hip`` kernel (one thread per env column, reverse scan over T)."""
from __future__ import annotations

from typing import Any, Dict

import numpy as np
import torch

from ...ops.rl import gae
from ..core.learner import Learner, _to_tensor
from .algorithm import Algorithm, AlgorithmConfig, concat_fragments


class PPOConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or PPO)
        self.lr = 5e-5
        self.lambda_ = 1.0
        self.use_gae = True
        self.use_critic = True
        self.clip_param = 0.3
        self.vf_clip_param = 10.0
        self.vf_loss_coeff = 1.0
        self.entropy_coeff = 0.0
        self.use_kl_loss = True
        self.kl_coeff = 0.2
        self.kl_target = 0.01
        self.num_epochs = 30
        self.minibatch_size = 128
        self.train_batch_size = 4000


class PPOLearner(Learner):
    def build(self):
        self.kl_coeff = self.config.get("kl_coeff", 0.2)

    def compute_loss(self, batch):
        c = self.config
        out = self.module.forward_train(batch)
        dist = self.module.dist_cls(out["action_dist_inputs"])
        logp = dist.logp(batch["actions"])
        ratio = torch.exp(logp - batch["action_logp"])
        adv = batch["advantages"]
        surr = torch.min(ratio * adv, ratio.clamp(1 - c["clip_param"], 1 + c["clip_param"]) * adv)
        v = out["vf_preds"]
        vf_loss = ((v - batch["value_targets"]) ** 2).clamp(max=c["vf_clip_param"])
        ent = dist.entropy()
        loss = -surr.mean() + c["vf_loss_coeff"] * vf_loss.mean() - c["entropy_coeff"] * ent.mean()
        old = self.module.dist_cls(batch["action_dist_inputs"])
        kl = old.kl(dist).mean()
        if c.get("use_kl_loss", True) and self.kl_coeff > 0:
            loss = loss + self.kl_coeff * kl
        self._last_kl = kl.detach()
        return {"default": loss}, {"total_loss": loss.detach(), "policy_loss": -surr.mean().detach(),
                                   "vf_loss": vf_loss.mean().detach(), "entropy": ent.mean().detach(),
                                   "mean_kl_loss": kl.detach()}

    def update_kl(self, kl: float):
        c = self.config
        if kl > 2.0 * c["kl_target"]:
            self.kl_coeff *= 1.5
        elif kl < 0.5 * c["kl_target"]:
            self.kl_coeff *= 0.5
        return self.kl_coeff

    @torch.no_grad()
    def postprocess(self, frag: Dict[str, Any]) -> Dict[str, Any]:
        """Bootstrap values + GAE on device; returns the flattened train batch."""
        c = self.config
        dev = self.device
        T, N = frag["rewards"].shape
        vf = _to_tensor(frag["vf_preds"], dev).float()
        last = self.module.compute_values({"obs": _to_tensor(frag["last_obs"], dev)}).float()
        values = torch.cat([vf, last[None]], 0)
        rew = _to_tensor(frag["rewards"], dev).float()
        nonterm = 1.0 - _to_tensor(frag["terminateds"], dev).float()
        adv, vt = gae(rew, values, nonterm, c["gamma"], c.get("lambda_", 1.0))
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        flat = lambda x: x.reshape((T * N,) + tuple(x.shape[2:]))
        return {"obs": flat(_to_tensor(frag["obs"], dev)), "actions": flat(_to_tensor(frag["actions"], dev)),
                "action_logp": flat(_to_tensor(frag["action_logp"], dev)),
                "action_dist_inputs": flat(_to_tensor(frag["action_dist_inputs"], dev)),
                "advantages": flat(adv), "value_targets": flat(vt)}


class PPO(Algorithm):
    config_class = PPOConfig
    learner_class = PPOLearner

    def training_step(self):
        import time

        c = self.algo_config
        t0 = time.perf_counter()
        frags = self.env_runner_group.sample()
        frag = concat_fragments(frags)
        t1 = time.perf_counter()
        steps = int(frag["rewards"].size)
        self.env_steps_sampled += steps
        lg = self.learner_group
        if lg.local is not None:
            batch = lg.local.postprocess(frag)
            stats = lg.local.update(batch, c.minibatch_size, c.num_epochs)
            stats["curr_kl_coeff"] = lg.local.update_kl(stats.get("mean_kl_loss", 0.0))
        else:
            batch = lg.call("postprocess", frag)
            batch = {k: v.cpu() for k, v in batch.items()}
            stats = lg.update(batch, c.minibatch_size, c.num_epochs)
            stats["curr_kl_coeff"] = lg.call("update_kl", stats.get("mean_kl_loss", 0.0))
        self.env_steps_trained += steps
        t2 = time.perf_counter()
        self._sync_weights()
        self._timers = {"sample_s": t1 - t0, "learn_s": t2 - t1, "sync_weights_s": time.perf_counter() - t2}
        return stats
