"""Offline RL: MARWIL and BC (reference: rllib/algorithms/marwil/marwil.py,
marwil_learner.py, torch/marwil_torch_learner.py; rllib/algorithms/bc/bc.py).

Input is offline experience: a ``cluster_anywhere_amd.data`` Dataset, a list of
column dicts, or parquet path(s) with columns ``obs, actions, rewards,
terminateds`` (+ optional ``eps_id``). Discounted returns are computed per
episode when the data is loaded. MARWIL weights the log-likelihood by
``exp(beta * A / sqrt(moving_avg(A^2)))``; BC is MARWIL with ``beta = 0``."""
from __future__ import annotations

from typing import Any, Dict

import numpy as np
import torch

from ..core.learner import Learner
from .algorithm import Algorithm, AlgorithmConfig


class MARWILConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or MARWIL)
        self.beta = 1.0
        self.vf_coeff = 1.0
        self.moving_average_sqd_adv_norm_update_rate = 1e-8
        self.moving_average_sqd_adv_norm_start = 100.0
        self.lr = 1e-4
        self.train_batch_size = 2000
        self.input_ = None
        self.updates_per_iteration = 1

    def offline_data(self, *, input_=None, **_):
        self.input_ = input_
        return self


class MARWILLearner(Learner):
    def build(self):
        self.ma_sqd = self.config.get("moving_average_sqd_adv_norm_start", 100.0)

    def compute_loss(self, b):
        c = self.config
        out = self.module.forward_train(b)
        dist = self.module.dist_cls(out["action_dist_inputs"])
        logp = dist.logp(b["actions"])
        beta = c["beta"]
        if beta != 0.0:
            v = out["vf_preds"]
            adv = b["returns"] - v
            with torch.no_grad():
                rate = c["moving_average_sqd_adv_norm_update_rate"]
                self.ma_sqd = self.ma_sqd + rate * (float((adv.detach() ** 2).mean()) - self.ma_sqd)
                w = torch.exp(beta * adv.detach() / (1e-8 + self.ma_sqd ** 0.5)).clamp(max=20.0)
            pi_loss = -(w * logp).mean()
            vf_loss = 0.5 * (adv ** 2).mean()
            loss = pi_loss + c["vf_coeff"] * vf_loss
            return {"default": loss}, {"policy_loss": pi_loss.detach(), "vf_loss": vf_loss.detach(),
                                       "total_loss": loss.detach()}
        loss = -logp.mean()
        return {"default": loss}, {"policy_loss": loss.detach(), "total_loss": loss.detach()}


def _load_offline(inp) -> Dict[str, np.ndarray]:
    if inp is None:
        raise ValueError("config.offline_data(input_=...) is required for offline algorithms")
    if isinstance(inp, (str, list)) and (isinstance(inp, str) or (inp and isinstance(inp[0], str))):
        from ... import data

        inp = data.read_parquet(inp)
    if hasattr(inp, "iter_batches"):
        parts = list(inp.iter_batches(batch_size=None, batch_format="numpy"))
        cols = {k: np.concatenate([np.asarray(p[k]) for p in parts]) for k in parts[0]}
    elif isinstance(inp, dict):
        cols = {k: np.asarray(v) for k, v in inp.items()}
    else:
        cols = {k: np.concatenate([np.asarray(p[k]) for p in inp]) for k in inp[0]}
    if cols["obs"].dtype == object:
        cols["obs"] = np.stack(cols["obs"])
    return cols


def _discounted_returns(rew, term, gamma):
    out = np.zeros_like(rew, dtype=np.float32)
    acc = 0.0
    for i in range(len(rew) - 1, -1, -1):
        if term[i]:
            acc = 0.0
        acc = rew[i] + gamma * acc
        out[i] = acc
    return out


class MARWIL(Algorithm):
    config_class = MARWILConfig
    learner_class = MARWILLearner

    def setup_algo(self):
        c = self.algo_config
        cols = _load_offline(c.input_)
        if "returns" not in cols:
            cols["returns"] = _discounted_returns(cols["rewards"].astype(np.float32),
                                                  cols["terminateds"].astype(bool), c.gamma)
        self.data = {"obs": cols["obs"], "actions": cols["actions"], "returns": cols["returns"].astype(np.float32)}
        self.n = len(self.data["obs"])
        self.rng = np.random.default_rng(c.seed)

    def training_step(self):
        c = self.algo_config
        stats = {}
        for _ in range(c.updates_per_iteration):
            idx = self.rng.integers(0, self.n, size=min(c.train_batch_size, self.n))
            b = {k: v[idx] for k, v in self.data.items()}
            stats = self.learner_group.update(b)
            self.env_steps_trained += len(idx)
        self._sync_weights()
        return stats


class BCConfig(MARWILConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or BC)
        self.beta = 0.0


class BC(MARWIL):
    config_class = BCConfig
