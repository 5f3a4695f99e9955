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
        self.updates_per_iteration = 1


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
    """All of a small offline input as one column dict (used by tools; training
    samples through :class:`~cluster_anywhere_amd.rllib.offline.OfflineData`)."""
    from ..offline import OfflineData

    od = OfflineData(inp)
    if od.memory is not None:
        return od.memory
    parts = [od.prelearner_class(od.gamma, None)(b) for b in od.dataset.iter_batches(batch_size=None,
                                                                                       batch_format="numpy")]
    return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}


class MARWIL(Algorithm):
    config_class = MARWILConfig
    learner_class = MARWILLearner

    def setup_algo(self):
        # streamed (paths / Dataset) or in-memory (column dicts) offline input; the
        # pre-learner adds per-episode discounted returns
        self.offline_data = self.algo_config.build_offline_data(columns=("obs", "actions", "returns"))

    def training_step(self):
        c = self.algo_config
        stats = {}
        for _ in range(c.updates_per_iteration):
            b = self.offline_data.sample(c.train_batch_size)
            b["returns"] = b["returns"].astype(np.float32, copy=False)
            stats = self.learner_group.update(b)
            self.env_steps_trained += len(b["returns"])
        self._sync_weights()
        return stats


class BCConfig(MARWILConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or BC)
        self.beta = 0.0


class BC(MARWIL):
    config_class = BCConfig
