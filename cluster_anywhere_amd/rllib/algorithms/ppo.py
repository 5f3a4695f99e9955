"""PPO (reference: rllib/algorithms/ppo/ppo.py, ppo_learner.py,
torch/ppo_torch_learner.py): clipped surrogate + clipped value loss + entropy
bonus + optional adaptive KL penalty. The train batch comes out of a learner
connector pipeline (``GeneralAdvantageEstimation``: GAE on the learner's device
with the ``rl_returns.hip`` kernel, one thread per column, reverse scan over T);
multi-agent PPO trains one learner per module on its own padded fragment."""
from __future__ import annotations

from typing import Any, Dict

import numpy as np
import torch

from ...ops.rl import gae
from ...ops.rl_encoder import ppo_loss_categorical
from ..core.learner import Learner, _to_tensor
from ..core.rl_module import Categorical
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


_SEQ_KEYS = ("actions", "action_logp", "action_dist_inputs", "advantages", "value_targets")


class PPOLearner(Learner):
    graph_capturable = True  # compute_loss has no host syncs / host-side state (KL coeff lives on device)

    def build(self):
        if self._stateful():  # sequence batches with padding masks: dynamic shapes, run eagerly
            self.graph_capturable = False
        self.kl_coeff = self.config.get("kl_coeff", 0.2)
        self._kl_dev = (torch.full((1,), float(self.kl_coeff), device=self.device)
                        if self.device.type == "cuda" else None)

    def _stateful(self) -> bool:
        return bool(getattr(self.module, "is_stateful", lambda: False)())

    def compute_loss(self, batch):
        c = self.config
        if self._stateful():  # sequences [S, L]: the module unrolls them; the loss sees flat steps
            st = {k[len("state_in_"):]: v for k, v in batch.items() if k.startswith("state_in_")}
            out = self.module.forward_train(dict(batch, state_in=st))
            batch = {k: (v.reshape((-1,) + tuple(v.shape[2:])) if k in _SEQ_KEYS else v) for k, v in batch.items()}
            if "loss_mask" in batch:  # multi-agent columns are padded to whole sequences
                keep = batch["loss_mask"].reshape(-1) > 0
                out = {k: v[keep] for k, v in out.items()}
                batch = {k: (v[keep] if k in _SEQ_KEYS else v) for k, v in batch.items()}
        else:
            out = self.module.forward_train(batch)
        if self.module.dist_cls is Categorical:
            # one fused kernel on GPU (ops/rl_encoder.py); the same math in torch on CPU
            use_kl = c.get("use_kl_loss", True)
            kl_coeff = self.kl_coeff if use_kl and self.kl_coeff > 0 else 0.0
            loss, st = ppo_loss_categorical(out["action_dist_inputs"], out["vf_preds"], batch["actions"],
                                            batch["action_logp"], batch["advantages"], batch["value_targets"],
                                            batch["action_dist_inputs"], c["clip_param"], c["vf_clip_param"],
                                            c["vf_loss_coeff"], c["entropy_coeff"], kl_coeff,
                                            self._kl_dev if use_kl else None)
            st = st / out["vf_preds"].shape[0]
            return {"default": loss}, {"total_loss": loss.detach(), "policy_loss": -st[0], "vf_loss": st[1],
                                       "entropy": st[2], "mean_kl_loss": st[3]}
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
        if self._kl_dev is not None:
            self._kl_dev.fill_(float(self.kl_coeff))
        return self.kl_coeff

    def build_learner_connector(self):
        """[user learner connectors..., NumpyToTensor, GeneralAdvantageEstimation, FlattenTimeMajor]."""
        from ..connectors import (ConnectorPipelineV2, FlattenTimeMajor, GeneralAdvantageEstimation, NumpyToTensor,
                                  build_pipeline)

        c = self.config
        user = c.get("learner_connector")
        p = build_pipeline(user, obs_space=self.obs_space, act_space=self.act_space) if user else ConnectorPipelineV2()
        p.append(NumpyToTensor(device=self.device))
        p.append(GeneralAdvantageEstimation(gamma=c["gamma"], lambda_=c.get("lambda_", 1.0)))
        if self._stateful():  # recurrent module: train on max_seq_len sequences
            from ..connectors import ChunkSequences

            p.append(ChunkSequences(max_seq_len=c.get("model_config", {}).get("max_seq_len", 20)))
        else:
            p.append(FlattenTimeMajor(keys=("obs", "actions", "action_logp", "action_dist_inputs", "advantages",
                                            "value_targets")))
        p.set_input_spaces(self.obs_space, self.act_space)
        return p

    @torch.no_grad()
    def postprocess(self, frag: Dict[str, Any]) -> Dict[str, Any]:
        """Run the learner connector pipeline (GAE on device) on one time-major
        fragment; returns the flattened train batch."""
        if getattr(self, "learner_connector", None) is None:
            self.learner_connector = self.build_learner_connector()
        return self.learner_connector(rl_module=self.module, batch=dict(frag), episodes=(), shared_data={})


class PPO(Algorithm):
    config_class = PPOConfig
    learner_class = PPOLearner
    supports_multi_agent = True
    supports_recurrent_multi_agent = True

    def training_step(self):
        import time

        from ..env.multi_agent_env_runner import concat_multi_agent

        c = self.algo_config
        t0 = time.perf_counter()
        frags = self.env_runner_group.sample()
        if self.is_multi_agent:
            frag = concat_multi_agent(frags)
            steps = sum(f["env_steps"] for f in frags)
            self.agent_steps_sampled += sum(f["agent_steps"] for f in frags)
        else:
            frag = concat_fragments(frags)
            steps = int(frag["rewards"].size)
        t1 = time.perf_counter()
        self.env_steps_sampled += steps
        lg = self.learner_group
        mbs = c.minibatch_size
        if c.model_config.get("use_lstm") or c.model_config.get("use_attention"):  # whole sequences
            mbs = max(1, mbs // int(c.model_config.get("max_seq_len", 20)))
        kl_of = (lambda st: {m: s.get("mean_kl_loss", 0.0) for m, s in st.items()}) if self.is_multi_agent \
            else (lambda st: st.get("mean_kl_loss", 0.0))
        if lg.local is not None:
            batch = lg.local.postprocess(frag)
            stats = lg.local.update(batch, mbs, c.num_epochs)
            kl = lg.local.update_kl(kl_of(stats))
        else:
            batch = _to_cpu(lg.call("postprocess", frag))
            stats = lg.update(batch, mbs, c.num_epochs)
            kl = lg.call("update_kl", kl_of(stats))
        if self.is_multi_agent:
            for m, k in kl.items():
                stats[m]["curr_kl_coeff"] = k
        else:
            stats["curr_kl_coeff"] = kl
        self.env_steps_trained += steps
        t2 = time.perf_counter()
        self._sync_weights()
        self._timers = {"sample_s": t1 - t0, "learn_s": t2 - t1, "sync_weights_s": time.perf_counter() - t2}
        return stats


def _to_cpu(b):
    if isinstance(b, dict):
        return {k: _to_cpu(v) for k, v in b.items()}
    return b.cpu() if isinstance(b, torch.Tensor) else b
