"""Old-stack ``Policy`` / ``TorchPolicy`` (reference role: rllib/policy/policy.py,
torch_policy_v2.py). The new stack here trains RLModules through Learners; these
classes keep code written against the old API working: a Policy maps observation
batches to actions and learns from :class:`SampleBatch` es.

* :class:`Policy`: the abstract interface (``compute_actions``,
  ``learn_on_batch``, weights / state, ``postprocess_trajectory``).
* :class:`TorchPolicy`: a concrete policy over the default actor-critic RLModule
  (or a given ``model``) with an Adam optimizer; subclasses override ``loss``
  (default: policy-gradient on ``advantages`` if present, else on discounted
  returns, plus a value loss).
* ``TFPolicy``: TensorFlow is not in the image.
"""
from __future__ import annotations

import os
import pickle
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from .sample_batch import SampleBatch


class Policy:
    def __init__(self, observation_space, action_space, config: Optional[Dict[str, Any]] = None):
        self.observation_space = observation_space
        self.action_space = action_space
        self.config = dict(config or {})
        self.global_timestep = 0

    # ------------------------------------------------------------------ acting
    def compute_actions(self, obs_batch, state_batches=None, prev_action_batch=None, prev_reward_batch=None,
                        info_batch=None, episodes=None, explore: Optional[bool] = None, timestep=None,
                        **kwargs) -> Tuple[Any, List[Any], Dict[str, Any]]:
        raise NotImplementedError

    def compute_single_action(self, obs=None, state=None, *, prev_action=None, prev_reward=None, info=None,
                              input_dict=None, episode=None, explore: Optional[bool] = None, timestep=None,
                              **kwargs):
        if input_dict is not None:
            obs = input_dict[SampleBatch.OBS]
        acts, state_out, extra = self.compute_actions(np.asarray(obs)[None], explore=explore, **kwargs)
        return acts[0], [s[0] for s in state_out], {k: v[0] for k, v in extra.items()}

    def compute_actions_from_input_dict(self, input_dict, explore: Optional[bool] = None, **kwargs):
        return self.compute_actions(input_dict[SampleBatch.OBS], explore=explore, **kwargs)

    def get_initial_state(self) -> List[Any]:
        return []

    def is_recurrent(self) -> bool:
        return False

    # ---------------------------------------------------------------- learning
    def postprocess_trajectory(self, sample_batch: SampleBatch, other_agent_batches=None, episode=None):
        return sample_batch

    def learn_on_batch(self, samples: SampleBatch) -> Dict[str, Any]:
        raise NotImplementedError

    def loss(self, model, dist_class, train_batch: SampleBatch):
        raise NotImplementedError

    # ----------------------------------------------------------------- state
    def get_weights(self) -> Dict[str, Any]:
        raise NotImplementedError

    def set_weights(self, weights: Dict[str, Any]) -> None:
        raise NotImplementedError

    def get_state(self) -> Dict[str, Any]:
        return {"weights": self.get_weights(), "global_timestep": self.global_timestep,
                "policy_spec": {"class": type(self), "observation_space": self.observation_space,
                                "action_space": self.action_space, "config": self.config}}

    def set_state(self, state: Dict[str, Any]) -> None:
        self.set_weights(state["weights"])
        self.global_timestep = state.get("global_timestep", 0)

    def export_checkpoint(self, export_dir: str) -> None:
        os.makedirs(export_dir, exist_ok=True)
        with open(os.path.join(export_dir, "policy_state.pkl"), "wb") as f:
            pickle.dump(self.get_state(), f)

    @staticmethod
    def from_checkpoint(checkpoint: str) -> "Policy":
        """Restore a policy this framework exported (``export_checkpoint``)."""
        with open(os.path.join(checkpoint, "policy_state.pkl"), "rb") as f:
            st = pickle.load(f)  # our own export, not a foreign file
        spec = st["policy_spec"]
        p = spec["class"](spec["observation_space"], spec["action_space"], spec["config"])
        p.set_state(st)
        return p

    def on_global_var_update(self, global_vars: Dict[str, Any]) -> None:
        self.global_timestep = global_vars.get("timestep", self.global_timestep)


class TorchPolicy(Policy):
    """A trainable policy over an RLModule (default: the actor-critic module of
    ``config["model"]``) with Adam (``config["lr"]``)."""

    def __init__(self, observation_space, action_space, config: Optional[Dict[str, Any]] = None, model=None):
        super().__init__(observation_space, action_space, config)
        from ..core.rl_module import DefaultActorCriticModule, dist_class

        self.model = model or DefaultActorCriticModule(observation_space, action_space,
                                                      dict(self.config.get("model", {})))
        self.dist_class = dist_class(action_space)
        self.device = torch.device(self.config.get("device", "cpu"))
        self.model.to(self.device)
        self.optimizer = torch.optim.Adam(self.model.parameters(), lr=float(self.config.get("lr", 3e-4)))
        self.gamma = float(self.config.get("gamma", 0.99))
        self.vf_coeff = float(self.config.get("vf_loss_coeff", 0.5))

    @torch.no_grad()
    def compute_actions(self, obs_batch, state_batches=None, prev_action_batch=None, prev_reward_batch=None,
                        info_batch=None, episodes=None, explore: Optional[bool] = None, timestep=None, **kwargs):
        explore = self.config.get("explore", True) if explore is None else explore
        obs = torch.as_tensor(np.asarray(obs_batch, dtype=np.float32), device=self.device)
        out = (self.model.forward_exploration if explore else self.model.forward_inference)({"obs": obs})
        if "actions" in out:
            acts = out["actions"]
        else:
            d = self.dist_class(out["action_dist_inputs"])
            acts = d.sample() if explore else d.deterministic()
        extra = {k: v.cpu().numpy() for k, v in out.items() if k in ("action_logp", "vf_preds",
                                                                       "action_dist_inputs")}
        self.global_timestep += len(obs)
        return acts.cpu().numpy(), [], extra

    def postprocess_trajectory(self, sample_batch: SampleBatch, other_agent_batches=None, episode=None):
        """Discounted returns (``value_targets``) and advantages (returns - V)."""
        if SampleBatch.REWARDS not in sample_batch or SampleBatch.ADVANTAGES in sample_batch:
            return sample_batch
        rew = np.asarray(sample_batch[SampleBatch.REWARDS], np.float32)
        done = np.zeros(len(rew), bool)
        for k in (SampleBatch.TERMINATEDS, SampleBatch.TRUNCATEDS):
            if k in sample_batch:
                done |= np.asarray(sample_batch[k]).astype(bool)
        ret, acc = np.zeros_like(rew), 0.0
        for i in range(len(rew) - 1, -1, -1):
            acc = rew[i] + self.gamma * (0.0 if done[i] else acc)
            ret[i] = acc
        sample_batch[SampleBatch.VALUE_TARGETS] = ret
        vf = np.asarray(sample_batch.get(SampleBatch.VF_PREDS, np.zeros_like(ret)), np.float32)
        sample_batch[SampleBatch.ADVANTAGES] = ret - vf
        return sample_batch

    def loss(self, model, dist_class, train_batch: Dict[str, torch.Tensor]):
        out = model.forward_train({"obs": train_batch[SampleBatch.OBS]})
        logp = dist_class(out["action_dist_inputs"]).logp(train_batch[SampleBatch.ACTIONS])
        adv = train_batch[SampleBatch.ADVANTAGES]
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        pg = -(logp * adv).mean()
        vf = ((out["vf_preds"] - train_batch[SampleBatch.VALUE_TARGETS]) ** 2).mean()
        return pg + self.vf_coeff * vf

    def learn_on_batch(self, samples: SampleBatch) -> Dict[str, Any]:
        samples = self.postprocess_trajectory(samples)
        batch = {}
        for k in (SampleBatch.OBS, SampleBatch.ACTIONS, SampleBatch.ADVANTAGES, SampleBatch.VALUE_TARGETS):
            v = np.asarray(samples[k])
            batch[k] = torch.as_tensor(v, device=self.device,
                                       dtype=torch.long if (k == SampleBatch.ACTIONS and v.dtype.kind in "iu")
                                       else torch.float32)
        loss = self.loss(self.model, self.dist_class, batch)
        self.optimizer.zero_grad()
        loss.backward()
        gc = self.config.get("grad_clip")
        if gc:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), gc)
        self.optimizer.step()
        return {"learner_stats": {"total_loss": float(loss.detach())}, "num_agent_steps_trained": len(samples)}

    def get_weights(self) -> Dict[str, Any]:
        return {k: v.detach().cpu().numpy() for k, v in self.model.state_dict().items()}

    def set_weights(self, weights: Dict[str, Any]) -> None:
        self.model.load_state_dict({k: torch.as_tensor(v) for k, v in weights.items()})


class TFPolicy(Policy):
    def __init__(self, *args, **kwargs):
        raise ImportError("TFPolicy needs TensorFlow, which is not installed in this image; use TorchPolicy")


TorchPolicyV2 = TorchPolicy
