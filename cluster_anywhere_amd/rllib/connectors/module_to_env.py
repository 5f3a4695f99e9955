"""module -> env connectors (reference role: rllib/connectors/module_to_env/:
normalize_and_clip_actions.py, get_actions.py).

They see the module's output dict for the B acting episodes (numpy arrays;
``batch["actions"]`` is what gets stored for training) and write
``batch["actions_for_env"]`` — what is sent to the env."""
from __future__ import annotations

import numpy as np

from ..env import Box
from .connector_v2 import ConnectorV2


class NormalizeAndClipActions(ConnectorV2):
    """For Box action spaces: ``normalize_actions`` maps the module's [-1, 1]
    actions onto [low, high]; ``clip_actions`` clips to [low, high]."""

    def __init__(self, input_observation_space=None, input_action_space=None, *, normalize_actions: bool = True,
                 clip_actions: bool = False, **kw):
        super().__init__(input_observation_space, input_action_space)
        self.normalize = normalize_actions
        self.clip = clip_actions

    def __call__(self, *, batch, **kw):
        sp = self.input_action_space
        a = batch.get("actions_for_env", batch["actions"])
        if isinstance(sp, Box):
            lo, hi = np.asarray(sp.low, np.float32), np.asarray(sp.high, np.float32)
            a = np.asarray(a, np.float32)
            if self.normalize:
                a = lo + (np.clip(a, -1.0, 1.0) + 1.0) * 0.5 * (hi - lo)
            elif self.clip:
                a = np.clip(a, lo, hi)
        batch["actions_for_env"] = a
        return batch


class GetActions(ConnectorV2):
    """Deterministic actions at inference time (``explore=False``) from the
    action-distribution inputs when the module did not emit actions."""

    def __call__(self, *, rl_module=None, batch, explore=None, **kw):
        if "actions" not in batch and "action_dist_inputs" in batch and rl_module is not None:
            import torch

            d = rl_module.dist_cls(torch.as_tensor(batch["action_dist_inputs"]))
            batch["actions"] = (d.sample() if explore else d.deterministic()).numpy()
        return batch


__all__ = ["NormalizeAndClipActions", "GetActions"]
