"""Learner connectors (reference role: rllib/connectors/learner/:
general_advantage_estimation.py, add_observations_from_episodes_to_batch.py).

The learner pipeline turns one time-major sample fragment (numpy ``[T, N, ...]``
from the env runners, plus ``last_obs`` ``[N, ...]`` and an optional validity
``mask`` ``[T, N]`` for padded multi-agent columns) into the flat train batch
of tensors on the learner's device. PPO's default pipeline is

    [user connectors..., NumpyToTensor, GeneralAdvantageEstimation, FlattenTimeMajor]

GAE runs on the learner's device with the ``rl_returns.hip`` kernel (one
thread per column, reverse scan over T) and advantages are standardised over
the valid steps only.
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import numpy as np
import torch

from ...ops.rl import gae
from .connector_v2 import ConnectorV2


def _to_tensor(x, device):
    if isinstance(x, torch.Tensor):
        return x.to(device, non_blocking=True)
    t = torch.from_numpy(np.ascontiguousarray(x))
    if device.type == "cuda":
        t = t.pin_memory().to(device, non_blocking=True)
    return t


class NumpyToTensor(ConnectorV2):
    def __init__(self, input_observation_space=None, input_action_space=None, *, device="cpu", **kw):
        super().__init__(input_observation_space, input_action_space)
        self.device = torch.device(device)

    def __call__(self, *, batch, **kw):
        return {k: (_to_tensor(v, self.device) if isinstance(v, (np.ndarray, torch.Tensor)) else v)
                for k, v in batch.items()}


class GeneralAdvantageEstimation(ConnectorV2):
    """Adds ``advantages`` and ``value_targets`` (time-major) from ``rewards``,
    ``vf_preds``, ``terminateds`` and the bootstrap value of ``last_obs``."""

    def __init__(self, input_observation_space=None, input_action_space=None, *, gamma: float = 0.99,
                 lambda_: float = 1.0, standardize: bool = True, **kw):
        super().__init__(input_observation_space, input_action_space)
        self.gamma, self.lambda_, self.standardize = gamma, lambda_, standardize

    @torch.no_grad()
    def __call__(self, *, rl_module=None, batch, **kw):
        vf = batch["vf_preds"].float()
        vb = {"obs": batch["last_obs"]}
        last_st = {k[len("last_state_"):]: v for k, v in batch.items() if k.startswith("last_state_")}
        if last_st:  # recurrent / attention module: V after the fragment's last state
            vb["state_in"] = last_st
        last = rl_module.compute_values(vb).float()
        values = torch.cat([vf, last[None]], 0)
        nonterm = 1.0 - batch["terminateds"].float()
        mask = batch.get("mask")
        if mask is not None:  # padded rows: zero reward / value and a terminal, so nothing leaks across columns
            values = torch.cat([vf * mask, last[None]], 0)
            nonterm = nonterm * mask
        adv, vt = gae(batch["rewards"].float(), values, nonterm, self.gamma, self.lambda_)
        if self.standardize:
            if mask is not None:
                m = mask.bool()
                sel = adv[m]
                mu, sd = sel.mean(), sel.std() if sel.numel() > 1 else torch.ones((), device=adv.device)
            else:
                mu, sd = adv.mean(), adv.std()
            adv = (adv - mu) / (sd + 1e-8)
        batch["advantages"] = adv
        batch["value_targets"] = vt
        return batch


class FlattenTimeMajor(ConnectorV2):
    """``[T, N, ...]`` -> ``[T*N, ...]`` for the per-step keys (only valid steps
    when a ``mask`` is present); fragment-level keys are dropped."""

    KEYS = ("obs", "actions", "action_logp", "action_dist_inputs", "advantages", "value_targets", "rewards",
            "terminateds", "vf_preds", "next_obs")

    def __init__(self, input_observation_space=None, input_action_space=None, *, keys=None, **kw):
        super().__init__(input_observation_space, input_action_space)
        self.keys = tuple(keys) if keys else None

    def __call__(self, *, batch, **kw):
        mask = batch.get("mask")
        keys = self.keys or [k for k in self.KEYS if k in batch]
        T, N = batch["rewards"].shape[:2]
        out = {}
        if mask is not None:
            idx = mask.reshape(-1).bool()
        for k in keys:
            v = batch[k]
            v = v.reshape((T * N,) + tuple(v.shape[2:]))
            out[k] = v[idx] if mask is not None else v
        return out


class ChunkSequences(ConnectorV2):
    """Recurrent modules: cut the time-major fragment ``[T, N, ...]`` into
    ``max_seq_len`` sequences ``[N*T/L, L, ...]`` (each env column cut along time),
    with the recurrent state at every sequence start (``state_in_*`` ``[S, cell]``)
    and ``resets [S, L]`` marking steps that begin a new episode inside a sequence."""

    KEYS = ("obs", "actions", "action_logp", "action_dist_inputs", "advantages", "value_targets")

    def __init__(self, input_observation_space=None, input_action_space=None, *, max_seq_len: int = 20, **kw):
        super().__init__(input_observation_space, input_action_space)
        self.L = int(max_seq_len)

    def _seq(self, v, T, N):
        L = self.L
        v = v.transpose(0, 1).contiguous()  # [N, T, ...]
        return v.reshape((N * (T // L), L) + tuple(v.shape[2:]))

    def __call__(self, *, batch, **kw):
        T, N = batch["rewards"].shape[:2]
        if T % self.L:
            raise ValueError(f"fragment length {T} is not a multiple of max_seq_len {self.L}")
        out = {k: self._seq(batch[k], T, N) for k in self.KEYS if k in batch}
        prev_term = torch.zeros_like(batch["terminateds"], dtype=torch.float32)
        prev_term[1:] = batch["terminateds"][:-1].float()
        out["resets"] = self._seq(prev_term, T, N)
        for k in [k for k in batch if k.startswith("state_in_")]:
            st = batch[k][:: self.L]  # [T/L, N, cell] state at each sequence start
            out[k] = st.transpose(0, 1).reshape(N * (T // self.L), -1).float()
        if "mask" in batch:  # padded multi-agent columns: the loss skips these steps
            out["loss_mask"] = self._seq(batch["mask"].float(), T, N)
        return out


__all__ = ["NumpyToTensor", "GeneralAdvantageEstimation", "FlattenTimeMajor", "ChunkSequences"]
