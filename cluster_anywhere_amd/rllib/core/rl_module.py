"""RLModules (reference: rllib/core/rl_module/rl_module.py,
rllib/core/models/catalog.py — default MLP / Nature-CNN encoders,
rllib/models/torch/torch_distributions.py).

``RLModule`` wraps a torch module with three forward modes:
  forward_inference  — greedy actions (evaluation / serving)
  forward_exploration— sampled actions + logp + value (EnvRunners)
  forward_train      — distribution inputs + values for the loss (Learner)
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..env import Box, Discrete, Space


# ---------------------------------------------------------- distributions
class Categorical:
    def __init__(self, logits):
        self.logits = logits - logits.logsumexp(-1, keepdim=True)

    def sample(self):
        return torch.multinomial(self.logits.exp(), 1).squeeze(-1)

    def deterministic(self):
        return self.logits.argmax(-1)

    def logp(self, a):
        return self.logits.gather(-1, a.long().unsqueeze(-1)).squeeze(-1)

    def entropy(self):
        return -(self.logits.exp() * self.logits).sum(-1)

    def kl(self, other: "Categorical"):
        p = self.logits.exp()
        return (p * (self.logits - other.logits)).sum(-1)


class DiagGaussian:
    def __init__(self, inputs):
        self.mean, log_std = inputs.chunk(2, dim=-1)
        self.log_std = log_std.clamp(-20, 2)
        self.std = self.log_std.exp()

    def sample(self):
        return self.mean + self.std * torch.randn_like(self.mean)

    def deterministic(self):
        return self.mean

    def logp(self, a):
        z = (a - self.mean) / self.std
        return (-0.5 * z * z - self.log_std - 0.5 * math.log(2 * math.pi)).sum(-1)

    def entropy(self):
        return (self.log_std + 0.5 * math.log(2 * math.pi * math.e)).sum(-1)

    def kl(self, other: "DiagGaussian"):
        return (other.log_std - self.log_std + (self.std ** 2 + (self.mean - other.mean) ** 2)
                / (2 * other.std ** 2) - 0.5).sum(-1)


def dist_class(action_space: Space):
    return Categorical if isinstance(action_space, Discrete) else DiagGaussian


def dist_input_dim(action_space: Space) -> int:
    if isinstance(action_space, Discrete):
        return action_space.n
    return 2 * int(np.prod(action_space.shape))


# --------------------------------------------------------------- encoders
def mlp(sizes: Sequence[int], act=nn.Tanh, out_act=False):
    layers = []
    for i in range(len(sizes) - 1):
        layers.append(nn.Linear(sizes[i], sizes[i + 1]))
        if i < len(sizes) - 2 or out_act:
            layers.append(act())
    return nn.Sequential(*layers)


class NatureCNN(nn.Module):
    """84x84xC uint8 NHWC -> 512 (Mnih et al. 2015). Parameters are kept in the
    layout of the MFMA kernels (``ops/rl_encoder.py``): conv weights
    ``[Cout, KH*KW*Cin]`` over NHWC windows, fc input flattened NHWC. On GPU the
    forward and backward run on those kernels; on CPU (env runners) the same
    parameters go through the fp32 PyTorch reference."""

    def __init__(self, in_ch: int = 4, out: int = 512, hw=(84, 84)):
        super().__init__()
        from ...ops.rl_encoder import NATURE_CONVS, nature_shapes

        shapes, flat = nature_shapes(hw[0], hw[1], in_ch)
        self.convs = nn.ParameterList()
        for (h, w, cin, cout, k, s, oh, ow) in shapes:
            wt = nn.Parameter(torch.empty(cout, k * k * cin))
            b = nn.Parameter(torch.empty(cout))
            _torch_default_init(wt, b)
            self.convs.append(wt)
            self.convs.append(b)
        self.fc_w = nn.Parameter(torch.empty(out, flat))
        self.fc_b = nn.Parameter(torch.empty(out))
        _torch_default_init(self.fc_w, self.fc_b)
        self.out_dim = out

    def params(self):
        return [*self.convs, self.fc_w, self.fc_b]

    def forward(self, x):
        from ...ops.rl_encoder import nature_cnn

        return nature_cnn(x, self.params())


def _torch_default_init(w: torch.Tensor, b: torch.Tensor):
    """nn.Linear / nn.Conv2d default init (kaiming-uniform(a=sqrt 5), fan_in = w.shape[1])."""
    with torch.no_grad():
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        bound = 1.0 / math.sqrt(w.shape[1])
        nn.init.uniform_(b, -bound, bound)


class TanhMLP(nn.Module):
    """The default vector-obs encoder (tanh MLP); on GPU via the MFMA kernels
    when every width is a multiple of 8, else plain torch."""

    def __init__(self, sizes: Sequence[int]):
        super().__init__()
        self.ws = nn.ParameterList()
        for i in range(len(sizes) - 1):
            w = nn.Parameter(torch.empty(sizes[i + 1], sizes[i]))
            b = nn.Parameter(torch.empty(sizes[i + 1]))
            _torch_default_init(w, b)
            self.ws.append(w)
            self.ws.append(b)
        from ...ops.rl_encoder import mlp_kernel_ok

        self.kernel_ok = mlp_kernel_ok(sizes[0], sizes[1:])

    def forward(self, x):
        from ...ops.rl_encoder import mlp_tanh, mlp_tanh_ref

        ps = list(self.ws)
        return mlp_tanh(x, ps) if self.kernel_ok else mlp_tanh_ref(x, ps)


def _act(name):
    return {"tanh": nn.Tanh, "relu": nn.ReLU, "silu": nn.SiLU, "elu": nn.ELU}[name]


class _GRUGate(nn.Module):
    """GTrXL gating layer: out = (1 - z) * x + z * tanh(W_g y + U_g (r * x))."""

    def __init__(self, d: int, bias_init: float = 2.0):
        super().__init__()
        self.w = nn.Linear(d, 3 * d, bias=False)
        self.u = nn.Linear(d, 2 * d, bias=False)
        self.ug = nn.Linear(d, d, bias=False)
        self.bz = nn.Parameter(torch.full((d,), float(bias_init)))

    def forward(self, x, y):
        wr, wz, wg = self.w(y).chunk(3, -1)
        ur, uz = self.u(x).chunk(2, -1)
        r = torch.sigmoid(wr + ur)
        z = torch.sigmoid(wz + uz - self.bz)
        h = torch.tanh(wg + self.ug(r * x))
        return (1 - z) * x + z * h


class GTrXLCore(nn.Module):
    """Gated transformer-XL core for partially observed tasks (reference: RLlib's
    attention net, ``use_attention`` / ``attention_dim`` / ``attention_num_heads`` /
    ``attention_num_transformer_units`` / ``attention_memory_inference`` /
    ``attention_init_gru_gate_bias``; Parisotto et al., "Stabilizing Transformers
    for RL"). Every unit keeps a memory of its last ``M`` inputs; one step attends
    from the current input over [memory, current] (pre-LayerNorm multi-head
    attention, then a position-wise MLP), each sub-layer joined by a GRU gate
    instead of a residual add. The recurrent state is the flat memory
    ``[units * M * dim]`` (zeros at episode start)."""

    def __init__(self, d_in: int, dim: int = 64, heads: int = 2, units: int = 1, memory: int = 16,
                 mlp_dim: int = 64, gate_bias: float = 2.0):
        super().__init__()
        self.dim, self.heads, self.units, self.M = dim, heads, units, memory
        self.inp = nn.Linear(d_in, dim)
        self.ln1 = nn.ModuleList([nn.LayerNorm(dim) for _ in range(units)])
        self.ln_kv = nn.ModuleList([nn.LayerNorm(dim) for _ in range(units)])
        self.q = nn.ModuleList([nn.Linear(dim, dim) for _ in range(units)])
        self.kv = nn.ModuleList([nn.Linear(dim, 2 * dim) for _ in range(units)])
        self.o = nn.ModuleList([nn.Linear(dim, dim) for _ in range(units)])
        self.g1 = nn.ModuleList([_GRUGate(dim, gate_bias) for _ in range(units)])
        self.ln2 = nn.ModuleList([nn.LayerNorm(dim) for _ in range(units)])
        self.mlp = nn.ModuleList([nn.Sequential(nn.Linear(dim, mlp_dim), nn.ReLU(), nn.Linear(mlp_dim, dim))
                                  for _ in range(units)])
        self.g2 = nn.ModuleList([_GRUGate(dim, gate_bias) for _ in range(units)])
        # learned position of each memory slot (oldest ... newest, current)
        self.pos = nn.Parameter(torch.zeros(memory + 1, dim))
        nn.init.normal_(self.pos, std=0.02)

    @property
    def state_size(self) -> int:
        return self.units * self.M * self.dim

    def step(self, z, mem_flat):
        """z [B, d_in], mem_flat [B, units*M*dim] -> (out [B, dim], new mem_flat)."""
        B = z.shape[0]
        mem = mem_flat.view(B, self.units, self.M, self.dim)
        x = self.inp(z)
        new = []
        H, hd = self.heads, self.dim // self.heads
        for u in range(self.units):
            new.append(torch.cat([mem[:, u, 1:], x[:, None]], 1))  # this unit's input joins its memory
            ctx = torch.cat([mem[:, u], x[:, None]], 1) + self.pos  # [B, M+1, dim]
            q = self.q[u](self.ln1[u](x)).view(B, H, 1, hd)
            k, v = self.kv[u](self.ln_kv[u](ctx)).chunk(2, -1)
            k = k.view(B, self.M + 1, H, hd).transpose(1, 2)
            v = v.view(B, self.M + 1, H, hd).transpose(1, 2)
            att = torch.softmax((q @ k.transpose(-1, -2)) / hd ** 0.5, -1) @ v  # [B, H, 1, hd]
            y = self.o[u](att.reshape(B, self.dim))
            x = self.g1[u](x, torch.relu(y))
            x = self.g2[u](x, torch.relu(self.mlp[u](self.ln2[u](x))))
        return x, torch.stack(new, 1).reshape(B, -1)


@dataclass
class RLModuleSpec:
    module_class: Optional[type] = None
    model_config: Dict = field(default_factory=dict)
    observation_space: Optional[Space] = None
    action_space: Optional[Space] = None
    inference_only: bool = False

    def build(self, observation_space: Optional[Space] = None, action_space: Optional[Space] = None) -> "RLModule":
        cls = self.module_class or DefaultActorCriticModule
        return cls(observation_space or self.observation_space, action_space or self.action_space,
                   dict(self.model_config or {}))


class RLModule(nn.Module):
    def __init__(self, observation_space: Space, action_space: Space, model_config: Optional[Dict] = None):
        super().__init__()
        self.observation_space, self.action_space = observation_space, action_space
        self.model_config = dict(model_config or {})
        self.setup()

    def setup(self):
        pass

    def forward_inference(self, batch: Dict) -> Dict:
        raise NotImplementedError

    def forward_exploration(self, batch: Dict) -> Dict:
        raise NotImplementedError

    def forward_train(self, batch: Dict) -> Dict:
        raise NotImplementedError

    def get_state(self):
        return {k: v.detach().cpu() for k, v in self.state_dict().items()}

    def set_state(self, state):
        self.load_state_dict(state)


class DefaultActorCriticModule(RLModule):
    """Encoder (MLP or Nature-CNN for image obs) + pi head + value head; the
    encoder is shared unless ``vf_share_layers`` is False.

    ``model_config["use_lstm"]`` adds a recurrent core (reference: the catalog's
    ``use_lstm`` / ``lstm_cell_size`` / ``max_seq_len``): encoder -> LSTM cell ->
    heads, with state ``{"h", "c"}``. Acting takes ``state_in`` ([B, cell]) and
    returns ``state_out``; training takes sequences ``obs [S, L, ...]`` with the
    state at each sequence start and ``resets [S, L]`` (1 where a new episode
    begins inside the sequence: the state is zeroed there)."""

    def setup(self):
        mc = self.model_config
        obs = self.observation_space
        hiddens = list(mc.get("fcnet_hiddens", [256, 256]))
        act = _act(mc.get("fcnet_activation", "tanh"))
        self.image = len(obs.shape) == 3
        self.use_lstm = bool(mc.get("use_lstm", False))
        self.use_attention = bool(mc.get("use_attention", False)) and not self.use_lstm
        self.share = mc.get("vf_share_layers", self.image or self.use_lstm or self.use_attention)
        if self.image:
            self.encoder = NatureCNN(obs.shape[-1], hw=obs.shape[:2])
            feat = self.encoder.out_dim
            self.vf_encoder = None
        else:
            d = int(np.prod(obs.shape))
            tanh = mc.get("fcnet_activation", "tanh") == "tanh"
            make = (lambda: TanhMLP([d] + hiddens)) if tanh else (lambda: mlp([d] + hiddens, act, out_act=True))
            self.encoder = make()
            feat = hiddens[-1]
            self.vf_encoder = None if self.share else make()
        if self.use_lstm:
            self.cell = int(mc.get("lstm_cell_size", 256))
            self.lstm = nn.LSTMCell(feat, self.cell)
            feat = self.cell
            self.vf_encoder = None  # value head shares the recurrent core
        elif self.use_attention:
            dim = int(mc.get("attention_dim", 64))
            self.gtrxl = GTrXLCore(feat, dim=dim, heads=int(mc.get("attention_num_heads", 2)),
                                   units=int(mc.get("attention_num_transformer_units", 1)),
                                   memory=int(mc.get("attention_memory_inference", mc.get("max_seq_len", 16))),
                                   mlp_dim=int(mc.get("attention_position_wise_mlp_dim", dim)),
                                   gate_bias=float(mc.get("attention_init_gru_gate_bias", 2.0)))
            feat = dim
            self.vf_encoder = None
        self.pi = nn.Linear(feat, dist_input_dim(self.action_space))
        self.vf = nn.Linear(feat, 1)
        nn.init.normal_(self.pi.weight, std=0.01)
        nn.init.zeros_(self.pi.bias)
        self.dist_cls = dist_class(self.action_space)
        if not isinstance(self.action_space, Discrete) and mc.get("free_log_std", True):
            # state-independent log std (as RLlib's free_log_std)
            self.log_std = nn.Parameter(torch.zeros(int(np.prod(self.action_space.shape))))
            with torch.no_grad():
                self.pi = nn.Linear(feat, int(np.prod(self.action_space.shape)))
                nn.init.normal_(self.pi.weight, std=0.01)
                nn.init.zeros_(self.pi.bias)
        else:
            self.log_std = None

    # ------------------------------------------------------------------ state
    def is_stateful(self) -> bool:
        return self.use_lstm or self.use_attention

    def get_initial_state(self) -> Dict[str, torch.Tensor]:
        if self.use_attention:
            return {"mem": torch.zeros(self.gtrxl.state_size)}
        if not self.use_lstm:
            return {}
        return {"h": torch.zeros(self.cell), "c": torch.zeros(self.cell)}

    def _state(self, batch, B, dev):
        st = batch.get("state_in")
        if st is None:
            z = torch.zeros(B, self.cell, device=dev)
            return z, z
        return st["h"].to(dev).float(), st["c"].to(dev).float()

    # ------------------------------------------------------------------ forward
    def _obs(self, batch):
        o = batch["obs"]
        return o if self.image else o.reshape(o.shape[0], -1).float()

    def _head_out(self, z):
        logits = self.pi(z)
        if self.log_std is not None:
            logits = torch.cat([logits, self.log_std.expand_as(logits)], -1)
        return logits

    def _heads(self, obs):
        z = self.encoder(obs)
        zv = z if self.vf_encoder is None else self.vf_encoder(obs)
        return self._head_out(z), self.vf(zv).squeeze(-1)

    def _step_lstm(self, batch):
        obs = self._obs(batch)
        z = self.encoder(obs)
        h, c = self._state(batch, obs.shape[0], z.device)
        h, c = self.lstm(z, (h, c))
        return h, c

    def _seq_lstm(self, batch):
        """obs [S, L, ...] -> core outputs [S*L, cell] (state zeroed at ``resets``)."""
        o = batch["obs"]
        S, L = o.shape[0], o.shape[1]
        flat = o.reshape((S * L,) + tuple(o.shape[2:]))
        z = self.encoder(flat if self.image else flat.reshape(S * L, -1).float()).view(S, L, -1)
        h, c = self._state(batch, S, z.device)
        resets = batch.get("resets")
        outs = []
        for t in range(L):
            if resets is not None and t > 0:
                keep = (1.0 - resets[:, t].float())[:, None]
                h, c = h * keep, c * keep
            h, c = self.lstm(z[:, t], (h, c))
            outs.append(h)
        return torch.stack(outs, 1).reshape(S * L, -1)

    def _step_attn(self, batch):
        obs = self._obs(batch)
        z = self.encoder(obs)
        st = batch.get("state_in")
        mem = (st["mem"].to(z.device).float() if st is not None
               else torch.zeros(z.shape[0], self.gtrxl.state_size, device=z.device))
        return self.gtrxl.step(z, mem)

    def _seq_attn(self, batch):
        """obs [S, L, ...] -> core outputs [S*L, dim]; memory zeroed at ``resets``."""
        o = batch["obs"]
        S, L = o.shape[0], o.shape[1]
        flat = o.reshape((S * L,) + tuple(o.shape[2:]))
        z = self.encoder(flat if self.image else flat.reshape(S * L, -1).float()).view(S, L, -1)
        st = batch.get("state_in")
        mem = (st["mem"].to(z.device).float() if st is not None
               else torch.zeros(S, self.gtrxl.state_size, device=z.device))
        resets = batch.get("resets")
        outs = []
        for t in range(L):
            if resets is not None and t > 0:
                mem = mem * (1.0 - resets[:, t].float())[:, None]
            y, mem = self.gtrxl.step(z[:, t], mem)
            outs.append(y)
        return torch.stack(outs, 1).reshape(S * L, -1)

    def forward_train(self, batch):
        if self.use_attention:
            core = self._seq_attn(batch)
            return {"action_dist_inputs": self._head_out(core), "vf_preds": self.vf(core).squeeze(-1)}
        if self.use_lstm:
            core = self._seq_lstm(batch)
            return {"action_dist_inputs": self._head_out(core), "vf_preds": self.vf(core).squeeze(-1)}
        logits, v = self._heads(self._obs(batch))
        return {"action_dist_inputs": logits, "vf_preds": v}

    @torch.no_grad()
    def forward_exploration(self, batch):
        if self.use_attention:
            y, mem = self._step_attn(batch)
            logits, v = self._head_out(y), self.vf(y).squeeze(-1)
        elif self.use_lstm:
            h, c = self._step_lstm(batch)
            logits, v = self._head_out(h), self.vf(h).squeeze(-1)
        else:
            logits, v = self._heads(self._obs(batch))
        d = self.dist_cls(logits)
        a = d.sample()
        out = {"actions": a, "action_logp": d.logp(a), "vf_preds": v, "action_dist_inputs": logits}
        if self.use_lstm:
            out["state_out"] = {"h": h, "c": c}
        elif self.use_attention:
            out["state_out"] = {"mem": mem}
        return out

    @torch.no_grad()
    def forward_inference(self, batch):
        if self.use_attention:
            y, mem = self._step_attn(batch)
            return {"actions": self.dist_cls(self._head_out(y)).deterministic(), "state_out": {"mem": mem}}
        if self.use_lstm:
            h, c = self._step_lstm(batch)
            return {"actions": self.dist_cls(self._head_out(h)).deterministic(), "state_out": {"h": h, "c": c}}
        logits, _ = self._heads(self._obs(batch))
        return {"actions": self.dist_cls(logits).deterministic()}

    def compute_values(self, batch):
        if self.use_attention:
            y, _ = self._step_attn(batch)
            return self.vf(y).squeeze(-1)
        if self.use_lstm:  # V of the state reached after ``state_in`` consumes ``obs``
            h, _ = self._step_lstm(batch)
            return self.vf(h).squeeze(-1)
        obs = self._obs(batch)
        z = self.encoder(obs) if self.vf_encoder is None else self.vf_encoder(obs)
        return self.vf(z).squeeze(-1)
