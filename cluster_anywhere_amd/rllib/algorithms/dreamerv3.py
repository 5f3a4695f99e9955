"""DreamerV3 (reference: rllib/algorithms/dreamerv3/ — dreamerv3.py,
dreamerv3_learner.py, tf/models/{world_model,actor_network,critic_network}.py;
Hafner et al. 2023). PyTorch, runs on the MI355X (or CPU) in the learner process.

World model (RSSM): MLP encoder of symlog(obs) -> posterior over ``num_latents``
categoricals of ``num_classes`` (1% unimix, straight-through samples); GRU
sequence model h_t = f(h_{t-1}, z_{t-1}, a_{t-1}); prior from h_t; heads:
symlog-MSE decoder, two-hot symlog reward (255 bins in [-20, 20]), Bernoulli
continue. KL balancing: 0.5 * max(1, KL[sg(post)||prior]) + 0.1 * max(1, KL[post||sg(prior)]).

Behaviour: actor and two-hot critic trained on ``horizon_H``-step imagined
rollouts from every posterior state; lambda-returns, return scale S = EMA of
(P95 - P5) (divided by max(1, S)), REINFORCE actor with entropy 3e-4, critic
regularised toward its EMA copy. Environment interaction keeps the recurrent
state per env; sequences of ``batch_length_T`` are drawn from a replay of
episodes with ``is_first`` resets.
"""
from __future__ import annotations

import math
import os
import time
from typing import Any, Dict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..env import Box, Discrete, make_env
from .algorithm import Algorithm, AlgorithmConfig

_SIZES = {  # model_size -> (dense units, mlp layers, gru units, latents, classes)
    "nano": (64, 1, 64, 4, 4), "micro": (128, 1, 128, 8, 8), "mini": (256, 2, 256, 16, 16),
    "XS": (256, 1, 256, 32, 32), "S": (512, 2, 512, 32, 32), "M": (640, 3, 1024, 32, 32),
    "L": (768, 4, 2048, 32, 32), "XL": (1024, 5, 4096, 32, 32),
}


def symlog(x):
    return torch.sign(x) * torch.log1p(x.abs())


def symexp(x):
    return torch.sign(x) * (torch.exp(x.abs()) - 1)


class TwoHot:
    def __init__(self, device, bins=255, lo=-20.0, hi=20.0):
        self.b = torch.linspace(lo, hi, bins, device=device)

    def encode(self, y):  # y: symlog target [...]
        y = y.clamp(self.b[0], self.b[-1])
        idx = torch.bucketize(y, self.b).clamp(1, len(self.b) - 1)
        lo, hi = self.b[idx - 1], self.b[idx]
        w_hi = (y - lo) / (hi - lo)
        out = torch.zeros(*y.shape, len(self.b), device=y.device)
        out.scatter_(-1, (idx - 1).unsqueeze(-1), (1 - w_hi).unsqueeze(-1))
        out.scatter_add_(-1, idx.unsqueeze(-1), w_hi.unsqueeze(-1))
        return out

    def mean(self, logits):  # -> value in real space
        return symexp((logits.softmax(-1) * self.b).sum(-1))

    def loss(self, logits, target):  # target in real space
        return -(self.encode(symlog(target)) * logits.log_softmax(-1)).sum(-1)


def _mlp(i, units, layers, out):
    mods, d = [], i
    for _ in range(layers):
        mods += [nn.Linear(d, units), nn.LayerNorm(units), nn.SiLU()]
        d = units
    mods.append(nn.Linear(d, out))
    return nn.Sequential(*mods)


class DreamerModel(nn.Module):
    def __init__(self, obs_dim, act_dim, discrete, size="nano"):
        super().__init__()
        units, layers, gru, nl, nc = _SIZES[size]
        self.nl, self.nc, self.gru_units = nl, nc, gru
        self.act_dim, self.discrete = act_dim, discrete
        z = nl * nc
        self.enc = _mlp(obs_dim, units, layers, units)
        self.post = _mlp(units + gru, units, 1, z)
        self.img_in = nn.Sequential(nn.Linear(z + act_dim, units), nn.LayerNorm(units), nn.SiLU())
        self.gru = nn.GRUCell(units, gru)
        self.prior = _mlp(gru, units, 1, z)
        feat = gru + z
        self.dec = _mlp(feat, units, layers, obs_dim)
        self.rew = _mlp(feat, units, layers, 255)
        self.cont = _mlp(feat, units, layers, 1)
        self.actor = _mlp(feat, units, layers, act_dim if discrete else 2 * act_dim)
        self.critic = _mlp(feat, units, layers, 255)
        for head in (self.rew[-1], self.critic[-1]):  # zero-init value heads (reference)
            nn.init.zeros_(head.weight)
            nn.init.zeros_(head.bias)

    # ---- latent helpers
    def _dist_logits(self, logits):
        p = logits.view(*logits.shape[:-1], self.nl, self.nc).softmax(-1)
        p = 0.99 * p + 0.01 / self.nc  # unimix
        return p.log()

    def _sample(self, logp):
        p = logp.exp()
        idx = torch.multinomial(p.reshape(-1, self.nc), 1).view(p.shape[:-1])
        onehot = F.one_hot(idx, self.nc).float()
        return (onehot + p - p.detach()).flatten(-2)  # straight-through

    def initial(self, b, device):
        return torch.zeros(b, self.gru_units, device=device), torch.zeros(b, self.nl * self.nc, device=device)

    def img_step(self, h, z, a):
        h = self.gru(self.img_in(torch.cat([z, a], -1)), h)
        return h, self._dist_logits(self.prior(h))

    def obs_step(self, h, z, a, emb, is_first, mode=False):
        keep = (1.0 - is_first).unsqueeze(-1)
        h, z, a = h * keep, z * keep, a * keep
        h, prior_lp = self.img_step(h, z, a)
        post_lp = self._dist_logits(self.post(torch.cat([emb, h], -1)))
        if mode:  # most likely latent (deterministic inference)
            z = F.one_hot(post_lp.argmax(-1), self.nc).float().flatten(-2)
            return h, z, post_lp, prior_lp
        return h, self._sample(post_lp), post_lp, prior_lp

    # ---- policy
    def act_dist(self, feat):
        out = self.actor(feat)
        if self.discrete:
            logits = out.log_softmax(-1)
            logits = torch.log(0.99 * logits.exp() + 0.01 / self.act_dim)
            return torch.distributions.Categorical(logits=logits)
        mean, std = out.chunk(2, -1)
        std = (2 - 0.1) * torch.sigmoid(std + 2.0) + 0.1
        return torch.distributions.Independent(torch.distributions.Normal(torch.tanh(mean), std), 1)


def _kl(lp_a, lp_b):  # categorical KL per latent, summed
    return (lp_a.exp() * (lp_a - lp_b)).sum(-1).sum(-1)


class DreamerV3Config(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or DreamerV3)
        self.model_size = "XS"
        self.batch_size_B = 16
        self.batch_length_T = 64
        self.horizon_H = 15
        self.gae_lambda = 0.95
        self.gamma = 0.997
        self.entropy_scale = 3e-4
        self.return_normalization_decay = 0.99
        self.world_model_lr = 1e-4
        self.actor_lr = 3e-5
        self.critic_lr = 3e-5
        self.world_model_grad_clip_by_global_norm = 1000.0
        self.actor_grad_clip_by_global_norm = 100.0
        self.critic_grad_clip_by_global_norm = 100.0
        self.training_ratio = 512
        self.num_envs = 1
        self.replay_capacity = 1_000_000
        self.symlog_obs = True
        self.use_float16 = False
        self.env_steps_per_iteration = 64

    def training(self, **kw):
        kw.pop("use_float16", None)
        return super().training(**kw)


class _Replay:
    """Per-step ring of (obs, action, reward, is_first, is_terminal) + sequence sampling."""

    def __init__(self, cap, obs_dim, act_dim, seed):
        self.cap, self.n, self.i = cap, 0, 0
        self.obs = np.zeros((cap, obs_dim), np.float32)
        self.act = np.zeros((cap, act_dim), np.float32)
        self.rew = np.zeros(cap, np.float32)
        self.first = np.zeros(cap, np.float32)
        self.term = np.zeros(cap, np.float32)
        self.rng = np.random.default_rng(seed)

    def add(self, o, a, r, first, term):
        j = self.i
        self.obs[j], self.act[j], self.rew[j], self.first[j], self.term[j] = o, a, r, first, term
        self.i = (j + 1) % self.cap
        self.n = min(self.n + 1, self.cap)

    def sample(self, B, T):
        start = self.rng.integers(0, max(1, self.n - T), size=B)
        idx = (start[:, None] + np.arange(T)[None]) % self.cap
        b = {"obs": self.obs[idx], "actions": self.act[idx], "rewards": self.rew[idx],
             "is_first": self.first[idx].copy(), "is_terminated": self.term[idx]}
        b["is_first"][:, 0] = 1.0
        return b


class DreamerV3(Algorithm):
    config_class = DreamerV3Config

    def setup(self, _config):
        c = self.algo_config
        if c.seed is not None:
            torch.manual_seed(c.seed)
            np.random.seed(c.seed)
        self.envs = [make_env(c.env, c.env_config) for _ in range(max(1, c.num_envs))]
        self.obs_space, self.act_space = self.envs[0].observation_space, self.envs[0].action_space
        self.discrete = isinstance(self.act_space, Discrete)
        self.obs_dim = int(np.prod(self.obs_space.shape))
        self.act_dim = int(self.act_space.n) if self.discrete else int(np.prod(self.act_space.shape))
        self.device = torch.device("cuda" if torch.cuda.is_available() and c.num_gpus_per_learner else "cpu")
        self.model = DreamerModel(self.obs_dim, self.act_dim, self.discrete, c.model_size).to(self.device)
        m = self.model
        wm = [*m.enc.parameters(), *m.post.parameters(), *m.img_in.parameters(), *m.gru.parameters(),
              *m.prior.parameters(), *m.dec.parameters(), *m.rew.parameters(), *m.cont.parameters()]
        self.wm_params = wm
        self.opt_wm = torch.optim.Adam(wm, lr=c.world_model_lr, eps=1e-8)
        self.opt_actor = torch.optim.Adam(m.actor.parameters(), lr=c.actor_lr, eps=1e-5)
        self.opt_critic = torch.optim.Adam(m.critic.parameters(), lr=c.critic_lr, eps=1e-5)
        import copy

        self.critic_ema = copy.deepcopy(m.critic)
        for p in self.critic_ema.parameters():
            p.requires_grad_(False)
        self.twohot = TwoHot(self.device)
        self.ret_scale = None
        self.replay = _Replay(min(c.replay_capacity, 1_000_000), self.obs_dim, self.act_dim, c.seed)
        self.env_steps_sampled = 0
        self.env_steps_trained = 0
        self._replayed = 0.0
        self._ep_ret = [0.0] * len(self.envs)
        self._returns = []
        self._obs = [e.reset(seed=(c.seed or 0) + i)[0] for i, e in enumerate(self.envs)]
        self._first = [1.0] * len(self.envs)
        self._h, self._z = m.initial(len(self.envs), self.device)
        self._a = torch.zeros(len(self.envs), self.act_dim, device=self.device)

    # ---------------------------------------------------------------- acting
    def _prep_obs(self, o):
        o = torch.as_tensor(np.asarray(o, np.float32).reshape(len(o), -1), device=self.device)
        return symlog(o) if self.algo_config.symlog_obs else o

    @torch.no_grad()
    def _policy_step(self, obs_list, first, explore=True):
        m = self.model
        emb = m.enc(self._prep_obs(obs_list))
        f = torch.tensor(first, device=self.device)
        self._h, self._z, _, _ = m.obs_step(self._h, self._z, self._a, emb, f)
        dist = m.act_dist(torch.cat([self._h, self._z], -1))
        if self.discrete:
            a = dist.sample() if explore else dist.probs.argmax(-1)
            self._a = F.one_hot(a, self.act_dim).float()
            return a.cpu().numpy(), self._a
        a = dist.sample() if explore else dist.mean
        a = a.clamp(-1, 1)
        self._a = a
        return a.cpu().numpy(), a

    def _env_action(self, a):
        if self.discrete:
            return int(a)
        lo, hi = self.act_space.low, self.act_space.high
        return (lo + (np.asarray(a) + 1) * 0.5 * (hi - lo)).astype(np.float32)

    def _collect(self, n_steps):
        for _ in range(n_steps):
            acts, a_vec = self._policy_step(self._obs, self._first)
            a_np = a_vec.cpu().numpy()
            for i, env in enumerate(self.envs):
                o2, r, te, tr, _ = env.step(self._env_action(acts[i]))
                self.replay.add(np.asarray(self._obs[i], np.float32).reshape(-1), a_np[i],
                                0.0 if self._first[i] else self._last_r[i], self._first[i], 0.0)
                self._ep_ret[i] += r
                self._last_r[i] = r
                self._first[i] = 0.0
                self._obs[i] = o2
                if te or tr:
                    # terminal observation row carries the final reward / termination flag
                    self.replay.add(np.asarray(o2, np.float32).reshape(-1), np.zeros(self.act_dim, np.float32),
                                    r, 0.0, float(te))
                    self._returns.append(self._ep_ret[i])
                    self._ep_ret[i] = 0.0
                    self._obs[i] = env.reset()[0]
                    self._first[i] = 1.0
            self.env_steps_sampled += len(self.envs)

    # -------------------------------------------------------------- learning
    def _train_batch(self, b):
        c, m, dev = self.algo_config, self.model, self.device
        t = {k: torch.as_tensor(v, device=dev) for k, v in b.items()}
        B, T = t["rewards"].shape
        obs = t["obs"].view(B, T, -1)
        sobs = symlog(obs) if c.symlog_obs else obs
        emb = m.enc(sobs)
        h, z = m.initial(B, dev)
        a_prev = torch.zeros(B, self.act_dim, device=dev)
        hs, zs, posts, priors = [], [], [], []
        for k in range(T):
            h, z, post_lp, prior_lp = m.obs_step(h, z, a_prev, emb[:, k], t["is_first"][:, k])
            hs.append(h)
            zs.append(z)
            posts.append(post_lp)
            priors.append(prior_lp)
            a_prev = t["actions"][:, k]
        H, Z = torch.stack(hs, 1), torch.stack(zs, 1)
        post, prior = torch.stack(posts, 1), torch.stack(priors, 1)
        feat = torch.cat([H, Z], -1)
        dec_loss = ((m.dec(feat) - sobs) ** 2).sum(-1)
        rew_loss = self.twohot.loss(m.rew(feat), t["rewards"])
        cont_loss = F.binary_cross_entropy_with_logits(m.cont(feat).squeeze(-1), 1.0 - t["is_terminated"],
                                                        reduction="none")
        dyn = _kl(post.detach(), prior).clamp(min=1.0)
        rep = _kl(post, prior.detach()).clamp(min=1.0)
        wm_loss = (dec_loss + rew_loss + cont_loss + 0.5 * dyn + 0.1 * rep).mean()
        self.opt_wm.zero_grad(set_to_none=True)
        wm_loss.backward()
        nn.utils.clip_grad_norm_(self.wm_params, c.world_model_grad_clip_by_global_norm)
        self.opt_wm.step()

        # ---- imagination from every posterior state
        Hs = c.horizon_H
        h = H.detach().reshape(B * T, -1)
        z = Z.detach().reshape(B * T, -1)
        feats, logps, ents = [torch.cat([h, z], -1)], [], []
        for _ in range(Hs):
            dist = m.act_dist(feats[-1].detach())
            a = dist.sample()
            logps.append(dist.log_prob(a))
            ents.append(dist.entropy())
            a_in = F.one_hot(a, self.act_dim).float() if self.discrete else a.clamp(-1, 1)
            with torch.no_grad():
                h, prior_lp = m.img_step(h, z, a_in)
                z = m._sample(prior_lp)
            feats.append(torch.cat([h, z], -1))
        F_ = torch.stack(feats, 0)  # [H+1, N, feat]
        with torch.no_grad():
            r = self.twohot.mean(m.rew(F_[1:]))
            cont = torch.sigmoid(m.cont(F_[1:]).squeeze(-1))
            disc = c.gamma * (cont > 0.5).float()
            v = self.twohot.mean(m.critic(F_))
            ret = [v[-1]]
            for k in range(Hs - 1, -1, -1):
                ret.append(r[k] + disc[k] * ((1 - c.gae_lambda) * v[k + 1] + c.gae_lambda * ret[-1]))
            R = torch.stack(ret[::-1][:-1], 0)  # [H, N]
            weight = torch.cumprod(torch.cat([torch.ones_like(disc[:1]), disc[:-1]], 0), 0)
            lo, hi = torch.quantile(R.flatten(), 0.05), torch.quantile(R.flatten(), 0.95)
            s = float(hi - lo)
            d = c.return_normalization_decay
            self.ret_scale = s if self.ret_scale is None else d * self.ret_scale + (1 - d) * s
            adv = (R - v[:-1]) / max(1.0, self.ret_scale)
        logp, ent = torch.stack(logps, 0), torch.stack(ents, 0)
        actor_loss = -(weight * (logp * adv + c.entropy_scale * ent)).mean()
        self.opt_actor.zero_grad(set_to_none=True)
        actor_loss.backward()
        nn.utils.clip_grad_norm_(m.actor.parameters(), c.actor_grad_clip_by_global_norm)
        self.opt_actor.step()
        cf = F_[:-1].detach()
        logits = m.critic(cf)
        with torch.no_grad():
            ema_t = self.twohot.mean(self.critic_ema(cf))
        critic_loss = (weight * (self.twohot.loss(logits, R) + self.twohot.loss(logits, ema_t))).mean()
        self.opt_critic.zero_grad(set_to_none=True)
        critic_loss.backward()
        nn.utils.clip_grad_norm_(m.critic.parameters(), c.critic_grad_clip_by_global_norm)
        self.opt_critic.step()
        with torch.no_grad():
            for pe, p in zip(self.critic_ema.parameters(), m.critic.parameters()):
                pe.mul_(0.98).add_(p, alpha=0.02)
        wm_loss, actor_loss, critic_loss = wm_loss.detach(), actor_loss.detach(), critic_loss.detach()
        dec_loss, rew_loss, dyn, ent = dec_loss.detach(), rew_loss.detach(), dyn.detach(), ent.detach()
        return {"WORLD_MODEL_L_total": float(wm_loss), "WORLD_MODEL_L_decoder": float(dec_loss.mean()),
                "WORLD_MODEL_L_reward": float(rew_loss.mean()), "WORLD_MODEL_L_dynamics": float(dyn.mean()),
                "ACTOR_L_total": float(actor_loss), "CRITIC_L_total": float(critic_loss),
                "ACTOR_entropy": float(ent.mean()), "return_scale": float(self.ret_scale)}

    def step(self) -> Dict[str, Any]:
        t0 = time.time()
        c = self.algo_config
        if not hasattr(self, "_last_r"):
            self._last_r = [0.0] * len(self.envs)
        self._collect(c.env_steps_per_iteration)
        stats = {}
        seq = c.batch_size_B * c.batch_length_T
        if self.replay.n >= c.batch_length_T + 1:
            # replayed steps / sampled steps == training_ratio
            self._replayed += c.env_steps_per_iteration * len(self.envs) * c.training_ratio
            while self._replayed >= seq:
                stats = self._train_batch(self.replay.sample(c.batch_size_B, c.batch_length_T))
                self._replayed -= seq
                self.env_steps_trained += seq
        rets = self._returns[-100:]
        m = {"episode_return_mean": float(np.mean(rets)) if rets else float("nan"),
             "num_episodes_lifetime": len(self._returns)}
        return {"env_runners": m, "learners": {"default_policy": stats},
                "num_env_steps_sampled_lifetime": self.env_steps_sampled,
                "num_env_steps_trained_lifetime": self.env_steps_trained,
                "episode_return_mean": m["episode_return_mean"], "timers": {"training_step_s": time.time() - t0}}

    # ------------------------------------------------------------ checkpoints
    def save_checkpoint(self, checkpoint_dir: str):
        torch.save({"model": self.model.state_dict(), "critic_ema": self.critic_ema.state_dict(),
                    "opt_wm": self.opt_wm.state_dict(), "opt_actor": self.opt_actor.state_dict(),
                    "opt_critic": self.opt_critic.state_dict(),
                    "ret_scale": -1.0 if self.ret_scale is None else float(self.ret_scale),
                    "steps": torch.tensor([self.env_steps_sampled, self.env_steps_trained])},
                   os.path.join(checkpoint_dir, "dreamer_state.pt"))

    def load_checkpoint(self, checkpoint):
        d = checkpoint if isinstance(checkpoint, str) else checkpoint.get("path")
        st = torch.load(os.path.join(d, "dreamer_state.pt"), weights_only=True, map_location=self.device)
        self.model.load_state_dict(st["model"])
        self.critic_ema.load_state_dict(st["critic_ema"])
        self.opt_wm.load_state_dict(st["opt_wm"])
        self.opt_actor.load_state_dict(st["opt_actor"])
        self.opt_critic.load_state_dict(st["opt_critic"])
        self.ret_scale = None if st["ret_scale"] < 0 else st["ret_scale"]
        self.env_steps_sampled, self.env_steps_trained = (int(x) for x in st["steps"])

    @torch.no_grad()
    def compute_single_action(self, obs, explore: bool = False, state=None):
        """Stateless convenience: a fresh recurrent state (is_first=1) per call."""
        m = self.model
        h, z = m.initial(1, self.device)
        a0 = torch.zeros(1, self.act_dim, device=self.device)
        emb = m.enc(self._prep_obs([obs]))
        h, z, _, _ = m.obs_step(h, z, a0, emb, torch.ones(1, device=self.device), mode=not explore)
        dist = m.act_dist(torch.cat([h, z], -1))
        if self.discrete:
            a = dist.sample() if explore else dist.probs.argmax(-1)
            return int(a[0])
        a = (dist.sample() if explore else dist.mean).clamp(-1, 1)[0].cpu().numpy()
        return self._env_action(a)

    def evaluate(self) -> Dict[str, Any]:
        return {}

    def get_module(self):
        return self.model

    def cleanup(self):
        pass
