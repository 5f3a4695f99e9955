"""Off-policy estimators (OPE): the value of a TARGET policy estimated from episodes
a BEHAVIOUR policy recorded (``config.offline_data(output=...)`` stores the
behaviour's ``action_prob``).

Reference: ``rllib/offline/estimators/`` (importance_sampling.py,
weighted_importance_sampling.py, direct_method.py, doubly_robust.py,
fqe_torch_model.py; Thomas & Brunskill 2016, Le et al. 2019). Per episode with
discount ``gamma``, behaviour probabilities ``mu_t = mu(a_t|s_t)`` and target
probabilities ``pi_t = pi(a_t|s_t)``, ``rho_t = prod_{t' <= t} pi_t' / mu_t'``:

* IS   ``V = sum_t gamma^t rho_t r_t``
* WIS  ``V = sum_t gamma^t rho_t / w_t r_t`` with ``w_t`` the mean of ``rho_t`` over
  the evaluated episodes that reach step ``t`` (a two-pass estimate)
* DM   ``V = V_Q(s_0) = sum_a pi(a|s_0) Q(s_0, a)`` with ``Q`` fitted by FQE
* DR   backward ``V_t = V_Q(s_t) + pi_t/mu_t (r_t + gamma V_{t+1} - Q(s_t, a_t))``

``estimate(episodes)`` returns ``v_behavior`` (the discounted return actually
observed), ``v_target``, their standard deviations over episodes, ``v_gain =
v_target / max(v_behavior, 1e-8)`` and ``v_delta = v_target - v_behavior``.
DM / DR need a discrete action space (as the reference's FQE model).
"""
from __future__ import annotations

import copy
from typing import Any, Dict, Iterable, List, Optional

import numpy as np
import torch
import torch.nn as nn


def target_action_probs(module, obs: np.ndarray, actions: np.ndarray) -> np.ndarray:
    """pi(a_t | s_t) of the target module for the logged actions."""
    with torch.no_grad():
        out = module.forward_train({"obs": torch.as_tensor(np.asarray(obs, np.float32))})
        d = module.dist_cls(out["action_dist_inputs"])
        lp = d.logp(torch.as_tensor(np.asarray(actions)))
    return lp.exp().double().numpy()


def target_policy_matrix(module, obs: np.ndarray) -> np.ndarray:
    """pi(. | s) for every discrete action, [T, A]."""
    with torch.no_grad():
        out = module.forward_train({"obs": torch.as_tensor(np.asarray(obs, np.float32))})
        return torch.softmax(out["action_dist_inputs"].double(), -1).numpy()


def _disc_return(r: np.ndarray, gamma: float) -> float:
    return float(np.sum(r * gamma ** np.arange(len(r))))


class OffPolicyEstimator:
    """Base: ``module`` is the target policy (an RLModule), ``gamma`` the discount."""

    requires_q_model = False

    def __init__(self, module, gamma: float = 0.99, **_):
        self.module = module
        self.gamma = float(gamma)

    # per-episode hooks ---------------------------------------------------------
    def peek_on_single_episode(self, ep: Dict[str, np.ndarray]) -> None:
        pass

    def estimate_on_single_episode(self, ep: Dict[str, np.ndarray]) -> Dict[str, float]:
        raise NotImplementedError

    def train(self, episodes: List[Dict[str, np.ndarray]]) -> Dict[str, Any]:
        return {}

    def _ratios(self, ep) -> np.ndarray:
        if "action_prob" not in ep or not np.all(np.isfinite(ep["action_prob"])):
            raise ValueError("off-policy estimation needs the behaviour policy's `action_prob` column "
                             "(recorded by config.offline_data(output=...))")
        pi = target_action_probs(self.module, ep["obs"], ep["actions"])
        return pi / np.maximum(np.asarray(ep["action_prob"], np.float64), 1e-12)

    def estimate(self, episodes: Iterable[Dict[str, np.ndarray]]) -> Dict[str, float]:
        eps = list(episodes)
        if not eps:
            raise ValueError("no episodes to estimate on")
        for ep in eps:
            self.peek_on_single_episode(ep)
        per = [self.estimate_on_single_episode(ep) for ep in eps]
        vb = np.array([p["v_behavior"] for p in per])
        vt = np.array([p["v_target"] for p in per])
        out = {"v_behavior": float(vb.mean()), "v_behavior_std": float(vb.std()),
               "v_target": float(vt.mean()), "v_target_std": float(vt.std()), "num_episodes": len(eps)}
        out["v_gain"] = out["v_target"] / max(out["v_behavior"], 1e-8)
        out["v_delta"] = out["v_target"] - out["v_behavior"]
        return out


class ImportanceSampling(OffPolicyEstimator):
    def estimate_on_single_episode(self, ep):
        r = np.asarray(ep["rewards"], np.float64)
        rho = np.cumprod(self._ratios(ep))
        disc = self.gamma ** np.arange(len(r))
        return {"v_behavior": float(np.sum(disc * r)), "v_target": float(np.sum(disc * rho * r))}


class WeightedImportanceSampling(OffPolicyEstimator):
    def __init__(self, module, gamma: float = 0.99, **kw):
        super().__init__(module, gamma, **kw)
        self._sum: List[float] = []
        self._cnt: List[float] = []
        self._rho: Dict[int, np.ndarray] = {}

    def peek_on_single_episode(self, ep):
        rho = np.cumprod(self._ratios(ep))
        self._rho[id(ep)] = rho
        for t, v in enumerate(rho):
            if t >= len(self._sum):
                self._sum.append(0.0)
                self._cnt.append(0.0)
            self._sum[t] += float(v)
            self._cnt[t] += 1.0

    def estimate_on_single_episode(self, ep):
        r = np.asarray(ep["rewards"], np.float64)
        rho = self._rho.pop(id(ep))
        w = np.array(self._sum[: len(r)]) / np.array(self._cnt[: len(r)])
        disc = self.gamma ** np.arange(len(r))
        return {"v_behavior": float(np.sum(disc * r)), "v_target": float(np.sum(disc * rho / np.maximum(w, 1e-12) * r))}

    def estimate(self, episodes):
        self._sum, self._cnt, self._rho = [], [], {}
        return super().estimate(episodes)


class FQETorchModel:
    """Fitted Q Evaluation of the target policy (discrete actions): ``Q(s, a)``
    regressed on ``r + gamma (1 - terminated) sum_a' pi(a'|s') Q_target(s', a')``,
    the target network refreshed every ``target_update_every`` updates
    (reference: ``rllib/offline/estimators/fqe_torch_model.py``)."""

    def __init__(self, module, obs_dim: int, num_actions: int, gamma: float = 0.99, *,
                 hiddens=(64, 64), lr: float = 1e-3, n_iters: int = 200, minibatch_size: int = 256,
                 target_update_every: int = 20, seed: int = 0, **_):
        torch.manual_seed(seed)
        layers, d = [], obs_dim
        for h in hiddens:
            layers += [nn.Linear(d, h), nn.ReLU()]
            d = h
        layers.append(nn.Linear(d, num_actions))
        self.q = nn.Sequential(*layers).double()
        self.q_target = copy.deepcopy(self.q)
        self.module = module
        self.gamma = gamma
        self.opt = torch.optim.Adam(self.q.parameters(), lr=lr)
        self.n_iters = n_iters
        self.mb = minibatch_size
        self.every = target_update_every
        self.rng = np.random.default_rng(seed)

    def train(self, episodes: List[Dict[str, np.ndarray]]) -> Dict[str, float]:
        cat = lambda k: np.concatenate([np.asarray(e[k]) for e in episodes])  # noqa: E731
        nxt = "new_obs" if "new_obs" in episodes[0] else "next_obs"
        obs = torch.as_tensor(cat("obs"), dtype=torch.float64)
        nobs = torch.as_tensor(cat(nxt), dtype=torch.float64)
        act = torch.as_tensor(cat("actions")).long()
        rew = torch.as_tensor(cat("rewards"), dtype=torch.float64)
        term = torch.as_tensor(cat("terminateds").astype(np.float64))
        pi_next = torch.as_tensor(target_policy_matrix(self.module, nobs.numpy()))
        n, losses = len(rew), []
        for it in range(self.n_iters):
            idx = torch.as_tensor(self.rng.integers(0, n, size=min(self.mb, n)))
            with torch.no_grad():
                v_next = (pi_next[idx] * self.q_target(nobs[idx])).sum(-1)
                y = rew[idx] + self.gamma * (1.0 - term[idx]) * v_next
            q = self.q(obs[idx]).gather(-1, act[idx].unsqueeze(-1)).squeeze(-1)
            loss = ((q - y) ** 2).mean()
            self.opt.zero_grad()
            loss.backward()
            self.opt.step()
            losses.append(float(loss.detach()))
            if (it + 1) % self.every == 0:
                self.q_target.load_state_dict(self.q.state_dict())
        return {"fqe_loss": float(np.mean(losses[-self.every:]))}

    @torch.no_grad()
    def estimate_q(self, obs, actions) -> np.ndarray:
        q = self.q(torch.as_tensor(np.asarray(obs), dtype=torch.float64))
        return q.gather(-1, torch.as_tensor(np.asarray(actions)).long().unsqueeze(-1)).squeeze(-1).numpy()

    @torch.no_grad()
    def estimate_v(self, obs) -> np.ndarray:
        q = self.q(torch.as_tensor(np.asarray(obs), dtype=torch.float64)).numpy()
        return (target_policy_matrix(self.module, obs) * q).sum(-1)


class _QModelEstimator(OffPolicyEstimator):
    requires_q_model = True

    def __init__(self, module, gamma: float = 0.99, q_model_config: Optional[Dict] = None, **kw):
        super().__init__(module, gamma, **kw)
        self.q_model_config = dict(q_model_config or {})
        self.model: Optional[FQETorchModel] = None

    def train(self, episodes):
        ep0 = episodes[0]
        obs_dim = int(np.prod(np.asarray(ep0["obs"]).shape[1:]))
        with torch.no_grad():
            out = self.module.forward_train({"obs": torch.as_tensor(np.asarray(ep0["obs"][:1], np.float32))})
        n_act = int(out["action_dist_inputs"].shape[-1])
        cfg = dict(self.q_model_config)
        cfg.pop("type", None)
        self.model = FQETorchModel(self.module, obs_dim, n_act, self.gamma, **cfg)
        return self.model.train(episodes)

    def estimate(self, episodes):
        eps = list(episodes)
        if self.model is None:
            self.train(eps)
        return super().estimate(eps)


class DirectMethod(_QModelEstimator):
    def estimate_on_single_episode(self, ep):
        r = np.asarray(ep["rewards"], np.float64)
        return {"v_behavior": _disc_return(r, self.gamma), "v_target": float(self.model.estimate_v(ep["obs"][:1])[0])}


class DoublyRobust(_QModelEstimator):
    def estimate_on_single_episode(self, ep):
        r = np.asarray(ep["rewards"], np.float64)
        w = self._ratios(ep)
        q = self.model.estimate_q(ep["obs"], ep["actions"])
        v = self.model.estimate_v(ep["obs"])
        vt = 0.0
        for t in range(len(r) - 1, -1, -1):
            vt = v[t] + w[t] * (r[t] + self.gamma * vt - q[t])
        return {"v_behavior": _disc_return(r, self.gamma), "v_target": float(vt)}


ESTIMATORS = {"is": ImportanceSampling, "wis": WeightedImportanceSampling, "dm": DirectMethod,
              "dr": DoublyRobust}


def make_estimator(spec, module, gamma: float):
    """``{"type": cls_or_name, ...kwargs}`` (the reference's
    ``off_policy_estimation_methods`` entry) -> an estimator instance."""
    spec = dict(spec or {})
    t = spec.pop("type", None)
    if isinstance(t, str):
        t = ESTIMATORS[t.lower()]
    if t is None:
        raise ValueError("off_policy_estimation_methods entries need a `type`")
    return t(module, gamma, **spec)
