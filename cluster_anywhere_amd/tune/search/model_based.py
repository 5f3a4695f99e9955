"""Model-based searchers implemented natively (no optuna / hyperopt / bayes_opt in
the image). Same constructor surface as the reference wrappers so a user script
switches over unchanged:

* :class:`OptunaSearch`   (python/ray/tune/search/optuna/optuna_search.py:81) -
  Optuna's default sampler, the Tree-structured Parzen Estimator.
* :class:`HyperOptSearch` (python/ray/tune/search/hyperopt/hyperopt_search.py) -
  HyperOpt's ``tpe.suggest`` (TPE with ``gamma`` and ``n_initial_points``).
* :class:`BayesOptSearch` (python/ray/tune/search/bayesopt/bayesopt_search.py:41) -
  Gaussian-process regression (Matern 5/2, fitted noise) with the UCB / EI / POI
  utilities of ``bayes_opt``, maximised by random sampling + L-BFGS-B polishing.

The search space is every :class:`~.sample.Domain` leaf of the ``param_space``
(nested dicts included); constants ride along. Each numeric hyperparameter is
mapped to [0, 1] (log domains on the log scale), categoricals to their index.
``mode="min"`` is handled by negating the objective. Parity against the
reference libraries is unpinned (they are not importable here); the tests check
that each searcher finds a known optimum faster than random search.
"""
from __future__ import annotations

import math
import random
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from . import Searcher
from .sample import Categorical, Domain, Float, Function, Grid, Integer, _copy, _set, _walk


class _Codec:
    """Domain leaves of a (nested) space <-> points of [0, 1]^d (+ category ids)."""

    def __init__(self, space: Dict[str, Any]):
        self.space = space
        self.leaves: List[Tuple[tuple, Domain]] = [(p, d) for p, d in _walk(space)
                                                   if not isinstance(d, (Function, Grid))]
        if any(isinstance(d, Grid) for _, d in _walk(space)):
            raise ValueError("grid_search is not supported by model-based searchers")

    @property
    def dim(self):
        return len(self.leaves)

    def is_cat(self, i):
        return isinstance(self.leaves[i][1], Categorical)

    def ncat(self, i):
        return len(self.leaves[i][1].categories)

    @staticmethod
    def _get(cfg, path):
        for k in path:
            cfg = cfg[k]
        return cfg

    def encode(self, cfg) -> List[float]:
        out = []
        for p, d in self.leaves:
            v = self._get(cfg, p)
            if isinstance(d, Categorical):
                out.append(float(d.categories.index(v)))
            elif getattr(d, "normal", None) is not None:
                mu, sd = d.normal
                out.append(min(1.0, max(0.0, 0.5 + (v - mu) / (8 * sd))))
            elif d.log:
                lo, hi = math.log(d.lower), math.log(d.upper)
                out.append((math.log(v) - lo) / (hi - lo) if hi > lo else 0.5)
            else:
                out.append((v - d.lower) / (d.upper - d.lower) if d.upper > d.lower else 0.5)
        return out

    def decode(self, vec) -> Dict:
        cfg = _copy(self.space)
        for (p, d), x in zip(self.leaves, vec):
            if isinstance(d, Categorical):
                v = d.categories[int(min(max(round(x), 0), len(d.categories) - 1))]
            else:
                x = min(max(float(x), 0.0), 1.0)
                if getattr(d, "normal", None) is not None:
                    mu, sd = d.normal
                    v = mu + (x - 0.5) * 8 * sd
                elif d.log:
                    lo, hi = math.log(d.lower), math.log(d.upper)
                    v = math.exp(lo + x * (hi - lo))
                else:
                    v = d.lower + x * (d.upper - d.lower)
                if isinstance(d, Integer):
                    v = int(min(max(round(v), d.lower), d.upper - 1))
                if d.q:
                    v = round(v / d.q) * d.q
                    v = int(v) if isinstance(d, Integer) else float(v)
                elif isinstance(d, Float):
                    v = float(v)
            _set(cfg, p, v)
        for p, d in _walk(cfg):  # sample_from leaves see the resolved config
            if isinstance(d, Function):
                from .sample import _Spec

                _set(cfg, p, d.sample(_Spec(cfg)))
        return cfg

    def random(self, rng: random.Random) -> List[float]:
        return [float(rng.randrange(self.ncat(i))) if self.is_cat(i) else rng.random() for i in range(self.dim)]


class _ModelSearcher(Searcher):
    """Shared bookkeeping: space resolution, points_to_evaluate, sign of the
    objective, the trial budget, observed (encoded point, score) pairs."""

    def __init__(self, space=None, metric=None, mode=None, points_to_evaluate=None, seed=None,
                 evaluated_rewards=None):
        super().__init__(metric, mode)
        self._space = space
        self.points = [dict(p) for p in (points_to_evaluate or [])]
        self.rng = random.Random(seed)
        self.np_rng = np.random.default_rng(seed)
        self.codec: Optional[_Codec] = None
        self.live: Dict[str, List[float]] = {}
        self.X: List[List[float]] = []
        self.y: List[float] = []
        self.limit = None
        self.count = 0
        if evaluated_rewards is not None:
            if len(evaluated_rewards) != len(self.points):
                raise ValueError("evaluated_rewards must match points_to_evaluate")
            self._preseeded = list(zip(self.points, evaluated_rewards))
            self.points = []
        else:
            self._preseeded = []
        if space is not None:
            self._setup(space)

    def _setup(self, space):
        self.codec = _Codec(space)
        for cfg, r in self._preseeded:
            full = self._merge(cfg)
            self.add_evaluated_point(full, r)
        self._preseeded = []

    def _merge(self, partial):
        cfg = self.codec.decode(self.codec.random(self.rng))
        for p, _ in self.codec.leaves:
            try:
                v = partial
                for k in p:
                    v = v[k]
            except (KeyError, TypeError):
                continue
            _set(cfg, p, v)
        return cfg

    def set_search_properties(self, metric, mode, config, **spec):
        super().set_search_properties(metric, mode, config, **spec)
        self.limit = spec.get("num_samples")
        if self.codec is None:
            if not config:
                return False
            self._setup(config)
        return True

    def _sign(self):
        return 1.0 if (self.mode or "max") == "max" else -1.0

    def add_evaluated_point(self, parameters: Dict, value: float, error: bool = False, pruned: bool = False,
                            intermediate_values=None):
        if error or value is None:
            return
        self.X.append(self.codec.encode(parameters))
        self.y.append(self._sign() * float(value))

    def suggest(self, trial_id):
        if self.codec is None:
            return None
        if self.limit is not None and self.count >= self.limit:
            return Searcher.FINISHED
        self.count += 1
        if self.points:
            cfg = self._merge(self.points.pop(0))
        else:
            cfg = self.codec.decode(self._propose())
        self.live[trial_id] = self.codec.encode(cfg)
        return cfg

    def on_trial_complete(self, trial_id, result=None, error=False):
        x = self.live.pop(trial_id, None)
        if x is None or error or not result or self.metric not in result:
            return
        self.X.append(x)
        self.y.append(self._sign() * float(result[self.metric]))

    def _propose(self) -> List[float]:
        raise NotImplementedError

    def __getstate__(self):
        d = dict(self.__dict__)
        d["np_rng"] = None
        return d

    def __setstate__(self, d):
        self.__dict__.update(d)
        self.np_rng = np.random.default_rng(self.rng.randrange(1 << 30))


# ------------------------------------------------------------------------- TPE
class _TPE(_ModelSearcher):
    """Tree-structured Parzen Estimator (Bergstra et al. 2011), per-dimension
    (independent) like Optuna's / HyperOpt's defaults: the observations are split
    at the gamma quantile; l(x) is a Parzen mixture over the good points, g(x)
    over the rest (truncated Gaussians on [0, 1] with neighbour-distance
    bandwidths + a uniform prior component; categoricals by prior-smoothed
    frequencies); ``n_ei_candidates`` draws from l maximise l(x) / g(x)."""

    def __init__(self, *a, n_startup_trials=10, n_ei_candidates=24, gamma=None, prior_weight=1.0, **kw):
        super().__init__(*a, **kw)
        self.n_startup, self.n_cand = n_startup_trials, n_ei_candidates
        self.gamma_frac = gamma
        self.prior_w = prior_weight

    def _n_good(self, n):
        if self.gamma_frac is not None:  # HyperOpt: min(ceil(gamma * sqrt(n)), 25)
            return max(1, min(int(math.ceil(self.gamma_frac * math.sqrt(n))), 25))
        return max(1, min(int(math.ceil(0.1 * n)), 25))  # Optuna: min(ceil(0.1 n), 25)

    @staticmethod
    def _bandwidths(mus):
        order = np.argsort(mus)
        s = np.concatenate([[0.0], mus[order], [1.0]])
        gaps = np.maximum(s[1:-1] - s[:-2], s[2:] - s[1:-1])
        bw = np.empty_like(mus)
        bw[order] = gaps
        n = len(mus)
        lo = 1.0 / min(100.0, 1.0 + n)  # magic clip
        return np.clip(bw, lo, 1.0)

    def _num_logpdf(self, x, mus):
        """log of the prior-weighted truncated-Gaussian mixture at points x."""
        mus = np.asarray(mus, float)
        if len(mus) == 0:
            return np.zeros_like(x)
        sig = self._bandwidths(mus)
        from scipy.special import ndtr

        mu_all = np.concatenate([mus, [0.5]])
        sig_all = np.concatenate([sig, [1.0]])
        w = np.concatenate([np.ones(len(mus)), [self.prior_w]])
        w = w / w.sum()
        z = (x[:, None] - mu_all[None]) / sig_all[None]
        mass = ndtr((1.0 - mu_all) / sig_all) - ndtr((0.0 - mu_all) / sig_all)
        pdf = np.exp(-0.5 * z * z) / (sig_all[None] * math.sqrt(2 * math.pi) * np.maximum(mass[None], 1e-12))
        return np.log(np.maximum((pdf * w[None]).sum(1), 1e-300))

    def _num_sample(self, mus, n):
        mus = np.asarray(mus, float)
        sig = self._bandwidths(mus) if len(mus) else np.zeros(0)
        mu_all = np.concatenate([mus, [0.5]])
        sig_all = np.concatenate([sig, [1.0]])
        w = np.concatenate([np.ones(len(mus)), [self.prior_w]])
        w = w / w.sum()
        out = np.empty(n)
        comp = self.np_rng.choice(len(w), size=n, p=w)
        for i, c in enumerate(comp):
            for _ in range(100):  # rejection into [0, 1]
                v = self.np_rng.normal(mu_all[c], sig_all[c])
                if 0.0 <= v <= 1.0:
                    break
            out[i] = min(max(v, 0.0), 1.0)
        return out

    def _cat_probs(self, vals, k):
        cnt = np.full(k, self.prior_w / k)
        for v in vals:
            cnt[int(v)] += 1.0
        return cnt / cnt.sum()

    def _propose(self):
        n = len(self.y)
        if n < self.n_startup:
            return self.codec.random(self.rng)
        X = np.asarray(self.X, float)
        order = np.argsort(-np.asarray(self.y))  # best first (scores are maximised)
        ng = self._n_good(n)
        good, bad = X[order[:ng]], X[order[ng:]]
        out = []
        for i in range(self.codec.dim):
            if self.codec.is_cat(i):
                k = self.codec.ncat(i)
                pl, pg = self._cat_probs(good[:, i], k), self._cat_probs(bad[:, i], k)
                cand = self.np_rng.choice(k, size=self.n_cand, p=pl)
                score = np.log(pl[cand]) - np.log(pg[cand])
            else:
                cand = self._num_sample(good[:, i], self.n_cand)
                score = self._num_logpdf(cand, good[:, i]) - self._num_logpdf(cand, bad[:, i])
            out.append(float(cand[int(np.argmax(score))]))
        return out


class OptunaSearch(_TPE):
    """Optuna-compatible searcher: ``sampler`` may be None / "tpe" (TPE with
    Optuna's defaults: 10 startup trials, 24 EI candidates, gamma = min(ceil(0.1 n),
    25)) or "random"."""

    def __init__(self, space=None, metric=None, mode=None, points_to_evaluate=None, sampler=None, seed=None,
                 evaluated_rewards=None):
        if sampler not in (None, "tpe", "random"):
            raise ValueError("OptunaSearch: sampler must be None, 'tpe' or 'random' (no optuna in this image)")
        super().__init__(space, metric, mode, points_to_evaluate, seed, evaluated_rewards,
                         n_startup_trials=10 if sampler != "random" else 1 << 30)


class HyperOptSearch(_TPE):
    """HyperOpt-compatible searcher (``tpe.suggest``): ``n_initial_points`` random
    trials, then TPE with the good set the top ``gamma`` fraction."""

    def __init__(self, space=None, metric=None, mode=None, points_to_evaluate=None, n_initial_points=20,
                 random_state_seed=None, gamma=0.25):
        super().__init__(space, metric, mode, points_to_evaluate, random_state_seed, None,
                         n_startup_trials=n_initial_points, gamma=gamma)


# ---------------------------------------------------------------- GP / BayesOpt
class BayesOptSearch(_ModelSearcher):
    """Gaussian-process Bayesian optimisation (numeric hyperparameters only, as in
    the reference): Matern-5/2 kernel with per-dimension length scales and noise
    fitted by maximising the log marginal likelihood, the ``utility_kwargs``
    acquisition (``kind`` in ucb / ei / poi, ``kappa``, ``xi``) maximised over
    random samples and polished with L-BFGS-B."""

    def __init__(self, space=None, metric=None, mode=None, points_to_evaluate=None, utility_kwargs=None,
                 random_state=42, random_search_steps=10, verbose=0, patience=5, skip_duplicate=True,
                 analysis=None):
        self.util = dict(kind="ucb", kappa=2.576, xi=0.0)
        self.util.update(utility_kwargs or {})
        if self.util["kind"] not in ("ucb", "ei", "poi"):
            raise ValueError("utility kind must be ucb, ei or poi")
        self.random_steps = random_search_steps
        self.skip_duplicate = skip_duplicate
        super().__init__(space, metric, mode, points_to_evaluate, random_state)

    def _setup(self, space):
        super()._setup(space)
        if any(self.codec.is_cat(i) for i in range(self.codec.dim)):
            raise ValueError("BayesOptSearch supports numeric (Float / Integer) domains only")

    @staticmethod
    def _matern(A, B, ls):
        d = np.sqrt(np.maximum(((A[:, None, :] - B[None, :, :]) / ls) ** 2, 0).sum(-1))
        s5 = math.sqrt(5.0) * d
        return (1.0 + s5 + 5.0 / 3.0 * d * d) * np.exp(-s5)

    def _fit(self, X, y):
        from scipy.optimize import minimize

        dim = X.shape[1]
        ym, ys = y.mean(), y.std() or 1.0
        yn = (y - ym) / ys

        def nll(theta):
            ls, noise = np.exp(theta[:dim]), np.exp(theta[dim])
            K = self._matern(X, X, ls) + (noise + 1e-8) * np.eye(len(X))
            try:
                L = np.linalg.cholesky(K)
            except np.linalg.LinAlgError:
                return 1e10
            a = np.linalg.solve(L.T, np.linalg.solve(L, yn))
            return 0.5 * yn @ a + np.log(np.diag(L)).sum()

        best = None
        for start in ([math.log(0.3)] * dim + [math.log(1e-3)], [math.log(1.0)] * dim + [math.log(1e-2)]):
            r = minimize(nll, np.asarray(start), method="L-BFGS-B",
                         bounds=[(math.log(1e-2), math.log(10.0))] * dim + [(math.log(1e-6), math.log(1.0))])
            if best is None or r.fun < best.fun:
                best = r
        ls, noise = np.exp(best.x[:dim]), np.exp(best.x[dim])
        K = self._matern(X, X, ls) + (noise + 1e-8) * np.eye(len(X))
        L = np.linalg.cholesky(K)
        alpha = np.linalg.solve(L.T, np.linalg.solve(L, yn))
        return ls, L, alpha, ym, ys

    def _acq(self, Z, X, model, ybest):
        from scipy.stats import norm

        ls, L, alpha, ym, ys = model
        Ks = self._matern(Z, X, ls)
        mu = Ks @ alpha
        v = np.linalg.solve(L, Ks.T)
        sd = np.sqrt(np.maximum(1.0 - (v * v).sum(0), 1e-12))
        kind, kappa, xi = self.util["kind"], self.util["kappa"], self.util["xi"]
        yb = (ybest - ym) / ys
        if kind == "ucb":
            return mu + kappa * sd
        z = (mu - yb - xi) / sd
        if kind == "ei":
            return (mu - yb - xi) * norm.cdf(z) + sd * norm.pdf(z)
        return norm.cdf(z)

    def _propose(self):
        from scipy.optimize import minimize

        if len(self.y) < max(1, self.random_steps):
            return self.codec.random(self.rng)
        X, y = np.asarray(self.X, float), np.asarray(self.y, float)
        model = self._fit(X, y)
        dim = X.shape[1]
        Z = self.np_rng.random((4096, dim))
        a = self._acq(Z, X, model, y.max())
        seeds = Z[np.argsort(-a)[:5]]
        best_x, best_a = seeds[0], a.max()
        for s in seeds:
            r = minimize(lambda z: -self._acq(z[None], X, model, y.max())[0], s, method="L-BFGS-B",
                         bounds=[(0.0, 1.0)] * dim)
            if -r.fun > best_a:
                best_x, best_a = r.x, -r.fun
        if self.skip_duplicate and np.min(np.abs(X - best_x).max(1)) < 1e-6:
            return self.codec.random(self.rng)
        return [float(v) for v in best_x]


__all__ = ["OptunaSearch", "HyperOptSearch", "BayesOptSearch"]
