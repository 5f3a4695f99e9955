"""Environments (gymnasium is not installed, so the env API, spaces, registry and
the classic-control / Atari-shaped envs used by RLlib's examples and tuned
benchmarks are built in; a gymnasium env is used when gymnasium is importable).

reference: rllib/env/ (env_context.py, vector_env.py, utils/), gymnasium
CartPole-v1 / Pendulum-v1 dynamics, rllib/env/wrappers/atari_wrappers.py
(84x84x4 uint8 frame stacks)."""
from __future__ import annotations

import math
from typing import Any, Callable, Dict, List, Optional, Tuple

import os

import numpy as np


# ----------------------------------------------------------------- spaces
class Space:
    shape: Tuple[int, ...] = ()
    dtype = np.float32

    def sample(self, rng: Optional[np.random.Generator] = None):
        raise NotImplementedError

    def contains(self, x) -> bool:
        raise NotImplementedError


class Discrete(Space):
    def __init__(self, n: int):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64

    def sample(self, rng=None):
        return int((rng or np.random.default_rng()).integers(self.n))

    def contains(self, x):
        return 0 <= int(x) < self.n

    def __repr__(self):
        return f"Discrete({self.n})"


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        shape = tuple(shape) if shape is not None else np.shape(low)
        self.low = np.broadcast_to(np.asarray(low, dtype=dtype), shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=dtype), shape).copy()
        self.shape = shape
        self.dtype = dtype

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        if np.issubdtype(self.dtype, np.integer):
            return rng.integers(lo, hi + 1, size=self.shape).astype(self.dtype)
        return rng.uniform(lo, hi, size=self.shape).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and np.all(x >= self.low) and np.all(x <= self.high)

    def __repr__(self):
        return f"Box({self.shape}, {np.dtype(self.dtype).name})"


# -------------------------------------------------------------------- envs
class Env:
    observation_space: Space
    action_space: Space
    spec_max_episode_steps: Optional[int] = None

    def reset(self, *, seed: Optional[int] = None, options=None):
        raise NotImplementedError

    def step(self, action):
        raise NotImplementedError

    def close(self):
        pass


class CartPoleEnv(Env):
    """Classic cart-pole (gymnasium CartPole-v1 dynamics: Euler integration,
    reward 1 per step, terminate at |x| > 2.4 or |theta| > 12 deg, truncate at 500)."""

    gravity, masscart, masspole, length, force_mag, tau = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02

    def __init__(self, config: Optional[Dict] = None):
        config = config or {}
        self.max_steps = config.get("max_episode_steps", 500)
        high = np.array([4.8, np.inf, 0.418, np.inf], dtype=np.float32)
        self.observation_space = Box(-high, high)
        self.action_space = Discrete(2)
        self.rng = np.random.default_rng()
        self.state = None
        self.t = 0

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.state = self.rng.uniform(-0.05, 0.05, size=4)
        self.t = 0
        return self.state.astype(np.float32), {}

    def step(self, action):
        x, xd, th, thd = self.state
        force = self.force_mag if int(action) == 1 else -self.force_mag
        ct, st = math.cos(th), math.sin(th)
        total = self.masspole + self.masscart
        pml = self.masspole * self.length
        temp = (force + pml * thd * thd * st) / total
        thacc = (self.gravity * st - ct * temp) / (self.length * (4.0 / 3.0 - self.masspole * ct * ct / total))
        xacc = temp - pml * thacc * ct / total
        x, xd = x + self.tau * xd, xd + self.tau * xacc
        th, thd = th + self.tau * thd, thd + self.tau * thacc
        self.state = np.array([x, xd, th, thd])
        self.t += 1
        terminated = bool(x < -2.4 or x > 2.4 or th < -0.2095 or th > 0.2095)
        truncated = self.t >= self.max_steps
        return self.state.astype(np.float32), 1.0, terminated, truncated, {}


class PendulumEnv(Env):
    """Inverted pendulum swing-up (gymnasium Pendulum-v1 dynamics, 200-step episodes)."""

    max_speed, max_torque, dt, g, m, l = 8.0, 2.0, 0.05, 10.0, 1.0, 1.0

    def __init__(self, config: Optional[Dict] = None):
        config = config or {}
        self.max_steps = config.get("max_episode_steps", 200)
        high = np.array([1.0, 1.0, self.max_speed], dtype=np.float32)
        self.observation_space = Box(-high, high)
        self.action_space = Box(-self.max_torque, self.max_torque, shape=(1,))
        self.rng = np.random.default_rng()

    def _obs(self):
        th, thd = self.state
        return np.array([math.cos(th), math.sin(th), thd], dtype=np.float32)

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.state = np.array([self.rng.uniform(-math.pi, math.pi), self.rng.uniform(-1, 1)])
        self.t = 0
        return self._obs(), {}

    def step(self, action):
        th, thd = self.state
        u = float(np.clip(np.asarray(action).reshape(-1)[0], -self.max_torque, self.max_torque))
        ang = ((th + math.pi) % (2 * math.pi)) - math.pi
        cost = ang ** 2 + 0.1 * thd ** 2 + 0.001 * u ** 2
        thd = thd + (3 * self.g / (2 * self.l) * math.sin(th) + 3.0 / (self.m * self.l ** 2) * u) * self.dt
        thd = float(np.clip(thd, -self.max_speed, self.max_speed))
        th = th + thd * self.dt
        self.state = np.array([th, thd])
        self.t += 1
        return self._obs(), -cost, False, self.t >= self.max_steps, {}


class FakeAtariEnv(Env):
    """Atari-shaped env for throughput benchmarks: 84x84x4 uint8 frame stacks,
    6 discrete actions, reward for matching a hidden target action that is
    encoded in the frame (so a conv policy can actually learn it)."""

    def __init__(self, config: Optional[Dict] = None):
        config = config or {}
        self.max_steps = config.get("max_episode_steps", 1000)
        self.observation_space = Box(0, 255, shape=(84, 84, 4), dtype=np.uint8)
        self.action_space = Discrete(6)
        self.rng = np.random.default_rng()
        self.frame = np.zeros((84, 84, 4), dtype=np.uint8)

    def _new_target(self):
        self.target = int(self.rng.integers(6))
        self.frame = np.roll(self.frame, -1, axis=2)
        f = self.rng.integers(0, 32, size=(84, 84), dtype=np.uint8)
        f[self.target * 14:(self.target + 1) * 14, :] = 200
        self.frame[..., -1] = f

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.t = 0
        self.frame[:] = 0
        self._new_target()
        return self.frame.copy(), {}

    def step(self, action):
        r = 1.0 if int(action) == self.target else 0.0
        self.t += 1
        self._new_target()
        return self.frame.copy(), r, False, self.t >= self.max_steps, {}


class FakeAtariVectorEnv:
    """``num_envs`` FakeAtari copies stepped as ONE batched numpy computation (the
    role of a natively vectorised env such as EnvPool / gymnasium's vector envs):
    the per-env Python step loop cost ~150 us per frame, about a third of a CPU env
    runner's time per step. Same dynamics, spaces and auto-reset contract as
    ``VectorEnv`` over ``FakeAtariEnv`` (per-env random streams differ)."""

    _POOL = 512

    def __init__(self, num_envs: int, config: Optional[Dict] = None, seed: Optional[int] = None):
        config = config or {}
        self.num_envs = num_envs
        self.max_steps = config.get("max_episode_steps", 1000)
        self.observation_space = Box(0, 255, shape=(84, 84, 4), dtype=np.uint8)
        self.action_space = Discrete(6)
        self.seed = seed
        self.rng = np.random.default_rng(seed)
        self.frames = np.zeros((num_envs, 84, 84, 4), dtype=np.uint8)
        self.target = np.zeros(num_envs, dtype=np.int64)
        self.t = np.zeros(num_envs, dtype=np.int64)
        self._rows = np.arange(84)[None, :]
        self._noise32 = self.rng.integers(0, 32, size=(self._POOL, 84, 84), dtype=np.uint32) << np.uint32(24)
        self._bufs = [np.empty((num_envs, 84, 84, 4), dtype=np.uint8) for _ in range(2)]
        self._flip = 0

    def _shift_in(self, frames, targets, out=None):
        """frames [n, 84, 84, 4] -> ``out`` (default: a new array): planes shifted by
        one, the last plane fresh background noise (one of ``_POOL`` pre-drawn planes
        per env and step) with the target band. A pixel's 4 channels are one
        little-endian uint32, so the plane shift is ``(px >> 8) | (new << 24)`` in
        place over 84 x 84 words, not a 4-byte-strided copy."""
        n = len(frames)
        new = self._noise32[self.rng.integers(self._POOL, size=n)]  # already << 24
        new[(self._rows // 14) == targets[:, None]] = np.uint32(200 << 24)  # rows of the target band
        if out is None:
            out = np.empty_like(frames)
        px = frames.view(np.uint32).reshape(n, 84, 84)
        o32 = out.view(np.uint32).reshape(n, 84, 84)
        np.right_shift(px, np.uint32(8), out=o32)
        np.bitwise_or(o32, new, out=o32)
        return out

    def reset(self):
        if self.seed is not None:
            self.rng = np.random.default_rng(self.seed)
        self.t[:] = 0
        self.target = self.rng.integers(6, size=self.num_envs)
        self.frames = self._shift_in(np.zeros((self.num_envs, 84, 84, 4), dtype=np.uint8), self.target)
        return self.frames

    def step(self, actions):
        """Observations alternate between two buffers: an array returned by step k
        stays valid until step k + 2 (callers copy what they keep)."""
        a = np.asarray(actions).reshape(-1).astype(np.int64)
        rew = (a == self.target).astype(np.float32)
        self.t += 1
        self.target = self.rng.integers(6, size=self.num_envs)
        self._flip ^= 1
        buf = self._bufs[self._flip]
        final = self.frames = self._shift_in(self.frames, self.target, out=buf)
        term = np.zeros(self.num_envs, dtype=bool)
        trunc = self.t >= self.max_steps
        if trunc.any():  # auto-reset (a fresh array: `final` keeps the last frames)
            idx = np.nonzero(trunc)[0]
            self.t[idx] = 0
            obs = self.frames.copy()
            obs[idx] = self._shift_in(np.zeros((len(idx), 84, 84, 4), dtype=np.uint8), self.target[idx])
            self.frames = obs
        return self.frames, rew, term, trunc, final


_NATIVE_VECTOR = {"FakeAtari-v0": FakeAtariVectorEnv}


class StatelessCartPoleEnv(CartPoleEnv):
    """CartPole without the velocity entries (x, theta only): partially observed, so
    a policy needs memory (reference: rllib/examples/envs/classes/stateless_cartpole.py)."""

    def __init__(self, config: Optional[Dict] = None):
        super().__init__(config)
        high = np.array([4.8, 0.418], dtype=np.float32)
        self.observation_space = Box(-high, high)

    def reset(self, *, seed=None, options=None):
        o, i = super().reset(seed=seed, options=options)
        return o[[0, 2]], i

    def step(self, action):
        o, r, te, tr, i = super().step(action)
        return o[[0, 2]], r, te, tr, i


class RepeatAfterMeEnv(Env):
    """Each step shows a random bit; the reward is +1 for playing the bit shown
    ``delay`` steps EARLIER (default 1), so only a policy with memory beats
    chance. Episodes are ``episode_len`` steps (default 20): chance ~= 0.5/step.
    (reference role: rllib/examples/envs/classes/repeat_after_me_env.py)"""

    def __init__(self, config: Optional[Dict] = None):
        config = config or {}
        self.delay = int(config.get("delay", 1))
        self.episode_len = int(config.get("episode_len", 20))
        self.observation_space = Box(0.0, 1.0, (2,))
        self.action_space = Discrete(2)
        self.rng = np.random.default_rng(config.get("seed"))
        self.hist: List[int] = []

    def _obs(self, b):
        o = np.zeros(2, np.float32)
        o[b] = 1.0
        return o

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        b = int(self.rng.integers(2))
        self.hist = [b]
        return self._obs(b), {}

    def step(self, action):
        want = self.hist[-1 - self.delay] if len(self.hist) > self.delay else None
        r = 1.0 if want is not None and int(action) == want else 0.0
        b = int(self.rng.integers(2))
        self.hist.append(b)
        done = len(self.hist) > self.episode_len
        return self._obs(b), r, False, done, {}


_REGISTRY: Dict[str, Callable[[Dict], Env]] = {
    "StatelessCartPole": lambda cfg: StatelessCartPoleEnv(cfg),
    "RepeatAfterMe-v0": lambda cfg: RepeatAfterMeEnv(cfg),
    "CartPole-v1": lambda cfg: CartPoleEnv(cfg),
    "CartPole-v0": lambda cfg: CartPoleEnv(dict({"max_episode_steps": 200}, **(cfg or {}))),
    "Pendulum-v1": lambda cfg: PendulumEnv(cfg),
    "FakeAtari-v0": lambda cfg: FakeAtariEnv(cfg),
    "ale_py:ALE/Pong-v5": lambda cfg: FakeAtariEnv(cfg),
}


def register_env(name: str, creator: Callable[[Dict], Env]):
    _REGISTRY[name] = creator


def make_env(env, config: Optional[Dict] = None) -> Env:
    config = config or {}
    if isinstance(env, str):
        if env in _REGISTRY:
            return _REGISTRY[env](config)
        try:  # optional gymnasium
            import gymnasium as gym

            return gym.make(env, **config)
        except ImportError:
            raise ValueError(f"unknown env {env!r} (registered: {sorted(_REGISTRY)})")
    if isinstance(env, type):
        return env(config)
    if callable(env):
        return env(config)
    raise TypeError(f"cannot build env from {env!r}")


class VectorEnv:
    """``num_envs`` copies stepped in lock-step with auto-reset (numpy batched).
    Envs with a native batched implementation (``_NATIVE_VECTOR``) get it instead of
    the per-env loop (``native=False`` keeps the loop)."""

    def __new__(cls, env=None, num_envs: int = 1, config: Optional[Dict] = None, seed: Optional[int] = None,
                native: bool = True):
        if native and cls is VectorEnv and isinstance(env, str) and env in _NATIVE_VECTOR \
                and os.environ.get("CAAMD_RLLIB_NATIVE_VECTOR_ENV", "1") == "1":
            return _NATIVE_VECTOR[env](num_envs, config, seed)
        return super().__new__(cls)

    def __init__(self, env, num_envs: int, config: Optional[Dict] = None, seed: Optional[int] = None,
                 native: bool = True):
        self.envs = [make_env(env, config) for _ in range(num_envs)]
        self.num_envs = num_envs
        self.observation_space = self.envs[0].observation_space
        self.action_space = self.envs[0].action_space
        self.seed = seed

    def reset(self):
        obs = []
        for i, e in enumerate(self.envs):
            o, _ = e.reset(seed=None if self.seed is None else self.seed + i)
            obs.append(o)
        return np.stack(obs)

    def step(self, actions):
        """Returns obs (after auto-reset), rewards, terminated, truncated, final_obs."""
        obs, rew, term, trunc, final = [], [], [], [], []
        for e, a in zip(self.envs, actions):
            o, r, te, tr, _ = e.step(a)
            final.append(o)
            if te or tr:
                o, _ = e.reset()
            obs.append(o)
            rew.append(r)
            term.append(te)
            trunc.append(tr)
        return (np.stack(obs), np.asarray(rew, np.float32), np.asarray(term), np.asarray(trunc), np.stack(final))


__all__ = ["Space", "Discrete", "Box", "Env", "CartPoleEnv", "StatelessCartPoleEnv", "RepeatAfterMeEnv",
           "PendulumEnv", "FakeAtariEnv", "FakeAtariVectorEnv", "register_env",
           "make_env", "VectorEnv"]
