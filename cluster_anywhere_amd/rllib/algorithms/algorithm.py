"""Algorithm / AlgorithmConfig (reference: rllib/algorithms/algorithm.py,
algorithm_config.py — builder methods ``environment``, ``env_runners``,
``learners``, ``training``, ``rl_module``, ``evaluation``, ``debugging``,
``reporting``, ``resources``, ``framework``, ``api_stack``).

``Algorithm`` is a Tune ``Trainable``: ``train()`` runs one
``training_step()`` and returns RLlib-style nested metrics
(``env_runners/episode_return_mean``, ``learners/...``,
``num_env_steps_sampled_lifetime``); ``save``/``restore`` checkpoint the
learner (module + optimizer) state and the config."""
from __future__ import annotations

import copy
import json
import os
import pickle
import time
from typing import Any, Callable, Dict, Optional

import numpy as np
import torch

from ...tune.trainable import Trainable
from ..core.learner import Learner, LearnerGroup
from ..core.rl_module import DefaultActorCriticModule
from ..env import make_env
from ..env.env_runner import EnvRunnerGroup


class _NotProvided:
    pass


NotProvided = _NotProvided()


class AlgorithmConfig:
    algo_class = None

    def __init__(self, algo_class=None):
        self.algo_class = algo_class or type(self).algo_class
        # environment
        self.env = None
        self.env_config: Dict = {}
        # env runners
        self.num_env_runners = 0
        self.num_envs_per_env_runner = 1
        self.rollout_fragment_length: Any = "auto"
        self.num_cpus_per_env_runner = 1
        # learners
        self.num_learners = 0
        self.num_gpus_per_learner = 1
        self.num_cpus_per_learner = 1
        # training
        self.gamma = 0.99
        self.lr = 5e-5
        self.train_batch_size = 4000
        self.train_batch_size_per_learner = None
        self.minibatch_size = 128
        self.num_epochs = 1
        self.grad_clip = None
        self.model_config: Dict = {}
        self.rl_module_class = None
        # misc
        self.seed = None
        self.evaluation_interval = None
        self.evaluation_duration = 10
        self.metrics_num_episodes_for_smoothing = 100
        self.framework_str = "torch"

    # ------------------------------------------------------------ builders
    def _set(self, **kw):
        for k, v in kw.items():
            if v is NotProvided:
                continue
            if not hasattr(self, k) and k not in ("lambda_",):
                raise AttributeError(f"{type(self).__name__} has no setting {k!r}")
            setattr(self, "lambda_" if k == "lambda_" else k, v)
        return self

    def environment(self, env=NotProvided, *, env_config=NotProvided, **_):
        return self._set(env=env, env_config=env_config)

    def env_runners(self, *, num_env_runners=NotProvided, num_envs_per_env_runner=NotProvided,
                    rollout_fragment_length=NotProvided, num_cpus_per_env_runner=NotProvided, **_):
        return self._set(num_env_runners=num_env_runners, num_envs_per_env_runner=num_envs_per_env_runner,
                         rollout_fragment_length=rollout_fragment_length,
                         num_cpus_per_env_runner=num_cpus_per_env_runner)

    rollouts = env_runners

    def learners(self, *, num_learners=NotProvided, num_gpus_per_learner=NotProvided,
                 num_cpus_per_learner=NotProvided, **_):
        return self._set(num_learners=num_learners, num_gpus_per_learner=num_gpus_per_learner,
                         num_cpus_per_learner=num_cpus_per_learner)

    def training(self, **kw):
        if "model" in kw:
            self.model_config.update(kw.pop("model") or {})
        if "num_sgd_iter" in kw:
            kw["num_epochs"] = kw.pop("num_sgd_iter")
        if "sgd_minibatch_size" in kw:
            kw["minibatch_size"] = kw.pop("sgd_minibatch_size")
        return self._set(**kw)

    def rl_module(self, *, model_config=NotProvided, rl_module_spec=NotProvided, model_config_dict=NotProvided, **_):
        for mc in (model_config, model_config_dict):
            if mc is not NotProvided and mc is not None:
                self.model_config.update(dict(mc))
        if rl_module_spec is not NotProvided and rl_module_spec is not None:
            self.rl_module_class = getattr(rl_module_spec, "module_class", None)
            self.model_config.update(getattr(rl_module_spec, "model_config", None) or {})
        return self

    def evaluation(self, *, evaluation_interval=NotProvided, evaluation_duration=NotProvided, **_):
        return self._set(evaluation_interval=evaluation_interval, evaluation_duration=evaluation_duration)

    def debugging(self, *, seed=NotProvided, **_):
        return self._set(seed=seed)

    def reporting(self, *, metrics_num_episodes_for_smoothing=NotProvided, **_):
        return self._set(metrics_num_episodes_for_smoothing=metrics_num_episodes_for_smoothing)

    def resources(self, **_):
        return self

    def framework(self, framework="torch", **_):
        if framework not in ("torch", None):
            raise ValueError("only the torch framework is supported")
        return self

    def api_stack(self, **_):
        return self

    def fault_tolerance(self, **_):
        return self

    def checkpointing(self, **_):
        return self

    # --------------------------------------------------------------- utils
    def copy(self, copy_frozen=None):
        return copy.deepcopy(self)

    def to_dict(self) -> Dict[str, Any]:
        d = {k: v for k, v in self.__dict__.items() if not k.startswith("_")}
        d["algo_class"] = self.algo_class
        return d

    @classmethod
    def from_dict(cls, d: Dict[str, Any]):
        c = cls()
        for k, v in d.items():
            if k == "algo_class":
                continue
            setattr(c, k, v)
        return c

    def update_from_dict(self, d: Dict[str, Any]):
        for k, v in d.items():
            if k != "algo_class":
                setattr(self, k, v)
        return self

    def get(self, k, default=None):
        return getattr(self, k, default)

    def __getitem__(self, k):
        return getattr(self, k)

    @property
    def total_train_batch_size(self):
        if self.train_batch_size_per_learner:
            return self.train_batch_size_per_learner * max(1, self.num_learners)
        return self.train_batch_size

    def get_rollout_fragment_length(self):
        if self.rollout_fragment_length != "auto":
            return int(self.rollout_fragment_length)
        per = max(1, self.num_env_runners) * self.num_envs_per_env_runner
        return max(1, int(np.ceil(self.total_train_batch_size / per)))

    def module_factory(self) -> Callable:
        cls = self.rl_module_class or self.default_module_class()
        mc = dict(self.model_config)
        return lambda obs, act: cls(obs, act, mc)

    def default_module_class(self):
        return DefaultActorCriticModule

    def runner_config(self) -> Dict[str, Any]:
        return {"env": self.env, "env_config": self.env_config,
                "num_envs_per_env_runner": self.num_envs_per_env_runner,
                "rollout_fragment_length": self.get_rollout_fragment_length(), "seed": self.seed,
                "gamma": self.gamma, "module_factory": self.module_factory(),
                "metrics_num_episodes_for_smoothing": self.metrics_num_episodes_for_smoothing,
                "need_next_obs": False}

    def learner_config(self) -> Dict[str, Any]:
        return dict(self.to_dict())

    def validate(self):
        if self.env is None:
            raise ValueError("config.environment(env=...) is required")

    def build_algo(self, env=None, logger_creator=None) -> "Algorithm":
        if env is not None:
            self.env = env
        self.validate()
        return self.algo_class(config=self)

    build = build_algo


class Algorithm(Trainable):
    config_class = AlgorithmConfig
    learner_class = Learner

    @classmethod
    def get_default_config(cls) -> AlgorithmConfig:
        return cls.config_class(cls)

    def __init__(self, config=None, trial_dir: str = "", trial_id: str = "", env=None, **kw):
        if isinstance(config, dict):
            d = dict(config)
            cfg = self.get_default_config()
            cfg.update_from_dict(d)
            config = cfg
        self.algo_config: AlgorithmConfig = config if config is not None else self.get_default_config()
        if env is not None:
            self.algo_config.env = env
        super().__init__(self.algo_config.to_dict(), trial_dir, trial_id)

    # Trainable hooks -------------------------------------------------------
    def setup(self, _config):
        c = self.algo_config
        c.validate()
        if c.seed is not None:
            torch.manual_seed(c.seed)
            np.random.seed(c.seed)
        self.env_runner_group = EnvRunnerGroup(c.runner_config(), c.num_env_runners, c.num_cpus_per_env_runner)
        self.obs_space, self.act_space = self.env_runner_group.spaces()
        self.learner_group = LearnerGroup(self.learner_class, c.learner_config(), c.module_factory(),
                                          self.obs_space, self.act_space)
        self.env_steps_sampled = 0
        self.env_steps_trained = 0
        self.setup_algo()
        self._sync_weights()

    def setup_algo(self):
        pass

    def _sync_weights(self, extra: Optional[Dict] = None):
        self.env_runner_group.sync_weights(self.learner_group.get_module_state(), extra)

    def training_step(self) -> Dict[str, Any]:
        raise NotImplementedError

    def step(self) -> Dict[str, Any]:
        t0 = time.time()
        learner_stats = self.training_step()
        m = self.env_runner_group.metrics()
        out = {"env_runners": m, "learners": {"default_policy": learner_stats},
               "num_env_steps_sampled_lifetime": self.env_steps_sampled,
               "num_env_steps_trained_lifetime": self.env_steps_trained,
               "episode_return_mean": m["episode_return_mean"],
               "timers": dict(getattr(self, "_timers", {}), training_step_s=time.time() - t0)}
        c = self.algo_config
        if c.evaluation_interval and (self.iteration + 1) % c.evaluation_interval == 0:
            out["evaluation"] = self.evaluate()
        return out

    def evaluate(self) -> Dict[str, Any]:
        c = self.algo_config
        env = make_env(c.env, c.env_config)
        module = c.module_factory()(self.obs_space, self.act_space)
        module.set_state(self.learner_group.get_module_state())
        rets = []
        for ep in range(c.evaluation_duration):
            obs, _ = env.reset(seed=10_000 + ep)
            done, ret = False, 0.0
            while not done:
                a = module.forward_inference({"obs": torch.from_numpy(np.asarray(obs)[None])})["actions"][0]
                obs, r, te, tr, _ = env.step(a.numpy())
                ret += r
                done = te or tr
            rets.append(ret)
        return {"env_runners": {"episode_return_mean": float(np.mean(rets)), "num_episodes": len(rets)}}

    def compute_single_action(self, obs, explore: bool = False):
        module = getattr(self, "_inference_module", None)
        if module is None:
            module = self._inference_module = self.algo_config.module_factory()(self.obs_space, self.act_space)
        module.set_state(self.learner_group.get_module_state())
        b = {"obs": torch.from_numpy(np.asarray(obs)[None])}
        out = module.forward_exploration(b) if explore else module.forward_inference(b)
        return out["actions"][0].numpy()

    def get_module(self):
        m = self.algo_config.module_factory()(self.obs_space, self.act_space)
        m.set_state(self.learner_group.get_module_state())
        return m

    def save_checkpoint(self, checkpoint_dir: str):
        torch.save(self.learner_group.get_state(), os.path.join(checkpoint_dir, "learner_state.pt"))
        extra = self.extra_state()
        with open(os.path.join(checkpoint_dir, "algorithm_state.json"), "w") as f:
            json.dump({"algo": type(self).__name__, "env_steps_sampled": self.env_steps_sampled,
                       "env_steps_trained": self.env_steps_trained, "extra": extra}, f)
        return None

    def extra_state(self) -> Dict:
        return {}

    def load_extra_state(self, st: Dict):
        pass

    def load_checkpoint(self, checkpoint):
        d = checkpoint if isinstance(checkpoint, str) else checkpoint.get("path")
        st = torch.load(os.path.join(d, "learner_state.pt"), weights_only=True)
        self.learner_group.set_state(st)
        with open(os.path.join(d, "algorithm_state.json")) as f:
            a = json.load(f)
        self.env_steps_sampled = a["env_steps_sampled"]
        self.env_steps_trained = a["env_steps_trained"]
        self.load_extra_state(a.get("extra", {}))
        self._sync_weights()

    def save_to_path(self, path: Optional[str] = None) -> str:
        path = path or os.path.join(self._trial_dir or ".", f"checkpoint_{self.iteration:06d}")
        self.save(path)
        with open(os.path.join(path, "algorithm_config.pkl"), "wb") as f:
            import cloudpickle

            cloudpickle.dump(self.algo_config, f)
        return path

    @classmethod
    def from_checkpoint(cls, path: str) -> "Algorithm":
        import cloudpickle

        # written by save_to_path() (our own file)
        with open(os.path.join(path, "algorithm_config.pkl"), "rb") as f:
            cfg = cloudpickle.load(f)
        algo = cfg.algo_class(config=cfg)
        algo.restore(path)
        return algo

    def restore_from_path(self, path: str):
        self.restore(path)

    def cleanup(self):
        self.env_runner_group.stop()
        self.learner_group.stop()


def concat_fragments(frags, keys=None):
    """Concatenate time-major fragments along the env axis."""
    keys = keys or [k for k, v in frags[0].items() if isinstance(v, np.ndarray) and k != "last_obs"]
    out = {k: np.concatenate([f[k] for f in frags], axis=1) for k in keys}
    out["last_obs"] = np.concatenate([f["last_obs"] for f in frags], axis=0)
    return out
