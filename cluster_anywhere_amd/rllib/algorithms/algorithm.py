"""Algorithm / AlgorithmConfig (reference: rllib/algorithms/algorithm.py,
algorithm_config.py — builder methods ``environment``, ``env_runners``,
``learners``, ``training``, ``rl_module``, ``evaluation``, ``debugging``,
``reporting``, ``resources``, ``framework``, ``api_stack``, ``multi_agent``,
``callbacks``; connector hooks ``env_runners(env_to_module_connector=...,
module_to_env_connector=...)`` and ``training(learner_connector=...)``).

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
from ..callbacks import RLlibCallback, make_callbacks
from ..core.learner import Learner, LearnerGroup, MultiLearner
from ..core.multi_rl_module import DEFAULT_MODULE_ID, MultiRLModuleSpec
from ..core.rl_module import DefaultActorCriticModule, RLModuleSpec
from ..env import make_env
from ..env.env_runner import EnvRunner, EnvRunnerGroup
from ..env.multi_agent_env_runner import MultiAgentEnvRunner


class _NotProvided:
    pass


NotProvided = _NotProvided()


class PolicySpec:
    """Per-module entry of ``config.multi_agent(policies={...})`` (reference:
    rllib/policy/policy.py PolicySpec): optional explicit spaces and a model
    config override for the module."""

    def __init__(self, policy_class=None, observation_space=None, action_space=None, config=None):
        self.policy_class = policy_class
        self.observation_space = observation_space
        self.action_space = action_space
        self.config = dict(config or {})


def _default_mapping(agent_id, episode, **kwargs):
    return DEFAULT_MODULE_ID


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
        # > 0: env runners act on a (fractional) GPU -- their module forward runs on
        # the device instead of the runner's one CPU thread (reference:
        # AlgorithmConfig.env_runners(num_gpus_per_env_runner=...))
        self.num_gpus_per_env_runner = 0
        # learners
        self.num_learners = 0
        self.num_gpus_per_learner = 1
        self.learner_batch_transport = None
        self.learner_checkpoint_interval = 10
        self.learner_dist_backend = None
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
        self.learner_connector = None
        # connectors
        self.env_to_module_connector = None
        self.module_to_env_connector = None
        # multi-agent
        self.policies: Optional[Dict[str, Any]] = None
        self.policy_mapping_fn: Callable = _default_mapping
        self.policies_to_train = None
        self.multi_rl_module_spec: Optional[MultiRLModuleSpec] = None
        # callbacks
        self.callbacks_class = None
        self.callbacks_functions: Dict[str, Callable] = {}
        # fault tolerance (reference: AlgorithmConfig.fault_tolerance)
        self.restart_failed_env_runners = True
        self.ignore_env_runner_failures = False
        self.max_num_env_runner_restarts = 1000
        self.delay_between_env_runner_restarts_s = 0.0
        self.env_runner_health_probe_timeout_s = 30.0
        # learner actors of a LearnerGroup are re-created from the last learner state
        self.restart_failed_learners = True
        self.max_num_learner_restarts = 100
        # offline data (reference: AlgorithmConfig.offline_data): input for BC / MARWIL /
        # CQL, streamed through a Data pipeline; `output` records env-runner episodes
        self.input_ = None
        self.input_read_method = "read_parquet"
        self.input_read_method_kwargs: Dict = {}
        self.map_batches_kwargs: Dict = {}
        self.iter_batches_kwargs: Dict = {}
        self.prelearner_class = None
        self.shuffle_buffer_rows = None
        self.output = None
        self.output_max_rows_per_file = 10_000
        self.output_write_episodes = True
        # off-policy estimation on offline episodes at evaluation time
        self.off_policy_estimation_methods: Dict = {}
        self.ope_max_rows = 50_000
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
                    rollout_fragment_length=NotProvided, num_cpus_per_env_runner=NotProvided,
                    num_gpus_per_env_runner=NotProvided,
                    env_to_module_connector=NotProvided, module_to_env_connector=NotProvided, **_):
        return self._set(num_env_runners=num_env_runners, num_envs_per_env_runner=num_envs_per_env_runner,
                         rollout_fragment_length=rollout_fragment_length,
                         num_cpus_per_env_runner=num_cpus_per_env_runner,
                         num_gpus_per_env_runner=num_gpus_per_env_runner,
                         env_to_module_connector=env_to_module_connector,
                         module_to_env_connector=module_to_env_connector)

    rollouts = env_runners

    def learners(self, *, num_learners=NotProvided, num_gpus_per_learner=NotProvided,
                 num_cpus_per_learner=NotProvided, learner_batch_transport=NotProvided,
                 learner_checkpoint_interval=NotProvided, learner_dist_backend=NotProvided, **_):
        """``learner_batch_transport``: "ipc" / "shm" / "pickle" (None: ipc for GPU
        learners on one node, else shm; see LearnerGroup); ``learner_checkpoint_interval``:
        updates between the learner-state snapshots a restarted group restores;
        ``learner_dist_backend``: the learners' process-group backend (None: nccl =
        RCCL on GPU, gloo on CPU)."""
        return self._set(num_learners=num_learners, num_gpus_per_learner=num_gpus_per_learner,
                         num_cpus_per_learner=num_cpus_per_learner, learner_batch_transport=learner_batch_transport,
                         learner_checkpoint_interval=learner_checkpoint_interval,
                         learner_dist_backend=learner_dist_backend)

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
        if isinstance(rl_module_spec, MultiRLModuleSpec):
            self.multi_rl_module_spec = rl_module_spec
        elif rl_module_spec is not NotProvided and rl_module_spec is not None:
            self.rl_module_class = getattr(rl_module_spec, "module_class", None)
            self.model_config.update(getattr(rl_module_spec, "model_config", None) or {})
        return self

    def multi_agent(self, *, policies=NotProvided, policy_mapping_fn=NotProvided, policies_to_train=NotProvided,
                    **_):
        """``policies``: a set/list of module ids or a dict id -> PolicySpec /
        RLModuleSpec / (obs_space, act_space) / None; ``policy_mapping_fn(agent_id,
        episode, **kw)`` -> module id (fixed per episode)."""
        if policies is not NotProvided:
            self.policies = {p: None for p in policies} if not isinstance(policies, dict) else dict(policies)
        if policy_mapping_fn is not NotProvided and policy_mapping_fn is not None:
            self.policy_mapping_fn = policy_mapping_fn
        if policies_to_train is not NotProvided:
            self.policies_to_train = None if policies_to_train is None else list(policies_to_train)
        return self

    def callbacks(self, callbacks_class=NotProvided, **on_hooks):
        """A callback class (or list of classes), and/or ``on_<hook>=fn`` functions."""
        if callbacks_class is not NotProvided:
            self.callbacks_class = callbacks_class
        for k, fn in on_hooks.items():
            if fn is not NotProvided and fn is not None:
                self.callbacks_functions[k] = fn
        return self

    @property
    def is_multi_agent(self) -> bool:
        return self.policies is not None

    def _module_specs(self) -> MultiRLModuleSpec:
        specs = dict(self.multi_rl_module_spec.rl_module_specs) if self.multi_rl_module_spec else {}
        for mid, ps in (self.policies or {}).items():
            if mid in specs:
                continue
            if isinstance(ps, RLModuleSpec):
                specs[mid] = ps
            elif isinstance(ps, PolicySpec):
                specs[mid] = RLModuleSpec(None, ps.config.get("model", ps.config), ps.observation_space,
                                          ps.action_space)
            elif isinstance(ps, tuple) and len(ps) == 2:
                specs[mid] = RLModuleSpec(None, {}, ps[0], ps[1])
        return MultiRLModuleSpec(specs)

    def module_ids(self):
        ids = list(self.policies or {})
        if self.multi_rl_module_spec:
            ids += [m for m in self.multi_rl_module_spec.rl_module_specs if m not in ids]
        return ids

    def algo_model_config(self) -> Dict[str, Any]:
        """``model_config`` plus the algorithm's own module settings (DQN's
        dueling flag, SAC's initial temperature ...)."""
        return dict(self.model_config)

    def multi_module_factory(self) -> Callable:
        spec = self._module_specs()
        cls = self.rl_module_class or self.default_module_class()
        mc = self.algo_model_config()
        return lambda spaces: spec.build(spaces, cls, mc)

    def module_factories(self) -> Dict[str, Callable]:
        spec = self._module_specs()
        cls = self.rl_module_class or self.default_module_class()
        return {mid: spec.module_factory(mid, cls, self.algo_model_config()) for mid in self.module_ids()}

    def policy_spaces(self) -> Dict[str, tuple]:
        out = {}
        for mid, sp in self._module_specs().rl_module_specs.items():
            if sp.observation_space is not None and sp.action_space is not None:
                out[mid] = (sp.observation_space, sp.action_space)
        return out

    def evaluation(self, *, evaluation_interval=NotProvided, evaluation_duration=NotProvided,
                   off_policy_estimation_methods=NotProvided, **_):
        """``off_policy_estimation_methods``: ``{name: {"type": ImportanceSampling |
        WeightedImportanceSampling | DirectMethod | DoublyRobust (or "is" / "wis" /
        "dm" / "dr"), **kwargs}}`` -- estimated on the offline ``input_`` episodes
        (which must carry the behaviour policy's ``action_prob``)."""
        return self._set(evaluation_interval=evaluation_interval, evaluation_duration=evaluation_duration,
                         off_policy_estimation_methods=(dict(off_policy_estimation_methods or {})
                                                        if off_policy_estimation_methods is not NotProvided
                                                        else NotProvided))

    def offline_data(self, *, input_=NotProvided, input_read_method=NotProvided,
                     input_read_method_kwargs=NotProvided, map_batches_kwargs=NotProvided,
                     iter_batches_kwargs=NotProvided, prelearner_class=NotProvided, shuffle_buffer_rows=NotProvided,
                     output=NotProvided, output_max_rows_per_file=NotProvided, output_write_episodes=NotProvided,
                     **_):
        """Offline input (paths / a Dataset -> streamed; column dicts -> in memory) and
        episode output (reference: ``AlgorithmConfig.offline_data``)."""
        return self._set(input_=input_, input_read_method=input_read_method,
                         input_read_method_kwargs=input_read_method_kwargs, map_batches_kwargs=map_batches_kwargs,
                         iter_batches_kwargs=iter_batches_kwargs, prelearner_class=prelearner_class,
                         shuffle_buffer_rows=shuffle_buffer_rows, output=output,
                         output_max_rows_per_file=output_max_rows_per_file,
                         output_write_episodes=output_write_episodes)

    def build_offline_data(self, columns=None):
        from ..offline import OfflineData

        return OfflineData(self.input_, gamma=self.gamma, columns=columns, input_read_method=self.input_read_method,
                           input_read_method_kwargs=self.input_read_method_kwargs,
                           map_batches_kwargs=self.map_batches_kwargs, iter_batches_kwargs=self.iter_batches_kwargs,
                           prelearner_class=self.prelearner_class, shuffle_buffer_rows=self.shuffle_buffer_rows,
                           seed=self.seed)

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

    def fault_tolerance(self, *, restart_failed_env_runners=NotProvided, ignore_env_runner_failures=NotProvided,
                        max_num_env_runner_restarts=NotProvided, delay_between_env_runner_restarts_s=NotProvided,
                        env_runner_health_probe_timeout_s=NotProvided, restart_failed_learners=NotProvided,
                        max_num_learner_restarts=NotProvided, **_):
        return self._set(restart_failed_env_runners=restart_failed_env_runners,
                         ignore_env_runner_failures=ignore_env_runner_failures,
                         max_num_env_runner_restarts=max_num_env_runner_restarts,
                         delay_between_env_runner_restarts_s=delay_between_env_runner_restarts_s,
                         env_runner_health_probe_timeout_s=env_runner_health_probe_timeout_s,
                         restart_failed_learners=restart_failed_learners,
                         max_num_learner_restarts=max_num_learner_restarts)

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
            n = int(self.rollout_fragment_length)
        else:
            per = max(1, self.num_env_runners) * self.num_envs_per_env_runner
            n = max(1, int(np.ceil(self.total_train_batch_size / per)))
        if self.model_config.get("use_lstm") or self.model_config.get("use_attention"):  # whole max_seq_len sequences
            L = int(self.model_config.get("max_seq_len", 20))
            n = ((n + L - 1) // L) * L
        return n

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
                "need_next_obs": False, "num_gpus_per_env_runner": self.num_gpus_per_env_runner,
                "output": self.output, "output_max_rows_per_file": self.output_max_rows_per_file,
                "output_write_episodes": self.output_write_episodes,
                "env_to_module_connector": self.env_to_module_connector,
                "module_to_env_connector": self.module_to_env_connector,
                "callbacks_class": self.callbacks_class, "callbacks_functions": dict(self.callbacks_functions),
                **({"policies": self.module_ids(), "policy_mapping_fn": self.policy_mapping_fn,
                    "policy_spaces": self.policy_spaces(), "multi_module_factory": self.multi_module_factory(),
                    "max_seq_len": (int(self.model_config.get("max_seq_len", 20))
                                    if self.model_config.get("use_lstm") or self.model_config.get("use_attention")
                                    else None)}
                   if self.is_multi_agent else {})}

    def learner_config(self) -> Dict[str, Any]:
        return dict(self.to_dict())

    def validate(self):
        if self.env is None:
            raise ValueError("config.environment(env=...) is required")
        if self.is_multi_agent:
            if not self.module_ids():
                raise ValueError("config.multi_agent(policies=...) needs at least one module id")
            if self.algo_class is not None and not getattr(self.algo_class, "supports_multi_agent", False):
                raise NotImplementedError(f"{self.algo_class.__name__} has no multi-agent training step")
            if ((self.model_config.get("use_lstm") or self.model_config.get("use_attention"))
                    and self.algo_class is not None
                    and not getattr(self.algo_class, "supports_recurrent_multi_agent", False)):
                raise NotImplementedError(f"{self.algo_class.__name__}: recurrent modules are single-agent only")

    def build_algo(self, env=None, logger_creator=None) -> "Algorithm":
        if env is not None:
            self.env = env
        self.validate()
        return self.algo_class(config=self)

    build = build_algo


class Algorithm(Trainable):
    config_class = AlgorithmConfig
    learner_class = Learner
    supports_multi_agent = False
    is_multi_agent = False
    callbacks = RLlibCallback()  # replaced per instance in setup()
    _connector_state = None

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
        self.callbacks = make_callbacks(c.callbacks_class, c.callbacks_functions)
        self.is_multi_agent = c.is_multi_agent
        runner_cls = MultiAgentEnvRunner if self.is_multi_agent else EnvRunner
        self.env_runner_group = EnvRunnerGroup(
            c.runner_config(), c.num_env_runners, c.num_cpus_per_env_runner, runner_cls=runner_cls,
            num_gpus_per_env_runner=c.num_gpus_per_env_runner,
            restart_failed=c.restart_failed_env_runners, ignore_failures=c.ignore_env_runner_failures,
            max_restarts=c.max_num_env_runner_restarts, restart_delay_s=c.delay_between_env_runner_restarts_s,
            on_recreated=self._on_env_runners_recreated)
        self.obs_space, self.act_space = self.env_runner_group.spaces()
        if self.is_multi_agent:
            self.module_spaces = self.obs_space  # module id -> (obs_space, act_space)
            train = c.policies_to_train or c.module_ids()
            facs = c.module_factories()
            self.learner_group = LearnerGroup(MultiLearner.of(self.learner_class), c.learner_config(),
                                              {m: facs[m] for m in train},
                                              {m: self.module_spaces[m][0] for m in train},
                                              {m: self.module_spaces[m][1] for m in train})
        else:
            self.learner_group = LearnerGroup(self.learner_class, c.learner_config(), c.module_factory(),
                                              self.obs_space, self.act_space)
        self.env_steps_sampled = 0
        self.env_steps_trained = 0
        self.agent_steps_sampled = 0
        self.setup_algo()
        self._sync_weights()
        self.callbacks.on_algorithm_init(algorithm=self, metrics_logger=None)

    def setup_algo(self):
        pass

    def _on_env_runners_recreated(self, indices):
        cb = getattr(self, "callbacks", None)
        if cb is not None:
            cb.on_env_runners_recreated(algorithm=self, env_runner_group=self.env_runner_group,
                                        env_runner_indices=indices, is_evaluation=False)

    def _sync_weights(self, extra: Optional[Dict] = None):
        g = self.env_runner_group
        if self._ipc_weights():
            # GPU runners on this node: a device snapshot shared by HIP IPC handles
            g.sync_weights(self.learner_group.get_module_state(on_device=True), extra, transport="ipc")
            return
        g.sync_weights(self.learner_group.get_module_state(), extra)

    def _ipc_weights(self) -> bool:
        """Weights go to the env runners over HIP IPC: remote runners acting on GPUs
        and a local learner whose module lives on a GPU of this node (single node)."""
        c = self.algo_config
        if not (c.num_gpus_per_env_runner and self.env_runner_group.remote and not self.is_multi_agent):
            return False
        lg = self.learner_group
        loc = getattr(lg, "local", None)
        if loc is None or not hasattr(loc, "module"):
            return False
        try:
            p = next(loc.module.parameters())
        except StopIteration:
            return False
        from ...core import api as core

        return p.is_cuda and len([n for n in core.nodes() if n.get("Alive")]) == 1

    def training_step(self) -> Dict[str, Any]:
        raise NotImplementedError

    def step(self) -> Dict[str, Any]:
        t0 = time.time()
        learner_stats = self.training_step()
        self._connector_state = self.env_runner_group.sync_connector_states()
        m = self.env_runner_group.metrics()
        learners = learner_stats if self.is_multi_agent else {"default_policy": learner_stats}
        out = {"env_runners": m, "learners": learners,
               "num_env_steps_sampled_lifetime": self.env_steps_sampled,
               "num_env_steps_trained_lifetime": self.env_steps_trained,
               "episode_return_mean": m["episode_return_mean"],
               "timers": dict(getattr(self, "_timers", {}), training_step_s=time.time() - t0)}
        if self.is_multi_agent:
            out["num_agent_steps_sampled_lifetime"] = self.agent_steps_sampled
        c = self.algo_config
        if c.evaluation_interval and (self.iteration + 1) % c.evaluation_interval == 0:
            out["evaluation"] = self.evaluate()
        self.callbacks.on_train_result(algorithm=self, metrics_logger=None, result=out)
        return out

    def _evaluation_runner(self):
        r = getattr(self, "_eval_runner", None)
        if r is None:
            c = self.algo_config
            cfg = dict(c.runner_config(), num_envs_per_env_runner=1, seed=10_000)
            cls = MultiAgentEnvRunner if self.is_multi_agent else EnvRunner
            r = self._eval_runner = cls(cfg, 0)
        return r

    def evaluate(self) -> Dict[str, Any]:
        """``evaluation_duration`` greedy episodes on a local evaluation runner
        (same connectors, with the training runners' merged connector state)."""
        c = self.algo_config
        self.callbacks.on_evaluate_start(algorithm=self, metrics_logger=None)
        r = self._evaluation_runner()
        r.set_weights(self.learner_group.get_module_state())
        if getattr(self, "_connector_state", None):
            r.set_connector_state(self._connector_state)
        r.reset_envs(10_000)
        rets = r.sample_episodes(c.evaluation_duration, explore=False)
        out = {"env_runners": {"episode_return_mean": float(np.mean(rets)), "num_episodes": len(rets)}}
        if c.off_policy_estimation_methods:
            out["off_policy_estimator"] = self.estimate_off_policy()
        if self.is_multi_agent:
            m = r.get_metrics()
            out["env_runners"]["module_episode_returns_mean"] = {
                k: float(np.mean(v[-len(rets):])) for k, v in m["module_episode_returns_mean"].items() if v}
        self.callbacks.on_evaluate_end(algorithm=self, metrics_logger=None, evaluation_metrics=out)
        return out

    def estimate_off_policy(self, episodes=None) -> Dict[str, Dict[str, float]]:
        """Every configured off-policy estimator on offline episodes (default: up to
        ``ope_max_rows`` rows of ``input_``), with the current module as the target
        policy (reference: ``evaluation/off_policy_estimator/<name>``)."""
        from ..offline import make_estimator

        c = self.algo_config
        if episodes is None:
            od = getattr(self, "offline_data", None)
            if od is None:
                if c.input_ is None:
                    raise ValueError("off-policy estimation needs config.offline_data(input_=...)")
                od = self.offline_data = c.build_offline_data()
            episodes = list(od.iter_episodes(max_rows=c.ope_max_rows))
        module = self.get_module()
        return {name: make_estimator(spec, module, c.gamma).estimate(episodes)
                for name, spec in c.off_policy_estimation_methods.items()}

    def compute_single_action(self, obs, explore: bool = False, policy_id: Optional[str] = None):
        module = self.get_module(policy_id)
        b = {"obs": torch.from_numpy(np.asarray(obs)[None])}
        out = module.forward_exploration(b) if explore else module.forward_inference(b)
        return out["actions"][0].numpy()

    def get_module(self, module_id: Optional[str] = None):
        c = self.algo_config
        if self.is_multi_agent:
            st = self.learner_group.get_module_state()
            mid = module_id or next(iter(st))
            obs, act = self.module_spaces[mid]
            m = c.module_factories()[mid](obs, act)
            m.set_state(st[mid])
            return m
        m = c.module_factory()(self.obs_space, self.act_space)
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
        self.callbacks.on_checkpoint_loaded(algorithm=self)

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
    """Concatenate time-major fragments along the env axis (``last_*`` entries,
    one row per env, along axis 0)."""
    keys = keys or [k for k, v in frags[0].items() if isinstance(v, np.ndarray) and not k.startswith("last_")]
    out = {k: np.concatenate([f[k] for f in frags], axis=1) for k in keys}
    for k in frags[0]:
        if k.startswith("last_") and isinstance(frags[0][k], np.ndarray):
            out[k] = np.concatenate([f[k] for f in frags], axis=0)
    return out


class OffPolicyMixin:
    """Replay-based training step shared by DQN and SAC (reference roles:
    dqn.py:610 ``training_step``, sac.py). Multi-agent: one replay buffer per
    trained module, filled from that module's transitions (padding dropped);
    every update samples each module's buffer and trains all modules in one
    learner call, priorities go back per module."""

    default_capacity = 50_000

    def _make_buffer(self):
        from ..utils.replay_buffers import PrioritizedReplayBuffer, ReplayBuffer

        c = self.algo_config
        rb = dict(c.replay_buffer_config)
        cap = rb.get("capacity", self.default_capacity)
        if "Prioritized" in rb.get("type", ""):
            return PrioritizedReplayBuffer(cap, rb.get("alpha", 0.6), rb.get("beta", 0.4), seed=c.seed)
        return ReplayBuffer(cap, seed=c.seed)

    def setup_replay(self):
        c = self.algo_config
        if self.is_multi_agent:
            train = c.policies_to_train or c.module_ids()
            self.buffers = {m: self._make_buffer() for m in train}
            self.buffer = None
        else:
            self.buffer = self._make_buffer()
            self.buffers = None

    def sample_into_replay(self) -> int:
        """One round of sampling into the buffer(s); returns env steps sampled."""
        from ..utils.replay_buffers import fragments_to_transitions

        frags = self.env_runner_group.sample()
        if self.is_multi_agent:
            from ..env.multi_agent_env_runner import concat_multi_agent

            for mid, f in concat_multi_agent(frags).items():
                if mid in self.buffers:
                    self.buffers[mid].add(fragments_to_transitions(f))
            self.agent_steps_sampled += sum(f["agent_steps"] for f in frags)
            steps = sum(f["env_steps"] for f in frags)
        else:
            frag = concat_fragments(frags)
            steps = int(frag["rewards"].size)
            self.buffer.add(fragments_to_transitions(frag))
        self.env_steps_sampled += steps
        return steps

    def replay_ready(self) -> bool:
        need = self.algo_config.num_steps_sampled_before_learning_starts
        if self.is_multi_agent:
            return all(len(b) >= need for b in self.buffers.values())
        return len(self.buffer) >= need

    def replay_update(self) -> Dict[str, Any]:
        """One learner update on a freshly sampled replay batch (per module when
        multi-agent); priorities are refreshed from the TD errors."""
        c = self.algo_config
        lg = self.learner_group
        call = (lambda b: lg.local.train_on(b)) if lg.local is not None else (lambda b: lg.call("train_on", b))
        if self.is_multi_agent:
            batches, idx = {}, {}
            for m, buf in self.buffers.items():
                b = buf.sample(c.train_batch_size)
                idx[m] = b.pop("batch_indexes")
                batches[m] = b
            res = call(batches)
            for m, (_, td) in res.items():
                self.buffers[m].update_priorities(idx[m], td)
            self.env_steps_trained += c.train_batch_size
            return {m: r[0] for m, r in res.items()}
        b = self.buffer.sample(c.train_batch_size)
        i = b.pop("batch_indexes")
        stats, td = call(b)
        self.buffer.update_priorities(i, td)
        self.env_steps_trained += c.train_batch_size
        return stats
