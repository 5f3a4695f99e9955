"""Reinforcement learning (reference: rllib/__init__.py)."""
from .algorithms import (ALGORITHMS, APPO, APPOConfig, BC, BCConfig, DQN, DQNConfig, IMPALA, IMPALAConfig, MARWIL,
                         MARWILConfig, PPO, PPOConfig, SAC, SACConfig, CQL, CQLConfig, DreamerV3, DreamerV3Config, Algorithm, AlgorithmConfig,
                         get_algorithm_class)
from .algorithms.algorithm import PolicySpec
from .callbacks import DefaultCallbacks, RLlibCallback
from .core import DefaultActorCriticModule, Learner, LearnerGroup, RLModule, RLModuleSpec
from .core.multi_rl_module import MultiRLModule, MultiRLModuleSpec
from .env import register_env
from .env.multi_agent_env import MultiAgentEnv, make_multi_agent
from .env import VectorEnv
from .env.base_env import BaseEnv
from .env.external_env import ExternalEnv
from .evaluation import RolloutWorker
from .policy import MultiAgentBatch, Policy, SampleBatch, TFPolicy, TorchPolicy

__all__ = [n for n in dir() if not n.startswith("_")]
