"""Reinforcement learning (reference: rllib/__init__.py)."""
from .algorithms import (ALGORITHMS, APPO, APPOConfig, BC, BCConfig, DQN, DQNConfig, IMPALA, IMPALAConfig, MARWIL,
                         MARWILConfig, PPO, PPOConfig, SAC, SACConfig, CQL, CQLConfig, DreamerV3, DreamerV3Config, Algorithm, AlgorithmConfig,
                         get_algorithm_class)
from .core import DefaultActorCriticModule, Learner, LearnerGroup, RLModule, RLModuleSpec
from .env import register_env

__all__ = [n for n in dir() if not n.startswith("_")]
