"""RL algorithms (reference: rllib/algorithms/)."""
from .algorithm import Algorithm, AlgorithmConfig
from .cql import CQL, CQLConfig
from .dqn import DQN, DQNConfig
from .dreamerv3 import DreamerV3, DreamerV3Config
from .impala import APPO, APPOConfig, IMPALA, IMPALAConfig
from .marwil import BC, BCConfig, MARWIL, MARWILConfig
from .ppo import PPO, PPOConfig
from .sac import SAC, SACConfig

ALGORITHMS = {"PPO": PPO, "APPO": APPO, "IMPALA": IMPALA, "DQN": DQN, "SAC": SAC, "BC": BC, "MARWIL": MARWIL, "CQL": CQL, "DreamerV3": DreamerV3}


def get_algorithm_class(name: str):
    return ALGORITHMS[name]
