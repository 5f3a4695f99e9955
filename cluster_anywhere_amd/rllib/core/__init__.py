"""RLModule / Learner core (reference: rllib/core/)."""
from .learner import Learner, LearnerGroup
from .rl_module import DefaultActorCriticModule, RLModule, RLModuleSpec
