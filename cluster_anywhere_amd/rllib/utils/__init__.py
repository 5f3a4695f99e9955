"""RLlib utilities (reference: rllib/utils/)."""
from .replay_buffers import PrioritizedReplayBuffer, ReplayBuffer
