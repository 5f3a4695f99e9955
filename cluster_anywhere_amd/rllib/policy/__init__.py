"""Old API stack policies and sample batches (reference: rllib/policy/)."""
from .policy import Policy, TFPolicy, TorchPolicy, TorchPolicyV2
from .sample_batch import DEFAULT_POLICY_ID, MultiAgentBatch, SampleBatch, concat_samples

__all__ = ["Policy", "TorchPolicy", "TorchPolicyV2", "TFPolicy", "SampleBatch", "MultiAgentBatch",
           "concat_samples", "DEFAULT_POLICY_ID"]
