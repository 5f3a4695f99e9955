"""Train v2 control plane (reference: python/ray/train/v2/_internal/execution/:
controller/controller.py:91 TrainController, controller/state.py, failure_handling/,
scaling_policy/). Enabled for every trainer with ``RAY_TRAIN_V2_ENABLED=1`` (the
reference's flag), or used directly::

    from cluster_anywhere_amd.train.v2 import TrainController
    result = TrainController(trainer).run()

The controller is a small state machine over the worker group of
:mod:`..trainer` (``_WorkerGroup``: one placement group + one actor per rank,
non-blocking ``poll()``): INITIALIZING -> SCHEDULING -> RUNNING ->
{FINISHED | RESTARTING (failure policy says retry) | RESIZING (scaling policy
found a better size) | ERRORED}, each new run attempt restoring from the
latest reported checkpoint. Scaling is a pluggable :class:`ScalingPolicy`
(fixed, or elastic between ``min_workers`` and ``max_workers`` by what the
cluster can place), failures a pluggable :class:`FailurePolicy` (default:
``FailureConfig.max_failures``, -1 = unlimited), and controller callbacks see
every state transition and decision.
"""
from .controller import (ControllerCallback, TrainController, TrainControllerState, TrainControllerStateType)
from .failure_policy import DefaultFailurePolicy, FailureDecision, FailurePolicy
from .scaling_policy import (ElasticScalingPolicy, FixedScalingPolicy, NoopDecision, ResizeDecision,
                             ScalingDecision, ScalingPolicy, create_scaling_policy)

__all__ = ["TrainController", "TrainControllerState", "TrainControllerStateType", "ControllerCallback",
           "FailurePolicy", "DefaultFailurePolicy", "FailureDecision", "ScalingPolicy", "FixedScalingPolicy",
           "ElasticScalingPolicy", "ScalingDecision", "ResizeDecision", "NoopDecision", "create_scaling_policy"]
