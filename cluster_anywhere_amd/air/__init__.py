"""AIR namespace (reference: python/ray/air/__init__.py): the shared config /
result types of Train and Tune, re-exported from their MI355X-native homes."""
from ..train.checkpoint import Checkpoint
from ..train.config import CheckpointConfig, DataConfig, FailureConfig, RunConfig, ScalingConfig
from ..train.trainer import Result
from . import session

DatasetConfig = DataConfig
DataBatchType = object  # numpy dict / pandas / arrow / torch batches are all accepted


class ResourceRequest:
    """Bundles of resources requested together (reference: air/execution/resources/request.py)."""

    def __init__(self, bundles, strategy: str = "PACK"):
        self.bundles = [dict(b) for b in bundles]
        self.strategy = strategy

    @property
    def head_bundle(self):
        return self.bundles[0] if self.bundles else {}

    def required_resources(self):
        out = {}
        for b in self.bundles:
            for k, v in b.items():
                out[k] = out.get(k, 0.0) + v
        return out

    def __eq__(self, other):
        return isinstance(other, ResourceRequest) and (self.bundles, self.strategy) == (other.bundles, other.strategy)

    def __hash__(self):
        return hash((tuple(tuple(sorted(b.items())) for b in self.bundles), self.strategy))

    def __repr__(self):
        return f"ResourceRequest(bundles={self.bundles}, strategy={self.strategy!r})"


class AcquiredResources:
    """Resources granted for a :class:`ResourceRequest` (a placement group underneath)."""

    def __init__(self, request: ResourceRequest, placement_group=None):
        self.resource_request = request
        self.placement_group = placement_group

    def annotate_remote_entities(self, entities):
        from ..util.scheduling_strategies import PlacementGroupSchedulingStrategy

        if self.placement_group is None:
            return list(entities)
        return [e.options(scheduling_strategy=PlacementGroupSchedulingStrategy(self.placement_group, i))
                for i, e in enumerate(entities)]


__all__ = ["Checkpoint", "CheckpointConfig", "DataConfig", "DatasetConfig", "FailureConfig",
           "RunConfig", "ScalingConfig", "Result", "session", "DataBatchType", "ResourceRequest",
           "AcquiredResources"]
