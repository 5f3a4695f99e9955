"""Autoscaler: node providers + resource-demand scaling (reference:
python/ray/autoscaler/). See :mod:`.autoscaler` for the algorithm."""
from .autoscaler import Monitor, StandardAutoscaler, load_config
from .node_provider import LocalNodeProvider, NodeProvider
from .sdk import request_resources

__all__ = ["StandardAutoscaler", "Monitor", "load_config", "NodeProvider", "LocalNodeProvider",
           "request_resources"]
