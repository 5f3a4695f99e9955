"""Model serving (reference: python/ray/serve/__init__.py)."""
from .api import (delete, get_app_handle, get_deployment_handle, grpc_port, http_port, run, shutdown, start,
                  status)
from .grpc_proxy import gRPCOptions
from .batching import batch
from .config import AutoscalingConfig, DeploymentConfig, HTTPOptions
from .context import get_multiplexed_model_id, get_replica_context
from .deployment import Application, Deployment, deployment, ingress
from .handle import DeploymentHandle, DeploymentResponse, DeploymentResponseGenerator
from .multiplex import multiplexed
from . import exceptions
from .exceptions import BackPressureError, RayServeException, RequestCancelledError

__all__ = ["run", "start", "shutdown", "delete", "status", "get_app_handle", "get_deployment_handle",
           "http_port", "grpc_port", "gRPCOptions", "batch", "multiplexed", "get_multiplexed_model_id", "get_replica_context",
           "deployment", "ingress", "Application", "Deployment", "DeploymentHandle", "DeploymentResponse",
           "DeploymentResponseGenerator", "AutoscalingConfig", "DeploymentConfig", "HTTPOptions", "exceptions"]
