"""Serve exceptions (reference: python/ray/serve/exceptions.py:9,14,34,48)."""
from __future__ import annotations

from ..exceptions import TaskCancelledError


class RayServeException(Exception):
    pass


class BackPressureError(RayServeException):
    """A handle's router already holds ``max_queued_requests`` requests that wait for
    a replica with a free ``max_ongoing_requests`` slot (the HTTP proxy answers 503)."""

    def __init__(self, num_queued_requests: int, max_queued_requests: int):
        super().__init__(num_queued_requests, max_queued_requests)
        self.num_queued_requests = num_queued_requests
        self.max_queued_requests = max_queued_requests

    @property
    def message(self) -> str:
        return (f"Request dropped due to backpressure (num_queued_requests={self.num_queued_requests}, "
                f"max_queued_requests={self.max_queued_requests}).")

    def __str__(self) -> str:
        return self.message


class RequestCancelledError(RayServeException, TaskCancelledError):
    def __init__(self, request_id: str = ""):
        super().__init__(request_id)
        self.request_id = request_id

    def __str__(self) -> str:
        return f"Request {self.request_id} was cancelled."


class DeploymentUnavailableError(RayServeException):
    def __init__(self, deployment_id=""):
        super().__init__(deployment_id)
        self.deployment_id = deployment_id

    @property
    def message(self) -> str:
        return f"Deployment {self.deployment_id!r} is unavailable."

    def __str__(self) -> str:
        return self.message
