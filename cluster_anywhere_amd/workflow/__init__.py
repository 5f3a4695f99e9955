"""Durable workflows (reference: python/ray/workflow/): a task DAG whose every
task output is checkpointed to storage, so a failed / interrupted / cancelled
workflow resumes from its last finished tasks.

Design: the workflow executor is itself a zero-CPU task (so ``run_async`` hands
back an ObjectRef, like the reference's workflow-management actor). It walks
the DAG with a ready-queue — every task whose inputs are finished is submitted
at once, independent branches overlap in the cluster scheduler — checkpoints
each output as it completes (``<storage>/<workflow_id>/tasks/<task_id>``) and
expands ``workflow.continuation(dag)`` returns in place (dynamic workflows).
"""
from .api import (EventListener, WorkflowCancellationError, WorkflowError, WorkflowExecutionError,
                  WorkflowNotFoundError, WorkflowStatus, cancel, continuation, delete, get_metadata,
                  get_output, get_output_async, get_status, init, list_all, options, resume, resume_all,
                  resume_async, run, run_async, sleep, wait_for_event)

globals().update(WorkflowStatus.__members__)

__all__ = ["init", "run", "run_async", "resume", "resume_async", "resume_all", "cancel", "list_all",
           "delete", "get_output", "get_output_async", "get_status", "get_metadata", "sleep",
           "wait_for_event", "options", "continuation", "EventListener", "WorkflowError",
           "WorkflowExecutionError", "WorkflowCancellationError", "WorkflowNotFoundError",
           "WorkflowStatus"]
