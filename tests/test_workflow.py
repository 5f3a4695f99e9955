"""Durable workflows (reference: python/ray/workflow/tests/test_basic_workflows*.py,
test_recovery.py, test_cancellation.py, test_dynamic_workflow_ref.py)."""
import os
import time

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import workflow


@pytest.fixture
def wf(tmp_path):
    ray.init(num_cpus=4)
    workflow.init(str(tmp_path / "wf"))
    yield tmp_path
    ray.shutdown()


@ray.remote
def add(a, b):
    return a + b


@ray.remote
def mul(a, b):
    return a * b


@ray.remote
def flaky(marker_dir, x):
    p = os.path.join(marker_dir, "ran")
    n = len(os.listdir(marker_dir)) if os.path.isdir(marker_dir) else 0
    os.makedirs(marker_dir, exist_ok=True)
    open(os.path.join(marker_dir, f"run{n}"), "w").close()
    if os.path.exists(os.path.join(marker_dir, "..", "FAIL")):
        raise ValueError("injected failure")
    return x * 10


@ray.remote
def fib(n):
    if n <= 1:
        return n
    return workflow.continuation(add.bind(fib.bind(n - 1), fib.bind(n - 2)))


@ray.remote
def slow():
    time.sleep(30)
    return 1


def test_run_diamond_and_outputs(wf):
    a = add.options(**workflow.options(task_id="a")).bind(1, 2)
    b = mul.bind(a, 10)
    c = add.bind(a, 100)
    d = add.bind(b, c)
    assert workflow.run(d, workflow_id="diamond", metadata={"owner": "t"}) == 30 + 103
    assert workflow.get_status("diamond") == workflow.SUCCESSFUL
    assert workflow.get_output("diamond") == 133
    assert workflow.get_output("diamond", task_id="a") == 3
    md = workflow.get_metadata("diamond")
    assert md["user_metadata"] == {"owner": "t"} and md["stats"]["end_time"] >= md["stats"]["start_time"]
    assert ("diamond", workflow.SUCCESSFUL) in workflow.list_all()
    # re-running a finished workflow returns the stored output
    assert workflow.run(d, workflow_id="diamond") == 133


@ray.remote
def counted(marker_dir, x):
    os.makedirs(marker_dir, exist_ok=True)
    open(os.path.join(marker_dir, f"run{len(os.listdir(marker_dir))}"), "w").close()
    return x * 10


@ray.remote
def gate(flag, y, x):
    if os.path.exists(flag):
        raise ValueError("injected failure")
    return x + y


def test_failure_and_resume_skips_finished_tasks(wf):
    flag, marks = str(wf / "FAIL"), str(wf / "runs")
    open(flag, "w").close()
    first = counted.options(**workflow.options(task_id="first")).bind(marks, 1)
    dag = gate.options(max_retries=0).bind(flag, 5, first)
    with pytest.raises(workflow.WorkflowExecutionError):
        workflow.run(dag, workflow_id="resumable")
    assert workflow.get_status("resumable") == workflow.FAILED
    assert ("resumable", workflow.FAILED) in workflow.list_all({workflow.FAILED})
    assert len(os.listdir(marks)) == 1
    os.unlink(flag)
    assert workflow.resume("resumable") == 15
    # "first" checkpointed before the failure: not re-executed on resume
    assert len(os.listdir(marks)) == 1
    assert workflow.get_status("resumable") == workflow.SUCCESSFUL


def test_catch_exceptions(wf):
    open(wf / "FAIL", "w").close()
    node = flaky.options(**workflow.options(catch_exceptions=True)).bind(str(wf / "m"), 1)
    out, err = workflow.run(node, workflow_id="caught")
    assert out is None and isinstance(err, Exception)


def test_dynamic_continuation(wf):
    assert workflow.run(fib.bind(8), workflow_id="fib") == 21


def test_cancel_and_delete(wf):
    ref = workflow.run_async(slow.bind(), workflow_id="slow")
    deadline = time.time() + 30
    while workflow.get_status("slow") != workflow.RUNNING and time.time() < deadline:
        time.sleep(0.05)
    workflow.cancel("slow")
    with pytest.raises(Exception):
        ray.get(ref, timeout=60)
    assert workflow.get_status("slow") == workflow.CANCELED
    workflow.delete("slow")
    with pytest.raises(workflow.WorkflowNotFoundError):
        workflow.get_status("slow")


class Ev(workflow.EventListener):
    async def poll_for_event(self, v):
        return v * 2


def test_sleep_and_events(wf):
    t0 = time.time()
    dag = add.bind(workflow.wait_for_event(Ev, 21), add.bind(0, 0))
    assert workflow.run(dag, workflow_id="ev") == 42
    workflow.run(workflow.sleep(0.3), workflow_id="nap")
    assert time.time() - t0 >= 0.3
