"""Smaller reference surfaces: experimental.get_object_locations, dag.DAGContext /
visualize / plot, job_submission.DriverInfo / JobType, LoggingConfig(JSON)
(reference: python/ray/experimental/locations.py, dag/context.py, dag/utils,
job_submission/__init__.py, _private/ray_logging/logging_config.py)."""
import json
import logging
import os
import subprocess
import sys

import numpy as np
import pytest

import cluster_anywhere_amd as ray

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=2)
    yield
    ray.shutdown()


@ray.remote
def small():
    return 1


@ray.remote
class Add:
    def add(self, x, y=1):
        return x + y


def test_object_locations(cluster):
    from cluster_anywhere_amd.experimental import get_local_object_locations, get_object_locations

    big = ray.put(np.zeros(1 << 20, np.uint8))
    s = small.remote()
    ray.get(s)
    locs = get_object_locations([big, s])
    node = ray.get_runtime_context().get_node_id()
    assert locs[big]["node_ids"] == [node] and locs[big]["object_size"] >= 1 << 20
    assert locs[s]["node_ids"] == []  # inline
    assert get_local_object_locations([big])[big]["node_ids"] == [node]


def test_dag_context_and_plot(cluster, tmp_path):
    from cluster_anywhere_amd.dag import DAGContext, InputNode, plot

    ctx = DAGContext.get_current()
    assert ctx.max_inflight_executions >= 1 and DAGContext.get_current() is ctx
    with pytest.raises(ValueError):
        DAGContext(read_iteration_timeout=100, get_timeout=1)
    a, b = Add.bind(), Add.bind()
    with InputNode() as inp:
        dag = b.add.bind(a.add.bind(inp), 5)
    dot = dag.visualize(str(tmp_path / "g"), return_dot=True)
    assert dot.startswith("digraph") and dot.count("->") >= 3 and "add" in dot
    assert os.path.exists(tmp_path / "g.dot")
    assert plot(dag, tmp_path / "p.dot") == dot
    assert ray.get(dag.execute(1)) == 7


def test_job_submission_names():
    from cluster_anywhere_amd.job_submission import DriverInfo, JobType

    assert JobType.SUBMISSION.value == "SUBMISSION" and JobType("DRIVER") is JobType.DRIVER
    d = DriverInfo(id="01", node_ip_address="127.0.0.1", pid="42")
    assert d.pid == "42"


def test_logging_config_json_reaches_workers(tmp_path):
    code = f"""
import logging, sys
sys.path.insert(0, {ROOT!r})
import cluster_anywhere_amd as ray
ray.init(num_cpus=1, logging_config=ray.LoggingConfig(encoding="JSON", log_level="INFO"),
         include_dashboard=False)

@ray.remote
def f():
    logging.getLogger("w").info("from-worker")
    return 1

logging.getLogger("d").info("from-driver")
assert ray.get(f.remote()) == 1
import time; time.sleep(1.5)
ray.shutdown()
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in (r.stderr + r.stdout).splitlines() if "from-" in ln]
    recs = []
    for ln in lines:
        i = ln.find("{")
        recs.append(json.loads(ln[i:]))
    assert any(x["message"] == "from-driver" and x["levelname"] == "INFO" for x in recs), lines
    worker = [x for x in recs if x["message"] == "from-worker"]
    assert worker and worker[0].get("job_id") and worker[0].get("worker_id"), lines
