"""CLI cluster lifecycle, dashboard REST/metrics and job submission
(reference: python/ray/tests/test_cli.py, dashboard/modules/job/tests/
test_job_manager.py, test_sdk.py, python/ray/tests/test_metrics_agent.py)."""
import json
import os
import subprocess
import sys
import time
import urllib.request

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cli(*args, tmp, check=True):
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-m", "cluster_anywhere_amd", *args], env=env, capture_output=True,
                       text=True, timeout=120)
    if check:
        assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


@pytest.fixture
def cluster(tmp_path):
    t = str(tmp_path / "caamd")
    _cli("start", "--head", "--port", "0", "--num-cpus", "2", "--dashboard-port", "0", "--temp-dir", t, tmp=t)
    info = json.load(open(os.path.join(t, "head.json")))
    _cli("start", "--address", info["address"], "--num-cpus", "1", "--num-gpus", "0", "--resources",
         '{"side": 1}', "--temp-dir", t, tmp=t)
    yield t, info
    _cli("stop", "--temp-dir", t, tmp=t)


def _get(url):
    with urllib.request.urlopen(url, timeout=30) as r:
        return r.read().decode()


def test_cli_cluster_dashboard_jobs_metrics(cluster):
    t, info = cluster
    dash = info["dashboard"]
    deadline = time.time() + 60
    while time.time() < deadline:
        nodes = json.loads(_get(dash + "/api/v0/nodes"))["data"]["result"]["result"]
        if sum(n["Alive"] for n in nodes) == 2:
            break
        time.sleep(0.2)
    assert sum(n["Alive"] for n in nodes) == 2
    out = _cli("status", "--temp-dir", t, tmp=t)
    assert "2 alive" in out and "side" in out
    # job submission through the dashboard REST API
    from cluster_anywhere_amd.job_submission import JobStatus, JobSubmissionClient

    c = JobSubmissionClient(dash)
    script = ("import cluster_anywhere_amd as ray; ray.init(); "
              "f = ray.remote(resources={'side': 1})(lambda: 41 + 1); print('answer', ray.get(f.remote()))")
    sid = c.submit_job(entrypoint=f"{sys.executable} -c \"{script}\"", runtime_env={"env_vars": {"FOO": "1"}})
    assert c.wait_until_finish(sid, 120) == JobStatus.SUCCEEDED, c.get_job_logs(sid)
    assert "answer 42" in c.get_job_logs(sid)
    bad = c.submit_job(entrypoint="exit 3")
    assert c.wait_until_finish(bad, 60) == JobStatus.FAILED
    assert c.get_job_info(bad).driver_exit_code == 3
    slow = c.submit_job(entrypoint="sleep 60")
    time.sleep(0.5)
    assert c.stop_job(slow)
    assert c.get_job_status(slow) == JobStatus.STOPPED
    assert {j.submission_id for j in c.list_jobs()} >= {sid, bad, slow}
    # application metrics recorded by a driver show up in the Prometheus export
    env = dict(os.environ, PYTHONPATH=ROOT, CAAMD_ADDRESS=info["unix"])
    code = ("import time, cluster_anywhere_amd as ray; from cluster_anywhere_amd.util.metrics import Counter, "
            "Histogram; ray.init(); c = Counter('app_requests', 'reqs', tag_keys=('route',)); "
            "c.inc(3, tags={'route': '/a'}); h = Histogram('app_lat', 'lat', boundaries=[0.1, 1.0]); "
            "h.observe(0.5); time.sleep(0.5); ray.shutdown()")
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=60)
    m = _get(dash + "/metrics")
    assert 'app_requests{route="/a"} 3.0' in m
    assert 'app_lat_bucket{le="1.0"} 1' in m and "ray_cluster_active_nodes 2" in m
    out = _cli("list", "nodes", "--address", info["unix"], tmp=t)
    assert len(json.loads(out)) == 2
