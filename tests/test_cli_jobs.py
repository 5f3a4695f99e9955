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


@pytest.fixture(scope="module")
def cluster(tmp_path_factory):
    t = str(tmp_path_factory.mktemp("cli") / "caamd")
    _cli("start", "--head", "--port", "0", "--num-cpus", "2", "--dashboard-port", "0", "--temp-dir", t, tmp=t)
    info = json.load(open(os.path.join(t, "head.json")))
    _cli("start", "--address", info["address"], "--num-cpus", "1", "--num-gpus", "0", "--resources",
         '{"side": 1}', "--temp-dir", t, tmp=t)
    deadline = time.time() + 60
    while time.time() < deadline:
        nodes = json.loads(_get(info["dashboard"] + "/api/v0/nodes"))["data"]["result"]["result"]
        if sum(n["Alive"] for n in nodes) == 2:
            break
        time.sleep(0.2)
    yield t, info
    _cli("stop", "--temp-dir", t, tmp=t)


def _get(url):
    with urllib.request.urlopen(url, timeout=30) as r:
        return r.read().decode()


@pytest.fixture(scope="module")
def jobs(cluster):
    from cluster_anywhere_amd.job_submission import JobSubmissionClient

    return JobSubmissionClient(cluster[1]["dashboard"])


def test_cli_status_and_dashboard_nodes(cluster):
    t, info = cluster
    nodes = json.loads(_get(info["dashboard"] + "/api/v0/nodes"))["data"]["result"]["result"]
    assert sum(n["Alive"] for n in nodes) == 2
    out = _cli("status", "--temp-dir", t, tmp=t)
    assert "2 alive" in out and "side" in out


def test_cli_list_nodes(cluster):
    t, info = cluster
    out = _cli("list", "nodes", "--address", info["unix"], tmp=t)
    assert len(json.loads(out)) == 2


def test_job_succeeds_with_runtime_env_and_logs(jobs):
    from cluster_anywhere_amd.job_submission import JobStatus

    script = ("import os, cluster_anywhere_amd as ray; ray.init(); "
              "f = ray.remote(resources={'side': 1})(lambda: 41 + 1); "
              "print('answer', ray.get(f.remote()), 'FOO', os.environ.get('FOO'))")
    sid = jobs.submit_job(entrypoint=f"{sys.executable} -c \"{script}\"", runtime_env={"env_vars": {"FOO": "1"}},
                          metadata={"owner": "tests"})
    assert jobs.wait_until_finish(sid, 120) == JobStatus.SUCCEEDED, jobs.get_job_logs(sid)
    logs = jobs.get_job_logs(sid)
    assert "answer 42" in logs and "FOO 1" in logs
    info = jobs.get_job_info(sid)
    assert info.metadata.get("owner") == "tests" and info.driver_exit_code == 0


def test_job_failure_reports_exit_code(jobs):
    from cluster_anywhere_amd.job_submission import JobStatus

    bad = jobs.submit_job(entrypoint="exit 3")
    assert jobs.wait_until_finish(bad, 60) == JobStatus.FAILED
    assert jobs.get_job_info(bad).driver_exit_code == 3


def test_job_stop_and_list(jobs):
    from cluster_anywhere_amd.job_submission import JobStatus

    slow = jobs.submit_job(entrypoint="sleep 60")
    time.sleep(0.5)
    assert jobs.stop_job(slow)
    assert jobs.get_job_status(slow) == JobStatus.STOPPED
    assert slow in {j.submission_id for j in jobs.list_jobs()}


def test_metrics_prometheus_export(cluster):
    t, info = cluster
    dash = info["dashboard"]
    env = dict(os.environ, PYTHONPATH=ROOT, CAAMD_ADDRESS=info["unix"])
    code = ("import time, cluster_anywhere_amd as ray; from cluster_anywhere_amd.util.metrics import Counter, "
            "Histogram; ray.init(); c = Counter('app_requests', 'reqs', tag_keys=('route',)); "
            "c.inc(3, tags={'route': '/a'}); h = Histogram('app_lat', 'lat', boundaries=[0.1, 1.0]); "
            "h.observe(0.5); time.sleep(0.5); ray.shutdown()")
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=60)
    m = _get(dash + "/metrics")
    assert 'app_requests{route="/a"} 3.0' in m
    assert 'app_lat_bucket{le="1.0"} 1' in m and "ray_cluster_active_nodes 2" in m


def test_cli_head_with_gcs_storage_restores_kv(tmp_path):
    """`start --head --gcs-storage`: a KV entry written through one head is served
    by the next head started on the same table log."""
    t = str(tmp_path / "caamd")
    store = str(tmp_path / "gcs.log")
    env = dict(os.environ, PYTHONPATH=ROOT)
    code = ("import sys, cluster_anywhere_amd as ray; from cluster_anywhere_amd.experimental import internal_kv as kv; "
            "ray.init(address=sys.argv[1]); op = sys.argv[2]; "
            "(kv._internal_kv_put(b'k', b'v1') if op == 'put' else print('VAL', kv._internal_kv_get(b'k'))); "
            "ray.shutdown()")
    for op in ("put", "get"):
        _cli("start", "--head", "--port", "0", "--num-cpus", "1", "--include-dashboard", "false", "--temp-dir", t,
             "--gcs-storage", store, tmp=t)
        info = json.load(open(os.path.join(t, "head.json")))
        p = subprocess.run([sys.executable, "-c", code, info["unix"], op], env=env, capture_output=True, text=True,
                           timeout=60)
        _cli("stop", "--temp-dir", t, tmp=t)
        assert p.returncode == 0, p.stdout + p.stderr
    assert "VAL b'v1'" in p.stdout, p.stdout
