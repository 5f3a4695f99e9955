"""Dashboard node / GPU physical metrics (reference:
python/ray/dashboard/modules/reporter/reporter_agent.py:89-140,489) and the Serve
REST API (dashboard/modules/serve/serve_rest_api_impl.py:116-157): amdsmi is
replaced by a fake that reports two busy GPUs; every node of a 2-node CLI cluster
publishes samples that show up in /api/v0/nodes and as ray_node_* Prometheus
gauges; PUT / GET / DELETE /api/serve/applications/ deploy, report and shut down an
application, also through ``serve deploy/status/shutdown --address http://...``."""
import json
import os
import socket
import subprocess
import sys
import textwrap
import time
import urllib.request

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _FakeSmi:
    ok = True

    def sample(self):
        return [{"index": 0, "name": "AMD Instinct MI355X", "utilization_gpu": 87.0, "memory_used": 5 << 30,
                 "memory_total": 288 << 30, "power_w": 910.0, "temperature_c": 71.0},
                {"index": 1, "name": "AMD Instinct MI355X", "utilization_gpu": 0.0, "memory_used": 1 << 30,
                 "memory_total": 288 << 30, "power_w": 250.0, "temperature_c": 40.0}]


def test_sample_node_with_mocked_amdsmi(monkeypatch):
    from cluster_anywhere_amd.dashboard import reporter

    monkeypatch.setattr(reporter, "_SMI", _FakeSmi())
    s = reporter.sample_node("/tmp")
    assert s["cpu_count"] >= 1 and s["mem_total"] > s["mem_used"] > 0 and "/" in s["disk"]
    assert [g["utilization_gpu"] for g in s["gpus"]] == [87.0, 0.0]
    lines = reporter.prometheus_lines([{"NodeManagerAddress": "10.0.0.1", "IsHeadNode": True, "stats": s}])
    text = "\n".join(lines)
    assert 'ray_node_gpus_utilization{ip="10.0.0.1"' in text and 'GpuIndex="0"' in text
    assert any(l.startswith("ray_node_gram_used") and l.endswith(str(float(5 << 30))) for l in lines)
    assert any(l.startswith("ray_node_gram_available") and l.endswith(str(float(283 << 30))) for l in lines)
    assert any(l.startswith("ray_node_mem_total") for l in lines)
    # amdsmi unusable -> sysfs fallback (no AMD GPU here: empty, no error)
    class _Dead:
        ok = False
    monkeypatch.setattr(reporter, "_SMI", _Dead())
    assert isinstance(reporter.sample_gpus(), list)


def _cli(*args, env):
    p = subprocess.run([sys.executable, "-m", "cluster_anywhere_amd", *args], env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


def _get(url):
    with urllib.request.urlopen(url, timeout=60) as r:
        return r.read().decode()


def _req(url, method, body=None):
    data = None if body is None else json.dumps(body).encode()
    r = urllib.request.Request(url, data=data, method=method, headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(r, timeout=300) as resp:
        return resp.status, resp.read().decode()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def cluster(tmp_path_factory):
    t = tmp_path_factory.mktemp("rep")
    (t / "restapp.py").write_text(textwrap.dedent('''
        from cluster_anywhere_amd import serve

        @serve.deployment
        class Echo:
            def __init__(self, tag="x"):
                self.tag = tag

            def __call__(self, request):
                return {"tag": self.tag}

        def build(args):
            return Echo.bind(args.get("tag", "x"))
        '''))
    # a sitecustomize that installs the fake amdsmi sampler in every node process
    (t / "sitecustomize.py").write_text(textwrap.dedent('''
        import os
        if os.environ.get("CAAMD_TEST_FAKE_SMI") == "1":
            try:
                from cluster_anywhere_amd.dashboard import reporter as _r
                class _F:
                    ok = True
                    def sample(self):
                        return [{"index": 0, "name": "AMD Instinct MI355X", "utilization_gpu": 55.0,
                                 "memory_used": 3 << 30, "memory_total": 288 << 30}]
                _r._SMI = _F()
            except Exception:
                pass
        '''))
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([str(t), ROOT]), CAAMD_TEST_FAKE_SMI="1",
               CAAMD_REPORTER_INTERVAL_S="0.3")
    tmp = str(t / "caamd")
    _cli("start", "--head", "--port", "0", "--num-cpus", "4", "--dashboard-port", "0", "--temp-dir", tmp, env=env)
    info = json.load(open(os.path.join(tmp, "head.json")))
    _cli("start", "--address", info["address"], "--num-cpus", "1", "--num-gpus", "0", "--temp-dir", tmp, env=env)
    yield t, tmp, info, env
    _cli("stop", "--temp-dir", tmp, env=env)


def test_every_node_reports_and_metrics_export(cluster):
    t, tmp, info, env = cluster
    dash = info["dashboard"]
    deadline = time.time() + 60
    while True:
        nodes = json.loads(_get(dash + "/api/v0/nodes"))["data"]["result"]["result"]
        if len(nodes) == 2 and all(n.get("stats") for n in nodes):
            break
        assert time.time() < deadline, nodes
        time.sleep(0.3)
    for n in nodes:
        st = n["stats"]
        assert st["cpu_count"] >= 1 and st["mem_total"] > 0
        assert st["gpus"][0]["utilization_gpu"] == 55.0
    assert sum(bool(n.get("IsHeadNode")) for n in nodes) == 1
    m = _get(dash + "/metrics")
    assert m.count("ray_node_gpus_utilization{") == 2  # one GPU per node
    assert 'IsHeadNode="true"' in m and 'IsHeadNode="false"' in m
    assert "ray_node_cpu_utilization{" in m and "ray_node_mem_used{" in m


def test_serve_rest_round_trip(cluster):
    t, tmp, info, env = cluster
    dash = info["dashboard"]
    url = dash + "/api/serve/applications/"
    port = _free_port()
    cfg = {"http_options": {"port": port},
           "applications": [{"name": "rest", "route_prefix": "/r", "import_path": "restapp:build",
                             "args": {"tag": "hello"}}]}
    code, _ = _req(url, "PUT", cfg)
    assert code == 200
    d = json.loads(_get(url))
    app = d["applications"]["rest"]
    assert app["status"] == "RUNNING" and app["route_prefix"] == "/r"
    assert app["deployed_app_config"]["import_path"] == "restapp:build"
    assert json.loads(_get(f"http://127.0.0.1:{port}/r"))["tag"] == "hello"
    # the CLI against the dashboard address
    (t / "cfg.yaml").write_text(yaml.safe_dump({"http_options": {"port": port}, "applications": [
        {"name": "rest2", "route_prefix": "/r2", "import_path": "restapp:build", "args": {"tag": "cli"}}]}))
    _cli("serve", "deploy", str(t / "cfg.yaml"), "--address", dash, env=env)
    st = yaml.safe_load(_cli("serve", "status", "--address", dash, env=env))
    assert set(st["applications"]) == {"rest2"}  # declarative: "rest" was removed
    assert json.loads(_get(f"http://127.0.0.1:{port}/r2"))["tag"] == "cli"
    code, _ = _req(url, "DELETE")
    assert code == 200
    assert json.loads(_get(url))["applications"] == {}
    # a bad config is a 400, not a crash of the agent
    bad = {"applications": [{"name": "x", "route_prefix": "no-slash", "import_path": "restapp:build"}]}
    try:
        _req(url, "PUT", bad)
        assert False, "expected HTTP 400"
    except urllib.error.HTTPError as e:
        assert e.code == 400
    assert json.loads(_get(url))["applications"] == {}


def test_serve_agent_request_times_out_and_restarts():
    """a hung agent answers 504 within the client's timeout (the lock is
    not held forever) and is replaced on the next request."""
    import subprocess
    import sys
    import time

    from cluster_anywhere_amd.dashboard.serve_agent import ServeAgentClient

    c = ServeAgentClient("unused", timeout_s=0.5)
    hung = subprocess.Popen([sys.executable, "-c", "import sys, time; sys.stdin.readline(); time.sleep(60)"],
                            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)
    c.proc = hung
    started = []
    c._ensure = lambda: started.append(1) if c.proc is None else None
    t0 = time.time()
    r = c.request("status")
    assert r["status"] == 504 and time.time() - t0 < 5
    assert hung.poll() is not None  # killed
    assert c.proc is None
