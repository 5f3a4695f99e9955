"""Dashboard UI and log endpoints (reference: python/ray/dashboard/client + the
logs module), exercised through the ASGI app with a fake state source."""
from starlette.testclient import TestClient

from cluster_anywhere_amd.dashboard import build_app
from cluster_anywhere_amd.dashboard.job_manager import JobManager


def _state(what, arg=None):
    return {"cluster_resources": {"CPU": 8.0, "GPU": 8.0, "node:127.0.0.1": 1.0},
            "available_resources": {"CPU": 6.0, "GPU": 8.0},
            "nodes": [{"NodeID": "ab" * 16, "Alive": True, "NodeManagerAddress": "127.0.0.1",
                       "Resources": {"CPU": 8.0}, "Labels": {}}],
            "actors": [{"actor_id": "1" * 32, "class_name": "A", "state": "ALIVE"}],
            "tasks": [], "objects": [], "workers": [], "placement_groups": [], "events": []}[what]


def _client(tmp_path):
    sess = tmp_path / "session"
    sess.mkdir()
    (sess / "worker-1.log").write_text("".join(f"line {i}\n" for i in range(50)))
    (sess / "secret.txt").write_text("no")
    jobs = JobManager("unused", str(tmp_path / "jobs"))
    return TestClient(build_app(_state, jobs, str(sess)))


def test_ui_page_and_rest(tmp_path):
    c = _client(tmp_path)
    r = c.get("/")
    assert r.status_code == 200 and "cluster_anywhere_amd" in r.text and "/api/cluster_status" in r.text
    st = c.get("/api/cluster_status").json()["data"]["clusterStatus"]
    assert st["total"]["CPU"] == 8.0 and st["available"]["CPU"] == 6.0
    actors = c.get("/api/v0/actors").json()["data"]["result"]["result"]
    assert actors[0]["class_name"] == "A"


def test_log_listing_and_tail(tmp_path):
    c = _client(tmp_path)
    files = c.get("/api/v0/logs").json()["files"]
    assert [f["name"] for f in files] == ["worker-1.log"]
    d = c.get("/api/v0/logs/file", params={"name": "worker-1.log", "lines": 3}).json()
    assert d["text"] == "line 47\nline 48\nline 49\n"
    # no path traversal out of the session directory
    assert c.get("/api/v0/logs/file", params={"name": "../jobs"}).status_code == 404
    assert c.get("/api/v0/logs/file", params={"name": "/etc/passwd"}).status_code == 404
