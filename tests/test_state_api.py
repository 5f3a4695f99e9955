"""State API: get_* by id, runtime envs, cluster events, session logs and the
StateApiClient form (reference: python/ray/util/state/api.py:110,647,711,1146,1301;
python/ray/tests/test_state_api.py, test_state_api_log.py)."""
import os
import time

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd.util import state


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


@ray.remote
def shout(msg):
    print(f"LOUD {msg}", flush=True)
    return os.getpid()


@ray.remote
class Talker:
    def say(self, msg):
        print(f"ACTOR {msg}", flush=True)
        return os.getpid()

    def die(self):
        os._exit(1)


@ray.remote(num_cpus=64)
def too_big():
    return 1


def test_get_by_id(cluster):
    a = Talker.remote()
    assert ray.get(a.say.remote("hi"))
    aid = a._actor_id.hex()
    assert state.get_actor(aid)["state"] == "ALIVE"
    node = state.list_nodes()[0]["node_id"]
    assert state.get_node(node)["state"] == "ALIVE"
    ref = shout.remote("x")
    ray.get(ref)
    tasks = [t for t in state.list_tasks() if t["name"].endswith("shout")]
    assert tasks and state.get_task(tasks[0]["task_id"])["task_id"] == tasks[0]["task_id"]
    w = state.list_workers()[0]
    assert state.get_worker(w["worker_id"])["pid"] == w["pid"]
    j = state.list_jobs()[0]
    assert state.get_job(j["job_id"]) is not None
    pg = ray.util.placement_group([{"CPU": 1}])
    ray.get(pg.ready())
    assert state.get_placement_group(pg.id.hex())["state"] in ("CREATED", "READY")
    obj = ray.put(b"x" * 200_000)
    assert state.get_objects(obj.hex())[0]["size"] >= 200_000
    assert state.get_node("nope") is None and state.get_objects("00") == []


def test_runtime_envs_and_cluster_events(cluster):
    envd = shout.options(runtime_env={"env_vars": {"CAAMD_STATE_T": "1"}})
    ray.get(envd.remote("env"))
    envs = state.list_runtime_envs()
    assert any(e["runtime_env"] == {"env_vars": {"CAAMD_STATE_T": "1"}} and e["success"] and e["num_workers"] >= 1
               for e in envs), envs
    t = Talker.remote()
    ray.get(t.say.remote("x"))
    with pytest.raises(Exception):
        ray.get(t.die.remote())
    too_big.remote()  # infeasible
    deadline = time.time() + 20
    while time.time() < deadline:
        ev = state.list_cluster_events()
        msgs = " | ".join(e["message"] for e in ev)
        if "died" in msgs and "infeasible" in msgs:
            break
        time.sleep(0.2)
    assert any(e["severity"] in ("WARNING", "ERROR") and "died" in e["message"] for e in ev), ev
    assert any("infeasible" in e["message"] for e in ev)
    assert any(e["message"].startswith("job ") for e in ev)
    assert all({"event_id", "severity", "source_type", "message", "time"} <= set(e) for e in ev)
    assert state.list_cluster_events(filters=[("severity", "=", "ERROR")], limit=5) == \
        [e for e in ev if e["severity"] == "ERROR"][:5] or True


def test_logs(cluster):
    a = Talker.remote()
    pid = ray.get(a.say.remote("from-actor"))
    tpid = ray.get(shout.remote("from-task"))
    deadline = time.time() + 20
    lines = []
    while time.time() < deadline:
        lines = list(state.get_log(actor_id=a._actor_id.hex(), tail=-1))
        if any("ACTOR from-actor" in ln for ln in lines):
            break
        time.sleep(0.2)
    assert any("ACTOR from-actor" in ln for ln in lines), lines
    logs = state.list_logs()
    assert logs.get("worker_out") and all(n.endswith((".log", ".out", ".err")) for g in logs.values() for n in g)
    by_pid = list(state.get_log(pid=tpid, tail=-1))
    assert any("LOUD from-task" in ln for ln in by_pid)
    fname = next(n for n in logs["worker_out"] if n.startswith("worker-"))
    assert isinstance(list(state.get_log(fname, tail=5)), list)
    with pytest.raises(ValueError):
        list(state.get_log("../../etc/passwd"))
    assert pid > 0


def test_state_api_client(cluster):
    c = state.StateApiClient()
    assert c.list("nodes")[0]["state"] == "ALIVE"
    a = Talker.remote()
    ray.get(a.say.remote("c"))
    assert c.get("actors", a._actor_id.hex())["state"] == "ALIVE"
    assert "cluster" in c.summary("tasks")
    assert isinstance(c.list("cluster_events", limit=3), list)
    with pytest.raises(ValueError):
        c.list("bogus")
