"""Head restart keeps the node running (reference: raylets and core workers
re-register with a restarted GCS, src/ray/gcs/gcs_server/gcs_server.cc:182
DoStart(GcsInitData); GCS pubsub tells subscribers about actor / node changes).

A standalone head with durable tables is SIGKILLed mid-workload and restarted on
the same ``--gcs-storage``. Its object-store arena, the actor and task workers and
the driver all outlive it: they reconnect, re-register and replay what was in
flight, so an actor keeps its in-memory state, a task that was running finishes
and delivers its result, objects in the arena stay readable, and new work runs."""
import json
import os
import signal
import subprocess
import sys
import time

import numpy as np
import pytest

import cluster_anywhere_amd as ray

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _start_head(tmp, store, log):
    env = dict(os.environ, PYTHONPATH=ROOT, CAAMD_HEAD_RECONNECT_S="60", CAAMD_GCS_REATTACH_S="4")
    info_path = os.path.join(tmp, "head.json")
    f = open(log, "ab")
    p = subprocess.Popen([sys.executable, "-m", "cluster_anywhere_amd.core.head_main", "--port", "0",
                          "--num-cpus", "4", "--num-gpus", "0", "--include-dashboard", "false",
                          "--temp-dir", tmp, "--gcs-storage", store, "--object-store-memory", str(256 << 20)],
                         env=env, stdout=f, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                         start_new_session=True)
    deadline = time.time() + 90
    while time.time() < deadline:
        try:
            with open(info_path) as fh:
                info = json.load(fh)
            if info.get("pid") == p.pid:
                return p, info
        except (OSError, ValueError):
            pass
        assert p.poll() is None, open(log).read()[-3000:]
        time.sleep(0.1)
    raise TimeoutError("head did not start")


@ray.remote
class Counter:
    def __init__(self, start):
        self.n = start

    def incr(self):
        self.n += 1
        return self.n

    def pid(self):
        return os.getpid()


@ray.remote
def sq(x):
    return x * x


@ray.remote
def slow(t, v):
    time.sleep(t)
    return v


def test_head_sigkill_and_restart_keeps_workers(tmp_path):
    tmp = str(tmp_path / "caamd")
    store = str(tmp_path / "gcs" / "tables.log")
    log = str(tmp_path / "head.log")
    head, info = _start_head(tmp, store, log)
    head2 = None
    try:
        ray.init(address=info["address"])
        c = Counter.options(name="ctr", namespace="ft").remote(5)
        assert ray.get(c.incr.remote()) == 6
        actor_pid = ray.get(c.pid.remote())
        big = ray.put(np.arange(300_000, dtype=np.int64))
        assert ray.get(sq.remote(3)) == 9
        running = slow.remote(3.0, "finished")  # runs across the head's death
        time.sleep(0.8)
        os.kill(head.pid, signal.SIGKILL)
        head.wait()
        head2, info2 = _start_head(tmp, store, log)
        assert info2["address"] == info["address"] and info2["session_dir"] == info["session_dir"]
        # the actor process survived and is re-attached: same process, same state
        c2 = ray.get_actor("ctr", namespace="ft")
        assert ray.get(c2.pid.remote(), timeout=60) == actor_pid
        assert ray.get(c2.incr.remote(), timeout=60) == 7
        # the task that was running when the head died delivers its result once
        assert ray.get(running, timeout=60) == "finished"
        # objects in the node's arena are still there
        assert int(ray.get(big, timeout=60).sum()) == int(np.arange(300_000).sum())
        # and new work runs
        assert ray.get([sq.remote(i) for i in range(20)], timeout=60) == [i * i for i in range(20)]
        d = Counter.remote(0)
        assert ray.get(d.incr.remote(), timeout=60) == 1
        from cluster_anywhere_amd.core.api import _state

        stats = _state("reattach_stats")
        assert stats["actors"] >= 1 and stats["workers"] >= 1 and stats["drivers"] >= 1, stats
    finally:
        ray.shutdown()
        for p in (head, head2):
            if p is not None and p.poll() is None:
                p.send_signal(signal.SIGTERM)
                try:
                    p.wait(30)
                except subprocess.TimeoutExpired:
                    p.kill()


def test_pubsub_actor_and_node_events(tmp_path):
    """Actor state changes (ALIVE -> DEAD, with the death cause) and node joins /
    deaths are pushed to subscribers (reference: src/ray/pubsub/publisher.h:297)."""
    import threading

    from cluster_anywhere_amd.util import state

    ctx = ray.init(num_cpus=2, _listen_tcp="127.0.0.1:0")
    try:
        events = []
        cv = threading.Condition()

        def on(kind):
            def cb(key, info):
                with cv:
                    events.append((kind, key, info))
                    cv.notify_all()
            return cb

        state.subscribe("actor", on("actor"))
        state.subscribe("node", on("node"))
        a = Counter.remote(0)
        assert ray.get(a.incr.remote()) == 1

        def wait_for(pred, t=30):
            deadline = time.time() + t
            with cv:
                while not any(pred(e) for e in events):
                    left = deadline - time.time()
                    assert left > 0, events
                    cv.wait(left)

        wait_for(lambda e: e[0] == "actor" and e[1] == a._actor_id and e[2]["state"] == "ALIVE")
        ray.kill(a)
        wait_for(lambda e: e[0] == "actor" and e[1] == a._actor_id and e[2]["state"] == "DEAD")
        # a node joins and dies
        addr = ctx["gcs_address"]
        env = dict(os.environ, PYTHONPATH=ROOT)
        agent = subprocess.Popen([sys.executable, "-m", "cluster_anywhere_amd.core.node_agent", "--address", addr,
                                  "--num-cpus", "1", "--num-gpus", "0", "--object-store-memory", str(64 << 20)],
                                 env=env)
        try:
            wait_for(lambda e: e[0] == "node" and e[2]["state"] == "ALIVE", 60)
            agent.kill()
            agent.wait()
            wait_for(lambda e: e[0] == "node" and e[2]["state"] == "DEAD", 60)
        finally:
            if agent.poll() is None:
                agent.kill()
    finally:
        ray.shutdown()


@ray.remote
def getenv(k):
    return os.environ.get(k)


def test_head_restart_keeps_env_pools_and_leases(tmp_path):
    """Workers started for a runtime env re-register into their own env's pool, and
    leases held across the restart are restored whichever of the driver or the
    leased worker re-registers first (ADVICE r3 on head.py:2116 / :2186)."""
    tmp = str(tmp_path / "caamd")
    store = str(tmp_path / "gcs" / "tables.log")
    log = str(tmp_path / "head.log")
    head, info = _start_head(tmp, store, log)
    head2 = None
    try:
        ray.init(address=info["address"])
        envd = getenv.options(runtime_env={"env_vars": {"CAAMD_T_FOO": "bar"}})
        assert ray.get(envd.remote("CAAMD_T_FOO")) == "bar"
        assert ray.get(getenv.remote("CAAMD_T_FOO")) is None
        burst = [slow.remote(2.0, i) for i in range(6)]  # leased workers busy across the restart
        time.sleep(0.6)
        os.kill(head.pid, signal.SIGKILL)
        head.wait()
        head2, _ = _start_head(tmp, store, log)
        assert ray.get(burst, timeout=120) == list(range(6))
        plain = ray.get([getenv.remote("CAAMD_T_FOO") for _ in range(40)], timeout=90)
        assert all(v is None for v in plain), plain
        assert ray.get(envd.remote("CAAMD_T_FOO"), timeout=60) == "bar"
    finally:
        ray.shutdown()
        for p in (head, head2):
            if p is not None and p.poll() is None:
                p.send_signal(signal.SIGTERM)
                try:
                    p.wait(30)
                except subprocess.TimeoutExpired:
                    p.kill()
