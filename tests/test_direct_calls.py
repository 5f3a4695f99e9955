"""Direct actor-call transport (core/direct.py): ordering across the head->direct
switch, refs escaping to other processes, nested refs in results, dropping refs
while calls are in flight, actor death with and without task retries, and that
the head is actually off the call path (reference test model:
python/ray/tests/test_actor.py, test_actor_failures.py, test_reference_counting.py)."""
import os
import signal
import time

import numpy as np
import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd.core import context


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=6, include_dashboard=False)
    yield
    ray.shutdown()


@ray.remote
class Log:
    def __init__(self):
        self.items = []

    def add(self, x):
        self.items.append(x)
        return len(self.items)

    def get(self):
        return list(self.items)

    def slow_add(self, x):
        time.sleep(0.05)  # keeps calls queued at the actor when it is killed
        return self.add(x)

    def big(self, n):
        return np.arange(n, dtype=np.int64)

    def nested(self):
        return [ray.put(np.ones(200_000)), ray.put("small")]

    def pid(self):
        return os.getpid()


@ray.remote
def consume(x):
    return int(np.asarray(x).sum()) if not isinstance(x, str) else len(x)


def _direct_client(actor):
    w = context.worker
    dc = w.actor_direct.get(actor._actor_id)
    return dc if dc is not None and not isinstance(dc, tuple) else None


def test_order_preserved_across_switch(cluster):
    a = Log.remote()
    refs = [a.add.remote(i) for i in range(300)]  # early calls may go through the head
    ray.get(refs[-1])
    refs += [a.add.remote(i) for i in range(300, 600)]  # then direct
    assert ray.get(refs) == list(range(1, 601))
    assert ray.get(a.get.remote()) == list(range(600))
    assert _direct_client(a) is not None, "calls should be on the direct transport by now"


def test_results_escape_and_large_objects(cluster):
    a = Log.remote()
    ray.get(a.pid.remote())
    ray.get(a.pid.remote())
    r_small = a.add.remote("x")
    r_big = a.big.remote(300_000)  # > inline limit: lives in the shm store
    # pass the direct-call refs (maybe still running) to other processes
    assert ray.get(consume.remote(r_big)) == int(np.arange(300_000).sum())
    assert ray.get(consume.remote(r_small)) == 1
    assert ray.get(r_big)[-1] == 299_999
    ready, _ = ray.wait([r_small, r_big], num_returns=2, timeout=30)
    assert len(ready) == 2


def test_nested_refs_survive(cluster):
    a = Log.remote()
    ray.get(a.pid.remote())
    inner = ray.get(a.nested.remote())
    time.sleep(0.3)  # the actor's own refs to the nested objects are gone by now
    assert ray.get(inner[0]).sum() == 200_000
    assert ray.get(inner[1]) == "small"
    assert ray.get(consume.remote(inner[0])) == 200_000


def test_drop_refs_in_flight_frees_objects(cluster):
    a = Log.remote()
    ray.get(a.pid.remote())
    for _ in range(5):
        rs = [a.big.remote(50_000) for _ in range(20)]
        del rs  # dropped before completion: decrefs are held until the seal
    ray.get(a.pid.remote())
    w = context.worker
    deadline = time.time() + 10
    while time.time() < deadline and (w.store.used > 10 * 400_000 or w.refs.direct_pending
                                      or w.refs.direct_dropped):
        time.sleep(0.1)  # seal notifications of the dropped calls may still be in flight
    # the store must not keep 100 x 400 KB of orphaned results
    assert w.store.used < 10 * 400_000, w.store.used
    assert not w.refs.direct_pending and not w.refs.direct_dropped


def test_actor_death_without_retries_fails_calls(cluster):
    a = Log.options(max_restarts=0).remote()
    pid = ray.get(a.pid.remote())
    ray.get(a.pid.remote())
    assert _direct_client(a) is not None
    slow = [a.slow_add.remote(i) for i in range(50)]
    os.kill(pid, signal.SIGKILL)
    errors = 0
    for r in slow:
        try:
            ray.get(r, timeout=60)
        except ray.exceptions.RayActorError:
            errors += 1
    assert errors >= 1
    with pytest.raises(ray.exceptions.RayActorError):
        ray.get(a.add.remote(1), timeout=60)


def test_actor_death_with_retries_resubmits(cluster):
    a = Log.options(max_restarts=1, max_task_retries=-1).remote()
    pid = ray.get(a.pid.remote())
    ray.get(a.pid.remote())
    refs = [a.add.remote(i) for i in range(20)]
    os.kill(pid, signal.SIGKILL)
    out = ray.get(refs, timeout=120)
    assert len(out) == 20  # every call completed (some on the restarted actor)
    assert ray.get(a.pid.remote(), timeout=60) != pid


@ray.remote
class SlowLog:
    def __init__(self):
        self.items = []

    def add(self, x):
        time.sleep(0.002)
        self.items.append(x)
        return x

    def stream(self, n):
        self.items.append("gen")
        for i in range(n):
            yield i

    def get(self):
        return list(self.items)


def test_order_direct_generator_direct(cluster):
    """A streaming call (head path) between direct calls must not overtake the
    direct calls sent before it, and later calls must not overtake it."""
    a = SlowLog.remote()
    ray.get(a.add.remote(-1))
    ray.get([a.add.remote(-2) for _ in range(3)])
    first = [a.add.remote(i) for i in range(40)]
    gen = a.stream.options(num_returns="streaming").remote(3)
    later = [a.add.remote(100 + i) for i in range(20)]
    assert [ray.get(r) for r in gen] == [0, 1, 2]
    ray.get(first + later)
    items = ray.get(a.get.remote())[4:]
    assert items == list(range(40)) + ["gen"] + [100 + i for i in range(20)]


def test_calls_after_kill_do_not_reach_actor(cluster):
    """ray.kill drops the caller's direct connection: later calls go through the
    head (ordered after the kill) and fail with ActorDiedError."""
    from cluster_anywhere_amd.exceptions import ActorDiedError, RayActorError

    a = Log.remote()
    for _ in range(50):
        ray.get([a.add.remote(i) for i in range(20)])
        if _direct_client(a) is not None:
            break
    assert _direct_client(a) is not None
    ray.kill(a)
    assert _direct_client(a) is None
    with pytest.raises((ActorDiedError, RayActorError)):
        ray.get(a.add.remote(99), timeout=60)


def test_dropping_last_handle_waits_for_direct_calls(cluster):
    """Dropping the last handle of an actor terminates it only after the calls
    already sent to it have run: the handle's decref (after which the head queues
    __ray_terminate__) is held back until the direct calls are answered, so the
    head-path terminate cannot overtake them (the multiprocessing.Pool
    maxtasksperchild race of round 3)."""
    import gc

    @ray.remote
    class Slow:
        def work(self, t, v):
            time.sleep(t)
            return v

    for _ in range(3):
        a = Slow.remote()
        assert ray.get(a.work.remote(0, -1)) == -1  # on the direct path now
        refs = [a.work.remote(0.05, i) for i in range(8)]
        del a
        gc.collect()
        assert ray.get(refs, timeout=60) == list(range(8))
