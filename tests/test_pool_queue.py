"""ActorPool and Queue semantics (reference test model: python/ray/tests/
test_actor_pool.py, test_queue.py): ordering, backlog, mixing ordered and
unordered consumption, timeouts, membership, capacity, blocking, batches."""
import threading
import time

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd.util import ActorPool
from cluster_anywhere_amd.util.queue import Empty, Full, Queue


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=6, include_dashboard=False)
    yield
    ray.shutdown()


@ray.remote
class Worker:
    def f(self, x):
        time.sleep(x[1])
        return x[0]


def test_pool_ordered_with_backlog(cluster):
    pool = ActorPool([Worker.remote() for _ in range(2)])
    # later items finish first; map() must still return submission order
    vals = [(i, 0.3 - 0.05 * i) for i in range(6)]
    assert list(pool.map(lambda a, v: a.f.remote(v), vals)) == list(range(6))
    assert not pool.has_next()


def test_pool_unordered_and_mixed(cluster):
    pool = ActorPool([Worker.remote() for _ in range(3)])
    for v in [(0, 0.4), (1, 0.0), (2, 0.0), (3, 0.0)]:
        pool.submit(lambda a, v: a.f.remote(v), v)
    first = pool.get_next_unordered()
    assert first in (1, 2, 3)
    rest = []
    while pool.has_next():
        rest.append(pool.get_next())
    # ordered consumption skips what was already taken
    assert sorted([first] + rest) == [0, 1, 2, 3] and len(rest) == 3
    assert rest[0] == 0


def test_pool_timeout_and_membership(cluster):
    a, b = Worker.remote(), Worker.remote()
    pool = ActorPool([a])
    pool.submit(lambda w, v: w.f.remote(v), (7, 1.0))
    with pytest.raises(TimeoutError):
        pool.get_next(timeout=0.05)
    assert pool.get_next() == 7
    assert pool.has_free()
    idle = pool.pop_idle()
    assert idle is a and not pool.has_free()
    pool.push(b)
    with pytest.raises(ValueError):
        pool.push(b)
    assert list(pool.map_unordered(lambda w, v: w.f.remote(v), [(1, 0), (2, 0)])) in ([1, 2], [2, 1])
    with pytest.raises(StopIteration):
        pool.get_next()


def test_queue_fifo_capacity_batches(cluster):
    q = Queue(maxsize=3)
    q.put_nowait_batch([1, 2])
    q.put(3)
    assert q.full() and len(q) == 3
    with pytest.raises(Full):
        q.put_nowait(4)
    with pytest.raises(Full):
        q.put(4, timeout=0.05)
    with pytest.raises(Full):
        q.put_nowait_batch([9, 9])  # all-or-nothing
    assert q.get_nowait_batch(2) == [1, 2]
    with pytest.raises(Empty):
        q.get_nowait_batch(5)
    assert q.get() == 3
    assert q.empty()
    with pytest.raises(Empty):
        q.get(timeout=0.05)
    with pytest.raises(ValueError):
        q.get(timeout=-1)


def test_queue_blocking_handoff(cluster):
    q = Queue()
    got = []
    t = threading.Thread(target=lambda: got.append(q.get(timeout=10)))
    t.start()
    time.sleep(0.2)
    q.put("x")
    t.join(10)
    assert got == ["x"]

    @ray.remote
    def producer(q, n):
        for i in range(n):
            q.put(i)
        return n

    ref = producer.remote(q, 5)
    assert [q.get(timeout=10) for _ in range(5)] == list(range(5))
    assert ray.get(ref) == 5
    q.shutdown()
