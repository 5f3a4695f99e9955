"""util.collective (gloo groups between actors), util.multiprocessing.Pool,
internal KV, and the OOM killer (reference: python/ray/util/collective/tests/,
python/ray/tests/test_multiprocessing.py, test_memory_pressure.py)."""
import os
import time

import numpy as np
import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd.exceptions import OutOfMemoryError


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4, object_store_memory=256 << 20)
    yield
    ray.shutdown()


@ray.remote
class Member:
    def __init__(self, rank=None, world=None, name=None):
        import cluster_anywhere_amd.util.collective as col

        if name is not None:
            col.init_collective_group(world, rank, backend="gloo", group_name=name)

    def allreduce(self, v, name):
        import torch

        import cluster_anywhere_amd.util.collective as col

        t = torch.full((4,), float(v))
        col.allreduce(t, group_name=name)
        return t.tolist()

    def numpy_allreduce_max(self, v, name):
        import cluster_anywhere_amd.util.collective as col

        a = np.full(3, float(v), dtype=np.float32)
        col.allreduce(a, group_name=name, op=col.ReduceOp.MAX)
        return a.tolist()

    def bcast(self, v, name):
        import torch

        import cluster_anywhere_amd.util.collective as col

        t = torch.full((2,), float(v))
        col.broadcast(t, src_rank=1, group_name=name)
        return t.tolist()

    def gather_scatter(self, rank, name):
        import torch

        import cluster_anywhere_amd.util.collective as col

        w = col.get_collective_group_size(name)
        outs = [torch.zeros(2) for _ in range(w)]
        col.allgather(outs, torch.full((2,), float(rank)), group_name=name)
        rs = torch.zeros(2)
        col.reducescatter(rs, [torch.full((2,), float(rank + i)) for i in range(w)], group_name=name)
        return [o.tolist() for o in outs], rs.tolist(), col.get_rank(name)

    def p2p(self, rank, name):
        import torch

        import cluster_anywhere_amd.util.collective as col

        t = torch.arange(3, dtype=torch.float32) * (rank + 1)
        if rank == 0:
            col.send(t, 1, group_name=name)
            return None
        col.recv(t, 0, group_name=name)
        return t.tolist()

    def destroy(self, name):
        import cluster_anywhere_amd.util.collective as col

        col.destroy_collective_group(name)
        return col.is_group_initialized(name)


def test_internal_kv(cluster):
    from cluster_anywhere_amd.experimental import internal_kv as kv

    assert kv._internal_kv_put("a", "1") is False
    assert kv._internal_kv_put("a", "2", overwrite=False) is True
    assert kv._internal_kv_get("a") == b"1"
    kv._internal_kv_put("ab", b"x", namespace="n")
    assert kv._internal_kv_get("ab") is None
    assert sorted(kv._internal_kv_list("a", namespace="n")) == [b"ab"]
    assert kv._internal_kv_exists("a")
    assert kv._internal_kv_del("a") == 1
    assert not kv._internal_kv_exists("a")


def test_collective_init_inside_actors(cluster):
    ms = [Member.remote(r, 3, "g1") for r in range(3)]
    out = ray.get([m.allreduce.remote(r + 1, "g1") for r, m in enumerate(ms)])
    assert out == [[6.0] * 4] * 3
    out = ray.get([m.numpy_allreduce_max.remote(r, "g1") for r, m in enumerate(ms)])
    assert out == [[2.0] * 3] * 3
    assert ray.get([m.bcast.remote(r * 10, "g1") for r, m in enumerate(ms)]) == [[10.0, 10.0]] * 3
    res = ray.get([m.gather_scatter.remote(r, "g1") for r, m in enumerate(ms)])
    for r, (gathered, rs, rank) in enumerate(res):
        assert gathered == [[0.0, 0.0], [1.0, 1.0], [2.0, 2.0]]
        assert rank == r
        # reducescatter: rank r gets sum_j (j + r)
        assert rs == [float(sum(j + r for j in range(3)))] * 2
    assert ray.get([m.destroy.remote("g1") for m in ms]) == [False] * 3


def test_collective_declarative_group(cluster):
    import cluster_anywhere_amd.util.collective as col

    ms = [Member.remote() for _ in range(2)]
    col.create_collective_group(ms, 2, [1, 0], backend="gloo", group_name="g2")
    with pytest.raises(RuntimeError):
        col.create_collective_group(ms, 2, [0, 1], backend="gloo", group_name="g2")
    out = ray.get([m.allreduce.remote(3, "g2") for m in ms])
    assert out == [[6.0] * 4] * 2
    # actor 1 holds rank 0 -> it sends; actor 0 (rank 1) receives
    res = ray.get([ms[1].p2p.remote(0, "g2"), ms[0].p2p.remote(1, "g2")])
    assert res == [None, [0.0, 1.0, 2.0]]


def _sq(x):
    return x * x


def _add(a, b):
    return a + b


def _boom(x):
    if x == 3:
        raise ValueError("three")
    return x


_INIT = {}


def _init(v):
    _INIT["v"] = v


def _read_init(_):
    return _INIT.get("v")


def test_multiprocessing_pool(cluster):
    from cluster_anywhere_amd.util.multiprocessing import Pool

    with Pool(2) as p:
        assert p.map(_sq, range(20)) == [i * i for i in range(20)]
        assert p.starmap(_add, [(1, 2), (3, 4)]) == [3, 7]
        assert p.apply(_add, (5, 6)) == 11
        r = p.apply_async(_sq, (7,))
        assert r.get(timeout=30) == 49 and r.successful()
        assert list(p.imap(_sq, range(5))) == [0, 1, 4, 9, 16]
        assert sorted(p.imap_unordered(_sq, range(5), chunksize=2)) == [0, 1, 4, 9, 16]
        with pytest.raises(ValueError, match="three"):
            p.map(_boom, range(5))
        got = []
        p.map_async(_sq, [2, 3], callback=got.append).wait(30)
        time.sleep(0.1)
        assert got == [[4, 9]]
    with Pool(2, initializer=_init, initargs=(42,), maxtasksperchild=1) as p:
        assert p.map(_read_init, range(6), chunksize=1) == [42] * 6


def _slow_sq(x):
    time.sleep(0.2)
    return x * x


def test_pool_reruns_chunks_of_a_killed_process(cluster):
    """A pool process that dies mid-map (OOM kill, crash) costs a re-run of its
    chunks on a fresh actor, not the map (ActorDiedError under load, round 3)."""
    from cluster_anywhere_amd.util.multiprocessing import Pool

    with Pool(2) as p:
        r = p.map_async(_slow_sq, range(12), chunksize=1)
        time.sleep(0.3)
        ray.kill(p._actors[0][0])
        assert r.get(timeout=120) == [i * i for i in range(12)]
        assert sorted(p.imap_unordered(_sq, range(6))) == [i * i for i in range(6)]


@ray.remote(max_retries=0)
def _hog(path):
    with open(path, "w") as f:
        f.write("0.99")
    time.sleep(60)
    return "survived"


@ray.remote(max_retries=1)
def _hog_then_ok(path, marker):
    if not os.path.exists(marker):
        open(marker, "w").close()
        with open(path, "w") as f:
            f.write("0.99")
        time.sleep(60)
        return "survived"
    with open(path, "w") as f:
        f.write("0.10")
    return "retried"


def test_oom_killer(tmp_path, monkeypatch):
    path = tmp_path / "usage"
    path.write_text("0.10")
    monkeypatch.setenv("CAAMD_MEMORY_MONITOR_TEST_FILE", str(path))
    monkeypatch.setenv("CAAMD_MEMORY_MONITOR_REFRESH_MS", "100")
    if ray.is_initialized():
        ray.shutdown()
    ray.init(num_cpus=2, object_store_memory=128 << 20)
    try:
        with pytest.raises(OutOfMemoryError):
            ray.get(_hog.remote(str(path)), timeout=30)
        path.write_text("0.10")
        time.sleep(1.0)
        assert ray.get(_hog_then_ok.remote(str(path), str(tmp_path / "m")), timeout=30) == "retried"
    finally:
        ray.shutdown()

