"""Head / GCS fault tolerance: the durable table log (native GcsStore) and a head
restarted on the same storage restoring KV, functions, jobs, detached actors and
detached placement groups (reference: GCS FT with an external store,
src/ray/gcs/store_client/redis_store_client.h, gcs_init_data.cc)."""
import os
import signal
import time

import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import _native


def test_gcs_store_replay_torn_tail_and_compaction(tmp_path):
    p = str(tmp_path / "gcs.log")
    s = _native.GcsStore(p)
    s.put("kv", b"a", b"1")
    s.put("kv", b"b", b"2")
    s.put("kv", b"a", b"3")
    assert s.delete("kv", b"b") and not s.delete("kv", b"zz")
    s.put("actor", b"\x00\x01", b"x" * 1000)
    s.clear_table("actor")
    del s
    s = _native.GcsStore(p)
    assert s.items("kv") == [(b"a", b"3")]
    assert s.items("actor") == [] and s.tables() == ["kv"]
    assert s.records_replayed == 6  # 4 puts, 1 delete, 1 clear (a miss writes nothing)
    # a crash mid-append leaves a torn record: replay drops it and truncates the file
    size = os.path.getsize(p)
    with open(p, "ab") as f:
        f.write(b"GCS1\x01\x02\x00\x00\x00partial")
    s = _native.GcsStore(p)
    assert s.items("kv") == [(b"a", b"3")] and s.torn_bytes_dropped > 0
    assert os.path.getsize(p) == size
    # overwrite churn is compacted away once dead records dominate
    for i in range(3000):
        s.put("kv", b"hot", os.urandom(700))
    assert s.log_bytes < 3 * 1024 * 1024, s.log_bytes
    last = s.get("kv", b"hot")
    s.compact()
    s2 = _native.GcsStore(p)
    assert s2.get("kv", b"hot") == last and s2.get("kv", b"a") == b"3"
    assert s2.log_bytes == s2.live_bytes


def _head_pid():
    from cluster_anywhere_amd.core import api

    return api._head_proc[0].pid if getattr(api, "_head_proc", None) is not None else None


@ray.remote
class Counter:
    def __init__(self, start):
        self.n = start

    def incr(self):
        self.n += 1
        return self.n


def test_gcs_store_failed_append_does_not_poison_later_records(tmp_path):
    """A short write (ENOSPC/EIO mid-record) is cut back off the log, so records
    appended after it survive a restart (replay stopped at the partial
    record and dropped everything behind it)."""
    p = str(tmp_path / "gcs.log")
    s = _native.GcsStore(p)
    s.put("kv", b"a", b"1")
    size = os.path.getsize(p)
    s._inject_write_fault(7)
    with pytest.raises(RuntimeError):
        s.put("kv", b"lost", b"x" * 100)
    assert os.path.getsize(p) == size and s.log_bytes == size
    s.put("kv", b"c", b"3")
    del s
    s = _native.GcsStore(p)
    assert sorted(s.items("kv")) == [(b"a", b"1"), (b"c", b"3")]
    assert s.torn_bytes_dropped == 0


@pytest.mark.parametrize("crash", [False, True])
def test_head_restart_restores_gcs_tables(tmp_path, crash):
    from cluster_anywhere_amd.experimental import internal_kv
    from cluster_anywhere_amd.util import placement_group, remove_placement_group
    from cluster_anywhere_amd.util.placement_group import get_placement_group, placement_group_table

    store = str(tmp_path / "gcs" / "tables.log")
    ray.init(num_cpus=4, _gcs_storage=store)
    try:
        internal_kv._internal_kv_put(b"model_uri", b"s3://bucket/ckpt-7")
        internal_kv._internal_kv_put(b"gone", b"x")
        internal_kv._internal_kv_del(b"gone")
        c = Counter.options(name="ctr", namespace="svc", lifetime="detached").remote(10)
        assert ray.get(c.incr.remote()) == 11
        tmp = Counter.options(name="tmp", namespace="svc").remote(0)  # not detached: not restored
        assert ray.get(tmp.incr.remote()) == 1
        pg = placement_group([{"CPU": 1}], name="keep", lifetime="detached")
        ray.get(pg.ready())
        pg2 = placement_group([{"CPU": 1}], name="dropped", lifetime="detached")
        ray.get(pg2.ready())
        remove_placement_group(pg2)
        dead = Counter.options(name="dead", namespace="svc", lifetime="detached").remote(0)
        ray.get(dead.incr.remote())
        ray.kill(dead)
        time.sleep(2.5)  # the head's health pass drops the killed detached actor's record
        if crash:
            pid = _head_pid()
            assert pid is not None
            os.kill(pid, signal.SIGKILL)  # the head dies without any shutdown path
            time.sleep(0.5)
    finally:
        ray.shutdown()

    ray.init(num_cpus=4, _gcs_storage=store)
    try:
        assert internal_kv._internal_kv_get(b"model_uri") == b"s3://bucket/ckpt-7"
        assert internal_kv._internal_kv_get(b"gone") is None
        c2 = ray.get_actor("ctr", namespace="svc")
        assert c2._actor_id == c._actor_id
        # the worker died with the old head: state restarts from __init__ (like an actor restart)
        assert ray.get(c2.incr.remote()) == 11
        with pytest.raises(ValueError):
            ray.get_actor("tmp", namespace="svc")
        with pytest.raises(ValueError):
            ray.get_actor("dead", namespace="svc")
        keep = get_placement_group("keep")
        deadline = time.time() + 30
        while placement_group_table(keep)["state"] != "CREATED" and time.time() < deadline:
            time.sleep(0.1)
        assert placement_group_table(keep)["state"] == "CREATED"
        with pytest.raises(ValueError):
            get_placement_group("dropped")
        ray.kill(c2)
    finally:
        ray.shutdown()
