"""``_system_config["object_spilling_config"]`` (reference:
python/ray/_private/external_storage.py:272 FileSystemStorage with several
directories, :481 the smart_open URI storage, :660 setup_external_storage;
tests modelled on python/ray/tests/test_object_spilling.py
test_spill_objects_automatically / test_multiple_directories)."""
import glob
import json
import os

import numpy as np
import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd.core.external_storage import (FileSystemStorage, URIStorage, parse_config,
                                                        setup_external_storage)

MB = 1 << 20


@ray.remote
def total(a):
    return float(a.sum())


def _fill_and_check(n=8):
    # 128 MiB store, 8 x 32 MiB objects: the early ones are spilled
    refs = [ray.put(np.full(4 * MB, i, dtype=np.float64)) for i in range(n)]
    # restored as task arguments (the workers map them from the store again)
    got = ray.get([total.remote(r) for r in refs])
    assert got == [float(i * 4 * MB) for i in range(n)]
    for i, r in enumerate(refs):
        v = ray.get(r)
        assert v[0] == i and v[-1] == i
    return refs


def test_parse_and_storage_units(tmp_path):
    assert parse_config(None) is None and parse_config("") is None
    cfg = parse_config(json.dumps({"type": "filesystem", "params": {"directory_path": str(tmp_path)}}))
    assert cfg["type"] == "filesystem"
    with pytest.raises(ValueError):
        parse_config({"params": {}})
    with pytest.raises(ValueError):
        setup_external_storage({"type": "bogus"}, "s", str(tmp_path))
    fs = FileSystemStorage([str(tmp_path / "a"), str(tmp_path / "b")], "sess")
    urls = [fs.spill(f"k{i}", memoryview(bytes([i]) * 100)) for i in range(4)]
    assert [os.path.dirname(u) for u in urls] == [fs.dirs[0], fs.dirs[1], fs.dirs[0], fs.dirs[1]]
    assert fs.restore(urls[3]) == bytes([3]) * 100
    fs.delete(urls[3])
    assert not os.path.exists(urls[3])
    us = URIStorage(["memory://caamd_unit/x", f"file://{tmp_path}/u"], "sess")
    u0, u1 = us.spill("o0", b"abc"), us.spill("o1", memoryview(b"defg"))
    assert us.restore(u0) == b"abc" and us.restore(u1) == b"defg"
    assert os.path.exists(u1.split("|", 1)[1])
    us.destroy()


def test_spill_round_robin_over_two_directories(tmp_path):
    d1, d2 = str(tmp_path / "spill1"), str(tmp_path / "spill2")
    ray.init(num_cpus=2, object_store_memory=128 * MB, _system_config={
        "object_spilling_config": json.dumps({"type": "filesystem", "params": {"directory_path": [d1, d2]}})})
    try:
        refs = _fill_and_check()
        # objects were spilled into BOTH directories (restored ones are deleted again,
        # so look at what is spilled after one more round of pressure)
        extra = [ray.put(np.full(4 * MB, 100 + i, dtype=np.float64)) for i in range(6)]
        f1 = glob.glob(os.path.join(d1, "caamd_spilled_objects_*", "*"))
        f2 = glob.glob(os.path.join(d2, "caamd_spilled_objects_*", "*"))
        assert f1 and f2, (f1, f2)
        assert all(ray.get(r)[0] == 100 + i for i, r in enumerate(extra))
        del refs, extra
    finally:
        ray.shutdown()
    # the session's spill directories are removed at shutdown
    assert not glob.glob(os.path.join(d1, "caamd_spilled_objects_*", "*"))


def test_spill_to_fsspec_memory_uri(monkeypatch):
    import fsspec

    monkeypatch.setenv("CAAMD_HEAD_IN_PROCESS", "1")  # the memory filesystem lives in the head's process
    ray.init(num_cpus=2, object_store_memory=128 * MB, _system_config={
        "object_spilling_config": {"type": "smart_open", "params": {"uri": "memory://caamd_spill_test"}}})
    try:
        refs = [ray.put(np.full(4 * MB, i, dtype=np.float64)) for i in range(8)]
        mem = fsspec.filesystem("memory")
        spilled = [p for p in mem.find("/caamd_spill_test")]
        assert spilled, "nothing was spilled to memory://"
        got = ray.get([total.remote(r) for r in refs])
        assert got == [float(i * 4 * MB) for i in range(8)]
    finally:
        ray.shutdown()


def test_bad_spilling_config_fails_init():
    with pytest.raises(ValueError):
        ray.init(num_cpus=1, _system_config={"object_spilling_config": {"type": "nope", "params": {}}})
    assert not ray.is_initialized()
