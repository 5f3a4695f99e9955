"""Client mode ``init("ray://host:port")`` against a standalone head process
(reference: python/ray/util/client/, tests/test_client*.py). The client maps no
shared memory: puts travel inline, gets of store objects are pulled over TCP."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import cluster_anywhere_amd as ray

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cli(*args):
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-m", "cluster_anywhere_amd", *args], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr


@pytest.fixture
def head(tmp_path):
    t = str(tmp_path / "caamd")
    _cli("start", "--head", "--port", "0", "--num-cpus", "2", "--include-dashboard", "false", "--temp-dir", t)
    info = json.load(open(os.path.join(t, "head.json")))
    yield info["address"]
    _cli("stop", "--temp-dir", t)


@ray.remote
def big(n):
    import numpy as np

    return np.arange(n, dtype=np.float64)


@ray.remote
def total(x):
    return float(x.sum())


@ray.remote
class Acc:
    def __init__(self):
        self.v = 0

    def add(self, x):
        self.v += x
        return self.v


def test_client_mode_roundtrip(head):
    ctx = ray.client(f"ray://{head}").namespace("clientns").connect()
    try:
        assert ray.is_initialized() and ray.get_runtime_context().namespace == "clientns"
        arr = np.ones(3_000_000)                     # 24 MB put shipped inline
        ref = ray.put(arr)
        assert ray.get(total.remote(ref)) == 3_000_000
        out = ray.get(big.remote(2_000_000))         # lives in the head's store: pulled over TCP
        assert out.shape == (2_000_000,) and out[-1] == 1_999_999
        a = Acc.options(name="acc").remote()
        assert ray.get([a.add.remote(1), a.add.remote(2)]) == [1, 3]
        assert ray.get(ray.get_actor("acc").add.remote(4)) == 7
        ready, _ = ray.wait([big.remote(10)], timeout=30)
        assert len(ready) == 1
        assert ray.cluster_resources()["CPU"] == 2
    finally:
        ctx.disconnect()
    assert not ray.is_initialized()


def test_init_with_ray_scheme(head):
    ray.init(f"ray://{head}")
    try:
        assert ray.get(total.remote(np.arange(5.0))) == 10.0
    finally:
        ray.shutdown()
