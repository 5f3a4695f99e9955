"""joblib backend (reference: util/joblib/tests), tqdm_ray, check_serialize."""
import threading

import joblib
import pytest

import cluster_anywhere_amd as ray


@pytest.fixture
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _sq(x):
    import os

    return x * x, os.getpid()


def test_joblib_backend(cluster):
    from cluster_anywhere_amd.util.joblib import register_ray

    register_ray()
    with joblib.parallel_backend("ray"):
        out = joblib.Parallel(n_jobs=2)(joblib.delayed(_sq)(i) for i in range(20))
    assert [v for v, _ in out] == [i * i for i in range(20)]
    import os

    assert all(pid != os.getpid() for _, pid in out)
    with joblib.parallel_backend("ray"):
        assert joblib.Parallel(n_jobs=-1)(joblib.delayed(_sq)(i) for i in range(3))[2][0] == 4


def test_check_serialize():
    from cluster_anywhere_amd.util import inspect_serializability

    ok, bad = inspect_serializability(lambda: 1, name="fn")
    assert ok and not bad
    lock = threading.Lock()
    ok, bad = inspect_serializability(lambda: lock, name="holds_lock")
    assert not ok and bad


def test_tqdm_ray(cluster):
    from cluster_anywhere_amd.experimental import tqdm_ray

    @ray.remote
    def work(n):
        bar = tqdm_ray.tqdm(total=n, desc="w")
        for _ in range(n):
            bar.update(1)
        bar.close()
        return bar.n

    assert ray.get(work.remote(5)) == 5
    assert list(tqdm_ray.tqdm(range(3))) == [0, 1, 2]
