"""Public API surface parity with the reference's __all__ lists, plus behaviour of
the smaller utilities (custom serializers, ParallelIterator, log_once, tune
registry, TorchCheckpoint/TorchPredictor)."""
import re

import numpy as np
import pytest

import cluster_anywhere_amd as ray

REF = "/root/reference/python/ray"


def _ref_all(path):
    try:
        src = open(path).read()
    except OSError:
        pytest.skip("reference tree not mounted")
    m = re.search(r"__all__ = \[(.*?)\]", src, re.S)
    return set(re.findall(r'"(\w+)"', m.group(1)))


@pytest.mark.parametrize("ref,ours", [
    ("__init__.py", "cluster_anywhere_amd"), ("train/__init__.py", "cluster_anywhere_amd.train"),
    ("tune/__init__.py", "cluster_anywhere_amd.tune"), ("util/__init__.py", "cluster_anywhere_amd.util"),
    ("train/torch/__init__.py", "cluster_anywhere_amd.train.torch"),
])
def test_all_names_present(ref, ours):
    import importlib

    mod = importlib.import_module(ours)
    missing = sorted(n for n in _ref_all(f"{REF}/{ref}") if not n.startswith("_") and not hasattr(mod, n))
    assert not missing, missing


class Point:
    def __init__(self, x):
        self.x = x

    def __reduce__(self):
        raise TypeError("not picklable by default")


def test_custom_serializer_and_iter():
    from cluster_anywhere_amd import util

    ray.init(num_cpus=2)
    try:
        util.register_serializer(Point, serializer=lambda p: p.x, deserializer=lambda x: Point(x * 10))

        @ray.remote
        def getx(p):
            return p.x

        assert ray.get(getx.remote(Point(4))) == 40
        util.deregister_serializer(Point)
        it = util.iter.from_range(10, num_shards=3).for_each(lambda x: x * 2).filter(lambda x: x % 4 == 0)
        assert sorted(it.gather_sync()) == [0, 4, 8, 12, 16]
        assert sorted(util.iter.from_items([1, 2, 3], 2).gather_async()) == [1, 2, 3]
    finally:
        ray.shutdown()
    assert util.log_once("k1") and not util.log_once("k1")


def test_tune_registry_and_torch_predictor(tmp_path):
    import torch

    from cluster_anywhere_amd import tune
    from cluster_anywhere_amd.train.torch import TorchCheckpoint, TorchPredictor

    tune.register_trainable("my_fn", lambda cfg: {"score": cfg["x"] * 2})
    assert tune.registry.get_trainable_cls("my_fn")({"x": 2}) == {"score": 4}
    assert isinstance(tune.create_scheduler("asha", metric="m", mode="max"), tune.ASHAScheduler)
    assert isinstance(tune.create_searcher("hyperopt", metric="m", mode="max"), tune.HyperOptSearch)
    with pytest.raises(ValueError):
        tune.create_searcher("no-such-searcher")
    m = torch.nn.Linear(3, 2)
    ck = TorchCheckpoint.from_model(m)
    p = TorchPredictor.from_checkpoint(ck, model=torch.nn.Linear(3, 2))
    x = np.random.rand(4, 3).astype(np.float32)
    out = p.predict({"x": x})["predictions"]
    assert np.allclose(out, m(torch.from_numpy(x)).detach().numpy(), atol=1e-6)
