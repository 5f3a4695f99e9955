"""Data: Arrow blocks with zero-copy numpy views, the per-execution object-store
budget and autoscaling actor pools (reference test model:
python/ray/data/tests/test_arrow_block.py, test_resource_manager.py,
test_autoscaler.py / test_actor_pool_map_operator.py)."""
import time

import numpy as np
import pyarrow as pa
import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import data
from cluster_anywhere_amd.data import block as B
from cluster_anywhere_amd.data.context import DataContext
from cluster_anywhere_amd.data.dataset import ActorPoolStrategy
from cluster_anywhere_amd.data.resource_manager import ResourceManager


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=6, include_dashboard=False)
    yield
    ray.shutdown()


# ------------------------------------------------------------------ blocks
def test_arrow_block_accessors_are_zero_copy():
    img = np.arange(6 * 4 * 4 * 3, dtype=np.uint8).reshape(6, 4, 4, 3)
    t = B.to_arrow({"id": np.arange(6), "img": img, "name": np.array(list("abcdef"), dtype=object)})
    assert B.is_arrow(t) and B.num_rows(t) == 6
    assert B.schema_of(t) == {"id": "int64", "img": "uint8(4, 4, 3)", "name": "string"}
    nb = B.to_numpy(t)
    assert np.shares_memory(nb["img"], img) and np.shares_memory(nb["id"], t.column("id").chunk(0).to_numpy())
    assert list(nb["name"]) == list("abcdef")
    s = B.slice_block(t, 2, 5)
    assert B.num_rows(s) == 3 and B.col(s, "id").tolist() == [2, 3, 4]
    tk = B.take_indices(t, [5, 0])
    assert B.col(tk, "img").shape == (2, 4, 4, 3) and (B.col(tk, "img")[0] == img[5]).all()
    both = B.concat([t, {"id": np.arange(6, 8), "img": img[:2], "name": np.array(["g", "h"], dtype=object)}])
    assert B.is_arrow(both) and B.col(both, "id").tolist() == list(range(8))
    rows = list(B.iter_rows(B.slice_block(t, 0, 2)))
    assert rows[1]["id"] == 1 and rows[1]["name"] == "b"


def test_arrow_blocks_travel_zero_copy_through_the_store(cluster):
    from cluster_anywhere_amd.core import serialization

    t = B.to_arrow({"x": np.arange(1 << 16, dtype=np.float64)})
    ref = ray.put(t)
    back = ray.get(ref)
    assert B.is_arrow(back) and B.col(back, "x")[123] == 123.0
    view = B.col(back, "x")
    assert not view.flags.writeable or view.base is not None  # a view, not a private copy
    parts = serialization.serialize(t)
    assert parts is not None


def test_readers_and_arrow_udfs_produce_arrow_blocks(cluster, tmp_path):
    import pyarrow.parquet as pq

    tbl = pa.table({"k": np.arange(100) % 7, "s": [f"row{i}" for i in range(100)],
                    "v": pa.array([None if i % 10 == 0 else float(i) for i in range(100)])})
    pq.write_table(tbl, tmp_path / "a.parquet")
    ds = data.read_parquet(str(tmp_path / "a.parquet"))
    blk = ray.get(next(iter(ds._execute()))[0])
    assert B.is_arrow(blk)  # strings and nulls stay columnar
    assert ds.count() == 100
    assert ds.filter(lambda r: r["v"] is not None and r["v"] > 90).count() == 9

    def arrow_udf(t: pa.Table) -> pa.Table:
        return t.append_column("s_len", pa.compute.utf8_length(t.column("s")))

    out = ds.map_batches(arrow_udf, batch_format="pyarrow", batch_size=None)
    b2 = ray.get(next(iter(out._execute()))[0])
    assert B.is_arrow(b2) and "s_len" in b2.column_names
    assert sorted(out.take_all(), key=lambda r: r["s_len"])[-1]["s_len"] == 5
    # numpy UDFs get zero-copy numpy views of Arrow columns
    seen = {}

    def np_udf(batch):
        seen["type"] = type(batch["k"]).__name__
        return {"k2": batch["k"] * 2}

    assert sum(r["k2"] for r in ds.map_batches(np_udf).take_all()) == 2 * int((np.arange(100) % 7).sum())
    g = ds.groupby("k").count().take_all()
    assert sum(r["count()"] for r in g) == 100
    assert [r["k"] for r in ds.sort("k").take(3)] == [0, 0, 0]
    pdf = ds.to_pandas()
    assert len(pdf) == 100 and pdf["s"].iloc[3] == "row3"


# ------------------------------------------------------------------ memory budget
def test_resource_manager_admission():
    rm = ResourceManager(budget_bytes=1000)
    a, b = rm.op("a"), rm.op("b")
    a.avg_out_bytes = b.avg_out_bytes = 100
    a.n_out = b.n_out = 1  # output sizes observed
    a.inflight = 2
    assert a.can_submit()  # 300 <= reserved 250 + shared 500
    a.inflight = 7
    assert not a.can_submit()  # 800 > 250 + 500
    b.inflight = 0
    assert b.can_submit()  # an idle op may always run one task
    b.inflight = 4
    a.inflight = 2
    assert b.can_submit() and a.can_submit()


def test_execution_budget_throttles_inflight(cluster):
    ctx = DataContext.get_current()
    old = (ctx.execution_object_store_bytes, ctx.max_tasks_in_flight_per_op)
    ctx.execution_object_store_bytes = 3 << 20  # 3 MiB for the whole execution
    ctx.max_tasks_in_flight_per_op = 64
    try:
        peak = {"n": 0}

        def big(batch):
            return {"x": np.zeros((len(batch["id"]), 1 << 18), np.uint8)}  # 256 KiB/row

        ds = data.range(64, override_num_blocks=64).map_batches(big, batch_size=None)
        n = 0
        for b in ds.iter_batches(batch_size=None):
            n += len(b["x"])
        assert n == 64
        op = ds._rm.ops[0]
        assert op.throttled > 0
        assert op.peak_bytes <= 6 << 20  # never far above the 3 MiB budget
        assert "throttled" in ds.stats()
    finally:
        ctx.execution_object_store_bytes, ctx.max_tasks_in_flight_per_op = old


# ------------------------------------------------------------------ autoscaling actor pool
class _Slow:
    def __init__(self):
        import os

        self.pid = os.getpid()

    def __call__(self, batch):
        time.sleep(0.12)  # long enough that the pool scales up under a loaded CI box
        return {"id": batch["id"], "pid": np.full(len(batch["id"]), self.pid)}


def test_actor_pool_autoscales_up_and_releases(cluster):
    ds = data.range(40, override_num_blocks=40).map_batches(
        _Slow, batch_size=None, compute=ActorPoolStrategy(min_size=1, max_size=3),
        num_cpus=1)
    rows = ds.take_all()
    assert sorted(r["id"] for r in rows) == list(range(40))
    pids = {r["pid"] for r in rows}
    op = [o for o in ds._rm.ops if o.name.startswith("ActorPoolMap")][0]
    assert op.actors_peak == 3 and 2 <= len(pids) <= 3
    assert op.scale_ups == 3 and op.scale_downs >= 1
    assert "actors min/peak" in ds.stats()


def test_concurrency_tuple_and_unordered_output(cluster):
    ctx = DataContext.get_current()
    ctx.execution_preserve_order = False
    try:
        ds = data.range(30, override_num_blocks=30).map_batches(_Slow, batch_size=None, concurrency=(1, 2),
                                                                num_cpus=1)
        assert sorted(r["id"] for r in ds.take_all()) == list(range(30))
    finally:
        ctx.execution_preserve_order = True
    ordered = data.range(30, override_num_blocks=10).map_batches(_Slow, batch_size=None, concurrency=(2, 2),
                                                                 num_cpus=1)
    assert [r["id"] for r in ordered.take_all()] == list(range(30))
