"""Data sources/sinks without third-party deps: TFRecord (own Example codec),
WebDataset tars, SQL (sqlite3), images, lineage serialization, random access
(reference: python/ray/data/tests/test_tfrecords.py, test_webdataset.py,
test_sql.py, test_image.py, test_random_access.py)."""
import os
import sqlite3

import numpy as np
import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import data
from cluster_anywhere_amd.data import formats


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_example_codec_roundtrip():
    row = {"i": np.int64(-7), "f": np.float32(1.5), "s": b"hi", "v": np.arange(3), "fl": np.array([0.5, 2.0])}
    out = formats.decode_example(formats.encode_example(row))
    assert out["i"] == -7 and out["f"] == 1.5 and out["s"] == b"hi"
    assert out["v"] == [0, 1, 2] and out["fl"] == [0.5, 2.0]
    assert formats.crc32c(b"123456789") == 0xE3069283  # CRC-32C check value


def test_tfrecords_roundtrip(cluster, tmp_path):
    ds = data.from_items([{"id": i, "x": float(i) / 2, "name": f"r{i}".encode()} for i in range(50)])
    ds.write_tfrecords(str(tmp_path / "tfr"))
    back = data.read_tfrecords(str(tmp_path / "tfr")).take_all()
    assert sorted(r["id"] for r in back) == list(range(50))
    r7 = [r for r in back if r["id"] == 7][0]
    assert r7["x"] == 3.5 and r7["name"] == b"r7"


def test_webdataset_roundtrip(cluster, tmp_path):
    rows = [{"__key__": f"s{i:03d}", "img": np.full((2, 2), i, np.uint8), "cls": i % 3, "txt": f"t{i}"}
            for i in range(20)]
    data.from_items(rows).write_webdataset(str(tmp_path / "wds"))
    back = sorted(data.read_webdataset(str(tmp_path / "wds")).take_all(), key=lambda r: r["__key__"])
    assert len(back) == 20 and back[5]["__key__"] == "s005"
    assert np.array_equal(back[5]["img"], np.full((2, 2), 5, np.uint8))
    assert back[5]["txt"] == "t5" and back[5]["cls"] == 2


def test_sql_roundtrip(cluster, tmp_path):
    db = str(tmp_path / "t.db")
    conn = sqlite3.connect(db)
    conn.execute("CREATE TABLE t (a INTEGER, b TEXT)")
    conn.commit()
    conn.close()
    factory = lambda: sqlite3.connect(db)  # noqa: E731
    data.from_items([{"a": i, "b": f"v{i}"} for i in range(30)]).write_sql("INSERT INTO t VALUES (?, ?)", factory)
    ds = data.read_sql("SELECT a, b FROM t WHERE a >= 10", factory)
    rows = sorted(ds.take_all(), key=lambda r: r["a"])
    assert len(rows) == 20 and rows[0] == {"a": 10, "b": "v10"}


def test_images_lineage_random_access(cluster, tmp_path):
    imgs = [{"image": np.full((4, 5, 3), i * 10, np.uint8)} for i in range(6)]
    data.from_items(imgs).write_images(str(tmp_path / "img"), column="image")
    back = data.read_images(str(tmp_path / "img")).take_all()
    assert len(back) == 6 and back[0]["image"].shape == (4, 5, 3)
    ds = data.range(100).map(lambda r: {"id": r["id"], "sq": r["id"] ** 2})
    assert ds.has_serializable_lineage()
    ds2 = data.Dataset.deserialize_lineage(ds.serialize_lineage())
    assert ds2.sum("sq") == ds.sum("sq")
    ra = data.range(1000).map(lambda r: {"k": r["id"] * 2, "v": -r["id"]}).to_random_access_dataset("k", 3)
    assert ra.multiget([0, 10, 1998, 7]) == [{"k": 0, "v": 0}, {"k": 10, "v": -5}, {"k": 1998, "v": -999}, None]
    with pytest.raises(TypeError):  # duck-typed over the Dask API: a non-Dask object fails loudly
        data.from_dask(None)
