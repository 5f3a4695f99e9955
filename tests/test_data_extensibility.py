"""Data extension points: custom Datasource / ReadTask, Datasink lifecycle with
distributed write tasks, file-sink bases, ExecutionOptions / ExecutionResources
(reference: python/ray/data/tests/test_datasource.py-style custom sources,
test_datasink.py, test_execution_options.py; datasource/datasink.py:31-64)."""
import csv
import os

import pyarrow as pa
import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import data as rd
from cluster_anywhere_amd.data import (BlockBasedFileDatasink, BlockMetadata, DataContext, Datasink, Datasource,
                                       ExecutionOptions, ExecutionResources, ReadTask, RowBasedFileDatasink)


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


class RangeSource(Datasource):
    """n rows split over the requested parallelism; each read task yields two
    blocks in different block formats."""

    def __init__(self, n):
        self.n = n

    def estimate_inmemory_data_size(self):
        return self.n * 8

    def get_read_tasks(self, parallelism):
        step = -(-self.n // parallelism)
        tasks = []
        for s in range(0, self.n, step):
            e = min(self.n, s + step)
            mid = (s + e) // 2

            def read(s=s, e=e, mid=mid):
                yield pa.table({"v": list(range(s, mid))})
                yield [{"v": i} for i in range(mid, e)]

            tasks.append(ReadTask(read, BlockMetadata(num_rows=e - s, size_bytes=(e - s) * 8)))
        return tasks


def test_custom_datasource(cluster):
    src = RangeSource(1000)
    assert src.get_name() == "RangeSource" and CollectSink("x").get_name() == "CollectSink"
    ds = rd.read_datasource(src, override_num_blocks=7)
    assert ds.num_blocks() == 7
    assert sorted(r["v"] for r in ds.take_all()) == list(range(1000))
    assert ds.map_batches(lambda b: {"v": b["v"] * 2}).sum("v") == 2 * sum(range(1000))


class CollectSink(Datasink):
    """Records where each callback ran; write returns (pid, rows)."""

    def __init__(self, path, fail_on=None, min_rows=None):
        self.path, self.fail_on, self._min_rows = path, fail_on, min_rows

    def _log(self, line):
        with open(self.path, "a") as f:
            f.write(line + "\n")

    def on_write_start(self):
        self._log(f"start {os.getpid()}")

    def write(self, blocks, ctx):
        rows = 0
        for b in blocks:
            vals = b["id"] if isinstance(b, dict) else b.column("id").to_pylist()
            if self.fail_on is not None and self.fail_on in list(vals):
                raise ValueError("bad row")
            rows += len(vals)
        return os.getpid(), rows, ctx.task_idx

    @property
    def min_rows_per_write(self):
        return self._min_rows

    def on_write_complete(self, result):
        self._log(f"complete {os.getpid()} {result.num_rows} {len(result.write_returns)} "
                  f"{sum(r[1] for r in result.write_returns)}")

    def on_write_failed(self, error):
        self._log(f"failed {type(error).__name__}")


def _lines(p):
    with open(p) as f:
        return [ln.split() for ln in f]


def test_datasink_lifecycle_and_distributed_writes(cluster, tmp_path):
    log = str(tmp_path / "log")
    sink = CollectSink(log)
    rd.range(500, override_num_blocks=10).write_datasink(sink)
    lines = _lines(log)
    assert lines[0] == ["start", str(os.getpid())]
    assert lines[-1][:3] == ["complete", str(os.getpid()), "500"] and lines[-1][3:] == ["10", "500"]
    # min_rows_per_write bundles blocks into fewer write tasks
    log2 = str(tmp_path / "log2")
    rd.range(500, override_num_blocks=10).write_datasink(CollectSink(log2, min_rows=200))
    assert _lines(log2)[-1][3] == "3"  # 200 + 200 + 100 rows


def test_datasink_remote_write_tasks_and_failure(cluster, tmp_path):
    class PidSink(CollectSink):
        def on_write_complete(self, result):
            pids = {r[0] for r in result.write_returns}
            self._log("pids " + " ".join(map(str, sorted(pids))))

    log = str(tmp_path / "log")
    rd.range(400, override_num_blocks=8).write_datasink(PidSink(log))
    pids = _lines(log)[-1][1:]
    assert pids and str(os.getpid()) not in pids  # write() ran in worker processes
    log3 = str(tmp_path / "log3")
    with pytest.raises(Exception, match="bad row"):
        rd.range(100, override_num_blocks=4).write_datasink(CollectSink(log3, fail_on=55))
    assert _lines(log3)[-1] == ["failed", "RayTaskError(ValueError)"] or _lines(log3)[-1][0] == "failed"


class CsvBlockSink(BlockBasedFileDatasink):
    def __init__(self, path):
        super().__init__(path, file_format="csv")

    def write_block_to_file(self, block, file):
        import pyarrow.csv as pcsv

        pcsv.write_csv(block, file)


class TextRowSink(RowBasedFileDatasink):
    def __init__(self, path):
        super().__init__(path, file_format="txt")

    def write_row_to_file(self, row, file):
        file.write(f"{row['id']}".encode())


def test_file_datasinks(cluster, tmp_path):
    out = tmp_path / "csv"
    rd.range(90, override_num_blocks=3).write_datasink(CsvBlockSink(str(out)))
    files = sorted(os.listdir(out))
    assert len(files) == 3 and all(f.endswith(".csv") for f in files)
    ids = []
    for f in files:
        with open(out / f) as fh:
            ids += [int(r["id"]) for r in csv.DictReader(fh)]
    assert sorted(ids) == list(range(90))
    rows = tmp_path / "rows"
    rd.range(12, override_num_blocks=2).write_datasink(TextRowSink(str(rows)))
    got = sorted(int(open(rows / f).read()) for f in os.listdir(rows))
    assert got == list(range(12))


def test_execution_options(cluster):
    ctx = DataContext.get_current()
    saved = ctx.execution_options
    try:
        opts = ExecutionOptions(resource_limits=ExecutionResources(cpu=1, object_store_memory=64 << 20),
                                preserve_order=False)
        ctx.execution_options = opts
        assert ctx.execution_preserve_order is False
        assert ctx.resource_limits() == (1, None, 64 << 20)
        from cluster_anywhere_amd.data.executor import _cluster_cpus

        assert _cluster_cpus() == 1
        assert sorted(rd.range(200, override_num_blocks=8).map(lambda r: {"id": r["id"] + 1})
                      .take_all(), key=lambda r: r["id"])[-1] == {"id": 200}
        with pytest.raises(ValueError):
            ctx.execution_options = ExecutionOptions(resource_limits=ExecutionResources(cpu=-1))
        r = ExecutionResources(cpu=2, gpu=1).add(ExecutionResources(cpu=1))
        assert (r.cpu, r.gpu, r.object_store_memory) == (3, 1, None)
        assert ExecutionResources(cpu=1).satisfies_limit(ExecutionResources(cpu=2))
        assert not ExecutionResources(cpu=3).satisfies_limit(ExecutionResources(cpu=2))
    finally:
        ctx.execution_options = ExecutionOptions(preserve_order=True)
        ctx.__dict__.pop("_execution_options", None)
        ctx.execution_preserve_order = saved.preserve_order


def test_reference_names(cluster):
    assert rd.DatasetIterator is rd.DataIterator and rd.DatasetContext is rd.DataContext
    from cluster_anywhere_amd.data.datasource import shuffle_paths

    assert sorted(shuffle_paths(["a", "b", "c"], rd.FileShuffleConfig(seed=1))) == ["a", "b", "c"]
    assert shuffle_paths(["a", "b"], None) == ["a", "b"]


def test_file_shuffle_config(cluster, tmp_path):
    for i in range(6):
        (tmp_path / f"f{i}.txt").write_text(f"line{i}\n")
    order = [r["text"] for r in rd.read_text(str(tmp_path), shuffle=rd.FileShuffleConfig(seed=3)).take_all()]
    again = [r["text"] for r in rd.read_text(str(tmp_path), shuffle=rd.FileShuffleConfig(seed=3)).take_all()]
    assert sorted(order) == [f"line{i}" for i in range(6)] and order == again
    assert [r["text"] for r in rd.read_text(str(tmp_path)).take_all()] == [f"line{i}" for i in range(6)]
