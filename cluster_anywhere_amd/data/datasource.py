"""Extension points of Data: custom sources (:class:`Datasource` / :class:`ReadTask`)
and sinks (:class:`Datasink`), plus the file-sink bases the built-in writers share.

Reference roles: ``python/ray/data/datasource/datasource.py:11`` (Datasource),
``:127`` (ReadTask), ``datasource/datasink.py:31-64`` (Datasink lifecycle),
``file_datasink.py`` (BlockBasedFileDatasink / RowBasedFileDatasink) and
``dataset.py:3991`` (write_datasink).

How they run here:

* ``read_datasource(ds)`` asks ``ds.get_read_tasks(parallelism)`` once on the
  driver; every ReadTask becomes one read operator input of the streaming
  executor, executed in a remote task (pickled with its closure), its blocks
  concatenated into one output block.
* ``Dataset.write_datasink(sink)`` calls ``on_write_start`` on the driver, streams
  the dataset's blocks into remote write tasks (``write(blocks, ctx)``; at least
  ``min_rows_per_write`` rows per task when the sink asks for it; at most the
  executor's task budget in flight), then ``on_write_complete(WriteResult)`` with
  every task's return value, or ``on_write_failed(error)`` and a raise.
"""
from __future__ import annotations

import os
import uuid
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Generic, Iterable, List, Optional, TypeVar

WriteReturnType = TypeVar("WriteReturnType")


@dataclass
class BlockMetadata:
    """What the planner may know about a block before reading it."""

    num_rows: Optional[int] = None
    size_bytes: Optional[int] = None
    schema: Any = None
    input_files: Optional[List[str]] = None
    exec_stats: Any = None


@dataclass
class TaskContext:
    """Passed to :meth:`Datasink.write`: which write task this is."""

    task_idx: int
    op_name: str = "Write"
    kwargs: Dict[str, Any] = field(default_factory=dict)


class ReadTask(Callable):
    """One unit of parallel reading: ``read_fn()`` returns an iterable of blocks
    (pyarrow Tables, pandas DataFrames, dicts of columns or lists of rows), and
    ``metadata`` describes them for planning."""

    def __init__(self, read_fn: Callable[[], Iterable[Any]], metadata: Optional[BlockMetadata] = None):
        self._read_fn = read_fn
        self._metadata = metadata or BlockMetadata()

    @property
    def metadata(self) -> BlockMetadata:
        return self._metadata

    @property
    def read_fn(self) -> Callable[[], Iterable[Any]]:
        return self._read_fn

    def __call__(self) -> Iterable[Any]:
        out = self._read_fn()
        if out is None:
            return []
        return out


class Datasource:
    """A custom source: subclass and implement :meth:`get_read_tasks` (and, if
    known, :meth:`estimate_inmemory_data_size`), then ``read_datasource(src)``."""

    def get_name(self) -> str:
        name = type(self).__name__
        return name[: -len("Datasource")] if name.endswith("Datasource") and name != "Datasource" else name

    def estimate_inmemory_data_size(self) -> Optional[int]:
        return None

    def get_read_tasks(self, parallelism: int) -> List[ReadTask]:
        raise NotImplementedError(f"{type(self).__name__}.get_read_tasks(parallelism)")

    @property
    def supports_distributed_reads(self) -> bool:
        return True


@dataclass
class WriteResult(Generic[WriteReturnType]):
    """What :meth:`Datasink.on_write_complete` gets: totals over every write task
    and each task's return value (in task order)."""

    num_rows: int
    size_bytes: int
    write_returns: List[Any]


class Datasink(Generic[WriteReturnType]):
    """A custom sink: subclass, implement :meth:`write`, then
    ``ds.write_datasink(sink)``. ``write`` runs in remote tasks (the sink object is
    pickled into them), the callbacks on the driver."""

    def on_write_start(self) -> None:
        pass

    def write(self, blocks: Iterable[Any], ctx: TaskContext) -> WriteReturnType:
        raise NotImplementedError(f"{type(self).__name__}.write(blocks, ctx)")

    def on_write_complete(self, write_result: WriteResult) -> None:
        pass

    def on_write_failed(self, error: Exception) -> None:
        pass

    def get_name(self) -> str:
        name = type(self).__name__.lstrip("_")
        return name[: -len("Datasink")] if name.endswith("Datasink") and name != "Datasink" else name

    @property
    def supports_distributed_writes(self) -> bool:
        return True

    @property
    def min_rows_per_write(self) -> Optional[int]:
        return None


@dataclass
class FileShuffleConfig:
    """``read_*(..., shuffle=FileShuffleConfig(seed))``: read the input files in a
    seeded random order (``shuffle="files"``: unseeded)."""

    seed: Optional[int] = None


def shuffle_paths(paths: List[str], shuffle) -> List[str]:
    if shuffle is None or shuffle is False:
        return paths
    import random

    seed = shuffle.seed if isinstance(shuffle, FileShuffleConfig) else None
    if not (isinstance(shuffle, FileShuffleConfig) or shuffle == "files"):
        raise ValueError(f"shuffle must be None, 'files' or a FileShuffleConfig, got {shuffle!r}")
    out = list(paths)
    random.Random(seed).shuffle(out)
    return out


class _FileDatasink(Datasink[List[str]]):
    """Writes each task's data to new files under ``path`` (created on write
    start); the task returns the paths it wrote."""

    def __init__(self, path: str, *, file_format: str = "bin", dataset_uuid: Optional[str] = None,
                 try_create_dir: bool = True):
        self.path = path
        self.file_format = file_format.lstrip(".")
        self.dataset_uuid = dataset_uuid or uuid.uuid4().hex[:12]
        self.try_create_dir = try_create_dir

    def on_write_start(self) -> None:
        if self.try_create_dir:
            os.makedirs(self.path, exist_ok=True)

    def _file(self, ctx: TaskContext, k: int) -> str:
        return os.path.join(self.path, f"{self.dataset_uuid}_{ctx.task_idx:06d}_{k:06d}.{self.file_format}")


class BlockBasedFileDatasink(_FileDatasink):
    """One file per block: implement ``write_block_to_file(block, file)`` (``block``
    is a pyarrow Table, ``file`` a binary file object)."""

    def write_block_to_file(self, block, file) -> None:
        raise NotImplementedError

    def write(self, blocks: Iterable[Any], ctx: TaskContext) -> List[str]:
        from . import block as B

        written = []
        for k, blk in enumerate(blocks):
            t = B.to_arrow(blk)
            if t.num_rows == 0:
                continue
            p = self._file(ctx, k)
            with open(p, "wb") as f:
                self.write_block_to_file(t, f)
            written.append(p)
        return written


class RowBasedFileDatasink(_FileDatasink):
    """One file per row: implement ``write_row_to_file(row, file)`` (``row`` a dict)."""

    def write_row_to_file(self, row: Dict[str, Any], file) -> None:
        raise NotImplementedError

    def write(self, blocks: Iterable[Any], ctx: TaskContext) -> List[str]:
        from . import block as B

        written = []
        k = 0
        for blk in blocks:
            for row in B.to_arrow(blk).to_pylist():
                p = self._file(ctx, k)
                k += 1
                with open(p, "wb") as f:
                    self.write_row_to_file(row, f)
                written.append(p)
        return written
