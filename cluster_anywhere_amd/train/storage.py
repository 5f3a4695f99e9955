"""Run storage for Train: where experiment results and checkpoints live
(reference: ``python/ray/train/_internal/storage.py:193,297,358,514`` --
``StorageContext``, ``get_fs_and_path``, ``persist_current_checkpoint``).

``RunConfig(storage_path=..., storage_filesystem=...)`` resolves to a
``pyarrow.fs.FileSystem`` plus a path inside it:

* ``storage_filesystem`` given: a pyarrow filesystem, or an fsspec one (wrapped in
  ``pyarrow.fs.PyFileSystem(FSSpecHandler(...))``); ``storage_path`` is then a path
  inside it.
* ``storage_path`` a URI (``file://``, ``s3://``, ``gs://``, ``hdfs://``,
  ``mock://`` ...): ``pyarrow.fs.FileSystem.from_uri``.
* a plain path: the local filesystem.

Workers write checkpoints to a directory of their own (node-local) and report it;
``persist_checkpoint`` uploads it into ``<experiment>/<checkpoint name>`` on the
storage filesystem from the WORKER's process, so a worker on a node without the
driver's disk still lands its checkpoint where the driver (and a restore on any
node) can read it. Every rank uploads its own files into the same directory
(sharded checkpoints merge). The storage context is picklable and travels to the
workers with the run.
"""
from __future__ import annotations

import os
import posixpath
import shutil
import tempfile
from typing import Any, Optional, Tuple


def _is_uri(p: str) -> bool:
    return "://" in p


def get_fs_and_path(storage_path: str, storage_filesystem: Any = None) -> Tuple[Any, str]:
    """(pyarrow filesystem, path inside it) for a storage path / filesystem pair."""
    import pyarrow.fs as pafs

    if storage_filesystem is not None:
        fs = storage_filesystem
        if not isinstance(fs, pafs.FileSystem):
            fs = pafs.PyFileSystem(pafs.FSSpecHandler(fs))  # an fsspec filesystem
        return fs, storage_path
    if _is_uri(storage_path):
        return pafs.FileSystem.from_uri(storage_path)
    return pafs.LocalFileSystem(), os.path.abspath(os.path.expanduser(storage_path))


def is_local(fs) -> bool:
    import pyarrow.fs as pafs

    return fs is None or isinstance(fs, pafs.LocalFileSystem)


def upload_dir(local_dir: str, fs, dest: str) -> None:
    """Copy a local directory's files into ``dest`` on ``fs`` (merging)."""
    import pyarrow.fs as pafs

    if is_local(fs):
        os.makedirs(dest, exist_ok=True)
        if os.path.abspath(local_dir) != os.path.abspath(dest):
            shutil.copytree(local_dir, dest, dirs_exist_ok=True)
        return
    fs.create_dir(dest, recursive=True)
    pafs.copy_files(local_dir, dest, source_filesystem=pafs.LocalFileSystem(), destination_filesystem=fs)


def download_dir(fs, src: str, local_dir: str) -> str:
    import pyarrow.fs as pafs

    os.makedirs(local_dir, exist_ok=True)
    if is_local(fs):
        if os.path.abspath(src) != os.path.abspath(local_dir):
            shutil.copytree(src, local_dir, dirs_exist_ok=True)
        return local_dir
    pafs.copy_files(src, local_dir, source_filesystem=fs, destination_filesystem=pafs.LocalFileSystem())
    return local_dir


class StorageContext:
    """Experiment storage: ``experiment_fs_path`` on ``storage_filesystem``."""

    def __init__(self, storage_path: str, experiment_name: str, storage_filesystem: Any = None):
        self.storage_path = storage_path
        self.experiment_name = experiment_name
        self.storage_filesystem, self.storage_fs_path = get_fs_and_path(storage_path, storage_filesystem)
        join = os.path.join if is_local(self.storage_filesystem) else posixpath.join
        self.experiment_fs_path = join(self.storage_fs_path, experiment_name)

    @property
    def local(self) -> bool:
        return is_local(self.storage_filesystem)

    def _join(self, *p) -> str:
        return (os.path.join if self.local else posixpath.join)(self.experiment_fs_path, *p)

    def create_experiment_dir(self) -> str:
        if self.local:
            os.makedirs(self.experiment_fs_path, exist_ok=True)
        else:
            self.storage_filesystem.create_dir(self.experiment_fs_path, recursive=True)
        return self.experiment_fs_path

    def checkpoint_fs_path(self, name: str) -> str:
        return self._join(name)

    def persist_checkpoint(self, local_dir: str, name: str) -> str:
        """Upload a worker-local checkpoint directory; returns its storage path."""
        dest = self.checkpoint_fs_path(name)
        upload_dir(local_dir, self.storage_filesystem, dest)
        return dest

    def delete(self, fs_path: str) -> None:
        try:
            if self.local:
                shutil.rmtree(fs_path, ignore_errors=True)
            else:
                self.storage_filesystem.delete_dir(fs_path)
        except Exception:
            pass

    def write_text(self, rel: str, text: str) -> None:
        p = self._join(rel)
        if self.local:
            with open(p, "w") as f:
                f.write(text)
            return
        with self.storage_filesystem.open_output_stream(p) as f:
            f.write(text.encode())

    def list_checkpoints(self):
        """Names of the ``checkpoint_*`` directories of the experiment, sorted."""
        import pyarrow.fs as pafs

        if self.local:
            if not os.path.isdir(self.experiment_fs_path):
                return []
            names = os.listdir(self.experiment_fs_path)
        else:
            infos = self.storage_filesystem.get_file_info(pafs.FileSelector(self.experiment_fs_path,
                                                                            allow_not_found=True))
            names = [posixpath.basename(i.path) for i in infos if i.type == pafs.FileType.Directory]
        return sorted(n for n in names if n.startswith("checkpoint_"))


def localize(path: str, filesystem: Any) -> Tuple[str, Optional[str]]:
    """(local directory with the checkpoint's files, temp dir to delete or None)."""
    if is_local(filesystem):
        return path, None
    tmp = tempfile.mkdtemp(prefix="caamd_ckpt_dl_")
    download_dir(filesystem, path, tmp)
    return tmp, tmp
