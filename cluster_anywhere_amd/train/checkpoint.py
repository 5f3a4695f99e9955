"""Directory checkpoints (reference: python/ray/train/_checkpoint.py:56): a
checkpoint IS a directory plus a metadata json, on the local filesystem or on a
run's storage filesystem (``filesystem``: a pyarrow filesystem, train/storage.py);
remote checkpoints are downloaded by ``to_directory`` / ``as_directory`` /
``to_dict``."""
from __future__ import annotations

import contextlib
import json
import os
import shutil
import tempfile
import uuid
from typing import Any, Dict, Optional

_META = ".metadata.json"


class Checkpoint:
    def __init__(self, path: str, filesystem: Any = None):
        self.path = os.fspath(path)
        self.filesystem = filesystem

    @classmethod
    def from_directory(cls, path) -> "Checkpoint":
        return cls(os.path.abspath(os.fspath(path)))

    @classmethod
    def from_dict(cls, data: Dict[str, Any]) -> "Checkpoint":
        d = tempfile.mkdtemp(prefix="caamd_ckpt_")
        import pickle

        with open(os.path.join(d, "dict_checkpoint.pkl"), "wb") as f:
            pickle.dump(data, f)
        return cls(d)

    @property
    def _remote(self) -> bool:
        from .storage import is_local

        return not is_local(self.filesystem)

    def to_dict(self) -> Dict[str, Any]:
        import pickle

        with self.as_directory() as d:
            with open(os.path.join(d, "dict_checkpoint.pkl"), "rb") as f:
                return pickle.load(f)

    def to_directory(self, path: Optional[str] = None) -> str:
        from .storage import download_dir

        path = path or tempfile.mkdtemp(prefix="caamd_ckpt_")
        os.makedirs(path, exist_ok=True)
        if self._remote:
            return download_dir(self.filesystem, self.path, path)
        if os.path.abspath(path) != os.path.abspath(self.path):
            shutil.copytree(self.path, path, dirs_exist_ok=True)
        return path

    @contextlib.contextmanager
    def as_directory(self):
        from .storage import localize

        d, tmp = localize(self.path, self.filesystem)
        try:
            yield d
        finally:
            if tmp:
                shutil.rmtree(tmp, ignore_errors=True)

    def _meta_path(self):
        return (self.path.rstrip("/") + "/" + _META) if self._remote else os.path.join(self.path, _META)

    def get_metadata(self) -> Dict[str, Any]:
        if self._remote:
            try:
                with self.filesystem.open_input_stream(self._meta_path()) as f:
                    return json.loads(f.read().decode())
            except (OSError, FileNotFoundError):
                return {}
        p = os.path.join(self.path, _META)
        if not os.path.exists(p):
            return {}
        with open(p) as f:
            return json.load(f)

    def set_metadata(self, metadata: Dict[str, Any]) -> None:
        if self._remote:
            with self.filesystem.open_output_stream(self._meta_path()) as f:
                f.write(json.dumps(metadata).encode())
            return
        with open(os.path.join(self.path, _META), "w") as f:
            json.dump(metadata, f)

    def update_metadata(self, metadata: Dict[str, Any]) -> None:
        m = self.get_metadata()
        m.update(metadata)
        self.set_metadata(m)

    def __repr__(self):
        fs = "local" if not self._remote else getattr(self.filesystem, "type_name", type(self.filesystem).__name__)
        return f"Checkpoint(filesystem={fs}, path={self.path})"

    def __eq__(self, other):
        return isinstance(other, Checkpoint) and other.path == self.path

    def __hash__(self):
        return hash(self.path)


def persist(src: Checkpoint, dest_dir: str) -> Checkpoint:
    """Copy a worker-local checkpoint into the run's storage (merging shards)."""
    os.makedirs(dest_dir, exist_ok=True)
    if os.path.abspath(src.path) != os.path.abspath(dest_dir):
        shutil.copytree(src.path, dest_dir, dirs_exist_ok=True)
    return Checkpoint(dest_dir)
