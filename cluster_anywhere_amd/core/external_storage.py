"""Where the head spills objects when the shared-memory store is full (reference:
python/ray/_private/external_storage.py: FileSystemStorage :272 -- one or several
local directories, round-robin; ExternalStorageSmartOpenImpl :481 -- any URI;
setup_external_storage :660).

Configured with ``init(_system_config={"object_spilling_config": cfg})`` where
``cfg`` is a dict or its JSON string, ``start --head --system-config JSON``, or
``CAAMD_OBJECT_SPILLING_CONFIG``:

* ``{"type": "filesystem", "params": {"directory_path": "/a" | ["/a", "/b"]}}``:
  spilled objects go to ``<dir>/caamd_spilled_objects_<session>/``, successive
  objects on successive directories (spreads spill I/O over several disks);
* ``{"type": "smart_open", "params": {"uri": "s3://bucket/prefix" | [uris]}}``
  (alias ``"uri"``): through ``pyarrow.fs.FileSystem.from_uri`` (local, S3, GCS,
  HDFS as built into pyarrow) or, for schemes pyarrow does not know (``memory://``,
  ``gs://`` through gcsfs, ...), through ``fsspec``. smart_open itself is not in
  the image; the URI form is the reference's.

Without a config the head spills to ``<session_dir>/spill``. One object per file;
each spill returns the URL the head keeps with the object (restore / delete).
"""
from __future__ import annotations

import itertools
import json
import os
import threading
from typing import List, Optional, Union


class ExternalStorage:
    def spill(self, key: str, data) -> str:
        raise NotImplementedError

    def restore(self, url: str) -> bytes:
        raise NotImplementedError

    def delete(self, url: str) -> None:
        raise NotImplementedError

    def destroy(self) -> None:
        pass

    def describe(self) -> str:
        return type(self).__name__


class FileSystemStorage(ExternalStorage):
    def __init__(self, directory_path: Union[str, List[str]], session_name: str = "session",
                 buffer_size: Optional[int] = None):
        paths = [directory_path] if isinstance(directory_path, str) else list(directory_path)
        if not paths:
            raise ValueError("object_spilling_config: directory_path is empty")
        self.dirs = []
        for p in paths:
            d = os.path.join(os.path.expanduser(p), f"caamd_spilled_objects_{session_name}")
            os.makedirs(d, exist_ok=True)
            if not os.access(d, os.W_OK):
                raise ValueError(f"object_spilling_config: {d} is not writable")
            self.dirs.append(d)
        self._next = itertools.cycle(range(len(self.dirs)))
        self._lock = threading.Lock()
        self.buffer_size = buffer_size

    def spill(self, key: str, data) -> str:
        with self._lock:
            d = self.dirs[next(self._next)]
        path = os.path.join(d, key)
        with open(path, "wb", buffering=self.buffer_size or -1) as f:
            f.write(data)
        return path

    def restore(self, url: str) -> bytes:
        with open(url, "rb") as f:
            return f.read()

    def delete(self, url: str) -> None:
        try:
            os.unlink(url)
        except OSError:
            pass

    def destroy(self) -> None:
        for d in self.dirs:
            try:
                for n in os.listdir(d):
                    os.unlink(os.path.join(d, n))
                os.rmdir(d)
            except OSError:
                pass

    def describe(self) -> str:
        return f"filesystem:{','.join(self.dirs)}"


class _Fs:
    """One URI root: a pyarrow filesystem when pyarrow knows the scheme, else fsspec."""

    def __init__(self, uri: str):
        self.uri = uri.rstrip("/")
        self.kind = None
        try:
            import pyarrow.fs as pafs

            self.fs, self.root = pafs.FileSystem.from_uri(self.uri)
            self.kind = "pyarrow"
            self.fs.create_dir(self.root, recursive=True)
        except Exception:
            import fsspec

            self.fs, self.root = fsspec.core.url_to_fs(self.uri)
            self.kind = "fsspec"
            try:
                self.fs.makedirs(self.root, exist_ok=True)
            except Exception:
                pass

    def write(self, name: str, data) -> str:
        path = f"{self.root}/{name}"
        if self.kind == "pyarrow":
            with self.fs.open_output_stream(path) as f:
                f.write(data)
        else:
            with self.fs.open(path, "wb") as f:
                f.write(bytes(data) if not isinstance(data, (bytes, bytearray)) else data)
        return path

    def read(self, path: str) -> bytes:
        if self.kind == "pyarrow":
            with self.fs.open_input_stream(path) as f:
                return f.read()
        with self.fs.open(path, "rb") as f:
            return f.read()

    def delete(self, path: str) -> None:
        try:
            if self.kind == "pyarrow":
                self.fs.delete_file(path)
            else:
                self.fs.rm(path)
        except Exception:
            pass

    def delete_dir(self):
        try:
            if self.kind == "pyarrow":
                self.fs.delete_dir(self.root)
            else:
                self.fs.rm(self.root, recursive=True)
        except Exception:
            pass


class URIStorage(ExternalStorage):
    """The reference's ``smart_open`` type: objects under ``<uri>/caamd_spilled_objects_<session>/``;
    with several URIs, successive objects go to successive ones."""

    def __init__(self, uri: Union[str, List[str]], session_name: str = "session", **_ignored):
        uris = [uri] if isinstance(uri, str) else list(uri)
        if not uris:
            raise ValueError("object_spilling_config: uri is empty")
        self.roots = [_Fs(f"{u.rstrip('/')}/caamd_spilled_objects_{session_name}") for u in uris]
        self._next = itertools.cycle(range(len(self.roots)))
        self._lock = threading.Lock()

    def spill(self, key: str, data) -> str:
        with self._lock:
            i = next(self._next)
        return f"{i}|{self.roots[i].write(key, data)}"

    def _split(self, url: str):
        i, path = url.split("|", 1)
        return self.roots[int(i)], path

    def restore(self, url: str) -> bytes:
        fs, path = self._split(url)
        return fs.read(path)

    def delete(self, url: str) -> None:
        fs, path = self._split(url)
        fs.delete(path)

    def destroy(self) -> None:
        for r in self.roots:
            r.delete_dir()

    def describe(self) -> str:
        return f"uri:{','.join(r.uri for r in self.roots)}"


def parse_config(cfg) -> Optional[dict]:
    if cfg is None or cfg == "" or cfg == {}:
        return None
    if isinstance(cfg, (bytes, bytearray)):
        cfg = cfg.decode()
    if isinstance(cfg, str):
        cfg = json.loads(cfg)
    if not isinstance(cfg, dict) or "type" not in cfg:
        raise ValueError(f"object_spilling_config needs a 'type': {cfg!r}")
    return cfg


def setup_external_storage(cfg, session_name: str, default_dir: str) -> ExternalStorage:
    cfg = parse_config(cfg)
    if cfg is None:
        return FileSystemStorage(default_dir, session_name)
    t, params = cfg["type"], dict(cfg.get("params") or {})
    if t == "filesystem":
        if "directory_path" not in params:
            raise ValueError("object_spilling_config type 'filesystem' needs params.directory_path")
        return FileSystemStorage(params["directory_path"], session_name, params.get("buffer_size"))
    if t in ("smart_open", "uri", "fsspec", "pyarrow"):
        if "uri" not in params:
            raise ValueError(f"object_spilling_config type {t!r} needs params.uri")
        return URIStorage(params.pop("uri"), session_name, **params)
    raise ValueError(f"unsupported object_spilling_config type {t!r} (filesystem, smart_open)")
