"""Dataset creation (reference: python/ray/data/read_api.py: range :228,
range_tensor :280, from_items :145, read_parquet :776, read_csv :1393,
read_json :1248, read_text :1562, read_numpy :1786, read_binary_files :2151,
read_images :955, from_pandas :2658, from_numpy :2780, from_arrow :2866,
from_torch :3262, from_huggingface :3058)."""
from __future__ import annotations

import glob
import math
import os
from typing import Any, Dict, List, Optional, Union

import numpy as np

from . import block as B
from .dataset import Dataset


def _default_blocks(n_rows: int, override: Optional[int]) -> int:
    if override:
        return max(1, int(override))
    try:
        from ..core.api import cluster_resources

        cpus = int(cluster_resources().get("CPU", 4))
    except Exception:
        cpus = 4
    return max(1, min(n_rows, max(2 * cpus, 8), 200)) if n_rows else 1


def _chunks(n: int, k: int):
    import builtins

    per = [n // k + (1 if i < n % k else 0) for i in builtins.range(k)]
    s = 0
    for p in per:
        yield s, s + p
        s += p


def range(n: int, *, override_num_blocks: Optional[int] = None, parallelism: int = -1) -> Dataset:
    k = _default_blocks(n, override_num_blocks or (parallelism if parallelism > 0 else None))
    reads = [(lambda s=s, e=e: {"id": np.arange(s, e, dtype=np.int64)}) for s, e in _chunks(n, k)]
    return Dataset(("read", reads))


def range_tensor(n: int, *, shape=(1,), override_num_blocks: Optional[int] = None, parallelism: int = -1) -> Dataset:
    k = _default_blocks(n, override_num_blocks or (parallelism if parallelism > 0 else None))
    shape = tuple(shape)

    def mk(s, e):
        a = np.arange(s, e, dtype=np.int64).reshape((-1,) + (1,) * len(shape))
        return {"data": np.broadcast_to(a, (e - s,) + shape).copy()}

    return Dataset(("read", [(lambda s=s, e=e: mk(s, e)) for s, e in _chunks(n, k)]))


def from_items(items: List[Any], *, override_num_blocks: Optional[int] = None, parallelism: int = -1) -> Dataset:
    from ..core.api import put

    k = _default_blocks(len(items), override_num_blocks or (parallelism if parallelism > 0 else None))
    refs = []
    for s, e in _chunks(len(items), k):
        b = B.from_rows(items[s:e])
        refs.append((put(b), {"num_rows": B.num_rows(b), "size_bytes": B.size_bytes(b),
                              "schema": B.schema_of(b)}))
    return Dataset(("refs", refs))


def from_blocks(blocks: List[Dict[str, np.ndarray]]) -> Dataset:
    from ..core.api import put

    return Dataset(("refs", [(put(b), {"num_rows": B.num_rows(b), "size_bytes": B.size_bytes(b),
                                       "schema": B.schema_of(b)}) for b in blocks]))


def from_numpy(ndarrays) -> Dataset:
    arrs = ndarrays if isinstance(ndarrays, list) else [ndarrays]
    return from_blocks([{"data": np.asarray(a)} for a in arrs])


def from_pandas(dfs) -> Dataset:
    dfs = dfs if isinstance(dfs, list) else [dfs]
    return from_blocks([B.from_batch(df) for df in dfs])


def from_arrow(tables) -> Dataset:
    tables = tables if isinstance(tables, list) else [tables]
    return from_blocks([B.from_batch(t) for t in tables])


def from_numpy_refs(refs) -> Dataset:
    from ..core.api import get

    return from_numpy(get(refs))


def from_pandas_refs(refs) -> Dataset:
    from ..core.api import get

    return from_pandas(get(refs))


def from_arrow_refs(refs) -> Dataset:
    from ..core.api import get

    return from_arrow(get(refs))


def from_torch(dataset) -> Dataset:
    return from_items([{"item": dataset[i]} for i in builtins_range(len(dataset))])


def from_huggingface(dataset, **kw) -> Dataset:
    if hasattr(dataset, "to_pandas"):
        return from_pandas(dataset.to_pandas())
    return from_items(list(dataset))


def builtins_range(n):
    import builtins

    return builtins.range(n)


def _expand(paths, exts=None) -> List[str]:
    if isinstance(paths, str):
        paths = [paths]
    out = []
    for p in paths:
        if os.path.isdir(p):
            for root, _, files in os.walk(p):
                for f in sorted(files):
                    if exts is None or any(f.endswith(e) for e in exts):
                        out.append(os.path.join(root, f))
        elif any(ch in p for ch in "*?["):
            out.extend(sorted(glob.glob(p)))
        else:
            out.append(p)
    if not out:
        raise ValueError(f"no input files found in {paths}")
    return out


def _file_ds(files, reader, **kw) -> Dataset:
    ds = Dataset(("read", [(lambda f=f: reader(f)) for f in files]))
    ds._input_files = files
    return ds


def _shuffled(files, shuffle):
    """``shuffle="files"`` / ``FileShuffleConfig(seed)``: read the files in random order."""
    from .datasource import shuffle_paths

    return shuffle_paths(files, shuffle)


def read_parquet(paths, *, columns: Optional[List[str]] = None, filter=None, **kw) -> Dataset:
    files = _shuffled(_expand(paths, [".parquet"]), kw.pop("shuffle", None))

    def rd(f):
        import pyarrow.parquet as pq

        return B.from_batch(pq.read_table(f, columns=columns, filters=filter))

    return _file_ds(files, rd)


def read_csv(paths, **arrow_csv_args) -> Dataset:
    files = _shuffled(_expand(paths, [".csv", ".csv.gz"]), arrow_csv_args.pop("shuffle", None))

    def rd(f):
        import pyarrow.csv as pcsv

        return B.from_batch(pcsv.read_csv(f))

    return _file_ds(files, rd)


def read_json(paths, *, lines: bool = True, **kw) -> Dataset:
    files = _shuffled(_expand(paths, [".json", ".jsonl"]), kw.pop("shuffle", None))

    def rd(f):
        import pandas as pd

        try:
            return B.from_batch(pd.read_json(f, lines=True))
        except ValueError:
            return B.from_batch(pd.read_json(f))

    return _file_ds(files, rd)


def read_text(paths, *, encoding: str = "utf-8", drop_empty_lines: bool = True, **kw) -> Dataset:
    files = _shuffled(_expand(paths), kw.pop("shuffle", None))

    def rd(f):
        with open(f, encoding=encoding) as fh:
            lines = [l.rstrip("\n") for l in fh]
        if drop_empty_lines:
            lines = [l for l in lines if l.strip()]
        return {"text": np.asarray(lines, dtype=object)}

    return _file_ds(files, rd)


def read_numpy(paths, **kw) -> Dataset:
    files = _shuffled(_expand(paths, [".npy"]), kw.pop("shuffle", None))
    return _file_ds(files, lambda f: {"data": np.load(f, allow_pickle=False)})


def read_binary_files(paths, *, include_paths: bool = False, **kw) -> Dataset:
    files = _shuffled(_expand(paths), kw.pop("shuffle", None))

    def rd(f):
        with open(f, "rb") as fh:
            data = fh.read()
        b = {"bytes": np.asarray([data], dtype=object)}
        if include_paths:
            b["path"] = np.asarray([f], dtype=object)
        return b

    return _file_ds(files, rd)


def read_images(paths, *, size=None, mode=None, include_paths: bool = False, **kw) -> Dataset:
    files = _shuffled(_expand(paths, [".png", ".jpg", ".jpeg", ".bmp", ".gif", ".npy"]), kw.pop("shuffle", None))

    def rd(f):
        if f.endswith(".npy"):
            img = np.load(f, allow_pickle=False)
        else:
            from PIL import Image  # optional dependency

            im = Image.open(f)
            if mode:
                im = im.convert(mode)
            if size:
                im = im.resize(size[::-1])
            img = np.asarray(im)
        b = {"image": img[None]}
        if include_paths:
            b["path"] = np.asarray([f], dtype=object)
        return b

    return _file_ds(files, rd)


def read_parquet_bulk(paths, *, columns: Optional[List[str]] = None, **kw) -> Dataset:
    """Many small parquet files, no metadata pre-pass (reference: read_parquet_bulk)."""
    return read_parquet(paths, columns=columns, **kw)


def read_tfrecords(paths, *, verify_crc: bool = True, **kw) -> Dataset:
    """TFRecord files of ``tf.train.Example`` (decoded without TensorFlow, see formats.py)."""
    from . import formats

    files = _expand(paths, [".tfrecords", ".tfrecord"])
    return _file_ds(files, lambda f: B.from_rows(formats.read_tfrecords(f, verify_crc)))


def read_webdataset(paths, *, decode: bool = True, **kw) -> Dataset:
    """WebDataset tar shards; one row per sample key, one column per member suffix."""
    from . import formats

    files = _expand(paths, [".tar"])
    return _file_ds(files, lambda f: B.from_rows(formats.read_webdataset(f, decode)))


def read_sql(sql: str, connection_factory, *, parallelism: int = -1, **kw) -> Dataset:
    """Run ``sql`` on a DB-API 2 connection from ``connection_factory()`` (reference: read_sql)."""

    def rd():
        conn = connection_factory()
        try:
            cur = conn.cursor()
            cur.execute(sql)
            names = [d[0] for d in cur.description]
            rows = cur.fetchall()
        finally:
            conn.close()
        return {n: B._to_array([r[i] for r in rows]) for i, n in enumerate(names)}

    return Dataset(("read", [rd]))


def read_avro(paths, **kw) -> Dataset:
    """Avro object-container files, one block per file (own decoder: data/avro.py;
    reference: datasource/avro_datasource.py)."""
    from .avro import read_avro_file

    files = _expand(paths, [".avro"])
    return _file_ds(files, lambda f: B.from_rows(list(read_avro_file(f))))


def _read_wav(path):
    import wave

    with wave.open(path, "rb") as w:
        ch, width, rate, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
        raw = w.readframes(n)
    if width == 1:
        a = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    elif width == 2:
        a = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
    elif width == 3:
        b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        a = v.astype(np.float32) / float(1 << 23)
    elif width == 4:
        a = np.frombuffer(raw, "<i4").astype(np.float32) / float(1 << 31)
    else:
        raise ValueError(f"unsupported WAV sample width {width}")
    return a.reshape(-1, ch).T.copy(), rate


def read_audio(paths, *, include_paths: bool = False, **kw) -> Dataset:
    """PCM WAV files -> ``amplitude [channels, samples]`` float32 in [-1, 1] and
    ``sample_rate`` (reference: datasource/audio_datasource.py; decoded with the
    standard-library ``wave`` module, no soundfile)."""
    files = _expand(paths, [".wav", ".wave"])

    def rd(f):
        amp, rate = _read_wav(f)
        b = {"amplitude": amp[None], "sample_rate": np.asarray([rate], dtype=np.int64)}
        if include_paths:
            b["path"] = np.asarray([f], dtype=object)
        return b

    return _file_ds(files, rd)


def _local(uri: str) -> str:
    return uri[len("file://"):] if uri.startswith("file://") else (uri[5:] if uri.startswith("file:") else uri)


def read_iceberg(table_identifier: str, *, snapshot_id: Optional[int] = None,
                 selected_fields: Optional[List[str]] = None, row_filter=None, **kw) -> Dataset:
    """An Iceberg table on a local / mounted filesystem (``table_identifier`` =
    the table directory): latest (or ``snapshot_id``) snapshot -> manifest list
    -> manifests (Avro, decoded by data/avro.py) -> live Parquet data files, one
    read task per file. Delete files (v2 row-level deletes) are refused.
    Reference: datasource/iceberg_datasource.py (which drives pyiceberg)."""
    import json as _json

    from .avro import read_avro_file

    root = _local(table_identifier)
    mdir = os.path.join(root, "metadata")
    hint = os.path.join(mdir, "version-hint.text")
    cands = sorted(glob.glob(os.path.join(mdir, "*.metadata.json")))
    if not cands:
        raise ValueError(f"no Iceberg metadata under {mdir}")
    meta_path = cands[-1]
    if os.path.exists(hint):
        v = open(hint).read().strip()
        for c in cands:
            b = os.path.basename(c)
            if b == f"v{v}.metadata.json" or b.startswith(f"{int(v):05d}-"):
                meta_path = c
    else:
        def ver(p):
            b = os.path.basename(p)
            head = b.split(".")[0].split("-")[0].lstrip("v")
            return int(head) if head.isdigit() else -1

        meta_path = max(cands, key=ver)
    with open(meta_path) as f:
        meta = _json.load(f)
    sid = snapshot_id if snapshot_id is not None else meta.get("current-snapshot-id")
    if sid is None or sid == -1:
        return from_items([])
    snap = next((s for s in meta.get("snapshots", []) if s["snapshot-id"] == sid), None)
    if snap is None:
        raise ValueError(f"snapshot {sid} not found in {meta_path}")
    files = []
    for m in read_avro_file(_local(snap["manifest-list"])):
        if int(m.get("content", 0) or 0) != 0:
            raise NotImplementedError("Iceberg row-level delete files are not supported")
        for ent in read_avro_file(_local(m["manifest_path"])):
            if int(ent.get("status", 1)) == 2:
                continue  # deleted in this snapshot
            df = ent["data_file"]
            if int(df.get("content", 0) or 0) != 0:
                raise NotImplementedError("Iceberg row-level delete files are not supported")
            if str(df.get("file_format", "PARQUET")).upper() != "PARQUET":
                raise NotImplementedError(f"Iceberg data file format {df.get('file_format')}")
            files.append(_local(df["file_path"]))
    if not files:
        return from_items([])

    def rd(f):
        import pyarrow.parquet as pq

        return B.from_batch(pq.read_table(f, columns=selected_fields, filters=row_filter))

    return _file_ds(sorted(set(files)), rd)


def read_hudi(table_uri: str, **kw) -> Dataset:
    """Snapshot query of a copy-on-write Hudi table on a local filesystem: for
    every file group the Parquet base file of the latest COMPLETED commit
    (``.hoodie/<instant>.commit``); merge-on-read log files are refused.
    Reference: datasource/hudi_datasource.py (which drives hudi-rs)."""
    root = _local(table_uri)
    hoodie = os.path.join(root, ".hoodie")
    if not os.path.isdir(hoodie):
        raise ValueError(f"{root} is not a Hudi table (no .hoodie directory)")
    done = {n.split(".")[0] for n in os.listdir(hoodie)
            if n.endswith(".commit") or n.endswith(".replacecommit")}
    latest: Dict[tuple, tuple] = {}
    for dirpath, dirnames, filenames in os.walk(root):
        dirnames[:] = [d for d in dirnames if d != ".hoodie"]
        for fn in filenames:
            if fn.endswith(".log") or ".log." in fn:
                raise NotImplementedError("Hudi merge-on-read log files are not supported")
            if not fn.endswith(".parquet"):
                continue
            parts = fn[: -len(".parquet")].split("_")
            if len(parts) < 3:
                continue
            file_id, instant = parts[0], parts[-1]
            if instant not in done:
                continue  # inflight / rolled back write
            key = (os.path.relpath(dirpath, root), file_id)
            if key not in latest or instant > latest[key][0]:
                latest[key] = (instant, os.path.join(dirpath, fn))
    files = sorted(p for _, p in latest.values())
    if not files:
        return from_items([])

    def rd(f):
        import pyarrow.parquet as pq

        return B.from_batch(pq.read_table(f))

    return _file_ds(files, rd)


def _unavailable(name: str, lib: str):
    def fn(*a, **k):
        raise ImportError(f"{name} needs {lib}, which is not installed in this image "
                          "(no package index on MI355X pods)")

    fn.__name__ = name
    return fn


for _n, _lib in (("read_lance", "lance"),):
    globals()[_n] = _unavailable(_n, _lib)


# ---- other dataframe / dataset libraries: duck-typed over their public export
# methods, so a user who has the library gets blocks without this package
# importing it (reference: read_api.py from_dask :2542, from_modin :2616,
# from_mars :2591, from_spark :2968, from_tf :3157).
def from_dask(df) -> Dataset:
    """One block per Dask partition (``df.to_delayed()`` computed lazily per read task)."""
    if not (hasattr(df, "to_delayed") or hasattr(df, "compute")):
        raise TypeError(f"from_dask expects a Dask DataFrame (to_delayed / compute), got {type(df).__name__}")
    parts = df.to_delayed() if hasattr(df, "to_delayed") else [df]

    def rd(p):
        out = p.compute() if hasattr(p, "compute") else p
        return B.from_batch(out)

    return Dataset(("read", [(lambda p=p: rd(p)) for p in parts]))


def from_modin(df) -> Dataset:
    """Modin frame -> pandas partitions (``_to_pandas`` / ``to_pandas``)."""
    pdf = df._to_pandas() if hasattr(df, "_to_pandas") else df.to_pandas()
    return from_pandas(pdf)


def from_mars(df) -> Dataset:
    pdf = df.to_pandas() if hasattr(df, "to_pandas") else df.execute().fetch()
    return from_pandas(pdf)


def from_spark(df, *, parallelism: Optional[int] = None, override_num_blocks: Optional[int] = None) -> Dataset:
    """Spark DataFrame -> Arrow (``toArrow`` on Spark >= 4, else ``toPandas``),
    split into ``override_num_blocks`` blocks."""
    t = df.toArrow() if hasattr(df, "toArrow") else df.toPandas()
    n = len(t)
    k = max(1, min(n, override_num_blocks or parallelism or 1)) if n else 1
    if k == 1:
        return from_blocks([B.from_batch(t)])
    return from_blocks([B.from_batch(t.slice(s, e - s) if hasattr(t, "slice") else t.iloc[s:e])
                        for s, e in _chunks(n, k)])


def from_tf(dataset) -> Dataset:
    """A ``tf.data.Dataset`` of dict / tuple / tensor elements, materialised
    through ``as_numpy_iterator()`` (the reference does the same)."""
    it = dataset.as_numpy_iterator() if hasattr(dataset, "as_numpy_iterator") else iter(dataset)
    rows = []
    for el in it:
        if isinstance(el, dict):
            rows.append(dict(el))
        elif isinstance(el, tuple):
            rows.append({f"item_{i}" if len(el) > 2 else ("features", "label")[i]: v for i, v in enumerate(el)})
        else:
            rows.append({"item": el})
    return from_items(rows)

# spoken over their HTTP protocols, no client library needed (data/connectors.py)
from .connectors import (read_bigquery, read_clickhouse, read_databricks_tables,  # noqa: E402
                         read_delta_sharing_tables, read_mongo, read_videos)


def _run_read_task(task):
    """One read operator input: a ReadTask (or any callable) -> one block."""
    out = task()
    if out is None:
        return {}
    if isinstance(out, dict) or B.is_arrow(out) or hasattr(out, "to_numpy") and hasattr(out, "columns"):
        return B.from_batch(out)  # a single block, not an iterable of blocks
    return B.concat([B.from_batch(x) for x in out])


def read_datasource(datasource, *, parallelism: int = -1, ray_remote_args: Optional[Dict[str, Any]] = None,
                    concurrency: Optional[int] = None, override_num_blocks: Optional[int] = None,
                    **read_args) -> Dataset:
    """Read a custom :class:`~.datasource.Datasource`: ``get_read_tasks`` runs here
    once; each :class:`~.datasource.ReadTask` is one read input of the streaming
    executor, run in a remote task. Reference: read_api.py read_datasource."""
    import functools

    from .context import DataContext
    from .executor import _cluster_cpus

    n = override_num_blocks or (parallelism if parallelism and parallelism > 0 else 0)
    if not n:
        n = max(DataContext.get_current().read_op_min_num_blocks, 2 * _cluster_cpus())
    tasks = datasource.get_read_tasks(int(n), **read_args) if read_args else datasource.get_read_tasks(int(n))
    fns = [functools.partial(_run_read_task, t) for t in tasks]
    return Dataset(("read", fns))
