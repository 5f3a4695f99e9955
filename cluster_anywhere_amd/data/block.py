"""Blocks: the unit of data movement (reference roles: python/ray/data/block.py
``BlockAccessor``, _internal/arrow_block.py:163, _internal/numpy_support.py).

Two physical block formats, both zero-copy through the shared-memory object
store (pickle-5 out-of-band buffers; pyarrow buffers travel the same way):

* **numpy blocks** ``Dict[str, np.ndarray]`` — columnar, tensor columns are
  N-d arrays. The format GPU consumers want (``torch.from_numpy`` -> pinned ->
  HBM), produced by numpy UDFs and tensor readers.
* **Arrow blocks** ``pyarrow.Table`` — what tabular readers (parquet / csv /
  json), pandas / Arrow UDFs and ``from_arrow`` produce: strings, nulls and
  nested types stay columnar instead of becoming Python object arrays. Tensor
  columns use Arrow's fixed-shape tensor extension type, so ``to_batch(...,
  "numpy")`` and ``col()`` hand out numpy VIEWS of the Arrow buffers (no copy)
  for primitive / tensor columns without nulls.

Every function here accepts either format. Mixed inputs to ``concat`` are
unified to Arrow when any input is Arrow (numpy -> Arrow is zero-copy for
primitive and tensor columns).
"""
from __future__ import annotations

from typing import Any, Dict, Iterator, List, Optional, Union

import numpy as np

Block = Union[Dict[str, np.ndarray], "pa.Table"]  # noqa: F821

_pa = None


def _arrow():
    global _pa
    if _pa is None:
        import pyarrow as pa

        _pa = pa
    return _pa


def is_arrow(b) -> bool:
    return type(b).__module__.startswith("pyarrow") and hasattr(b, "schema")


# ------------------------------------------------------------------ arrow <-> numpy
def _is_tensor_type(t) -> bool:
    pa = _arrow()
    return isinstance(t, pa.FixedShapeTensorType) if hasattr(pa, "FixedShapeTensorType") else False


def _array_to_numpy(arr) -> np.ndarray:
    """One Arrow array -> numpy, zero-copy when the layout allows it."""
    if _is_tensor_type(arr.type):
        return arr.to_numpy_ndarray()
    if arr.null_count == 0:
        try:
            return arr.to_numpy(zero_copy_only=True)
        except Exception:
            pass
    try:
        v = arr.to_numpy(zero_copy_only=False)
    except Exception:
        return np.asarray(arr.to_pylist(), dtype=object)
    if v.dtype == object and len(v) and isinstance(v[0], np.ndarray):  # list<...> of equal-length rows
        try:
            return np.stack(v)
        except ValueError:
            pass
    return v


def _chunked_to_numpy(col) -> np.ndarray:
    if hasattr(col, "num_chunks"):
        if col.num_chunks == 1:
            return _array_to_numpy(col.chunk(0))
        if col.num_chunks == 0:
            return _array_to_numpy(_arrow().array([], type=col.type))
        if _is_tensor_type(col.type):
            return np.concatenate([c.to_numpy_ndarray() for c in col.chunks])
        return _array_to_numpy(col.combine_chunks())
    return _array_to_numpy(col)


def _numpy_to_arrow_col(v):
    pa = _arrow()
    v = _to_array(v)
    if v.ndim > 1:
        return pa.FixedShapeTensorArray.from_numpy_ndarray(np.ascontiguousarray(v))
    if v.dtype == object:
        return pa.array(list(v))
    return pa.array(v)


def to_arrow(b: Block):
    """Any block -> ``pyarrow.Table`` (zero-copy for primitive / tensor columns)."""
    if is_arrow(b):
        return b
    pa = _arrow()
    if not b:
        return pa.table({})
    return pa.table({k: _numpy_to_arrow_col(v) for k, v in b.items()})


def to_numpy(b: Block) -> Dict[str, np.ndarray]:
    """Any block -> dict of numpy arrays (views of Arrow buffers when possible)."""
    if is_arrow(b):
        return {name: _chunked_to_numpy(b.column(name)) for name in b.column_names}
    return b


def col(b: Block, name: str) -> np.ndarray:
    return _chunked_to_numpy(b.column(name)) if is_arrow(b) else b[name]


def columns(b: Block) -> List[str]:
    return list(b.column_names) if is_arrow(b) else list(b.keys())


# ------------------------------------------------------------------ accessors
def num_rows(b: Block) -> int:
    if is_arrow(b):
        return b.num_rows
    for v in b.values():
        return len(v)
    return 0


def size_bytes(b: Block) -> int:
    if is_arrow(b):
        return int(b.nbytes)
    return int(sum(getattr(v, "nbytes", 0) for v in b.values()))


def slice_block(b: Block, start: int, end: int) -> Block:
    if is_arrow(b):
        return b.slice(start, max(0, end - start))
    return {k: v[start:end] for k, v in b.items()}


def take_indices(b: Block, idx) -> Block:
    if is_arrow(b):
        return b.take(_arrow().array(np.asarray(idx, dtype=np.int64)))
    return {k: v[idx] for k, v in b.items()}


def concat(blocks: List[Block]) -> Block:
    blocks = [b for b in blocks if (num_rows(b) > 0 or (b if not is_arrow(b) else b.num_columns))]
    if not blocks:
        return {}
    if len(blocks) == 1:
        return blocks[0]
    if any(is_arrow(b) for b in blocks):
        pa = _arrow()
        tables = [to_arrow(b) for b in blocks]
        try:
            return pa.concat_tables(tables, promote_options="default")
        except (pa.ArrowInvalid, TypeError):
            return pa.concat_tables([t.cast(tables[0].schema) for t in tables])
    keys = list(blocks[0].keys())
    return {k: np.concatenate([np.asarray(b[k]) for b in blocks]) for k in keys}


def _to_array(v) -> np.ndarray:
    if isinstance(v, np.ndarray):
        return v
    if "torch" in str(type(v)):
        import torch

        if isinstance(v, torch.Tensor):
            return v.detach().cpu().numpy()
    if type(v).__module__.startswith("pyarrow"):
        return _chunked_to_numpy(v)
    try:
        a = np.asarray(v)
        if a.dtype == object:
            raise ValueError
        return a
    except Exception:
        a = np.empty(len(v), dtype=object)
        for i, x in enumerate(v):
            a[i] = x
        return a


def from_rows(rows: List[Any]) -> Block:
    if not rows:
        return {}
    if isinstance(rows[0], dict):
        keys = list(rows[0].keys())
        return {k: _to_array([r[k] for r in rows]) for k in keys}
    return {"item": _to_array(rows)}


def iter_rows(b: Block) -> Iterator[Dict[str, Any]]:
    nb = to_numpy(b)
    keys = list(nb.keys())
    n = num_rows(b)
    cols = [nb[k] for k in keys]
    for i in range(n):
        yield {k: _scalar(c[i]) for k, c in zip(keys, cols)}


def _scalar(x):
    if isinstance(x, np.generic):
        return x.item()
    return x


def from_batch(batch: Any) -> Block:
    """UDF output (dict / pandas / pyarrow / list of rows) -> block. Arrow tables
    stay Arrow (zero-copy); pandas frames become Arrow tables."""
    if batch is None:
        return {}
    if isinstance(batch, dict):
        return {k: _to_array(v) for k, v in batch.items()}
    mod = type(batch).__module__
    if mod.startswith("pandas"):
        return _pandas_to_arrow(batch)
    if mod.startswith("pyarrow"):
        pa = _arrow()
        if isinstance(batch, pa.Table):
            return batch
        if isinstance(batch, pa.RecordBatch):
            return pa.Table.from_batches([batch])
        raise TypeError(f"unsupported pyarrow object {type(batch)}")
    if isinstance(batch, list):
        return from_rows(batch)
    raise TypeError(f"UDF returned unsupported batch type {type(batch)}; return a dict of arrays, "
                    "a pandas.DataFrame or a pyarrow.Table")


def _pandas_to_arrow(df):
    pa = _arrow()
    cols = {}
    for c in df.columns:
        s = df[c]
        v = s.to_numpy()
        if v.dtype == object and len(v) and isinstance(v[0], np.ndarray):
            try:
                cols[str(c)] = _numpy_to_arrow_col(np.stack(v))
                continue
            except ValueError:
                pass
        try:
            cols[str(c)] = pa.array(s, from_pandas=True)
        except (pa.ArrowInvalid, pa.ArrowTypeError, TypeError):
            cols[str(c)] = pa.array(list(v))
    return pa.table(cols)


def to_batch(b: Block, fmt: Optional[str]):
    if fmt in (None, "default", "numpy"):
        return to_numpy(b)
    if fmt == "pandas":
        import pandas as pd

        if is_arrow(b) and not any(_is_tensor_type(f.type) for f in b.schema):
            return b.to_pandas()
        cols = {}
        for k, v in to_numpy(b).items():
            cols[k] = list(v) if v.ndim > 1 else v
        return pd.DataFrame(cols)
    if fmt in ("pyarrow", "arrow"):
        return to_arrow(b)
    raise ValueError(f"unknown batch_format {fmt!r}")


def batches(b: Block, batch_size: Optional[int]) -> Iterator[Block]:
    n = num_rows(b)
    if batch_size is None or batch_size >= n:
        yield b
        return
    for s in range(0, n, batch_size):
        yield slice_block(b, s, min(n, s + batch_size))


def _type_str(t) -> str:
    if _is_tensor_type(t):
        return f"{t.value_type.to_pandas_dtype().__name__}{tuple(t.shape)}"
    try:
        d = np.dtype(t.to_pandas_dtype())
    except (NotImplementedError, TypeError):
        return str(t)
    return str(t) if d == object else str(d)


def schema_of(b: Block) -> Dict[str, Any]:
    if is_arrow(b):
        return {f.name: _type_str(f.type) for f in b.schema}
    return {k: (str(v.dtype) if v.ndim == 1 else f"{v.dtype}{tuple(v.shape[1:])}") for k, v in b.items()}
