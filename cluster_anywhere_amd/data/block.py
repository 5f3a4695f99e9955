"""Blocks: the unit of data movement (reference: python/ray/data/block.py).

A block is a ``Dict[str, np.ndarray]`` (columnar numpy, every column the same
length; tensor columns are N-d arrays). This is the zero-copy format of the
object store (arrays are out-of-band pickle-5 buffers) and the format GPU
consumers want (``torch.from_numpy`` → pinned → HBM). pandas / pyarrow batches
are converted at the UDF boundary only.
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, Iterator, List, Optional

import numpy as np

Block = Dict[str, np.ndarray]


def num_rows(b: Block) -> int:
    for v in b.values():
        return len(v)
    return 0


def size_bytes(b: Block) -> int:
    return int(sum(getattr(v, "nbytes", 0) for v in b.values()))


def slice_block(b: Block, start: int, end: int) -> Block:
    return {k: v[start:end] for k, v in b.items()}


def take_indices(b: Block, idx) -> Block:
    return {k: v[idx] for k, v in b.items()}


def concat(blocks: List[Block]) -> Block:
    blocks = [b for b in blocks if num_rows(b) > 0 or b]
    if not blocks:
        return {}
    if len(blocks) == 1:
        return blocks[0]
    keys = list(blocks[0].keys())
    return {k: np.concatenate([np.asarray(b[k]) for b in blocks]) for k in keys}


def _to_array(v) -> np.ndarray:
    if isinstance(v, np.ndarray):
        return v
    if "torch" in str(type(v)):
        import torch

        if isinstance(v, torch.Tensor):
            return v.detach().cpu().numpy()
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
    keys = list(b.keys())
    n = num_rows(b)
    cols = [b[k] for k in keys]
    for i in range(n):
        yield {k: _scalar(c[i]) for k, c in zip(keys, cols)}


def _scalar(x):
    if isinstance(x, np.generic):
        return x.item()
    return x


def from_batch(batch: Any) -> Block:
    """UDF output (dict / pandas / pyarrow / list of rows) -> block."""
    if batch is None:
        return {}
    if isinstance(batch, dict):
        return {k: _to_array(v) for k, v in batch.items()}
    mod = type(batch).__module__
    if mod.startswith("pandas"):
        return {str(c): _col_from_pandas(batch[c]) for c in batch.columns}
    if mod.startswith("pyarrow"):
        return {name: _col_from_arrow(batch.column(name)) for name in batch.column_names}
    if isinstance(batch, list):
        return from_rows(batch)
    raise TypeError(f"UDF returned unsupported batch type {type(batch)}; return a dict of arrays, "
                    "a pandas.DataFrame or a pyarrow.Table")


def _col_from_pandas(s):
    v = s.to_numpy()
    if v.dtype == object and len(v) and isinstance(v[0], np.ndarray):
        try:
            return np.stack(v)
        except ValueError:
            pass
    return v


def _col_from_arrow(col):
    try:
        return col.to_numpy(zero_copy_only=False)
    except Exception:
        return np.asarray(col.to_pylist(), dtype=object)


def to_batch(b: Block, fmt: Optional[str]):
    if fmt in (None, "default", "numpy"):
        return b
    if fmt == "pandas":
        import pandas as pd

        cols = {}
        for k, v in b.items():
            cols[k] = list(v) if v.ndim > 1 else v
        return pd.DataFrame(cols)
    if fmt in ("pyarrow", "arrow"):
        import pyarrow as pa

        return pa.table({k: (pa.array(list(v)) if v.ndim > 1 else v) for k, v in b.items()})
    raise ValueError(f"unknown batch_format {fmt!r}")


def batches(b: Block, batch_size: Optional[int]) -> Iterator[Block]:
    n = num_rows(b)
    if batch_size is None or batch_size >= n:
        yield b
        return
    for s in range(0, n, batch_size):
        yield slice_block(b, s, min(n, s + batch_size))


def schema_of(b: Block) -> Dict[str, Any]:
    return {k: (str(v.dtype) if v.ndim == 1 else f"{v.dtype}{tuple(v.shape[1:])}") for k, v in b.items()}
