"""Preprocessors (reference: python/ray/data/preprocessors/): fit on a Dataset
(aggregations run distributed), transform with map_batches."""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import numpy as np


class Preprocessor:
    _is_fittable = True

    def __init__(self):
        self.stats_: Optional[Dict[str, Any]] = None

    def fit(self, ds):
        if self._is_fittable:
            self.stats_ = self._fit(ds)
        return self

    def fit_transform(self, ds):
        return self.fit(ds).transform(ds)

    def transform(self, ds):
        if self._is_fittable and self.stats_ is None:
            raise RuntimeError(f"{type(self).__name__} must be fit before transform")
        fn = self._transform_numpy
        return ds.map_batches(fn, batch_format="numpy", batch_size=None)

    def transform_batch(self, batch: Dict[str, np.ndarray]):
        return self._transform_numpy(dict(batch))

    def _fit(self, ds):
        return {}

    def _transform_numpy(self, batch):
        raise NotImplementedError


class StandardScaler(Preprocessor):
    def __init__(self, columns: List[str], ddof: int = 0):
        super().__init__()
        self.columns = columns
        self.ddof = ddof

    def _fit(self, ds):
        from .aggregate import Mean, Std

        aggs = [a for c in self.columns for a in (Mean(c), Std(c, ddof=self.ddof))]
        r = ds.aggregate(*aggs)
        return {c: (r[f"mean({c})"], r[f"std({c})"]) for c in self.columns}

    def _transform_numpy(self, batch):
        out = dict(batch)
        for c in self.columns:
            m, s = self.stats_[c]
            out[c] = (batch[c] - m) / (s if s else 1.0)
        return out


class MinMaxScaler(Preprocessor):
    def __init__(self, columns: List[str]):
        super().__init__()
        self.columns = columns

    def _fit(self, ds):
        from .aggregate import Max, Min

        r = ds.aggregate(*[a for c in self.columns for a in (Min(c), Max(c))])
        return {c: (r[f"min({c})"], r[f"max({c})"]) for c in self.columns}

    def _transform_numpy(self, batch):
        out = dict(batch)
        for c in self.columns:
            lo, hi = self.stats_[c]
            rng = (hi - lo) or 1.0
            out[c] = (batch[c] - lo) / rng
        return out


class LabelEncoder(Preprocessor):
    def __init__(self, label_column: str):
        super().__init__()
        self.label_column = label_column

    def _fit(self, ds):
        vals = sorted(ds.unique(self.label_column))
        return {v: i for i, v in enumerate(vals)}

    def _transform_numpy(self, batch):
        out = dict(batch)
        out[self.label_column] = np.asarray([self.stats_[v.item() if hasattr(v, "item") else v]
                                             for v in batch[self.label_column]])
        return out


class OneHotEncoder(Preprocessor):
    def __init__(self, columns: List[str]):
        super().__init__()
        self.columns = columns

    def _fit(self, ds):
        return {c: sorted(ds.unique(c)) for c in self.columns}

    def _transform_numpy(self, batch):
        out = dict(batch)
        for c in self.columns:
            cats = self.stats_[c]
            idx = {v: i for i, v in enumerate(cats)}
            oh = np.zeros((len(batch[c]), len(cats)), dtype=np.int8)
            for r, v in enumerate(batch[c]):
                v = v.item() if hasattr(v, "item") else v
                if v in idx:
                    oh[r, idx[v]] = 1
            out[c] = oh
        return out


class Concatenator(Preprocessor):
    _is_fittable = False

    def __init__(self, columns: Optional[List[str]] = None, output_column_name: str = "concat_out",
                 dtype=np.float32, exclude: Optional[List[str]] = None):
        super().__init__()
        self.columns = columns
        self.output_column_name = output_column_name
        self.dtype = dtype
        self.exclude = exclude or []

    def _transform_numpy(self, batch):
        cols = self.columns or [k for k in batch if k not in self.exclude]
        parts = [np.asarray(batch[c], dtype=self.dtype).reshape(len(batch[c]), -1) for c in cols]
        out = {k: v for k, v in batch.items() if k not in cols}
        out[self.output_column_name] = np.concatenate(parts, axis=1)
        return out


class SimpleImputer(Preprocessor):
    def __init__(self, columns: List[str], strategy: str = "mean", fill_value=None):
        super().__init__()
        self.columns, self.strategy, self.fill_value = columns, strategy, fill_value

    def _fit(self, ds):
        if self.strategy == "constant":
            return {c: self.fill_value for c in self.columns}
        from .aggregate import Mean

        r = ds.aggregate(*[Mean(c) for c in self.columns])
        return {c: r[f"mean({c})"] for c in self.columns}

    def _transform_numpy(self, batch):
        out = dict(batch)
        for c in self.columns:
            v = np.asarray(batch[c], dtype=np.float64).copy()
            v[np.isnan(v)] = self.stats_[c]
            out[c] = v
        return out


class Chain(Preprocessor):
    def __init__(self, *preprocessors: Preprocessor):
        super().__init__()
        self.preprocessors = preprocessors

    def fit(self, ds):
        for p in self.preprocessors:
            ds = p.fit_transform(ds)
        self.stats_ = {}
        return self

    def transform(self, ds):
        for p in self.preprocessors:
            ds = p.transform(ds)
        return ds

    def transform_batch(self, batch):
        for p in self.preprocessors:
            batch = p.transform_batch(batch)
        return batch


class BatchMapper(Preprocessor):
    _is_fittable = False

    def __init__(self, fn, batch_format="numpy", batch_size=None):
        super().__init__()
        self.fn = fn

    def _transform_numpy(self, batch):
        return self.fn(batch)
