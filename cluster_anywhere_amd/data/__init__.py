"""Distributed streaming datasets (reference: python/ray/data/)."""
from . import preprocessors
from .aggregate import AbsMax, AggregateFn, Count, Max, Mean, Min, Std, Sum
from .context import DataContext
from .dataset import ActorPoolStrategy, Dataset, GroupedData, MaterializedDataset, Schema, TaskPoolStrategy
from .iterator import DataIterator
from .datasource import (BlockBasedFileDatasink, BlockMetadata, Datasink, Datasource, FileShuffleConfig, ReadTask,
                         RowBasedFileDatasink, TaskContext, WriteResult)
from .execution_options import ExecutionOptions, ExecutionResources
from .preprocessors import Preprocessor

DatasetIterator = DataIterator  # the reference's older name of the iterator class
DatasetContext = DataContext  # ditto for the context
NodeIdStr = str  # node ids are hex strings


class TFXReadOptions:
    """``read_tfrecords(tfx_read_options=...)`` (reference: tfrecords_datasource.py):
    accepted for parity; the own tf.train.Example codec needs no TFX batching."""

    def __init__(self, batch_size: int = 2048, auto_infer_schema: bool = True):
        self.batch_size = batch_size
        self.auto_infer_schema = auto_infer_schema
from .read_api import (
    from_arrow,
    from_arrow_refs,
    from_blocks,
    from_huggingface,
    from_items,
    from_numpy,
    from_numpy_refs,
    from_pandas,
    from_pandas_refs,
    from_torch,
    range,
    range_tensor,
    read_binary_files,
    read_csv,
    read_datasource,
    read_images,
    read_json,
    read_numpy,
    read_parquet,
    read_text,
)
from .read_api import (  # noqa: E402  (formats without extra deps + honest stubs)
    read_parquet_bulk,
    read_tfrecords,
    read_webdataset,
    read_sql,
    from_dask,
    from_spark,
    from_modin,
    from_mars,
    from_tf,
    read_bigquery,
    read_mongo,
    read_lance,
    read_iceberg,
    read_hudi,
    read_delta_sharing_tables,
    read_databricks_tables,
    read_clickhouse,
    read_avro,
    read_audio,
    read_videos,
)

__all__ = [
    "Dataset", "MaterializedDataset", "GroupedData", "DataIterator", "DataContext", "Schema",
    "ActorPoolStrategy", "TaskPoolStrategy", "AggregateFn", "Count", "Sum", "Min", "Max", "Mean",
    "Std", "AbsMax", "range", "range_tensor", "from_items", "from_blocks", "from_numpy",
    "from_pandas", "from_arrow", "from_numpy_refs", "from_pandas_refs", "from_arrow_refs",
    "from_torch", "from_huggingface", "read_parquet", "read_csv", "read_json", "read_text",
    "read_numpy", "read_binary_files", "read_images", "read_datasource", "preprocessors",
    "Datasource", "ReadTask", "Datasink", "BlockBasedFileDatasink", "RowBasedFileDatasink", "BlockMetadata",
    "TaskContext", "WriteResult", "FileShuffleConfig", "ExecutionOptions", "ExecutionResources",
    "DatasetIterator", "DatasetContext", "NodeIdStr", "Preprocessor", "TFXReadOptions",
] + ['read_parquet_bulk', 'read_tfrecords', 'read_webdataset', 'read_sql', 'from_dask', 'from_spark', 'from_modin', 'from_mars', 'from_tf', 'read_bigquery', 'read_mongo', 'read_lance', 'read_iceberg', 'read_hudi', 'read_delta_sharing_tables', 'read_databricks_tables', 'read_clickhouse', 'read_avro', 'read_audio', 'read_videos']


def __getattr__(name):
    # ``data.llm`` imports pydantic / the LLM stack: load it on first use only
    if name == "llm":
        import importlib

        return importlib.import_module(".llm", __name__)
    raise AttributeError(name)
