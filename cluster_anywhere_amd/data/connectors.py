"""Database / lakehouse connectors spoken over their public HTTP protocols, so they
need no client library (none of clickhouse-connect, delta-sharing,
databricks-sql-connector or google-cloud-bigquery is in the image):

* :func:`read_clickhouse`  - ClickHouse HTTP interface (``POST /?database=``,
  ``FORMAT Parquet``), split into ORDER BY / LIMIT / OFFSET read tasks.
  Reference: python/ray/data/_internal/datasource/clickhouse_datasource.py.
* :func:`read_delta_sharing_tables` - the open Delta Sharing REST protocol
  (profile file -> ``POST .../tables/{t}/query`` -> NDJSON ``file`` actions ->
  pre-signed Parquet URLs), one read task per data file, partition values added
  as columns. Reference: datasource/delta_sharing_datasource.py.
* :func:`read_databricks_tables` - Databricks SQL Statement Execution API
  (``POST /api/2.0/sql/statements`` with ``ARROW_STREAM`` + ``EXTERNAL_LINKS``,
  polling while PENDING / RUNNING), one read task per result chunk.
  Reference: datasource/databricks_uc_datasource.py.
* :func:`read_mongo` - pymongo (in the image; pymongoarrow is not), ``_id``-range
  partitions, documents -> Arrow. Reference: datasource/mongo_datasource.py.
* :func:`read_bigquery` - BigQuery REST (``tables.get`` for the schema,
  ``tabledata.list`` pages, or ``jobs.query`` for a query), rows typed from the
  schema. Reference: datasource/bigquery_datasource.py (which uses the storage
  read API through the client library).

Endpoints and credentials follow each service's conventions (DSN / profile file
/ ``DATABRICKS_HOST`` + ``DATABRICKS_TOKEN`` / ``GOOGLE_OAUTH_ACCESS_TOKEN``,
with ``BIGQUERY_API_ENDPOINT`` to point at another server). The tests run each
connector against a local HTTP server that implements the protocol.
"""
from __future__ import annotations

import io
import json
import math
import os
import time
import urllib.parse
from typing import Any, Dict, List, Optional

from . import block as B
from .dataset import Dataset


def _http(method: str, url: str, *, headers=None, data=None, json_body=None, timeout: float = 60.0) -> bytes:
    import requests

    r = requests.request(method, url, headers=headers or {}, data=data, json=json_body, timeout=timeout)
    if r.status_code >= 400:
        raise RuntimeError(f"{method} {url} -> HTTP {r.status_code}: {r.text[:500]}")
    return r.content


def _read_ds(tasks) -> Dataset:
    return Dataset(("read", list(tasks)))


def _arrow_from_parquet(raw: bytes):
    import pyarrow.parquet as pq

    return pq.read_table(io.BytesIO(raw))


# ----------------------------------------------------------------- ClickHouse
def _parse_dsn(dsn: str):
    u = urllib.parse.urlparse(dsn)
    scheme = "https" if u.scheme.endswith("https") else "http"
    host = u.hostname or "localhost"
    port = u.port or (8443 if scheme == "https" else 8123)
    db = (u.path or "/").lstrip("/") or "default"
    q = dict(urllib.parse.parse_qsl(u.query))
    return f"{scheme}://{host}:{port}", db, u.username, u.password, q


def read_clickhouse(*, table: str, dsn: str, columns: Optional[List[str]] = None, filter: Optional[str] = None,
                    order_by: Optional[tuple] = None, client_settings: Optional[Dict[str, Any]] = None,
                    client_kwargs: Optional[Dict[str, Any]] = None, concurrency: Optional[int] = None,
                    override_num_blocks: Optional[int] = None, ray_remote_args=None) -> Dataset:
    """``SELECT columns FROM table [WHERE filter] [ORDER BY ...]`` over the HTTP
    interface. Parallel blocks need ``order_by`` (a stable split); without it the
    table is read as one block. ``order_by=(["col", ...], descending)``."""
    base, db, user, pwd, q = _parse_dsn(dsn)
    settings = dict(q)
    settings.update(client_settings or {})
    headers = {}
    if user:
        headers["X-ClickHouse-User"] = user
    if pwd:
        headers["X-ClickHouse-Key"] = pwd
    params = {"database": db, **{k: str(v) for k, v in settings.items()}}
    url = base + "/?" + urllib.parse.urlencode(params)
    cols = ", ".join(columns) if columns else "*"
    where = f" WHERE {filter}" if filter else ""
    order = ""
    if order_by:
        ocols, desc = order_by if isinstance(order_by, tuple) and len(order_by) == 2 and \
            isinstance(order_by[0], (list, tuple)) else (order_by, False)
        order = " ORDER BY " + ", ".join(ocols) + (" DESC" if desc else "")
    base_q = f"SELECT {cols} FROM {table}{where}{order}"
    nblocks = 1
    total = None
    if order:
        total = int(_http("POST", url, headers=headers, data=f"SELECT count() FROM {table}{where} FORMAT TSV"
                          .encode()).decode().strip() or 0)
        nblocks = max(1, min(override_num_blocks or max(1, math.ceil(total / 100_000)), max(1, total)))

    def task(limit=None, offset=None):
        sql = base_q + (f" LIMIT {limit} OFFSET {offset}" if limit is not None else "") + " FORMAT Parquet"
        return B.from_batch(_arrow_from_parquet(_http("POST", url, headers=headers, data=sql.encode())))

    if nblocks == 1:
        return _read_ds([lambda: task()])
    per = math.ceil(total / nblocks)
    return _read_ds([(lambda o=o: task(per, o)) for o in range(0, total, per)])


# --------------------------------------------------------------- Delta Sharing
def _delta_profile(path: str) -> Dict[str, Any]:
    with open(path) as f:
        prof = json.load(f)
    if "endpoint" not in prof:
        raise ValueError(f"{path}: not a Delta Sharing profile (no endpoint)")
    return prof


def read_delta_sharing_tables(url: str, *, limit: Optional[int] = None, version: Optional[int] = None,
                              timestamp: Optional[str] = None, json_predicate_hints: Optional[str] = None,
                              ray_remote_args=None, concurrency: Optional[int] = None,
                              override_num_blocks: Optional[int] = None) -> Dataset:
    """``url`` = ``<profile file>#<share>.<schema>.<table>``."""
    if "#" not in url:
        raise ValueError("url must be '<profile-file>#<share>.<schema>.<table>'")
    prof_path, coords = url.split("#", 1)
    share, schema, table = coords.split(".", 2)
    prof = _delta_profile(prof_path)
    endpoint = prof["endpoint"].rstrip("/")
    headers = {"Content-Type": "application/json; charset=utf-8"}
    if prof.get("bearerToken"):
        headers["Authorization"] = f"Bearer {prof['bearerToken']}"
    body: Dict[str, Any] = {}
    if limit is not None:
        body["limitHint"] = int(limit)
    if version is not None:
        body["version"] = int(version)
    if timestamp is not None:
        body["timestamp"] = timestamp
    if json_predicate_hints is not None:
        body["jsonPredicateHints"] = json_predicate_hints
    q = urllib.parse.quote
    raw = _http("POST", f"{endpoint}/shares/{q(share)}/schemas/{q(schema)}/tables/{q(table)}/query",
                headers=headers, json_body=body).decode()
    files = []
    for line in raw.splitlines():
        if not line.strip():
            continue
        obj = json.loads(line)
        if "file" in obj:
            files.append(obj["file"])
    if not files:
        from .read_api import from_items

        return from_items([])

    def task(f):
        import pyarrow as pa

        t = _arrow_from_parquet(_http("GET", f["url"]))
        for k, v in (f.get("partitionValues") or {}).items():
            if k not in t.column_names:
                t = t.append_column(k, pa.array([v] * t.num_rows))
        return B.from_batch(t)

    ds = _read_ds([(lambda f=f: task(f)) for f in files])
    if limit is not None:
        ds = ds.limit(int(limit))
    return ds


# ------------------------------------------------------------------ Databricks
def read_databricks_tables(*, warehouse_id: str, table: Optional[str] = None, query: Optional[str] = None,
                           catalog: Optional[str] = None, schema: Optional[str] = None,
                           parallelism: int = -1, ray_remote_args=None,
                           override_num_blocks: Optional[int] = None) -> Dataset:
    """Runs ``query`` (or ``SELECT * FROM table``) on a SQL warehouse; credentials
    from ``DATABRICKS_HOST`` / ``DATABRICKS_TOKEN``."""
    if (table is None) == (query is None):
        raise ValueError("give exactly one of table / query")
    host = os.environ.get("DATABRICKS_HOST")
    token = os.environ.get("DATABRICKS_TOKEN")
    if not host or not token:
        raise ValueError("set DATABRICKS_HOST and DATABRICKS_TOKEN")
    if not host.startswith("http"):
        host = "https://" + host
    host = host.rstrip("/")
    headers = {"Authorization": f"Bearer {token}", "Content-Type": "application/json"}
    body = {"statement": query or f"SELECT * FROM {table}", "warehouse_id": warehouse_id, "wait_timeout": "10s",
            "on_wait_timeout": "CONTINUE", "disposition": "EXTERNAL_LINKS", "format": "ARROW_STREAM"}
    if catalog:
        body["catalog"] = catalog
    if schema:
        body["schema"] = schema
    resp = json.loads(_http("POST", f"{host}/api/2.0/sql/statements/", headers=headers, json_body=body))
    sid = resp["statement_id"]
    deadline = time.monotonic() + 3600
    while resp["status"]["state"] in ("PENDING", "RUNNING"):
        if time.monotonic() > deadline:
            raise TimeoutError(f"statement {sid} still {resp['status']['state']}")
        time.sleep(0.5)
        resp = json.loads(_http("GET", f"{host}/api/2.0/sql/statements/{sid}", headers=headers))
    state = resp["status"]["state"]
    if state != "SUCCEEDED":
        raise RuntimeError(f"statement {sid} {state}: {resp['status'].get('error')}")
    chunks = (resp.get("manifest") or {}).get("chunks") or [{"chunk_index": 0}]
    first = {l["chunk_index"]: l["external_link"] for l in (resp.get("result") or {}).get("external_links", [])}

    def task(i):
        import pyarrow.ipc as ipc

        link = first.get(i)
        if link is None:
            r = json.loads(_http("GET", f"{host}/api/2.0/sql/statements/{sid}/result/chunks/{i}", headers=headers))
            link = r["external_links"][0]["external_link"]
        raw = _http("GET", link)  # pre-signed: no Databricks credentials on it
        return B.from_batch(ipc.open_stream(io.BytesIO(raw)).read_all())

    return _read_ds([(lambda i=c["chunk_index"]: task(i)) for c in chunks])


# -------------------------------------------------------------------- BigQuery
def _bq_cast(v, typ: str):
    if v is None:
        return None
    typ = typ.upper()
    if typ in ("INTEGER", "INT64"):
        return int(v)
    if typ in ("FLOAT", "FLOAT64", "NUMERIC", "BIGNUMERIC"):
        return float(v)
    if typ in ("BOOLEAN", "BOOL"):
        return v in (True, "true", "TRUE", "1")
    if typ == "TIMESTAMP":
        return float(v)
    return v


def read_bigquery(project_id: str, dataset: Optional[str] = None, query: Optional[str] = None, *,
                  parallelism: int = -1, ray_remote_args=None, concurrency: Optional[int] = None,
                  override_num_blocks: Optional[int] = None, page_size: int = 10000) -> Dataset:
    """``dataset`` = ``"<dataset>.<table>"`` (table read) or ``query`` (standard SQL)."""
    if (dataset is None) == (query is None):
        raise ValueError("give exactly one of dataset / query")
    api = os.environ.get("BIGQUERY_API_ENDPOINT", "https://bigquery.googleapis.com").rstrip("/") + "/bigquery/v2"
    token = os.environ.get("GOOGLE_OAUTH_ACCESS_TOKEN")
    if not token:
        raise ValueError("set GOOGLE_OAUTH_ACCESS_TOKEN (an OAuth2 access token for BigQuery)")
    headers = {"Authorization": f"Bearer {token}"}
    if query is not None:
        r = json.loads(_http("POST", f"{api}/projects/{project_id}/queries", headers=headers,
                             json_body={"query": query, "useLegacySql": False, "maxResults": page_size}))
        job = r["jobReference"]["jobId"]
        while not r.get("jobComplete", True):
            time.sleep(0.5)
            r = json.loads(_http("GET", f"{api}/projects/{project_id}/queries/{job}?maxResults={page_size}",
                                 headers=headers))
        fields = r["schema"]["fields"]
        pages = [r.get("rows", [])]
        tok = r.get("pageToken")
        while tok:
            r = json.loads(_http("GET", f"{api}/projects/{project_id}/queries/{job}?pageToken="
                                 f"{urllib.parse.quote(tok)}&maxResults={page_size}", headers=headers))
            pages.append(r.get("rows", []))
            tok = r.get("pageToken")
        loaders = [(lambda rows=rows: rows) for rows in pages]
    else:
        ds_id, table = dataset.split(".", 1)
        base = f"{api}/projects/{project_id}/datasets/{ds_id}/tables/{table}"
        meta = json.loads(_http("GET", base, headers=headers))
        fields = meta["schema"]["fields"]
        n = int(meta.get("numRows", 0))
        per = max(1, page_size)
        loaders = [(lambda s=s: json.loads(_http("GET", f"{base}/data?startIndex={s}&maxResults={per}",
                                                 headers=headers)).get("rows", []))
                   for s in range(0, max(n, 1), per)]

    names = [f["name"] for f in fields]
    types = [f.get("type", "STRING") for f in fields]

    def task(load):
        rows = load()
        cols = {nm: [_bq_cast(r["f"][i]["v"], types[i]) for r in rows] for i, nm in enumerate(names)}
        import pyarrow as pa

        return B.from_batch(pa.table(cols))

    return _read_ds([(lambda ld=ld: task(ld)) for ld in loaders])




# --------------------------------------------------------------------- MongoDB
def _docs_to_block(docs, schema=None):
    import pyarrow as pa

    if not docs:
        return B.from_batch(pa.table({}))
    cols: Dict[str, list] = {}
    keys = list(schema) if schema else []
    for d in docs:
        for k in d:
            if k not in cols and (not schema or k in schema):
                cols[k] = []
                if not schema:
                    keys.append(k)
    out = {}
    for k in keys:
        vals = [d.get(k) for d in docs]
        if vals and all(type(v).__name__ == "ObjectId" or v is None for v in vals):
            vals = [str(v) if v is not None else None for v in vals]
        out[k] = vals
    if schema:
        return B.from_batch(pa.table({k: pa.array(out[k], type=schema[k]) for k in keys}))
    return B.from_batch(pa.table(out))


def read_mongo(uri: str, database: str, collection: str, *, pipeline: Optional[List[Dict]] = None,
               schema: Optional[Dict[str, Any]] = None, parallelism: int = -1, ray_remote_args=None,
               concurrency: Optional[int] = None, override_num_blocks: Optional[int] = None,
               **mongo_args) -> Dataset:
    """Reads ``collection`` (through ``pipeline`` when given) with pymongo. The
    collection is cut into ``_id`` ranges (boundaries from a sorted ``_id``
    projection sampled every N documents) and each read task runs
    ``[{$match: {_id: range}}] + pipeline``; ObjectIds become strings. ``schema``:
    optional ``{column: pyarrow type}`` (pymongoarrow is not in the image)."""
    import pymongo

    pipeline = list(pipeline or [])

    def client():
        return pymongo.MongoClient(uri, **mongo_args)

    with client() as c:
        coll = c[database][collection]
        n = coll.estimated_document_count()
        k = max(1, min(n, override_num_blocks or (parallelism if parallelism > 0 else max(1, math.ceil(n / 100_000)))))
        bounds = []
        if k > 1:
            step = max(1, n // k)
            ids = [d["_id"] for d in coll.find({}, {"_id": 1}).sort("_id", 1)]
            bounds = [ids[i] for i in range(step, len(ids), step)][: k - 1]
    edges = [None] + bounds + [None]

    def task(lo, hi):
        m: Dict[str, Any] = {}
        if lo is not None:
            m["$gte"] = lo
        if hi is not None:
            m["$lt"] = hi
        stages = ([{"$match": {"_id": m}}] if m else []) + [{"$sort": {"_id": 1}}] + pipeline
        with client() as c:
            docs = list(c[database][collection].aggregate(stages))
        return _docs_to_block(docs, schema)

    return _read_ds([(lambda lo=lo, hi=hi: task(lo, hi)) for lo, hi in zip(edges[:-1], edges[1:])])




# ---------------------------------------------------------------------- videos
def _y4m_frames(raw: bytes):
    import numpy as np

    nl = raw.index(b"\n")
    hdr = raw[:nl].split()
    if hdr[0] != b"YUV4MPEG2":
        raise ValueError("not a YUV4MPEG2 stream")
    w = h = None
    cs = b"420"
    for t in hdr[1:]:
        if t[:1] == b"W":
            w = int(t[1:])
        elif t[:1] == b"H":
            h = int(t[1:])
        elif t[:1] == b"C":
            cs = t[1:]
    sub = 1 if cs.startswith(b"444") else 2
    cw, ch = -(-w // sub), -(-h // sub)
    fsize = w * h + 2 * cw * ch
    pos = nl + 1
    while pos < len(raw):
        e = raw.index(b"\n", pos)
        if not raw[pos:e].startswith(b"FRAME"):
            raise ValueError("bad Y4M frame header")
        buf = np.frombuffer(raw, np.uint8, fsize, e + 1)
        pos = e + 1 + fsize
        y = buf[: w * h].reshape(h, w).astype(np.float32)
        u = buf[w * h: w * h + cw * ch].reshape(ch, cw).astype(np.float32)
        v = buf[w * h + cw * ch:].reshape(ch, cw).astype(np.float32)
        if sub == 2:
            u = u.repeat(2, 0).repeat(2, 1)[:h, :w]
            v = v.repeat(2, 0).repeat(2, 1)[:h, :w]
        c, d, e_ = y - 16.0, u - 128.0, v - 128.0  # BT.601 limited range
        rgb = np.stack([1.164 * c + 1.596 * e_, 1.164 * c - 0.392 * d - 0.813 * e_, 1.164 * c + 2.017 * d], -1)
        yield np.clip(rgb + 0.5, 0, 255).astype(np.uint8)


def _avi_frames(raw: bytes):
    """RIFF AVI with Motion-JPEG ('00dc' JPEG chunks) or uncompressed 24-bit DIB frames."""
    import struct

    import numpy as np
    from PIL import Image

    if raw[:4] != b"RIFF" or raw[8:12] != b"AVI ":
        raise ValueError("not an AVI file")
    w = h = 0
    i = raw.find(b"strf")
    if i >= 0:
        w, h = struct.unpack("<ii", raw[i + 12:i + 20])
    m = raw.find(b"movi")
    if m < 0:
        raise ValueError("AVI without a movi list")
    pos = m + 4
    while pos + 8 <= len(raw):
        cid, size = raw[pos:pos + 4], struct.unpack("<I", raw[pos + 4:pos + 8])[0]
        data = raw[pos + 8:pos + 8 + size]
        if cid == b"LIST":
            pos += 12
            continue
        if cid == b"idx1":
            break
        if cid[2:] in (b"dc", b"db") and size:
            if data[:2] == b"\xff\xd8":
                yield np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
            else:
                stride = (w * 3 + 3) & ~3
                img = np.frombuffer(data, np.uint8, stride * abs(h)).reshape(abs(h), stride)[:, : w * 3]
                img = img.reshape(abs(h), w, 3)[:, :, ::-1]
                yield np.ascontiguousarray(img[::-1] if h > 0 else img)
        pos += 8 + size + (size & 1)


def _pil_frames(raw: bytes):
    import numpy as np
    from PIL import Image, ImageSequence

    for fr in ImageSequence.Iterator(Image.open(io.BytesIO(raw))):
        yield np.asarray(fr.convert("RGB"))


_VIDEO_DECODERS = {".y4m": _y4m_frames, ".avi": _avi_frames, ".gif": _pil_frames, ".webp": _pil_frames,
                   ".png": _pil_frames, ".apng": _pil_frames}


def read_videos(paths, *, include_paths: bool = False, file_extensions: Optional[List[str]] = None,
                override_num_blocks: Optional[int] = None, concurrency: Optional[int] = None,
                ray_remote_args=None, **kw) -> Dataset:
    """One row per frame: ``{"frame": uint8 [H, W, 3], "frame_index": int}`` (+ ``path``).
    Decoded here without a codec library: YUV4MPEG2 (``.y4m``), AVI with
    Motion-JPEG or uncompressed frames, and animated GIF / WebP / PNG. Codec-
    compressed containers (H.264 / HEVC / VP9 in .mp4 / .mkv / .webm) need a video
    decoder, which this image does not have: they raise NotImplementedError."""
    from .read_api import _expand, _file_ds

    exts = file_extensions or list(_VIDEO_DECODERS) + [".mp4", ".mkv", ".mov", ".webm"]
    files = _expand(paths, exts)

    def rd(f):
        import numpy as np

        ext = os.path.splitext(f)[1].lower()
        dec = _VIDEO_DECODERS.get(ext)
        if dec is None:
            raise NotImplementedError(f"{f}: decoding {ext} needs a video codec library (not in this image); "
                                      f"supported here: {sorted(_VIDEO_DECODERS)}")
        with open(f, "rb") as fh:
            raw = fh.read()
        frames = list(dec(raw))
        out = {"frame": np.stack(frames) if frames else np.zeros((0, 0, 0, 3), np.uint8),
               "frame_index": np.arange(len(frames), dtype=np.int64)}
        if include_paths:
            out["path"] = np.array([f] * len(frames), dtype=object)
        return out

    return _file_ds(files, rd)


__all__ = ["read_clickhouse", "read_delta_sharing_tables", "read_databricks_tables", "read_bigquery", "read_mongo",
           "read_videos"]


# ------------------------------------------------------------------------ sinks
from .datasource import Datasink as _Datasink  # noqa: E402


def _plain_value(v):
    import numpy as _np

    if isinstance(v, _np.generic):
        return v.item()
    if isinstance(v, _np.ndarray):
        return v.tolist()
    return v


class MongoDatasink(_Datasink):
    """``Dataset.write_mongo``: each write task opens its own client and inserts
    its blocks' rows (``insert_many``, unordered); returns the count inserted."""

    def __init__(self, uri: str, database: str, collection: str, **mongo_args):
        self.uri, self.database, self.collection = uri, database, collection
        self.mongo_args = mongo_args

    def write(self, blocks, ctx) -> int:
        import pymongo

        n = 0
        client = pymongo.MongoClient(self.uri, **self.mongo_args)
        try:
            coll = client[self.database][self.collection]
            for blk in blocks:
                docs = [{k: _plain_value(v) for k, v in r.items()} for r in B.to_arrow(blk).to_pylist()]
                if docs:
                    n += len(coll.insert_many(docs, ordered=False).inserted_ids)
        finally:
            client.close()
        return n


_BQ_TYPES = (("bool", "BOOLEAN"), ("int", "INTEGER"), ("uint", "INTEGER"), ("float", "FLOAT"),
             ("double", "FLOAT"), ("timestamp", "TIMESTAMP"), ("datetime", "TIMESTAMP"), ("date", "DATE"),
             ("binary", "BYTES"), ("bytes", "BYTES"))


def _bq_type(t: str) -> str:
    t = str(t).lower()
    for prefix, bq in _BQ_TYPES:
        if t.startswith(prefix):
            return bq
    return "STRING"


class BigQueryDatasink(_Datasink):
    """``Dataset.write_bigquery`` over the REST API (the client library is not in
    the image): ``on_write_start`` drops the table when ``overwrite_table`` and
    creates it from the Dataset schema; write tasks stream rows with
    ``tabledata.insertAll`` (500 rows per request, 429 / 5xx retried with backoff)."""

    ROWS_PER_REQUEST = 500

    def __init__(self, project_id: str, dataset: str, schema: Optional[Dict[str, str]], *,
                 max_retry_cnt: int = 10, overwrite_table: bool = True):
        if "." not in dataset:
            raise ValueError('dataset must be "<dataset>.<table>"')
        self.project_id = project_id
        self.dataset_id, self.table = dataset.split(".", 1)
        self.schema = dict(schema or {})
        self.max_retry_cnt = max_retry_cnt
        self.overwrite_table = overwrite_table
        # resolved on the driver: the write tasks' workers need not share its environment
        self._endpoint = os.environ.get("BIGQUERY_API_ENDPOINT", "https://bigquery.googleapis.com").rstrip("/")
        self._token = os.environ.get("GOOGLE_OAUTH_ACCESS_TOKEN")
        if not self._token:
            raise ValueError("set GOOGLE_OAUTH_ACCESS_TOKEN (an OAuth2 access token for BigQuery)")

    def _api(self):
        return (f"{self._endpoint}/bigquery/v2/projects/{self.project_id}/datasets/{self.dataset_id}",
                {"Authorization": f"Bearer {self._token}"})

    def _call(self, method, url, headers, body=None, ok=()):
        """JSON response of one REST call; 429 / 5xx retried with backoff; status
        codes in ``ok`` (e.g. 404 on a DELETE) are not errors."""
        import requests

        for attempt in range(self.max_retry_cnt + 1):
            r = requests.request(method, url, headers=headers, json=body, timeout=120)
            if (r.status_code == 429 or r.status_code >= 500) and attempt < self.max_retry_cnt:
                time.sleep(min(8.0, 0.25 * (2 ** attempt)))
                continue
            if r.status_code >= 400 and r.status_code not in ok:
                raise RuntimeError(f"BigQuery {method} {url} -> HTTP {r.status_code}: {r.text[:500]}")
            return r.json() if r.content and r.status_code < 300 else {}

    def on_write_start(self) -> None:
        base, headers = self._api()
        if self.overwrite_table:
            self._call("DELETE", f"{base}/tables/{self.table}", headers, ok=(404,))
        fields = [{"name": k, "type": _bq_type(v), "mode": "NULLABLE"} for k, v in self.schema.items()]
        self._call("POST", f"{base}/tables", headers,
                   {"tableReference": {"projectId": self.project_id, "datasetId": self.dataset_id,
                                       "tableId": self.table}, "schema": {"fields": fields}},
                   ok=(409,))  # 409: it exists (overwrite_table=False) -> append

    def write(self, blocks, ctx) -> int:
        import base64

        base, headers = self._api()
        n = 0
        for blk in blocks:
            rows = B.to_arrow(blk).to_pylist()
            for s in range(0, len(rows), self.ROWS_PER_REQUEST):
                chunk = []
                for r in rows[s:s + self.ROWS_PER_REQUEST]:
                    row = {}
                    for k, v in r.items():
                        v = _plain_value(v)
                        if isinstance(v, (bytes, bytearray)):
                            v = base64.b64encode(bytes(v)).decode()
                        elif hasattr(v, "isoformat"):
                            v = v.isoformat()
                        row[k] = v
                    chunk.append({"json": row})
                out = self._call("POST", f"{base}/tables/{self.table}/insertAll", headers,
                                 {"rows": chunk, "skipInvalidRows": False, "ignoreUnknownValues": False})
                if out.get("insertErrors"):
                    raise RuntimeError(f"BigQuery insertAll rejected rows: {out['insertErrors'][:3]}")
                n += len(chunk)
        return n
