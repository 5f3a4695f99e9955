"""HTTP-protocol connectors (data/connectors.py) against a local server that
implements each protocol: ClickHouse HTTP interface (FORMAT Parquet), Delta
Sharing REST (NDJSON file actions + pre-signed Parquet URLs), Databricks SQL
Statement Execution (PENDING -> SUCCEEDED, ARROW_STREAM external links, chunks),
BigQuery REST (tables.get + tabledata.list pages, jobs.query). Reference tests:
python/ray/data/tests/test_clickhouse.py, test_delta_sharing.py,
test_databricks_uc_datasource.py, test_bigquery.py (mocked clients there)."""
import io
import os
import json
import re
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

import pyarrow as pa
import pyarrow.ipc as ipc
import pyarrow.parquet as pq
import pytest

import cluster_anywhere_amd as ray
from cluster_anywhere_amd import data

TABLE = pa.table({"id": list(range(25)), "name": [f"n{i}" for i in range(25)], "x": [i * 0.5 for i in range(25)]})


def _parquet(t):
    b = io.BytesIO()
    pq.write_table(t, b)
    return b.getvalue()


def _arrow_stream(t):
    b = io.BytesIO()
    with ipc.new_stream(b, t.schema) as w:
        w.write_table(t)
    return b.getvalue()


class State:
    polls = 0
    auth = []
    bq_tables = {}
    bq_inserts = 0


class Handler(BaseHTTPRequestHandler):
    def log_message(self, *a):
        pass

    def _send(self, code, body, ctype="application/octet-stream"):
        if isinstance(body, (dict, list)):
            body, ctype = json.dumps(body).encode(), "application/json"
        elif isinstance(body, str):
            body = body.encode()
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def _body(self):
        n = int(self.headers.get("Content-Length", 0))
        return self.rfile.read(n) if n else b""

    def do_POST(self):
        u = urlparse(self.path)
        State.auth.append(self.headers.get("Authorization") or self.headers.get("X-ClickHouse-User"))
        body = self._body()
        if u.path == "/" and "database" in parse_qs(u.query):  # ClickHouse
            sql = body.decode()
            assert parse_qs(u.query)["database"] == ["db1"]
            if sql.startswith("SELECT count()"):
                t = TABLE.filter(pa.compute.greater_equal(TABLE["id"], 5)) if "WHERE id >= 5" in sql else TABLE
                return self._send(200, f"{t.num_rows}\n", "text/tab-separated-values")
            t = TABLE
            if "WHERE id >= 5" in sql:
                t = t.filter(pa.compute.greater_equal(t["id"], 5))
            m = re.search(r"LIMIT (\d+) OFFSET (\d+)", sql)
            if m:
                t = t.slice(int(m.group(2)), int(m.group(1)))
            if "SELECT id, name" in sql:
                t = t.select(["id", "name"])
            return self._send(200, _parquet(t))
        if u.path.startswith("/delta/shares/"):
            req = json.loads(body or b"{}")
            port = self.server.server_address[1]
            lines = [{"protocol": {"minReaderVersion": 1}}, {"metaData": {"id": "t1", "format": {"provider": "parquet"}}}]
            for part in ("a", "b"):
                lines.append({"file": {"url": f"http://127.0.0.1:{port}/files/{part}.parquet", "id": part,
                                       "partitionValues": {"part": part}, "size": 1}})
            State.delta_req = req
            return self._send(200, "\n".join(json.dumps(x) for x in lines), "application/x-ndjson")
        if u.path == "/api/2.0/sql/statements/":
            req = json.loads(body)
            State.dbx_req = req
            return self._send(200, {"statement_id": "s1", "status": {"state": "PENDING"}})
        if u.path == "/bigquery/v2/projects/p1/datasets/d1/tables":
            req = json.loads(body)
            name = req["tableReference"]["tableId"]
            if name in State.bq_tables:
                return self._send(409, {"error": {"code": 409, "message": "Already Exists"}})
            State.bq_tables[name] = {"schema": req["schema"], "rows": []}
            return self._send(200, req)
        m = re.match(r"^/bigquery/v2/projects/p1/datasets/d1/tables/(\w+)/insertAll$", u.path)
        if m:
            State.bq_inserts += 1
            if State.bq_inserts == 1:  # the first request is throttled: the sink retries
                return self._send(503, {"error": {"code": 503}})
            State.bq_tables[m.group(1)]["rows"].extend(r["json"] for r in json.loads(body)["rows"])
            return self._send(200, {"kind": "bigquery#tableDataInsertAllResponse"})
        if u.path.startswith("/bigquery/v2/projects/p1/queries"):
            return self._send(200, {"jobReference": {"jobId": "j1"}, "jobComplete": True,
                                    "schema": {"fields": [{"name": "id", "type": "INTEGER"},
                                                          {"name": "ok", "type": "BOOLEAN"}]},
                                    "rows": [{"f": [{"v": "1"}, {"v": "true"}]}], "pageToken": "t2"})
        self._send(404, "no")

    def do_DELETE(self):
        m = re.match(r"^/bigquery/v2/projects/p1/datasets/d1/tables/(\w+)$", urlparse(self.path).path)
        if m and m.group(1) in State.bq_tables:
            del State.bq_tables[m.group(1)]
            self.send_response(204)
            self.end_headers()
            return
        self._send(404, {"error": {"code": 404}})

    def do_GET(self):
        u = urlparse(self.path)
        port = self.server.server_address[1]
        if u.path.startswith("/files/"):
            part = u.path.split("/")[-1].split(".")[0]
            t = TABLE.slice(0, 10) if part == "a" else TABLE.slice(10, 15)
            return self._send(200, _parquet(t))
        if u.path == "/api/2.0/sql/statements/s1":
            State.polls += 1
            if State.polls < 2:
                return self._send(200, {"statement_id": "s1", "status": {"state": "RUNNING"}})
            return self._send(200, {"statement_id": "s1", "status": {"state": "SUCCEEDED"},
                                    "manifest": {"chunks": [{"chunk_index": 0}, {"chunk_index": 1}]},
                                    "result": {"external_links": [{"chunk_index": 0,
                                                                   "external_link": f"http://127.0.0.1:{port}/ext/0"}]}})
        if u.path == "/api/2.0/sql/statements/s1/result/chunks/1":
            return self._send(200, {"external_links": [{"chunk_index": 1, "external_link": f"http://127.0.0.1:{port}/ext/1"}]})
        if u.path.startswith("/ext/"):
            i = int(u.path.split("/")[-1])
            return self._send(200, _arrow_stream(TABLE.slice(i * 12, 12 if i == 0 else 13)))
        if u.path == "/bigquery/v2/projects/p1/datasets/d1/tables/t1":
            return self._send(200, {"numRows": "25", "schema": {"fields": [
                {"name": "id", "type": "INTEGER"}, {"name": "name", "type": "STRING"}, {"name": "x", "type": "FLOAT"}]}})
        if u.path == "/bigquery/v2/projects/p1/datasets/d1/tables/t1/data":
            q = parse_qs(u.query)
            s, n = int(q["startIndex"][0]), int(q["maxResults"][0])
            rows = [{"f": [{"v": str(i)}, {"v": f"n{i}"}, {"v": str(i * 0.5)}]} for i in range(s, min(25, s + n))]
            return self._send(200, {"rows": rows})
        if u.path == "/bigquery/v2/projects/p1/queries/j1":
            return self._send(200, {"jobComplete": True, "rows": [{"f": [{"v": "2"}, {"v": "false"}]}]})
        self._send(404, "no")


@pytest.fixture(scope="module")
def server():
    srv = ThreadingHTTPServer(("127.0.0.1", 0), Handler)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    ray.init(num_cpus=2, ignore_reinit_error=True)
    yield f"http://127.0.0.1:{srv.server_address[1]}"
    ray.shutdown()
    srv.shutdown()


def test_clickhouse(server):
    port = server.rsplit(":", 1)[1]
    dsn = f"clickhouse+http://user:pw@127.0.0.1:{port}/db1"
    ds = data.read_clickhouse(table="t", dsn=dsn, filter="id >= 5", order_by=(["id"], False),
                              override_num_blocks=4)
    rows = ds.take_all()
    assert [r["id"] for r in rows] == list(range(5, 25))
    assert ds.num_blocks() == 4 if hasattr(ds, "num_blocks") else True
    one = data.read_clickhouse(table="t", dsn=dsn, columns=["id", "name"]).take_all()
    assert len(one) == 25 and set(one[0]) == {"id", "name"}


def test_delta_sharing(server, tmp_path):
    prof = tmp_path / "p.share"
    prof.write_text(json.dumps({"shareCredentialsVersion": 1, "endpoint": server + "/delta", "bearerToken": "tok"}))
    rows = data.read_delta_sharing_tables(f"{prof}#s1.sch.t1", version=3).take_all()
    assert sorted(r["id"] for r in rows) == list(range(25))
    assert {r["part"] for r in rows} == {"a", "b"}
    assert State.delta_req == {"version": 3}
    assert "Bearer tok" in State.auth


def test_databricks(server, monkeypatch):
    monkeypatch.setenv("DATABRICKS_HOST", server)
    monkeypatch.setenv("DATABRICKS_TOKEN", "dtok")
    rows = data.read_databricks_tables(warehouse_id="w1", table="cat.sch.t", catalog="cat").take_all()
    assert sorted(r["id"] for r in rows) == list(range(25))
    assert State.dbx_req["statement"] == "SELECT * FROM cat.sch.t" and State.dbx_req["format"] == "ARROW_STREAM"
    assert State.polls >= 2
    with pytest.raises(ValueError):
        data.read_databricks_tables(warehouse_id="w1")


def test_bigquery(server, monkeypatch):
    monkeypatch.setenv("BIGQUERY_API_ENDPOINT", server)
    monkeypatch.setenv("GOOGLE_OAUTH_ACCESS_TOKEN", "gtok")
    rows = data.read_bigquery("p1", dataset="d1.t1", page_size=10).take_all()
    assert [r["id"] for r in rows] == list(range(25)) and rows[3]["x"] == 1.5 and rows[2]["name"] == "n2"
    q = data.read_bigquery("p1", query="SELECT 1").take_all()
    assert [(r["id"], r["ok"]) for r in q] == [(1, True), (2, False)]


def test_from_other_frameworks_duck_typed(server):
    import numpy as np
    import pandas as pd

    df = pd.DataFrame({"a": range(6), "b": list("abcdef")})

    class Delayed:
        def __init__(self, d):
            self.d = d

        def compute(self):
            return self.d

    class DaskLike:
        def to_delayed(self):
            return [Delayed(df.iloc[:3]), Delayed(df.iloc[3:])]

    class ModinLike:
        def _to_pandas(self):
            return df

    class SparkLike:
        def toArrow(self):
            return pa.Table.from_pandas(df, preserve_index=False)

    class TfLike:
        def as_numpy_iterator(self):
            return iter([{"x": np.float32(i)} for i in range(4)])

    assert [r["a"] for r in data.from_dask(DaskLike()).take_all()] == list(range(6))
    assert data.from_modin(ModinLike()).count() == 6
    sp = data.from_spark(SparkLike(), override_num_blocks=3)
    assert [r["b"] for r in sp.take_all()] == list("abcdef")
    assert [float(r["x"]) for r in data.from_tf(TfLike()).take_all()] == [0.0, 1.0, 2.0, 3.0]


# ---- MongoDB: a minimal OP_MSG server (hello / ping / count / find / aggregate) ----
class _MiniMongo:
    """Speaks enough of the MongoDB wire protocol (OP_MSG, plus legacy OP_QUERY
    hello) for pymongo: handshake, count, find with projection + sort, aggregate
    with $match on an _id range, $sort on _id, $project of fields."""

    def __init__(self, docs):
        import socket

        self.docs = docs
        self.sock = socket.socket()
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(16)
        self.port = self.sock.getsockname()[1]
        threading.Thread(target=self._accept, daemon=True).start()

    def _accept(self):
        while True:
            try:
                conn, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(conn,), daemon=True).start()

    @staticmethod
    def _recv(conn, n):
        buf = b""
        while len(buf) < n:
            c = conn.recv(n - len(buf))
            if not c:
                raise EOFError
            buf += c
        return buf

    def _reply(self, conn, req_id, doc, legacy):
        import struct

        import bson

        body = bson.encode(doc)
        if legacy:  # OP_REPLY
            payload = struct.pack("<iqii", 0, 0, 0, 1) + body
            op = 1
        else:
            payload = struct.pack("<I", 0) + b"\x00" + body
            op = 2013
        conn.sendall(struct.pack("<iiii", 16 + len(payload), 0, req_id, op) + payload)

    def _run(self, cmd):
        import datetime

        name = next(iter(cmd)).lower()
        if name in ("hello", "ismaster"):
            return {"ok": 1.0, "isWritablePrimary": True, "ismaster": True, "helloOk": True, "maxWireVersion": 17,
                    "minWireVersion": 0, "maxBsonObjectSize": 16 * 1024 * 1024, "maxMessageSizeBytes": 48000000,
                    "maxWriteBatchSize": 100000, "localTime": datetime.datetime.now(datetime.timezone.utc),
                    "logicalSessionTimeoutMinutes": 30, "connectionId": 1}
        if name in ("ping", "endsessions", "killcursors"):
            return {"ok": 1.0}
        if name == "count":
            return {"ok": 1.0, "n": len(self.docs)}
        if name == "insert":
            self.docs.extend(cmd.get("documents") or [])
            return {"ok": 1.0, "n": len(cmd.get("documents") or [])}
        ns = f"{cmd.get('$db', 'db')}.{cmd[next(iter(cmd))]}"
        if name == "find":
            out = sorted(self.docs, key=lambda d: d["_id"])
            proj = cmd.get("projection") or {}
            if proj:
                out = [{k: d[k] for k in d if k in proj or k == "_id"} for d in out]
            return {"ok": 1.0, "cursor": {"firstBatch": out, "id": 0, "ns": ns}}
        if name == "aggregate":
            out = list(self.docs)
            for st in cmd["pipeline"]:
                if "$match" in st:
                    rng = st["$match"].get("_id", {})
                    out = [d for d in out if ("$gte" not in rng or d["_id"] >= rng["$gte"])
                           and ("$lt" not in rng or d["_id"] < rng["$lt"])]
                elif "$sort" in st:
                    out.sort(key=lambda d: d["_id"])
                elif "$project" in st:
                    keep = st["$project"]
                    out = [{k: d[k] for k in d if keep.get(k) or k == "_id"} for d in out]
            return {"ok": 1.0, "cursor": {"firstBatch": out, "id": 0, "ns": ns}}
        return {"ok": 0.0, "errmsg": f"unsupported {name}", "code": 59}

    def _serve(self, conn):
        import struct

        import bson

        try:
            while True:
                ln, req_id, _, op = struct.unpack("<iiii", self._recv(conn, 16))
                body = self._recv(conn, ln - 16)
                if op == 2013:
                    n0 = struct.unpack("<i", body[5:9])[0]
                    doc = bson.decode(body[5:5 + n0])
                    i = 5 + n0
                    while i < len(body) and body[i] == 1:  # kind-1 document sequence (insert documents)
                        size = struct.unpack("<i", body[i + 1:i + 5])[0]
                        end = i + 1 + size
                        j = body.index(b"\x00", i + 5)
                        ident = body[i + 5:j].decode()
                        j += 1
                        seq = []
                        while j < end:
                            dl = struct.unpack("<i", body[j:j + 4])[0]
                            seq.append(bson.decode(body[j:j + dl]))
                            j += dl
                        doc[ident] = seq
                        i = end
                    self._reply(conn, req_id, self._run(doc), False)
                elif op == 2004:  # legacy OP_QUERY handshake
                    i = 4 + body[4:].index(b"\x00") + 1 + 8
                    doc = bson.decode(body[i:i + struct.unpack("<i", body[i:i + 4])[0]])
                    self._reply(conn, req_id, self._run(doc), True)
                else:
                    return
        except (EOFError, OSError):
            conn.close()


def test_read_mongo(server):
    docs = [{"_id": i, "name": f"n{i}", "v": i * 2} for i in range(20)]
    srv = _MiniMongo(docs)
    uri = f"mongodb://127.0.0.1:{srv.port}/?directConnection=true&serverSelectionTimeoutMS=3000"
    ds = data.read_mongo(uri, "db", "c", override_num_blocks=4)
    rows = ds.take_all()
    assert [r["_id"] for r in rows] == list(range(20)) and rows[3]["v"] == 6
    proj = data.read_mongo(uri, "db", "c", pipeline=[{"$project": {"name": 1}}]).take_all()
    assert set(proj[0]) == {"_id", "name"} and len(proj) == 20


def test_read_videos_native_containers(server, tmp_path):
    """Y4M (raw YUV 4:2:0), Motion-JPEG AVI (hand-built RIFF) and animated GIF."""
    import struct

    import numpy as np
    from PIL import Image

    w, h, n = 16, 8, 3
    # Y4M: mid-grey luma, neutral chroma -> RGB ~ (1.164 * (y - 16)) on every channel
    with open(tmp_path / "a.y4m", "wb") as f:
        f.write(f"YUV4MPEG2 W{w} H{h} F25:1 Ip A1:1 C420jpeg\n".encode())
        for i in range(n):
            f.write(b"FRAME\n" + bytes([100 + i * 10]) * (w * h) + bytes([128]) * (2 * (w // 2) * (h // 2)))
    # MJPEG AVI: three solid-colour JPEG frames
    frames = []
    for c in [(255, 0, 0), (0, 255, 0), (0, 0, 255)]:
        b = io.BytesIO()
        Image.new("RGB", (w, h), c).save(b, format="JPEG", quality=95)
        frames.append(b.getvalue())
    chunks = b"".join(b"00dc" + struct.pack("<I", len(fr)) + fr + (b"\x00" if len(fr) & 1 else b"") for fr in frames)
    movi = b"LIST" + struct.pack("<I", 4 + len(chunks)) + b"movi" + chunks
    strf = b"strf" + struct.pack("<I", 40) + struct.pack("<iiiHH", 40, w, h, 1, 24) + b"MJPG" + b"\x00" * 20
    hdrl = b"LIST" + struct.pack("<I", 4 + len(strf)) + b"hdrl" + strf
    body = b"AVI " + hdrl + movi
    (tmp_path / "b.avi").write_bytes(b"RIFF" + struct.pack("<I", len(body)) + body)
    # animated GIF
    ims = [Image.new("RGB", (w, h), (i * 80, 0, 0)) for i in range(n)]
    ims[0].save(tmp_path / "c.gif", save_all=True, append_images=ims[1:], duration=40)

    rows = data.read_videos(str(tmp_path), include_paths=True).take_all()
    by = {}
    for r in rows:
        by.setdefault(os.path.basename(r["path"]), []).append(r)
    assert [r["frame_index"] for r in by["a.y4m"]] == [0, 1, 2]
    y = by["a.y4m"][1]["frame"]
    assert y.shape == (h, w, 3) and abs(int(y[0, 0, 0]) - round(1.164 * (110 - 16))) <= 1
    av = by["b.avi"]
    assert len(av) == 3 and av[0]["frame"][..., 0].mean() > 200 and av[2]["frame"][..., 2].mean() > 200
    assert len(by["c.gif"]) == 3
    (tmp_path / "d.mp4").write_bytes(b"\x00" * 16)
    with pytest.raises(Exception):
        data.read_videos(str(tmp_path / "d.mp4")).take_all()


def test_write_mongo_round_trip(server):
    srv = _MiniMongo([])
    uri = f"mongodb://127.0.0.1:{srv.port}/?directConnection=true&serverSelectionTimeoutMS=3000"
    data.range(60, override_num_blocks=6).map(lambda r: {"_id": r["id"], "sq": r["id"] ** 2}).write_mongo(
        uri, "db", "w")
    assert sorted(d["_id"] for d in srv.docs) == list(range(60))
    back = data.read_mongo(uri, "db", "w").take_all()
    assert {r["_id"]: r["sq"] for r in back} == {i: i * i for i in range(60)}


def test_write_bigquery_creates_table_and_inserts(server, monkeypatch):
    monkeypatch.setenv("BIGQUERY_API_ENDPOINT", server)
    monkeypatch.setenv("GOOGLE_OAUTH_ACCESS_TOKEN", "tok")
    State.bq_tables["t2"] = {"schema": {}, "rows": [{"stale": 1}]}  # dropped by overwrite_table
    ds = data.from_items([{"id": i, "name": f"r{i}", "x": i / 4, "ok": i % 2 == 0} for i in range(1200)])
    ds.write_bigquery("p1", "d1.t2")
    t = State.bq_tables["t2"]
    types = {f["name"]: f["type"] for f in t["schema"]["fields"]}
    assert types == {"id": "INTEGER", "name": "STRING", "x": "FLOAT", "ok": "BOOLEAN"}
    assert sorted(r["id"] for r in t["rows"]) == list(range(1200))
    assert State.bq_inserts >= 4  # 500-row requests, one retried after a 503
    ds.limit(10).write_bigquery("p1", "d1.t2", overwrite_table=False)  # 409 on create -> append
    assert len(State.bq_tables["t2"]["rows"]) == 1210
