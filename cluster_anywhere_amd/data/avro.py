"""Avro object-container files without fastavro (reference role:
python/ray/data/_internal/datasource/avro_datasource.py, which wraps fastavro).

Implements the Avro 1.x binary encoding and the object-container framing
(``Obj\\x01`` magic, metadata map with ``avro.schema`` / ``avro.codec``, 16-byte
sync marker, blocks of ``count, size, data``) for the ``null`` and ``deflate``
codecs. Types: null, boolean, int, long (zig-zag varints), float, double, bytes,
string, record, enum, array, map, union, fixed, plus logical types passed through
as their underlying values. ``write_avro_file`` is the matching encoder (used by
tests and by ``Dataset.write_avro``-style round trips).
"""
from __future__ import annotations

import io
import json
import os
import struct
import zlib
from typing import Any, Dict, Iterator, List, Optional

MAGIC = b"Obj\x01"


class _Reader:
    __slots__ = ("b", "p")

    def __init__(self, b: bytes):
        self.b = b
        self.p = 0

    def long(self) -> int:
        shift = 0
        acc = 0
        b = self.b
        while True:
            x = b[self.p]
            self.p += 1
            acc |= (x & 0x7F) << shift
            if not x & 0x80:
                break
            shift += 7
        return (acc >> 1) ^ -(acc & 1)

    def raw(self, n: int) -> bytes:
        out = self.b[self.p: self.p + n]
        self.p += n
        return out

    def bytes_(self) -> bytes:
        return self.raw(self.long())


def _named(schema, names: Dict[str, Any], ns: Optional[str] = None):
    """Resolve named-type references; register named types."""
    if isinstance(schema, str):
        if schema in names:
            return names[schema]
        if ns and f"{ns}.{schema}" in names:
            return names[f"{ns}.{schema}"]
        return schema
    if isinstance(schema, list):
        return [_named(s, names, ns) for s in schema]
    t = schema.get("type")
    if t in ("record", "error", "enum", "fixed"):
        nm = schema["name"]
        sns = schema.get("namespace", ns)
        full = nm if "." in nm or not sns else f"{sns}.{nm}"
        names[full] = schema
        names[nm] = schema
        if t in ("record", "error"):
            for f in schema["fields"]:
                f["type"] = _named(f["type"], names, sns)
        return schema
    if t == "array":
        schema["items"] = _named(schema["items"], names, ns)
    elif t == "map":
        schema["values"] = _named(schema["values"], names, ns)
    elif isinstance(t, (dict, list)):
        schema["type"] = _named(t, names, ns)
    return schema


def _decode(r: _Reader, s) -> Any:
    if isinstance(s, list):  # union
        return _decode(r, s[r.long()])
    t = s if isinstance(s, str) else s["type"]
    if isinstance(t, (dict, list)):
        return _decode(r, t)
    if t == "null":
        return None
    if t == "boolean":
        v = r.b[r.p]
        r.p += 1
        return v != 0
    if t in ("int", "long"):
        return r.long()
    if t == "float":
        return struct.unpack("<f", r.raw(4))[0]
    if t == "double":
        return struct.unpack("<d", r.raw(8))[0]
    if t == "bytes":
        return r.bytes_()
    if t == "string":
        return r.bytes_().decode("utf-8")
    if t in ("record", "error"):
        return {f["name"]: _decode(r, f["type"]) for f in s["fields"]}
    if t == "enum":
        return s["symbols"][r.long()]
    if t == "fixed":
        return r.raw(s["size"])
    if t in ("array", "map"):
        out = [] if t == "array" else {}
        while True:
            n = r.long()
            if n == 0:
                break
            if n < 0:
                n = -n
                r.long()  # block byte size
            for _ in range(n):
                if t == "array":
                    out.append(_decode(r, s["items"]))
                else:
                    k = r.bytes_().decode("utf-8")
                    out[k] = _decode(r, s["values"])
        return out
    raise ValueError(f"unsupported avro type {t!r}")


def read_avro_file(path_or_bytes) -> Iterator[Dict[str, Any]]:
    """Yield the records of one object-container file."""
    if isinstance(path_or_bytes, (bytes, bytearray)):
        data = bytes(path_or_bytes)
    else:
        with open(path_or_bytes, "rb") as f:
            data = f.read()
    if data[:4] != MAGIC:
        raise ValueError("not an Avro object container file")
    r = _Reader(data)
    r.p = 4
    meta = _decode(r, {"type": "map", "values": "bytes"})
    sync = r.raw(16)
    schema = _named(json.loads(meta["avro.schema"].decode()), {})
    codec = meta.get("avro.codec", b"null").decode()
    if codec not in ("null", "deflate"):
        raise ValueError(f"avro codec {codec!r} is not supported (null, deflate)")
    while r.p < len(data):
        count = r.long()
        size = r.long()
        block = r.raw(size)
        if codec == "deflate":
            block = zlib.decompress(block, -15)
        br = _Reader(block)
        for _ in range(count):
            yield _decode(br, schema)
        if r.raw(16) != sync:
            raise ValueError("avro sync marker mismatch (corrupt file)")


def read_avro_schema(path) -> Any:
    with open(path, "rb") as f:
        data = f.read(1 << 20)
    r = _Reader(data)
    r.p = 4
    meta = _decode(r, {"type": "map", "values": "bytes"})
    return json.loads(meta["avro.schema"].decode())


# ------------------------------------------------------------------ encoder
def _zz(n: int) -> bytes:
    n = (n << 1) ^ (n >> 63)
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _encode(buf: io.BytesIO, s, v):
    if isinstance(s, list):
        for i, branch in enumerate(s):
            if _matches(branch, v):
                buf.write(_zz(i))
                return _encode(buf, branch, v)
        raise ValueError(f"value {v!r} matches no branch of union {s}")
    t = s if isinstance(s, str) else s["type"]
    if isinstance(t, (dict, list)):
        return _encode(buf, t, v)
    if t == "null":
        return
    if t == "boolean":
        buf.write(b"\x01" if v else b"\x00")
    elif t in ("int", "long"):
        buf.write(_zz(int(v)))
    elif t == "float":
        buf.write(struct.pack("<f", v))
    elif t == "double":
        buf.write(struct.pack("<d", v))
    elif t in ("bytes", "string"):
        b = v.encode("utf-8") if t == "string" else bytes(v)
        buf.write(_zz(len(b)))
        buf.write(b)
    elif t in ("record", "error"):
        for f in s["fields"]:
            _encode(buf, f["type"], v.get(f["name"]) if isinstance(v, dict) else getattr(v, f["name"]))
    elif t == "enum":
        buf.write(_zz(s["symbols"].index(v)))
    elif t == "fixed":
        buf.write(bytes(v))
    elif t == "array":
        if v:
            buf.write(_zz(len(v)))
            for x in v:
                _encode(buf, s["items"], x)
        buf.write(b"\x00")
    elif t == "map":
        if v:
            buf.write(_zz(len(v)))
            for k, x in v.items():
                kb = k.encode()
                buf.write(_zz(len(kb)))
                buf.write(kb)
                _encode(buf, s["values"], x)
        buf.write(b"\x00")
    else:
        raise ValueError(f"unsupported avro type {t!r}")


def _matches(s, v) -> bool:
    t = s if isinstance(s, str) else s.get("type")
    if t == "null":
        return v is None
    if t == "boolean":
        return isinstance(v, bool)
    if t in ("int", "long"):
        return isinstance(v, int) and not isinstance(v, bool)
    if t in ("float", "double"):
        return isinstance(v, float)
    if t == "string":
        return isinstance(v, str)
    if t in ("bytes", "fixed"):
        return isinstance(v, (bytes, bytearray))
    if t in ("record", "map"):
        return isinstance(v, dict)
    if t == "array":
        return isinstance(v, (list, tuple))
    if t == "enum":
        return isinstance(v, str)
    return False


def write_avro_file(path: str, schema: dict, records: List[dict], codec: str = "deflate",
                    block_records: int = 1000):
    """Write ``records`` as an object-container file (null / deflate codec)."""
    resolved = _named(json.loads(json.dumps(schema)), {})
    sync = os.urandom(16)
    out = io.BytesIO()
    out.write(MAGIC)
    meta = io.BytesIO()
    _encode(meta, {"type": "map", "values": "bytes"},
            {"avro.schema": json.dumps(schema).encode(), "avro.codec": codec.encode()})
    out.write(meta.getvalue())
    out.write(sync)
    for i in range(0, len(records), block_records):
        chunk = records[i: i + block_records]
        b = io.BytesIO()
        for rec in chunk:
            _encode(b, resolved, rec)
        data = b.getvalue()
        if codec == "deflate":
            c = zlib.compressobj(6, zlib.DEFLATED, -15)
            data = c.compress(data) + c.flush()
        out.write(_zz(len(chunk)))
        out.write(_zz(len(data)))
        out.write(data)
        out.write(sync)
    with open(path, "wb") as f:
        f.write(out.getvalue())
