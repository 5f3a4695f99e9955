"""File-format codecs for Data sources/sinks that need no third-party library
(reference: python/ray/data/_internal/datasource/{tfrecords,webdataset,sql,
image}_datasource.py and their datasinks).

* TFRecord: length-prefixed records with masked CRC32C, each a ``tf.train.Example``
  protobuf — encoded/decoded here directly on the protobuf wire format, so
  TensorFlow is not needed.
* WebDataset: tar shards, one member per ``<key>.<ext>`` (row = shared key).
* SQL: any DB-API 2 connection factory (sqlite3 ships with Python).
"""
from __future__ import annotations

import io
import json
import struct
import tarfile
from typing import Any, Dict, Iterator, List

import numpy as np

# ---------------------------------------------------------------- CRC32C
_CRC_TABLE = None


def _crc_table():
    global _CRC_TABLE
    if _CRC_TABLE is None:
        poly = 0x82F63B78
        t = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ poly if c & 1 else c >> 1
            t.append(c)
        _CRC_TABLE = t
    return _CRC_TABLE


def crc32c(data: bytes) -> int:
    t = _crc_table()
    c = 0xFFFFFFFF
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ------------------------------------------------------- protobuf wire format
def _varint(n: int) -> bytes:
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: memoryview, i: int):
    shift = n = 0
    while True:
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        if not b & 0x80:
            return n, i
        shift += 7


def _ld(field: int, payload: bytes) -> bytes:  # length-delimited field
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def _fields(buf: memoryview):
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        f, wt = key >> 3, key & 7
        if wt == 2:
            n, i = _read_varint(buf, i)
            yield f, wt, buf[i:i + n]
            i += n
        elif wt == 0:
            v, i = _read_varint(buf, i)
            yield f, wt, v
        elif wt == 5:
            yield f, wt, buf[i:i + 4]
            i += 4
        elif wt == 1:
            yield f, wt, buf[i:i + 8]
            i += 8
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")


def _feature(value) -> bytes:
    arr = np.asarray(value)
    if arr.dtype == object or arr.dtype.kind in "SU":
        vals = [v.encode() if isinstance(v, str) else bytes(v) for v in np.ravel(arr)]
        return _ld(1, b"".join(_ld(1, v) for v in vals))
    if arr.dtype.kind == "f":
        return _ld(2, _ld(1, np.ravel(arr).astype("<f4").tobytes()))
    if arr.dtype.kind in "iub":
        return _ld(3, _ld(1, b"".join(_varint(int(v)) for v in np.ravel(arr))))
    raise TypeError(f"cannot encode {arr.dtype} in a tf.train.Example")


def encode_example(row: Dict[str, Any]) -> bytes:
    entries = b"".join(_ld(1, _ld(1, k.encode()) + _ld(2, _feature(v))) for k, v in row.items())
    return _ld(1, entries)


def decode_example(data: bytes) -> Dict[str, Any]:
    out = {}
    for f, _, feats in _fields(memoryview(data)):
        if f != 1:
            continue
        for f2, _, entry in _fields(feats):
            if f2 != 1:
                continue
            key, val = None, None
            for f3, _, x in _fields(entry):
                if f3 == 1:
                    key = bytes(x).decode()
                elif f3 == 2:
                    val = x
            vals: List[Any] = []
            for kind, _, lst in _fields(val):
                for f4, wt, x in _fields(lst):
                    if kind == 1:
                        vals.append(bytes(x))
                    elif kind == 2:
                        vals.extend(np.frombuffer(bytes(x), "<f4").tolist() if wt == 2 else
                                    [struct.unpack("<f", bytes(x))[0]])
                    elif kind == 3:
                        if wt == 2:
                            j, xb = 0, x
                            while j < len(xb):
                                v, j = _read_varint(xb, j)
                                vals.append(v - (1 << 64) if v >= 1 << 63 else v)
                        else:
                            vals.append(x - (1 << 64) if x >= 1 << 63 else x)
            out[key] = vals[0] if len(vals) == 1 else vals
    return out


def write_tfrecords(rows: Iterator[Dict[str, Any]], fn: str):
    with open(fn, "wb") as f:
        for row in rows:
            data = encode_example(row)
            ln = struct.pack("<Q", len(data))
            f.write(ln + struct.pack("<I", _masked(ln)) + data + struct.pack("<I", _masked(data)))


def read_tfrecords(fn: str, verify: bool = True) -> List[Dict[str, Any]]:
    rows = []
    with open(fn, "rb") as f:
        while True:
            hdr = f.read(12)
            if not hdr:
                break
            (n,) = struct.unpack("<Q", hdr[:8])
            if verify and struct.unpack("<I", hdr[8:])[0] != _masked(hdr[:8]):
                raise ValueError(f"{fn}: corrupt TFRecord length crc")
            data = f.read(n)
            (crc,) = struct.unpack("<I", f.read(4))
            if verify and crc != _masked(data):
                raise ValueError(f"{fn}: corrupt TFRecord data crc")
            rows.append(decode_example(data))
    return rows


# ------------------------------------------------------------- webdataset
def _wds_encode(v) -> (str, bytes):
    if isinstance(v, (bytes, bytearray)):
        return "bin", bytes(v)
    if isinstance(v, str):
        return "txt", v.encode()
    if isinstance(v, np.ndarray):
        b = io.BytesIO()
        np.save(b, v, allow_pickle=False)
        return "npy", b.getvalue()
    if isinstance(v, (np.generic,)):
        v = v.item()
    return "json", json.dumps(v).encode()


def write_webdataset(rows: Iterator[Dict[str, Any]], fn: str, start_key: int = 0):
    with tarfile.open(fn, "w") as tar:
        for i, row in enumerate(rows):
            key = str(row.get("__key__", f"{start_key + i:09d}"))
            for col, v in row.items():
                if col == "__key__":
                    continue
                ext, data = _wds_encode(v)
                name = f"{key}.{col}" if "." in col else f"{key}.{col}.{ext}"
                ti = tarfile.TarInfo(name)
                ti.size = len(data)
                tar.addfile(ti, io.BytesIO(data))


def _wds_decode(ext: str, data: bytes, decode: bool):
    if not decode:
        return data
    if ext == "npy":
        return np.load(io.BytesIO(data), allow_pickle=False)
    if ext in ("txt", "text"):
        return data.decode()
    if ext in ("json", "cls"):
        return json.loads(data.decode()) if ext == "json" else int(data.decode())
    if ext in ("png", "jpg", "jpeg"):
        try:
            from PIL import Image

            return np.asarray(Image.open(io.BytesIO(data)))
        except ImportError:
            return data
    return data


def read_webdataset(fn: str, decode: bool = True) -> List[Dict[str, Any]]:
    rows: Dict[str, Dict[str, Any]] = {}
    order = []
    with tarfile.open(fn, "r") as tar:
        for m in tar.getmembers():
            if not m.isfile():
                continue
            base = m.name.rsplit("/", 1)[-1]
            key, _, rest = base.partition(".")
            parts = rest.split(".")
            col, ext = (parts[0], parts[-1]) if len(parts) > 1 else (rest, rest)
            data = tar.extractfile(m).read()
            if key not in rows:
                rows[key] = {"__key__": key}
                order.append(key)
            rows[key][col] = _wds_decode(ext, data, decode)
    return [rows[k] for k in order]
