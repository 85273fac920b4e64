"""TF-free TFRecord + tf.train.Example IO.

Framing, CRC32C and Example decoding run in the native host runtime (csrc/host/io.cpp ->
``deep_vision_amd._io``); Example *encoding* (the offline builders' side) is done here from the
protobuf wire format, so no TensorFlow and no generated protobuf classes are needed. Files
written here are byte-compatible with ``tf.io.TFRecordWriter`` + ``tf.train.Example``.

Feature helpers mirror the reference builders (R/Datasets/MSCOCO/tfrecords.py:19-34):
``bytes_feature``, ``float_feature``, ``int64_feature`` (and ``*_list_feature``).
"""
from __future__ import annotations

import os
import struct
from typing import Dict, Iterator, List, Sequence, Tuple

_io_mod = None


def native():
    """The ``_io`` host extension (built on first use)."""
    global _io_mod
    if _io_mod is None:
        try:
            from .. import _io  # type: ignore
        except ImportError:
            from .. import _build

            _build.build_host(verbose=False)
            from .. import _io  # type: ignore
        _io_mod = _io
    return _io_mod


# ------------------------------------------------------------------ Example encoding
def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _ld(field: int, payload: bytes) -> bytes:  # length-delimited field
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def bytes_feature(value) -> Tuple[str, list]:
    return ("bytes", [value if isinstance(value, bytes) else str(value).encode()])


def bytes_list_feature(values: Sequence) -> Tuple[str, list]:
    return ("bytes", [v if isinstance(v, bytes) else str(v).encode() for v in values])


def float_feature(value) -> Tuple[str, list]:
    return ("float", [float(value)])


def float_list_feature(values: Sequence[float]) -> Tuple[str, list]:
    return ("float", [float(v) for v in values])


def int64_feature(value) -> Tuple[str, list]:
    return ("int64", [int(value)])


def int64_list_feature(values: Sequence[int]) -> Tuple[str, list]:
    return ("int64", [int(v) for v in values])


def _encode_feature(kind: str, values: list) -> bytes:
    if kind == "bytes":
        body = b"".join(_ld(1, v) for v in values)
        return _ld(1, body)
    if kind == "float":
        packed = struct.pack(f"<{len(values)}f", *values)
        return _ld(2, _ld(1, packed) if values else b"")
    if kind == "int64":
        packed = b"".join(_varint(v) for v in values)
        return _ld(3, _ld(1, packed) if values else b"")
    raise ValueError(kind)


def encode_example(features: Dict[str, Tuple[str, list]]) -> bytes:
    """{name: (kind, values)} -> serialized tf.train.Example."""
    entries = b""
    for name in sorted(features):
        kind, values = features[name]
        entry = _ld(1, name.encode()) + _ld(2, _encode_feature(kind, list(values)))
        entries += _ld(1, entry)
    return _ld(1, entries)


def decode_example(data: bytes) -> Dict[str, Tuple[str, list]]:
    """serialized tf.train.Example -> {name: (kind, values)} (native decoder)."""
    return native().parse_example(data)


def example_values(ex: Dict[str, Tuple[str, list]], name: str, default=None):
    v = ex.get(name)
    return default if v is None else v[1]


# ------------------------------------------------------------------ record files
class TFRecordWriter:
    def __init__(self, path: str):
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        self._w = native().RecordWriter(path)

    def write(self, record: bytes) -> None:
        self._w.write(record)

    def close(self) -> None:
        self._w.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def tfrecord_iterator(path: str, check_crc: bool = True) -> Iterator[bytes]:
    r = native().RecordReader(path, check_crc)
    while True:
        rec = r.next()
        if rec is None:
            return
        yield rec


class TFRecordIndex:
    """Random access over a list of TFRecord files: (file, offset) per record."""

    def __init__(self, files: Sequence[str]):
        self.files = list(files)
        self.entries: List[Tuple[int, int]] = []
        for fi, f in enumerate(self.files):
            self.entries += [(fi, off) for off in native().index_file(f)]
        self._readers = {}

    def __len__(self):
        return len(self.entries)

    def __getitem__(self, i: int) -> bytes:
        fi, off = self.entries[i]
        # one reader per file per process (DataLoader workers get their own after fork)
        key = (os.getpid(), fi)
        r = self._readers.get(key)
        if r is None:
            r = self._readers[key] = native().RecordReader(self.files[fi], True)
        return r.read_at(off)

    def __getstate__(self):
        st = dict(self.__dict__)
        st["_readers"] = {}
        return st


def shard_name(prefix: str, idx: int, total: int) -> str:
    """TF-models shard naming: ``{prefix}-00003-of-00064``."""
    return "%s-%.5d-of-%.5d" % (prefix, idx, total)
