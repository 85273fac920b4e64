"""TensorBoard scalar event files without TensorFlow.

The reference writes TensorBoard logs through the Keras callback
(R/ResNet/tensorflow/train.py:268-269, R/LeNet/tensorflow/train.py:134-135) and ``tf.summary``
writers (R/YOLO/tensorflow/train.py:196-199, R/Hourglass/tensorflow/train.py:134-135,
R/CycleGAN/tensorflow/train.py:267-312). ``tensorboard`` / ``tensorflow`` are not installed
on this stack, so ``SummaryWriter`` emits the same on-disk format itself:

  file   ``events.out.tfevents.{int(time)}.{hostname}`` in the log directory
  record TFRecord framing (length, masked CRC32C; data/tfrecord.py + the native _io writer)
  data   a serialized ``tensorflow.Event`` protobuf:
           wall_time = 1 (double), step = 2 (int64), file_version = 3 (string, first record
           "brain.Event:2"), summary = 5 (Summary { repeated Value value = 1 },
           Value { tag = 1 (string), simple_value = 2 (float) })

``read_scalars`` decodes such files (ours or TensorFlow's: it is validated against the
reference's checked-in Keras event file) into ``{tag: [(step, value, wall_time)]}``.
Only rank 0 writes (``SummaryWriter(enabled=...)``).
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Dict, List, Tuple

from ..data.tfrecord import TFRecordWriter, _ld, _varint, tfrecord_iterator


def _event(wall_time: float, step: int = 0, file_version: str | None = None, summary: bytes | None = None) -> bytes:
    out = bytearray()
    out += _varint((1 << 3) | 1) + struct.pack("<d", wall_time)
    if step:
        out += _varint((2 << 3) | 0) + _varint(int(step))
    if file_version is not None:
        out += _ld(3, file_version.encode())
    if summary is not None:
        out += _ld(5, summary)
    return bytes(out)


def _scalar_summary(tag: str, value: float) -> bytes:
    val = _ld(1, tag.encode()) + _varint((2 << 3) | 5) + struct.pack("<f", float(value))
    return _ld(1, val)


class SummaryWriter:
    """``add_scalar(tag, value, step)`` -> a TensorBoard event file under ``log_dir``."""

    def __init__(self, log_dir: str, enabled: bool = True, filename_suffix: str = ""):
        self.log_dir = log_dir
        self.enabled = enabled
        self._w = None
        self.path = None
        if enabled:
            os.makedirs(log_dir, exist_ok=True)
            name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}{filename_suffix}"
            self.path = os.path.join(log_dir, name)
            self._w = TFRecordWriter(self.path)
            self._w.write(_event(time.time(), file_version="brain.Event:2"))

    def add_scalar(self, tag: str, value: float, step: int = 0, walltime: float | None = None) -> None:
        if self._w is None:
            return
        self._w.write(_event(walltime if walltime is not None else time.time(), step, summary=_scalar_summary(tag, value)))

    def add_scalars(self, values: Dict[str, float], step: int = 0) -> None:
        for k, v in values.items():
            self.add_scalar(k, v, step)

    def flush(self) -> None:
        pass  # records are written through (the native writer flushes on close)

    def close(self) -> None:
        if self._w is not None:
            self._w.close()
            self._w = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# ------------------------------------------------------------------ reading
def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    v = shift = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if not c & 0x80:
            return v, i
        shift += 7


def _fields(b: bytes):
    """Yield (field number, wire type, value) of one protobuf message (values: int / bytes)."""
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield fn, wt, v


def parse_event(rec: bytes) -> dict:
    ev = {"wall_time": 0.0, "step": 0, "file_version": None, "scalars": []}
    for fn, wt, v in _fields(rec):
        if fn == 1 and wt == 1:
            ev["wall_time"] = struct.unpack("<d", v)[0]
        elif fn == 2 and wt == 0:
            ev["step"] = v
        elif fn == 3 and wt == 2:
            ev["file_version"] = v.decode()
        elif fn == 5 and wt == 2:
            for sfn, swt, sv in _fields(v):
                if sfn != 1 or swt != 2:
                    continue
                tag, val = None, None
                for vfn, vwt, vv in _fields(sv):
                    if vfn == 1 and vwt == 2:
                        tag = vv.decode()
                    elif vfn == 2 and vwt == 5:
                        val = struct.unpack("<f", vv)[0]
                if tag is not None and val is not None:
                    ev["scalars"].append((tag, val))
    return ev


def read_scalars(path: str) -> Dict[str, List[Tuple[int, float, float]]]:
    out: Dict[str, List[Tuple[int, float, float]]] = {}
    for rec in tfrecord_iterator(path):
        ev = parse_event(rec)
        for tag, val in ev["scalars"]:
            out.setdefault(tag, []).append((ev["step"], val, ev["wall_time"]))
    return out
