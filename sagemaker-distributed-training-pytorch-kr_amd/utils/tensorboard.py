"""TensorBoard event-file writer with no TensorFlow / tensorboard dependency.

The reference's Megatron recipe writes scalars through ``torch.utils.tensorboard.SummaryWriter``
when ``--tensorboard-dir`` is set (/root/reference/3_training_megatron-lm/megatron/arguments.py:
652-679, 812-813). Neither the ``tensorboard`` package nor TensorFlow is in this
image, so this module writes the on-disk format directly — it is small and stable:

  * a file ``events.out.tfevents.<unix time>.<host>.<pid>.<n>`` of TFRecords, each
    ``uint64 len | uint32 masked_crc32c(len) | bytes data | uint32 masked_crc32c(data)``;
  * ``data`` is a serialized ``tensorflow.Event`` protobuf: ``wall_time`` (field 1, double),
    ``step`` (2, int64), then either ``file_version`` (3, string; the first record) or
    ``summary`` (5): ``Summary { repeated Value value = 1 }``, ``Value { string tag = 1;
    float simple_value = 2 }``.

The protobuf wire encoding is done by hand (varints + fixed64/32) so nothing needs generated
message classes. ``read_scalars`` parses the same format back (CRC-checked) for tests and tools.
Stock TensorBoard reads these files unchanged.
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Dict, Iterator, List, Optional, Tuple

# ---- CRC-32C (Castagnoli), table driven ------------------------------------------------------
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    tb = _TABLE
    for b in data:
        c = tb[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---- protobuf wire helpers --------------------------------------------------------------------
def _varint(n: int) -> bytes:
    if n < 0:
        n += 1 << 64
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _len_field(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _event(wall_time: float, step: int, *, file_version: Optional[str] = None,
           scalars: Optional[List[Tuple[str, float]]] = None) -> bytes:
    ev = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        ev += _len_field(3, file_version.encode())
    if scalars:
        summ = b"".join(_len_field(1, _len_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(v)))
                        for tag, v in scalars)
        ev += _len_field(5, summ)
    return ev


def _record(data: bytes) -> bytes:
    hdr = struct.pack("<Q", len(data))
    return hdr + struct.pack("<I", _masked_crc(hdr)) + data + struct.pack("<I", _masked_crc(data))


class SummaryWriter:
    """The subset of ``torch.utils.tensorboard.SummaryWriter`` Megatron uses: ``add_scalar``,
    ``add_scalars`` (flattened to ``main/sub`` tags), ``add_text`` (as a scalar-free no-op record),
    ``flush``, ``close``. Records are buffered up to ``max_queue`` (``--tensorboard-queue-size``)."""

    _counter = 0

    def __init__(self, log_dir: str, max_queue: int = 1000, filename_suffix: str = ""):
        os.makedirs(log_dir, exist_ok=True)
        SummaryWriter._counter += 1
        name = (f"events.out.tfevents.{int(time.time()):010d}.{socket.gethostname()}."
                f"{os.getpid()}.{SummaryWriter._counter}{filename_suffix}")
        self.log_dir = log_dir
        self.path = os.path.join(log_dir, name)
        self.max_queue = max(int(max_queue), 1)
        self._buf: List[bytes] = []
        self._f = open(self.path, "ab")
        self._f.write(_record(_event(time.time(), 0, file_version="brain.Event:2")))
        self._f.flush()

    def add_scalar(self, tag: str, value, global_step: int = 0, walltime: Optional[float] = None):
        v = float(value.item() if hasattr(value, "item") else value)
        self._buf.append(_record(_event(walltime or time.time(), global_step, scalars=[(tag, v)])))
        if len(self._buf) >= self.max_queue:
            self.flush()

    def add_scalars(self, main_tag: str, tag_scalar_dict: Dict[str, float], global_step: int = 0,
                    walltime: Optional[float] = None):
        for k, v in tag_scalar_dict.items():
            self.add_scalar(f"{main_tag}/{k}", v, global_step, walltime)

    def add_text(self, tag: str, text: str, global_step: int = 0):  # kept for API compatibility
        pass

    def flush(self):
        if self._buf and self._f is not None:
            self._f.write(b"".join(self._buf))
            self._f.flush()
            self._buf.clear()

    def close(self):
        self.flush()
        if self._f is not None:
            self._f.close()
            self._f = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- reader -------------------------------------------------------------------------------------
def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    n, shift = 0, 0
    while True:
        x = b[i]
        i += 1
        n |= (x & 0x7F) << shift
        if not x & 0x80:
            return n, i
        shift += 7


def _fields(b: bytes) -> Iterator[Tuple[int, int, object]]:
    i = 0
    while i < len(b):
        k, i = _read_varint(b, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _read_varint(b, i)
        elif w == 1:
            v = b[i:i + 8]
            i += 8
        elif w == 5:
            v = b[i:i + 4]
            i += 4
        elif w == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError(f"unsupported wire type {w}")
        yield f, w, v


def read_records(path: str) -> Iterator[bytes]:
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        hdr = data[i:i + 8]
        (n,) = struct.unpack("<Q", hdr)
        (hc,) = struct.unpack("<I", data[i + 8:i + 12])
        if hc != _masked_crc(hdr):
            raise ValueError(f"{path}: corrupt record header at byte {i}")
        payload = data[i + 12:i + 12 + n]
        (pc,) = struct.unpack("<I", data[i + 12 + n:i + 16 + n])
        if pc != _masked_crc(payload):
            raise ValueError(f"{path}: corrupt record payload at byte {i}")
        yield payload
        i += 16 + n


def read_scalars(path: str) -> List[Tuple[int, str, float]]:
    """[(step, tag, value)] of every scalar in an event file (CRC-checked)."""
    out = []
    for rec in read_records(path):
        step = 0
        for f, w, v in _fields(rec):
            if f == 2:
                step = v
            elif f == 5:
                for vf, _, val in _fields(v):
                    if vf != 1:
                        continue
                    tag, x = None, None
                    for ff, _, vv in _fields(val):
                        if ff == 1:
                            tag = vv.decode()
                        elif ff == 2:
                            (x,) = struct.unpack("<f", vv)
                    if tag is not None and x is not None:
                        out.append((step, tag, x))
    return out
