"""Minimal TensorBoard event-file writer (no tensorboard/tensorflow dependency).

The reference logs through Lightning's ``TensorBoardLogger`` (`train.py:143-148`):
epoch scalars, ``log_hyperparams`` with final metrics (`train.py:201-211`) and
matplotlib figures from `test.py:91-145`.  TensorBoard is not installed on the
MI355X image, so this module writes the on-disk format directly:

* TFRecord framing: ``u64 len | u32 masked_crc32c(len) | data | u32 masked_crc32c(data)``;
* hand-encoded ``Event`` / ``Summary`` protobufs: scalars (``simple_value``),
  PNG images, and the ``hparams`` plugin (experiment / session start / session end),
  which is what ``torch.utils.tensorboard.summary.hparams`` emits.

Files are readable by stock TensorBoard; ``read_events`` parses them back (tests).
"""
from __future__ import annotations

import os
import socket
import struct
import threading
import time
from pathlib import Path
from typing import Any, Dict, Iterator, List, Optional, Tuple

# --------------------------------------------------------------------------- #
# CRC32C (Castagnoli), table driven
# --------------------------------------------------------------------------- #
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    t = _TABLE
    for b in data:
        crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# --------------------------------------------------------------------------- #
# protobuf wire encoding
# --------------------------------------------------------------------------- #
def _varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def f_varint(field: int, v: int) -> bytes:
    return _key(field, 0) + _varint(int(v))


def f_double(field: int, v: float) -> bytes:
    return _key(field, 1) + struct.pack("<d", float(v))


def f_float(field: int, v: float) -> bytes:
    return _key(field, 5) + struct.pack("<f", float(v))


def f_bytes(field: int, b: bytes) -> bytes:
    return _key(field, 2) + _varint(len(b)) + b


def f_str(field: int, s: str) -> bytes:
    return f_bytes(field, s.encode("utf-8"))


# Summary.Value
def value_scalar(tag: str, v: float) -> bytes:
    return f_str(1, tag) + f_float(2, v)


def value_image(tag: str, png: bytes, height: int, width: int, channels: int = 4) -> bytes:
    img = f_varint(1, height) + f_varint(2, width) + f_varint(3, channels) + f_bytes(4, png)
    return f_str(1, tag) + f_bytes(4, img)


def value_plugin(tag: str, plugin: str, content: bytes) -> bytes:
    plugin_data = f_str(1, plugin) + f_bytes(2, content)
    metadata = f_bytes(1, plugin_data)
    # a zero-length tensor keeps the value well-formed for the hparams plugin
    tensor = f_varint(1, 7)  # DT_STRING dtype, empty
    return f_str(1, tag) + f_bytes(9, metadata) + f_bytes(8, tensor)


def summary(values: List[bytes]) -> bytes:
    return b"".join(f_bytes(1, v) for v in values)


def event(wall_time: float, step: int, *, summary_bytes: Optional[bytes] = None,
          file_version: Optional[str] = None) -> bytes:
    out = f_double(1, wall_time) + f_varint(2, step)
    if file_version is not None:
        out += f_str(3, file_version)
    if summary_bytes is not None:
        out += f_bytes(5, summary_bytes)
    return out


# hparams plugin (tensorboard/plugins/hparams/api.proto + plugin_data.proto)
def _pb_value(v: Any) -> bytes:
    if v is None:
        return f_varint(1, 0)
    if isinstance(v, bool):
        return f_varint(4, int(v))
    if isinstance(v, (int, float)):
        return f_double(2, float(v))
    return f_str(3, str(v))


def hparams_plugin_contents(hparams: Dict[str, Any], metric_tags: List[str],
                            start_time: float) -> Tuple[bytes, bytes, bytes]:
    infos = b""
    for k, v in hparams.items():
        dtype = 2 if isinstance(v, bool) else 3 if isinstance(v, (int, float)) else 1
        infos += f_bytes(4, f_str(1, k) + f_varint(4, dtype))
    metrics = b"".join(f_bytes(5, f_bytes(1, f_str(2, t))) for t in metric_tags)
    experiment = f_bytes(2, infos + metrics)  # HParamsPluginData.experiment (version 0)
    hp_map = b"".join(f_bytes(1, f_str(1, k) + f_bytes(2, _pb_value(v))) for k, v in hparams.items())
    start = f_bytes(3, hp_map + f_double(5, start_time))
    end = f_bytes(4, f_varint(1, 1) + f_double(2, time.time()))
    return experiment, start, end


# --------------------------------------------------------------------------- #
# writer
# --------------------------------------------------------------------------- #
class EventFileWriter:
    def __init__(self, logdir: os.PathLike, filename_suffix: str = ""):
        self.logdir = Path(logdir)
        self.logdir.mkdir(parents=True, exist_ok=True)
        fname = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}.0{filename_suffix}"
        self.path = self.logdir / fname
        self._f = open(self.path, "ab")
        self._lock = threading.Lock()
        self._write(event(time.time(), 0, file_version="brain.Event:2"))

    def _write(self, data: bytes) -> None:
        header = struct.pack("<Q", len(data))
        rec = header + struct.pack("<I", masked_crc(header)) + data + struct.pack("<I", masked_crc(data))
        with self._lock:
            self._f.write(rec)

    def add_summary(self, values: List[bytes], step: int, wall_time: Optional[float] = None) -> None:
        self._write(event(time.time() if wall_time is None else wall_time, int(step), summary_bytes=summary(values)))

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        self.add_summary([value_scalar(tag, float(value))], step)

    def add_image_png(self, tag: str, png: bytes, height: int, width: int, step: int = 0) -> None:
        self.add_summary([value_image(tag, png, height, width)], step)

    def add_figure(self, tag: str, figure, global_step: int = 0, close: bool = True) -> None:
        import io

        import matplotlib

        matplotlib.use("Agg", force=False)
        import matplotlib.pyplot as plt

        buf = io.BytesIO()
        figure.canvas.draw()
        w, h = figure.canvas.get_width_height()
        figure.savefig(buf, format="png")
        if close:
            plt.close(figure)
        self.add_image_png(tag, buf.getvalue(), h, w, global_step)

    def add_hparams(self, hparams: Dict[str, Any], metrics: Dict[str, float], step: int = 0) -> None:
        exp, start, end = hparams_plugin_contents(hparams, list(metrics), time.time())
        self.add_summary([value_plugin("_hparams_/experiment", "hparams", exp)], step)
        self.add_summary([value_plugin("_hparams_/session_start_info", "hparams", start)], step)
        self.add_summary([value_plugin("_hparams_/session_end_info", "hparams", end)], step)
        for k, v in metrics.items():
            self.add_scalar(k, v, step)

    def flush(self) -> None:
        with self._lock:
            self._f.flush()

    def close(self) -> None:
        with self._lock:
            if not self._f.closed:
                self._f.flush()
                self._f.close()


# --------------------------------------------------------------------------- #
# reader (tests / tooling)
# --------------------------------------------------------------------------- #
def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            return v, i


def parse_message(b: bytes) -> Dict[int, list]:
    out: Dict[int, list] = {}
    i = 0
    while i < len(b):
        k, i = _read_varint(b, i)
        field, wire = k >> 3, k & 7
        if wire == 0:
            v, i = _read_varint(b, i)
        elif wire == 1:
            v = struct.unpack_from("<d", b, i)[0]
            i += 8
        elif wire == 5:
            v = struct.unpack_from("<f", b, i)[0]
            i += 4
        elif wire == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError(f"unsupported wire type {wire}")
        out.setdefault(field, []).append(v)
    return out


def read_records(path: os.PathLike) -> Iterator[bytes]:
    data = Path(path).read_bytes()
    i = 0
    while i < len(data):
        header = data[i:i + 8]
        (n,) = struct.unpack("<Q", header)
        (hc,) = struct.unpack_from("<I", data, i + 8)
        if hc != masked_crc(header):
            raise ValueError("corrupt record header")
        body = data[i + 12:i + 12 + n]
        (bc,) = struct.unpack_from("<I", data, i + 12 + n)
        if bc != masked_crc(body):
            raise ValueError("corrupt record body")
        yield body
        i += 16 + n


def read_scalars(path: os.PathLike) -> Dict[str, List[Tuple[int, float]]]:
    """tag -> [(step, value)] for every simple_value in an event file."""
    out: Dict[str, List[Tuple[int, float]]] = {}
    for rec in read_records(path):
        ev = parse_message(rec)
        step = ev.get(2, [0])[0]
        for s in ev.get(5, []):
            for v in parse_message(s).get(1, []):
                vm = parse_message(v)
                if 2 in vm:
                    out.setdefault(vm[1][0].decode(), []).append((step, vm[2][0]))
    return out


def read_tags(path: os.PathLike) -> List[str]:
    tags = []
    for rec in read_records(path):
        ev = parse_message(rec)
        for s in ev.get(5, []):
            for v in parse_message(s).get(1, []):
                tags.append(parse_message(v)[1][0].decode())
    return tags
