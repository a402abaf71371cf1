"""TensorBoard event files through the native writer (csrc/io/event_writer.cpp).

``EventFileWriter(logdir)`` creates ``events.out.tfevents.<time>.<host>`` and writes
the ``brain.Event:2`` header; ``add_scalars(step, {tag: value})`` appends one
Event with a Summary of simple values (tags ``loss``, ``accuracy``,
``global_step/sec`` — SURVEY.md §5.5).  ``read_events`` parses them back
(tests/tools; verifies both TFRecord CRCs natively).
"""
from __future__ import annotations

import ctypes as C
import socket
import struct
import time
from pathlib import Path

from .. import _native as N

N.register_host({
    "tde_events_open": (C.c_void_p, [C.c_char_p]),
    "tde_events_write_version": (C.c_int, [C.c_void_p, C.c_double]),
    "tde_events_write_scalars": (C.c_int, [C.c_void_p, C.c_double, C.c_longlong, C.c_int, C.POINTER(C.c_char_p),
                                           C.POINTER(C.c_float)]),
    "tde_events_write_raw": (C.c_int, [C.c_void_p, C.c_void_p, C.c_longlong]),
    "tde_events_flush": (C.c_int, [C.c_void_p]),
    "tde_events_close": (None, [C.c_void_p]),
    "tde_tfrecord_scan": (C.c_longlong, [C.c_char_p, C.c_longlong, C.c_void_p, C.c_longlong,
                                         C.POINTER(C.c_longlong)]),
})


class EventFileWriter:
    def __init__(self, logdir, filename_suffix=""):
        self.logdir = Path(logdir)
        self.logdir.mkdir(parents=True, exist_ok=True)
        self.path = self.logdir / f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}{filename_suffix}"
        self._lib = N.host()
        self._h = self._lib.tde_events_open(str(self.path).encode())
        if not self._h:
            raise IOError(f"cannot open {self.path}")
        self._lib.tde_events_write_version(self._h, time.time())

    def add_scalars(self, step, values: dict, wall_time=None):
        tags = list(values)
        n = len(tags)
        ct = (C.c_char_p * n)(*[t.encode() for t in tags])
        cv = (C.c_float * n)(*[float(values[t]) for t in tags])
        rc = self._lib.tde_events_write_scalars(self._h, wall_time or time.time(), int(step), n, ct, cv)
        if rc != 0:
            raise IOError("event write failed")

    def add_scalar(self, tag, value, step, wall_time=None):
        self.add_scalars(step, {tag: value}, wall_time)

    def flush(self):
        self._lib.tde_events_flush(self._h)

    def close(self):
        if self._h:
            self._lib.tde_events_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ minimal proto decoding (tests/tools)
def _varint(b, i):
    r = s = 0
    while True:
        x = b[i]
        i += 1
        r |= (x & 0x7F) << s
        if x < 0x80:
            return r, i
        s += 7


def _fields(b):
    i = 0
    while i < len(b):
        tag, i = _varint(b, i)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 2:
            n, i = _varint(b, i)
            v = b[i:i + n]
            i += n
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        else:
            raise ValueError("bad wire type")
        yield f, wt, v


def parse_event(rec: bytes) -> dict:
    ev = {"scalars": {}, "step": 0}   # proto3: a zero step is not on the wire
    for f, wt, v in _fields(rec):
        if f == 1 and wt == 1:
            ev["wall_time"] = struct.unpack("<d", v)[0]
        elif f == 2 and wt == 0:
            ev["step"] = v
        elif f == 3 and wt == 2:
            ev["file_version"] = v.decode()
        elif f == 5 and wt == 2:
            for f2, _, val in _fields(v):
                if f2 != 1:
                    continue
                tag, sv = None, None
                for f3, wt3, x in _fields(val):
                    if f3 == 1:
                        tag = x.decode()
                    elif f3 == 2 and wt3 == 5:
                        sv = struct.unpack("<f", x)[0]
                if tag is not None:
                    ev["scalars"][tag] = sv
    return ev


def read_events(path) -> list:
    lib = N.host()
    n = lib.tde_tfrecord_scan(str(path).encode(), -1, None, 0, None)
    if n < 0:
        raise IOError(f"corrupt TFRecord {path} at record {-n - 1}")
    out = []
    buf = C.create_string_buffer(1 << 20)
    ln = C.c_longlong()
    for i in range(n):
        lib.tde_tfrecord_scan(str(path).encode(), i, buf, len(buf), C.byref(ln))
        out.append(parse_event(buf.raw[:ln.value]))
    return out
