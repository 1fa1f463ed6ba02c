"""TensorBoard event-file writer (no TensorFlow): scalar and histogram
summaries encoded as tensorflow.Event protos inside TFRecord framing, written
through the native runtime.  Role of tf.summary.FileWriter + the
--summary_verbosity summaries of tcb/benchmark_cnn.py:2811-2846."""

from __future__ import annotations

import os
import socket
import struct
import time
from typing import Dict, Optional

import numpy as np

from .. import runtime

_v = runtime._varint


def _fb(field, payload: bytes) -> bytes:
    return _v((field << 3) | 2) + _v(len(payload)) + payload


def _fd(field, x: float) -> bytes:  # double
    return _v((field << 3) | 1) + struct.pack("<d", x)


def _ff(field, x: float) -> bytes:  # float
    return _v((field << 3) | 5) + struct.pack("<f", x)


def _fi(field, x: int) -> bytes:
    return _v(field << 3) + _v(int(x))


def _event(step: int, summary: Optional[bytes] = None, file_version: Optional[str] = None,
           wall_time: Optional[float] = None) -> bytes:
    b = _fd(1, wall_time if wall_time is not None else time.time())
    b += _fi(2, step)
    if file_version:
        b += _fb(3, file_version.encode())
    if summary is not None:
        b += _fb(5, summary)
    return b


def scalar_value(tag: str, value: float) -> bytes:
    return _fb(1, _fb(1, tag.encode()) + _ff(2, float(value)))


def histogram_value(tag: str, values) -> bytes:
    a = np.asarray(values, dtype=np.float64).ravel()
    if a.size == 0:
        a = np.zeros(1)
    edges = _default_buckets()
    idx = np.searchsorted(edges, a, side="left")
    counts = np.bincount(np.minimum(idx, len(edges) - 1), minlength=len(edges)).astype(np.float64)
    keep = counts > 0
    limits, cnt = edges[keep], counts[keep]
    h = (_fd(1, float(a.min())) + _fd(2, float(a.max())) + _fd(3, float(a.size)) +
         _fd(4, float(a.sum())) + _fd(5, float((a * a).sum())) +
         _fb(6, struct.pack("<%dd" % len(limits), *limits)) +
         _fb(7, struct.pack("<%dd" % len(cnt), *cnt)))
    return _fb(1, _fb(1, tag.encode()) + _fb(5, h))


_BUCKETS = None


def _default_buckets():
    global _BUCKETS
    if _BUCKETS is None:
        pos = []
        v = 1e-12
        while v < 1e20:
            pos.append(v)
            v *= 1.1
        _BUCKETS = np.array([-x for x in reversed(pos)] + [0.0] + pos + [np.finfo(np.float64).max])
    return _BUCKETS


class SummaryWriter:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        name = "events.out.tfevents.%d.%s" % (int(time.time()), socket.gethostname())
        self.path = os.path.join(logdir, name)
        self._w = runtime.TFRecordWriter(self.path)
        self._w.write(_event(0, file_version="brain.Event:2"))

    def add_summary_values(self, values: bytes, step: int):
        self._w.write(_event(step, summary=values))

    def add_scalars(self, scalars: Dict[str, float], step: int):
        self.add_summary_values(b"".join(scalar_value(k, v) for k, v in scalars.items()), step)

    def add_histograms(self, hists: Dict[str, object], step: int):
        self.add_summary_values(b"".join(histogram_value(k, v) for k, v in hists.items()), step)

    def flush(self):
        pass

    def close(self):
        self._w.close()


def read_events(path: str):
    """Decodes an event file written by SummaryWriter: [(step, {tag: value})]."""
    from .checkpoint import _parse_fields
    out = []
    for rec in runtime.tf_record_iterator(path):
        step, vals = 0, {}
        for f, wt, v in _parse_fields(rec):
            if f == 2:
                step = v
            elif f == 5:
                for f2, _, val in _parse_fields(v):
                    if f2 != 1:
                        continue
                    tag, sv = None, None
                    for f3, wt3, v3 in _parse_fields(val):
                        if f3 == 1:
                            tag = v3.decode()
                        elif f3 == 2:
                            sv = struct.unpack("<f", struct.pack("<I", v3))[0]
                        elif f3 == 5:
                            sv = "histogram"
                    vals[tag] = sv
        out.append((step, vals))
    return out
