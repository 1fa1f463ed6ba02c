"""ctypes binding of the native host runtime ``_lib/libkfb_rt.so``
(csrc/runtime/kfb_runtime.cpp): CRC32C, TFRecord reader/writer,
tf.train.Example decoding and the LevelDB-format table used by TF V2
checkpoint indexes."""

from __future__ import annotations

import ctypes
import os
import struct
import threading
from typing import Dict, Iterator, List, Tuple

from .. import build as _build

_LIB = None
_LOCK = threading.Lock()

c_char_p_p = ctypes.POINTER(ctypes.c_char_p)


def _load():
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        if not os.path.exists(_build.RT_LIB):
            _build.build_rt()
        lib = ctypes.CDLL(_build.RT_LIB)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        sz = ctypes.c_size_t
        lib.kfbrt_crc32c.argtypes = [ctypes.c_char_p, sz]
        lib.kfbrt_crc32c.restype = ctypes.c_uint32
        lib.kfbrt_crc32c_extend.argtypes = [ctypes.c_uint32, ctypes.c_char_p, sz]
        lib.kfbrt_crc32c_extend.restype = ctypes.c_uint32
        lib.kfbrt_masked_crc32c.argtypes = [ctypes.c_char_p, sz]
        lib.kfbrt_masked_crc32c.restype = ctypes.c_uint32
        lib.kfbrt_record_reader_open.argtypes = [ctypes.c_char_p, ctypes.c_int]
        lib.kfbrt_record_reader_open.restype = ctypes.c_void_p
        lib.kfbrt_record_reader_next.argtypes = [ctypes.c_void_p, ctypes.POINTER(u8p)]
        lib.kfbrt_record_reader_next.restype = ctypes.c_long
        lib.kfbrt_record_reader_close.argtypes = [ctypes.c_void_p]
        lib.kfbrt_record_writer_open.argtypes = [ctypes.c_char_p]
        lib.kfbrt_record_writer_open.restype = ctypes.c_void_p
        lib.kfbrt_record_writer_write.argtypes = [ctypes.c_void_p, ctypes.c_char_p, sz]
        lib.kfbrt_record_writer_write.restype = ctypes.c_int
        lib.kfbrt_record_writer_close.argtypes = [ctypes.c_void_p]
        lib.kfbrt_table_write.argtypes = [ctypes.c_char_p, ctypes.c_int, c_char_p_p,
                                          ctypes.POINTER(sz), c_char_p_p, ctypes.POINTER(sz)]
        lib.kfbrt_table_write.restype = ctypes.c_int
        lib.kfbrt_table_read.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
        lib.kfbrt_table_read.restype = ctypes.c_void_p
        lib.kfbrt_table_size.argtypes = [ctypes.c_void_p]
        lib.kfbrt_table_size.restype = ctypes.c_int
        cpp = ctypes.POINTER(ctypes.c_void_p)
        lib.kfbrt_table_entry.argtypes = [ctypes.c_void_p, ctypes.c_int, cpp, ctypes.POINTER(sz),
                                          cpp, ctypes.POINTER(sz)]
        lib.kfbrt_table_free.argtypes = [ctypes.c_void_p]
        lib.kfbrt_adjust_sat_hue.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_float,
                                             ctypes.c_float]
        lib.kfbrt_adjust_sat_hue.restype = None
        lib.kfbrt_parse_example.argtypes = [ctypes.c_char_p, sz, ctypes.c_void_p, sz]
        lib.kfbrt_parse_example.restype = ctypes.c_long
        _LIB = lib
        return lib


def crc32c(data: bytes, crc: int = 0) -> int:
    lib = _load()
    if crc:
        return lib.kfbrt_crc32c_extend(crc, data, len(data))
    return lib.kfbrt_crc32c(data, len(data))


def masked_crc32c(data: bytes) -> int:
    return _load().kfbrt_masked_crc32c(data, len(data))


def mask(crc: int) -> int:
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ------------------------------------------------------------------ TFRecord
class TFRecordCorrupt(IOError):
    pass


def tf_record_iterator(path: str, verify: bool = True) -> Iterator[bytes]:
    lib = _load()
    h = lib.kfbrt_record_reader_open(path.encode(), int(verify))
    if not h:
        raise IOError("cannot open %s" % path)
    try:
        out = ctypes.POINTER(ctypes.c_uint8)()
        while True:
            n = lib.kfbrt_record_reader_next(h, ctypes.byref(out))
            if n == -1:
                return
            if n < 0:
                raise TFRecordCorrupt("corrupt record in %s" % path)
            yield ctypes.string_at(out, n)
    finally:
        lib.kfbrt_record_reader_close(h)


class TFRecordWriter:
    def __init__(self, path: str):
        self._lib = _load()
        self._h = self._lib.kfbrt_record_writer_open(path.encode())
        if not self._h:
            raise IOError("cannot open %s for writing" % path)

    def write(self, record: bytes):
        if self._lib.kfbrt_record_writer_write(self._h, record, len(record)) != 0:
            raise IOError("write failed")

    def close(self):
        if self._h:
            self._lib.kfbrt_record_writer_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ------------------------------------------------------------- tf.Example
def parse_example(record: bytes) -> Dict[str, list]:
    """{feature key: list of bytes | float | int}."""
    lib = _load()
    cap = max(4 * len(record) + 256, 4096)
    while True:
        buf = ctypes.create_string_buffer(cap)
        n = lib.kfbrt_parse_example(record, len(record), buf, cap)
        if n == -2:
            cap *= 4
            continue
        if n < 0:
            raise ValueError("malformed tf.Example")
        break
    raw = buf.raw[:n]
    out: Dict[str, list] = {}
    i = 0
    while i < n:
        (klen,) = struct.unpack_from("<I", raw, i)
        i += 4
        key = raw[i:i + klen].decode()
        i += klen
        kind = raw[i]
        (count,) = struct.unpack_from("<I", raw, i + 1)
        i += 5
        vals: list = []
        if kind == 1:
            for _ in range(count):
                (bl,) = struct.unpack_from("<I", raw, i)
                i += 4
                vals.append(raw[i:i + bl])
                i += bl
        elif kind == 2:
            vals = list(struct.unpack_from("<%df" % count, raw, i))
            i += 4 * count
        elif kind == 3:
            vals = list(struct.unpack_from("<%dq" % count, raw, i))
            i += 8 * count
        out[key] = vals
    return out


# --- minimal protobuf encoding used by the writers (tf.Example for test data)
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _ld(field: int, payload: bytes) -> bytes:
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def make_example(features: Dict[str, list]) -> bytes:
    """Encode a tf.train.Example from {key: [bytes...] | [float...] | [int...]}."""
    entries = b""
    for key in sorted(features):
        vals = features[key]
        if vals and isinstance(vals[0], (bytes, bytearray)):
            lst = b"".join(_ld(1, bytes(v)) for v in vals)
            feat = _ld(1, lst)
        elif vals and isinstance(vals[0], float):
            lst = _ld(1, struct.pack("<%df" % len(vals), *vals))
            feat = _ld(2, lst)
        else:
            lst = _ld(1, b"".join(_varint(int(v)) for v in vals))
            feat = _ld(3, lst)
        entries += _ld(1, _ld(1, key.encode()) + _ld(2, feat))
    return _ld(1, entries)


def _feature_bytes(vals) -> bytes:
    if vals and isinstance(vals[0], (bytes, bytearray)):
        return _ld(1, b"".join(_ld(1, bytes(v)) for v in vals))
    if vals and isinstance(vals[0], float):
        return _ld(2, _ld(1, struct.pack("<%df" % len(vals), *vals)))
    return _ld(3, _ld(1, b"".join(_varint(int(v)) for v in vals)))


def _features_bytes(features: Dict[str, list]) -> bytes:
    return b"".join(_ld(1, _ld(1, k.encode()) + _ld(2, _feature_bytes(features[k])))
                    for k in sorted(features))


def make_sequence_example(context: Dict[str, list], feature_lists: Dict[str, list]) -> bytes:
    """Encode a tf.train.SequenceExample: ``feature_lists`` maps a key to a
    list of per-step value lists."""
    fl = b"".join(_ld(1, _ld(1, k.encode()) +
                      _ld(2, b"".join(_ld(1, _feature_bytes(step)) for step in feature_lists[k])))
                  for k in sorted(feature_lists))
    return _ld(1, _features_bytes(context)) + _ld(2, fl)


# --- protobuf wire decoding (SequenceExample; tf.Example goes through C++)
def _read_varint(b: bytes, i: int):
    shift = v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if c < 0x80:
            return v, i
        shift += 7


def _fields(b: bytes):
    """Yields (field number, wire type, value) of one message."""
    i, n = 0, len(b)
    while i < n:
        key, i = _read_varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 2:
            ln, i = _read_varint(b, i)
            v = b[i:i + ln]
            i += ln
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        else:
            raise ValueError("unsupported protobuf wire type %d" % wt)
        yield f, wt, v


def _decode_feature(b: bytes) -> list:
    for f, wt, v in _fields(b):
        if f == 1:
            return [bytes(x) for ff, _, x in _fields(v) if ff == 1]
        if f == 2:
            out = []
            for ff, w2, x in _fields(v):
                if w2 == 2:
                    out.extend(struct.unpack("<%df" % (len(x) // 4), x))
                elif w2 == 5:
                    out.append(struct.unpack("<f", x)[0])
            return out
        if f == 3:
            out = []
            for ff, w2, x in _fields(v):
                if w2 == 2:
                    j = 0
                    while j < len(x):
                        val, j = _read_varint(x, j)
                        out.append(val - (1 << 64) if val >= 1 << 63 else val)
                else:
                    out.append(x - (1 << 64) if x >= 1 << 63 else x)
            return out
    return []


def _decode_map(b: bytes, value_fn) -> Dict[str, object]:
    out = {}
    for f, _, entry in _fields(b):
        if f != 1:
            continue
        key, val = "", b""
        for ef, _, ev in _fields(entry):
            if ef == 1:
                key = bytes(ev).decode()
            elif ef == 2:
                val = ev
        out[key] = value_fn(val)
    return out


def parse_sequence_example(record: bytes):
    """-> (context {key: values}, feature_lists {key: [values per step]})."""
    ctx, lists = {}, {}
    for f, _, v in _fields(record):
        if f == 1:
            ctx = _decode_map(v, _decode_feature)
        elif f == 2:
            lists = _decode_map(v, lambda fl: [_decode_feature(x) for ff, _, x in _fields(fl)
                                               if ff == 1])
    return ctx, lists


# -------------------------------------------------------------------- tables
def table_write(path: str, items: List[Tuple[bytes, bytes]]):
    lib = _load()
    items = sorted(items)
    n = len(items)
    keys = (ctypes.c_char_p * n)(*[k for k, _ in items])
    klens = (ctypes.c_size_t * n)(*[len(k) for k, _ in items])
    vals = (ctypes.c_char_p * n)(*[v for _, v in items])
    vlens = (ctypes.c_size_t * n)(*[len(v) for _, v in items])
    rc = lib.kfbrt_table_write(path.encode(), n, keys, klens, vals, vlens)
    if rc != 0:
        raise IOError("table write failed (%d): %s" % (rc, path))


def table_read(path: str) -> List[Tuple[bytes, bytes]]:
    lib = _load()
    err = ctypes.c_int(0)
    h = lib.kfbrt_table_read(path.encode(), ctypes.byref(err))
    if not h:
        raise IOError("table read failed (%d): %s" % (err.value, path))
    try:
        out = []
        kp, vp = ctypes.c_void_p(), ctypes.c_void_p()
        kl, vl = ctypes.c_size_t(), ctypes.c_size_t()
        for i in range(lib.kfbrt_table_size(h)):
            lib.kfbrt_table_entry(h, i, ctypes.byref(kp), ctypes.byref(kl), ctypes.byref(vp),
                                  ctypes.byref(vl))
            out.append((ctypes.string_at(kp, kl.value), ctypes.string_at(vp, vl.value)))
        return out
    finally:
        lib.kfbrt_table_free(h)


def adjust_saturation_hue(img, sat: float, hue: float):
    """In place on a C-contiguous float32 [..., 3] RGB array (see
    kfbrt_adjust_sat_hue); returns the array."""
    import numpy as np
    assert img.dtype == np.float32 and img.flags["C_CONTIGUOUS"] and img.shape[-1] == 3
    _load().kfbrt_adjust_sat_hue(img.ctypes.data, img.size // 3, float(sat), float(hue))
    return img


class ImagePipe:
    """Native batch image pipeline (csrc/runtime/kfb_images.cpp): records ->
    uint8 [n, height, width, 3] crops, [n, 8] device-augmentation parameters
    and int32 labels, on ``threads`` native threads (the calling thread one
    of them), the GIL released for the whole batch."""

    def __init__(self, threads: int, height: int, width: int, distortions: bool,
                 distort_color_in_yiq: bool, draft: bool = True):
        lib = _load()
        if not getattr(lib, "_imgpipe_sigs", False):
            lib.kfbrt_imgpipe_available.restype = ctypes.c_int
            lib.kfbrt_imgpipe_create.argtypes = [ctypes.c_int] * 6
            lib.kfbrt_imgpipe_create.restype = ctypes.c_void_p
            lib.kfbrt_imgpipe_run.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 7
            lib.kfbrt_imgpipe_run.restype = ctypes.c_int
            lib.kfbrt_imgpipe_destroy.argtypes = [ctypes.c_void_p]
            lib._imgpipe_sigs = True
        self._lib = lib
        self.height, self.width = height, width
        self._h = lib.kfbrt_imgpipe_create(int(threads), int(height), int(width),
                                           int(bool(distortions)), int(bool(distort_color_in_yiq)),
                                           int(bool(draft)))

    @staticmethod
    def available() -> bool:
        try:
            lib = _load()
            lib.kfbrt_imgpipe_available.restype = ctypes.c_int
            return bool(lib.kfbrt_imgpipe_available())
        except (OSError, AttributeError):
            return False

    def run(self, records, seeds, positions=None):
        """-> (images uint8 [n,H,W,3], params float32 [n,8], labels int32 [n],
        number of undecodable images)."""
        import numpy as np
        n = len(records)
        bufs = (ctypes.c_char_p * n)(*records)
        lens = np.asarray([len(r) for r in records], dtype=np.uint64)
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        pos = np.ascontiguousarray(np.arange(n) if positions is None else positions, dtype=np.int32)
        images = np.empty((n, self.height, self.width, 3), dtype=np.uint8)
        params = np.empty((n, 8), dtype=np.float32)
        labels = np.empty((n,), dtype=np.int32)
        bad = self._lib.kfbrt_imgpipe_run(self._h, n, ctypes.cast(bufs, ctypes.c_void_p),
                                          lens.ctypes.data, seeds.ctypes.data, pos.ctypes.data,
                                          images.ctypes.data, params.ctypes.data,
                                          labels.ctypes.data)
        return images, params, labels, bad

    def run_coef(self, records, seeds, slot, positions=None):
        """GPU-reconstruction form of :meth:`run` into the (pinned) buffers of
        ``slot`` (``descs`` uint8, ``blocks`` int16 [cap, 64], ``images``,
        ``params``, ``labels``): the host entropy-decodes and packs each
        crop's coefficient blocks (ops/jpeg.decode finishes on the GPU);
        images whose layout the device path does not cover are decoded here
        into ``images``.  -> (blocks used, images decoded on the host,
        undecodable images)."""
        import numpy as np
        lib = self._lib
        if not getattr(lib, "_coef_sigs", False):
            lib.kfbrt_imgpipe_run_coef.argtypes = [ctypes.c_void_p, ctypes.c_int] + \
                [ctypes.c_void_p] * 6 + [ctypes.c_long] + [ctypes.c_void_p] * 4
            lib.kfbrt_imgpipe_run_coef.restype = ctypes.c_int
            lib._coef_sigs = True
        n = len(records)
        bufs = (ctypes.c_char_p * n)(*records)
        lens = np.asarray([len(r) for r in records], dtype=np.uint64)
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        pos = np.ascontiguousarray(np.arange(n) if positions is None else positions, dtype=np.int32)
        out2 = (ctypes.c_long * 3)()
        bad = lib.kfbrt_imgpipe_run_coef(
            self._h, n, ctypes.cast(bufs, ctypes.c_void_p), lens.ctypes.data, seeds.ctypes.data,
            pos.ctypes.data, slot.descs.data_ptr(), slot.blocks.data_ptr(),
            slot.blocks.shape[0], slot.images.data_ptr(), slot.params.data_ptr(),
            slot.labels.data_ptr(), out2)
        self.crop_pixels = int(out2[2])
        return int(out2[0]), int(out2[1]), bad

    def close(self):
        if getattr(self, "_h", None):
            self._lib.kfbrt_imgpipe_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def jpeg_desc_bytes() -> int:
    lib = _load()
    lib.kfbrt_jpeg_desc_bytes.restype = ctypes.c_int
    return int(lib.kfbrt_jpeg_desc_bytes())


def coef_pipeline_available() -> bool:
    """The host half of the GPU JPEG path (libjpeg with
    jpeg_read_coefficients) is loadable."""
    if not ImagePipe.available():
        return False
    try:
        return jpeg_desc_bytes() > 0
    except (OSError, AttributeError):
        return False


def jpeg_reconstruct(descs, n, blocks, images, height, width, out):
    """Host reference of csrc/jpeg.hip (numpy arrays; ``out`` uint8
    [n, height, width, 3] is filled)."""
    import numpy as np
    lib = _load()
    lib.kfbrt_jpeg_reconstruct.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_long, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_void_p]
    lib.kfbrt_jpeg_reconstruct.restype = None
    descs = np.ascontiguousarray(descs)
    blocks = np.ascontiguousarray(blocks, dtype=np.int16)
    img = None if images is None else np.ascontiguousarray(images)
    lib.kfbrt_jpeg_reconstruct(descs.ctypes.data, int(n), blocks.ctypes.data, blocks.size // 64,
                               None if img is None else img.ctypes.data, int(height), int(width),
                               out.ctypes.data)
    return out


def jpeg_decode_coef(data: bytes):
    """Test hook: the whole JPEG through the coefficient path (host form) ->
    uint8 [h, w, 3], or None when its layout is not covered."""
    import numpy as np
    lib = _load()
    lib.kfbrt_jpeg_decode_coef.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p,
                                           ctypes.c_size_t, ctypes.c_void_p]
    cap = 64 << 20
    buf = np.empty((cap,), np.uint8)
    hw = (ctypes.c_int * 2)()
    if lib.kfbrt_jpeg_decode_coef(data, len(data), buf.ctypes.data, cap, hw) != 0:
        return None
    h, w = hw[0], hw[1]
    return buf[:h * w * 3].reshape(h, w, 3).copy()
