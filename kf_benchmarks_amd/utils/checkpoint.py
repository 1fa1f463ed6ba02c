"""TF-V2-bundle-compatible checkpoints (role of tf.train.Saver in
tcb/benchmark_cnn.py:905-950, 2076-2082, 2304-2309, 2374-2378).

Layout written into ``train_dir``::

    model.ckpt-<step>.index                   LevelDB table: name -> BundleEntryProto
    model.ckpt-<step>.data-00000-of-00001     tensor bytes, concatenated
    checkpoint                                text CheckpointState (latest + history)

Variable names follow the reference graph: ``v0/cg/<scope>/conv2d/kernel``
(kernels in TF layout [KH, KW, Cin, Cout]), ``.../batchnorm<i>/{gamma,beta,
moving_mean,moving_variance}``, ``.../affine<i>/{weights,biases}``,
optimizer slots ``<var>/Momentum`` (``RMSProp``/``RMSProp_1``,
``Adam``/``Adam_1`` + ``beta1_power``/``beta2_power``) and ``global_step``
(int64).  In parameter_server mode the prefix is ``v/cg/`` as in the
reference's shared-variable scope.

The .index table and CRC32C go through the native runtime
(csrc/runtime/kfb_runtime.cpp); the small protobufs are encoded here.
"""

from __future__ import annotations

import glob
import os
import re
import struct
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import cnn_util, runtime

_DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3,
       np.dtype(np.uint8): 4, np.dtype(np.int64): 9, np.dtype(np.float16): 19}
_DT_BF16 = 14
_NP = {v: k for k, v in _DT.items()}


class CheckpointNotFoundException(Exception):
    pass


# --------------------------------------------------------- protobuf helpers
def _varint(v: int) -> bytes:
    return runtime._varint(v)


def _field_varint(field: int, v: int) -> bytes:
    return _varint(field << 3) + _varint(v)


def _field_bytes(field: int, b: bytes) -> bytes:
    return _varint((field << 3) | 2) + _varint(len(b)) + b


def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    v, shift = 0, 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if not c & 0x80:
            return v, i
        shift += 7


def _parse_fields(b: bytes) -> List[Tuple[int, int, object]]:
    out, i = [], 0
    while i < len(b):
        tag, i = _read_varint(b, i)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 2:
            ln, i = _read_varint(b, i)
            v = b[i:i + ln]
            i += ln
        elif wt == 5:
            v = struct.unpack_from("<I", b, i)[0]
            i += 4
        elif wt == 1:
            v = struct.unpack_from("<Q", b, i)[0]
            i += 8
        else:
            raise ValueError("bad wire type %d" % wt)
        out.append((f, wt, v))
    return out


def _encode_entry(dtype_enum: int, shape, offset: int, size: int, crc: int) -> bytes:
    dims = b"".join(_field_bytes(2, _field_varint(1, int(d))) for d in shape)
    b = _field_varint(1, dtype_enum) + _field_bytes(2, dims)
    if offset:
        b += _field_varint(4, offset)
    if size:
        b += _field_varint(5, size)
    b += _varint((6 << 3) | 5) + struct.pack("<I", crc)
    return b


def _decode_entry(b: bytes):
    dtype, shape, offset, size, crc, shard = 1, [], 0, 0, None, 0
    for f, wt, v in _parse_fields(b):
        if f == 1:
            dtype = v
        elif f == 2:
            for f2, _, v2 in _parse_fields(v):
                if f2 == 2:
                    size_d = 0
                    for f3, _, v3 in _parse_fields(v2):
                        if f3 == 1:
                            size_d = v3
                    shape.append(size_d)
        elif f == 3:
            shard = v
        elif f == 4:
            offset = v
        elif f == 5:
            size = v
        elif f == 6:
            crc = v
    return dtype, shape, offset, size, crc, shard


def _header() -> bytes:
    # BundleHeaderProto{num_shards=1, endianness=LITTLE(0), version{producer=1}}
    return _field_varint(1, 1) + _field_bytes(3, _field_varint(1, 1))


# ------------------------------------------------------------- bundle I/O
def _to_numpy(t) -> Tuple[np.ndarray, int]:
    if isinstance(t, torch.Tensor):
        t = t.detach()
        if t.dtype == torch.bfloat16:
            a = t.cpu().contiguous().view(torch.int16).numpy()
            return a, _DT_BF16
        a = t.cpu().contiguous().numpy()
    else:
        a = np.asarray(t)
        if not a.flags["C_CONTIGUOUS"]:
            a = a.copy(order="C")  # (np.ascontiguousarray would turn scalars 1-d)
    return a, _DT[a.dtype]


def write_bundle(prefix: str, tensors: Dict[str, object]):
    """Writes ``prefix.index`` + ``prefix.data-00000-of-00001``."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    items = [(b"", _header())]
    offset = 0
    data_path = prefix + ".data-00000-of-00001"
    tmp = data_path + ".tmp"
    with open(tmp, "wb") as f:
        for name in sorted(tensors):
            arr, dt = _to_numpy(tensors[name])
            raw = arr.tobytes()
            f.write(raw)
            crc = runtime.mask(runtime.crc32c(raw)) if raw else runtime.mask(0)
            items.append((name.encode(), _encode_entry(dt, arr.shape, offset, len(raw), crc)))
            offset += len(raw)
    os.replace(tmp, data_path)
    runtime.table_write(prefix + ".index", items)


def read_bundle(prefix: str, verify: bool = True) -> Dict[str, np.ndarray]:
    index = prefix + ".index"
    if not os.path.exists(index):
        raise CheckpointNotFoundException("no checkpoint index at %s" % index)
    entries = runtime.table_read(index)
    out = {}
    data = {}
    for key, val in entries:
        if key == b"":
            continue
        dtype, shape, offset, size, crc, shard = _decode_entry(val)
        dpath = prefix + ".data-%05d-of-%05d" % (shard, _num_shards(entries))
        if dpath not in data:
            with open(dpath, "rb") as fh:
                data[dpath] = fh.read()
        raw = data[dpath][offset:offset + size]
        if verify and crc is not None and runtime.mask(runtime.crc32c(raw)) != crc:
            raise IOError("checksum mismatch for %s" % key.decode())
        if dtype == _DT_BF16:
            a = torch.frombuffer(bytearray(raw), dtype=torch.bfloat16).float().numpy()
        else:
            a = np.frombuffer(raw, dtype=_NP[dtype]).copy()
        out[key.decode()] = a.reshape(tuple(shape))
    return out


def _num_shards(entries) -> int:
    for key, val in entries:
        if key == b"":
            for f, _, v in _parse_fields(val):
                if f == 1:
                    return v
    return 1


# ------------------------------------------------------- checkpoint state
def write_checkpoint_state(train_dir: str, latest: str, all_paths: List[str]):
    lines = ['model_checkpoint_path: "%s"' % latest]
    lines += ['all_model_checkpoint_paths: "%s"' % p for p in all_paths]
    tmp = os.path.join(train_dir, "checkpoint.tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(train_dir, "checkpoint"))


def get_checkpoint_state(train_dir: str):
    path = os.path.join(train_dir, "checkpoint")
    if not os.path.exists(path):
        return None
    latest, allp = None, []
    with open(path) as f:
        for line in f:
            m = re.match(r'\s*(\w+):\s*"(.*)"', line)
            if not m:
                continue
            if m.group(1) == "model_checkpoint_path":
                latest = m.group(2)
            elif m.group(1) == "all_model_checkpoint_paths":
                allp.append(m.group(2))
    if latest is None:
        return None
    if not os.path.isabs(latest):
        latest = os.path.join(train_dir, latest)
    allp = [p if os.path.isabs(p) else os.path.join(train_dir, p) for p in allp]
    return {"model_checkpoint_path": latest, "all_model_checkpoint_paths": allp}


def get_checkpoint_to_load(ckpt_dir: str) -> str:
    """Full checkpoint prefix for a ``.../model.ckpt-N`` path or a directory
    (latest), as tcb/benchmark_cnn.py:927-950."""
    if re.search(r"ckpt-\d+$", ckpt_dir):
        return ckpt_dir
    st = get_checkpoint_state(ckpt_dir)
    if st and st["model_checkpoint_path"]:
        return st["model_checkpoint_path"]
    raise CheckpointNotFoundException("No checkpoint file found in dir:{}".format(ckpt_dir))


def step_from_path(path: str) -> int:
    step = path.split("/")[-1].split("-")[-1]
    return int(step) if step.isdigit() else 0


# ------------------------------------------------------------------- Saver
_SLOT_NAMES = {"momentum": ("Momentum", None), "rmsprop": ("RMSProp_1", "RMSProp"),
               "adam": ("Adam", "Adam_1"), "sgd": (None, None)}


class Saver:
    """Saves/restores a BenchmarkCNN's model, optimizer slots and global step."""

    def __init__(self, bench, max_to_keep=5):
        self.bench = bench
        self.max_to_keep = max_to_keep
        vu = bench.params.variable_update
        # PS mode keeps one shared copy under scope "v"; per-tower modes save tower 0.
        self.prefix = "v/cg/" if vu == "parameter_server" else "v0/cg/"
        self._kept: List[str] = []

    # -- tensors
    def _collect(self) -> Dict[str, object]:
        b = self.bench
        with b.flat.real_values():  # staged_vars: save the real variables
            out = {k: (v.detach().cpu().clone() if torch.is_tensor(v) else v)
                   for k, v in b.net.tf_variables(prefix=self.prefix).items()}
        out["global_step"] = np.array(b.global_step, dtype=np.int64)
        opt = b.optimizer
        s1n, s2n = _SLOT_NAMES[opt.kind]
        flat = b.flat
        for name, p, off, n in flat.segments():
            tf_name = self.prefix + name
            shape = self._tf_shape(name, p)
            for slot, sname in ((opt.s1, s1n), (opt.s2, s2n)):
                if slot is None or sname is None:
                    continue
                out[tf_name + "/" + sname] = self._to_tf_layout(name, slot[off:off + n].view(
                    p.shape)).cpu()
        if opt.kind == "adam":
            out["beta1_power"] = np.array(opt.adam[0] ** (opt.t + 1), dtype=np.float32)
            out["beta2_power"] = np.array(opt.adam[1] ** (opt.t + 1), dtype=np.float32)
        return out

    @staticmethod
    def _tf_shape(name, p):
        return p.shape

    @staticmethod
    def _to_tf_layout(name, t):
        return t.permute(1, 2, 3, 0) if name.endswith("conv2d/kernel") and t.dim() == 4 else t

    @staticmethod
    def _from_tf_layout(name, a):
        t = torch.as_tensor(a)
        return t.permute(3, 0, 1, 2) if name.endswith("conv2d/kernel") and t.dim() == 4 else t

    def save(self, train_dir: str, global_step: int) -> str:
        prefix = os.path.join(train_dir, "model.ckpt-%d" % global_step)
        write_bundle(prefix, self._collect())
        if prefix in self._kept:
            self._kept.remove(prefix)
        self._kept.append(prefix)
        while self.max_to_keep and len(self._kept) > self.max_to_keep:
            old = self._kept.pop(0)
            for f in glob.glob(old + ".*"):
                os.remove(f)
        write_checkpoint_state(train_dir, os.path.basename(prefix),
                               [os.path.basename(p) for p in self._kept])
        return prefix

    def restore(self, path: str, strict: bool = True) -> int:
        values = read_bundle(path)
        b = self.bench
        prefix = self.prefix
        if not any(k.startswith(prefix) for k in values):
            alt = "v/cg/" if prefix == "v0/cg/" else "v0/cg/"
            if any(k.startswith(alt) for k in values):
                prefix = alt
        b.net.load_tf_variables(values, prefix=prefix, strict=strict)
        opt = b.optimizer
        s1n, s2n = _SLOT_NAMES[opt.kind]
        with torch.no_grad():
            for name, p, off, n in b.flat.segments():
                for slot, sname in ((opt.s1, s1n), (opt.s2, s2n)):
                    key = prefix + name + "/" + str(sname)
                    if slot is not None and sname is not None and key in values:
                        t = self._from_tf_layout(name, values[key]).reshape(-1)
                        slot[off:off + n].copy_(t.to(slot.device))
        b.flat.refresh_lp()
        step = int(values["global_step"]) if "global_step" in values else step_from_path(path)
        b.global_step = step
        if opt.kind == "adam":
            opt.t = step
        cnn_util.log_fn("Successfully loaded model from %s." % path)
        return step

    def restore_latest(self, train_dir: str) -> Optional[int]:
        try:
            path = get_checkpoint_to_load(train_dir)
        except CheckpointNotFoundException:
            return None
        return self.restore(path)

    def restore_partial(self, path: str) -> int:
        """--backbone_model_path: load whatever variables match by name."""
        path = get_checkpoint_to_load(path)
        values = read_bundle(path)
        n = self.bench.net.load_tf_variables(values, prefix=self.prefix, strict=False)
        self.bench.flat.refresh_lp()
        cnn_util.log_fn("Loaded %d backbone variables from %s" % (n, path))
        return n


def load_checkpoint(saver: Saver, ckpt_dir: str) -> int:
    """Returns the global step of the restored checkpoint."""
    path = get_checkpoint_to_load(ckpt_dir)
    saver.restore(path)
    return step_from_path(path)
