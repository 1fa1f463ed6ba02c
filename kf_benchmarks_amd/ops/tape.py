"""Recording and replaying a training step as a launch tape (csrc/tape.hip).

The reference executes a step as one call into TF's C++ executor
(tcb/benchmark_cnn.py:821, ``sess.run(fetches)``); eager PyTorch spends
~20 us of Python per kernel launch instead.  A :class:`StepTape` records
one eager step - every native call it makes, with its raw arguments - and
replays it from C++ afterwards, so a step costs one Python call.

What makes a recorded step replayable:

* every GPU operation of the step goes through :func:`_native.call`
  (kernels, zero fills :func:`_native.zero_`, cross-stream waits
  :func:`_native.stream_wait`); a torch kernel inside the step would be
  silently skipped at replay, so :meth:`StepTape.record` checks with the
  profiler-free counter below that no torch op ran on the device;
* the step allocates from a private memory pool that nothing else allocates
  from afterwards, so every recorded address stays owned by the tape;
  tensors handed to another stream (``record_stream``) are held until the
  step ends, so no address is reused within the step across streams;
* per-step scalars are passed as :func:`_native.dyn` values (learning rate,
  RNG seeds) and patched at every replay.

Used by ``BenchmarkCNN.train_step`` under ``--launch_tape`` (single-process
runs and runs whose gradient collectives are native calls).
"""

from __future__ import annotations

import ctypes
import struct
from typing import Callable, Dict, List, Optional, Tuple

import torch

from . import _native as N

_CODE = {ctypes.c_int: "i", ctypes.c_uint32: "u", ctypes.c_long: "l", ctypes.c_longlong: "l",
         ctypes.c_size_t: "q", ctypes.c_uint64: "q", ctypes.c_void_p: "p", ctypes.c_char_p: "p",
         ctypes.c_float: "f"}
_MASK = (1 << 64) - 1


class TapeError(RuntimeError):
    def __init__(self, msg, outputs=None):
        super().__init__(msg)
        self.outputs = outputs  # the step's results when the step itself completed


def _pack(v, code, keep=None):
    if isinstance(v, ctypes._SimpleCData):
        v = v.value
    if code == "f":
        return struct.unpack("<I", struct.pack("<f", float(v)))[0]
    if code == "p":
        if v is None:
            return 0
        if isinstance(v, int):
            return v & _MASK
        if isinstance(v, ctypes.Array) and keep is not None:
            # a host argument table (e.g. the concat kernel's pointer list):
            # the tape keeps its own copy alive and passes that every replay
            copy = (v._type_ * len(v))(*v)
            keep.append(copy)
            return ctypes.addressof(copy)
        raise TapeError("pointer argument %r cannot be recorded" % (v,))
    return int(v) & _MASK


# Entry points whose work is not only kernel launches on the given streams
# (collectives, host registration, events, stream creation): a replay always
# calls them, never the raw launches recorded under them.
_NO_RAW_PREFIX = ("kfb_rccl_", "kfb_host_", "kfb_event_", "kfb_stream_create", "kfb_tape_",
                  "kfb_seqlock_")


class Recorder:
    """One native launch tape: ``add`` appends calls, ``replay`` re-issues them.

    Calls recorded through ``call`` also capture the device work they issued
    (kernel function + grid + argument bytes, memsets, stream waits, copies):
    a replay re-issues that with ``hipLaunchKernel`` directly, skipping the
    entry point's host logic (shape checks, algorithm choice, argument
    packing), unless the op has a per-step argument (Dyn) or did something
    else (an RCCL call) while recorded.  KFB_TAPE_RAW=0 turns this off."""

    def __init__(self):
        lib = N.load()
        if not lib.kfb_tape_available():
            raise TapeError("launch tape unavailable (libffi not loadable)")
        self.h = lib.kfb_tape_new()
        self.dyn: List[Tuple[int, int, str, str]] = []  # (op, arg, key, code)
        self._codes = {}
        self.names: List[str] = []
        self._keep = []  # host argument tables the recorded calls point into

    def _types(self, name, fn):
        t = self._codes.get(name)
        if t is None:
            try:
                t = "".join(_CODE[a] for a in fn.argtypes)
            except KeyError as e:
                raise TapeError("%s: argument type %s cannot be recorded" % (name, e))
            self._codes[name] = t
        return t

    def add(self, name, fn, args):
        types = self._types(name, fn)
        if len(args) != len(types):
            raise TapeError("%s: %d args for %d types" % (name, len(args), len(types)))
        slots = (ctypes.c_uint64 * max(len(args), 1))()
        out = list(args)
        op = len(self.names)
        dyn = []
        for k, (a, c) in enumerate(zip(args, types)):
            if isinstance(a, N.Dyn):
                dyn.append((op, k, a.key, c))
                a = out[k] = a.value
            slots[k] = _pack(a, c, self._keep)
        fp = ctypes.cast(fn, ctypes.c_void_p).value
        got = N.load().kfb_tape_add(self.h, fp, types.encode(), slots, len(args))
        if got != op:
            raise TapeError("kfb_tape_add(%s) failed" % name)
        self.names.append(name)
        self.dyn.extend(dyn)
        return out

    def call(self, name, fn, args):
        """Records ``name(*args)`` and executes it, capturing its device work."""
        n0 = len(self.names)
        out = self.add(name, fn, args)
        if len(self.names) != n0 + 1:  # (not appended: a test's dropped op)
            return fn(*out)
        op = n0
        lib = N.load()
        lib.kfb_tape_begin_op(self.h, op)
        err = -1
        try:
            err = fn(*out)
        finally:
            allow = 0 if (err != 0 or name.startswith(_NO_RAW_PREFIX)) else 1
            lib.kfb_tape_end_op(self.h, op, allow)
        return err

    def raw_ops(self) -> int:
        """Ops a replay re-issues as raw launches (the rest call their entry point)."""
        return N.load().kfb_tape_raw_ops(self.h)

    def keys(self):
        return sorted({k for _, _, k, _ in self.dyn})

    def replay(self, values: Dict[str, float]):
        n = len(self.dyn)
        if n:
            po = (ctypes.c_int * n)()
            pa = (ctypes.c_int * n)()
            pv = (ctypes.c_uint64 * n)()
            for i, (op, arg, key, code) in enumerate(self.dyn):
                if key not in values:
                    raise TapeError("no value for per-step argument %r" % key)
                po[i], pa[i], pv[i] = op, arg, _pack(values[key], code)
        else:
            po = pa = pv = None
        bad = ctypes.c_int(-1)
        rc = N.load().kfb_tape_replay(self.h, po, pa, pv, n, ctypes.byref(bad))
        if rc != 0:
            name = self.names[bad.value] if 0 <= bad.value < len(self.names) else "?"
            raise TapeError("tape replay failed at op %d (%s): error %d" % (bad.value, name, rc))

    def __len__(self):
        return len(self.names)

    def host_profile(self, replays: int, top: int = 12) -> str:
        """Host time per replayed step by native entry point (KFB_TAPE_PROFILE)."""
        n = len(self.names)
        buf = (ctypes.c_double * n)()
        N.load().kfb_tape_host_times(self.h, buf)
        by: Dict[str, List[float]] = {}
        for name, t in zip(self.names, buf):
            by.setdefault(name, []).append(t)
        tot = sum(buf) / max(replays, 1)
        rows = sorted(by.items(), key=lambda kv: -sum(kv[1]))[:top]
        out = ["tape host time per replayed step: %.3f ms over %d calls (%d raw, %d device ops)"
               % (1e3 * tot, n, self.raw_ops(), N.load().kfb_tape_raw_launches(self.h))]
        for name, ts in rows:
            out.append("  %-28s %5d calls %8.3f ms  %6.2f us/call" % (
                name, len(ts), 1e3 * sum(ts) / max(replays, 1),
                1e6 * sum(ts) / max(replays, 1) / len(ts)))
        return "\n".join(out)

    def close(self):
        if self.h:
            N.load().kfb_tape_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class _TorchKernelProbe:
    """Counts torch device work launched while recording (a torch op inside
    the step would be missing from the tape): wraps the dispatcher with a
    TorchDispatchMode that flags every op producing or mutating a CUDA
    tensor, except allocation/view ops, which launch nothing."""

    _HOST_ONLY = {"empty", "empty_strided", "empty_like", "view", "_unsafe_view", "reshape",
                  "as_strided", "slice", "select", "detach", "alias", "t", "transpose",
                  "permute", "expand", "unsqueeze", "squeeze", "split", "split_with_sizes",
                  "narrow", "_reshape_alias", "lift_fresh", "unbind", "chunk",
                  "tensor_split", "view_as", "_to_copy_noop", "set_", "resize_",
                  "new_empty", "new_empty_strided", "clone_noop", "is_same_size", "sym_size",
                  "sym_stride", "sym_numel", "sym_storage_offset", "record_stream"}

    def __init__(self):
        from torch.utils._python_dispatch import TorchDispatchMode
        probe = self

        class Mode(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                name = func.__name__.split(".")[0]
                if name in ("add", "add_"):
                    # the autograd engine's own sums of a multi-use tensor's
                    # incoming gradients (no Python frame of ours): run as
                    # the native add, a recorded call, instead of a torch
                    # kernel the tape would miss
                    y = _native_add(func, args, kwargs)
                    if y is not None:
                        probe.native_adds += 1
                        return y
                out = func(*args, **(kwargs or {}))
                if name not in probe._HOST_ONLY:
                    flat = [out] if isinstance(out, torch.Tensor) else (
                        list(out) if isinstance(out, (tuple, list)) else [])
                    flat += [a for a in args if isinstance(a, torch.Tensor)]
                    if any(isinstance(t, torch.Tensor) and t.is_cuda for t in flat):
                        import traceback
                        where = [f for f in traceback.extract_stack()
                                 if "kf_benchmarks_amd" in f.filename and "tape.py" not in f.filename]
                        site = ("%s:%d" % (where[-1].filename.split("kf_benchmarks_amd/")[-1],
                                           where[-1].lineno)) if where else "?"
                        probe.ops.append("%s@%s" % (name, site))
                return out

        self.mode = Mode()
        self.ops: List[str] = []
        self.native_adds = 0


def _native_add(func, args, kwargs):
    """``a + b`` / ``a += b`` as kfb_add when it is a plain same-shape sum of
    contiguous, 16-byte aligned CUDA tensors of a native dtype (None: leave
    it to torch)."""
    aten = torch.ops.aten
    inplace = func is aten.add_.Tensor
    if not (inplace or func is aten.add.Tensor) or len(args) != 2:
        return None
    a, b = args
    if (kwargs or {}).get("alpha", 1) != 1 or not isinstance(a, torch.Tensor) \
            or not isinstance(b, torch.Tensor):
        return None
    if not (a.is_cuda and b.is_cuda and a.device == b.device and a.dtype == b.dtype
            and a.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and a.shape == b.shape and a.is_contiguous() and b.is_contiguous()
            and a.numel() > 0 and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0):
        return None
    y = a if inplace else torch.empty_like(a)
    N.call("kfb_add", N.dt(a), a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), 0,
           N.stream(a.device))
    return y


class StepTape:
    """A recorded training step for one device (see module docstring)."""

    def __init__(self, device: torch.device):
        self.device = device
        self.recorder: Optional[Recorder] = None
        self.pool = None
        self.outputs = None
        self.replays = 0

    @property
    def ready(self) -> bool:
        return self.recorder is not None

    def record(self, step: Callable[[], object], check_torch_ops: bool = True):
        """Runs ``step()`` once eagerly while recording it; returns its result
        (tensors in it stay valid and are rewritten by every replay)."""
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        torch.cuda.synchronize(self.device)
        rec = Recorder()
        self.pool = torch.cuda.MemPool()
        keep = []
        orig_rs = torch.Tensor.record_stream

        def record_stream(t, s):
            keep.append(t)  # no cross-stream reuse inside the recorded step
            return orig_rs(t, s)

        probe = _TorchKernelProbe() if check_torch_ops else None
        # torch's stream-ordering calls are neither native calls nor
        # dispatcher ops: recorded silently they would vanish at replay and
        # leave a consumer stream unordered behind its producer, so any made
        # while recording refuses the tape (use _native.stream_wait)
        waits: List[str] = []
        orig_ws, orig_we = torch.cuda.Stream.wait_stream, torch.cuda.Stream.wait_event

        def _flag(kind):
            import traceback
            where = [f for f in traceback.extract_stack()
                     if "kf_benchmarks_amd" in f.filename and "tape.py" not in f.filename]
            waits.append("%s@%s" % (kind, ("%s:%d" % (where[-1].filename.split(
                "kf_benchmarks_amd/")[-1], where[-1].lineno)) if where else "?"))

        def wait_stream(s, other):
            _flag("Stream.wait_stream")
            return orig_ws(s, other)

        def wait_event(s, ev):
            _flag("Stream.wait_event")
            return orig_we(s, ev)

        # the per-step statistics arena (conv_hip.STATS_ARENA) is global: the
        # tape keeps the buffers its replays write alive, and a buffer the
        # arena grows into while recording (from this tape's pool) is dropped
        # from the arena when the tape closes
        from . import conv_hip
        self._arena_before = conv_hip.STATS_ARENA.snapshot()
        torch._C._cuda_beginAllocateToPool(dev, self.pool.id)
        torch.Tensor.record_stream = record_stream
        torch.cuda.Stream.wait_stream, torch.cuda.Stream.wait_event = wait_stream, wait_event
        N._TAPE = rec
        try:
            if probe is not None:
                with probe.mode:
                    out = step()
            else:
                out = step()
        except BaseException:
            self._release_arena()
            raise
        finally:
            N._TAPE = None
            torch.Tensor.record_stream = orig_rs
            torch.cuda.Stream.wait_stream, torch.cuda.Stream.wait_event = orig_ws, orig_we
            torch._C._cuda_endAllocateToPool(dev, self.pool.id)
        torch.cuda.synchronize(self.device)
        del keep
        self._arena_keep = conv_hip.STATS_ARENA.snapshot()
        if waits:
            self._release_arena()
            rec.close()
            raise TapeError("torch stream waits inside the recorded step (not replayable): %s"
                            % sorted(set(waits)), outputs=out)
        if probe is not None and probe.ops:
            self._release_arena()
            rec.close()
            raise TapeError("torch device ops inside the recorded step (not replayable): %s"
                            % sorted(set(probe.ops)), outputs=out)
        self.recorder = rec
        self.outputs = out
        return out

    def replay(self, values: Dict[str, float]):
        self.recorder.replay(values)
        self.replays += 1
        return self.outputs

    def _release_arena(self):
        before = getattr(self, "_arena_before", None)
        if before is not None:
            from . import conv_hip
            conv_hip.STATS_ARENA.forget_new(before)
            self._arena_before = None
        self._arena_keep = None

    def close(self):
        if self.recorder is not None:
            self.recorder.close()
            self.recorder = None
        self._release_arena()
        self.outputs = None
        self.pool = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass
