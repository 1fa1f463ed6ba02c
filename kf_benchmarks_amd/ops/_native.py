"""ctypes binding of ``_lib/libkfb_hip.so`` (our gfx950 kernels).

Every op in :mod:`kf_benchmarks_amd.ops` that runs on a GPU tensor goes
through this module.  If the library is missing or fails to load while a GPU
is in use we raise immediately: there is deliberately no silent PyTorch
fallback on the GPU path (the CPU path exists only for the ``--device=cpu``
plumbing config and for numerics references in tests).
"""

from __future__ import annotations

import ctypes
import os
import threading

import torch

from .. import build as _build

_LIB = None
_LOCK = threading.Lock()

F32, BF16, F16 = 0, 1, 2
_DT = {torch.float32: F32, torch.bfloat16: BF16, torch.float16: F16}

c_void_p, c_int, c_long, c_float, c_uint32 = (ctypes.c_void_p, ctypes.c_int, ctypes.c_long,
                                               ctypes.c_float, ctypes.c_uint32)
P = c_void_p
I = c_int
L = c_long
F = c_float

# name -> argtypes (restype is int = hipError_t unless listed in _RESTYPES)
_SIGS = {
    "kfb_bn_num_slabs": [L, I],
    "kfb_bn_fwd_train": [I, P, P, P, L, I, P, P, F, F, P, P, P, P, P, P, P, P, I, I, I, P, P, P],
    "kfb_bn_fwd_train_dual": [I, P, P, P, L, I, P, P, F, F, P, P, P, P, P, P, P, P, I,
                              P, P, F, F, P, P, P, P, P, P, P, P, I, I, P, P, P, P],
    "kfb_bn_bwd_dual": [I, P, P, P, P, P, L, I, P, P, P, P, P, P, P, I, P, P, P, I,
                        P, P, P, P, P, P, P, I, P, P, P, I, I, P],
    "kfb_bn_fwd_train_recompute": [I, P, P, P, P, P, I, I, I, I, I, P, P, F, F, P, P, P, P, P, P,
                                   P, P, I, I, P, I, P, P],
    "kfb_conv_s1_apply": [I, P, P, P, P, P, I, I, I, I, I, P, P, I, P, P],
    "kfb_bn_fwd_infer": [I, P, P, P, L, I, P, P, P, P, F, P, P, I, P],
    "kfb_bn_bwd": [I, P, P, P, P, P, L, I, P, P, P, P, P, P, P, I, P, P, P, I, I, I, P],
    "kfb_opt_step": [I, P, P, P, P, P, I, P, L, F, F, F, F, F, F, F, F, F, I, P, F, F, P, P, P],
    "kfb_seqlock_check": [P, ctypes.c_longlong, P, P, P],
    "kfb_event_create": [P],
    "kfb_event_create_device": [P],
    "kfb_event_destroy": [P],
    "kfb_stream_wait": [P, P, P],
    "kfb_event_timer_new": [I, P],
    "kfb_event_timer_mark": [P, I, P],
    "kfb_event_timer_read": [P, P, I],
    "kfb_event_timer_free": [P],
    "kfb_memset": [P, I, ctypes.c_size_t, P],
    "kfb_memcpy_d2d": [P, P, ctypes.c_size_t, P],
    "kfb_tape_available": [],
    "kfb_tape_new": [],
    "kfb_tape_free": [P],
    "kfb_tape_size": [P],
    "kfb_tape_add": [P, P, ctypes.c_char_p, P, I],
    "kfb_tape_patch": [P, I, I, ctypes.c_uint64],
    "kfb_tape_replay": [P, P, P, P, I, P],
    "kfb_tape_host_times": [P, P],
    "kfb_tape_begin_op": [P, I],
    "kfb_tape_end_op": [P, I, I],
    "kfb_tape_raw_ops": [P],
    "kfb_tape_raw_launches": [P],
    "kfb_tape_set_raw": [I],
    "kfb_host_register": [P, ctypes.c_size_t, P],
    "kfb_host_unregister": [P],
    "kfb_ipc_export": [P, P, P],
    "kfb_ipc_handle_bytes": [],
    "kfb_ipc_open": [P, I, P],
    "kfb_ipc_close": [P],
    "kfb_enable_peer": [I, I],
    "kfb_nonfinite": [P, L, P, P],
    "kfb_half_sumsq": [P, L, P, P],
    "kfb_cast_f32": [P, P, I, L, P],
    "kfb_cast_to_f32": [P, I, P, L, P],
    "kfb_xent_fwd": [I, P, P, L, I, P, P, P],
    "kfb_mean_f32": [P, L, P, P],
    "kfb_xent_bwd": [I, P, P, P, P, F, L, I, P, P],
    "kfb_in_top_k": [I, P, P, L, I, P, P, P],
    "kfb_maxpool_fwd": [I, P, P, P] + [I] * 12 + [P],
    "kfb_maxpool_bwd": [I, P, P, P] + [I] * 12 + [P],
    "kfb_avgpool_fwd": [I, P, P] + [I] * 12 + [P],
    "kfb_avgpool_bwd": [I, P, P] + [I] * 12 + [P],
    "kfb_gap_fwd": [I, P, P, I, I, I, P],
    "kfb_gap_bwd": [I, P, P, I, I, I, P],
    "kfb_bias_act": [I, P, P, P, L, I, I, P],
    "kfb_colsum_num_slabs": [L, I],
    "kfb_act_bwd_bias": [I, P, P, P, L, I, I, P, I, P, I, P],
    "kfb_dropout": [I, P, P, L, F, c_uint32, P],
    "kfb_synthetic_images": [I, P, L, F, F, c_uint32, P],
    "kfb_augment": [I, P, P, P, I, I, I, P, P],
    "kfb_augment_blocks": [],
    "kfb_synthetic_labels": [P, L, I, c_uint32, P],
    "kfb_synthetic_uniform": [I, P, L, F, F, c_uint32, c_uint32, P],
    "kfb_synthetic_ints": [P, L, I, c_uint32, c_uint32, P],
    "kfb_mul": [I, P, P, P, L, P],
    "kfb_mul_bwd": [I, P, P, P, P, P, L, P],
    "kfb_add": [I, P, P, P, L, I, P],
    "kfb_gemm": [I, I, P, I, P, I, I, I, I, P, I, P, I, I, P, L, I, P],
    "kfb_gemm_splits": [I, I, I, I],
    "kfb_lrn_fwd": [I, P, P, L, I, I, F, F, F, P],
    "kfb_lrn_bwd": [I, P, P, P, L, I, I, F, F, F, P],
    "kfb_embedding_fwd": [I, P, L, P, P, L, I, P],
    "kfb_embedding_bwd": [I, P, P, P, L, L, I, P],
    "kfb_concat": [I, P, P, P, I, L, I, I, I, P],
    "kfb_ssd_loss_fwd": [I, P, P, P, P, I, I, I, I, P, P, P],
    "kfb_ssd_loss_bwd": [I, P, P, P, P, P, P, I, I, I, P, P],
    "kfb_rnn_fwd": [I, I, P, P, P, P, P, P, P, I, I, I, I, P],
    "kfb_rnn_bwd": [I, I, P, P, P, P, P, P, P, P, P, I, I, I, I, P],
    "kfb_transpose_cast": [I, P, P, I, I, I, P],
    "kfb_permute01": [I, P, P, I, I, I, P],
    "kfb_ctc_loss": [I, P, L, L, P, P, P, I, I, I, I, P, P, I, P, P, P],
    "kfb_ctc_grad_scale": [I, P, P, P, L, L, I, I, I, P],
    "kfb_ctc_max_states": [],
    "kfb_ssd_heads": [I, P, P, I, I, I, I, L, I, L, I, I, P],
    "kfb_slab_colsum": [P, I, I, P, I, P],
}
_RESTYPES = {"kfb_ipc_handle_bytes": c_int, "kfb_bn_num_slabs": c_int, "kfb_colsum_num_slabs": c_int,
             "kfb_gemm_splits": c_int, "kfb_ctc_max_states": c_int, "kfb_tape_new": c_void_p,
             "kfb_tape_free": None, "kfb_tape_set_raw": None,
             "kfb_tape_raw_launches": ctypes.c_long}
# Optional symbols (added by later kernel files); bound if present.
_OPTIONAL = {}


class NativeError(RuntimeError):
    pass


def lib_path() -> str:
    # KFB_HIP_LIB: load an alternative build (kernel A/B experiments)
    return os.environ.get("KFB_HIP_LIB") or _build.HIP_LIB


def available() -> bool:
    return os.path.exists(lib_path())


def load():
    """Loads (building first if the .so is absent) and binds the library."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        path = lib_path()
        if not os.path.exists(path):
            if os.environ.get("KFB_NO_AUTOBUILD"):
                raise NativeError("native kernel library missing: %s (run "
                                  "`python -m kf_benchmarks_amd.build`)" % path)
            _build.build_all()
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, args in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, c_int)
        for name, (args, res) in _OPTIONAL.items():
            if hasattr(lib, name):
                fn = getattr(lib, name)
                fn.argtypes = args
                fn.restype = res
        _LIB = lib
        return lib


def register_optional(name, argtypes, restype=c_int):
    _OPTIONAL[name] = (argtypes, restype)
    if _LIB is not None and hasattr(_LIB, name):
        fn = getattr(_LIB, name)
        fn.argtypes = argtypes
        fn.restype = restype


_FN = {}

# The launch tape being recorded (ops/tape.py), or None.  While set, every
# call() is appended to it (and still executed).
_TAPE = None


class Dyn:
    """A per-step argument of a recorded call (learning rate, RNG seed): the
    tape patches it with the value for ``key`` at every replay."""
    __slots__ = ("key", "value")

    def __init__(self, key, value):
        self.key, self.value = key, value


def dyn(key, value):
    """``value``, marked as the per-step scalar ``key`` while a tape is being
    recorded (a plain value otherwise)."""
    return Dyn(key, value) if _TAPE is not None else value


def recording() -> bool:
    return _TAPE is not None


def call(name, *args):
    """Calls a kernel entry point and raises on a non-zero hipError_t."""
    fn = _FN.get(name)
    if fn is None:
        fn = _FN[name] = getattr(load(), name)
    if _TAPE is not None:
        err = _TAPE.call(name, fn, args)
    else:
        err = fn(*args)
    if err != 0:
        raise NativeError("%s failed with hipError %d" % (name, err))
    return err


def query(name, *args):
    return getattr(load(), name)(*args)


def dt(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise NativeError("unsupported dtype %s for native kernels" % t.dtype)


def ptr(t):
    return None if t is None else t.data_ptr()


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream(device=None) -> int:
    """hipStream_t of the current torch stream of ``device``.  The raw C
    accessor skips torch.cuda.current_stream's Stream-object construction
    (~5 us per kernel launch on the host, which the forward pass is bound by)."""
    if _RAW_STREAM is not None:
        if device is None:
            idx = torch.cuda.current_device()
        elif isinstance(device, int):
            idx = device
        else:
            if isinstance(device, str):
                device = torch.device(device)
            idx = device.index if device.index is not None else torch.cuda.current_device()
        return _RAW_STREAM(idx)
    return torch.cuda.current_stream(device).cuda_stream


def loaded_path():
    return lib_path() if _LIB is not None else None


# ------------------------------------------------- stream ordering / memory
_EVENTS = {}


def _pair_event(dst, src, device_only=False):
    key = (dst, src, device_only)
    ev = _EVENTS.get(key)
    if ev is None:
        h = ctypes.c_void_p()
        lib = load()
        err = (lib.kfb_event_create_device if device_only and _DEVICE_EVENTS
               else lib.kfb_event_create)(ctypes.byref(h))
        if err != 0:
            raise NativeError("kfb_event_create failed with hipError %d" % err)
        ev = _EVENTS[key] = h.value
    return ev


# compute-to-compute waits skip the system-scope fence (False: every
# cross-stream wait records with it)
_DEVICE_EVENTS = True


def stream_wait(dst_stream: int, src_stream: int, device_only: bool = False):
    """``dst`` waits for the work enqueued on ``src`` so far (raw hipStream_t
    handles) - the recordable form of torch's Stream.wait_stream.
    ``device_only``: both streams run kernels of this device and nothing on
    the host or another device reads what ``src`` wrote through this
    ordering, so the event skips the system-scope release fence."""
    if dst_stream == src_stream:
        return
    call("kfb_stream_wait", dst_stream, src_stream,
         _pair_event(dst_stream, src_stream, device_only))


def zero_(t: torch.Tensor):
    """Recordable zero fill of a contiguous device tensor."""
    if t.numel():
        call("kfb_memset", t.data_ptr(), 0, t.numel() * t.element_size(), stream(t.device))
    return t
