"""Python face of the native RCCL communicator (csrc/comm.hip).

One communicator per process (one process per GPU).  Rank 0 creates the
RCCL unique id and publishes it in the job's TCP store (the rendezvous of
``torch.distributed``'s env:// init, which here only carries host-side
traffic over gloo); every rank then calls ``ncclCommInitRank`` on its GPU.

Collectives run on the caller's current stream, as RCCL's own API does:
the bucket reducer issues them from the weight-gradient side stream, which
has already caught up with the compute stream, so the collective follows
both producers without a stream of its own; :meth:`Work.wait` makes the
then-current stream wait for the issuing one.  Both are native calls
(``kfb_rccl_*``, ``kfb_stream_wait``), so a recorded launch tape replays
them with the rest of the step.  (A dedicated collective stream - one more
stream waiting on the side stream - cost 28.5 vs 17.6 ms/step at one rank
at either priority, 24.3 at ordinary priority; profiles/r13_comm_stream_ab.txt.)
Replaces the reference's NCCL / Horovod / KungFu device collectives
(tcb/allreduce.py:297-299, tcb/benchmark_cnn.py:3122-3130, 2094-2100);
SURVEY section 7.1.
"""

from __future__ import annotations

import ctypes
import os

import torch

from ..ops import _native as N

_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3}
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3,
       torch.float64: 4}

N.register_optional("kfb_rccl_available", [], N.c_int)
N.register_optional("kfb_rccl_error_string", [N.c_int], ctypes.c_char_p)
N.register_optional("kfb_rccl_unique_id", [N.P], N.c_int)
N.register_optional("kfb_rccl_init", [N.I, N.P, N.I, N.I, N.P], N.c_int)
N.register_optional("kfb_rccl_destroy", [N.P, N.I], N.c_int)
N.register_optional("kfb_rccl_async_error", [N.P], N.c_int)
N.register_optional("kfb_rccl_all_reduce", [N.P, N.P, N.P, ctypes.c_size_t, N.I, N.I, N.P],
                    N.c_int)
N.register_optional("kfb_rccl_reduce", [N.P, N.P, N.P, ctypes.c_size_t, N.I, N.I, N.I, N.P],
                    N.c_int)
N.register_optional("kfb_rccl_broadcast", [N.P, N.P, N.P, ctypes.c_size_t, N.I, N.I, N.P],
                    N.c_int)
N.register_optional("kfb_rccl_all_gather", [N.P, N.P, N.P, ctypes.c_size_t, N.I, N.P], N.c_int)
N.register_optional("kfb_rccl_send", [N.P, N.P, ctypes.c_size_t, N.I, N.I, N.P], N.c_int)
N.register_optional("kfb_rccl_recv", [N.P, N.P, ctypes.c_size_t, N.I, N.I, N.P], N.c_int)
N.register_optional("kfb_rccl_group_start", [], N.c_int)
N.register_optional("kfb_rccl_group_end", [], N.c_int)


class RcclError(RuntimeError):
    pass


_LIVE = set()  # handles of this process's communicators not yet destroyed


def live_count() -> int:
    """Native communicators alive in this process (world + subgroups)."""
    return len(_LIVE)


def available() -> bool:
    try:
        return bool(N.load().kfb_rccl_available())
    except (OSError, AttributeError, N.NativeError):
        return False


def mode() -> str:
    """KFB_NATIVE_COMM: ``auto`` (default) - device collectives of a
    multi-process run on this communicator, validated at startup against
    torch's gloo group (:func:`comm.selftest_device_collectives`), falling
    back to torch's ProcessGroupNCCL if the check fails; ``1`` - this
    communicator, no fallback; ``0`` - torch's ProcessGroupNCCL only.  With
    the native communicator no ProcessGroupNCCL exists unless the fallback
    creates one: subgroups are native communicators too (:func:`subgroup`)."""
    v = os.environ.get("KFB_NATIVE_COMM", "auto").strip().lower()
    return v if v in ("0", "1", "auto") else "auto"


def enabled() -> bool:
    return mode() != "0"


def subgroup(world_native: "NativeComm", ranks, store, tag: str):
    """A native communicator over ``ranks`` (global ranks, ascending) for
    this process if it is a member, else None.  Collective over the members
    only: the first member publishes the RCCL unique id under ``tag`` in the
    job's TCP store (the same rendezvous as the world communicator)."""
    ranks = list(ranks)
    if world_native.rank not in ranks:
        return None
    return NativeComm(ranks.index(world_native.rank), len(ranks), world_native.device.index,
                      store, tag="sub/%s/%s" % (tag, ",".join(map(str, ranks))))


class Work:
    """Completion handle of a collective: the stream it was issued on."""

    __slots__ = ("stream_h", "device")

    def __init__(self, stream_h, device):
        self.stream_h, self.device = stream_h, device

    def wait(self):
        """The caller's current stream waits for the collective (no host wait)."""
        cur = N.stream(self.device)
        if cur != self.stream_h:
            N.stream_wait(cur, self.stream_h)

    def synchronize(self):
        torch.cuda.synchronize(self.device)


class NativeComm:
    """This rank's RCCL communicator (see module docstring)."""

    def __init__(self, rank: int, size: int, device_index: int, store, tag: str = "world"):
        lib = N.load()
        if not lib.kfb_rccl_available():
            raise RcclError("RCCL could not be loaded")
        self.rank, self.size = rank, size
        self.device = torch.device("cuda", device_index)
        key = "kfb_rccl_id/%s" % tag
        uid = ctypes.create_string_buffer(128)
        if rank == 0:
            self._check(lib.kfb_rccl_unique_id(uid), "ncclGetUniqueId")
            store.set(key, bytes(uid.raw))
        else:
            raw = store.get(key)
            ctypes.memmove(uid, raw, 128)
        h = ctypes.c_void_p()
        self._check(lib.kfb_rccl_init(size, uid, rank, device_index, ctypes.byref(h)),
                    "ncclCommInitRank")
        self.h = h.value
        self.collectives = 0
        _LIVE.add(self.h)
        from . import watchdog
        watchdog.add_comm(self.h)  # polled for async errors, aborted on a hang

    def _check(self, rc, what):
        if rc != 0:
            msg = N.load().kfb_rccl_error_string(rc)
            raise RcclError("%s failed: %s (%d)" % (what, msg.decode() if msg else "?", rc))

    def _enter(self, t: torch.Tensor) -> int:
        """The stream to issue on: the caller's current one."""
        if not t.is_cuda or not t.is_contiguous():
            raise RcclError("native collectives take contiguous device tensors")
        if t.dtype not in _DT:
            raise RcclError("dtype %s not supported by the native communicator" % t.dtype)
        self.collectives += 1
        return N.stream(t.device)

    def all_reduce(self, t, op="sum"):
        s = self._enter(t)
        N.call("kfb_rccl_all_reduce", self.h, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
               _OPS[op], s)
        return Work(s, t.device)

    def reduce(self, t, dst=0, op="sum"):
        s = self._enter(t)
        N.call("kfb_rccl_reduce", self.h, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
               _OPS[op], int(dst), s)
        return Work(s, t.device)

    def broadcast(self, t, src=0):
        s = self._enter(t)
        N.call("kfb_rccl_broadcast", self.h, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
               int(src), s)
        return Work(s, t.device)

    def all_gather(self, out, t):
        """out [size * t.numel()] receives every rank's t, rank-major."""
        s = self._enter(t)
        N.call("kfb_rccl_all_gather", self.h, t.data_ptr(), out.data_ptr(), t.numel(),
               _DT[t.dtype], s)
        return Work(s, t.device)

    def send(self, t, peer):
        s = self._enter(t)
        N.call("kfb_rccl_send", self.h, t.data_ptr(), t.numel(), _DT[t.dtype], int(peer), s)
        return Work(s, t.device)

    def recv(self, t, peer):
        s = self._enter(t)
        N.call("kfb_rccl_recv", self.h, t.data_ptr(), t.numel(), _DT[t.dtype], int(peer), s)
        return Work(s, t.device)

    def group_start(self):
        N.call("kfb_rccl_group_start")

    def group_end(self):
        N.call("kfb_rccl_group_end")

    def barrier(self):
        t = torch.zeros(1, device=self.device)
        self.all_reduce(t).wait()
        torch.cuda.synchronize(self.device)

    def check(self):
        rc = N.load().kfb_rccl_async_error(self.h)
        if rc != 0 and rc != 1007:  # (1007: ncclInProgress)
            self._check(rc, "RCCL asynchronous error")

    def close(self, abort=False):
        if getattr(self, "h", None):
            from . import watchdog
            watchdog.remove_comm(self.h)
            try:
                torch.cuda.synchronize(self.device)
            except RuntimeError:
                abort = True
            N.load().kfb_rccl_destroy(self.h, int(abort))
            _LIVE.discard(self.h)
            self.h = None
