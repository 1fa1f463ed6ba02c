"""Failure detection of a multi-process job (csrc/watchdog.hip).

One native thread per rank watches a heartbeat and the rank's RCCL
communicators.  The step loops beat it (:func:`beat`) before every step and
every host wait (barrier, final synchronize, replica-consistency gather);
when a beat's allowance runs out, an RCCL asynchronous error appears, or the
launcher sends SIGTERM (a peer failed), the thread aborts the communicators
(ncclCommAbort), writes one JSON line ``{"status": "comm_error", "rank",
"step", "phase", ...}`` (rank 0 on stdout) and exits the process non-zero.

The reference's equivalent is its launcher's fail-fast (kungfu-run stops the
job when a peer exits, tcb/slurm-2810438.out:133-137) plus TF's collective
timeouts; torch's ProcessGroupNCCL watchdog does not watch our native
communicator, so this replaces it.  SURVEY section 5 (failure detection).

Knobs: ``KFB_COMM_TIMEOUT_S`` (default 300; 0 disables the watchdog) is the
allowance of a step / host wait; startup-like phases get
``STARTUP_FACTOR`` times that.
"""

from __future__ import annotations

import ctypes
import json
import os
from typing import Optional

from ..ops import _native as N

N.register_optional("kfb_watchdog_start", [N.I, ctypes.c_double, ctypes.c_double, N.I, N.I, N.I])
N.register_optional("kfb_watchdog_beat", [ctypes.c_char_p, ctypes.c_long, ctypes.c_double])
N.register_optional("kfb_watchdog_pause", [])
N.register_optional("kfb_watchdog_add_comm", [N.P])
N.register_optional("kfb_watchdog_remove_comm", [N.P])
N.register_optional("kfb_watchdog_set_abort_hook", [N.P])
N.register_optional("kfb_watchdog_fired", [N.P, N.I])
N.register_optional("kfb_watchdog_aborts", [])
N.register_optional("kfb_watchdog_stop", [])

STARTUP_FACTOR = 3.0  # warmup / recording phases (autotune, tape recording)
EXIT_CODE = 3

_STATE = {"running": False, "timeout": 0.0, "rank": 0}


def timeout_s() -> float:
    """KFB_COMM_TIMEOUT_S (seconds; 0 or negative disables the watchdog)."""
    try:
        return float(os.environ.get("KFB_COMM_TIMEOUT_S", "300"))
    except ValueError:
        return 300.0


def _lib():
    try:
        lib = N.load()
    except (OSError, N.NativeError):
        return None
    return lib if hasattr(lib, "kfb_watchdog_start") else None


def running() -> bool:
    return _STATE["running"]


def start(rank: int, timeout: Optional[float] = None, poll_s: float = 0.25,
          dry_run: bool = False, handle_sigterm: bool = True) -> bool:
    """Starts this rank's watchdog (idempotent).  Returns False when disabled
    (timeout <= 0) or the native library lacks it."""
    t = timeout_s() if timeout is None else float(timeout)
    if t <= 0:
        return False
    lib = _lib()
    if lib is None:
        return False
    lib.kfb_watchdog_start(int(rank), t, float(poll_s), EXIT_CODE, int(dry_run),
                           int(handle_sigterm))
    if not _STATE.get("atexit"):
        import atexit
        atexit.register(stop)  # a finished process is not a hung one
        _STATE["atexit"] = True
    _STATE.update(running=True, timeout=t, rank=int(rank))
    return True


def beat(phase: str, step: int = -1, timeout: Optional[float] = None, startup: bool = False):
    """The rank entered ``phase`` (of ``step``); it must beat again within
    ``timeout`` seconds (default: the watchdog's; x STARTUP_FACTOR for
    startup-like phases)."""
    if not _STATE["running"]:
        return
    t = float(timeout) if timeout is not None else _STATE["timeout"]
    if startup:
        t *= STARTUP_FACTOR
    N.load().kfb_watchdog_beat(phase.encode(), int(step), t)


def pause():
    if _STATE["running"]:
        N.load().kfb_watchdog_pause()


def add_comm(handle: int):
    """Registers an RCCL communicator: polled for asynchronous errors and
    aborted when the watchdog fires."""
    lib = _lib()
    if lib is not None and handle:
        lib.kfb_watchdog_add_comm(handle)


def remove_comm(handle: int):
    lib = _lib()
    if lib is not None and handle:
        lib.kfb_watchdog_remove_comm(handle)


def fired() -> Optional[dict]:
    """The firing record (dry-run mode / after the fact), else None."""
    lib = _lib()
    if lib is None:
        return None
    buf = ctypes.create_string_buffer(4096)
    if not lib.kfb_watchdog_fired(buf, len(buf)):
        return None
    txt = buf.value.decode(errors="replace").strip()
    try:
        return json.loads(txt) if txt else {"status": "comm_error"}
    except ValueError:
        return {"status": "comm_error", "raw": txt}


def aborts() -> int:
    lib = _lib()
    return int(lib.kfb_watchdog_aborts()) if lib is not None else 0


_HOOK_KEEP = []


def set_abort_hook(fn):
    """Test hook: ``fn(comm_handle) -> int`` replaces ncclCommAbort (None
    restores it)."""
    lib = _lib()
    if lib is None:
        return
    if fn is None:
        lib.kfb_watchdog_set_abort_hook(None)
        _HOOK_KEEP.clear()
        return
    cb = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)(fn)
    _HOOK_KEEP.append(cb)
    lib.kfb_watchdog_set_abort_hook(ctypes.cast(cb, ctypes.c_void_p))


def stop():
    if not _STATE["running"]:
        return
    lib = _lib()
    if lib is not None:
        lib.kfb_watchdog_stop()
    _STATE["running"] = False
