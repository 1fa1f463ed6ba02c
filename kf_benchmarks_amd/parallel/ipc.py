"""Device memory shared between the ranks of one node over HIP IPC.

Exporter: the IPC handle of the allocation holding a tensor plus the tensor's
byte offset inside it (torch's caching allocator hands out sub-ranges of
larger blocks).  Importer: the handle is opened on the importing rank's OWN
device (csrc/optim.hip kfb_ipc_open), so no process ever creates a context on
a peer's GPU, and peer access is enabled explicitly where both ranks see the
whole node.  Used by the KungFu PairAveraging model store (peer pulls over
xGMI, tcb/benchmark_cnn.py:1196-1198) and the asynchronous parameter server
(shared model on rank 0).
"""

from __future__ import annotations

import os

import torch


def _visible_devices_env():
    for name in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        v = os.environ.get(name)
        if v is not None:
            return "%s=%s" % (name, v)
    return ""


def export_view(device: torch.device) -> dict:
    """This rank's view of the node: its device index and device visibility."""
    return {"device": device.index, "visible": _visible_devices_env(),
            "count": torch.cuda.device_count()}


def export_slots(slots: torch.Tensor) -> dict:
    """What a peer needs to map ``slots``: the IPC handle of the allocation
    holding them, their byte offset in it, and this rank's view of the node
    (its device index and device visibility), for the peer-access choice."""
    import ctypes
    from ..ops import _native as N
    lib = N.load()
    hb = int(lib.kfb_ipc_handle_bytes())
    buf = ctypes.create_string_buffer(hb)
    off = ctypes.c_longlong()
    N.call("kfb_ipc_export", slots.data_ptr(), buf, ctypes.byref(off))
    return dict(export_view(slots.device), handle=bytes(buf.raw), offset=int(off.value))


def peer_access_target(mine: dict, theirs: dict):
    """The peer's device index as THIS process sees it, if peer access can be
    enabled explicitly: both ranks see the same set of several devices (a
    launcher that exposes the whole node).  None when each rank sees only its
    own GPU (the IPC mapping then enables peer access lazily by itself)."""
    if mine["visible"] != theirs["visible"] or mine["count"] != theirs["count"] \
            or mine["count"] < 2:
        return None
    if theirs["device"] == mine["device"] or not 0 <= theirs["device"] < mine["count"]:
        return None
    return theirs["device"]


def open_peer_slots(theirs: dict, mine: dict) -> int:
    """Maps a peer's slot allocation into THIS rank's device (its own
    ``device`` index; the calling thread's current device is kept) and
    returns the mapped base address."""
    import ctypes
    from ..ops import _native as N
    tgt = peer_access_target(mine, theirs)
    if tgt is not None:
        try:
            N.call("kfb_enable_peer", mine["device"], tgt)
        except N.NativeError:
            pass  # (the lazy peer access of the IPC mapping still applies)
    base = ctypes.c_void_p()
    N.call("kfb_ipc_open", theirs["handle"], mine["device"], ctypes.byref(base))
    return int(base.value)


_TYPESTR = {torch.float32: "<f4", torch.float16: "<f2", torch.int32: "<i4", torch.int64: "<i8"}


def wrap(addr: int, numel: int, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
    """A tensor over ``numel`` elements at device address ``addr`` (a mapped
    peer allocation; not owned: freed by :func:`close_mapping`)."""
    class _Arr:
        __cuda_array_interface__ = {
            "shape": (int(numel),), "typestr": _TYPESTR[dtype],
            "data": (int(addr), False), "version": 2}
    with torch.cuda.device(device):
        t = torch.as_tensor(_Arr(), device=device)
    if t.data_ptr() != int(addr) or t.device != torch.device(device):
        # a copy (or another device's tensor) would silently break the
        # sharing: writes must land in the peer's allocation
        raise RuntimeError("ipc.wrap: tensor at 0x%x on %s is not a view of the mapping at 0x%x "
                           "on %s" % (t.data_ptr(), t.device, int(addr), device))
    return t


def close_mapping(base: int):
    from ..ops import _native as N
    try:
        N.call("kfb_ipc_close", base)
    except N.NativeError:
        pass
