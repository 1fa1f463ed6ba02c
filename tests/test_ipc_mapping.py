"""Peer-slot mapping over HIP IPC (parallel/ipc.py), CPU side: which device
a rank opens a peer's handle on, and when peer access is enabled
explicitly - with per-rank device visibility (HIP_VISIBLE_DEVICES set) and
with the whole node visible.  The native calls are recorded, not run."""

import pytest

from kf_benchmarks_amd.parallel import ipc


def _view(device, count, visible=""):
    return {"device": device, "count": count, "visible": visible}


def test_visible_devices_env(monkeypatch):
    for v in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert ipc._visible_devices_env() == ""
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "3")
    assert ipc._visible_devices_env() == "HIP_VISIBLE_DEVICES=3"


@pytest.mark.parametrize("mine,theirs,want", [
    (_view(0, 8), _view(5, 8), 5),                       # whole node visible
    (_view(2, 8), _view(2, 8), None),                    # same GPU (shared-device rehearsal)
    (_view(0, 1, "HIP_VISIBLE_DEVICES=0"), _view(0, 1, "HIP_VISIBLE_DEVICES=1"), None),
    (_view(0, 8, "HIP_VISIBLE_DEVICES=0,1,2,3,4,5,6,7"), _view(3, 8, ""), None),  # views differ
    (_view(0, 4), _view(6, 8), None),                    # counts differ
])
def test_peer_access_target(mine, theirs, want):
    assert ipc.peer_access_target(mine, theirs) == want


class _Rec:
    def __init__(self):
        self.calls = []

    def __call__(self, name, *args):
        self.calls.append((name, args))
        if name == "kfb_ipc_open":
            args[2]._obj.value = 0x7000_0000_0000
        return 0


@pytest.mark.parametrize("visible", [None, "per_rank"])
def test_open_uses_own_device(monkeypatch, visible):
    """The importer always maps on ITS OWN device index (never the
    exporter's); peer access is enabled only with the whole node visible."""
    from kf_benchmarks_amd.ops import _native as N
    rec = _Rec()
    monkeypatch.setattr(N, "call", rec)
    if visible is None:
        mine, theirs = _view(3, 8), dict(_view(6, 8), handle=b"h" * 64, offset=256)
    else:
        mine = _view(0, 1, "HIP_VISIBLE_DEVICES=3")
        theirs = dict(_view(0, 1, "HIP_VISIBLE_DEVICES=6"), handle=b"h" * 64, offset=256)
    base = ipc.open_peer_slots(theirs, mine)
    assert base == 0x7000_0000_0000
    names = [c[0] for c in rec.calls]
    opened = [c for c in rec.calls if c[0] == "kfb_ipc_open"]
    assert len(opened) == 1 and opened[0][1][1] == mine["device"]
    if visible is None:
        assert ("kfb_enable_peer", (3, 6)) in rec.calls
    else:
        assert "kfb_enable_peer" not in names
