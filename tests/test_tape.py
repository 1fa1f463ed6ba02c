"""The launch tape's C++ replay (csrc/tape.hip) on the host: recorded calls
of a probe entry point with every argument type the kernels use (int,
float, long, pointer, uint32; more than fit in registers), replayed with a
per-step patch, and an error return reported with its op index."""

import ctypes

import pytest

from kf_benchmarks_amd.ops import _native as N
from kf_benchmarks_amd.ops import tape


@pytest.fixture
def probe():
    lib = N.load()
    fn = lib.kfb_tape_probe
    fn.argtypes = [N.I, N.F, N.L, N.P, ctypes.c_uint32, N.I, N.F, N.L, N.I, N.I, N.F]
    fn.restype = N.I
    lib.kfb_tape_probe_sum.restype = ctypes.c_uint64
    return lib, fn


def _expected(a, b, c, d, e, f, g, h, i, j, k):
    return a + int(b * 4) + c + d + e + f + int(g * 4) + h + i + j + int(k * 4)


def test_record_and_replay_with_patches(probe):
    lib, fn = probe
    rec = tape.Recorder()
    args = [3, 1.5, 10, 1000, 7, 2, 0.25, 100, 4, 5, 2.0]
    out = rec.add("kfb_tape_probe", fn, [args[0], N.Dyn("lr", args[1])] + args[2:])
    assert out[1] == 1.5  # the recording call itself gets plain values
    assert rec.keys() == ["lr"] and len(rec) == 1
    s0 = lib.kfb_tape_probe_sum()
    rec.replay({"lr": 1.5})
    assert lib.kfb_tape_probe_sum() - s0 == _expected(*args)
    rec.replay({"lr": 3.0})
    assert lib.kfb_tape_probe_sum() - s0 == _expected(*args) + _expected(*([3, 3.0] + args[2:]))
    with pytest.raises(tape.TapeError):
        rec.replay({})  # a per-step argument without a value
    rec.close()


def test_replay_reports_failing_op(probe):
    lib, fn = probe
    rec = tape.Recorder()
    rec.add("kfb_tape_probe", fn, [1, 0.0, 0, None, 0, 0, 0.0, 0, 0, 0, 0.0])
    rec.add("kfb_tape_probe", fn, [N.Dyn("a", 1), 0.0, 0, None, 0, 0, 0.0, 0, 0, 0, 0.0])
    rec.replay({"a": 2})
    with pytest.raises(tape.TapeError, match="op 1"):
        rec.replay({"a": -7})  # the probe returns 5 for a == -7
    rec.close()


def test_dyn_is_plain_value_when_not_recording():
    assert N.dyn("lr", 0.5) == 0.5 and not N.recording()
