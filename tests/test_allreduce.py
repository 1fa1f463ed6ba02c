"""All-reduce spec grammar and the per-bucket algorithm choice
(tcb/allreduce.py:58-104; tcb/batch_allreduce.py).  The algorithms
themselves run as process-level collectives; multi-rank numerics are pinned
against the analytic oracle in tests/test_variable_update.py."""

import pytest

from kf_benchmarks_amd.parallel import allreduce


def test_parse_spec():
    assert allreduce.parse_general_int("32k") == 32768
    assert allreduce.parse_general_int("2M") == 2 << 20
    s = allreduce.parse_all_reduce_spec("psgpu#4:32k:xring")
    assert s == [allreduce.AllReduceSpecTuple("psgpu", 4, 32768),
                 allreduce.AllReduceSpecTuple("xring", 1, -1)]
    with pytest.raises(ValueError):
        allreduce.parse_all_reduce_spec("bogus")
    with pytest.raises(ValueError):
        allreduce.parse_all_reduce_spec("nccl:32k")
    with pytest.raises(ValueError):
        allreduce.parse_all_reduce_spec("nccl#x")
    assert allreduce.rccl_env_for_spec("xring#2") == {"NCCL_ALGO": "Ring",
                                                      "NCCL_MIN_NCHANNELS": "2"}
    assert allreduce.rccl_env_for_spec("nccl/rechd") == {"NCCL_ALGO": "Tree"}
    assert allreduce.rccl_env_for_spec(None) == {}


def test_algorithm_by_bucket_size():
    spec = allreduce.parse_all_reduce_spec("psgpu#4:32k:nccl/xring#2")
    assert allreduce.algorithm_for(spec, 1000) == ("psgpu", 4, 32768)
    assert allreduce.algorithm_for(spec, 32768) == ("psgpu", 4, 32768)
    assert allreduce.algorithm_for(spec, 32769) == ("nccl/xring", 2, -1)
    assert allreduce.algorithm_for(None, 5) == ("nccl", 1, -1)
    assert allreduce.is_parameter_server("pscpu/pscpu")
    assert not allreduce.is_parameter_server("nccl/xring")


class _Work:
    def __init__(self, calls, name):
        self.calls, self.name = calls, name

    def wait(self):
        self.calls.append(("wait", self.name))


class _FakeComm:
    def __init__(self):
        self.calls = []

    def all_reduce(self, buf, op="sum", async_op=False):
        self.calls.append(("all_reduce",))
        return _Work(self.calls, "a")

    def reduce(self, buf, dst=0, op="sum", async_op=False):
        self.calls.append(("reduce", dst))
        return _Work(self.calls, "r")

    def broadcast(self, buf, src=0, async_op=False):
        self.calls.append(("broadcast", src))
        return _Work(self.calls, "b")


def test_launch_collective_ps_root_rotates():
    """PS algorithms: reduce to the bucket's root, wait (ordering), then
    broadcast from it; the root rotates with the bucket index."""
    import torch
    buf = torch.zeros(4)
    c = _FakeComm()
    ws = allreduce.launch_collective(c, buf, "psgpu", 5, 4)
    assert [w.name for w in ws] == ["b"]
    assert c.calls == [("reduce", 1), ("wait", "r"), ("broadcast", 1)]
    c = _FakeComm()
    ws = allreduce.launch_collective(c, buf, "nccl/xring", 5, 4)
    assert [w.name for w in ws] == ["a"] and c.calls == [("all_reduce",)]
