"""Diagnosis (run after tests/test_tape_gpu.py::test_nasnet_tape_bitwise_matches_eager):
MobileNet-v2 gradients, ReLU6 in the BN vs a separate pass, repeated; prints
the worst per-tensor relative differences of each pair."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import relu6_diag as D  # noqa: E402  (its module body only defines helpers when imported)


@pytest.fixture
def cuda():
    return torch.device("cuda", 0)


@pytest.mark.gpu
def test_relu6_probe(cuda, monkeypatch):
    from kf_benchmarks_amd.ops import nn as nn_ops
    from kf_benchmarks_amd.ops import conv_hip
    if os.environ.get("PROBE_RESET_ARENA") == "1":
        conv_hip.STATS_ARENA.buf.clear()  # hypothesis: a buffer left in a dropped tape pool
        print("arena dropped", flush=True)
    f1 = D.run()
    f2 = D.run()
    monkeypatch.setattr(nn_ops, "_RELU6_IN_BN", False)
    u1 = D.run()
    u2 = D.run()
    D.cmp("fused vs fused", f1, f2)
    D.cmp("unfused vs unfused", u1, u2)
    D.cmp("fused vs unfused", f1, u1)
    D.cmp("fused2 vs unfused2", f2, u2)
