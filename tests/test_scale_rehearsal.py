"""CPU rehearsals of the multi-GPU BASELINE configs through bench.py at 4 and
8 ranks (gloo stands in for RCCL; the rank/device plumbing, collective
sequence, bucket schedule and JSON contract are the ones the round-end
8-GPU driver run uses).

BASELINE.json configs rehearsed (reference: tcb/benchmark_cnn_distributed_test.py:261-414
for the multi-worker matrix this mirrors):
  #3  ResNet-50, --variable_update=kungfu --kungfu_option=sync_sgd
  #4  ResNet-152, --kungfu_option=async_sgd (PairAveraging)
  #5  VGG-16, gradients on the wire in fp16
plus the parameter-server (``pscpu``) and two-level (hierarchical) reductions
at 8 ranks.  Synchronous strategies must end with bit-identical weights on
every rank (``weights_in_sync``); every run must exit 0 on all ranks.
"""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "1"
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR",
              "KFB_FORCE_PG", "KFB_BENCH_NO_SELF_LAUNCH"):
        env.pop(k, None)
    return env


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout[-3000:]
    return json.loads(lines[0])


def _run(n, args, torchrun=False, timeout=900):
    common = ["--gpus", str(n), "--device", "cpu", "--dtype", "fp32", "--steps", "2",
              "--warmup", "1"] + args
    if torchrun:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), BENCH] + common
    else:
        cmd = [sys.executable, BENCH] + common
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    out = _json(r.stdout)
    assert out["n_gpus"] == n and out["ranks"] == n and out["backend"] == "gloo"
    assert out["steps"] == 2 and out["value"] > 0
    assert out["config"]["parallelism"] == "dp%d" % n
    return out


def _no_leftover_shm():
    return [f for f in os.listdir("/dev/shm") if f.startswith(("kfb_model_", "kfb_ver_"))]


@pytest.mark.parametrize("n,torchrun", [(8, False), (4, True)])
def test_config3_sync_sgd_resnet50(n, torchrun):
    out = _run(n, ["--model", "resnet50", "--batch_size", "1"], torchrun=torchrun)
    assert out["config"]["variable_update"] == "kungfu/sync_sgd"
    assert out["config"]["global_batch"] == n
    assert out["weights_in_sync"] is True
    c = out["comm"]
    assert c["buckets"] >= 4 and c["collectives_per_step"] == c["buckets"]
    loss = out["config"]["loss_last"]
    assert loss == loss and abs(loss) < 1e4


@pytest.mark.parametrize("n,torchrun", [(4, False), (8, True)])
def test_config4_pair_averaging_resnet152(n, torchrun):
    before = set(_no_leftover_shm())
    out = _run(n, ["--model", "resnet152", "--batch_size", "1", "--kungfu_option",
                   "async_sgd"], torchrun=torchrun)
    assert out["config"]["variable_update"] == "kungfu/async_sgd"
    loss = out["config"]["loss_last"]
    assert loss == loss and abs(loss) < 1e4
    # asynchronous model averaging: no gradient all-reduce at all
    assert out["comm"]["buckets"] == 0
    # the model store's shared-memory files are removed at shutdown
    assert set(_no_leftover_shm()) <= before


@pytest.mark.parametrize("n,torchrun", [(4, False), (8, True)])
def test_config5_vgg16_fp16_wire(n, torchrun):
    out = _run(n, ["--model", "vgg16", "--batch_size", "1", "--wire_dtype", "fp16"],
               torchrun=torchrun)
    assert out["comm"]["wire_dtype"] == "fp16"
    assert out["weights_in_sync"] is True


@pytest.mark.parametrize("spec,extra", [("pscpu", []), (None, ["--hierarchical_copy"])])
def test_ps_and_hierarchical_8_ranks(spec, extra):
    args = ["--model", "resnet50", "--batch_size", "1", "--variable_update", "replicated"]
    if spec:
        args += ["--all_reduce_spec", spec]
    out = _run(8, args + extra)
    assert out["weights_in_sync"] is True
    assert out["config"]["all_reduce_spec"] == spec


def test_sma_4_ranks_in_sync_after_averaging():
    """SMA (kungfu_option=sma) moves every replica toward the all-reduced
    model average each step; with identical initial weights the replicas
    differ only by their local gradients, so they drift apart far less than
    independently trained replicas on the same data (the exact update rule is
    pinned by tests/test_variable_update.py::test_workers_sma_exact)."""
    sma = _run(4, ["--model", "trivial", "--batch_size", "2", "--kungfu_option", "sma"])
    ind = _run(4, ["--model", "trivial", "--batch_size", "2", "--variable_update",
                   "independent"])
    assert sma["config"]["variable_update"] == "kungfu/sma"
    assert sma["weights_in_sync"] is False and ind["weights_in_sync"] is False
    assert 0.0 < sma["replica_spread"] < ind["replica_spread"], (sma["replica_spread"],
                                                                 ind["replica_spread"])
    loss = sma["config"]["loss_last"]
    assert loss == loss
