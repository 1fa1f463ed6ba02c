"""2-rank data-parallel rehearsal on the GPU: both ranks run the HIP-kernel
training step with the bucketed all-reduce (overlapped with backward) and
must end every step with bit-identical weights (S-SGD keeps replicas in
lock step) after starting from rank 0's broadcast model."""

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(kw, steps, tmp_path, n=2):
    port = _port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KFB_DIST_BACKEND="gloo",
                   KFB_TEST_GRAD_SEGS="1",
                   PYTHONPATH=ROOT)
        out = tmp_path / ("rank%d.json" % r)
        cmd = [sys.executable, os.path.join(ROOT, "tests", "dist_gpu_worker.py"), str(out),
               json.dumps(kw), str(steps)]
        procs.append((subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE,
                                       stderr=subprocess.STDOUT, text=True), out))
    res = []
    for p, out in procs:
        try:
            log, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q, _ in procs:
                q.kill()
            raise
        assert p.returncode == 0, log[-4000:]
        with open(out) as f:
            res.append(json.load(f))
    return res


@pytest.mark.parametrize("extra", [
    dict(variable_update="kungfu", kungfu_option="sync_sgd", bucket_size_mb=4.0),
    dict(variable_update="horovod", gradient_wire_dtype="bf16", bucket_size_mb=2.0),
    dict(variable_update="replicated", gradient_repacking=3),
], ids=["kungfu_ssgd", "horovod_bf16wire", "replicated_repack3"])
def test_two_ranks_stay_in_lock_step(cuda, tmp_path, extra):
    kw = dict(model="resnet50", batch_size=8, num_gpus=1, use_bf16=True, optimizer="momentum",
              data_format="NHWC", **extra)
    r0, r1 = _run(kw, 3, tmp_path)
    assert r0["size"] == r1["size"] == 2
    assert r0["w0"] == r1["w0"]  # broadcast initial model
    for step, (g0, g1) in enumerate(zip(r0["gsegs"], r1["gsegs"])):
        gd = [k for k in g0 if g0[k] != g1[k]]
        assert not gd, "step %d: reduced gradients differ in %d variables, e.g. %s" % (
            step, len(gd), [(k, g0[k], g1[k]) for k in gd[:4]])
    diff = [k for k in r0["segs"] if r0["segs"][k] != r1["segs"][k]]
    assert not diff, "replicas differ in %d of %d variables, e.g. %s" % (
        len(diff), len(r0["segs"]), diff[:8])
    assert r0["wsum"] == r1["wsum"] and r0["wabs"] == r1["wabs"]
    assert r0["head"] == r1["head"] and r0["tail"] == r1["tail"]
    assert r0["wsum"] != r0["w0"]  # the step changed the weights
    for l0, l1 in zip(r0["losses"], r1["losses"]):
        assert l0 == l0 and l1 == l1 and abs(l0) < 1e3


def test_two_ranks_async_parameter_server(cuda, tmp_path):
    """--cross_replica_sync=False: the shared model lives in rank 0's device
    memory (HIP IPC); every rank applies its gradients to it under the PS
    lock, and the shared global step counts every apply."""
    kw = dict(model="resnet50", batch_size=8, num_gpus=1, use_bf16=True, optimizer="momentum",
              data_format="NHWC", variable_update="parameter_server", cross_replica_sync=False)
    r0, r1 = _run(kw, 3, tmp_path)
    assert r0["ps_global_step"] == r1["ps_global_step"] == 6
    assert r0["w0"] == r1["w0"]
    for r in (r0, r1):
        assert r["wsum"] != r["w0"] and r["wsum"] == r["wsum"]
        assert all(l == l and abs(l) < 1e3 for l in r["losses"])
