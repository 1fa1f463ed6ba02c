"""Native-communicator startup self-test and its fallback (parallel/comm.py
selftest_device_collectives / validate_native), on 2 and 4 gloo ranks with a
stand-in communicator: a correct one passes everywhere and is kept; one
rank's wrong sums fail the check on EVERY rank, which then drop it (the
torch-group fallback)."""

import json
import os
import subprocess
import sys

import pytest

from test_variable_update import _free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, kind, tmp_path, timeout=180):
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1",
                   PYTHONPATH=ROOT + os.pathsep + os.path.join(ROOT, "tests"))
        env.pop("KFB_NATIVE_COMM", None)
        out = tmp_path / ("r%d.json" % r)
        cmd = [sys.executable, os.path.join(ROOT, "tests", "selftest_worker.py"), str(out), kind]
        procs.append((subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE,
                                       stderr=subprocess.STDOUT, text=True), out))
    res = []
    for p, out in procs:
        try:
            log, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q, _ in procs:
                q.kill()
            raise
        assert p.returncode == 0, log
        with open(out) as f:
            res.append(json.load(f))
    return res


@pytest.mark.parametrize("n", [2, 4])
def test_selftest_passes_and_keeps_native(n, tmp_path):
    res = _run(n, "good", tmp_path)
    for r in res:
        # 3 sizes x 2 dtypes x (broadcast, sum, max, reduce)
        assert r["selftest"]["ok"] and r["selftest"]["checked"] == 3 * 2 * 4
        assert r["validate"]["ok"] and "fallback" not in r["validate"]
        assert r["native_after"] and not r["closed"]


@pytest.mark.parametrize("n", [2, 4])
def test_selftest_failure_on_one_rank_falls_back_everywhere(n, tmp_path):
    res = _run(n, "bad", tmp_path)
    for r in res:
        st = r["selftest"]
        assert not st["ok"]
        # rank 1's wrong sums are reported by every rank (one verdict)
        assert st["failed"] == ["sum n=4097 bfloat16", "sum n=4097 float32",
                                "sum n=65536 bfloat16", "sum n=65536 float32"]
        assert not r["validate"]["ok"] and r["validate"]["fallback"]
        assert not r["native_after"] and r["closed"]


def test_selftest_cost_bounded_on_vgg16_8_ranks(tmp_path):
    """VGG-16's 138 M parameters (BASELINE #5): every distinct bucket size is
    checked once, capped (64 MB on a GPU; 8 MB for these host stand-ins), on
    data each rank generates itself; the whole startup check on 8 gloo ranks
    stays within 10 s."""
    res = _run(8, "vgg16", tmp_path, timeout=300)
    for r in res:
        assert r["selftest"]["ok"], r["selftest"]
        assert max(r["sizes"]) > 100_000_000  # (the whole model is one size)
        assert r["seconds"] <= 10.0, r["seconds"]
