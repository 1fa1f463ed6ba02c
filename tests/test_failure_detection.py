"""Failure detection of multi-rank runs (parallel/watchdog.py, csrc/watchdog.hip).

The reference's launcher fails the job fast when a peer exits
(tcb/slurm-2810438.out:133-137, "exit on error: <k> tasks failed"); our
kfb-run does the same for exits, and the per-rank watchdog turns a peer that
stalls (no exit, a collective that never completes) into a non-zero exit
with one JSON line {"status": "comm_error", ...} on rank 0's stdout.

* a 4-rank CPU rehearsal of bench.py (gloo) where rank 2 stalls before timed
  step 1: the job exits non-zero within the deadline plus the launcher's
  grace, and rank 0 printed the comm_error line naming its phase and step;
* the deadline path aborts every registered communicator (a test hook
  stands in for ncclCommAbort), in-process, without exiting;
* heartbeats keep a healthy run alive past many deadlines;
* torchrun (the driver's launcher) also ends with the JSON line.
"""

import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "1"
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR",
              "KFB_FORCE_PG", "KFB_BENCH_NO_SELF_LAUNCH"):
        env.pop(k, None)
    env.update(extra)
    return env


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_lines(stdout):
    out = []
    for ln in stdout.splitlines():
        if ln.startswith("{"):
            try:
                out.append(json.loads(ln))
            except ValueError:
                pass
    return out


_ARGS = ["--device", "cpu", "--dtype", "fp32", "--model", "trivial", "--batch_size", "2",
         "--steps", "4", "--warmup", "1"]


@pytest.mark.parametrize("torchrun", [False, True])
def test_stalled_rank_ends_job_with_comm_error(torchrun):
    deadline = 6.0
    env = _env(KFB_COMM_TIMEOUT_S=str(deadline), KFB_TEST_STALL="2:1")
    if torchrun:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               "--nproc-per-node", "4", "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), BENCH, "--gpus", "4"] + _ARGS
    else:
        cmd = [sys.executable, BENCH, "--gpus", "4", "--job_timeout", "600"] + _ARGS
    t0 = time.time()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    took = time.time() - t0
    assert r.returncode != 0, r.stdout[-2000:]
    lines = [j for j in _json_lines(r.stdout) if j.get("status") == "comm_error"]
    assert len(lines) == 1, (r.stdout[-3000:], r.stderr[-3000:])
    j = lines[0]
    assert j["rank"] == 0 and j["kind"] in ("deadline", "terminated")
    if j["kind"] == "deadline":
        # rank 0 blocked in the gradient all-reduce of the step rank 2 never ran
        # (the first steps, which autotune and record the tape, get 3x)
        assert j["phase"] == "step" and j["timeout_s"] in (deadline, 3 * deadline)
    # no throughput line: a failed job reports only the error
    assert not [x for x in _json_lines(r.stdout) if "metric" in x]
    # startup (imports, model build) plus the deadline plus the launcher's
    # grace; far below the job timeout
    assert took < 240, took


def test_deadline_aborts_registered_communicators():
    code = r"""
import json, time
from kf_benchmarks_amd.parallel import watchdog as W
seen = []
W.set_abort_hook(lambda h: seen.append(h) or 0)
assert W.start(0, timeout=0.4, poll_s=0.05, dry_run=True, handle_sigterm=False)
W.add_comm(0x1000); W.add_comm(0x2000); W.add_comm(0x3000)
W.remove_comm(0x2000)
for i in range(10):          # healthy heartbeats: no firing
    W.beat("step", i)
    time.sleep(0.1)
assert W.fired() is None
W.beat("barrier", 10)         # then the rank stalls in a barrier
time.sleep(1.0)
rec = W.fired()
print(json.dumps({"rec": rec, "aborted": sorted(seen), "aborts": W.aborts()}))
W.stop()
"""
    r = subprocess.run([sys.executable, "-c", code], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"rec"')][0])
    rec = out["rec"]
    assert rec["status"] == "comm_error" and rec["kind"] == "deadline"
    assert rec["phase"] == "barrier" and rec["step"] == 10 and rec["rank"] == 0
    assert out["aborted"] == [0x1000, 0x3000] and out["aborts"] == 2
    assert rec["communicators_aborted"] == 2


def test_sigterm_becomes_comm_error_line():
    """The launcher's SIGTERM (a peer failed) is answered with the JSON line
    and the watchdog's exit code, not a silent kill."""
    code = r"""
import os, signal, time
from kf_benchmarks_amd.parallel import watchdog as W
assert W.start(0, timeout=60, poll_s=0.05)
W.beat("step", 3)
os.kill(os.getpid(), signal.SIGTERM)
time.sleep(5)
print("not reached")
"""
    r = subprocess.run([sys.executable, "-c", code], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 3, (r.returncode, r.stdout, r.stderr[-2000:])
    j = _json_lines(r.stdout)[0]
    assert j["kind"] == "terminated" and j["step"] == 3 and "not reached" not in r.stdout


def test_disabled_by_zero_timeout():
    code = r"""
import os
os.environ["KFB_COMM_TIMEOUT_S"] = "0"
from kf_benchmarks_amd.parallel import watchdog as W
print("started" if W.start(0) else "off")
"""
    r = subprocess.run([sys.executable, "-c", code], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert r.stdout.strip().endswith("off"), r.stderr[-2000:]
