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


def _run(kw, steps, tmp_path, n=2, env_extra=None, tag=""):
    port = _port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KFB_DIST_BACKEND="gloo",
                   KFB_TEST_GRAD_SEGS="1",
                   PYTHONPATH=ROOT)
        env.update(env_extra or {})
        for k in [k for k, v in env.items() if v is None]:
            del env[k]
        out = tmp_path / ("%srank%d.json" % (tag, r))
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
    # rank 1's applies landed in rank 0's shared model: both ranks read the
    # same bytes (ipc.wrap raises if the mapping came back as a copy)
    assert r0["ps_shared_sum"] == r1["ps_shared_sum"]
    assert all(s == s for s in r0["ps_shared_sum"])
    for r in (r0, r1):
        assert r["wsum"] != r["w0"] and r["wsum"] == r["wsum"]
        assert all(l == l and abs(l) < 1e3 for l in r["losses"])


# RCCL proper: a 1-rank "nccl" process group (KFB_FORCE_PG=1).  RCCL refuses
# two ranks on one device, so on the 1-GPU box the real communicator runs at
# size 1: same bucket hooks, same async all-reduce issued from the weight-
# gradient side stream, same broadcast; the result must match the run without any group.
_RCCL = dict(KFB_FORCE_PG="1", KFB_DIST_BACKEND=None, WORLD_SIZE=None, RANK=None,
             LOCAL_RANK=None)
_NOCOMM = dict(KFB_DIST_BACKEND=None, WORLD_SIZE=None, RANK=None, LOCAL_RANK=None)


@pytest.mark.parametrize("native", ["1", "0"], ids=["native_comm", "torch_pg"])
def test_one_rank_rccl_is_identity(cuda, tmp_path, native):
    """FC-only model through a real 1-rank RCCL communicator - ours
    (csrc/comm.hip) or torch's ProcessGroupNCCL: every bucket launches every
    step, a synchronous all-reduce of the gradient returns it bit for bit,
    and training tracks the run without any process group."""
    kw = dict(model="trivial", batch_size=16, num_gpus=1, use_bf16=True, optimizer="momentum",
              data_format="NHWC", variable_update="kungfu", kungfu_option="sync_sgd",
              bucket_size_mb=8.0)
    env = dict(_RCCL, KFB_TEST_REDUCE_IDENTITY="1", KFB_NATIVE_COMM=native, KFB_TEST_HIER="1")
    (a,) = _run(kw, 3, tmp_path, n=1, env_extra=env, tag="rccl")
    (b,) = _run(kw, 3, tmp_path, n=1, env_extra=_NOCOMM, tag="nocomm")
    assert a["backend"] == ("rccl" if native == "1" else "nccl") and a["size"] == 1
    assert a["hier_identity"] is True
    # one RCCL communicator family: a native-communicator run (world and the
    # hierarchical subgroups) creates no ProcessGroupNCCL at all
    if native == "1":
        assert a["nccl_pgs"] == 0, a["nccl_pgs"]
    else:
        assert a["nccl_pgs"] >= 1
    # 3 steps + the identity check's synchronous reduction
    assert a["bucket_launches"] == 4 * a["num_buckets"] > 0
    assert b["bucket_launches"] == 0
    assert a["reduce_identity"] is True
    # (the first loss to fp32 rounding: the 150528-deep FC forward is a
    # split-K GEMM whose partial sums land in either order)
    assert a["w0"] == b["w0"]
    assert abs(a["losses"][0] - b["losses"][0]) <= 1e-6 * abs(b["losses"][0])
    for la, lb in zip(a["losses"], b["losses"]):
        assert abs(la - lb) <= 1e-4 * max(1.0, abs(lb)), (a["losses"], b["losses"])


@pytest.mark.parametrize("native,tape", [("1", False), ("0", False), ("1", True)],
                         ids=["native_comm", "torch_pg", "native_comm_taped"])
def test_one_rank_rccl_resnet50_overlap(cuda, tmp_path, native, tape):
    """ResNet-50 bs 8 through RCCL with backward-overlapped buckets and the
    side-stream weight gradients: every bucket launches every step, and the
    weights track the no-comm run (the BN statistics' fp32 atomics make
    either run non-bitwise at these shapes, so the bound is a tolerance).
    Taped: the bucket all-reduces are replayed from the launch tape with
    the kernels (2 eager steps, 1 recorded, the rest replayed)."""
    kw = dict(model="resnet50", batch_size=8, num_gpus=1, use_bf16=True, optimizer="momentum",
              data_format="NHWC", variable_update="kungfu", kungfu_option="sync_sgd",
              bucket_size_mb=4.0, launch_tape=tape)
    steps = 5 if tape else 3
    # (taped: no per-step gradient probe - its torch reads inside the step
    # would make the recording fall back to eager)
    env = dict(_RCCL, KFB_NATIVE_COMM=native, KFB_TAPE_STRICT="1" if tape else None)
    if tape:
        env["KFB_TEST_GRAD_SEGS"] = None
    (a,) = _run(kw, steps, tmp_path, n=1, env_extra=env, tag="rccl")
    (b,) = _run(dict(kw, launch_tape=False), steps, tmp_path, n=1, env_extra=_NOCOMM,
                tag="nocomm")
    assert a["backend"] == ("rccl" if native == "1" else "nccl")
    assert a["taped"] == (2 if tape else 0)
    launches = 3 * a["num_buckets"] if not tape else 3 * a["num_buckets"]  # eager+recorded
    assert a["num_buckets"] >= 4 and a["bucket_launches"] == launches
    # the exposed-communication probe: one interval per step, replayed
    # steps included (its marks are native calls inside the recorded step)
    import math
    assert len(a["exposed_ms"]) == steps, a["exposed_ms"]
    assert all(math.isfinite(x) and 0.0 <= x < 1000.0 for x in a["exposed_ms"]), a["exposed_ms"]
    assert a["w0"] == b["w0"]
    import math
    for k in a["segs"]:
        x, y = a["segs"][k], b["segs"][k]
        assert math.isfinite(x) and abs(x - y) <= 2e-3 * max(1.0, abs(y)), (k, x, y)
    for la, lb in zip(a["losses"], b["losses"]):
        assert abs(la - lb) <= 0.05 * max(1.0, abs(lb)), (a["losses"], b["losses"])


def test_pair_averaging_store_never_tears_over_hip_ipc(cuda, tmp_path):
    """KungFu async_sgd's model store on device memory shared over HIP IPC
    (both ranks on the box's one GPU): a publisher hammering constant-valued
    snapshots, a reader pulling on its side stream; every accepted snapshot
    is uniform."""
    from test_variable_update import _hammer
    pub, rd = _hammer(tmp_path, "cuda", 16 << 20, 4.0, pace_us=100)
    assert pub["publishes"] > 10 and rd["pulls"] > 10
    assert rd["torn"] == 0, rd
    assert rd["distinct"] > 2


def test_two_ranks_pair_averaging_training(cuda, tmp_path):
    """ResNet-50 bs 8 under --kungfu_option=async_sgd, two ranks on the GPU:
    prefetched peer pulls and event-committed publishes; both ranks train."""
    kw = dict(model="resnet50", batch_size=8, num_gpus=1, use_bf16=True, optimizer="momentum",
              data_format="NHWC", variable_update="kungfu", kungfu_option="async_sgd")
    r0, r1 = _run(kw, 4, tmp_path)
    assert r0["w0"] == r1["w0"]
    for r in (r0, r1):
        assert r["wsum"] != r["w0"] and r["wsum"] == r["wsum"]
        assert all(l == l and abs(l) < 1e3 for l in r["losses"])


@pytest.mark.parametrize("vu", ["replicated", "parameter_server"])
def test_tower_mode_taped_over_rccl(cuda, tmp_path, vu):
    """--num_gpus=N runs as N tower processes (KFB_TOWER_GROUP); the
    reported loss is the mean over the towers, a one-element all-reduce
    issued outside the recorded step, so tower mode tapes like any
    native-communicator run.  Here the single-tower stand-in
    over a real 1-rank RCCL group (KFB_FORCE_PG=1): taped and eager runs
    agree."""
    kw = dict(model="resnet50", batch_size=8, num_gpus=2, use_bf16=True, optimizer="momentum",
              data_format="NHWC", variable_update=vu, bucket_size_mb=4.0)
    env = dict(_RCCL, KFB_NATIVE_COMM="1", KFB_TOWER_GROUP="1", KFB_TEST_GRAD_SEGS=None)
    (a,) = _run(dict(kw, launch_tape=True), 6, tmp_path, n=1,
                env_extra=dict(env, KFB_TAPE_STRICT="1"), tag="taped")
    (b,) = _run(dict(kw, launch_tape=False), 6, tmp_path, n=1, env_extra=env, tag="eager")
    assert a["backend"] == "rccl" and a["tower_mode"] is True
    assert a["taped"] == 3, a["taped"]  # 2 eager, 1 recorded, 3 replayed
    assert a["w0"] == b["w0"]
    for la, lb in zip(a["losses"], b["losses"]):
        assert la == la and abs(la - lb) <= 0.05 * max(1.0, abs(lb)), (a["losses"], b["losses"])


def test_pair_averaging_torn_snapshot_skips_averaging(cuda, tmp_path):
    """PairAveraging's device-side torn-snapshot guard: rank 0's pull at
    step 3 sees a sequence word that moved during the copy (injected); the
    seqlock check kernel clears the flag, the fused update applies the plain
    gradient step without the averaging, and the rejection is counted.  The
    steps around it average normally (lock-step mode, 2 ranks, 1 GPU)."""
    kw = dict(model="trivial", batch_size=16, num_gpus=1, use_bf16=True, optimizer="sgd",
              data_format="NHWC", variable_update="kungfu", kungfu_option="async_sgd",
              kungfu_pair_lockstep=True)
    env = dict(KFB_TEST_TORN_STEP="3", KFB_TEST_GRAD_SEGS=None)
    r0, r1 = _run(kw, 5, tmp_path, env_extra=env)
    t = r0["torn_check"]
    assert t["ok_flag"] == 0 and t["peer_differs"], t
    assert t["err_nomix"] < 1e-6 < t["err_mix"], t
    assert r0["pa_torn"] == 1 and r1["pa_torn"] == 0
    assert r0["pa_publishes"] == r1["pa_publishes"] == 5


@pytest.mark.parametrize("option", ["sma", "ada_sgd"])
def test_one_rank_rccl_model_averaging_taped(cuda, tmp_path, option):
    """KungFu SMA / ada_sgd through the native 1-rank RCCL communicator from
    a launch tape: the model all-reduce (launched after each update, waited
    for by the next) is replayed with the step; ada_sgd re-records the tape
    when it switches phase (last averaging step, then S-SGD).  The taped run
    tracks the eager one."""
    kw = dict(model="resnet50", batch_size=8, num_gpus=1, use_bf16=True, optimizer="momentum",
              data_format="NHWC", variable_update="kungfu", kungfu_option=option,
              kungfu_sma_alpha=0.5, kungfu_ada_switch_step=4, bucket_size_mb=4.0)
    env = dict(_RCCL, KFB_NATIVE_COMM="1", KFB_TAPE_STRICT="1", KFB_TEST_GRAD_SEGS=None)
    (a,) = _run(dict(kw, launch_tape=True), 8, tmp_path, n=1, env_extra=env, tag="taped")
    (b,) = _run(dict(kw, launch_tape=False), 8, tmp_path, n=1, env_extra=env, tag="eager")
    assert a["backend"] == "rccl" and a["nccl_pgs"] == 0
    # sma: 2 eager, 1 recorded, 5 replayed; ada_sgd: recorded again at steps
    # 3 and 4 (phase changes), then 3 replays
    assert a["taped"] == (5 if option == "sma" else 3), a["taped"]
    assert a["w0"] == b["w0"]
    for la, lb in zip(a["losses"], b["losses"]):
        assert la == la and abs(la - lb) <= 0.05 * max(1.0, abs(lb)), (a["losses"], b["losses"])


def test_two_ranks_pair_averaging_taped(cuda, tmp_path):
    """KungFu async_sgd from a launch tape, two ranks on the GPU: the peer
    pull (device copy from the peer's IPC slot + device seqlock check) and
    the update into the publish slot are replayed with per-step peer-slot
    addresses, sequence words and publish slots; every step publishes."""
    kw = dict(model="resnet50", batch_size=8, num_gpus=1, use_bf16=True, optimizer="momentum",
              data_format="NHWC", variable_update="kungfu", kungfu_option="async_sgd",
              launch_tape=True)
    env = dict(KFB_TAPE_STRICT="1", KFB_TEST_GRAD_SEGS=None)
    r0, r1 = _run(kw, 6, tmp_path, env_extra=env)
    assert r0["w0"] == r1["w0"]
    for r in (r0, r1):
        assert r["taped"] == 3, r["taped"]
        assert r["pa_publishes"] == 6
        assert r["wsum"] != r["w0"] and r["wsum"] == r["wsum"]
        assert all(l == l and abs(l) < 1e3 for l in r["losses"])


@pytest.mark.parametrize("inject", [False, True], ids=["selftest_passes", "selftest_fails"])
def test_bench_native_selftest_and_fallback(cuda, inject):
    """bench.py through a real 1-rank RCCL group (KFB_FORCE_PG=1) with the
    default KFB_NATIVE_COMM=auto: the native communicator's startup self-test
    (every bucket size, broadcast / sum / max, bitwise against the gloo
    group) passes and the step is taped with its collectives; with a wrong
    sum injected into the check, the run falls back in-process to torch's
    ProcessGroupNCCL and stays eager - the JSON says which path ran."""
    env = dict(os.environ, PYTHONPATH=ROOT, KFB_FORCE_PG="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "KFB_DIST_BACKEND", "KFB_NATIVE_COMM"):
        env.pop(k, None)
    if inject:
        env["KFB_SELFTEST_INJECT"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "4",
           "--batch_size", "32"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    st = out["comm"]["selftest"]
    assert st is not None and st["checked"] > 0 and st["mode"] == "auto"
    if inject:
        assert not st["ok"] and st["fallback"] and st["failed"]
        assert out["backend"] == "nccl" and out["config"]["launch_tape"] is False
        assert "torch.distributed" in out["config"]["launch_tape_off_reason"]
    else:
        assert st["ok"] and "fallback" not in st
        assert out["backend"] == "rccl" and out["config"]["launch_tape"] is True
    assert out["weights_in_sync"] is True and out["value"] > 0
    if not inject:
        # the exposed-communication probe runs inside the taped step
        c = out["comm"]
        assert c["exposed_allreduce_ms"] is not None and c["exposed_allreduce_ms"] >= 0
        assert c["collectives_per_step"] == c["buckets"] > 0
        assert c["native_comms_live"] == 1  # the world communicator


def test_bench_selftest_fallback_rebuilds_hierarchical(cuda):
    """--hierarchical_copy on the native communicator builds its subgroup
    communicators with the strategy; when the startup self-test fails (a
    wrong sum injected), the fallback rebuilds the strategy on torch groups,
    so NO native communicator is left (the subgroups used to keep
    reducing on native RCCL after the self-test declared it bad)."""
    env = dict(os.environ, PYTHONPATH=ROOT, KFB_FORCE_PG="1", KFB_SELFTEST_INJECT="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "KFB_DIST_BACKEND", "KFB_NATIVE_COMM"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "2",
           "--batch_size", "16", "--hierarchical_copy"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    st = out["comm"]["selftest"]
    assert not st["ok"] and st["fallback"] and st.get("rebuilt_strategy") is True
    # the subgroup was checked as well as the world
    assert any(f.startswith("hier:") for f in st["failed"]), st["failed"]
    assert out["backend"] == "nccl" and out["comm"]["native_comms_live"] == 0
    assert out["weights_in_sync"] is True and out["value"] > 0
