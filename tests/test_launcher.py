"""kfb-run (the kungfu-run equivalent): env, prefixed output, per-peer logs,
fail-fast, and a 2-peer gloo training run through it."""

import os
import subprocess
import sys

import pytest

from kf_benchmarks_amd.parallel import launcher

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return env


def test_env_prefix_and_logs(tmp_path):
    code = ("import os,sys; print('rank', os.environ['RANK'], os.environ['WORLD_SIZE'], "
            "os.environ['LOCAL_RANK'], os.environ['MASTER_ADDR'], os.environ['KUNGFU_SELF_SPEC']);"
            "print('warn', file=sys.stderr)")
    r = launcher.run(3, [sys.executable, "-c", code], logdir=str(tmp_path), capture=True,
                     port_range="23000-23100", env=_env())
    assert r.returncode == 0, r.stderr
    for k in range(3):
        port = 23000 + k
        assert "127.0.0.1.%d" % port in r.stdout
        with open(tmp_path / ("127.0.0.1.%d.stdout.log" % port)) as f:
            line = f.read().split()
        assert line[:6] == ["rank", str(k), "3", str(k), "127.0.0.1", "127.0.0.1:%d" % port]
        with open(tmp_path / ("127.0.0.1.%d.stderr.log" % port)) as f:
            assert f.read().strip() == "warn"
    assert "all 3/3 local peers finished" in r.stdout


def test_fail_fast(tmp_path):
    code = ("import os,sys,time; r=int(os.environ['RANK']); "
            "time.sleep(0.2 if r == 1 else 60); sys.exit(3 if r == 1 else 0)")
    r = launcher.run(3, [sys.executable, "-c", code], logdir=str(tmp_path), capture=True,
                     port_range="23100-23200", env=_env(), timeout=120)
    assert r.returncode == 1
    assert "exited with error: exit status 3" in r.stderr
    assert "tasks failed" in r.stderr


def test_two_peer_kungfu_training(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "tf_cnn_benchmarks.py"), "--device=cpu",
           "--data_format=NHWC", "--model=trivial", "--batch_size=4", "--num_batches=3",
           "--num_warmup_batches=1", "--variable_update=kungfu", "--kungfu_option=sync_sgd"]
    r = launcher.run(2, cmd, logdir=str(tmp_path), quiet=True, capture=True,
                     port_range="23200-23300", env=_env(), timeout=300)
    assert r.returncode == 0, r.stderr
    for port in (23200, 23201):
        with open(tmp_path / ("127.0.0.1.%d.stdout.log" % port)) as f:
            assert "total images/sec" in f.read()


def test_num_gpus_runs_as_tower_processes(tmp_path):
    """One --num_gpus=2 command -> 2 tower ranks; the console shows one
    worker's output (tower 0) with the 2-device global batch."""
    code = ("import sys; from kf_benchmarks_amd import cli, params as P, flags;"
            "argv=sys.argv[1:]; p=P.make_params(**flags.parse_flags(argv));"
            "sys.exit(cli._launch_towers(p, argv))")
    args = ["--device=cpu", "--data_format=NHWC", "--model=trivial", "--batch_size=4",
            "--num_batches=3", "--num_warmup_batches=1", "--num_gpus=2",
            "--variable_update=replicated"]
    env = _env()
    env["KFB_TOWER_LOGDIR"] = str(tmp_path)
    r = subprocess.run([sys.executable, "-c", code] + args, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("total images/sec") == 1
    assert "8 global" in r.stdout and "[127.0.0.1" not in r.stdout
    assert len(list(tmp_path.glob("127.0.0.1.*.stdout.log"))) == 2


def test_all_reduce_benchmark_two_ranks(tmp_path):
    """tcb/all_reduce_benchmark_test.py: the last log line is
    'Average time per step: <float>' (here per rank, via kfb-run)."""
    import re
    cmd = [sys.executable, "-m", "kf_benchmarks_amd.all_reduce_benchmark", "--device=cpu",
           "--data_format=NHWC", "--model=lenet", "--variable_update=replicated",
           "--num_batches=3", "--num_warmup_batches=1", "--iters_per_step=2",
           "--gradient_repacking=2", "--compact_gradient_transfer=false"]
    r = launcher.run(2, cmd, logdir=str(tmp_path), quiet=True, capture=True,
                     port_range="23300-23400", env=_env(), timeout=300)
    assert r.returncode == 0, r.stderr
    for port in (23300, 23301):
        with open(tmp_path / ("127.0.0.1.%d.stdout.log" % port)) as f:
            lines = [ln for ln in f.read().splitlines() if ln.strip()]
        avg = [ln for ln in lines if ln.startswith("Average time per step")]
        assert avg and re.match(r"^Average time per step: [0-9.e-]+$", avg[-1])


def test_ps_worker_cluster_flags(tmp_path):
    """--job_name/--task_index/--worker_hosts/--ps_hosts (the reference's
    gRPC cluster) as a torch.distributed world; the ps task waits for the
    workers and exits cleanly."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    common = ["--device=cpu", "--data_format=NHWC", "--model=trivial", "--batch_size=4",
              "--num_batches=3", "--num_warmup_batches=1", "--variable_update=parameter_server",
              "--worker_hosts=127.0.0.1:%d,127.0.0.1:%d" % (port, port + 1),
              "--ps_hosts=127.0.0.1:%d" % (port + 2)]
    env = _env()
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    script = os.path.join(ROOT, "tf_cnn_benchmarks.py")
    procs = [subprocess.Popen([sys.executable, script, "--job_name=ps", "--task_index=0"] + common,
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True)]
    for t in range(2):
        procs.append(subprocess.Popen([sys.executable, script, "--job_name=worker",
                                       "--task_index=%d" % t] + common, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=240)
            outs.append(out)
            assert p.returncode == 0, out
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert "total images/sec" in outs[1] and "total images/sec" in outs[2]
    assert "Running ps 0" in outs[0]


def _bench_json(stdout):
    import json
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_bench_self_launches_n_ranks():
    """bench.py --gpus 2 without an external launcher starts 2 ranks itself
    (kfb-run) and reports the whole 2-rank job; the driver contract."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
           "--model", "trivial", "--batch_size", "4", "--steps", "2", "--warmup", "1",
           "--dtype", "fp32"]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = _bench_json(r.stdout)
    assert out["n_gpus"] == 2 and out["ranks"] == 2 and out["backend"] == "gloo"
    assert out["config"]["global_batch"] == 8 and out["config"]["parallelism"] == "dp2"


def test_bench_refuses_mismatched_world():
    """A launcher that started fewer ranks than --gpus is an error, never a
    1-rank number labelled as N GPUs."""
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    env["KFB_BENCH_NO_SELF_LAUNCH"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
           "--model", "trivial", "--batch_size", "2", "--steps", "1", "--warmup", "0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and not r.stdout.strip(), (r.stdout, r.stderr)


def test_bench_forced_one_rank_group():
    """KFB_FORCE_PG=1: a 1-rank process group is created, so the bucketed
    all-reduce and the broadcast run (gloo here; RCCL on the GPU box)."""
    env = _env()
    env["KFB_FORCE_PG"] = "1"
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--model",
           "trivial", "--batch_size", "2", "--steps", "2", "--warmup", "1", "--dtype", "fp32"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = _bench_json(r.stdout)
    assert out["ranks"] == 1 and out["backend"] == "gloo"


def test_openmpi_environment_gives_one_rank_per_process(tmp_path):
    """mpirun -np N exports OMPI_COMM_WORLD_{RANK,SIZE,LOCAL_RANK} only
    (tcb/run_hv.sh:15-18): the world is read from them (horovod mode)."""
    port = 23450
    code = ("from kf_benchmarks_amd.parallel import comm; import torch;"
            "w=comm.init_world('cpu'); t=torch.ones(1); comm.all_reduce(t);"
            "print('W', w.rank, w.size, w.local_rank, int(t.item()))")
    procs = []
    for r in range(2):
        env = _env()
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
            env.pop(k, None)
        env.update(OMPI_COMM_WORLD_RANK=str(r), OMPI_COMM_WORLD_SIZE="2",
                   OMPI_COMM_WORLD_LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, text=True,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    outs = [p.communicate(timeout=120) for p in procs]
    for r, (o, e) in enumerate(outs):
        assert procs[r].returncode == 0, e
        assert ("W %d 2 %d 2" % (r, r)) in o


@pytest.mark.parametrize("model,batch", [("trivial", 4), ("resnet50", 2)])
def test_bench_under_torchrun(model, batch):
    """The driver's multi-GPU invocation, verbatim apart from --device cpu:
    torch.distributed.run starts the ranks, bench.py joins them (no self
    launch) and rank 0 prints one JSON line for the whole job."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = _env()
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--device", "cpu", "--model", model, "--batch_size", str(batch), "--dtype", "fp32"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _bench_json(r.stdout)
    assert out["n_gpus"] == 2 and out["ranks"] == 2 and out["steps"] == 2
    assert out["config"]["global_batch"] == 2 * batch
    assert out["value"] > 0 and out["higher_is_better"] is True
