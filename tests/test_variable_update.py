"""Analytic-oracle tests of every --variable_update mode (the role of
tcb/benchmark_cnn_test.py:1236-1365 VariableUpdateTest and
tcb/benchmark_cnn_distributed_test.py DistributedVariableUpdateTest).

Single-process runs check the update rule; 2-rank gloo runs (one OS process
per rank, rendezvous on 127.0.0.1) check the cross-worker aggregation."""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import kfb_test_util as tu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("vu", ["parameter_server", "replicated", "independent", "horovod",
                                "collective_all_reduce", "distributed_replicated",
                                "distributed_all_reduce", "kungfu"])
def test_single_worker_updates(vu):
    params = tu.get_var_update_params(variable_update=vu)
    losses, _ = tu.run_test_model(params)
    expected = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), 1, params, "sum")[0]
    np.testing.assert_allclose(losses, expected, rtol=1e-5, atol=0)


@pytest.mark.parametrize("opt", ["sgd", "momentum"])
@pytest.mark.parametrize("loss_type", ["base_loss", "total_loss"])
def test_optimizer_and_loss_type(opt, loss_type):
    params = tu.get_var_update_params(optimizer=opt, loss_type_to_report=loss_type,
                                      num_batches=6)
    losses, _ = tu.run_test_model(params)
    expected = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), 1, params, "sum")[0]
    np.testing.assert_allclose(losses, expected, rtol=1e-5, atol=0)


def test_print_training_accuracy_columns():
    params = tu.get_var_update_params(print_training_accuracy=True)
    _, logs = tu.run_test_model(params)
    outs = tu.get_training_outputs_from_logs(logs, True)
    assert len(outs) == params.num_batches


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_workers(nworkers, flag_kwargs, tmp_path, timeout=240, extra_env=None):
    """Launch nworkers processes of tests/dist_worker.py; returns per-rank losses."""
    port = _free_port()
    procs = []
    for r in range(nworkers):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(nworkers), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1",
                   PYTHONPATH=ROOT + os.pathsep + os.path.join(ROOT, "tests"),
                   **(extra_env or {}))
        out = tmp_path / ("rank%d.json" % r)
        cmd = [sys.executable, os.path.join(ROOT, "tests", "dist_worker.py"), str(out),
               json.dumps(flag_kwargs)]
        procs.append((subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE,
                                       stderr=subprocess.STDOUT, text=True), out))
    results = []
    for p, out in procs:
        try:
            log, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q, _ in procs:
                q.kill()
            raise
        assert p.returncode == 0, log
        with open(out) as f:
            results.append(json.load(f))
    return results


@pytest.mark.parametrize("vu,kopt,agg", [("parameter_server", None, "sum"),
                                         ("replicated", None, "sum"),
                                         ("horovod", None, "sum"),
                                         ("independent", None, "none"),
                                         ("kungfu", "sync_sgd", "mean")])
def test_two_workers(vu, kopt, agg, tmp_path):
    kw = dict(variable_update=vu, num_batches=4)
    if kopt:
        kw["kungfu_option"] = kopt
    res = run_workers(2, kw, tmp_path)
    params = tu.get_var_update_params(**kw)
    expected = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), 2, params, agg)
    for r in range(2):
        np.testing.assert_allclose(res[r]["losses"], expected[r], rtol=1e-5, atol=0)


@pytest.mark.parametrize("n", [2, 4])
@pytest.mark.parametrize("opt", ["sgd", "momentum"])
def test_workers_sma_exact(n, opt, tmp_path):
    """kungfu sma (SynchronousAveragingOptimizer): every step each worker
    moves to (1 - alpha) w + alpha * mean_r(w_r), then applies its own
    gradient - deterministic, so every worker's reported loss matches the
    analytic oracle (tcb/benchmark_cnn_test.py:1236-1365 style)."""
    kw = dict(variable_update="kungfu", kungfu_option="sma", num_batches=6,
              kungfu_sma_alpha=0.3, optimizer=opt)
    res = run_workers(n, kw, tmp_path)
    params = tu.get_var_update_params(**kw)
    expected = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), n, params, "sma")
    for r in range(n):
        np.testing.assert_allclose(res[r]["losses"], expected[r], rtol=1e-5, atol=0)
    # the averaging is real: the oracle's workers differ from independent ones
    ind = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), n, params, "none")
    assert any(abs(a - b) > 1e-3 for a, b in zip(expected[1][1:], ind[1][1:]))


@pytest.mark.parametrize("n", [2, 4])
def test_workers_ada_sgd_exact(n, tmp_path):
    """kungfu ada_sgd: SMA for the first kungfu_ada_switch_step steps, then
    synchronous SGD (mean gradient) on each worker's own weights."""
    kw = dict(variable_update="kungfu", kungfu_option="ada_sgd", num_batches=7,
              kungfu_sma_alpha=0.5, kungfu_ada_switch_step=3)
    res = run_workers(n, kw, tmp_path)
    params = tu.get_var_update_params(**kw)
    expected = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), n, params, "ada_sgd")
    for r in range(n):
        np.testing.assert_allclose(res[r]["losses"], expected[r], rtol=1e-5, atol=0)
    # the switch matters: pure SMA and pure S-SGD both differ from it
    for other in ("sma", "mean"):
        o = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), n, params, other)
        assert any(abs(a - b) > 1e-6 for a, b in zip(expected[0], o[0])), other


@pytest.mark.parametrize("n,seed", [(2, 0), (4, 0), (4, 5)])
def test_workers_pair_averaging_exact(n, seed, tmp_path):
    """kungfu async_sgd (PairAveragingOptimizer) in its lock-step mode (pull
    at update time; all pulls before any publish; each publish committed
    before the next step): worker r averages with the step-t model of the
    peer its own RNG drew, w <- (w + w_peer) / 2, then applies its own
    gradient - the oracle replays the same peer draws."""
    kw = dict(variable_update="kungfu", kungfu_option="async_sgd", num_batches=6,
              kungfu_pair_lockstep=True, kungfu_peer_seed=seed)
    res = run_workers(n, kw, tmp_path)
    params = tu.get_var_update_params(**kw)
    expected = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), n, params, "pair")
    for r in range(n):
        np.testing.assert_allclose(res[r]["losses"], expected[r], rtol=1e-5, atol=0)


def test_two_workers_async_pair_averaging(tmp_path):
    """kungfu async_sgd (PairAveraging), the default asynchronous mode: every
    worker trains and publishes without a global barrier per step; models
    stay finite and every step's loss lies between the independent and the
    fully averaged (S-SGD) oracles' ranges."""
    res = run_workers(2, dict(variable_update="kungfu", kungfu_option="async_sgd",
                              num_batches=6), tmp_path)
    for r in res:
        assert len(r["losses"]) == 6
        assert all(np.isfinite(r["losses"]))


def test_two_workers_async_parameter_server(tmp_path):
    """--variable_update=parameter_server --cross_replica_sync=False: each
    worker applies its own (possibly stale) gradient to the shared model under
    the PS lock; every apply is counted in the shared global step that times
    the run (GlobalStepWatcher), and the first step of each worker sees the
    initial model."""
    kw = dict(variable_update="parameter_server", cross_replica_sync=False, num_batches=6,
              loss_type_to_report="base_loss")
    res = run_workers(2, kw, tmp_path)
    params = tu.get_var_update_params(**kw)
    expected = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), 2, params, "none")
    for r in range(2):
        assert len(res[r]["losses"]) == 6
        np.testing.assert_allclose(res[r]["losses"][0], expected[r][0], rtol=1e-6)
        assert res[r]["stats"]["ps_global_step"] >= 6
    assert max(r["stats"]["ps_global_step"] for r in res) == 12
    # the workers trained one shared model, not two independent ones
    ind = run_workers(2, dict(variable_update="independent", num_batches=6), tmp_path)
    assert res[0]["vars"] != ind[0]["vars"]


def _tower_oracle(inputs, ntowers, params, mean):
    """One worker with ``ntowers`` towers (tower t reads the data rolled by
    t/ntowers): tower gradients averaged (parameter_server) or summed
    (replicated), L2 counted once per tower sum as the reference's
    last-tower x num_devices term; reported loss = mean tower loss."""
    bs = params.batch_size
    x = inputs.astype(np.float64) / 127.5 - 1.0
    nb = x.shape[0] // bs
    from kf_benchmarks_amd import cnn_util
    data = [cnn_util.roll_numpy_batches(x, bs, t / float(ntowers)).reshape(nb, bs)
            for t in range(ntowers)]
    a, b = tu.TestCNNModel.VAR_A_INITIAL_VALUE, tu.TestCNNModel.VAR_B_INITIAL_VALUE
    wd, lr = params.weight_decay, params.init_learning_rate
    losses = []
    for step in range(params.num_batches):
        ms = [data[t][step % nb].mean() for t in range(ntowers)]
        losses.append(float(np.mean([m * a * b for m in ms])))
        ga = sum(m * b for m in ms)
        gb = sum(m * a for m in ms)
        if mean:
            ga, gb = ga / ntowers + wd * a, gb / ntowers + wd * b
        else:
            ga, gb = ga + ntowers * wd * a, gb + ntowers * wd * b
        a, b = a - lr * ga, b - lr * gb
    return losses


@pytest.mark.parametrize("vu,mean", [("parameter_server", True), ("replicated", False)])
def test_two_towers_one_worker(vu, mean, tmp_path):
    """--num_gpus=2 in one command runs as 2 tower processes (KFB_TOWER_GROUP)
    reporting as one worker."""
    kw = dict(variable_update=vu, num_batches=4, num_gpus=2, loss_type_to_report="base_loss")
    res = run_workers(2, kw, tmp_path, extra_env={"KFB_TOWER_GROUP": "1"})
    params = tu.get_var_update_params(**kw)
    expected = _tower_oracle(tu.get_fake_var_update_inputs(), 2, params, mean)
    np.testing.assert_allclose(res[0]["losses"], expected, rtol=1e-5, atol=0)


@pytest.mark.parametrize("extra", [dict(gradient_repacking=3, compact_gradient_transfer=False),
                                   dict(gradient_repacking=3),  # fp16 on the wire
                                   dict(all_reduce_spec="xring#2"), dict(bucket_size_mb=1e-6)])
def test_two_workers_bucket_options_match_sum(extra, tmp_path):
    """Repacking into k buckets, sharded collectives and one-tensor buckets
    reduce exactly like the default plan."""
    kw = dict(variable_update="replicated", num_batches=4, **extra)
    res = run_workers(2, kw, tmp_path)
    params = tu.get_var_update_params(**kw)
    expected = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), 2, params, "sum")
    compact = params.gradient_repacking and params.compact_gradient_transfer
    for r in range(2):
        np.testing.assert_allclose(res[r]["losses"], expected[r], rtol=1e-3 if compact else 1e-5,
                                   atol=0)


def test_two_workers_relaxed_consistency(tmp_path):
    """--variable_consistency=relaxed applies the previous step's reduced
    gradients (nothing at the first step)."""
    kw = dict(variable_update="replicated", num_batches=5, variable_consistency="relaxed",
              loss_type_to_report="base_loss")
    res = run_workers(2, kw, tmp_path)
    params = tu.get_var_update_params(**kw)
    from kf_benchmarks_amd import cnn_util
    x = tu.get_fake_var_update_inputs().astype(np.float64) / 127.5 - 1.0
    bs = params.batch_size
    data = [cnn_util.roll_numpy_batches(x, bs, w / 2.0).reshape(-1, bs) for w in range(2)]
    a, b = tu.TestCNNModel.VAR_A_INITIAL_VALUE, tu.TestCNNModel.VAR_B_INITIAL_VALUE
    wd, lr = params.weight_decay, params.init_learning_rate
    prev = None
    exp = [[], []]
    for step in range(params.num_batches):
        ms = [data[w][step % data[w].shape[0]].mean() for w in range(2)]
        for w in range(2):
            exp[w].append(ms[w] * a * b)
        cur = (sum(m * b for m in ms), sum(m * a for m in ms))
        if prev is not None:
            a, b = a - lr * (prev[0] + 2 * wd * a), b - lr * (prev[1] + 2 * wd * b)
        prev = cur
    for r in range(2):
        np.testing.assert_allclose(res[r]["losses"], exp[r], rtol=1e-5, atol=0)


def _hammer(tmp_path, device, numel, seconds, pace_us=0):
    import json
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONPATH=root)
        out = tmp_path / ("hammer%d.json" % r)
        procs.append((subprocess.Popen(
            [sys.executable, os.path.join(root, "tests", "pairavg_hammer.py"), str(out),
             device, str(numel), str(seconds), str(pace_us)], env=env, stdout=subprocess.PIPE,
            stderr=subprocess.STDOUT, text=True), out))
    res = []
    for p, out in procs:
        log, _ = p.communicate(timeout=240)
        assert p.returncode == 0, log[-3000:]
        with open(out) as f:
            res.append(json.load(f))
    return res


def test_pair_averaging_store_never_tears(tmp_path):
    """The seqlock model store under a publisher hammering constant-valued
    snapshots: every snapshot a reader accepts is uniform."""
    pub, rd = _hammer(tmp_path, "cpu", 4 << 20, 3.0)
    # (counts vary with machine load; the property is that no accepted
    # snapshot tears)
    assert pub["publishes"] > 3 and rd["pulls"] > 3
    assert rd["torn"] == 0, rd
    assert rd["distinct"] > 2  # the reader saw the publisher advancing


@pytest.mark.parametrize("opt", ["sgd", "momentum"])
def test_staged_vars_parameter_server(opt):
    """--staged_vars (PS mode): step t's loss and gradients use the variables
    as read one update earlier, checked against the analytic oracle
    (tcb/benchmark_cnn_test.py:197 _testVariables('parameter_server',
    staged_vars=True))."""
    params = tu.get_var_update_params(variable_update="parameter_server", staged_vars=True,
                                      optimizer=opt, num_batches=6)
    losses, _ = tu.run_test_model(params)
    expected = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), 1, params, "sum",
                                          staged=True)[0]
    np.testing.assert_allclose(losses, expected, rtol=1e-5, atol=0)
    plain = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), 1, params, "sum")[0]
    assert not np.allclose(plain, expected)  # staging changes the trajectory


@pytest.mark.parametrize("spec", ["psgpu#2", "pscpu/pscpu", "nccl/xring:64:psgpu"])
def test_two_workers_all_reduce_specs(spec, tmp_path):
    """--all_reduce_spec algorithms as process-level collectives (RCCL on the
    GPU, gloo here): parameter-server reduce+broadcast with rotating roots,
    sharded pieces, size-ranged choice; same sums as the plain all-reduce."""
    kw = dict(variable_update="replicated", num_batches=4, all_reduce_spec=spec)
    res = run_workers(2, kw, tmp_path)
    params = tu.get_var_update_params(**kw)
    expected = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), 2, params, "sum")
    for r in range(2):
        np.testing.assert_allclose(res[r]["losses"], expected[r], rtol=1e-5, atol=0)


def test_hierarchical_copy_eight_workers(tmp_path):
    """--hierarchical_copy with the DGX-1 topology over 8 ranks: reduce inside
    {0-3} / {4-7}, all-reduce between the two leaders, broadcast back
    (tcb/batch_allreduce.py:173-267); same sums as the flat all-reduce."""
    kw = dict(variable_update="replicated", num_batches=3, hierarchical_copy=True,
              network_topology="dgx1", bucket_size_mb=1e-5)
    res = run_workers(8, kw, tmp_path)
    params = tu.get_var_update_params(**kw)
    expected = tu.manually_compute_losses(tu.get_fake_var_update_inputs(), 8, params, "sum")
    for r in range(8):
        np.testing.assert_allclose(res[r]["losses"], expected[r], rtol=1e-5, atol=0)


def test_strategy_tape_hooks():
    """Launch-tape hooks of the KungFu strategies (the GPU tests replay
    them): ada_sgd's three launch sequences re-record the tape at the
    switch; the averaging strategies accept taping, per-step collectives
    are declared."""
    from kf_benchmarks_amd.parallel import variable_mgr as vm
    from kf_benchmarks_amd.parallel.kungfu import PairAveraging
    ada = vm.KungFuAdaSGD.__new__(vm.KungFuAdaSGD)
    ada.switch_step = 4
    phases = [ada.tape_phase(s) for s in range(7)]
    assert phases == [(True, True)] * 3 + [(True, False)] + [(False, False)] * 3
    assert ada.steps_use_collectives() and vm.KungFuSMA.steps_use_collectives(None)
    assert not PairAveraging.steps_use_collectives(None)
    assert vm.IndependentStrategy.tape_blocker(None) is None
