"""End-to-end engine tests on the CPU path (role of TfCnnBenchmarksTest in
tcb/benchmark_cnn_test.py:429-1233 and tcb/test_util.py:202-299):
train -> checkpoint -> resume -> eval, forward-only, eval during training,
checkpoint retention, tracing outputs, summaries and optimizers."""

import glob
import json
import os

import numpy as np
import pytest

import kfb_test_util as tu
from kf_benchmarks_amd import benchmark, datasets


def _bw_data(n=16, size=32):
    """Black images labelled 0, white images labelled 1 (the reference's
    black/white fixture, tcb/test_data/tfrecord_image_generator.py)."""
    imgs = np.zeros((n, size, size, 3), np.float32)
    labels = np.zeros((n,), np.int64)
    imgs[1::2] = 255.0
    labels[1::2] = 1
    return imgs, labels


def _params(train_dir=None, **kw):
    base = dict(model="trivial", data_name="cifar10", batch_size=4, num_batches=20,
                num_warmup_batches=0, display_every=5, device="cpu", data_format="NHWC",
                optimizer="sgd", init_learning_rate=0.005, weight_decay=0,
                print_training_accuracy=True, train_dir=train_dir)
    base.update(kw)
    return benchmark.make_params(**base)


def _run(params, data=None):
    data = data or _bw_data()
    with tu.capture_logs() as logs:
        b = benchmark.BenchmarkCNN(params)
        b.set_fake_data(*data)
        stats = b.run()
    return b, stats, logs


def test_train_resume_eval(tmp_path):
    d = str(tmp_path / "train")
    b, stats, logs = _run(_params(d))
    outs = tu.get_training_outputs_from_logs(logs, True)
    assert stats["num_steps"] == 20
    assert os.path.exists(os.path.join(d, "model.ckpt-20.index"))
    assert outs[-1].loss < outs[0].loss
    # resume: the global step is restored, only the remaining steps run
    b2, stats2, logs2 = _run(_params(d, num_batches=30))
    assert stats2["num_steps"] == 10
    assert b2.global_step == 30
    assert os.path.exists(os.path.join(d, "model.ckpt-30.index"))
    outs2 = tu.get_training_outputs_from_logs(logs2, True)
    assert outs2[-1].loss <= outs[0].loss
    # eval from the latest checkpoint
    _, ev_stats, ev_logs = _run(_params(d, eval=True, num_eval_batches=4))
    ev = tu.get_evaluation_outputs_from_logs(ev_logs)
    assert ev[-1].top_1_accuracy == pytest.approx(1.0)
    assert ev[-1].top_5_accuracy == pytest.approx(1.0)
    assert ev_stats["global_step"] == 30
    # moved train dir still loads (checkpoint state uses relative paths)
    moved = str(tmp_path / "moved")
    os.rename(d, moved)
    _, _, ev_logs2 = _run(_params(moved, eval=True, num_eval_batches=2))
    assert tu.get_evaluation_outputs_from_logs(ev_logs2)


def test_forward_only():
    _, stats, logs = _run(_params(forward_only=True, num_batches=4, print_training_accuracy=False))
    assert stats["num_steps"] == 4
    assert any("total images/sec" in l for l in logs)


def test_eval_during_training(tmp_path):
    _, stats, logs = _run(_params(eval_during_training_every_n_steps=10, num_eval_batches=2))
    assert len(tu.get_evaluation_outputs_from_logs(logs)) == 2


def test_stop_at_top_1_accuracy():
    _, stats, logs = _run(_params(eval_during_training_every_n_steps=5, num_eval_batches=2,
                                  stop_at_top_1_accuracy=0.5, num_batches=40,
                                  init_learning_rate=0.01))
    assert stats["num_steps"] < 40
    assert any("Stopping" in l for l in logs)


def test_save_model_steps_and_retention(tmp_path):
    d = str(tmp_path / "t")
    _run(_params(d, save_model_steps=2, max_ckpts_to_keep=3, num_batches=10))
    idx = sorted(glob.glob(os.path.join(d, "*.index")))
    assert len(idx) == 3
    assert os.path.basename(idx[-1]) == "model.ckpt-8.index" or \
        "model.ckpt-10.index" in [os.path.basename(i) for i in idx]


def test_trace_tfprof_graph_files(tmp_path):
    tr, tp, gf = (str(tmp_path / n) for n in ("trace.json", "tfprof.txt", "graph.txt"))
    _run(_params(num_warmup_batches=3, num_batches=12, trace_file=tr, tfprof_file=tp,
                 graph_file=gf))
    with open(tr) as f:
        trace = json.load(f)
    assert trace.get("traceEvents")
    assert os.path.getsize(tp) > 0 and os.path.getsize(gf) > 0


def test_summaries_written(tmp_path):
    from kf_benchmarks_amd.utils import summary as sm
    d = str(tmp_path / "s")
    _run(_params(d, summary_verbosity=3, save_summaries_steps=5, num_batches=10))
    ev = glob.glob(os.path.join(d, "events.out.tfevents.*"))
    assert ev
    tags = set()
    for _, vals in sm.read_events(ev[0]):
        tags.update(vals)
    assert {"learning_rate", "total_loss", "log_gradients"} <= tags


@pytest.mark.parametrize("opt", ["momentum", "rmsprop", "adam"])
def test_optimizers_train(opt):
    _, stats, logs = _run(_params(optimizer=opt, num_batches=10, init_learning_rate=0.001,
                                  gradient_clip=1.0))
    assert np.isfinite(stats["last_average_loss"])


def test_benchmark_logger(tmp_path):
    d = str(tmp_path / "bl")
    _run(_params(num_batches=5, benchmark_log_dir=d))
    with open(os.path.join(d, "metric.log")) as f:
        names = {json.loads(l)["name"] for l in f}
    assert "average_examples_per_sec" in names


def test_failed_update_releases_strategy(tmp_path):
    """An exception between before_update and after_update (optimizer,
    non-finite check) reaches the strategy's abort_update, and the async
    PS lock is released so the other workers do not block forever."""
    import fcntl
    from kf_benchmarks_amd.parallel import async_ps
    b = benchmark.BenchmarkCNN(_params(num_batches=2))
    b.set_fake_data(*_bw_data())
    b.build()
    calls = []
    b.strategy.abort_update = lambda step: calls.append(step)

    def boom(*a, **k):
        raise FloatingPointError("injected")
    b.optimizer.step = boom
    with pytest.raises(FloatingPointError):
        b.train_step()
    assert calls == [0]
    # the PS strategy's lock bookkeeping: abort releases a held lock
    st = async_ps._SharedState.__new__(async_ps._SharedState)
    st._lock_f = open(tmp_path / "ps.lock", "w")
    strat = async_ps.AsyncParameterServer.__new__(async_ps.AsyncParameterServer)
    strat.state = st
    st.lock()
    strat.abort_update(0)
    with open(tmp_path / "ps.lock", "w") as f2:
        fcntl.flock(f2, fcntl.LOCK_EX | fcntl.LOCK_NB)  # would raise if still held
        fcntl.flock(f2, fcntl.LOCK_UN)
    st._lock_f.close()


def test_synthetic_seed_streams_are_independent():
    """Synthetic batches: every (rank, step) gets its own mixed seed; a
    step's label seed (seed + 1) is never another step's or rank's image
    seed (it used to be the next step's, and ranks were 1000 steps apart)."""
    from kf_benchmarks_amd.data.input_pipeline import _mix32
    seeds = {(r, s): _mix32(1234, r, s) for r in range(8) for s in range(2000)}
    vals = list(seeds.values())
    assert len(set(vals)) == len(vals)
    assert all(v % 2 == 0 and 0 <= v < 2 ** 31 for v in vals)
    assert not (set(vals) & {v + 1 for v in vals})
