"""Test harness (role of tcb/test_util.py): log capture and parsing, the
analytic TestCNNModel (loss = mean(x * A * B)), a 1x1-image dataset and a
manual loss oracle for every gradient-aggregation mode."""

from __future__ import annotations

import collections
import contextlib
import math
import os
import sys

import numpy as np
import torch

from kf_benchmarks_amd import benchmark, cnn_util, datasets
from kf_benchmarks_amd.models import model as model_lib

TrainingOutput = collections.namedtuple("TrainingOutput",
                                        ["loss", "top_1_accuracy", "top_5_accuracy"])
EvalOutput = collections.namedtuple("EvalOutput", ["top_1_accuracy", "top_5_accuracy"])


@contextlib.contextmanager
def monkey_patch(obj, **kwargs):
    old = {k: getattr(obj, k) for k in kwargs}
    for k, v in kwargs.items():
        setattr(obj, k, v)
    try:
        yield
    finally:
        for k, v in old.items():
            setattr(obj, k, v)


def print_and_add_to_list(lst):
    def f(s):
        print(s)
        lst.append(s)
    return f


def capture_logs():
    """Context manager yielding a list that receives every log_fn line."""
    logs = []
    fn = print_and_add_to_list(logs)

    @contextlib.contextmanager
    def cm():
        import kf_benchmarks_amd.eval as ev
        with monkey_patch(benchmark, log_fn=fn), monkey_patch(cnn_util, log_fn=fn), \
                monkey_patch(ev, log_fn=fn):
            yield logs
    return cm()


def get_training_outputs_from_logs(logs, print_training_accuracy):
    outputs = []
    for log in logs:
        if "images/sec" in log and "+/-" in log:
            parts = log.split()
            if print_training_accuracy:
                assert len(parts) == 11, log
                t1, t5 = float(parts[9]), float(parts[10])
            else:
                assert len(parts) == 9, log
                t1 = t5 = -1
            outputs.append(TrainingOutput(float(parts[8]), t1, t5))
    assert len(outputs) >= 1
    return outputs


def get_evaluation_outputs_from_logs(logs):
    out = []
    for log in logs:
        if "Accuracy @ " in log:
            parts = log.split()
            assert len(parts) == 12, log
            out.append(EvalOutput(float(parts[4]), float(parts[9])))
    assert out
    return out


class TestCNNModel(model_lib.CNNModel):
    """1x1x1 images; two scalar variables A=1, B=2 (1x1 convs); loss = mean(x*A*B)."""

    VAR_A_INITIAL_VALUE = 1.0
    VAR_B_INITIAL_VALUE = 2.0

    def __init__(self, params=None):
        super().__init__("test_cnn_model", image_size=1, batch_size=1, learning_rate=1,
                         params=params)
        self.depth = 1

    def add_inference(self, cnn):
        assert tuple(cnn.top_layer.shape[1:]) == (1, 1, 1)
        cnn.conv(1, 1, 1, 1, 1, use_batch_norm=False, activation=None, bias=None,
                 kernel_initializer=self.VAR_A_INITIAL_VALUE)
        cnn.conv(1, 1, 1, 1, 1, use_batch_norm=False, activation=None, bias=None,
                 kernel_initializer=self.VAR_B_INITIAL_VALUE)
        cnn.reshape([-1, 1])

    def skip_final_affine_layer(self):
        return True

    def loss_function(self, inputs, build_network_result):
        return build_network_result.logits.float().mean()

    def accuracy_function(self, inputs, logits):
        s = logits.float().sum()
        return {"top_1_accuracy": s, "top_5_accuracy": s}


class TestDataSet(datasets.ImageDataset):
    def __init__(self, height=1, width=1, depth=1):
        super().__init__("test_dataset", height=height, width=width, depth=depth,
                         data_dir=None, queue_runner_required=True, num_classes=1)

    def num_examples_per_epoch(self, subset="train"):
        return 1


def get_fake_var_update_inputs():
    """16 images whose normalized values are -1, 0, 1, ..., 14."""
    return np.resize(127.5 * np.array(range(16)), (16, 1, 1, 1))


def manually_compute_losses(inputs, num_workers, params, aggregation, staged=False):
    """Simulates ``num_workers`` workers on the analytic model.

    aggregation: 'sum' (parameter_server/replicated/... all-reduce SUM),
    'mean' (kungfu sync_sgd), 'none' (independent), and KungFu's model
    averaging optimizers (the wrappers of
    tcb/benchmark_cnn.py:1196-1201):

    * 'sma' (SynchronousAveragingOptimizer): every worker moves to
      (1 - alpha) w + alpha * mean_r(w_r), then applies its own gradient;
    * 'ada_sgd': 'sma' until --kungfu_ada_switch_step, 'mean' afterwards;
    * 'pair' (PairAveragingOptimizer, lock-step): worker r averages with the
      step-t model of a peer drawn by its own RNG (seed
      kungfu_peer_seed * 7919 + r), w <- (w + w_peer) / 2, then applies its
      own gradient.

    In the averaging modes the gradient is of the loss the step's forward
    computed, so its L2 term uses the forward's (pre-average) weights.
    Returns losses[w][step] as reported with loss_type_to_report.
    ``staged``: --staged_vars, the loss and gradients of step t use the
    variables as they were before the previous update
    (tcb/variable_mgr_util.py:236-393).
    """
    import random
    bs = params.batch_size
    n_batches = inputs.shape[0] // bs
    x_all = inputs.astype(np.float64) / 127.5 - 1.0
    wd = params.weight_decay or 0.0
    lr = params.init_learning_rate
    mom = params.momentum
    workers = []
    for w in range(num_workers):
        shifted = cnn_util.roll_numpy_batches(x_all, bs, w / float(num_workers))
        workers.append(shifted.reshape(n_batches, bs))
    A = [TestCNNModel.VAR_A_INITIAL_VALUE] * num_workers
    B = [TestCNNModel.VAR_B_INITIAL_VALUE] * num_workers
    acc = [[0.0, 0.0] for _ in range(num_workers)]
    losses = [[] for _ in range(num_workers)]
    RA, RB = list(A), list(B)  # staged reads
    alpha = float(getattr(params, "kungfu_sma_alpha", 0.1))
    switch = int(getattr(params, "kungfu_ada_switch_step", 100))
    rngs = [random.Random(int(getattr(params, "kungfu_peer_seed", 0)) * 7919 + w)
            for w in range(num_workers)]
    for step in range(params.num_batches):
        grads = []
        for w in range(num_workers):
            xb = workers[w][step % n_batches]
            m = xb.mean()
            a, b = (RA[w], RB[w]) if staged else (A[w], B[w])
            base = m * a * b
            total = base + wd * (a * a + b * b) / 2
            losses[w].append(base if params.loss_type_to_report == "base_loss" else total)
            grads.append((m * b, m * a, a, b))  # data gradient; wd added at update
        mode = aggregation
        if mode == "ada_sgd":
            mode = "sma" if step < switch else "mean"
        mixA, mixB = list(A), list(B)  # the weights the update starts from
        if mode == "sma":
            avgA, avgB = sum(A) / num_workers, sum(B) / num_workers
            mixA = [(1 - alpha) * a + alpha * avgA for a in A]
            mixB = [(1 - alpha) * b + alpha * avgB for b in B]
            agg = [(g[0], g[1]) for g in grads]
        elif mode == "pair":
            agg = [(g[0], g[1]) for g in grads]
            for w in range(num_workers):
                if num_workers > 1:
                    q = rngs[w].randrange(num_workers - 1)
                    q = q + 1 if q >= w else q
                    mixA[w], mixB[w] = 0.5 * (A[w] + A[q]), 0.5 * (B[w] + B[q])
        elif mode == "sum":
            # every worker's gradient carries its own wd * w term (the
            # reference oracle applies each worker's total-loss gradient,
            # tcb/test_util.py:365-443); replicas are identical in sum modes
            agg = [(sum(g[0] for g in grads) + (num_workers - 1) * wd * A[0],
                    sum(g[1] for g in grads) + (num_workers - 1) * wd * B[0])] * num_workers
        elif mode == "mean":
            agg = [(sum(g[0] for g in grads) / num_workers,
                    sum(g[1] for g in grads) / num_workers)] * num_workers
        else:
            agg = grads
        for w in range(num_workers):
            wa, wb = (grads[w][2], grads[w][3]) if staged else (A[w], B[w])
            ga = agg[w][0] + wd * wa
            gb = agg[w][1] + wd * wb
            RA[w], RB[w] = A[w], B[w]
            A[w], B[w] = mixA[w], mixB[w]
            if params.optimizer == "sgd":
                A[w] -= lr * ga
                B[w] -= lr * gb
            elif params.optimizer == "momentum":
                acc[w][0] = acc[w][0] * mom + ga
                acc[w][1] = acc[w][1] * mom + gb
                A[w] -= lr * (ga + mom * acc[w][0])
                B[w] -= lr * (gb + mom * acc[w][1])
            else:
                raise NotImplementedError(params.optimizer)
    return losses


def get_var_update_params(**kw):
    base = dict(batch_size=2, model="test_model", num_gpus=1, display_every=1,
                num_warmup_batches=0, num_batches=4, weight_decay=2 ** -4,
                init_learning_rate=2 ** -4, optimizer="sgd", device="cpu",
                data_format="NHWC")
    base.update(kw)
    return benchmark.make_params(**base)


def run_test_model(params, inputs=None, digits=15):
    """Runs BenchmarkCNN with the analytic model and returns (losses, logs)."""
    inputs = get_fake_var_update_inputs() if inputs is None else inputs
    with capture_logs() as logs, monkey_patch(benchmark, LOSS_AND_ACCURACY_DIGITS_TO_SHOW=digits):
        bench = benchmark.BenchmarkCNN(params, dataset=TestDataSet(), model=TestCNNModel(params))
        bench.set_fake_data(inputs, np.ones(inputs.shape[0], dtype=np.int64))
        stats = bench.run()
    global LAST_VARS, LAST_STATS
    LAST_STATS = stats
    LAST_VARS = [float(p.detach().float().sum()) for _, p in bench.net.trainable_variables()]
    outs = get_training_outputs_from_logs(logs, params.print_training_accuracy)
    return [o.loss for o in outs], logs


LAST_VARS = None
LAST_STATS = None
