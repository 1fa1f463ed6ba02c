"""Evaluation: --eval from checkpoints and --eval_during_training_*.

Role of tcb/benchmark_cnn.py:1757-1923 (_run_eval / _eval_once /
_do_eval) and the eval-during-training hooks of the hot loop
(tcb/benchmark_cnn.py:2310-2326, 2393-2403).  Log lines are verbatim:
``'%i\\t%.1f examples/sec'`` and
``'Accuracy @ 1 = %.4f Accuracy @ 5 = %.4f [%d examples]'``.
"""

from __future__ import annotations

import time

import torch

from . import cnn_util
from .constants import BenchmarkMode
from .utils import checkpoint as ckpt_lib

from .parallel import comm  # noqa: E402

log_fn = cnn_util.log_fn


def _make_eval_input(bench):
    from .data.input_pipeline import make_input_source
    return make_input_source(bench, subset="validation")


def eval_once(bench, input_source, num_batches, global_step, summary_writer=None):
    p = bench.params
    top1 = top5 = 0.0
    batch = bench.batch_size
    loop_start = start = time.time()
    from .parallel import watchdog
    for step in range(num_batches):
        watchdog.beat("eval", step, startup=step < 2)
        inputs = tuple(input_source.next())
        with torch.no_grad():
            res = bench.net.forward_inputs(inputs, phase_train=False)
            acc = bench.model.accuracy_function(inputs, res.logits)
            if "top_1_accuracy" not in acc:
                # unreduced outputs (e.g. DeepSpeech2 probabilities): the model
                # reduces them on the host (tcb/benchmark_cnn.py postprocess)
                host = bench.model.postprocess(
                    {k: v.detach().float().cpu().numpy() for k, v in acc.items()})
                acc = {"top_1_accuracy": host["top_1_accuracy"] * batch,
                       "top_5_accuracy": host["top_5_accuracy"] * batch}
            counts = torch.stack([torch.as_tensor(acc["top_1_accuracy"], dtype=torch.float32),
                                  torch.as_tensor(acc["top_5_accuracy"], dtype=torch.float32)])
            if getattr(bench, "tower_mode", False):
                # towers of one worker: the accuracy is over the global batch
                counts = counts.to(bench.device)
                comm.all_reduce(counts)
            counts = counts.cpu()
        results = {"top_1_accuracy": float(counts[0]) / batch,
                   "top_5_accuracy": float(counts[1]) / batch,
                   "global_step": global_step}
        top1 += results["top_1_accuracy"]
        top5 += results["top_5_accuracy"]
        if (step + 1) % p.display_every == 0:
            duration = time.time() - start
            log_fn("%i\t%.1f examples/sec" % (step + 1, batch * p.display_every / duration))
            start = time.time()
    loop_end = time.time()
    acc1 = top1 / num_batches if num_batches else 0.0
    acc5 = top5 / num_batches if num_batches else 0.0
    log_fn("Accuracy @ 1 = %.4f Accuracy @ 5 = %.4f [%d examples]"
           % (acc1, acc5, num_batches * batch))
    if summary_writer is not None:
        summary_writer.add_scalars({"eval/Accuracy@1": acc1, "eval/Accuracy@5": acc5},
                                   global_step)
    elapsed = max(loop_end - loop_start, 1e-9)
    ips = num_batches * batch / elapsed
    if bench.mode != BenchmarkMode.TRAIN_AND_EVAL:
        log_fn("-" * 64)
        log_fn("total images/sec: %.2f" % ips)
        log_fn("-" * 64)
    if bench.benchmark_logger:
        bench.benchmark_logger.log_evaluation_result({
            "eval_top_1_accuracy": acc1, "eval_top_5_accuracy": acc5,
            "eval_average_examples_per_sec": ips, "global_step": global_step})
    return acc1, acc5, ips


def run_eval(bench):
    p = bench.params
    if p.train_dir is None:
        raise ValueError("Trained model directory not specified")
    bench.build()
    saver = ckpt_lib.Saver(bench, max_to_keep=p.max_ckpts_to_keep)
    writer = None
    if p.eval_dir and p.summary_verbosity > 0:
        from .utils.summary import SummaryWriter
        writer = SummaryWriter(p.eval_dir)
    stats = {}
    while True:
        try:
            global_step = ckpt_lib.load_checkpoint(saver, p.train_dir)
        except ckpt_lib.CheckpointNotFoundException:
            log_fn("Checkpoint not found in %s" % p.train_dir)
        else:
            acc1, acc5, ips = eval_once(bench, bench.input, bench.num_batches, global_step,
                                        writer)
            stats = {"top_1_accuracy": acc1, "top_5_accuracy": acc5, "images_per_sec": ips,
                     "global_step": global_step}
        if p.eval_interval_secs <= 0:
            break
        time.sleep(p.eval_interval_secs)
    return stats


class EvalDuringTraining:
    """Runs evaluation inside the training loop at the configured cadence."""

    def __init__(self, bench):
        self.bench = bench
        p = bench.params
        ex = bench.dataset.num_examples_per_epoch("train")
        per_epoch = ex / float(bench.batch_size * bench.num_workers)
        self.steps = set()
        self.every = None
        if p.eval_during_training_every_n_steps:
            self.every = p.eval_during_training_every_n_steps
        elif p.eval_during_training_every_n_epochs:
            self.every = max(int(p.eval_during_training_every_n_epochs * per_epoch), 1)
        elif p.eval_during_training_at_specified_steps:
            self.steps = {int(s) for s in p.eval_during_training_at_specified_steps}
        elif p.eval_during_training_at_specified_epochs:
            self.steps = {int(float(e) * per_epoch) for e in
                          p.eval_during_training_at_specified_epochs}
        self.num_eval_batches = p.num_eval_batches or max(
            int(bench.dataset.num_examples_per_epoch("validation") / bench.batch_size), 1)
        if p.num_eval_epochs:
            self.num_eval_batches = max(int(
                p.num_eval_epochs * bench.dataset.num_examples_per_epoch("validation")
                / bench.batch_size), 1)
        self._input = None
        self.history = []

    def should_eval(self, global_step):
        if self.every:
            return global_step > 0 and global_step % self.every == 0
        return global_step in self.steps

    def maybe_eval(self, global_step) -> bool:
        """Returns True if training should stop (accuracy target reached)."""
        if not self.should_eval(global_step):
            return False
        if self._input is None:
            self._input = _make_eval_input(self.bench)
        acc1, acc5, _ = eval_once(self.bench, self._input, self.num_eval_batches, global_step)
        self.history.append((global_step, acc1, acc5))
        target = self.bench.params.stop_at_top_1_accuracy
        if target and acc1 >= target:
            log_fn("Stopping, as eval accuracy at least %s was reached" % target)
            return True
        return False

    def stats(self):
        if not self.history:
            return {}
        step, a1, a5 = self.history[-1]
        return {"last_eval_step": step, "top_1_accuracy": a1, "top_5_accuracy": a5}
