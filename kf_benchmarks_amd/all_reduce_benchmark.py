"""Gradient all-reduce micro-benchmark (role of tcb/all_reduce_benchmark.py).

Times only the cross-GPU reduction of a model's gradients: the model is
built (to get its exact variable set in flat-buffer order), then every step
runs ``--iters_per_step`` back-to-back all-reduces of the whole gradient
through the same bucketed RCCL path training uses (parallel/bucket.py, with
--bucket_size_mb / --gradient_repacking / --gradient_wire_dtype /
--all_reduce_spec shards).  Output keeps the reference's lines
("Running all-reduce ops", "Iteration: N. Average time per step so far: T",
"Average time per step: T") and adds the RCCL-style algorithm and bus
bandwidth of one all-reduce.

    python -m kf_benchmarks_amd.parallel.launcher -np 8 \\
        python3 -m kf_benchmarks_amd.all_reduce_benchmark --model=resnet50 \\
        --variable_update=replicated --num_batches=50 --iters_per_step=5

``--num_gpus=N`` in one command is relaunched as N tower processes like the
training CLI.
"""

from __future__ import annotations

import sys
import time

import torch

from . import benchmark, flags, optim, params as params_lib
from .cnn_util import log_fn
from .models.model import make_network
from .parallel.bucket import BucketReducer
from .parallel.variable_mgr import make_strategy


def get_var_shapes(net):
    return [list(p.shape) for _, p in net.trainable_variables()]


def run_benchmark(bench, num_iters: int):
    p = bench.params
    if p.variable_update != "replicated":
        raise ValueError("--variable_update=replicated must be specified to use "
                         "the all-reduce benchmark")
    if p.variable_consistency == "relaxed":
        raise ValueError("--variable_consistency=relaxed is not supported")
    net = make_network(bench.model, bench.dataset.num_classes, bench.device, bench.compute_dtype,
                  kernel_impl=p.kernel_impl, seed=p.tf_random_seed)
    flat = optim.FlatParams(net, None)
    strategy = make_strategy(p, bench.world, flat, bench.tower_mode, bench.num_gpus)
    reducer = strategy.reducer
    if reducer is None:  # single process: still exercise the bucket plan
        reducer = BucketReducer(flat, p.bucket_size_mb, None, overlap=False,
                                num_buckets=p.gradient_repacking)
    flat.grad.normal_()
    nbytes = flat.numel * (reducer.wire_dtype.itemsize if reducer.wire_dtype else 4)
    log_fn("Variables:   %d tensors, %d elements, %.1f MB per all-reduce in %d buckets"
           % (len(get_var_shapes(net)), flat.numel, nbytes / 1e6, reducer.num_buckets))
    sync = (lambda: torch.cuda.synchronize(bench.device)) if bench.device_type == "cuda" \
        else (lambda: None)
    log_fn("Running warmup")
    start = None
    for i in range(-bench.num_warmup_batches, bench.num_batches):
        if i == 0:
            sync()
            bench.world.barrier(bench.device if bench.device_type == "cuda" else None)
            log_fn("Running all-reduce ops")
            start = time.time()
        if i > 0 and i % p.display_every == 0:
            sync()
            log_fn("Iteration: %d. Average time per step so far: %s"
                   % (i, (time.time() - start) / i))
        for _ in range(num_iters):
            reducer.reduce_now()
            flat.grad.mul_(1.0 / max(bench.world.size, 1))  # keep values bounded
    sync()
    per_step = (time.time() - start) / max(bench.num_batches, 1)
    log_fn("Average time per step: %s" % per_step)
    n = bench.world.size
    t = per_step / max(num_iters, 1)
    if t > 0:
        algbw = nbytes / t / 1e9
        busbw = algbw * (2.0 * (n - 1) / n if n > 1 else 0.0)
        log_fn("All-reduce: %.3f ms  algbw %.2f GB/s  busbw %.2f GB/s  (%d ranks)"
               % (t * 1e3, algbw, busbw, n))
    return per_step


def _split_iters(argv):
    iters, rest = 5, []
    it = iter(argv)
    for a in it:
        if a.startswith("--iters_per_step="):
            iters = int(a.split("=", 1)[1])
        elif a == "--iters_per_step":
            iters = int(next(it))
        else:
            rest.append(a)
    return iters, rest


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    iters, rest = _split_iters(argv)
    try:
        values = flags.parse_flags(rest)
    except flags.FlagError as e:
        print("FATAL Flags parsing error: %s" % e, file=sys.stderr)
        return 2
    params = params_lib.make_params(**values)
    from . import cli
    if cli._needs_tower_launch(params):
        import os
        import subprocess
        from .parallel import launcher
        env = dict(os.environ, KFB_TOWER_GROUP="1")
        return subprocess.call([launcher.launcher_binary(), "-np", str(params.num_gpus),
                                "-chief-only", "--", sys.executable, "-m",
                                "kf_benchmarks_amd.all_reduce_benchmark"] + argv, env=env)
    params = benchmark.setup(params)
    bench = benchmark.BenchmarkCNN(params)
    log_fn("TensorFlow:  kf_benchmarks_amd %s / torch %s"
           % (__import__("kf_benchmarks_amd").__version__, torch.__version__))
    run_benchmark(bench, iters)
    bench.world.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
