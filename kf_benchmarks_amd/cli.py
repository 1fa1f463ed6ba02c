"""Command-line entry point (role of tcb/tf_cnn_benchmarks.py:33-64).

    python -m kf_benchmarks_amd.cli --model=resnet50 --batch_size=256 --use_bf16 \
        --variable_update=kungfu --num_gpus=1 ...

Multi-GPU: one process per GPU, launched by ``python -m
kf_benchmarks_amd.parallel.launcher -np N`` (KungFu ``kungfu-run``
compatible) or ``torch.distributed.run``.
"""

from __future__ import annotations

import sys

import torch

from . import benchmark, cnn_util, flags, params as params_lib
from .parallel import comm


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    try:
        values = flags.parse_flags(argv)
    except flags.FlagError as e:
        print("FATAL Flags parsing error: %s" % e, file=sys.stderr)
        return 2
    params = params_lib.make_params(**values)
    params = benchmark.setup(params)
    bench = benchmark.BenchmarkCNN(params)
    tfversion = "kf_benchmarks_amd %s / torch %s" % (
        __import__("kf_benchmarks_amd").__version__, torch.__version__)
    if getattr(torch.version, "hip", None):
        tfversion += " / HIP %s" % torch.version.hip
    cnn_util.log_fn("TensorFlow:  %s" % tfversion)
    bench.print_info()
    bench.run()
    if params.variable_update == "kungfu":
        bench.world.barrier(bench.device if bench.device_type == "cuda" else None)
    comm.get_world().shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
