"""Command-line entry point (role of tcb/tf_cnn_benchmarks.py:33-64).

    python -m kf_benchmarks_amd.cli --model=resnet50 --batch_size=256 --use_bf16 \
        --variable_update=kungfu --num_gpus=1 ...

Multi-GPU: one process per GPU, launched by ``python -m
kf_benchmarks_amd.parallel.launcher -np N`` (KungFu ``kungfu-run``
compatible) or ``torch.distributed.run``.  A single command with
``--num_gpus=N`` (the reference's in-process towers) is relaunched here as N
tower processes through ``kfb-run -chief-only`` with KFB_TOWER_GROUP=1; the
console shows tower 0, which reports for the whole worker.
"""

from __future__ import annotations

import os
import subprocess
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
    if _needs_tower_launch(params):
        return _launch_towers(params, argv)
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


def _needs_tower_launch(params) -> bool:
    return (params.num_gpus > 1 and params.device.lower() == "gpu"
            and "WORLD_SIZE" not in os.environ
            and params.variable_update not in ("horovod", "kungfu")
            and not params.job_name and os.environ.get("KFB_NO_TOWER_LAUNCH") != "1")


def _launch_towers(params, argv) -> int:
    """Runs this command as params.num_gpus tower processes (no GPU has been
    touched in this process; the towers are children, not an exec)."""
    from .parallel import launcher
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, KFB_TOWER_GROUP="1",
               PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    logdir = os.environ.get("KFB_TOWER_LOGDIR", os.path.join(
        params.train_dir or "/tmp", "kfb_towers"))
    cmd = [launcher.launcher_binary(), "-np", str(params.num_gpus), "-chief-only",
           "-logdir", logdir, "--", sys.executable, "-m", "kf_benchmarks_amd.cli"] + list(argv)
    return subprocess.call(cmd, env=env)


if __name__ == "__main__":
    sys.exit(main())
