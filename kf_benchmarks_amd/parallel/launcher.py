"""KungFu-compatible launcher front end (role of ``kungfu-run``,
tcb/README.md:95-105, tcb/run_kf.sh).

    python -m kf_benchmarks_amd.parallel.launcher -np 8 \\
        python3 tf_cnn_benchmarks.py --variable_update=kungfu --num_gpus=1 ...

The process management is native: this module builds (if needed) and runs
``_lib/kfb-run`` (csrc/launcher/kfb_run.cpp), which forks one peer per GPU
with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT,
prefixes each peer's output with ``[127.0.0.1.<port>::stdout]``, writes
``127.0.0.1.<port>.{stdout,stderr}.log`` and fails fast when a peer exits
non-zero ("exit on error: N tasks failed").  Peers then join the RCCL
world through ``torch.distributed`` (parallel/comm.py).
"""

from __future__ import annotations

import os
import subprocess
import sys
from typing import List, Optional


def launcher_binary() -> str:
    from .. import build
    path = build.RUN_BIN
    if not os.path.exists(path) or os.environ.get("KFB_NO_AUTOBUILD") != "1":
        path = build.build_launcher() or path
    if not os.path.exists(path):
        raise RuntimeError("kfb-run launcher is not built (python -m kf_benchmarks_amd.build)")
    return path


def run(np_: int, cmd: List[str], logdir: Optional[str] = None, quiet: bool = False,
        timeout: Optional[float] = None, port_range: Optional[str] = None,
        env: Optional[dict] = None, capture: bool = False):
    """Runs ``cmd`` on ``np_`` local peers; returns the CompletedProcess."""
    argv = [launcher_binary(), "-np", str(np_)]
    if logdir:
        os.makedirs(logdir, exist_ok=True)
        argv += ["-logdir", logdir]
    if quiet:
        argv.append("-q")
    if timeout:
        argv += ["-timeout", str(timeout)]
    if port_range:
        argv += ["-port-range", port_range]
    argv.append("--")
    argv += list(cmd)
    return subprocess.run(argv, env=env, capture_output=capture, text=capture)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    # the child is started as a subprocess (never exec'd over this process)
    return subprocess.call([launcher_binary()] + argv)


if __name__ == "__main__":
    sys.exit(main())
