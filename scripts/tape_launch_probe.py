#!/usr/bin/env python3
"""Host cost of one replayed launch: a tape of N tiny native adds (4 KB
tensors, a chain on one stream) replayed raw (hipLaunchKernel from the
recorded arguments) and through the entry points (libffi + host logic);
host time per launch without waiting for the GPU, and GPU-inclusive time
per launch with a synchronize after each replay."""
import sys
import time

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

import torch  # noqa: E402

from kf_benchmarks_amd.ops import _native as N  # noqa: E402
from kf_benchmarks_amd.ops import tape as T  # noqa: E402


def main(n=1000, reps=20):
    dev = torch.device("cuda", 0)
    lib = N.load()
    a = torch.randn(2048, device=dev).to(torch.bfloat16)
    b = torch.randn(2048, device=dev).to(torch.bfloat16)

    def step():
        x = a
        for _ in range(n):
            x = torch.add(x, b)  # recorded as kfb_add (tape probe)
        return x
    t = T.StepTape(dev)
    t.record(step)
    torch.cuda.synchronize()
    for mode in (1, 0, 1, 0):
        lib.kfb_tape_set_raw(mode)
        t.replay({})
        torch.cuda.synchronize()
        host = wall = 0.0
        for _ in range(reps):
            t0 = time.perf_counter()
            t.replay({})
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            host += t1 - t0
            wall += t2 - t0
        print("%-5s replay: host %.2f us/launch, host+GPU %.2f us/launch (%d launches)"
              % ("raw" if mode else "entry", 1e6 * host / reps / n, 1e6 * wall / reps / n, n))
    lib.kfb_tape_set_raw(1)


if __name__ == "__main__":
    main()
