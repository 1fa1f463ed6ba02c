#!/usr/bin/env python3
"""Times the implicit-GEMM kernels on the ResNet-50 "conv a" data gradient
(1x1, K = the conv's output channels) with its full fused epilogue: the
other branch's gradient as addend, the producer BN's ReLU bit mask, its raw
input x_bn and the BN backward partial sums.  Prints us and the achieved
HBM rate of the operand + epilogue bytes per kernel, next to a 3-read /
1-write streaming reference of the same tensor size.
usage: bench_dgrad_epilogue.py [algo,algo,...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from kf_benchmarks_amd.ops import conv_hip  # noqa: E402

# (H, K = conv cout, ncol = conv cin) at batch 256
SHAPES = [(56, 64, 256), (28, 128, 512), (14, 256, 1024), (7, 512, 2048)]
ALGOS = ["classic", "glds", "onebuf", "tall256", "small", "gshort64", "gshort128", "gmulti64",
         "gmulti128", "gbig256", "g8p", "classic_n64", "glds_n64", "onebuf_n64", "onebuf_n64_e",
         "classic_n64_e", "db"]


def timeit(fn, reps=10, rounds=5):
    for _ in range(3):
        fn()
    best = float("inf")
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best * 1e3  # us


def main():
    algos = sys.argv[1].split(",") if len(sys.argv) > 1 else ALGOS
    dev = torch.device("cuda", 0)
    n = 256
    for H, K, ncol in SHAPES:
        M = n * H * H
        dy = torch.randn(n, H, H, K, device=dev).to(torch.bfloat16)
        wt = (torch.randn(ncol, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        y = torch.empty(n, H, H, ncol, device=dev, dtype=torch.bfloat16)
        add = torch.randn_like(y)
        xbn = torch.randn_like(y)
        bits = torch.randint(0, 256, (M * ncol // 8,), device=dev, dtype=torch.uint8)
        mean = torch.zeros(ncol, device=dev)
        stats = torch.zeros(2 * conv_hip.STATS_SPREAD * ncol, device=dev)
        geo = (n, H, H, K, H, H, 1, 1, 1, 1, 0, 0, ncol, H, H, 1, ncol, 0)
        nbytes = dy.numel() * 2 + 3 * y.numel() * 2 + bits.numel()
        ref = timeit(lambda: torch.add(add, xbn, out=y))
        print("-- %dx%d K=%d -> %d: %.0f MB; torch add (2 reads + 1 write of y) %.1f us = %.2f TB/s"
              % (H, H, K, ncol, nbytes / 1e6, ref, 3 * y.numel() * 2 / ref / 1e6), flush=True)
        for a in algos:
            run = lambda: conv_hip._igemm_call(conv_hip.IG_ALGOS[a], dy, wt, y, geo, stats, bits,
                                               xbn, mean, add, None, None, 4)
            t = timeit(run)
            print("   %-12s %8.1f us  %5.2f TB/s" % (a, t, nbytes / t / 1e6), flush=True)


if __name__ == "__main__":
    main()
