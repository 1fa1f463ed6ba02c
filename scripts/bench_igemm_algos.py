#!/usr/bin/env python3
"""Times implicit-GEMM kernel choices on one conv geometry (forward, bf16,
random operands, stats epilogue), reps back-to-back per timing.
usage: bench_igemm_algos.py N H W Cin Cout KH KW stride algo[,algo...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from kf_benchmarks_amd.ops import conv_hip  # noqa: E402
from kf_benchmarks_amd.ops import nn as F  # noqa: E402


def main():
    n, H, W, cin, cout, kh, kw, s = map(int, sys.argv[1:9])
    algos = sys.argv[9].split(",")
    dev = torch.device("cuda", 0)
    x = torch.randn(n, H, W, cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(cout, kh * kw * cin, device=dev) / (kh * kw * cin) ** 0.5).to(torch.bfloat16)
    pt, pb, pl, pr = F.resolve_pads("SAME_RESNET", H, W, kh, kw, s, s)
    OH = (H + pt + pb - kh) // s + 1
    OW = (W + pl + pr - kw) // s + 1
    y = torch.empty(n, OH, OW, cout, device=dev, dtype=torch.bfloat16)
    stats = torch.zeros(2 * conv_hip.STATS_SPREAD * cout, device=dev)
    geo = (n, H, W, cin, OH, OW, kh, kw, s, s, pt, pl, cout, OH, OW, 1, cout, 0)
    flops = 2.0 * n * OH * OW * cout * kh * kw * cin
    for a in algos:
        run = lambda: conv_hip._igemm_call(conv_hip.IG_ALGOS[a], x, w, y, geo, stats)
        for _ in range(3):
            run()
        best = float("inf")
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1) / 10)
        print("%-12s %8.1f us  %7.1f TF/s" % (a, best * 1e3, flops / best / 1e9), flush=True)


if __name__ == "__main__":
    main()
