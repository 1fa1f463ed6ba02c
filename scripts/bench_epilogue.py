#!/usr/bin/env python3
"""Implicit-GEMM kernel variants on the memory-heavy short-K conv shapes,
with and without the fused BN-statistics epilogue (isolates the epilogue
cost), next to a plain device copy of the output size (bandwidth yardstick).

usage: bench_epilogue.py [--iters N] [--algos a,b,...]
"""
import argparse
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd.ops import conv_hip  # noqa: E402

# name, (N, H, W, C, KH, KW, Cout)  stride 1, no padding
SHAPES = [
    ("56x56 64->256 1x1", (256, 56, 56, 64, 1, 1, 256)),
    ("stem s2d 112x115 64->64 1x4", (256, 112, 115, 64, 1, 4, 64)),
    ("56x56 256->64 1x1", (256, 56, 56, 256, 1, 1, 64)),
    ("28x28 128->512 1x1", (256, 28, 28, 128, 1, 1, 512)),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--algos", default="classic,glds,classic_n64,glds_n64,onebuf,onebuf_n64")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    for name, (n, H, W, C, KH, KW, cout) in SHAPES:
        OH, OW = H - KH + 1, W - KW + 1
        x = torch.randn(n, H, W, C, device=dev, dtype=dt)
        w = torch.randn(cout, KH, KW, C, device=dev, dtype=dt) * 0.05
        y = torch.empty(n, OH, OW, cout, device=dev, dtype=dt)
        stats = torch.zeros(2 * conv_hip.STATS_SPREAD * cout, device=dev)
        geo = (n, H, W, C, OH, OW, KH, KW, 1, 1, 0, 0, cout, OH, OW, 1, cout, 0)
        # dgrad-style epilogue operands: ReLU mask, producer-BN input, mean, addend
        mask, xbn, addend = (torch.randn_like(y) for _ in range(3))
        mean = torch.zeros(cout, device=dev)
        ybytes = y.numel() * 2
        xbytes = x.numel() * 2
        tc = timeit(lambda: y.copy_(torch.empty_like(y)), a.iters) if False else \
            timeit(lambda: torch.empty_like(y).copy_(y), a.iters)
        print("%s: out %.0f MB, in %.0f MB; copy of out: %.1f us (%.2f TB/s r+w)"
              % (name, ybytes / 1e6, xbytes / 1e6, tc, 2 * ybytes / tc / 1e6))
        for al in a.algos.split(","):
            algo = conv_hip.IG_ALGOS[al]
            t0 = timeit(lambda: conv_hip._igemm_call(algo, x, w, y, geo), a.iters)
            t1 = timeit(lambda: conv_hip._igemm_call(algo, x, w, y, geo, stats), a.iters)
            t2 = timeit(lambda: conv_hip._igemm_call(algo, x, w, y, geo, stats, mask, xbn, mean,
                                                     addend), a.iters)
            print("  %-11s plain %7.1f us (%.2f TB/s)   +stats %7.1f us   dgrad-fused %7.1f us"
                  % (al, t0, (ybytes + xbytes) / t0 / 1e6, t1, t2))


if __name__ == "__main__":
    main()
