#!/usr/bin/env python3
"""ResNet-50 stem (batch 256, 224x224x3 -> 112x112x64, bf16) as the pixel-pair
8x4-tap conv with the BN-statistics epilogue: the streaming kernel (s7) vs
the autotuned tiled kernels; us and % of the memory speed of light."""
import argparse
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd.ops import conv_hip  # noqa: E402


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--algos", default="auto,s7")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = a.batch
    xv = torch.randn(n, 230, 115, 8, device=dev, dtype=torch.bfloat16)
    w2 = torch.randn(64, 8, 4, 8, device=dev, dtype=torch.bfloat16) * 0.06
    st = conv_hip.stats_buffer(64, dev, shift=torch.zeros(64, device=dev))
    nb = xv.numel() * 2 + n * 112 * 112 * 64 * 2
    res = {}
    for _ in range(a.rounds):
        for al in a.algos.split(","):
            conv_hip._IG_FORCE = None if al == "auto" else conv_hip.IG_ALGOS[al]
            conv_hip._NO_S7 = al == "auto"
            res.setdefault(al, []).append(timeit(
                lambda: conv_hip.conv_fwd(xv, w2, (2, 1), (0, 0, 0, 0), st.zero_()), a.iters))
    sol = nb / 6e12 * 1e6
    for al, ts in res.items():
        t = min(ts)
        print("stem fwd %-6s %8.1f us  %5.2f TB/s  %5.1f%% of SOL (%.1f us)"
              % (al, t, nb / t / 1e6, 100 * sol / t, sol))


if __name__ == "__main__":
    main()
