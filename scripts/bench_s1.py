#!/usr/bin/env python3
"""ResNet-50 1x1 expand layers (K -> 4K channels at 56/28/14/7, batch 256,
bf16) with the fused epilogues the training step uses: forward + shifted BN
statistics, and the data gradient of the 4K -> K reduce conv + the producer
BN's ReLU bit mask (+ the residual addend) + BN backward partials.  Times
the streaming kernel (s1) against the autotuned choice among the tiled
kernels ("auto") and any forced ones (interleaved rounds); prints us and %
of the memory speed of light (bytes / 6 TB/s)."""

import argparse
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd.ops import conv_hip  # noqa: E402

LAYERS = {56: 64, 28: 128, 14: 256, 7: 512}


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
    ap.add_argument("--hw", default="56,28,14,7")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--algos", default="auto,s1")
    ap.add_argument("--passes", default="fwd,dgrad,dgrad_noadd")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    for H in [int(h) for h in a.hw.split(",")]:
        K = LAYERS[H]
        C = 4 * K
        n = a.batch
        x = torch.randn(n, H, H, K, device=dev, dtype=dt)
        w = torch.randn(C, 1, 1, K, device=dev, dtype=dt) * K ** -0.5
        wr = torch.randn(K, 1, 1, C, device=dev, dtype=dt) * K ** -0.5  # the reduce conv
        dy = torch.randn(n, H, H, K, device=dev, dtype=dt)
        xb = torch.randn(n, H, H, C, device=dev, dtype=dt)
        add = torch.randn(n, H, H, C, device=dev, dtype=dt)
        bits = torch.randint(0, 255, (n * H * H * C // 8,), device=dev, dtype=torch.uint8)
        mean = torch.randn(C, device=dev)
        shift = torch.randn(C, device=dev)
        st = conv_hip.stats_buffer(C, dev, shift=shift)
        px = n * H * H
        nb = {"fwd": px * (2 * K + 2 * C), "dgrad": px * (2 * K + 6 * C + C // 8),
              "dgrad_noadd": px * (2 * K + 4 * C + C // 8)}
        passes = {
            "fwd": lambda: conv_hip.conv_fwd(x, w, (1, 1), (0, 0, 0, 0), st.zero_()),
            "dgrad": lambda: conv_hip.conv_dgrad(dy, wr, (n, H, H, C), (1, 1), (0, 0, 0, 0),
                                                 (st.zero_(), bits, xb, mean), addend=add),
            "dgrad_noadd": lambda: conv_hip.conv_dgrad(dy, wr, (n, H, H, C), (1, 1),
                                                       (0, 0, 0, 0), (st.zero_(), bits, xb, mean)),
        }
        passes = {k: v for k, v in passes.items() if k in a.passes.split(",")}
        algos = a.algos.split(",")
        res = {}
        for _ in range(a.rounds):
            for al in algos:
                conv_hip._IG_FORCE = None if al == "auto" else conv_hip.IG_ALGOS[al]
                conv_hip._NO_S1 = al == "auto"
                for pn, fn in passes.items():
                    res.setdefault((al, pn), []).append(timeit(fn, a.iters))
        conv_hip._IG_FORCE = None
        conv_hip._NO_S1 = False
        print("1x1 %dx%d %d<->%d batch %d, fused epilogues (min over %d rounds)"
              % (H, H, K, C, n, a.rounds), flush=True)
        for pn in passes:
            sol = nb[pn] / 6e12 * 1e6
            for al in algos:
                t = min(res[(al, pn)])
                print("  %-12s %-10s %8.1f us  %6.2f TB/s  %5.1f%% of SOL (%.1f us)"
                      % (pn, al, t, nb[pn] / t / 1e6, 100 * sol / t, sol), flush=True)
        del x, w, wr, dy, xb, add, bits
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
