#!/usr/bin/env python3
"""ResNet-50 conv2_x 3x3 (56x56, 64 -> 64, batch 256, bf16) with the fused
epilogues the training step uses: forward + BN statistics, dgrad + producer
BN ReLU bit mask + BN backward partials.  Times each igemm kernel choice
(interleaved rounds) and prints us / TFLOP/s / % of the speed of light
(max(bytes / 6 TB/s, flops / 2.5 PF/s))."""

import argparse
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd.ops import conv_hip  # noqa: E402
from kf_benchmarks_amd.ops import nn as F  # noqa: E402


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
    ap.add_argument("--hw", type=int, default=56)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--algos", default="onebuf,s3")
    ap.add_argument("--passes", default="fwd,dgrad,wgrad")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, H = a.batch, a.hw
    dt = torch.bfloat16
    x = torch.randn(n, H, H, 64, device=dev, dtype=dt)
    w = torch.randn(64, 3, 3, 64, device=dev, dtype=dt) * 0.05
    dy = torch.randn(n, H, H, 64, device=dev, dtype=dt)
    xb = torch.randn(n, H, H, 64, device=dev, dtype=dt)
    bits = torch.randint(0, 255, (n * H * H * 8,), device=dev, dtype=torch.uint8)
    mean = torch.randn(64, device=dev)
    st = conv_hip.stats_buffer(64, dev)
    pads = F.resolve_pads("SAME_RESNET", H, H, 3, 3, 1, 1)
    flops = 2.0 * n * H * H * 64 * 576
    act = n * H * H * 64 * 2
    sol = {"fwd": max(2 * act / 6e12, flops / 2.5e15) * 1e6,
           "dgrad": max((3 * act + act / 16) / 6e12, flops / 2.5e15) * 1e6}
    passes = {
        "fwd": lambda: conv_hip.conv_fwd(x, w, (1, 1), pads, st.zero_()),
        "dgrad": lambda: conv_hip.conv_dgrad(dy, w, x.shape, (1, 1), pads,
                                             (st.zero_(), bits, xb, mean)),
        "wgrad": lambda: conv_hip.conv_wgrad(dy, x, (64, 3, 3, 64), (1, 1), pads, out=dwb),
    }
    dwb = torch.zeros(64, 3, 3, 64, device=dev)
    sol["wgrad"] = max(2 * act / 6e12, flops / 2.5e15) * 1e6
    passes = {k: v for k, v in passes.items() if k in a.passes.split(",")}
    algos = a.algos.split(",")
    res = {}
    for _ in range(a.rounds):
        for al in algos:
            conv_hip._IG_FORCE = conv_hip.IG_ALGOS[al]
            # wgrad: the streaming kernel vs the autotuned tiled kernels
            conv_hip._WGRAD_ALGO = "s3" if al == "s3" else ""
            conv_hip._NO_S3 = al != "s3"
            conv_hip._wgrad_tuned.clear()
            for pn, fn in passes.items():
                res.setdefault((al, pn), []).append(timeit(fn, a.iters))
    conv_hip._IG_FORCE = None
    print("conv2_x 3x3 %dx%d 64->64 batch %d, fused epilogues (min over %d rounds)"
          % (H, H, n, a.rounds))
    for pn in passes:
        for al in algos:
            t = min(res[(al, pn)])
            print("  %-6s %-8s %8.1f us  %6.1f TF/s  %5.1f%% of SOL (%.1f us)"
                  % (pn, al, t, flops / t / 1e6, 100 * sol[pn] / t, sol[pn]))


if __name__ == "__main__":
    main()
