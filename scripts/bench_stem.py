#!/usr/bin/env python3
"""ResNet stem (7x7/2, 3 -> 64, bs256, bf16) through the model's conv path:
the pixel-pair strided conv vs the space-to-depth repack, forward and
forward + weight gradient, plus the kernels each runs (torch.profiler)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd.ops import conv as conv_ops  # noqa: E402
from kf_benchmarks_amd.ops import conv_hip  # noqa: E402
from kf_benchmarks_amd.ops import nn as F  # noqa: E402


def timeit(fn, iters=20):
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
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev, dt = torch.device("cuda", 0), torch.bfloat16
    x = torch.randn(bs, 224, 224, 3, device=dev, dtype=dt)
    w = (torch.randn(64, 7, 7, 3, device=dev) * 0.05).requires_grad_(True)
    pads = F.resolve_pads("SAME_RESNET", 224, 224, 7, 7, 2, 2)
    dy = torch.randn(bs, 112, 112, 64, device=dev, dtype=dt)
    for mode in ("pairs", "s2d"):
        conv_hip._STEM_MODE = mode

        def fwd():
            with torch.no_grad():
                return conv_ops.conv2d(x, w, w.detach().to(dt), (2, 2), pads, "hip")

        def fwd_bwd():
            y = conv_ops.conv2d(x, w, w.detach().to(dt), (2, 2), pads, "hip")
            y.backward(dy)

        tf = timeit(fwd)
        tb = timeit(fwd_bwd)
        print("%-6s fwd %8.1f us   fwd+wgrad %8.1f us" % (mode, tf, tb), flush=True)
        acts = [torch.profiler.ProfilerActivity.CUDA]
        with torch.profiler.profile(activities=acts) as prof:
            fwd_bwd()
            torch.cuda.synchronize()
        for ev in prof.key_averages():
            if ev.device_time_total > 0:
                print("   %-80s %8.1f us" % (ev.key[:80], ev.device_time_total))


if __name__ == "__main__":
    main()
