#!/usr/bin/env python3
"""Weight-gradient kernel timing for one ResNet-50 geometry at batch 256,
bf16: every launch-shape candidate of the autotune (``conv_hip``'s
_wgrad_candidates, slab reduce included), or the ones given with
--targets (e.g. 512,glds/512).  For profiling a single kernel:

  python scripts/bench_wgrad.py --hw 14 --cin 256 --cout 256 --k 3 --targets glds/512
"""
import argparse
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd.ops import conv_hip  # noqa: E402


def parse_target(t):
    if t.startswith("glds/"):
        return int(t.split("/")[1]) | conv_hip._WGRAD_GLDS
    if t == "s3w":
        return conv_hip._WGRAD_S3
    return int(t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--hw", type=int, default=14)
    ap.add_argument("--cin", type=int, default=256)
    ap.add_argument("--cout", type=int, default=256)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--targets", default=None)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, H, C, K = a.batch, a.hw, a.cin, a.k
    pad = K // 2
    x = torch.randn(n, H, H, C, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(n, H, H, a.cout, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(a.cout, K, K, C, device=dev, dtype=torch.float32)
    geo = (n, H, H, C, H, H, K, K, 1, 1, pad, pad, a.cout)
    cands = ([parse_target(t) for t in a.targets.split(",")] if a.targets
             else conv_hip._wgrad_candidates(geo))
    flops = 2.0 * n * H * H * a.cout * K * K * C
    for t in cands:
        for _ in range(2):
            conv_hip._wgrad_launch(dy, x, dw, geo, t)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            conv_hip._wgrad_launch(dy, x, dw, geo, t)
        e.record()
        e.synchronize()
        us = s.elapsed_time(e) * 1e3 / a.iters
        name = ("glds/%d" % (t & 0xFFFF)) if t >> 16 == 1 else "s3w" if t >> 16 == 2 else str(t)
        print("%dx%d %d->%d k%d  %-10s %8.1f us  %6.0f TF/s" % (H, H, C, a.cout, K, name, us,
                                                               flops / us / 1e6), flush=True)


if __name__ == "__main__":
    main()
