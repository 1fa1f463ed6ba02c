#!/usr/bin/env python3
"""HBM streaming rate (write-only fill, read-only sum, copy) and of the elementwise passes on a ResNet-50 activation
([256, 56, 56, 256] bf16 = 411 MB): our BN apply (residual + ReLU, via the
inference entry point that shares bn_apply_k) and add kernels next to
PyTorch's own copy / add as the achievable-rate yardstick."""

import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd.ops import _native as N  # noqa: E402


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
    return s.elapsed_time(e) / iters * 1e-3


def main():
    dev = torch.device("cuda", 0)
    shapes = [tuple(int(v) for v in s.split("x")) for s in (sys.argv[1].split(",") if len(sys.argv) > 1 else
              ["256x56x56x256", "256x28x28x512", "256x14x14x1024", "256x56x56x64"])]
    for shp in shapes:
        x = torch.randn(shp, device=dev, dtype=torch.bfloat16)
        r = torch.randn(shp, device=dev, dtype=torch.bfloat16)
        y = torch.empty_like(x)
        C = shp[-1]
        rows = x.numel() // C
        g = torch.rand(C, device=dev) + 0.5
        b = torch.randn(C, device=dev)
        rm = torch.randn(C, device=dev)
        rv = torch.rand(C, device=dev) + 0.5
        sc = torch.empty(C, device=dev)
        sh = torch.empty(C, device=dev)
        nb = x.numel() * 2
        st = N.stream(dev)
        cases = {
            "torch fill (0R1W)": (lambda: y.fill_(1.0), 1),
            "torch sum (1R)": (lambda: x.view(-1, 4096).sum(dim=0), 1),
            "torch copy (1R1W)": (lambda: y.copy_(x), 2),
            "torch add (2R1W)": (lambda: torch.add(x, r, out=y), 3),
            "kfb_add (2R1W)": (lambda: N.call("kfb_add", N.dt(x), x.data_ptr(), r.data_ptr(),
                                              y.data_ptr(), x.numel(), 0, st), 3),
            "bn_apply res+relu (2R1W)": (lambda: N.call(
                "kfb_bn_fwd_infer", N.dt(x), x.data_ptr(), r.data_ptr(), y.data_ptr(), rows, C,
                g.data_ptr(), b.data_ptr(), rm.data_ptr(), rv.data_ptr(), 1e-5, sc.data_ptr(),
                sh.data_ptr(), 1, st), 3),
            "bn_apply relu (1R1W)": (lambda: N.call(
                "kfb_bn_fwd_infer", N.dt(x), x.data_ptr(), None, y.data_ptr(), rows, C,
                g.data_ptr(), b.data_ptr(), rm.data_ptr(), rv.data_ptr(), 1e-5, sc.data_ptr(),
                sh.data_ptr(), 1, st), 2),
        }
        print("shape %s (%.0f MB per tensor)" % (shp, nb / 1e6))
        for name, (fn, k) in cases.items():
            t = timeit(fn)
            print("  %-28s %8.1f us  %6.2f TB/s" % (name, t * 1e6, k * nb / t / 1e12))


if __name__ == "__main__":
    main()
