#!/usr/bin/env python3
"""hipBLASLt (torch.matmul, bf16) on the ResNet-50 1x1-conv GEMM shapes, as a
yardstick for the implicit-GEMM kernels: fwd [M,K]x[K,N], dgrad [M,N]x[N,K],
wgrad [N,M]x[M,K] with M = batch * H * W."""
import torch

SHAPES = [(56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024),
          (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]


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
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    for H, cin, cout in SHAPES:
        M = 256 * H * H
        x = torch.randn(M, cin, device=dev, dtype=dt)
        w = torch.randn(cin, cout, device=dev, dtype=dt)
        dy = torch.randn(M, cout, device=dev, dtype=dt)
        fl = 2.0 * M * cin * cout
        tf = timeit(lambda: x @ w)
        td = timeit(lambda: dy @ w.t())
        tw = timeit(lambda: dy.t() @ x)
        print("%2dx%-2d %4d->%-4d  fwd %7.1f us %6.0f TF/s  dgrad %7.1f us %6.0f TF/s  "
              "wgrad %7.1f us %6.0f TF/s" % (H, H, cin, cout, tf, fl / tf / 1e6, td,
                                            fl / td / 1e6, tw, fl / tw / 1e6))


if __name__ == "__main__":
    main()
