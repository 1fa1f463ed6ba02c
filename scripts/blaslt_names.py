#!/usr/bin/env python3
"""hipBLASLt (torch.matmul) on the large-K ResNet-50 1x1 GEMMs where it beats
our igemm: run under rocprofv3 --kernel-trace to read its kernel choices
(macro tile, depth, wave layout) from the Cijk_* names."""
import torch

dev = torch.device("cuda", 0)
dt = torch.bfloat16
for M, N, K in ((50176, 256, 1024), (50176, 1024, 256), (12544, 2048, 512), (12544, 512, 2048)):
    a = torch.randn(M, K, device=dev, dtype=dt)
    b = torch.randn(N, K, device=dev, dtype=dt)
    for _ in range(5):
        a @ b.t()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        a @ b.t()
    e.record()
    e.synchronize()
    t = s.elapsed_time(e) / 20 * 1e3
    print("M=%d N=%d K=%d  %.1f us  %.0f TF/s" % (M, N, K, t, 2 * M * N * K / t / 1e6), flush=True)
