#!/usr/bin/env python3
"""Gradient agreement of the GPU path with the CPU fp32 reference.

usage: diag_grads.py MODEL DATASET [IMAGE_SIZE] [BATCH]
Prints, for CPU bf16 / GPU fp32 / GPU bf16 fused / GPU bf16 unfused, the
minimum and median per-variable cosine against CPU fp32 - the CPU-bf16 row
shows how well-conditioned the configuration is (small BN populations make
bf16 gradients chaotic regardless of the kernels).
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from kf_benchmarks_amd.ops import conv as conv_ops
from test_model_gpu import _grads, _cos

name, ds = sys.argv[1], sys.argv[2]
size = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3] != "0" else None
batch = int(sys.argv[4]) if len(sys.argv) > 4 else 4
dev = torch.device("cuda", 0)
lr, ref = _grads(name, ds, "cpu", torch.float32, size, batch)
runs = {"cpu_bf16": ("cpu", torch.bfloat16, True), "gpu_fp32": (dev, torch.float32, True),
        "gpu_bf16_fused": (dev, torch.bfloat16, True),
        "gpu_bf16_unfused": (dev, torch.bfloat16, False)}
print("%s %s size=%s batch=%d  cpu fp32 loss %.5f" % (name, ds, size, batch, lr))
for tag, (d, dt, fuse) in runs.items():
    conv_ops.FUSE_BN = fuse
    try:
        l, g = _grads(name, ds, d, dt, size, batch)
    finally:
        conv_ops.FUSE_BN = True
    cs = sorted((_cos(g[k], r), k) for k, r in ref.items() if r.norm() > 0)
    print("%-18s loss %.5f  min cos %.4f (%s)  median %.4f" %
          (tag, l, cs[0][0], cs[0][1], cs[len(cs) // 2][0]))
