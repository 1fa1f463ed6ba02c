#!/usr/bin/env python3
"""Per-variable gradient error of the GPU path vs the CPU fp32 reference."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from test_model_gpu import _grads
name, ds, size = sys.argv[1], sys.argv[2], (int(sys.argv[3]) if len(sys.argv) > 3 else None)
dt = {"bf16": torch.bfloat16, "fp32": torch.float32}[os.environ.get("DT", "bf16")]
lr, gr = _grads(name, ds, "cpu", torch.float32, size)
lg, gg = _grads(name, ds, torch.device("cuda", 0), dt, size)
print("loss cpu %.5f gpu %.5f" % (lr, lg))
for k, ref in gr.items():
    got = gg[k]
    print("%-50s rel %.4f  |ref| %.3e" % (k, float((got - ref).norm() / (ref.norm() + 1e-12)), float(ref.norm())))
