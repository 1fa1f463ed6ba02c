"""Prints the autotuned igemm kernel per ResNet-50 bs256 conv geometry (after 3 steps)
and its fused-epilogue flags.  Usage (GPU): python scripts/dump_igemm_algos.py"""
import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from kf_benchmarks_amd import params as P
from kf_benchmarks_amd.benchmark import BenchmarkCNN
from kf_benchmarks_amd.ops import conv_hip
p = P.make_params(model="resnet50", batch_size=256, num_gpus=1, use_bf16=True, optimizer="momentum",
                  data_format="NHWC", variable_update="kungfu")
b = BenchmarkCNN(p); b.build()
for _ in range(3):
    b.train_step()
torch.cuda.synchronize()
names = {v: k for k, v in conv_hip.IG_ALGOS.items()}
for key, algo in sorted(conv_hip._ig_tuned.items(), key=lambda kv: str(kv[0][9:])):
    geo = key[9:]
    flags = "stats=%d mask=%d xbn=%d add=%d mcoef=%d bias=%d fl=%d" % tuple(int(x) for x in key[2:9])
    print("N%d H%d W%d C%d OH%d OW%d K%dx%d s%d ncol%d ys%d" % (geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[12], geo[15]), flags, "->", names.get(algo, algo))
