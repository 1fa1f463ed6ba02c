#!/usr/bin/env python3
"""Which PyTorch (non-kfb) ops run inside one ResNet-50 training step, and
from where: torch.profiler with Python stacks over a few steps, printing the
aten ops that launch device work grouped by their nearest framework frame."""

import collections
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd import params as P  # noqa: E402
from kf_benchmarks_amd.benchmark import BenchmarkCNN  # noqa: E402


def main():
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    p = P.make_params(model="resnet50", batch_size=bs, num_gpus=1, use_bf16=True,
                      optimizer="momentum", data_format="NHWC", variable_update="kungfu")
    bench = BenchmarkCNN(p)
    bench.build()
    for _ in range(3):
        bench.train_step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True) as prof:
        for _ in range(2):
            bench.train_step()
        torch.cuda.synchronize()
    groups = collections.Counter()
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.device_type != torch.autograd.DeviceType.CPU:
            continue
        if ev.name in ("aten::empty", "aten::empty_strided", "aten::view", "aten::reshape",
                       "aten::as_strided", "aten::slice", "aten::select", "aten::detach",
                       "aten::_reshape_alias", "aten::alias", "aten::t", "aten::transpose",
                       "aten::permute", "aten::expand", "aten::unsqueeze", "aten::squeeze",
                       "aten::lift_fresh", "aten::result_type", "aten::is_nonzero",
                       "aten::item", "aten::_local_scalar_dense", "aten::resolve_conj",
                       "aten::resolve_neg", "aten::split", "aten::tensor_split", "aten::narrow"):
            continue
        frame = next((f for f in ev.stack if "kf_benchmarks_amd" in f and "torch/" not in f),
                     ev.stack[0] if ev.stack else "?")
        groups[(ev.name, frame)] += 1
    print("calls/step  op  <- frame")
    for (name, frame), n in groups.most_common(60):
        print("%6.1f  %-28s %s" % (n / 2, name, frame))
    # device kernels of the two steady-state steps
    kern = collections.defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA:
            k = kern[ev.name[:90]]
            k[0] += 1
            k[1] += ev.device_time
    tot = sum(v[1] for v in kern.values())
    print("\ndevice time per step: %.2f ms" % (tot / 2 / 1000))
    print("%-90s %8s %10s" % ("kernel", "calls/st", "us/step"))
    for name, (n, t) in sorted(kern.items(), key=lambda kv: -kv[1][1])[:60]:
        print("%-90s %8.1f %10.1f" % (name, n / 2, t / 2))


if __name__ == "__main__":
    main()
