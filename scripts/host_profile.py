#!/usr/bin/env python3
"""Host-side (Python) cost of the training step: cProfile over K steps of
the 1-GPU ResNet-50 bench configuration after warmup.  The GPU runs
asynchronously, so this is the launch path's CPU time per step; where it
exceeds the GPU time of a phase the GPU idles (the wall-vs-busy gap of
scripts/kernel_stats.py --last-steps).

usage: host_profile.py [--steps K] [--top N]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch_size", type=int, default=256)
    a = ap.parse_args()
    import torch
    from kf_benchmarks_amd import params as P
    from kf_benchmarks_amd.benchmark import BenchmarkCNN
    p = P.make_params(model=a.model, batch_size=a.batch_size, num_gpus=1, use_bf16=True,
                      optimizer="momentum", data_format="NHWC", variable_update="kungfu")
    bench = BenchmarkCNN(p)
    bench.build()
    for _ in range(5):
        bench.train_step()
    torch.cuda.synchronize()
    # host time of forward vs backward vs update, GPU drained before each
    t = {"fwd": 0.0, "bwd": 0.0}
    orig = bench.forward_backward

    def fb(inputs, need_accuracy=False):
        t0 = time.perf_counter()
        res = bench.net.forward_inputs(inputs, phase_train=True)
        loss = bench.model.loss_function(inputs, res)
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        t["fwd"] += t1 - t0
        t["bwd"] += t2 - t1
        return loss.detach(), None
    bench.forward_backward = fb
    pr = cProfile.Profile()
    w0 = time.perf_counter()
    pr.enable()
    for _ in range(a.steps):
        bench.train_step()
    pr.disable()
    host = time.perf_counter() - w0
    torch.cuda.synchronize()
    wall = time.perf_counter() - w0
    print("host %.2f ms/step (fwd %.2f, bwd %.2f), wall %.2f ms/step (profiled)"
          % (1e3 * host / a.steps, 1e3 * t["fwd"] / a.steps, 1e3 * t["bwd"] / a.steps,
             1e3 * wall / a.steps))
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
    print(s.getvalue())
    bench.forward_backward = orig


if __name__ == "__main__":
    main()
