"""Probe: eager ResNet-50 bs256 training step vs the same step captured in a
HIP graph and replayed (constant LR / fixed synthetic seed inside the graph;
measurement only, not the product path)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from kf_benchmarks_amd import params as P  # noqa: E402
from kf_benchmarks_amd.benchmark import BenchmarkCNN  # noqa: E402


def timeit(fn, n):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    p = P.make_params(model="resnet50", batch_size=bs, num_gpus=1, use_bf16=True,
                      optimizer="momentum", data_format="NHWC", variable_update="kungfu",
                      init_learning_rate=0.1, display_every=10 ** 9)
    b = BenchmarkCNN(p)
    b.build()
    for _ in range(10):
        b.train_step()
    eager = timeit(lambda: b.train_step(), 20)
    print("eager  %.3f ms/step" % eager, flush=True)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            b.train_step()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        b.train_step()
    g.replay()
    torch.cuda.synchronize()
    graph = timeit(g.replay, 20)
    print("graph  %.3f ms/step  (%.1f%% faster)" % (graph, 100 * (eager / graph - 1)), flush=True)


if __name__ == "__main__":
    main()
