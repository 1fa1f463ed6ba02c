"""One rank of the 2-rank GPU rehearsal (tests/test_dist_gpu.py): a real
model stepping through the HIP kernels with bucketed all-reduce hooks
overlapped with backward.  Both ranks share the box's one GPU, so the
process group is gloo over CUDA tensors (KFB_DIST_BACKEND=gloo); the
collective call sequence is the one RCCL runs on an 8-GPU node.

usage: dist_gpu_worker.py <out.json> '<json flag kwargs>' <steps>"""

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    out, kw, steps = sys.argv[1], json.loads(sys.argv[2]), int(sys.argv[3])
    import torch
    from kf_benchmarks_amd import params as P
    from kf_benchmarks_amd.benchmark import BenchmarkCNN
    from kf_benchmarks_amd.parallel import comm
    p = P.make_params(**kw)
    bench = BenchmarkCNN(p)
    bench.build()
    bench.strategy.broadcast_initial_model(bench.optimizer.slot_tensors().values())
    w0 = bench.flat.flat.detach().double().sum().item()
    losses = []
    for _ in range(steps):
        loss, _ = bench.train_step(need_loss=True)
        losses.append(float(loss))
    torch.cuda.synchronize()
    flat = bench.flat.flat.detach()
    res = {"losses": losses, "w0": w0, "wsum": flat.double().sum().item(),
           "wabs": flat.double().abs().sum().item(), "head": flat[:64].cpu().tolist(),
           "tail": flat[-64:].cpu().tolist(), "rank": comm.get_world().rank,
           "size": comm.get_world().size}
    with open(out, "w") as f:
        json.dump(res, f)
    comm.get_world().shutdown()


if __name__ == "__main__":
    main()
