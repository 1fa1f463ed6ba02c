#!/usr/bin/env python3
"""Diagnostic: one ResNet training step with the BN finalize in the conv's
last workgroup vs the BN's own finalize launch; prints the BN layers whose
running statistics / statistics shift / finalize outputs differ."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd import params as P  # noqa: E402
from kf_benchmarks_amd.benchmark import BenchmarkCNN  # noqa: E402
from kf_benchmarks_amd.ops import conv_hip  # noqa: E402


def run(fin, steps, model, bs):
    conv_hip._BN_FIN = fin
    p = P.make_params(model=model, batch_size=bs, num_gpus=1, use_bf16=True,
                      optimizer="momentum", data_format="NHWC", variable_update="kungfu",
                      init_learning_rate=0.002, display_every=10 ** 9)
    b = BenchmarkCNN(p)
    b.build()
    losses = [float(b.train_step(need_loss=True)[0]) for _ in range(steps)]
    torch.cuda.synchronize()
    bufs = {k: t.detach().float().cpu().clone() for k, t in b.net.named_buffers()}
    return losses, bufs


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    for steps in (1, 2):
        la, ba = run(True, steps, model, bs)
        lb, bb = run(False, steps, model, bs)
        print("steps %d losses fin %s nofin %s" % (steps, la, lb))
        bad = []
        for k in bb:
            if k.endswith(("fin_st", "fin_coef")):
                continue
            d = (ba[k] - bb[k]).abs().max().item()
            if d > 1e-3 * max(1.0, bb[k].abs().max().item()):
                bad.append((k, d))
        print("  %d differing buffers; first: %s" % (len(bad), bad[:6]))


if __name__ == "__main__":
    main()
