"""Diagnosis: MobileNet-v2 (bf16, 64 px, batch 4) gradients - ReLU6 in the BN
vs a separate pass, each twice, with and without the weight-gradient side
stream; prints the worst per-tensor relative differences of each pair."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from kf_benchmarks_amd import datasets, params as P  # noqa: E402
from kf_benchmarks_amd.models import model_config  # noqa: E402
from kf_benchmarks_amd.models.model import make_network  # noqa: E402
from kf_benchmarks_amd.ops import conv_hip, nn as nn_ops  # noqa: E402

dev = torch.device("cuda", 0)


def run():
    d = datasets.create_dataset(None, "imagenet")
    m = model_config.get_model_config("mobilenet", d, P.make_params(model="mobilenet"))
    m.image_size = 64
    torch.manual_seed(0)
    net = make_network(m, d.num_classes, str(dev), torch.bfloat16)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 64, 64, 3, generator=g).to(dev, torch.bfloat16)
    lab = torch.randint(0, d.num_classes - 1, (4,), generator=g).to(dev)
    loss = m.loss_function((x, lab), net(x))
    loss.backward()
    torch.cuda.synchronize()
    names = [n for n, p in net.trainable_variables() if p.grad is not None]
    return float(loss), names, [p.grad.float().cpu().reshape(-1) for _, p in net.trainable_variables()
                                if p.grad is not None]


def cmp(tag, a, b):
    (la, names, ga), (lb, _, gb) = a, b
    rows = sorted(((float((x - y).norm()) / max(float(y.norm()), 1e-12), n, float(y.norm()))
                   for n, x, y in zip(names, ga, gb)), reverse=True)[:5]
    print("%-28s loss %s | worst rel diffs: %s" % (tag, la == lb, ["%s %.3g (|g| %.3g)" % (n[-40:], r, nm) for r, n, nm in rows]), flush=True)


if __name__ != "__main__":
    pass
elif len(sys.argv) > 1 and sys.argv[1] == "after_nasnet":
    # the state the pytest order left: the NASNet exact-oracle runs first
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))), "tests"))
    from kf_benchmarks_amd.ops import _native as N
    import test_tape_gpu as T
    conv_hip._NO_S3 = True
    conv_hip._AUTOTUNE = False
    N.load().kfb_set_deterministic(1)
    T._run_exact_nasnet(False)
    N.load().kfb_set_deterministic(0)
    conv_hip._NO_S3 = False
    conv_hip._AUTOTUNE = True
    print("ran the NASNet exact run first", flush=True)
    f0 = run()
    nn_ops._RELU6_IN_BN = False
    u0 = run()
    nn_ops._RELU6_IN_BN = True
    cmp("after nasnet: fused vs unfused", f0, u0)
    f1 = run()
    cmp("after nasnet: fused vs fused(2nd)", f0, f1)
    sys.exit(0)

for side in ((True, False) if __name__ == "__main__" else ()):
    conv_hip._WGRAD_SIDE = side
    nn_ops._RELU6_IN_BN = True
    f1 = run()
    f2 = run()
    nn_ops._RELU6_IN_BN = False
    u1 = run()
    u2 = run()
    cmp("side=%s fused vs fused" % side, f1, f2)
    cmp("side=%s unfused vs unfused" % side, u1, u2)
    cmp("side=%s fused vs unfused" % side, f1, u1)
