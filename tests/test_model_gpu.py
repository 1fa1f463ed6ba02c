"""Whole-network numerics on the GPU path (every fused kernel: conv + BN
statistics epilogue, dgrad + producer-BN ReLU/partials epilogue, direct
gradient sinks, fused optimizer) against the fp32 CPU reference of the same
network, weights and inputs."""

import pytest
import torch

from kf_benchmarks_amd import datasets, optim, params as P
from kf_benchmarks_amd.models import model_config
from kf_benchmarks_amd.models.model import Network

pytestmark = pytest.mark.gpu


def _grads(name, ds, dev, dtype, image_size=None, batch=4, seed=3):
    d = datasets.create_dataset(None, ds)
    m = model_config.get_model_config(name, d, P.make_params(model=name, data_name=ds))
    if image_size:
        m.image_size = image_size
    net = Network(m, d.num_classes, dev, dtype, seed=7)
    flat = optim.FlatParams(net, dtype if dtype != torch.float32 else None)
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(batch, m.image_size, m.image_size, 3, generator=g).to(dtype)
    y = torch.randint(0, d.num_classes - 1, (batch,), generator=g)
    flat.zero_grad()
    res = net(x.to(dev), phase_train=True)
    loss = m.loss_function((x, y.to(dev)), res)
    loss.backward()
    out = {n: p.grad.detach().float().cpu().clone() for n, p in net.trainable_variables()}
    return float(loss), out


@pytest.mark.parametrize("name,ds,size", [("resnet20", "cifar10", None),
                                          ("resnet50", "imagenet", 64),
                                          ("resnet50_v1.5", "imagenet", 64),
                                          ("resnet50_v2", "imagenet", 64),
                                          ("googlenet", "imagenet", 64)])
def test_network_grads_match_cpu(cuda, name, ds, size):
    loss_ref, g_ref = _grads(name, ds, "cpu", torch.float32, size)
    loss_gpu, g_gpu = _grads(name, ds, cuda, torch.bfloat16, size)
    assert abs(loss_gpu - loss_ref) < 0.05 * max(1.0, abs(loss_ref))
    bad = []
    for k, ref in g_ref.items():
        got = g_gpu[k]
        rel = (got - ref).norm() / (ref.norm() + 1e-12)
        if rel > 0.12:
            bad.append((k, float(rel)))
    assert not bad, bad[:10]
