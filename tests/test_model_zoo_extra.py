"""MobileNet-v2, official ResNets and NASNet: parameter counts against the
published architectures and a CPU forward/backward."""

import pytest
import torch

from kf_benchmarks_amd import datasets, params as P
from kf_benchmarks_amd.models import model_config
from kf_benchmarks_amd.models.model import make_network


def _net(name, ds="imagenet", size=None):
    d = datasets.create_dataset(None, ds)
    m = model_config.get_model_config(name, d, P.make_params(model=name))
    if size:
        m.image_size = size
    return d, m, make_network(m, d.num_classes, "cpu", torch.float32)


# published parameter counts (+ the CNNModel's final 1001/11-way affine)
@pytest.mark.parametrize("name,ds,expected", [
    ("mobilenet", "imagenet", 3.504e6 + 1001 * 1001 + 1001),
    ("official_resnet18", "imagenet", 11.69e6), ("official_resnet34", "imagenet", 21.80e6),
    ("official_resnet50", "imagenet", 25.56e6), ("official_resnet101_v2", "imagenet", 44.55e6),
    ("nasnet", "imagenet", 5.29e6), ("nasnet", "cifar10", 3.35e6)])
def test_param_counts(name, ds, expected):
    _, _, net = _net(name, ds)
    assert abs(net.num_params() - expected) / expected < 0.02, net.num_params()


@pytest.mark.parametrize("name,ds,size", [("mobilenet", "imagenet", 64),
                                          ("official_resnet18_v2", "imagenet", 64),
                                          ("nasnet", "cifar10", None)])
def test_forward_backward(name, ds, size):
    d, m, net = _net(name, ds, size)
    x = torch.randn(2, m.image_size, m.image_size, 3)
    y = torch.randint(0, d.num_classes - 1, (2,))
    res = net(x)
    loss = m.loss_function((x, y), res)
    loss.backward()
    assert torch.isfinite(loss)
    grads = [p.grad for _, p in net.trainable_variables()]
    assert all(g is not None and torch.isfinite(g).all() for g in grads)


def test_mobilenet_block_structure():
    _, _, net = _net("mobilenet")
    names = [n for n, _ in net.trainable_variables()]
    assert sum("depthwise_weights" in n for n in names) == 17
    # first block has no expansion conv; later ones do
    assert not any(n.startswith("MobilenetV2/expanded_conv/expand") for n in names)
    assert any(n.startswith("MobilenetV2/expanded_conv_1/expand") for n in names)
