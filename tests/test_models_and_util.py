"""Model zoo shapes / parameter counts (CPU, meta materialization), the
layer DSL, and cnn_util concurrency helpers (tcb/cnn_util_test.py)."""

import threading
import time

import numpy as np
import pytest
import torch

from kf_benchmarks_amd import cnn_util, datasets, params as P
from kf_benchmarks_amd.models import model_config
from kf_benchmarks_amd.models.model import Network

# name, dataset, expected params (millions, 1001/11 classes), tolerance
ZOO = [("resnet50", "imagenet", 25.56), ("resnet50_v1.5", "imagenet", 25.56),
       ("resnet50_v2", "imagenet", 25.54), ("resnet101", "imagenet", 44.55),
       ("resnet152", "imagenet", 60.19), ("vgg11", "imagenet", 132.87),
       ("vgg16", "imagenet", 138.36), ("vgg19", "imagenet", 143.67),
       ("alexnet", "imagenet", 61.84), ("googlenet", "imagenet", 7.00),
       ("inception3", "imagenet", 23.82), ("inception4", "imagenet", 42.65),
       ("overfeat", "imagenet", 145.92), ("lenet", "imagenet", 2.17),
       ("trivial", "imagenet", 4.26), ("resnet20", "cifar10", 0.27),
       ("resnet110_v2", "cifar10", 1.73), ("densenet40_k12", "cifar10", 1.02),
       ("alexnet", "cifar10", 1.76)]


@pytest.mark.parametrize("name,ds,mparams", ZOO, ids=["%s-%s" % (a, b) for a, b, _ in ZOO])
def test_model_builds_with_expected_params(name, ds, mparams):
    d = datasets.create_dataset(None, ds)
    m = model_config.get_model_config(name, d, P.make_params(model=name, data_name=ds))
    net = Network(m, d.num_classes, "cpu")
    assert net.num_params() / 1e6 == pytest.approx(mparams, abs=0.01)


@pytest.mark.parametrize("name", ["resnet50", "inception3", "googlenet"])
def test_forward_backward_cpu_small_batch(name):
    d = datasets.create_dataset(None, "imagenet")
    m = model_config.get_model_config(name, d, P.make_params(model=name))
    net = Network(m, d.num_classes, "cpu")
    m.set_batch_size(1)
    x = torch.randn(1, m.image_size, m.image_size, 3)
    res = net(x, phase_train=True)
    assert tuple(res.logits.shape) == (1, 1001)
    loss = m.loss_function((x, torch.tensor([3])), res)
    loss.backward()
    grads = [p.grad for _, p in net.trainable_variables()]
    assert all(g is not None for g in grads)


def test_inception3_aux_head():
    from kf_benchmarks_amd.models.inception_model import Inceptionv3Model
    m = Inceptionv3Model(P.make_params(model="inception3"), auxiliary=True)
    net = Network(m, 1001, "cpu")
    x = torch.randn(2, 299, 299, 3)
    res = net(x, phase_train=True)
    assert res.extra_info is not None and tuple(res.extra_info.shape) == (2, 1001)


def test_checkpoint_variable_names_follow_reference_layout():
    d = datasets.create_dataset(None, "imagenet")
    m = model_config.get_model_config("resnet50", d, P.make_params(model="resnet50"))
    names = set(Network(m, 1001, "cpu").tf_variables())
    assert "v0/cg/conv0/conv2d/kernel" in names
    assert "v0/cg/conv0/batchnorm0/gamma" in names
    assert "v0/cg/resnet_v10/conv1/conv2d/kernel" in names
    assert "v0/cg/affine0/weights" in names
    k = Network(m, 1001, "cpu").tf_variables()["v0/cg/conv0/conv2d/kernel"]
    assert tuple(k.shape) == (7, 7, 3, 64)  # TF [KH, KW, Cin, Cout]


def test_unknown_model_raises():
    d = datasets.create_dataset(None, "imagenet")
    with pytest.raises(ValueError):
        model_config.get_model_config("no_such_model", d, P.make_params())


def test_register_model():
    model_config.register_model("my_trivial_x", "imagenet",
                                model_config._IMAGENET["trivial"])
    with pytest.raises(ValueError):
        model_config.register_model("my_trivial_x", "imagenet", model_config._IMAGENET["trivial"])


def test_roll_numpy_batches():
    a = np.arange(8)
    np.testing.assert_array_equal(cnn_util.roll_numpy_batches(a, 2, 0.5), [4, 5, 6, 7, 0, 1, 2, 3])
    np.testing.assert_array_equal(cnn_util.roll_numpy_batches(a, 2, 0.0), a)


def test_barrier_orders_threads():
    """20 threads x 5 rounds: nobody starts round r+1 before all finished round r."""
    n, rounds = 20, 5
    bar = cnn_util.Barrier(n)
    done = [[False] * n for _ in range(rounds)]
    bad = []

    def worker(i):
        for r in range(rounds):
            done[r][i] = True
            bar.wait()
            if not all(done[r]):
                bad.append((i, r))
            bar.wait()

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert not bad


def test_barrier_abort_releases_waiters():
    bar = cnn_util.Barrier(3)
    released = []

    def w():
        bar.wait()
        released.append(1)

    ts = [threading.Thread(target=w) for _ in range(2)]
    for t in ts:
        t.start()
    time.sleep(0.1)
    bar.abort()
    for t in ts:
        t.join(5)
    assert len(released) == 2


def test_image_producer_back_pressure():
    produced = []
    prod = cnn_util.ImageProducer(lambda: produced.append(1), batch_group_size=2)
    prod.start()
    time.sleep(0.2)
    assert len(produced) <= 4  # at most 2 groups ahead of an idle consumer
    for _ in range(4):
        prod.notify_image_consumption()
    time.sleep(0.2)
    assert len(produced) >= 6
    prod.done()
