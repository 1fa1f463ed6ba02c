"""Learnability of the bf16 HIP training path: a CIFAR ResNet (BN, convs,
residual adds, fused epilogues, momentum step - all HIP kernels) memorises
a fixed batch of 64 random images, tracking the CPU fp32 run of the same
network, weights and data (role of tcb/benchmark_cnn_test.py's train ->
eval runs asserting top-1 = 1.0, tcb/test_util.py:202-299).

Random-init bf16 gradients of deep nets are chaotic step by step
(profiles/r1_grad_conditioning.txt), so the check is on the trajectory:
both runs must drive the loss below 0.1, and the bf16 curve must stay within
a band of the fp32 one while it descends."""

import numpy as np
import pytest
import torch

from kf_benchmarks_amd import benchmark

pytestmark = pytest.mark.gpu

STEPS = 60


def _curve(device, use_bf16):
    params = benchmark.make_params(model="resnet20", data_name="cifar10", batch_size=64,
                                   device=device, use_bf16=use_bf16, data_format="NHWC",
                                   optimizer="momentum", init_learning_rate=0.05,
                                   weight_decay=0.0, num_warmup_batches=0,
                                   num_batches=STEPS, tf_random_seed=1234)
    b = benchmark.BenchmarkCNN(params)
    rng = np.random.default_rng(0)
    imgs = rng.uniform(0, 255, size=(64, 32, 32, 3)).astype(np.float32)
    labels = rng.integers(0, 10, size=(64,))
    b.set_fake_data(imgs, labels)
    b.build()
    out = []
    for _ in range(STEPS):
        loss, _ = b.train_step(need_loss=True)
        out.append(float(loss))
    return np.array(out)


def test_bf16_hip_memorises_fixed_batch(cuda):
    gpu = _curve("gpu", True)
    cpu = _curve("cpu", False)
    assert np.isfinite(gpu).all() and np.isfinite(cpu).all()
    assert cpu[-10:].mean() < 0.1, cpu[::10]
    assert gpu[-10:].mean() < 0.1, gpu[::10]
    # same starting point (same weights, data), and the descent tracks fp32
    assert abs(gpu[0] - cpu[0]) < 0.05 * abs(cpu[0])
    first_below = lambda c, t: int(np.argmax(c < t)) if (c < t).any() else len(c)  # noqa: E731
    assert abs(first_below(gpu, 0.5) - first_below(cpu, 0.5)) <= 10
