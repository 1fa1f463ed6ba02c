"""Numerics of the gfx950 kernels against plain PyTorch fp32 references.

Every test runs the op on cuda:0 through libkfb_hip.so and the same op on
CPU in fp32 (stock PyTorch), for forward and backward.
"""

import os

import pytest
import torch

from kf_benchmarks_amd.ops import nn as F

pytestmark = pytest.mark.gpu

DT = [torch.float32, torch.bfloat16]


def tol(dt):
    return dict(rtol=2e-2, atol=2e-2) if dt == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)


def _pair(x, dev, dt):
    # the fp32 reference sees the same (rounded) input values as the kernel
    a = x.clone().to(dev, dt).requires_grad_(True)
    b = x.clone().to(dt).float().requires_grad_(True)
    return a, b


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("shape", [(4, 7, 7, 64), (2, 5, 6, 24), (3, 4, 4, 2048), (2, 3, 3, 20),
                                   # > 4 x the capped grid: the unrolled streaming loop + tail
                                   (81, 32, 32, 256),
                                   # >= 64 MB: the flat passes
                                   (64, 64, 64, 256)])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
def test_batch_norm_train(cuda, dt, shape, relu, res):
    if relu and shape[0] * shape[1] * shape[2] * shape[3] > (1 << 24):
        # 6.7e7 outputs: a handful sit within rounding of 0, where the
        # kernel's ReLU gate (on its own output) and the fp32 reference's
        # disagree by a full gradient element (and its dgamma term); the
        # flat passes with the gate are covered by test_batch_norm_relu6
        pytest.skip("ReLU gate ambiguity at 6.7e7 elements")
    torch.manual_seed(0)
    C = shape[-1]
    x = torch.randn(shape) * 2 + 0.5
    r = torch.randn(shape)
    g0 = torch.rand(C) + 0.5
    b0 = torch.randn(C)
    xa, xb = _pair(x, cuda, dt)
    ra, rb = (_pair(r, cuda, dt) if res else (None, None))
    ga, gb = g0.clone().to(cuda).requires_grad_(True), g0.clone().requires_grad_(True)
    ba, bb = b0.clone().to(cuda).requires_grad_(True), b0.clone().requires_grad_(True)
    rma, rva = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    rmb, rvb = torch.zeros(C), torch.ones(C)
    ya = F.batch_norm(xa, ga, ba, rma, rva, 0.9, 1e-5, True, relu, ra)
    yb = F.batch_norm(xb, gb, bb, rmb, rvb, 0.9, 1e-5, True, relu, rb)
    torch.testing.assert_close(ya.float().cpu(), yb, **tol(dt))
    torch.testing.assert_close(rma.cpu(), rmb, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(rva.cpu(), rvb, rtol=1e-3, atol=1e-3)
    dy = torch.randn(shape).to(dt).float()  # both sides see the same rounded gradient
    ya.backward(dy.to(cuda, dt))
    yb.backward(dy)
    t = tol(dt)
    # bf16 output rounding: ~1 ulp of |dx| up to ~8 over 2e7 elements
    torch.testing.assert_close(xa.grad.float().cpu(), xb.grad, rtol=t["rtol"] * 4, atol=t["atol"] * 4)
    torch.testing.assert_close(ga.grad.cpu(), gb.grad, rtol=5e-2 if dt != torch.float32 else 1e-3,
                               atol=0.5 if dt != torch.float32 else 1e-3)
    torch.testing.assert_close(ba.grad.cpu(), bb.grad, rtol=5e-2 if dt != torch.float32 else 1e-3,
                               atol=0.5 if dt != torch.float32 else 1e-3)
    if res:
        # the residual gradient is dy masked by the kernel's own output: a
        # y within bf16 rounding of 0 may fall on either side of the fp32 mask
        exp = dy * (ya.detach().float().cpu() > 0) if relu else dy
        torch.testing.assert_close(ra.grad.float().cpu(), exp, **tol(dt))
        assert (ra.grad.float().cpu() - rb.grad).abs().gt(0.05).float().mean() < 1e-5


@pytest.mark.parametrize("shape", [(4, 7, 7, 64), (2, 5, 6, 24), (3, 4, 4, 2048),
                                   (128, 64, 64, 256)])  # last: >= 256 MB, the flat passes
def test_batch_norm_relu6(cuda, shape):
    """BN + ReLU6 in one apply pass (MobileNet-v2; csrc/bn.hip act_apply /
    act_pass): y = min(max(bn(x), 0), 6), its bit mask, and the backward
    gated by 0 < y < 6 on the stored output - against an fp32 reference that
    uses the kernel's own output for the gate (bf16 rounding puts values
    within an ulp of 6 on either side)."""
    torch.manual_seed(0)
    dt = torch.bfloat16
    C = shape[-1]
    x = (torch.randn(shape) * 2 + 0.5).to(dt).float()
    g0 = torch.rand(C) + 0.5
    b0 = torch.randn(C) * 2 + 4  # a good share of the outputs above 6
    xa = x.to(cuda, dt).requires_grad_(True)
    ga = g0.clone().to(cuda).requires_grad_(True)
    ba = b0.clone().to(cuda).requires_grad_(True)
    rma, rva = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    ya = F.batch_norm(xa, ga, ba, rma, rva, 0.9, 1e-5, True, 2, None)
    xf = x.view(-1, C)
    mean, var = xf.mean(0), xf.var(0, unbiased=False)
    xhat = (xf - mean) / torch.sqrt(var + 1e-5)
    yref = (xhat * g0 + b0).clamp(0.0, 6.0).view(shape)
    y = ya.detach().float().cpu()
    torch.testing.assert_close(y, yref, rtol=2e-2, atol=4e-2)
    assert (y >= 6).float().mean() > 0.05 and (y <= 0).float().mean() > 0.01
    gate = (y > 0) & (y < 6)
    mb = ya._kfb_bn_link.mbits
    assert mb is not None
    bits = torch.stack([(mb.cpu() >> k) & 1 for k in range(8)], -1).view(shape).bool()
    assert torch.equal(bits, gate)
    dy = torch.randn(shape).to(dt).float()
    ya.backward(dy.to(cuda, dt))
    n = xf.shape[0]
    dyp = (dy * gate).view(-1, C)
    dbeta = dyp.sum(0)
    dgamma = (dyp * xhat).sum(0)
    dx = (g0 / torch.sqrt(var + 1e-5)) * (dyp - dbeta / n - xhat * dgamma / n)
    torch.testing.assert_close(xa.grad.float().cpu(), dx.view(shape), rtol=8e-2, atol=8e-2)
    torch.testing.assert_close(ba.grad.cpu(), dbeta, rtol=1e-2, atol=0.5)
    torch.testing.assert_close(ga.grad.cpu(), dgamma, rtol=1e-2, atol=0.5)


def test_mobilenet_relu6_in_bn_matches_separate_pass(cuda, monkeypatch):
    """MobileNet-v2 (bf16, 64 px, batch 4): with ReLU6 applied by the BN
    (default) the loss is bitwise the separate-pass loss (clamping commutes
    with rounding) and the gradients agree to fp32 summation order."""
    from kf_benchmarks_amd import datasets, params as P
    from kf_benchmarks_amd.models import model_config
    from kf_benchmarks_amd.models.model import make_network
    from kf_benchmarks_amd.ops import nn as nn_ops

    def run():
        d = datasets.create_dataset(None, "imagenet")
        m = model_config.get_model_config("mobilenet", d, P.make_params(model="mobilenet"))
        m.image_size = 64
        torch.manual_seed(0)
        net = make_network(m, d.num_classes, str(cuda), torch.bfloat16)
        g = torch.Generator().manual_seed(3)
        x = torch.randn(4, 64, 64, 3, generator=g).to(cuda, torch.bfloat16)
        lab = torch.randint(0, d.num_classes - 1, (4,), generator=g).to(cuda)
        loss = m.loss_function((x, lab), net(x))
        loss.backward()
        return float(loss), [p.grad.float().cpu().reshape(-1) for _, p in net.trainable_variables()
                             if p.grad is not None]

    la, ga = run()
    monkeypatch.setattr(nn_ops, "_RELU6_IN_BN", False)
    lb, gb = run()
    assert la == lb, (la, lb)
    # the two backwards differ in fp32 summation order only (BN partial sums
    # in the consumer's dgrad epilogue vs a separate pass), so every gradient
    # tensor agrees to ~1e-3 of its own norm or, for the near-cancelling ones
    # (a BN beta whose true gradient is ~0), of the typical gradient norm
    norms = sorted(float(b.norm()) for b in gb)
    floor = 1e-3 * norms[len(norms) // 2]
    bad = [(i, float((a - b).norm()), float(b.norm())) for i, (a, b) in enumerate(zip(ga, gb))
           if float((a - b).norm()) > 2e-2 * float(b.norm()) + floor]
    assert not bad, bad[:8]
    allc = float(torch.nn.functional.cosine_similarity(torch.cat(ga), torch.cat(gb), dim=0))
    assert allc > 0.9999, allc


@pytest.mark.parametrize("dt", DT)
def test_batch_norm_infer(cuda, dt):
    C = 32
    x = torch.randn(2, 5, 5, C)
    g, b, rm, rv = torch.rand(C) + 0.5, torch.randn(C), torch.randn(C), torch.rand(C) + 0.5
    ya = F.batch_norm(x.to(cuda, dt), g.to(cuda), b.to(cuda), rm.to(cuda), rv.to(cuda), 0.9,
                      1e-3, False, True)
    yb = F.batch_norm(x, g, b, rm.clone(), rv.clone(), 0.9, 1e-3, False, True)
    torch.testing.assert_close(ya.float().cpu(), yb, **tol(dt))


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("kind,k,s,mode,hw", [("max", 3, 2, "SAME", 16), ("max", 2, 2, "VALID", 8),
                                              ("avg", 3, 1, "SAME", 9), ("avg", 3, 2, "VALID", 9),
                                              ("max", 3, 2, "VALID", 13)])
def test_pool(cuda, dt, kind, k, s, mode, hw):
    torch.manual_seed(1)
    x = torch.randn(2, hw, hw, 16)
    xa, xb = _pair(x, cuda, dt)
    fn = F.max_pool if kind == "max" else F.avg_pool
    ya, yb = fn(xa, k, k, s, s, mode), fn(xb, k, k, s, s, mode)
    torch.testing.assert_close(ya.float().cpu(), yb, **tol(dt))
    dy = torch.randn(yb.shape)
    ya.backward(dy.to(cuda, dt))
    yb.backward(dy)
    torch.testing.assert_close(xa.grad.float().cpu(), xb.grad, **tol(dt))


@pytest.mark.parametrize("dt", DT)
def test_spatial_mean(cuda, dt):
    x = torch.randn(3, 7, 7, 256)
    xa, xb = _pair(x, cuda, dt)
    ya, yb = F.spatial_mean(xa), F.spatial_mean(xb)
    torch.testing.assert_close(ya.float().cpu(), yb, **tol(dt))
    dy = torch.randn(yb.shape)
    ya.backward(dy.to(cuda, dt))
    yb.backward(dy)
    torch.testing.assert_close(xa.grad.float().cpu(), xb.grad, **tol(dt))


@pytest.mark.parametrize("dt", DT)
def test_softmax_xent_and_topk(cuda, dt):
    torch.manual_seed(2)
    logits = torch.randn(16, 1001) * 3
    labels = torch.randint(0, 1000, (16,), dtype=torch.int32)
    la, lb = _pair(logits, cuda, dt)
    a = F.softmax_cross_entropy(la, labels.to(cuda))
    b = F.softmax_cross_entropy(lb, labels)
    torch.testing.assert_close(a.cpu(), b, rtol=1e-2 if dt != torch.float32 else 1e-5, atol=1e-2)
    (a * 2).backward()
    (b * 2).backward()
    torch.testing.assert_close(la.grad.float().cpu(), lb.grad, rtol=2e-2, atol=1e-3)
    t1a, t5a = F.in_top_k(la.detach().float(), labels.to(cuda))
    t1b, t5b = F.in_top_k(lb.detach(), labels)
    assert float(t1a) == float(t1b) and float(t5a) == float(t5b)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("relu", [False, True])
def test_bias_act(cuda, dt, relu):
    x = torch.randn(4, 6, 6, 40)
    bias = torch.randn(40)
    xa, xb = _pair(x, cuda, dt)
    ba, bb = bias.clone().to(cuda).requires_grad_(True), bias.clone().requires_grad_(True)
    ya, yb = F.bias_act(xa, ba, relu), F.bias_act(xb, bb, relu)
    torch.testing.assert_close(ya.float().cpu(), yb, **tol(dt))
    dy = torch.randn(yb.shape)
    ya.backward(dy.to(cuda, dt))
    yb.backward(dy)
    torch.testing.assert_close(xa.grad.float().cpu(), xb.grad, **tol(dt))
    torch.testing.assert_close(ba.grad.cpu(), bb.grad, rtol=2e-2, atol=0.2 if dt != torch.float32 else 1e-3)


@pytest.mark.parametrize("relu", [False, True])
def test_add(cuda, relu):
    a, b = torch.randn(3, 4, 4, 8), torch.randn(3, 4, 4, 8)
    aa, ab = _pair(a, cuda, torch.float32)
    ba, bb = _pair(b, cuda, torch.float32)
    ya, yb = F.add(aa, ba, relu), F.add(ab, bb, relu)
    torch.testing.assert_close(ya.cpu(), yb)
    dy = torch.randn(yb.shape)
    ya.backward(dy.to(cuda))
    yb.backward(dy)
    torch.testing.assert_close(aa.grad.cpu(), ab.grad)
    torch.testing.assert_close(ba.grad.cpu(), bb.grad)


def test_dropout_statistics(cuda):
    x = torch.ones(1 << 20, device=cuda)
    y = F.dropout(x, 0.5, True, seed=123)
    keep = (y > 0).float().mean().item()
    assert abs(keep - 0.5) < 0.01
    assert torch.allclose(y[y > 0], torch.full_like(y[y > 0], 2.0))
    x.requires_grad_(True)
    y = F.dropout(x, 0.5, True, seed=123)
    y.sum().backward()
    assert torch.equal((x.grad > 0), (y.detach() > 0))


def test_synthetic_inputs(cuda):
    img = F.synthetic_images((8, 32, 32, 3), torch.float32, cuda, 7)
    assert abs(img.mean().item() - 127) < 3
    assert img.min().item() >= 127 - 120 - 1e-3 and img.max().item() <= 127 + 120 + 1e-3
    lab = F.synthetic_labels(4096, 1001, cuda, 7)
    assert lab.min().item() >= 0 and lab.max().item() < 1000


def test_synthetic_images_truncated_normal_bf16(cuda):
    """The per-step synthetic batch (bf16, 8 values per thread, drawn by
    inverting the truncated normal's CDF): mean 127, std 60 * 0.87963 (the
    std of a normal truncated at +-2), every value within +-2 std, and the
    histogram matches the truncated normal's CDF."""
    img = F.synthetic_images((64, 64, 64, 3), torch.bfloat16, cuda, 11).float().cpu()
    z = (img.reshape(-1) - 127.0) / 60.0
    assert abs(z.mean().item()) < 5e-3
    assert abs(z.std().item() - 0.87963) < 5e-3
    assert z.min().item() >= -2.0 - 1e-2 and z.max().item() <= 2.0 + 1e-2
    from math import erf, sqrt
    norm = erf(sqrt(2.0))
    for t in (-1.5, -0.5, 0.0, 0.7, 1.9):
        want = 0.5 + 0.5 * erf(t / sqrt(2.0)) / norm
        assert abs((z <= t).float().mean().item() - want) < 1.2e-2, t  # (bf16 bins)
    again = F.synthetic_images((64, 64, 64, 3), torch.bfloat16, cuda, 11).float().cpu()
    other = F.synthetic_images((64, 64, 64, 3), torch.bfloat16, cuda, 12).float().cpu()
    assert torch.equal(img, again) and not torch.equal(img, other)


@pytest.mark.parametrize("kind", ["sgd", "momentum", "rmsprop", "adam"])
def test_fused_optimizer(cuda, kind):
    from kf_benchmarks_amd import optim
    from kf_benchmarks_amd.models.model import Network
    from kf_benchmarks_amd.models.resnet_model import create_resnet20_cifar_model

    res = {}
    for dev in ("cpu", cuda):
        model = create_resnet20_cifar_model(None)
        net = Network(model, 11, dev, torch.float32, seed=5)
        flat = optim.FlatParams(net, torch.bfloat16)
        opt = optim.FusedOptimizer(flat, kind)
        g = torch.Generator().manual_seed(3)
        for i in range(3):
            flat.grad.copy_(torch.randn(flat.numel, generator=g).to(flat.grad.device))
            opt.step(0.01, grad_scale=0.5, weight_decay=1e-3, clip=1.5)
        res[str(dev)] = (flat.flat.cpu().clone(), flat.lp.float().cpu().clone())
    a, b = res["cpu"], res[str(cuda)]
    torch.testing.assert_close(b[0], a[0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(b[1], a[1], rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_mul_forward_backward(cuda, dtype):
    """Native elementwise product (NCF's GMF layer) vs the fp32 torch formula."""
    a = torch.randn(513, 64, device=cuda).to(dtype).requires_grad_(True)
    b = torch.randn(513, 64, device=cuda).to(dtype).requires_grad_(True)
    dy = torch.randn(513, 64, device=cuda).to(dtype)
    y = F.mul(a, b)
    y.backward(dy)
    af, bf, gf = a.detach().float(), b.detach().float(), dy.float()
    tol = dict(rtol=1e-2, atol=1e-2) if dtype == torch.bfloat16 else dict(rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(y.float(), af * bf, **tol)
    torch.testing.assert_close(a.grad.float(), gf * bf, **tol)
    torch.testing.assert_close(b.grad.float(), gf * af, **tol)


def test_synthetic_ints_and_uniform(cuda):
    """Device-drawn integers / uniforms: in range, roughly uniform, the salt
    separates tensors of one seed, the seed re-draws them."""
    a = F.synthetic_ints(1 << 16, 138493, cuda, 5, 21)
    b = F.synthetic_ints(1 << 16, 138493, cuda, 5, 22)
    c = F.synthetic_ints(1 << 16, 138493, cuda, 6, 21)
    assert a.dtype == torch.int32 and int(a.min()) >= 0 and int(a.max()) < 138493
    assert abs(a.float().mean().item() / 138492 - 0.5) < 0.01
    assert not torch.equal(a, b) and not torch.equal(a, c)
    assert torch.equal(a, F.synthetic_ints(1 << 16, 138493, cuda, 5, 21))
    u = F.synthetic_uniform((4096, 4), torch.float32, cuda, 3, 14, 1.0, 10.0)
    assert float(u.min()) >= 1.0 and float(u.max()) < 10.0
    assert abs(u.mean().item() - 5.5) < 0.1


@pytest.mark.parametrize("kind", ["momentum", "adam"])
def test_fused_optimizer_decay_mask(cuda, kind):
    """Weight decay on a subset of the variables (a model's L2 filter, e.g.
    SSD without batch-norm variables) applied inside the update kernel from a
    uint8 per-element mask vs the CPU formula; masked-off elements get none."""
    from kf_benchmarks_amd import optim
    from kf_benchmarks_amd.models.model import Network
    from kf_benchmarks_amd.models.resnet_model import create_resnet20_cifar_model

    res = {}
    for dev in ("cpu", cuda):
        model = create_resnet20_cifar_model(None)
        net = Network(model, 11, dev, torch.float32, seed=5)
        flat = optim.FlatParams(net, torch.bfloat16)
        opt = optim.FusedOptimizer(flat, kind)
        mask = torch.zeros(flat.numel, dtype=torch.uint8)
        for n, _, o, k in flat.segments():
            if "batchnorm" not in n:
                mask[o:o + k] = 1
        assert 0 < int(mask.sum()) < flat.numel
        opt.decay_mask = mask.to(flat.flat.device)
        for i in range(3):
            flat.grad.zero_()
            opt.step(0.01, grad_scale=0.5, weight_decay=0.3)
        res[str(dev)] = (flat.flat.cpu().clone(), mask)
    (a, mask), (b, _) = res["cpu"], res[str(cuda)]
    torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
    net = Network(create_resnet20_cifar_model(None), 11, "cpu", torch.float32, seed=5)
    w0 = optim.FlatParams(net, torch.bfloat16).flat
    off = mask == 0
    assert torch.equal(b[off], w0[off])  # zero gradient, no decay: unchanged
    assert not torch.equal(b[~off], w0[~off])


@pytest.mark.parametrize("ok", [None, 1, 0])
def test_fused_optimizer_model_averaging(cuda, ok):
    """The averaging folded into the optimizer pass (PairAveraging / SMA):
    w <- a*w + b*src before the update, gated by a device flag, and the
    updated weights copied to ``wout``; the HIP pass vs the CPU path (the
    explicit formula)."""
    from kf_benchmarks_amd import optim
    from kf_benchmarks_amd.models.model import Network
    from kf_benchmarks_amd.models.resnet_model import create_resnet20_cifar_model

    res = {}
    for dev in ("cpu", cuda):
        model = create_resnet20_cifar_model(None)
        net = Network(model, 11, dev, torch.float32, seed=5)
        flat = optim.FlatParams(net, torch.bfloat16)
        opt = optim.FusedOptimizer(flat, "momentum")
        g = torch.Generator().manual_seed(3)
        src = torch.randn(flat.numel, generator=g).to(flat.flat.device)
        wout = torch.zeros_like(flat.flat)
        flag = None if ok is None else torch.tensor([ok], dtype=torch.int32,
                                                     device=flat.flat.device)
        for i in range(2):
            flat.grad.copy_(torch.randn(flat.numel, generator=g).to(flat.grad.device))
            opt.step(0.01, grad_scale=0.5, weight_decay=1e-3, mix=(src, 0.75, 0.25, flag),
                     wout=wout)
        res[str(dev)] = (flat.flat.cpu().clone(), wout.cpu().clone())
    a, b = res["cpu"], res[str(cuda)]
    torch.testing.assert_close(b[0], a[0], rtol=1e-5, atol=1e-6)
    assert torch.equal(b[1], b[0]) and torch.equal(a[1], a[0])


def test_seqlock_check_reads_host_word(cuda):
    """The device-side PairAveraging snapshot check reads the peer's sequence
    word from page-locked host memory (a /dev/shm mapping) at kernel time."""
    import ctypes
    import mmap
    import struct
    from kf_benchmarks_amd.ops import _native as N
    path = "/dev/shm/kfb_test_seq_%d" % os.getpid()
    with open(path, "wb") as f:
        f.write(b"\0" * 64)
    f = open(path, "r+b")
    m = mmap.mmap(f.fileno(), 64)
    try:
        host = ctypes.addressof(ctypes.c_char.from_buffer(m))
        dev = ctypes.c_void_p()
        N.call("kfb_host_register", host, 64, ctypes.byref(dev))
        ok = torch.zeros(1, dtype=torch.int32, device=cuda)
        torn = torch.zeros(1, dtype=torch.int32, device=cuda)
        s = N.stream(cuda)
        for word, val, expect, good in ((0, 4, 4, 1), (1, 7, 6, 0), (0, 6, 4, 0), (1, 8, 8, 1)):
            struct.pack_into("<q", m, 8 * word, val)
            N.call("kfb_seqlock_check", dev.value + 8 * word, expect, ok.data_ptr(),
                   torn.data_ptr(), s)
            torch.cuda.synchronize()
            assert int(ok.item()) == good, (word, val, expect)
        assert int(torn.item()) == 2
        N.call("kfb_host_unregister", host)
    finally:
        m.close()
        f.close()
        os.remove(path)


def _epilogue_stats(x):
    """[2][32][C] partial sums as a conv epilogue leaves them (slot 0 only)."""
    from kf_benchmarks_amd.ops import conv_hip
    C = x.shape[-1]
    xf = x.float().reshape(-1, C)
    st = torch.zeros(2, conv_hip.STATS_SPREAD, C, device=x.device)
    st[0, 0] = xf.sum(0)
    st[1, 0] = (xf * xf).sum(0)
    return st.reshape(-1)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(4, 7, 7, 64), (2, 5, 6, 256)])
@pytest.mark.parametrize("relu", [True, False])
def test_batch_norm_dual(cuda, dt, shape, relu):
    """relu?(bn(x) + bn_r(xr)) in one apply pass (kfb_bn_fwd_train_dual,
    DeferredBN) vs the fp32 reference of two BNs and the add."""
    from kf_benchmarks_amd.ops import nn as KF
    torch.manual_seed(2)
    C = shape[-1]
    x, xr = torch.randn(shape) * 2 + 0.5, torch.randn(shape) * 0.5 - 1
    g0, b0, g1, b1 = torch.rand(C) + 0.5, torch.randn(C), torch.rand(C) + 0.5, torch.randn(C)
    xa, xb = _pair(x, cuda, dt)
    ra, rb = _pair(xr, cuda, dt)
    pa = [t.clone().to(cuda).requires_grad_(True) for t in (g0, b0, g1, b1)]
    pb = [t.clone().requires_grad_(True) for t in (g0, b0, g1, b1)]
    rms = [torch.zeros(C, device=cuda), torch.ones(C, device=cuda),
           torch.zeros(C, device=cuda), torch.ones(C, device=cuda)]
    d = KF.DeferredBN(ra, pa[2], pa[3], rms[2], rms[3], 0.9, 1e-5, _epilogue_stats(ra.detach()))
    ya = KF.batch_norm_dual(xa, pa[0], pa[1], rms[0], rms[1], 0.9, 1e-5, relu,
                            _epilogue_stats(xa.detach()), d)
    rm_b = [torch.zeros(C), torch.ones(C), torch.zeros(C), torch.ones(C)]
    yr = F.batch_norm(rb, pb[2], pb[3], rm_b[2], rm_b[3], 0.9, 1e-5, True, False)
    yb = F.batch_norm(xb, pb[0], pb[1], rm_b[0], rm_b[1], 0.9, 1e-5, True, relu, yr)
    t = dict(rtol=2e-2, atol=2e-2) if dt == torch.bfloat16 else dict(rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(ya.float().cpu(), yb, rtol=t["rtol"] * 2, atol=t["atol"] * 2)
    for a, b in zip(rms, rm_b):
        torch.testing.assert_close(a.cpu(), b, rtol=1e-3, atol=1e-3)
    dy = torch.randn(shape).to(dt).float()
    ya.backward(dy.to(cuda, dt))
    yb.backward(dy)
    torch.testing.assert_close(xa.grad.float().cpu(), xb.grad, rtol=t["rtol"] * 4, atol=t["atol"] * 4)
    torch.testing.assert_close(ra.grad.float().cpu(), rb.grad, rtol=t["rtol"] * 4, atol=t["atol"] * 4)
    for a, b in zip(pa, pb):
        torch.testing.assert_close(a.grad.cpu(), b.grad, rtol=5e-2, atol=0.5)


@pytest.mark.parametrize("cin,cout,x_grad", [(4099, 1, False), (512, 1000, True), (300, 7, True)])
def test_linear_fwd_bwd(cuda, cin, cout, x_grad):
    """F.linear (+bias, ReLU) vs fp32 PyTorch, including the narrow-output
    dW path (Cout < 16) and the no-input-gradient first layer."""
    g = torch.Generator().manual_seed(cin + cout)
    x = torch.randn(33, cin, generator=g)
    w = torch.randn(cin, cout, generator=g) / cin ** 0.5
    b = torch.randn(cout, generator=g)
    dy = torch.randn(33, cout, generator=g)
    xd = x.to(cuda, torch.bfloat16).requires_grad_(x_grad)
    wd, bd = w.to(cuda).requires_grad_(), b.to(cuda).requires_grad_()
    y = F.linear(xd, wd, bd, relu=True)
    y.backward(dy.to(cuda, torch.bfloat16))
    xr = x.to(torch.bfloat16).float().requires_grad_(x_grad)
    wr, br = w.to(torch.bfloat16).float().requires_grad_(), b.clone().requires_grad_()
    yl = xr @ wr + br
    assert torch.allclose(y.float().cpu(), torch.relu(yl), atol=3e-2, rtol=2e-2)
    # ReLU mask from the kernel's own output (bf16 ties at y ~ 0)
    yl.backward(dy.to(torch.bfloat16).float() * (y.float().cpu() > 0))
    for got, ref in ((wd.grad, wr.grad), (bd.grad, br.grad)) + (((xd.grad, xr.grad),) if x_grad else ()):
        err = float((got.float().cpu() - ref).abs().max() / (ref.abs().max() + 1e-6))
        assert err < 2e-2, err
    if not x_grad:
        assert xd.grad is None


def _rel_err(got, ref):
    return float((got.double() - ref.double()).abs().max() / (ref.double().abs().max() + 1e-6))


@pytest.mark.parametrize("B,cin,cout", [
    (128, 25088, 4096),   # VGG-16 fc6 at bs 128 (split-K forward, KS weight operand)
    (128, 4096, 4096),    # fc7
    (128, 4096, 1001),    # logits: Cout % 8 != 0 (per-element loads / stores)
    (512, 9216, 4096),    # AlexNet fc6 at bs 512
    (37, 203, 77),        # ragged everything
    (2048, 256, 256),     # NCF MLP at batch 2048: split-K weight gradient
    (2048, 128, 64),
    (4099, 203, 77),      # ragged split-K weight gradient
])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_linear_production_shapes(cuda, B, cin, cout, dt):
    """The affine op's three GEMMs (csrc/gemm.hip) at the zoo's FC shapes
    against an fp32 oracle on the same bf16-rounded inputs (torch fp32 on
    the GPU: this is the reference, not the op under test)."""
    g = torch.Generator(device="cpu").manual_seed(B + cin + cout)
    x = torch.randn(B, cin, generator=g).to(cuda, dt)
    w = (torch.randn(cin, cout, generator=g) / cin ** 0.5).to(cuda)
    b = torch.randn(cout, generator=g).to(cuda)
    dy = torch.randn(B, cout, generator=g).to(cuda, dt)
    wl = w.to(dt)
    xd = x.clone().requires_grad_(True)
    wd, bd = w.clone().requires_grad_(), b.clone().requires_grad_()
    y = F.linear(xd, wd, bd, w_lp=wl, relu=False)
    y.backward(dy)
    xf, wf, dyf = x.double(), wl.double(), dy.double()
    yr = xf @ wf + b.double()
    lim = 1e-2 if dt == torch.bfloat16 else 1e-5
    assert _rel_err(y, yr) < lim
    assert _rel_err(xd.grad, dyf @ wf.t()) < lim
    assert _rel_err(wd.grad, xf.t() @ dyf) < lim
    assert _rel_err(bd.grad, dyf.sum(0)) < lim


@pytest.mark.parametrize("B", [64, 2048])
def test_linear_grad_sink_accumulates(cuda, B):
    """A FlatParams-managed weight: dW is accumulated in place in the flat
    gradient view (no autograd tensor returned) and the ready callback fires
    (B=2048: through the split-K slab and its accumulating reduce)."""
    torch.manual_seed(3)
    x = torch.randn(B, 256, device=cuda).to(torch.bfloat16)
    w = torch.nn.Parameter(torch.randn(256, 128, device=cuda) / 16)
    sink = torch.full((256, 128), 0.5, device=cuda)
    w._kfb_grad_sink = sink
    fired = []
    w._kfb_ready_cb = lambda p: fired.append(p)
    dy = torch.randn(B, 128, device=cuda).to(torch.bfloat16)
    y = F.linear(x, w, None, w_lp=w.detach().to(torch.bfloat16), relu=False)
    y.backward(dy)
    ref = x.float().t() @ dy.float() + 0.5
    assert _rel_err(sink, ref) < 1e-2 and fired == [w] and w.grad is None


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("shape,r", [((4, 8, 8, 64), 4), ((2, 5, 5, 20), 2), ((3, 3, 3, 96), 5)])
def test_lrn(cuda, dt, shape, r):
    torch.manual_seed(1)
    x = torch.randn(shape) * 2
    bias, alpha, beta = 1.0, 0.001 / 9.0, 0.75
    xa, xb = _pair(x, cuda, dt)
    ya = F.lrn(xa, r, bias, alpha, beta)
    yb = F.lrn(xb, r, bias, alpha, beta)
    torch.testing.assert_close(ya.float().cpu(), yb.float(), **tol(dt))
    dy = torch.randn(shape).to(dt).float()
    ya.backward(dy.to(cuda, dt))
    yb.float().backward(dy)
    torch.testing.assert_close(xa.grad.float().cpu(), xb.grad, **tol(dt))


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("widths", [(64, 128, 32), (3, 5, 8, 1), (96, 96), (16,) * 16,
                                    tuple(8 + (i % 3) * 8 for i in range(37))])
def test_concat_channels(cuda, dt, widths):
    """Channel concat (csrc/gather.hip) and its split backward vs torch.cat."""
    torch.manual_seed(4)
    xs = [torch.randn(3, 5, 7, w) for w in widths]
    xa = [x.to(cuda, dt).requires_grad_(True) for x in xs]
    y = F.concat_channels(xa)
    ref = torch.cat([x.to(dt) for x in xs], dim=-1)
    assert torch.equal(y.cpu(), ref)
    dy = torch.randn(ref.shape).to(dt)
    y.backward(dy.to(cuda))
    off = 0
    for x, w in zip(xa, widths):
        assert torch.equal(x.grad.cpu(), dy[..., off:off + w])
        off += w


@pytest.mark.parametrize("dim", [64, 128, 5])
def test_embedding_lookup_and_grad(cuda, dim):
    """Embedding gather and the scatter-add gradient (repeated ids) vs torch."""
    torch.manual_seed(5)
    rows = 1000
    table = torch.randn(rows, dim)
    idx = torch.randint(0, rows, (4096,), dtype=torch.int32)
    idx[:100] = 7  # many duplicates -> atomics on one row
    ta = table.to(cuda).requires_grad_(True)
    y = F.embedding(idx.to(cuda), ta)
    assert torch.equal(y.cpu(), table[idx.long()])
    dy = torch.randn(4096, dim)
    y.backward(dy.to(cuda))
    ref = torch.zeros(rows, dim).index_add_(0, idx.long(), dy)
    torch.testing.assert_close(ta.grad.cpu(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("case", ["mixed", "all_negative", "many_matched", "few_classes"])
def test_ssd_loss(cuda, dt, case):
    """Fused SSD loss (csrc/ssd_loss.hip: per-row lse over 16 lanes + per-image
    radix select of the hard negatives) vs the stable-sort tensor form in fp32
    (few_classes: C < 16, so some lanes of a row hold no class)."""
    B, A, C = 4, 8732, (5 if case == "few_classes" else 81)
    g = torch.Generator().manual_seed(7)
    logits = torch.randn(B, A, 4 + C, generator=g) * 2
    gt_loc = torch.randn(B, A, 4, generator=g)
    if case == "all_negative":  # the synthetic-data configuration: every label 0
        label = torch.zeros(B, A, 1)
        nm = torch.rand(B, generator=g) * 9 + 1
    else:
        frac = 0.2 if case == "many_matched" else 0.02
        pos = torch.rand(B, A, 1, generator=g) < frac
        label = torch.where(pos, torch.randint(1, C, (B, A, 1), generator=g).float(),
                            torch.zeros(B, A, 1)) + 0.3  # truncation like .long()
        nm = pos.reshape(B, A).sum(1).float()
        if case == "many_matched":  # k = 3 n exceeds A: every negative is mined
            nm = nm * 2
    a, b = _pair(logits, "cuda", dt)
    got = F.ssd_loss(a, gt_loc.cuda(), label.cuda(), nm.cuda())
    ref = F.ssd_loss_reference(b, gt_loc, label, nm)
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-4, atol=1e-4)
    (got * 1.7).backward()
    (ref * 1.7).backward()
    t = dict(rtol=2e-2, atol=1e-6) if dt == torch.bfloat16 else dict(rtol=1e-4, atol=1e-8)
    torch.testing.assert_close(a.grad.float().cpu(), b.grad, **t)


def test_ssd_loss_bwd_past_2g_elements(cuda):
    """The SSD loss backward at B*A*(4+C) >= 2^31 elements (~2,900 images of
    8732 anchors x 85 logits) runs its 64-bit-index form (it used
    to refuse that size): its first and last images equal a small call over
    those images bitwise (32-bit form, same arithmetic)."""
    from kf_benchmarks_amd.ops import _native as N
    A, C = 8732, 81
    B = (1 << 31) // (A * (4 + C)) + 2
    assert B * A * (4 + C) >= (1 << 31)
    dev = torch.device(cuda)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn((B, A, 4 + C), generator=g, device=dev, dtype=torch.bfloat16)
    gt = torch.randn((B, A, 4), generator=g, device=dev)
    label = torch.randint(0, C, (B, A), generator=g, device=dev).float() + 0.3
    nm = torch.rand((B,), generator=g, device=dev) * 50 + 1
    lse = torch.randn((B, A), generator=g, device=dev)
    w = torch.rand((B, A), generator=g, device=dev)

    def work_of(imgs):
        n = len(imgs)
        wk = torch.zeros(n + 3 * n * A, device=dev)
        wk[n:n + n * A] = lse[imgs].reshape(-1)
        wk[n + 2 * n * A:] = w[imgs].reshape(-1)
        return wk

    def bwd(xx, gg, ll, nn_, wk, b):
        dx = torch.empty_like(xx)
        gs = torch.full((1,), float(b), device=dev)  # g / B = 1 in every call
        N.call("kfb_ssd_loss_bwd", N.dt(xx), xx.data_ptr(), gg.data_ptr(), ll.data_ptr(),
               nn_.data_ptr(), wk.data_ptr(), gs.data_ptr(), b, A, C, dx.data_ptr(),
               N.stream(dev))
        return dx

    big = bwd(x, gt, label, nm, work_of(list(range(B))), B)
    for imgs in ([0, 1], [B - 2, B - 1]):
        small = bwd(x[imgs].contiguous(), gt[imgs].contiguous(), label[imgs].contiguous(),
                    nm[imgs].contiguous(), work_of(imgs), 2)
        assert torch.equal(big[imgs], small), imgs
    del big, x
    torch.cuda.empty_cache()


@pytest.mark.parametrize("dt", DT)
def test_ssd_heads(cuda, dt):
    """Anchor-major SSD logits from NHWC heads (kfb_ssd_heads) vs the
    permute + concat reference, forward and backward."""
    torch.manual_seed(5)
    B, ncls, nds, hw = 3, 5, [4, 6, 4], [(5, 5), (3, 3), (1, 1)]
    locs = [torch.randn(B, h, w, nd * 4) for nd, (h, w) in zip(nds, hw)]
    confs = [torch.randn(B, h, w, nd * ncls) for nd, (h, w) in zip(nds, hw)]
    la = [t.to(cuda, dt).requires_grad_(True) for t in locs + confs]
    lb = [t.to(dt).float().requires_grad_(True) for t in locs + confs]
    ya = F.ssd_heads(la[:3], la[3:], nds, ncls)
    yb = F.ssd_heads(lb[:3], lb[3:], nds, ncls)
    assert torch.equal(ya.float().cpu(), yb.to(dt).float())
    g = torch.randn(yb.shape).to(dt)
    ya.backward(g.to(cuda))
    yb.backward(g.float())
    for a, b in zip(la, lb):
        assert torch.equal(a.grad.float().cpu(), b.grad.to(dt).float())


@pytest.mark.parametrize("dt", DT)
def test_channel_pad(cuda, dt):
    x = torch.randn(3, 4, 5, 16)
    xa = x.to(cuda, dt).requires_grad_(True)
    y = F.channel_pad(xa, 8, 8)
    assert torch.equal(y.float().cpu(), torch.nn.functional.pad(x.to(dt).float(), (8, 8)))
    g = torch.randn(y.shape).to(dt)
    y.backward(g.to(cuda))
    assert torch.equal(xa.grad.float().cpu(), g[..., 8:24].float())


@pytest.mark.parametrize("kind", ["relu6", "tanh"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(2, 7, 7, 96), (3, 5, 5, 3)])
def test_activation_native(cuda, kind, dt, shape):
    """relu6 / tanh forward and backward (csrc/elementwise.hip act_fwd_k /
    act_bwd_k) against the fp32 torch ops."""
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(shape, generator=g) * 4).to(dt)
    dy = torch.randn(shape, generator=g).to(dt)
    xa = x.to(cuda).requires_grad_(True)
    ya = F.activation(xa, kind)
    ya.backward(dy.to(cuda))
    xr = x.float().requires_grad_(True)
    yr = torch.clamp(xr, 0.0, 6.0) if kind == "relu6" else torch.tanh(xr)
    yr.backward(dy.float())
    gref = xr.grad
    if kind == "relu6":
        # tf.nn.relu6's gradient: dy * (0 < x < 6), strict at both ends
        # (torch.clamp's passes the gradient at x == 0 and x == 6)
        gref = dy.float() * ((x.float() > 0) & (x.float() < 6)).float()
    tol = 2e-2 if dt == torch.bfloat16 else 1e-5
    torch.testing.assert_close(ya.float().cpu(), yr.detach(), rtol=tol, atol=tol)
    torch.testing.assert_close(xa.grad.float().cpu(), gref, rtol=tol, atol=tol)
