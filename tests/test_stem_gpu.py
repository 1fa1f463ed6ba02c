"""ResNet stem fusions on the GPU vs fp32 PyTorch references:

* the space-to-depth stride-2 conv over a 3-channel input (csrc/stem.hip +
  the FAST implicit-GEMM kernels): forward and weight gradient;
* the fused BN(train) + ReLU + 3x3/2 max-pool (csrc/bn.hip): pooled output,
  running statistics, input gradient and dgamma/dbeta.
"""

import pytest
import torch

from kf_benchmarks_amd.ops import conv as conv_ops
from kf_benchmarks_amd.ops import nn as F

pytestmark = pytest.mark.gpu

STEM_SHAPES = [
    (2, 224, 224, 3, 64, 7, 7, "SAME_RESNET"),   # the ResNet stem
    (3, 37, 30, 3, 64, 7, 7, "SAME_RESNET"),     # odd height, M not a tile multiple
    (2, 33, 33, 4, 32, 5, 5, "SAME"),            # 4 channels, 5x5, TF SAME pads
    (2, 31, 32, 1, 64, 8, 8, "VALID"),           # even kernel, one channel
]


@pytest.mark.parametrize("mode", ["pairs", "s2d"])
@pytest.mark.parametrize("shape", STEM_SHAPES, ids=[str(s) for s in STEM_SHAPES])
def test_s2d_stem_conv(cuda, shape, mode, monkeypatch):
    """Both stem forms: the pixel-pair strided conv (default) and the
    space-to-depth repack."""
    from kf_benchmarks_amd.ops import conv_hip
    monkeypatch.setattr(conv_hip, "_STEM_MODE", mode)
    n, H, W, cin, cout, kh, kw, mode = shape
    g = torch.Generator().manual_seed(3)
    dt = torch.bfloat16
    x = torch.randn(n, H, W, cin, generator=g).to(dt).float()
    w = (torch.randn(cout, kh, kw, cin, generator=g) / (kh * kw * cin) ** 0.5).to(dt).float()
    pads = F.resolve_pads(mode, H, W, kh, kw, 2, 2)
    assert conv_hip.use_s2d(x.to(cuda, dt), (cout, kh, kw, cin), (2, 2), False, pads)
    wa = w.to(cuda).requires_grad_(True)
    ya = conv_ops.conv2d(x.to(cuda, dt), wa, wa.detach().to(dt), (2, 2), pads, "hip")
    wb = w.clone().requires_grad_(True)
    yb = conv_ops.conv2d_reference(x, wb, (2, 2), pads)
    assert ya.shape == yb.shape
    torch.testing.assert_close(ya.float().cpu(), yb, rtol=2e-2, atol=2e-2)
    dy = torch.randn(yb.shape, generator=g).to(dt).float()
    ya.backward(dy.to(cuda, dt))
    yb.backward(dy)
    gw = wb.grad
    torch.testing.assert_close(wa.grad.cpu(), gw, rtol=3e-2, atol=2e-2 * gw.abs().max().item())


def test_s2d_weight_roundtrip():
    from kf_benchmarks_amd.ops import conv_hip
    w = torch.randn(16, 7, 7, 3)
    w2 = conv_hip.s2d_weight(w)
    assert w2.shape == (16, 1, 4, 64)
    assert torch.equal(conv_hip.s2d_weight_grad(w2, w.shape), w)
    # channel kh*8 + t*4 + c of tap j holds w[:, kh, 2j+t, c]
    assert torch.equal(w2[:, 0, 1, 2 * 8 + 1 * 4 + 2], w[:, 2, 3, 2])


POOL_SHAPES = [
    (4, 112, 112, 64, 3, 2, "SAME"),    # ResNet stem (3x3/2 block kernels)
    (3, 13, 11, 16, 3, 2, "SAME"),      # odd sizes, top/left padding
    (2, 15, 14, 24, 3, 2, "VALID"),     # C/8 = 3: generic gather kernels
    (2, 12, 12, 32, 2, 2, "VALID"),     # 2x2/2: generic gather kernels
]


@pytest.mark.parametrize("shape", POOL_SHAPES, ids=[str(s) for s in POOL_SHAPES])
def test_bn_relu_maxpool_fused(cuda, shape):
    from kf_benchmarks_amd.ops import conv_hip
    n, H, W, C, pk, ps, pmode = shape
    g = torch.Generator().manual_seed(5)
    dt = torch.bfloat16
    x = (torch.randn(n, H, W, C, generator=g) * 2 + 0.5).to(dt)
    gamma = (torch.rand(C, generator=g) + 0.5)
    beta = torch.randn(C, generator=g) * 0.3
    decay, eps = 0.9, 1e-5
    xa = x.to(cuda)
    # the producing conv's epilogue statistics: [2][32][C] slabs of sum / sum^2
    stats = torch.zeros(2 * conv_hip.STATS_SPREAD * C, device=cuda)
    xf = xa.float().reshape(-1, C)
    stats.view(2, conv_hip.STATS_SPREAD, C)[0, 0] = xf.sum(0)
    stats.view(2, conv_hip.STATS_SPREAD, C)[1, 0] = (xf * xf).sum(0)
    ga = gamma.to(cuda).requires_grad_(True)
    ba = beta.to(cuda).requires_grad_(True)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    xa.requires_grad_(True)
    za = F.bn_relu_max_pool(xa, ga, ba, rm, rv, decay, eps, stats, pk, pk, ps, ps, pmode)

    xb = x.float().requires_grad_(True)
    gb, bb = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    xc = xb.permute(0, 3, 1, 2)
    yb = torch.nn.functional.batch_norm(xc, None, None, gb, bb, training=True, eps=eps)
    yb = torch.relu(yb).to(dt).float()  # the unfused path stores the BN output in bf16
    pads, OH, OW = F.pool_geometry(x.shape, pk, pk, ps, ps, pmode)
    pt, pb, pl, pr = pads
    zb = torch.nn.functional.max_pool2d(
        torch.nn.functional.pad(yb, (pl, pr, pt, pb), value=-1.0), pk, ps).permute(0, 2, 3, 1)
    assert za.shape == zb.shape
    torch.testing.assert_close(za.float().cpu(), zb, rtol=2e-2, atol=2e-2)
    mean = x.float().reshape(-1, C).mean(0)
    var = x.float().reshape(-1, C).var(0, unbiased=True)
    torch.testing.assert_close(rm.cpu(), 0.1 * mean, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(rv.cpu(), 0.9 + 0.1 * var, rtol=1e-3, atol=1e-4)

    dz = torch.randn(zb.shape, generator=g).to(dt).float()
    za.backward(dz.to(cuda, dt))
    zb.backward(dz)
    sc = xb.grad.abs().max().item()
    torch.testing.assert_close(xa.grad.float().cpu(), xb.grad, rtol=5e-2, atol=3e-2 * sc)
    torch.testing.assert_close(ba.grad.cpu(), bb.grad, rtol=2e-2, atol=2e-2 * bb.grad.abs().max().item())
    torch.testing.assert_close(ga.grad.cpu(), gb.grad, rtol=3e-2, atol=3e-2 * gb.grad.abs().max().item())


# (the multi-tile kernels take the 64-channel geometry only; forced for an
# 8-channel conv they fall back to the one-tile kernel)
C8_ALGOS = ["classic", "glds", "classic_n64", "glds_n64", "onebuf", "onebuf_n64", "tall256",
            "small", "gshort64", "gshort128", "gshort64_3", "gbig512", "multi2", "gmulti64"]
C8_SHAPES = [  # (N, H, W, Cout, KH, KW, stride): 8-channel FAST geometry (C == 8, KW | 8)
    (2, 30, 20, 64, 8, 4, (2, 1)),     # the stem's pixel-pair conv
    (3, 17, 13, 32, 4, 2, (1, 1)),
    (1, 21, 19, 128, 1, 8, (2, 2)),
]


@pytest.mark.parametrize("algo", C8_ALGOS)
@pytest.mark.parametrize("shape", C8_SHAPES, ids=[str(s) for s in C8_SHAPES])
def test_c8_fast_conv_every_kernel(cuda, shape, algo, monkeypatch):
    """The FAST implicit-GEMM kernels in 8-channel geometry (each lane's
    16-byte chunk is its own tap) vs an fp32 reference, every kernel."""
    from kf_benchmarks_amd.ops import conv_hip
    monkeypatch.setattr(conv_hip, "_IG_FORCE", conv_hip.IG_ALGOS[algo])
    n, H, W, cout, kh, kw, stride = shape
    g = torch.Generator().manual_seed(11)
    dt = torch.bfloat16
    x = torch.randn(n, H, W, 8, generator=g).to(dt).float()
    w = (torch.randn(cout, kh, kw, 8, generator=g) / (kh * kw * 8) ** 0.5).to(dt).float()
    y = conv_hip.conv_fwd(x.to(cuda, dt), w.to(cuda, dt), stride, (0, 0, 0, 0))
    ref = conv_ops.conv2d_reference(x, w, stride, (0, 0, 0, 0))
    assert y.shape == ref.shape
    torch.testing.assert_close(y.float().cpu(), ref, rtol=2e-2, atol=2e-2)


S7_SHAPES = [(2, 112, 112), (3, 19, 15), (1, 9, 40), (4, 56, 128)]  # (N, OH, OW)


@pytest.mark.parametrize("shape", S7_SHAPES, ids=[str(s) for s in S7_SHAPES])
def test_s7_streaming_stem_conv(cuda, shape, monkeypatch):
    """The streaming stem kernel (csrc/conv_s7.hip, IG_ALGO_S7) on the
    pixel-pair view: 8x4 taps, stride (2, 1), 64 channels, with the shifted
    BN statistics, vs the fp32 reference - full rows (112), rows shorter
    than a wave's 32 pixels, the 128-pixel maximum, and bands of a few rows
    (small batches split each image over several workgroups)."""
    from kf_benchmarks_amd.ops import conv_hip
    n, OH, OW = shape
    Hp, Wp2 = 2 * (OH - 1) + 8, OW + 3
    g = torch.Generator().manual_seed(17)
    dt = torch.bfloat16
    xv = torch.randn(n, Hp, Wp2, 8, generator=g).to(dt)
    w2 = (torch.randn(64, 8, 4, 8, generator=g) / 16.0).to(dt)
    shift = torch.randn(64, generator=g) * 0.2
    ref = conv_ops.conv2d_reference(xv.float(), w2.float(), (2, 1), (0, 0, 0, 0))
    assert ref.shape == (n, OH, OW, 64)
    monkeypatch.setattr(conv_hip, "_IG_FORCE", conv_hip.IG_S7)
    st = conv_hip.stats_buffer(64, cuda, shift=shift.to(cuda)).zero_()
    y = conv_hip.conv_fwd(xv.to(cuda), w2.to(cuda), (2, 1), (0, 0, 0, 0), st)
    yf = y.float().cpu()
    torch.testing.assert_close(yf, ref, rtol=2e-2, atol=2e-2)
    p = st.view(2, conv_hip.STATS_SPREAD, 64).sum(1).cpu()
    d = yf.reshape(-1, 64) - shift
    tol = 4e-3 * (d.abs() + d * d).sum(0).max().item()
    torch.testing.assert_close(p[0], d.sum(0), rtol=1e-2, atol=tol)
    torch.testing.assert_close(p[1], (d * d).sum(0), rtol=1e-2, atol=tol)
    # the same through the tiled kernel agrees to output rounding
    monkeypatch.setattr(conv_hip, "_IG_FORCE", conv_hip.IG_CLASSIC)
    y2 = conv_hip.conv_fwd(xv.to(cuda), w2.to(cuda), (2, 1), (0, 0, 0, 0)).float().cpu()
    assert (yf - y2).abs().max().item() <= 1e-2 * y2.abs().max().item()


def test_s7_applicability():
    from kf_benchmarks_amd.ops import _native as N
    lib = N.load()
    assert lib.kfb_conv_s7_applicable(8, 64, 8, 4, 2, 1, 0, 0, 230, 115, 112, 112) == 1
    assert lib.kfb_conv_s7_applicable(8, 32, 8, 4, 2, 1, 0, 0, 230, 115, 112, 112) == 0
    assert lib.kfb_conv_s7_applicable(8, 64, 8, 4, 2, 1, 0, 0, 230, 200, 112, 197) == 0
