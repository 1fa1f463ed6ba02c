"""Streaming 3x3 64-channel conv kernel (csrc/conv_stream.hip, IG_ALGO_S3)
vs a PyTorch fp32 reference: forward with the BN-statistics epilogue,
stride-1 dgrad with the fused producer-BN backward epilogue (ReLU mask from
bits / values / recomputed, addend, partial sums), and the ring / multi-tile
logic forced by a small grid (every workgroup then streams many tiles and
wraps its 5-block LDS ring several times)."""

import pytest
import torch

from kf_benchmarks_amd.ops import _native as N
from kf_benchmarks_amd.ops import conv as conv_ops
from kf_benchmarks_amd.ops import nn as F

pytestmark = pytest.mark.gpu

# (N, H, W): all 64 -> 64, 3x3, stride 1, SAME
SHAPES = [(2, 14, 14), (3, 9, 11), (1, 56, 56), (5, 7, 5), (4, 28, 28), (2, 17, 62)]
GRIDS = [0, 3, 1]  # 0 = one workgroup per CU; 1 / 3 = many tiles per workgroup


@pytest.fixture
def s3(monkeypatch, cuda):
    from kf_benchmarks_amd.ops import conv_hip
    monkeypatch.setattr(conv_hip, "_IG_FORCE", conv_hip.IG_S3)
    yield
    N.load().kfb_conv_s3_set_grid(0)


def test_s3_applicability():
    lib = N.load()
    assert lib.kfb_conv_s3_applicable(64, 64, 3, 3, 1, 1, 1, 1, 56, 56, 56, 56) == 1
    assert lib.kfb_conv_s3_applicable(64, 128, 3, 3, 1, 1, 1, 1, 56, 56, 56, 56) == 0
    assert lib.kfb_conv_s3_applicable(64, 64, 3, 3, 2, 2, 1, 1, 56, 56, 28, 28) == 0
    assert lib.kfb_conv_s3_applicable(64, 64, 3, 3, 1, 1, 1, 1, 63, 63, 63, 63) == 0  # halo > block


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
@pytest.mark.parametrize("grid", GRIDS)
def test_s3_fwd_stats_and_dgrad(s3, cuda, shape, grid):
    from kf_benchmarks_amd.ops import conv_hip
    N.load().kfb_conv_s3_set_grid(grid)
    n, H, W = shape
    g = torch.Generator().manual_seed(3)
    dt = torch.bfloat16
    x = torch.randn(n, H, W, 64, generator=g).to(dt)
    w = (torch.randn(64, 3, 3, 64, generator=g) / 24.0).to(dt)
    pads = F.resolve_pads("SAME_RESNET", H, W, 3, 3, 1, 1)
    ref = conv_ops.conv2d_reference(x.float(), w.float(), (1, 1), pads)
    st = conv_hip.stats_buffer(64, cuda).zero_()
    y = conv_hip.conv_fwd(x.to(cuda), w.to(cuda), (1, 1), pads, st)
    torch.testing.assert_close(y.float().cpu(), ref, rtol=2e-2, atol=2e-2)
    yf = y.float().cpu()
    p = st.view(2, conv_hip.STATS_SPREAD, 64).sum(1).cpu()
    tol = 4e-3 * (yf.abs() + yf * yf).sum((0, 1, 2)).max().item()
    torch.testing.assert_close(p[0], yf.sum((0, 1, 2)), rtol=1e-2, atol=tol)
    torch.testing.assert_close(p[1], (yf * yf).sum((0, 1, 2)), rtol=1e-2, atol=tol)
    # plain dgrad (stride-1 transposed conv = forward conv with flipped weights)
    dy = torch.randn(ref.shape, generator=g).to(dt)
    xr = x.float().requires_grad_(True)
    conv_ops.conv2d_reference(xr, w.float(), (1, 1), pads).backward(dy.float())
    dx = conv_hip.conv_dgrad(dy.to(cuda), w.to(cuda), x.shape, (1, 1), pads)
    torch.testing.assert_close(dx.float().cpu(), xr.grad, rtol=3e-2, atol=3e-2)


def _bits(y):
    b = (y.float().reshape(-1, 8) > 0).to(torch.int32)
    return (b * (1 << torch.arange(8, dtype=torch.int32))).sum(1).to(torch.uint8)


@pytest.mark.parametrize("shape", SHAPES[:4], ids=[str(s) for s in SHAPES[:4]])
@pytest.mark.parametrize("mask_src", ["read", "recompute", "bits"])
@pytest.mark.parametrize("with_addend", [False, True])
def test_s3_dgrad_fused_epilogue(s3, cuda, shape, mask_src, with_addend):
    from kf_benchmarks_amd.ops import conv_hip
    N.load().kfb_conv_s3_set_grid(2)
    n, H, W = shape
    g = torch.Generator().manual_seed(5)
    dt = torch.bfloat16
    w = (torch.randn(64, 3, 3, 64, generator=g) / 24.0).to(dt)
    pads = F.resolve_pads("SAME_RESNET", H, W, 3, 3, 1, 1)
    dy = torch.randn(n, H, W, 64, generator=g).to(dt)
    xb = torch.randn(n, H, W, 64, generator=g).to(dt)
    mean = torch.randn(64, generator=g)
    x = torch.randn(n, H, W, 64, generator=g).to(dt)
    mcoef = None
    if mask_src == "recompute":
        scale, shift = torch.rand(64, generator=g) + 0.5, torch.randn(64, generator=g) * 0.5
        x = torch.relu(xb.float() * scale + shift).to(dt)
        mcoef = torch.cat([scale, shift])
    add = torch.randn(n, H, W, 64, generator=g).to(dt) if with_addend else None
    xr = x.float().requires_grad_(True)
    conv_ops.conv2d_reference(xr, w.float(), (1, 1), pads).backward(dy.float())
    ref = (xr.grad + (add.float() if add is not None else 0)) * (x.float() > 0)
    parts = conv_hip.stats_buffer(64, cuda).zero_()
    if mask_src == "bits":
        fuse = (parts, _bits(x).to(cuda), xb.to(cuda), mean.to(cuda))
    elif mask_src == "read":
        fuse = (parts, x.to(cuda), xb.to(cuda), mean.to(cuda))
    else:
        fuse = (parts, None, xb.to(cuda), mean.to(cuda), mcoef.to(cuda))
    dx = conv_hip.conv_dgrad(dy.to(cuda), w.to(cuda), x.shape, (1, 1), pads, fuse,
                             addend=add.to(cuda) if add is not None else None)
    torch.testing.assert_close(dx.float().cpu(), ref, rtol=3e-2, atol=3e-2)
    p = parts.view(2, conv_hip.STATS_SPREAD, 64).sum(1).cpu()
    r = dx.float().cpu()
    s1 = r.sum((0, 1, 2))
    s2 = (r * (xb.float() - mean)).sum((0, 1, 2))
    tol = 4e-3 * (r.abs() * (1 + (xb.float() - mean).abs())).sum((0, 1, 2)).max().item()
    torch.testing.assert_close(p[0], s1, rtol=1e-2, atol=tol)
    torch.testing.assert_close(p[1], s2, rtol=1e-2, atol=tol)


def test_s3_matches_tiled_kernel_at_resnet_shape(cuda, monkeypatch):
    """ResNet-50 conv2_x shape at batch 32: the streaming kernel and the
    register-staged tiled kernel agree to bf16 output rounding."""
    from kf_benchmarks_amd.ops import conv_hip
    g = torch.Generator().manual_seed(7)
    x = torch.randn(32, 56, 56, 64, generator=g).to(torch.bfloat16).to(cuda)
    w = (torch.randn(64, 3, 3, 64, generator=g) / 24.0).to(torch.bfloat16).to(cuda)
    pads = F.resolve_pads("SAME_RESNET", 56, 56, 3, 3, 1, 1)
    monkeypatch.setattr(conv_hip, "_IG_FORCE", conv_hip.IG_S3)
    a = conv_hip.conv_fwd(x, w, (1, 1), pads).float()
    monkeypatch.setattr(conv_hip, "_IG_FORCE", conv_hip.IG_ONEBUF)
    b = conv_hip.conv_fwd(x, w, (1, 1), pads).float()
    err = (a - b).abs().max().item()
    assert err <= 1e-2 * b.abs().max().item(), err


@pytest.fixture
def s3w(monkeypatch, cuda):
    from kf_benchmarks_amd.ops import conv_hip
    monkeypatch.setattr(conv_hip, "_WGRAD_ALGO", "s3")
    monkeypatch.setattr(conv_hip, "_wgrad_tuned", {})
    yield
    N.load().kfb_conv_s3_set_grid(0)


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
@pytest.mark.parametrize("grid", GRIDS)
def test_s3_wgrad(s3w, cuda, shape, grid):
    """Streaming weight gradient vs the fp32 reference, and bitwise
    repeatable (fixed-order slab fold, no atomics)."""
    from kf_benchmarks_amd.ops import conv_hip
    N.load().kfb_conv_s3_set_grid(grid)
    n, H, W = shape
    g = torch.Generator().manual_seed(11)
    dt = torch.bfloat16
    x = torch.randn(n, H, W, 64, generator=g).to(dt)
    dy = torch.randn(n, H, W, 64, generator=g).to(dt)
    pads = F.resolve_pads("SAME_RESNET", H, W, 3, 3, 1, 1)
    wr = torch.zeros(64, 3, 3, 64, requires_grad=True)
    conv_ops.conv2d_reference(x.float(), wr, (1, 1), pads).backward(dy.float())
    dw = conv_hip.conv_wgrad(dy.to(cuda), x.to(cuda), (64, 3, 3, 64), (1, 1), pads)
    ref = wr.grad
    torch.testing.assert_close(dw.float().cpu(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
    dw2 = conv_hip.conv_wgrad(dy.to(cuda), x.to(cuda), (64, 3, 3, 64), (1, 1), pads)
    assert torch.equal(dw, dw2)
