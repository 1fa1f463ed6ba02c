"""Implicit-GEMM conv kernels (fwd / dgrad / wgrad) vs a PyTorch fp32 reference."""

import pytest
import torch

from kf_benchmarks_amd.ops import conv as conv_ops
from kf_benchmarks_amd.ops import nn as F

pytestmark = pytest.mark.gpu

# (N, H, W, Cin, Cout, KH, KW, stride, mode)
SHAPES = [
    (2, 14, 14, 64, 256, 1, 1, 1, "SAME"),        # 1x1 expand
    (2, 14, 14, 256, 64, 1, 1, 1, "SAME"),        # 1x1 reduce (Cout=64 tile)
    (2, 14, 14, 256, 512, 1, 1, 2, "SAME"),       # strided 1x1 projection
    (2, 13, 13, 64, 64, 3, 3, 1, "SAME_RESNET"),  # 3x3, odd spatial
    (2, 14, 14, 128, 128, 3, 3, 2, "SAME_RESNET"),  # 3x3 s2 (v1.5)
    (2, 32, 32, 3, 64, 7, 7, 2, "SAME_RESNET"),   # RGB stem (channel pad)
    (3, 9, 9, 48, 64, 5, 5, 1, "SAME"),           # K steps spanning taps
    (2, 17, 17, 160, 192, 1, 7, 1, "SAME"),       # asymmetric kernel
    (2, 17, 17, 128, 96, 7, 1, 1, "SAME"),
    (2, 11, 11, 64, 96, 3, 3, 2, "VALID"),
    (1, 7, 7, 512, 2048, 1, 1, 1, "SAME"),        # M < one tile
    (2, 8, 8, 20, 36, 3, 3, 1, "SAME"),           # Cin, Cout not multiples of 8
]


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_conv_fwd_bwd(cuda, shape, dt):
    n, H, W, cin, cout, kh, kw, s, mode = shape
    torch.manual_seed(0)
    x = torch.randn(n, H, W, cin).to(dt).float()
    w = (torch.randn(cout, kh, kw, cin) / (kh * kw * cin) ** 0.5).to(dt).float()
    pads = F.resolve_pads(mode, H, W, kh, kw, s, s)
    xa = x.to(cuda, dt).requires_grad_(True)
    wa = w.to(cuda).requires_grad_(True)
    ya = conv_ops.conv2d(xa, wa, wa.detach().to(dt), (s, s), pads, "hip")
    xb = x.clone().requires_grad_(True)
    wb = w.clone().requires_grad_(True)
    yb = conv_ops.conv2d_reference(xb, wb, (s, s), pads)
    assert ya.shape == yb.shape
    torch.testing.assert_close(ya.float().cpu(), yb, rtol=2e-2, atol=2e-2)
    dy = torch.randn(yb.shape).to(dt).float()
    ya.backward(dy.to(cuda, dt))
    yb.backward(dy)
    scale = dy.abs().mean().item()
    torch.testing.assert_close(xa.grad.float().cpu(), xb.grad, rtol=3e-2, atol=3e-2 * scale * 4)
    gw = wb.grad
    torch.testing.assert_close(wa.grad.cpu(), gw, rtol=3e-2, atol=2e-2 * gw.abs().max().item())


def test_dgrad_weight_relayout_matches(cuda):
    from kf_benchmarks_amd import datasets, optim, params as P
    from kf_benchmarks_amd.models import model_config
    from kf_benchmarks_amd.models.model import Network
    from kf_benchmarks_amd.ops.conv_hip import DgradWeights
    d = datasets.create_dataset(None, "imagenet")
    for name in ("resnet50", "inception3"):
        m = model_config.get_model_config(name, d, P.make_params(model=name))
        net = Network(m, 1001, cuda, torch.bfloat16, seed=1)
        flat = optim.FlatParams(net, torch.bfloat16)
        DgradWeights(net, flat)
        n = 0
        for layer in net.ordered_layers():
            wt = getattr(layer, "weight_t", None)
            if wt is None:
                continue
            wl = layer.weight_lp
            if tuple(layer.stride) == (1, 1) and wl.shape[1:3] != (1, 1):
                ref = wl.flip(1, 2).permute(3, 1, 2, 0)
            else:
                ref = wl.permute(3, 1, 2, 0)
            assert torch.equal(wt, ref.contiguous()), layer.tf_scope
            n += 1
        assert n > 10
