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
    (9, 2, 2, 64, 64, 3, 3, 1, "SAME"),           # rows wrap several images per K step
    (40, 1, 1, 256, 128, 1, 1, 1, "SAME"),        # 1x1 spatial (FC-like)
    (3, 19, 21, 128, 192, 3, 3, 1, "SAME_RESNET"),  # M = 1197: several 256-row tiles + remainder
    (2, 23, 23, 64, 320, 1, 1, 1, "SAME"),        # Ncol not a multiple of 128
]


@pytest.fixture(params=["classic", "glds", "classic_n64", "glds_n64", "onebuf", "onebuf_n64",
                        "tall512", "tall256", "small", "gshort64", "gshort128",
                        "gshort64_3", "gshort128_3", "multi2", "multi4", "small_multi4",
                        "gmulti64", "gmulti128", "gbig256", "gbig512", "generic",
                        "sk128", "g8p", "onebuf_n64_e", "classic_n64_e", "db",
                        "gbig256_32", "gshort128_32", "gshort64_32", "gbig224", "gbig448"])
def ig_algo(request, monkeypatch):
    """Runs a test once per igemm kernel (register-staged / LDS-DMA ring /
    single LDS stage, 128- or 64-channel-wide tiles)."""
    from kf_benchmarks_amd.ops import conv_hip
    monkeypatch.setattr(conv_hip, "_IG_FORCE", conv_hip.IG_ALGOS[request.param])
    return request.param


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_conv_fwd_bwd(cuda, shape, dt, ig_algo):
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


# (N, H, W, Cin, Cout, KH, KW): tile counts around the stream-K boundaries
# (P = 512 slots): fewer tiles than slots, several data-parallel rounds plus a
# split tail, and a 1-tile launch whose 18 K steps span many workgroups
SK_SHAPES = [
    (16, 100, 100, 128, 128, 3, 3),   # 1250 tiles: 512 data-parallel + 738 split
    (8, 14, 14, 256, 256, 3, 3),      # 25 x 2 tiles, K = 2304
    (1, 7, 7, 512, 256, 3, 3),        # one 128-row tile x 2, 72 K steps
    (4, 28, 28, 1024, 256, 1, 1),     # 1x1, 25 x 2 tiles
]


@pytest.mark.parametrize("shape", SK_SHAPES, ids=[str(s) for s in SK_SHAPES])
def test_stream_k_matches_one_tile_kernel(cuda, shape):
    """Stream-K (IG_SK128) against the one-tile LDS-DMA kernel of the same
    tile on the same operands: equal to fp32-rounding of the split sums, and
    bitwise repeatable (the last contributor sums the partials in fixed
    order; the tickets reset themselves between launches)."""
    from kf_benchmarks_amd.ops import conv_hip
    n, H, W, cin, cout, kh, kw = shape
    g = torch.Generator().manual_seed(3)
    x = torch.randn(n, H, W, cin, generator=g).to(cuda, torch.bfloat16)
    w = (torch.randn(cout, kh, kw, cin, generator=g) / (kh * kw * cin) ** 0.5).to(
        cuda, torch.bfloat16)
    wmat = w.reshape(cout, -1).contiguous()
    pt, pl = (kh - 1) // 2, (kw - 1) // 2
    geo = (n, H, W, cin, H, W, kh, kw, 1, 1, pt, pl, cout, H, W, 1, cout, 0)
    outs = {}
    for algo in ("gshort128", "sk128", "sk128", "sk128"):
        y = torch.empty(n, H, W, cout, device=cuda, dtype=torch.bfloat16)
        stats = torch.zeros(2 * conv_hip.STATS_SPREAD * cout, device=cuda)
        conv_hip._igemm_call(conv_hip.IG_ALGOS[algo], x, wmat, y, geo, stats)
        outs.setdefault(algo, []).append((y, stats))
    torch.cuda.synchronize()
    ref, sref = outs["gshort128"][0]
    y0, s0 = outs["sk128"][0]
    torch.testing.assert_close(y0.float(), ref.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(s0.view(2, -1, cout).sum(1), sref.view(2, -1, cout).sum(1),
                               rtol=1e-3, atol=1e-1)
    for y1, _ in outs["sk128"][1:]:
        assert torch.equal(y1, y0)
    want = conv_ops.conv2d_reference(x.float().cpu(), w.float().cpu(), (1, 1),
                                     F.resolve_pads("SAME", H, W, kh, kw, 1, 1))
    torch.testing.assert_close(y0.float().cpu(), want, rtol=2e-2, atol=2e-2)


FUSED_SHAPES = [
    (2, 14, 14, 64, 256, 1, 1, 1, "SAME"),
    (2, 7, 7, 128, 128, 3, 3, 1, "SAME_RESNET"),     # M=98 < one tile
    (3, 9, 9, 64, 96, 3, 3, 2, "SAME_RESNET"),       # transposed gather
    (4, 2, 2, 512, 2048, 1, 1, 1, "SAME"),           # M=16
    (2, 13, 13, 64, 128, 1, 1, 2, "SAME"),           # scatter (addend only)
    (2, 20, 20, 128, 192, 3, 3, 1, "SAME_RESNET"),   # M = 800: 256-row tiles + remainder
    # MobileNet-v2 projection / expansion widths (ReLU6 bit masks since round 6):
    # dX channels not a multiple of 64
    (2, 14, 14, 144, 24, 1, 1, 1, "SAME"),
    (2, 9, 9, 96, 40, 3, 3, 1, "SAME_RESNET"),
]


def pack_relu_bits(y):
    """Host form of the BN apply pass's ReLU bit mask (csrc/bn.hip relu_bits):
    bit k of byte e/8 = y[e + k] > 0 over the flattened tensor."""
    b = (y.float().reshape(-1, 8) > 0).to(torch.int32)
    return (b * (1 << torch.arange(8, dtype=torch.int32))).sum(1).to(torch.uint8)


@pytest.mark.parametrize("shape", FUSED_SHAPES, ids=[str(s) for s in FUSED_SHAPES])
@pytest.mark.parametrize("with_addend", [False, True])
@pytest.mark.parametrize("mask_src", ["read", "recompute", "bits"])
def test_dgrad_fused_epilogue(cuda, shape, with_addend, ig_algo, mask_src):
    """dgrad epilogue: dX = (conv^T(dY) + addend) * [x > 0] and the producer
    BN's backward partials sum(dX), sum(dX * (x_bn - mean)) per channel.  The
    ReLU mask is read from x (the BN output), from its bit mask (one byte
    per 8 channels, IgArgs::maskbits) or recomputed as x_bn * scale + shift > 0
    (BNs without a residual add)."""
    from kf_benchmarks_amd.ops import conv_hip
    n, H, W, cin, cout, kh, kw, s, mode = shape
    scatter = kh == 1 and s > 1
    if scatter and not with_addend:
        pytest.skip("scatter path: the BN epilogue needs the (sparse) pending gradient")
    g = torch.Generator().manual_seed(1)
    dt = torch.bfloat16
    x = torch.randn(n, H, W, cin, generator=g).to(dt)
    w = (torch.randn(cout, kh, kw, cin, generator=g) / (kh * kw * cin) ** 0.5).to(dt)
    pads = F.resolve_pads(mode, H, W, kh, kw, s, s)
    yb = conv_ops.conv2d_reference(x.float(), w.float(), (s, s), pads)
    dy = torch.randn(yb.shape, generator=g).to(dt)
    xb = torch.randn(n, H, W, cin, generator=g).to(dt)
    mean = torch.randn(cin, generator=g)
    mcoef = None
    if mask_src == "recompute":
        # x = relu(xb * scale + shift) as the BN forward stores it
        scale, shift = torch.rand(cin, generator=g) + 0.5, torch.randn(cin, generator=g) * 0.5
        x = torch.relu(xb.float() * scale + shift).to(dt)
        mcoef = torch.cat([scale, shift])
    add = torch.randn(n, H, W, cin, generator=g).to(dt) if with_addend else None
    if scatter:
        # the other contributor was a scatter of the same stride: zero off-grid
        keep = torch.zeros(n, H, W, 1, dtype=dt)
        keep[:, ::s, ::s] = 1
        add = add * keep
    xr = x.float().requires_grad_(True)
    conv_ops.conv2d_reference(xr, w.float(), (s, s), pads).backward(dy.float())
    ref = xr.grad + (add.float() if add is not None else 0)
    parts = None
    fuse = None
    if True:
        ref = ref * (x.float() > 0)
        parts = conv_hip.stats_buffer(cin, cuda).zero_()
        if mask_src == "bits":
            fuse = (parts, pack_relu_bits(x).to(cuda), xb.to(cuda), mean.to(cuda))
        elif mcoef is None:
            fuse = (parts, x.to(cuda), xb.to(cuda), mean.to(cuda))
        else:
            fuse = (parts, None, xb.to(cuda), mean.to(cuda), mcoef.to(cuda))
    dx = conv_hip.conv_dgrad(dy.to(cuda), w.to(cuda), x.shape, (s, s), pads, fuse,
                             addend=add.to(cuda) if add is not None else None)
    torch.testing.assert_close(dx.float().cpu(), ref, rtol=3e-2, atol=3e-2)
    if parts is not None:
        p = parts.view(2, conv_hip.STATS_SPREAD, cin).sum(1).cpu()
        r = dx.float().cpu()
        s1 = r.sum((0, 1, 2))
        s2 = (r * (xb.float() - mean)).sum((0, 1, 2))
        tol = 4e-3 * (r.abs() * (1 + (xb.float() - mean).abs())).sum((0, 1, 2)).max().item()
        torch.testing.assert_close(p[0], s1, rtol=1e-2, atol=tol)
        torch.testing.assert_close(p[1], s2, rtol=1e-2, atol=tol)


@pytest.mark.parametrize("cin,cout", [(144, 24), (96, 24), (576, 96), (960, 160), (32, 16)])
@pytest.mark.parametrize("algo", ["auto", "s1"])
def test_dgrad_bits_mobilenet_widths(cuda, monkeypatch, cin, cout, algo):
    """The 1x1 dgrad with the producer BN's bit mask, pending gradient and
    partial sums at MobileNet-v2 widths (dX channels 32-960, not multiples of
    64), autotuned or on the streaming 1x1 kernel where it applies."""
    from kf_benchmarks_amd.ops import conv_hip
    if algo == "s1":
        if not conv_hip.N.load().kfb_conv_s1_applicable(cout, cin, 1, 1, 1, 1, 0, 0, 28, 28, 28, 28):
            pytest.skip("streaming 1x1 kernel does not apply")
        monkeypatch.setattr(conv_hip, "_IG_FORCE", conv_hip.IG_S1)
    g = torch.Generator().manual_seed(7)
    dt = torch.bfloat16
    n, H, W = 4, 28, 28
    x = torch.relu(torch.randn(n, H, W, cin, generator=g)).clamp(max=6.0).to(dt)
    x[torch.rand(x.shape, generator=g) < 0.2] = 6.0  # clamped outputs: gate closed
    w = (torch.randn(cout, 1, 1, cin, generator=g) / cin ** 0.5).to(dt)
    dy = torch.randn(n, H, W, cout, generator=g).to(dt)
    xb = torch.randn(n, H, W, cin, generator=g).to(dt)
    mean = torch.randn(cin, generator=g)
    add = torch.randn(n, H, W, cin, generator=g).to(dt)
    gate = (x.float() > 0) & (x.float() < 6)
    b = gate.reshape(-1, 8).to(torch.int32)
    bits = (b * (1 << torch.arange(8, dtype=torch.int32))).sum(1).to(torch.uint8)
    ref = (dy.float().reshape(-1, cout) @ w.float().reshape(cout, cin)).reshape(n, H, W, cin)
    ref = (ref + add.float()) * gate
    parts = conv_hip.stats_buffer(cin, cuda).zero_()
    dx = conv_hip.conv_dgrad(dy.to(cuda), w.to(cuda), x.shape, (1, 1), (0, 0, 0, 0),
                             (parts, bits.to(cuda), xb.to(cuda), mean.to(cuda)),
                             addend=add.to(cuda))
    torch.testing.assert_close(dx.float().cpu(), ref, rtol=3e-2, atol=3e-2)
    p = parts.view(2, conv_hip.STATS_SPREAD, cin).sum(1).cpu()
    r = dx.float().cpu()
    tol = 4e-3 * (r.abs() * (1 + (xb.float() - mean).abs())).sum((0, 1, 2)).max().item()
    torch.testing.assert_close(p[0], r.sum((0, 1, 2)), rtol=1e-2, atol=tol)
    torch.testing.assert_close(p[1], (r * (xb.float() - mean)).sum((0, 1, 2)), rtol=1e-2,
                               atol=tol)


@pytest.mark.parametrize("shape", FUSED_SHAPES[:4], ids=[str(s) for s in FUSED_SHAPES[:4]])
def test_fwd_stats_epilogue(cuda, shape, ig_algo):
    from kf_benchmarks_amd.ops import conv_hip
    n, H, W, cin, cout, kh, kw, s, mode = shape
    g = torch.Generator().manual_seed(2)
    x = torch.randn(n, H, W, cin, generator=g).to(torch.bfloat16)
    w = (torch.randn(cout, kh, kw, cin, generator=g) / (kh * kw * cin) ** 0.5).to(torch.bfloat16)
    pads = F.resolve_pads(mode, H, W, kh, kw, s, s)
    st = conv_hip.stats_buffer(cout, cuda).zero_()
    y = conv_hip.conv_fwd(x.to(cuda), w.to(cuda), (s, s), pads, st).float().cpu()
    p = st.view(2, conv_hip.STATS_SPREAD, cout).sum(1).cpu()
    tol = 4e-3 * (y.abs() + y * y).sum((0, 1, 2)).max().item()
    torch.testing.assert_close(p[0], y.sum((0, 1, 2)), rtol=1e-2, atol=tol)
    torch.testing.assert_close(p[1], (y * y).sum((0, 1, 2)), rtol=1e-2, atol=tol)


DW_SHAPES = [(2, 14, 14, 32, 3, 1), (2, 15, 15, 24, 3, 2), (2, 9, 9, 16, 5, 1),
             (1, 11, 11, 8, 7, 2), (2, 8, 8, 11, 3, 1),
             # filter gradient: > 256 channel groups (two chunks, the second
             # partial), 256 % groups != 0 (idle lanes), many workgroups
             (2, 7, 7, 2560, 3, 1), (4, 28, 28, 144, 3, 1), (16, 56, 56, 32, 3, 2),
             (2, 12, 12, 44, 5, 1), (2, 12, 12, 40, 7, 1),
             (2, 12, 12, 16, 9, 1)]  # 9 columns: two column groups per filter row


@pytest.mark.parametrize("shape", DW_SHAPES, ids=[str(s) for s in DW_SHAPES])
def test_depthwise_fwd_bwd(cuda, shape):
    """csrc/depthwise.hip fwd / dgrad / wgrad vs the fp32 PyTorch grouped conv."""
    from kf_benchmarks_amd.ops import depthwise as dw
    n, H, W, C, k, s = shape
    g = torch.Generator().manual_seed(4)
    dt = torch.bfloat16
    x = torch.randn(n, H, W, C, generator=g).to(dt).float()
    w = (torch.randn(k, k, C, generator=g) / k).to(dt).float()
    pads = F.resolve_pads("SAME", H, W, k, k, s, s)
    xa = x.to(cuda, dt).requires_grad_(True)
    wa = w.to(cuda).requires_grad_(True)
    ya = dw.depthwise_conv2d(xa, wa, wa.detach().to(dt), (s, s), pads, "hip")
    xb = x.clone().requires_grad_(True)
    wb = w.clone().requires_grad_(True)
    yb = dw.depthwise_reference(xb, wb, (s, s), pads)
    torch.testing.assert_close(ya.float().cpu(), yb, rtol=2e-2, atol=2e-2)
    dy = torch.randn(yb.shape, generator=g).to(dt).float()
    ya.backward(dy.to(cuda, dt))
    yb.backward(dy)
    torch.testing.assert_close(xa.grad.float().cpu(), xb.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(wa.grad.cpu(), wb.grad, rtol=3e-2,
                               atol=2e-2 * wb.grad.abs().max().item())


@pytest.mark.parametrize("products,tol", [("exact", 1e-5), ("bf16x3", 1e-4)])
@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_conv_fp32_fwd_bwd(cuda, shape, products, tol, monkeypatch):
    """fp32 convs (csrc/conv_f32.hip) vs the CPU fp64 reference: forward,
    data and weight gradients.  exact: fp32 MFMA products (error at fp32
    rounding); bf16x3: three bf16 MFMAs per product on the operands' bf16
    splits (~2^-16 per product, far below TF32's 2^-11)."""
    from kf_benchmarks_amd.ops import conv_f32
    monkeypatch.setattr(conv_f32, "_products", products)
    n, H, W, cin, cout, kh, kw, s, mode = shape
    torch.manual_seed(0)
    x = torch.randn(n, H, W, cin)
    w = torch.randn(cout, kh, kw, cin) / (kh * kw * cin) ** 0.5
    pads = F.resolve_pads(mode, H, W, kh, kw, s, s)
    xa = x.to(cuda).requires_grad_(True)
    wa = w.to(cuda).requires_grad_(True)
    ya = conv_ops.conv2d(xa, wa, None, (s, s), pads, "hip")
    xb = x.clone().double().requires_grad_(True)
    wb = w.clone().double().requires_grad_(True)
    yb = conv_ops._torch_conv(xb, wb, (s, s), pads)
    assert ya.dtype == torch.float32 and ya.shape == yb.shape
    dy = torch.randn(yb.shape)
    ya.backward(dy.to(cuda))
    yb.backward(dy.double())
    for got, ref in ((ya, yb), (xa.grad, xb.grad), (wa.grad, wb.grad)):
        err = float((got.detach().cpu().double() - ref.detach()).abs().max()
                    / (ref.detach().abs().max() + 1e-12))
        assert err < tol, err
        if products == "bf16x3":  # genuinely more precise than one bf16 product
            assert err > 0


BACT_SHAPES = [
    (2, 14, 14, 64, 256, 3, 3, 1, "SAME"),
    (2, 17, 17, 3, 64, 3, 3, 1, "SAME"),          # RGB input (channel pad)
    (2, 13, 13, 96, 36, 1, 1, 1, "SAME"),         # Cout not a multiple of 8
    (2, 32, 32, 3, 64, 7, 7, 2, "SAME_RESNET"),   # s2d stem path
]


@pytest.mark.parametrize("shape", BACT_SHAPES, ids=[str(s) for s in BACT_SHAPES])
@pytest.mark.parametrize("relu", [True, False])
def test_conv_bias_relu_epilogue(cuda, shape, relu):
    """conv + bias (+ ReLU) fused in the forward epilogue (VGG/AlexNet-style
    layers without BN); backward = one mask + bias-sum pass, then dgrad /
    wgrad; vs the fp32 CPU reference."""
    n, H, W, cin, cout, kh, kw, s, mode = shape
    torch.manual_seed(2)
    dt = torch.bfloat16
    x = torch.randn(n, H, W, cin).to(dt).float()
    w = (torch.randn(cout, kh, kw, cin) / (kh * kw * cin) ** 0.5).to(dt).float()
    b = torch.randn(cout) * 0.3
    pads = F.resolve_pads(mode, H, W, kh, kw, s, s)
    xa = x.to(cuda, dt).requires_grad_(True)
    wa = w.to(cuda).requires_grad_(True)
    ba = b.to(cuda).requires_grad_(True)
    assert conv_ops.fuses_bias_act(xa)
    ya = conv_ops.conv2d(xa, wa, wa.detach().to(dt), (s, s), pads, "hip", bias=ba, relu=relu)
    xb, wb, bb = (t.clone().requires_grad_(True) for t in (x, w, b))
    ylin = conv_ops.conv2d_reference(xb, wb, (s, s), pads) + bb
    yb = torch.relu(ylin) if relu else ylin
    torch.testing.assert_close(ya.float().cpu(), yb.detach(), rtol=2e-2, atol=2e-2)
    dy = torch.randn(yb.shape).to(dt).float()
    ya.backward(dy.to(cuda, dt))
    # the ReLU mask of the kernel's own (bf16-rounded) output decides ties at 0
    mask = (ya.detach().float().cpu() > 0).float() if relu else 1.0
    ylin.backward(dy * mask)
    scale = dy.abs().mean().item()
    torch.testing.assert_close(xa.grad.float().cpu(), xb.grad, rtol=3e-2, atol=3e-2 * scale * 4)
    torch.testing.assert_close(wa.grad.cpu(), wb.grad, rtol=3e-2,
                               atol=2e-2 * wb.grad.abs().max().item())
    torch.testing.assert_close(ba.grad.cpu(), bb.grad, rtol=2e-2, atol=2e-2 * scale * 50)


@pytest.mark.parametrize("shifted", [True, False])
def test_bn_stats_large_mean_shifted(cuda, shifted):
    """Conv-epilogue BN statistics of a channel whose mean is ~500x its
    spread (fp16 identity 1x1 conv over 500 + N(0, 1)): with the partials
    centered on the previous batch mean (stats_buffer(shift=...), as the
    model builder wires it) the batch variance is exact to fp32 rounding,
    and the BN writes this step's mean back as the next step's shift."""
    from kf_benchmarks_amd.ops import conv_hip
    g = torch.Generator().manual_seed(11)
    C = 64
    x = (500.0 + torch.randn(16, 16, 16, C, generator=g)).to(torch.float16)
    w = torch.eye(C).view(C, 1, 1, C).to(torch.float16)
    shift = torch.full((C,), 499.5, device=cuda) if shifted else None
    st = conv_hip.stats_buffer(C, cuda, shift=shift).zero_()
    y = conv_hip.conv_fwd(x.to(cuda), w.to(cuda), (1, 1), (0, 0, 0, 0), st)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    out = F.batch_norm(y, None, torch.zeros(C, device=cuda), rm, rv, 0.9, 1e-5, True,
                       stats=st).double().cpu()
    yd = y.double().cpu().view(-1, C)
    mean, var = yd.mean(0), yd.var(0, unbiased=False)
    ref = ((yd - mean) / (var + 1e-5).sqrt()).view(out.shape)
    if shifted:
        torch.testing.assert_close(out, ref, rtol=0, atol=2e-2)
        torch.testing.assert_close(shift.double().cpu(), mean, rtol=0, atol=1e-3)
        # running variance (unbiased, decay 0.9) from the exact batch variance
        n = yd.shape[0]
        torch.testing.assert_close(rv.double().cpu(), 0.9 + 0.1 * var * n / (n - 1),
                                   rtol=1e-3, atol=0)
    else:  # uncentered fp32 partials: finite, but only the shifted path is pinned
        assert torch.isfinite(out).all()


@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("consumers", [1, 2])
def test_act_link_fused_backward(cuda, relu, consumers, monkeypatch):
    """conv+bias(+ReLU) -> conv(s) without BN (VGG/AlexNet): the consumers'
    dgrad epilogue applies the producer's ReLU mask and sums its bias
    gradient (act link, _Conv2d.forward), so the producer runs no separate
    act/bias backward pass; vs the fp32 CPU reference."""
    from kf_benchmarks_amd.ops import conv_hip
    monkeypatch.setattr(conv_hip, "_ACT_FUSE", True)  # opt-in (KFB_ACT_FUSE=1)
    calls = []
    real = conv_hip._bias_act_backward
    monkeypatch.setattr(conv_hip, "_bias_act_backward",
                        lambda *a: calls.append(1) or real(*a))
    torch.manual_seed(5)
    dt = torch.bfloat16
    n, H, W, c0, c1, c2 = 4, 12, 12, 32, 64, 48
    x = torch.randn(n, H, W, c0).to(dt).float()
    w1 = (torch.randn(c1, 3, 3, c0) / (9 * c0) ** 0.5).to(dt).float()
    b1 = torch.randn(c1) * 0.3
    w2s = [(torch.randn(c2, 3, 3, c1) / (9 * c1) ** 0.5).to(dt).float() for _ in range(consumers)]
    pads = F.resolve_pads("SAME", H, W, 3, 3, 1, 1)
    xa = x.to(cuda, dt).requires_grad_(True)
    w1a, b1a = w1.to(cuda).requires_grad_(True), b1.to(cuda).requires_grad_(True)
    w2a = [w.to(cuda).requires_grad_(True) for w in w2s]
    y1 = conv_ops.conv2d(xa, w1a, w1a.detach().to(dt), (1, 1), pads, "hip", bias=b1a, relu=relu)
    link = y1._kfb_bn_link  # the builder counts the consumers (ConvNetBuilder._use)
    link.convs += consumers
    outs = [conv_ops.conv2d(y1, w, w.detach().to(dt), (1, 1), pads, "hip") for w in w2a]
    dys = [torch.randn(o.shape).to(dt).float() for o in outs]
    sum((o.float() * d.to(cuda)).sum() for o, d in zip(outs, dys)).backward()
    assert not calls, "producer ran its own act/bias backward pass"
    # reference, with the kernel's own (bf16-rounded) output deciding the mask
    xb, w1b, b1b = (t.clone().requires_grad_(True) for t in (x, w1, b1))
    w2b = [w.clone().requires_grad_(True) for w in w2s]
    ylin = conv_ops.conv2d_reference(xb, w1b, (1, 1), pads) + b1b
    mask = (y1.detach().float().cpu() > 0).float() if relu else torch.ones_like(ylin)
    y1b = ylin * mask
    sum((conv_ops.conv2d_reference(y1b, w, (1, 1), pads) * d).sum()
        for w, d in zip(w2b, dys)).backward()
    gs = max(t.grad.abs().max().item() for t in (xb,))
    torch.testing.assert_close(xa.grad.float().cpu(), xb.grad, rtol=3e-2, atol=3e-2 * gs)
    torch.testing.assert_close(w1a.grad.cpu(), w1b.grad, rtol=3e-2,
                               atol=2e-2 * w1b.grad.abs().max().item())
    torch.testing.assert_close(b1a.grad.cpu(), b1b.grad, rtol=2e-2,
                               atol=2e-2 * b1b.grad.abs().max().item())
    for wa, wb in zip(w2a, w2b):
        torch.testing.assert_close(wa.grad.cpu(), wb.grad, rtol=3e-2,
                                   atol=2e-2 * wb.grad.abs().max().item())


# (N, H, W, Cin, Cout, KH, KW, stride, mode): LDS-DMA wgrad geometries - 3x3
# gathers with padding, a strided gather, plain 1x1, Cout / K not multiples of
# 128, reduction lengths not multiples of the 64-row step
WGRAD_SHAPES = [
    (4, 14, 14, 64, 128, 3, 3, 1, "SAME_RESNET"),
    (2, 13, 13, 128, 192, 3, 3, 1, "SAME_RESNET"),
    (3, 15, 15, 64, 256, 1, 1, 2, "SAME"),
    (5, 7, 7, 256, 128, 1, 1, 1, "SAME"),
    (2, 9, 11, 32, 136, 3, 3, 2, "VALID"),
]


@pytest.mark.parametrize("shape", WGRAD_SHAPES, ids=[str(s) for s in WGRAD_SHAPES])
@pytest.mark.parametrize("target", [1024, 64])
def test_wgrad_glds_kernel(cuda, shape, target):
    """wgrad_glds_k (forced: bit 16 of the launch target) vs the fp32
    reference; target 1024 splits the reduction into slabs, 64 keeps one
    split (fp32 atomics epilogue)."""
    from kf_benchmarks_amd.ops import conv_hip
    n, H, W, cin, cout, kh, kw, s, mode = shape
    g = torch.Generator().manual_seed(5)
    x = torch.randn(n, H, W, cin, generator=g).to(torch.bfloat16)
    pads = F.resolve_pads(mode, H, W, kh, kw, s, s)
    w = torch.randn(cout, kh, kw, cin, generator=g)
    y = conv_ops.conv2d_reference(x.float(), w, (s, s), pads)
    dy = torch.randn(y.shape, generator=g).to(torch.bfloat16)
    xb = x.float().requires_grad_(True)
    wb = w.clone().requires_grad_(True)
    conv_ops.conv2d_reference(xb, wb, (s, s), pads).backward(dy.float())
    want = wb.grad
    geo = (n, H, W, cin, y.shape[1], y.shape[2], kh, kw, s, s, pads[0], pads[2], cout)
    for t in (target, target | conv_hip._WGRAD_GLDS):
        dw = torch.zeros(cout, kh, kw, cin, device=cuda)
        conv_hip._wgrad_launch(dy.to(cuda), x.to(cuda), dw, geo, t)
        torch.testing.assert_close(dw.cpu(), want, rtol=2e-3, atol=2e-3 * want.abs().max().item())


@pytest.mark.parametrize("dual", [False, True])
@pytest.mark.parametrize("shape", [(2, 7, 7, 64), (4, 14, 14, 256), (1, 3, 5, 8)])
def test_bn_apply_writes_relu_bits(cuda, shape, dual):
    """The residual / dual BN apply pass writes y's ReLU bit mask (the byte a
    consumer dgrad epilogue reads instead of y): equal to packing y > 0."""
    from kf_benchmarks_amd.ops import conv_hip
    n, H, W, C = shape
    g = torch.Generator().manual_seed(3)
    dt = torch.bfloat16
    x = torch.randn(n, H, W, C, generator=g).to(dt).to(cuda)
    gamma = (torch.rand(C, generator=g).to(cuda) + 0.5).requires_grad_(True)
    beta = torch.randn(C, generator=g).to(cuda).requires_grad_(True)
    stats = conv_hip.stats_buffer(C, cuda).zero_()
    xs = x.float().reshape(-1, C)
    stats.view(2, conv_hip.STATS_SPREAD, C)[0, 0] = xs.sum(0)
    stats.view(2, conv_hip.STATS_SPREAD, C)[1, 0] = (xs * xs).sum(0)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    if dual:
        xr = torch.randn(n, H, W, C, generator=g).to(dt).to(cuda)
        sr = conv_hip.stats_buffer(C, cuda).zero_()
        xrs = xr.float().reshape(-1, C)
        sr.view(2, conv_hip.STATS_SPREAD, C)[0, 0] = xrs.sum(0)
        sr.view(2, conv_hip.STATS_SPREAD, C)[1, 0] = (xrs * xrs).sum(0)
        r = F.DeferredBN(xr, gamma, beta, rm.clone(), rv.clone(), 0.9, 1e-3, sr)
        y = F.batch_norm_dual(x, gamma, beta, rm, rv, 0.9, 1e-3, True, stats, r)
    else:
        res = torch.randn(n, H, W, C, generator=g).to(dt).to(cuda)
        y = F.batch_norm(x, gamma, beta, rm, rv, 0.9, 1e-3, True, True, res, stats=stats)
    link = y._kfb_bn_link
    assert link.mbits is not None and link.mbits.dtype == torch.uint8
    torch.cuda.synchronize()
    assert torch.equal(link.mbits.cpu(), pack_relu_bits(y.detach().cpu()))
