"""In-kernel BN finalize (csrc/igemm_args.h BnFin): the last workgroup of
the conv that accumulates a BN's statistics folds them into mean / invstd,
scale / shift, the running statistics and the statistics shift - checked
against the same quantities computed from the conv output on the host, for
every igemm kernel family (one-tile, multi-tile, LDS-DMA, 8-phase, the
streaming 3x3 kernel, and stream-K, which takes the separate finalize
launch instead), and end to end: a ResNet trains the same with the
finalize in the conv as with the BN's own finalize launch."""

import pytest
import torch

from kf_benchmarks_amd.ops import conv_hip
from kf_benchmarks_amd.ops import nn as F

pytestmark = pytest.mark.gpu

CASES = [
    ((4, 14, 14, 64, 64, 3, 3), "onebuf"),
    ((4, 14, 14, 64, 256, 1, 1), "multi2"),
    ((4, 14, 14, 128, 128, 3, 3), "gshort128"),
    ((2, 28, 28, 64, 256, 1, 1), "gmulti64"),
    ((4, 16, 16, 256, 256, 1, 1), "g8p"),
    ((8, 28, 28, 64, 64, 3, 3), "s3"),
    ((4, 14, 14, 128, 128, 3, 3), "sk128"),
]


@pytest.mark.parametrize("case", CASES, ids=[c[1] for c in CASES])
def test_conv_finalizes_bn(cuda, monkeypatch, case):
    (n, H, W, cin, cout, kh, kw), algo = case
    monkeypatch.setattr(conv_hip, "_IG_FORCE", conv_hip.IG_ALGOS[algo])
    monkeypatch.setattr(conv_hip, "_BN_FIN_MODE", "1")
    g = torch.Generator().manual_seed(4)
    x = torch.randn(n, H, W, cin, generator=g).to(torch.bfloat16).to(cuda)
    w = (torch.randn(cout, kh, kw, cin, generator=g) / (kh * kw * cin) ** 0.5).to(torch.bfloat16)
    w = w.to(cuda)
    pads = F.resolve_pads("SAME_RESNET", H, W, kh, kw, 1, 1)
    gamma = (torch.rand(cout, generator=g) + 0.5).to(cuda)
    beta = torch.randn(cout, generator=g).to(cuda)
    shift = (torch.randn(cout, generator=g) * 0.1).to(cuda)
    rm0 = torch.randn(cout, generator=g).to(cuda)
    rv0 = (torch.rand(cout, generator=g) + 0.5).to(cuda)
    rm, rv = rm0.clone(), rv0.clone()
    st = torch.zeros(2, cout, device=cuda)
    coef = torch.zeros(2 * cout, device=cuda)
    kshift = shift.clone()
    stats = conv_hip.stats_buffer(cout, cuda, shift=kshift).zero_()
    stats._kfb_counter.zero_()
    decay, eps = 0.9, 1e-3
    conv_hip.attach_bn_finalize(stats, gamma, beta, rm, rv, decay, eps, st, coef)
    y = conv_hip.conv_fwd(x, w, (1, 1), pads, stats)
    torch.cuda.synchronize()
    assert stats._kfb_finalized
    yd = y.double().reshape(-1, cout)
    rows = yd.shape[0]
    mean = yd.mean(0)
    var = yd.var(0, unbiased=False)
    invstd = 1.0 / torch.sqrt(var + eps)
    tol = dict(rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(st[0].double(), mean, **tol)
    torch.testing.assert_close(st[1].double(), invstd, rtol=5e-3, atol=5e-3)
    torch.testing.assert_close(coef[:cout].double(), gamma.double() * invstd, rtol=5e-3,
                               atol=5e-3)
    torch.testing.assert_close(coef[cout:].double(),
                               beta.double() - mean * gamma.double() * invstd, rtol=5e-3,
                               atol=5e-3)
    torch.testing.assert_close(rm.double(), rm0.double() * decay + mean * (1 - decay), **tol)
    unb = var * rows / (rows - 1)
    torch.testing.assert_close(rv.double(), rv0.double() * decay + unb * (1 - decay), **tol)
    torch.testing.assert_close(kshift.double(), mean, **tol)  # next step's shift


@pytest.mark.parametrize("force", [None, "s1"])
def test_resnet_trains_same_with_in_kernel_finalize(cuda, monkeypatch, force):
    """ResNet-50 at batch 8: the finalize in the conv's last workgroup and
    the BN's own finalize launch give the same training trajectory (up to
    the run-to-run spread of the statistics atomics).  force="s1": every
    eligible 1x1 conv on the streaming kernel, whose dgrad form also runs the
    producer BN's backward finalize in its last workgroup (BnGFin)."""
    from kf_benchmarks_amd import params as P
    from kf_benchmarks_amd.benchmark import BenchmarkCNN

    if force is not None:
        monkeypatch.setattr(conv_hip, "_IG_FORCE", conv_hip.IG_ALGOS[force])

    def run(fin):
        monkeypatch.setattr(conv_hip, "_BN_FIN", fin)
        monkeypatch.setattr(conv_hip, "_BN_FIN_MODE", "1" if fin else "0")
        p = P.make_params(model="resnet50", batch_size=8, num_gpus=1, use_bf16=True,
                          optimizer="momentum", data_format="NHWC", variable_update="kungfu",
                          init_learning_rate=0.002, display_every=10 ** 9)
        b = BenchmarkCNN(p)
        b.build()
        losses = [float(b.train_step(need_loss=True)[0]) for _ in range(4)]
        torch.cuda.synchronize()
        bufs = {k: t.detach().float().cpu().clone() for k, t in b.net.named_buffers()
                if k.endswith("moving_mean") or k.endswith("moving_variance")}
        return losses, bufs

    # (batch 8 has more pixel tiles than statistics slots, so even two
    # runs of one configuration differ in the last bits and bf16 training
    # amplifies that: the bound is the eager-vs-eager spread, as in
    # tests/test_tape_gpu.py)
    lb, bb = run(False)
    lb2, bb2 = run(False)
    la, ba = run(True)
    spread = 0.0
    for x, y, y2 in zip(la, lb, lb2):
        spread = max(spread, abs(y - y2))
        assert abs(x - y) <= max(4 * spread, 2.5e-2 * max(1.0, abs(y))), (la, lb, lb2)
    for k in bb:
        ref = (bb[k] - bb2[k]).abs().max().item()
        assert (ba[k] - bb[k]).abs().max().item() <= max(8 * ref, 2e-2 * bb[k].abs().max().item()
                                                         + 2e-3), k


@pytest.fixture
def fold_bwd(cuda):
    from kf_benchmarks_amd.ops import _native as N
    prev = N.load().kfb_bn_get_fold_bwd()
    yield lambda on: N.load().kfb_bn_set_fold_bwd(2 if on else 0)  # (2: at every size)
    N.load().kfb_bn_set_fold_bwd(prev)


def _bwd_case(cuda, rows, C, seed):
    g = torch.Generator().manual_seed(seed)
    t = dict(
        dy=torch.randn(rows, C, generator=g).to(torch.bfloat16).to(cuda),
        x=(torch.randn(rows, C, generator=g) * 2 + 0.3).to(torch.bfloat16).to(cuda),
        xr=torch.randn(rows, C, generator=g).to(torch.bfloat16).to(cuda),
        gamma=(torch.rand(C, generator=g) + 0.5).to(cuda),
        mean=(torch.randn(C, generator=g) * 0.1).to(cuda),
        invstd=(torch.rand(C, generator=g) + 0.5).to(cuda),
        # the 32 conv-epilogue slots of sum(dy') and sum(dy' (x - mean))
        parts=(torch.randn(2, 32, C, generator=g) * 50).to(cuda),
        gamma_r=(torch.rand(C, generator=g) + 0.5).to(cuda),
        mean_r=(torch.randn(C, generator=g) * 0.1).to(cuda),
        invstd_r=(torch.rand(C, generator=g) + 0.5).to(cuda))
    return t


@pytest.mark.parametrize("rows,C,dres", [(1000, 64, False), (12544, 2048, True),
                                         (6272, 256, False), (3136, 512, True)])
def test_bn_bwd_fold_matches_finalize_launch(cuda, fold_bwd, rows, C, dres):
    """The backward apply pass with the gradient finalize folded in (every
    workgroup folds its 64-channel slice of the conv-epilogue slots,
    bn_bwd_apply_fold_k) gives exactly the finalize launch + apply pass:
    coefficients, dgamma / dbeta (accumulated), dx and the residual
    gradient, bitwise."""
    from kf_benchmarks_amd.ops import _native as N
    t = _bwd_case(cuda, rows, C, 7 + C)
    out = {}
    for on in (False, True):
        fold_bwd(on)
        dx = torch.empty_like(t["dy"])
        dr = torch.empty_like(t["dy"]) if dres else None
        coef = torch.full((3, C), float("nan"), device=cuda)
        dgamma = torch.ones(C, device=cuda)
        dbeta = torch.ones(C, device=cuda)
        parts = t["parts"].clone()
        N.call("kfb_bn_bwd", N.dt(t["dy"]), t["dy"].data_ptr(), None, t["x"].data_ptr(),
               dx.data_ptr(), N.ptr(dr), rows, C, t["gamma"].data_ptr(), t["mean"].data_ptr(),
               t["invstd"].data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), parts[0].data_ptr(),
               parts[1].data_ptr(), 32, coef[0].data_ptr(), coef[1].data_ptr(),
               coef[2].data_ptr(), 0, 1, 1, N.stream(cuda))
        torch.cuda.synchronize()
        out[on] = (dx, dr, coef, dgamma, dbeta)
    for k, (a, b) in enumerate(zip(out[False], out[True])):
        if a is not None:
            assert torch.equal(a, b), k
    # against the formula on the host
    s1, s2 = t["parts"][0].double().sum(0), t["parts"][1].double().sum(0)
    A = t["gamma"].double() * t["invstd"].double()
    B = -A * t["invstd"].double() ** 2 * s2 / rows
    Cc = -A * s1 / rows - t["mean"].double() * B
    ref = t["dy"].double() * A + t["x"].double() * B + Cc
    torch.testing.assert_close(out[True][0].double(), ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(out[True][3].double(), 1 + s2 * t["invstd"].double(), rtol=1e-5,
                               atol=1e-3)


@pytest.mark.parametrize("rows,C", [(3136, 256), (12544, 2048)])
def test_bn_bwd_dual_fold_matches_finalize_launch(cuda, fold_bwd, rows, C):
    """kfb_bn_bwd_dual (y = relu(bn(x) + bn_r(xr)) backward) with the main
    BN's finalize folded into the apply pass equals the two finalize
    launches + apply, bitwise (the residual branch keeps its launch)."""
    from kf_benchmarks_amd.ops import _native as N
    t = _bwd_case(cuda, rows, C, 11 + C)
    out = {}
    for on in (False, True):
        fold_bwd(on)
        dx, dxr = torch.empty_like(t["dy"]), torch.empty_like(t["dy"])
        coef = torch.full((6, C), float("nan"), device=cuda)
        dg = torch.zeros(4, C, device=cuda)
        parts = t["parts"].clone()
        nr = 64
        pr = torch.zeros(2, nr, C, device=cuda)
        N.call("kfb_bn_bwd_dual", N.dt(t["dy"]), t["dy"].data_ptr(), t["x"].data_ptr(),
               t["xr"].data_ptr(), dx.data_ptr(), dxr.data_ptr(), rows, C,
               t["gamma"].data_ptr(), t["mean"].data_ptr(), t["invstd"].data_ptr(),
               dg[0].data_ptr(), dg[1].data_ptr(), parts[0].data_ptr(), parts[1].data_ptr(), 32,
               coef[0].data_ptr(), coef[1].data_ptr(), coef[2].data_ptr(), 0,
               t["gamma_r"].data_ptr(), t["mean_r"].data_ptr(), t["invstd_r"].data_ptr(),
               dg[2].data_ptr(), dg[3].data_ptr(), pr[0].data_ptr(), pr[1].data_ptr(), nr,
               coef[3].data_ptr(), coef[4].data_ptr(), coef[5].data_ptr(), 0, 0, N.stream(cuda))
        torch.cuda.synchronize()
        out[on] = (dx, dxr, coef, dg)
    for k, (a, b) in enumerate(zip(out[False], out[True])):
        assert torch.equal(a, b), k


@pytest.mark.parametrize("rows,C", [(3136, 256), (12544, 2048), (50176, 64)])
def test_bn_bwd_dual_fold_r_matches_finalize_launch(cuda, fold_bwd, rows, C):
    """kfb_bn_bwd_dual with the second BN's partials from the dual dgrad
    epilogue (partials_r_ready: its sum dy' is the first BN's slot array):
    folding that BN's finalize into the apply pass as well equals its
    finalize launch, bitwise (coefficients, dgamma / dbeta, dx, dxr)."""
    from kf_benchmarks_amd.ops import _native as N
    lib = N.load()
    t = _bwd_case(cuda, rows, C, 23 + C)
    pr = (torch.randn(32, C, generator=torch.Generator().manual_seed(C)) * 50).to(cuda)
    prev = lib.kfb_bn_get_fold_r()
    fold_bwd(True)
    out = {}
    try:
        for on in (False, True):
            lib.kfb_bn_set_fold_r(1 if on else 0)
            dx, dxr = torch.empty_like(t["dy"]), torch.empty_like(t["dy"])
            coef = torch.full((6, C), float("nan"), device=cuda)
            dg = torch.zeros(4, C, device=cuda)
            parts = t["parts"].clone()
            N.call("kfb_bn_bwd_dual", N.dt(t["dy"]), t["dy"].data_ptr(), t["x"].data_ptr(),
                   t["xr"].data_ptr(), dx.data_ptr(), dxr.data_ptr(), rows, C,
                   t["gamma"].data_ptr(), t["mean"].data_ptr(), t["invstd"].data_ptr(),
                   dg[0].data_ptr(), dg[1].data_ptr(), parts[0].data_ptr(), parts[1].data_ptr(),
                   32, coef[0].data_ptr(), coef[1].data_ptr(), coef[2].data_ptr(), 0,
                   t["gamma_r"].data_ptr(), t["mean_r"].data_ptr(), t["invstd_r"].data_ptr(),
                   dg[2].data_ptr(), dg[3].data_ptr(), parts[0].data_ptr(), pr.data_ptr(), 32,
                   coef[3].data_ptr(), coef[4].data_ptr(), coef[5].data_ptr(), 0, 1,
                   N.stream(cuda))
            torch.cuda.synchronize()
            out[on] = (dx, dxr, coef, dg)
    finally:
        lib.kfb_bn_set_fold_r(prev)
    for k, (a, b) in enumerate(zip(out[False], out[True])):
        assert torch.equal(a, b), k
    # the second BN against the formula on the host
    s1, s2 = t["parts"][0].double().sum(0), pr.double().sum(0)
    A = t["gamma_r"].double() * t["invstd_r"].double()
    B = -A * t["invstd_r"].double() ** 2 * s2 / rows
    Cc = -A * s1 / rows - t["mean_r"].double() * B
    ref = t["dy"].double() * A + t["xr"].double() * B + Cc
    torch.testing.assert_close(out[True][1].double(), ref, rtol=2e-2, atol=2e-2)
