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
