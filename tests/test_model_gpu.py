"""Whole-network numerics on the GPU path (every fused kernel: conv + BN
statistics epilogue, dgrad + producer-BN ReLU/partials epilogue, direct
gradient sinks) against the CPU reference of the same network, weights and
inputs.

* fp32: GPU (our BN/pool/xent kernels, fp32 convs) must match the CPU fp32
  reference (per-variable cosine >= 0.999).
* bf16: compared with the CPU path run in bf16 (activations rounded to bf16
  at the same tensor boundaries).  BN backward at small batches amplifies
  rounding-order differences (dy - mean(dy) - xhat*mean(dy*xhat) cancels),
  so the bf16 check is on direction (cosine) rather than elementwise values;
  the fused-vs-unfused comparison pins the fusions themselves.
"""

import pytest
import torch

from kf_benchmarks_amd import datasets, optim, params as P
from kf_benchmarks_amd.models import model_config
from kf_benchmarks_amd.models.model import Network
from kf_benchmarks_amd.ops import conv as conv_ops

pytestmark = pytest.mark.gpu


def _grads(name, ds, dev, dtype, image_size=None, batch=4, seed=3):
    d = datasets.create_dataset(None, ds)
    m = model_config.get_model_config(name, d, P.make_params(model=name, data_name=ds))
    if image_size:
        m.image_size = image_size
    net = Network(m, d.num_classes, dev, dtype, seed=7)
    flat = optim.FlatParams(net, dtype if dtype != torch.float32 else None)
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(batch, m.image_size, m.image_size, 3, generator=g).to(dtype)
    y = torch.randint(0, d.num_classes - 1, (batch,), generator=g)
    flat.zero_grad()
    res = net(x.to(dev), phase_train=True)
    loss = m.loss_function((x, y.to(dev)), res)
    loss.backward()
    out = {n: p.grad.detach().float().cpu().clone() for n, p in net.trainable_variables()}
    return float(loss.detach()), out


def _cos(a, b):
    return float((a * b).sum() / (a.norm() * b.norm() + 1e-20))


# ResNet-50-class networks at random init have chaotic bf16 gradients: even
# the CPU bf16 path reaches only ~0.2 median cosine against CPU fp32
# (scripts/diag_grads.py; profiles/r1_grad_conditioning.txt), so their kernels
# are pinned in fp32 here and by the per-kernel bf16 tests in
# test_conv_gpu.py / test_kernels_gpu.py.  The bf16 whole-network checks run
# on well-conditioned networks (CPU bf16 min cosine > 0.9).
FP32_MODELS = [("resnet20", "cifar10", None, 4), ("resnet50", "imagenet", 64, 4),
               ("resnet50_v1.5", "imagenet", 64, 4), ("resnet50_v2", "imagenet", 64, 4),
               ("googlenet", "imagenet", 224, 2)]
BF16_MODELS = [("resnet20", "cifar10", None, 8), ("googlenet", "imagenet", 224, 2)]


@pytest.mark.parametrize("name,ds,size,batch", FP32_MODELS)
def test_network_grads_fp32(cuda, name, ds, size, batch):
    lr, gr = _grads(name, ds, "cpu", torch.float32, size, batch)
    lg, gg = _grads(name, ds, cuda, torch.float32, size, batch)
    assert abs(lr - lg) < 1e-3
    bad = [(k, _cos(gg[k], ref)) for k, ref in gr.items()
           if ref.norm() > 0 and _cos(gg[k], ref) < 0.999]
    assert not bad, bad[:10]


@pytest.mark.parametrize("name,ds,size,batch", BF16_MODELS)
def test_network_grads_bf16(cuda, name, ds, size, batch):
    lr, gr = _grads(name, ds, "cpu", torch.float32, size, batch)
    lg, gg = _grads(name, ds, cuda, torch.bfloat16, size, batch)
    assert abs(lg - lr) < 0.02 * max(1.0, abs(lr))
    cos = sorted(_cos(gg[k], ref) for k, ref in gr.items() if ref.norm() > 0)
    assert cos[0] > 0.85 and cos[len(cos) // 2] > 0.95, (cos[0], cos[len(cos) // 2])


@pytest.mark.parametrize("name,ds,size,batch", BF16_MODELS[:1] + [("resnet20", "cifar10", None, 64)])
def test_fused_matches_unfused(cuda, name, ds, size, batch):
    """(The batch-64 case has 512 pixel tiles per 32x32 layer, far more than
    the 32 statistics slots: the conv-epilogue BN statistics then depend on
    the order of their fp32 atomics, and the tolerance must hold anyway.)"""
    conv_ops.FUSE_BN = True
    _, fused = _grads(name, ds, cuda, torch.bfloat16, size, batch)
    conv_ops.FUSE_BN = False
    try:
        _, plain = _grads(name, ds, cuda, torch.bfloat16, size, batch)
    finally:
        conv_ops.FUSE_BN = True
    cos = sorted(_cos(fused[k], ref) for k, ref in plain.items() if ref.norm() > 0)
    assert cos[0] > 0.9 and cos[len(cos) // 2] > 0.97, (cos[0], cos[len(cos) // 2])


def test_scatter_dgrad_bn_fusion_matches(cuda, monkeypatch):
    """ResNet-50 v1 stage transitions: the block input feeds two strided 1x1
    convs (conv a, projection shortcut), whose scatter dgrads now also apply
    the producer BN's ReLU mask and accumulate its backward partials.  The
    backward is identical up to the first such BN, so every gradient is
    (nearly) unchanged against the unfused path; deeper ones drift only by
    bf16 rounding order."""
    from kf_benchmarks_amd.ops import conv_hip
    monkeypatch.setattr(conv_hip, "_SCATTER_BN_FUSE", True)
    _, new = _grads("resnet50", "imagenet", cuda, torch.bfloat16, 64, 8)
    monkeypatch.setattr(conv_hip, "_SCATTER_BN_FUSE", False)
    _, old = _grads("resnet50", "imagenet", cuda, torch.bfloat16, 64, 8)
    cos = {k: _cos(new[k], ref) for k, ref in old.items() if ref.norm() > 0}
    vals = sorted(cos.values())
    print("scatter fusion cosines: min %.4f median %.4f" % (vals[0], vals[len(vals) // 2]))
    assert vals[len(vals) // 2] > 0.99 and vals[0] > 0.9, (vals[0], vals[len(vals) // 2])


def test_stem_pool_link_partials_match(cuda, monkeypatch):
    """ResNet-50 stem: the fused BN+ReLU+max-pool backward takes its BN
    partials from the dgrad epilogue of the convs consuming the pooled output
    z (sum dz', sum dz' (z - beta) / (gamma * invstd), ops/nn.py _POOL_LINK)
    instead of its own pass over x.  The forward is unchanged and the
    backward identical down to the stem BN, whose partials now come from the
    bf16 z instead of the bf16 x: the stem gradients agree to bf16 rounding,
    every other gradient to the atomics' order."""
    from kf_benchmarks_amd.ops import nn as F
    monkeypatch.setattr(F, "_POOL_LINK", True)
    loss_new, new = _grads("resnet50", "imagenet", cuda, torch.bfloat16, 64, 8)
    monkeypatch.setattr(F, "_POOL_LINK", False)
    loss_old, old = _grads("resnet50", "imagenet", cuda, torch.bfloat16, 64, 8)
    assert abs(loss_new - loss_old) < 5e-3 * abs(loss_old), (loss_new, loss_old)
    cos = {k: _cos(new[k], ref) for k, ref in old.items() if ref.norm() > 0}
    vals = sorted(cos.values())
    print("pool-link cosines: min %.5f median %.5f" % (vals[0], vals[len(vals) // 2]))
    assert vals[len(vals) // 2] > 0.99 and vals[0] > 0.95, (vals[0], vals[len(vals) // 2])


def test_deferred_shortcut_bn_network(cuda, monkeypatch):
    """ResNet-50 v1 projection shortcuts take the deferred-BN path (the
    shortcut BN applied inside the block-output BN's apply pass) on the GPU:
    4 dual BNs, the same loss as the materialized path up to the bf16
    rounding of the shortcut BN output, finite gradients for every variable
    (numerics of the dual op: test_kernels_gpu.py::test_batch_norm_dual)."""
    from kf_benchmarks_amd.models import builder
    from kf_benchmarks_amd.ops import nn as F
    calls = []
    orig = F._BatchNormTrainDual.apply
    monkeypatch.setattr(F._BatchNormTrainDual, "apply",
                        lambda *a: calls.append(1) or orig(*a))
    monkeypatch.setattr(builder, "_DEFER_BN", True)
    loss_new, new = _grads("resnet50", "imagenet", cuda, torch.bfloat16, 64, 8)
    assert len(calls) == 4
    monkeypatch.setattr(builder, "_DEFER_BN", False)
    loss_old, old = _grads("resnet50", "imagenet", cuda, torch.bfloat16, 64, 8)
    assert len(calls) == 4
    assert set(new) == set(old)
    assert abs(loss_new - loss_old) < 2e-2 * abs(loss_old), (loss_new, loss_old)
    assert all(torch.isfinite(g).all() for g in new.values())
    # (bf16 ResNet-50 gradients are chaotic under a forward rounding change,
    # see FP32_MODELS above, so the backward is pinned with the forward fixed:)
    # the fused dual backward (one apply pass; kfb_bn_bwd_dual) == two
    # separate BN backwards with the masked dy written out as a copy
    monkeypatch.setattr(builder, "_DEFER_BN", True)
    monkeypatch.setattr(F, "_DUAL_ALIAS_RES", False)
    monkeypatch.setattr(F, "_DUAL_BWD_FUSE", False)
    loss_copy, copy = _grads("resnet50", "imagenet", cuda, torch.bfloat16, 64, 8)
    assert loss_copy == loss_new
    cos = sorted(_cos(new[k], ref) for k, ref in copy.items() if ref.norm() > 0)
    print("fused vs separate dual-BN backward cosines: min %.4f median %.4f" % (cos[0], cos[len(cos) // 2]))
    assert cos[len(cos) // 2] > 0.99 and cos[0] > 0.9, (cos[0], cos[len(cos) // 2])


def test_s1_dual_partials_network(cuda, monkeypatch):
    """ResNet-50's four projection-block outputs relu(bn(x) + bn_r(x_r)):
    with the streaming 1x1 kernel forced, the next block's conv-a data
    gradient sums bn_r's backward partials too (kfb_conv_s1_dgrad_dual, so
    the dual backward skips its partial pass); the gradients agree with the
    partial-pass path (forward identical; bf16 backward by cosine, as above)."""
    from kf_benchmarks_amd.models import builder
    from kf_benchmarks_amd.ops import _native as N, conv_hip, nn as F
    monkeypatch.setattr(builder, "_DEFER_BN", True)
    monkeypatch.setattr(conv_hip, "_IG_FORCE", conv_hip.IG_S1)
    names = []
    orig = N.call
    monkeypatch.setattr(N, "call", lambda name, *a: names.append(name) or orig(name, *a))
    loss_d, dual = _grads("resnet50", "imagenet", cuda, torch.bfloat16, 64, 8)
    assert names.count("kfb_conv_s1_dgrad_dual") == 4, names.count("kfb_conv_s1_dgrad_dual")
    monkeypatch.setattr(F, "_S1_DUAL", False)
    names.clear()
    loss_p, sep = _grads("resnet50", "imagenet", cuda, torch.bfloat16, 64, 8)
    assert "kfb_conv_s1_dgrad_dual" not in names
    assert loss_d == loss_p
    cos = sorted(_cos(dual[k], ref) for k, ref in sep.items() if ref.norm() > 0)
    print("dual-partial vs partial-pass cosines: min %.4f median %.4f" % (cos[0], cos[len(cos) // 2]))
    assert cos[len(cos) // 2] > 0.99 and cos[0] > 0.9, (cos[0], cos[len(cos) // 2])


def _kernel_names(fn):
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    return {e.name for e in prof.events() if e.device_type.name == "CUDA"}


@pytest.mark.parametrize("name,ds,size,batch", [("resnet20", "cifar10", None, 4),
                                                ("googlenet", "imagenet", 224, 2)])
def test_fp32_network_runs_only_our_kernels(cuda, name, ds, size, batch):
    """One GPU path: an fp32 training step launches our HIP kernels (plus
    torch's own fill/copy/elementwise helpers), never MIOpen or hipBLASLt."""
    names = _kernel_names(lambda: _grads(name, ds, cuda, torch.float32, size, batch))
    ours = [n for n in names if "kfb" in n]
    foreign = [n for n in names if "kfb" not in n and "at::native" not in n
               and not n.startswith("Memset") and not n.startswith("Memcpy")]
    assert ours and not foreign, foreign[:10]


def _bf16_vs_fp32(cuda):
    """(loss, grads) of ResNet-20 on CIFAR-10 shapes at batch 8 on the CPU in
    fp32: the bf16 whole-network reference (a well-conditioned network; the
    ResNet-50 class is chaotic in bf16 at random init, see above)."""
    return _grads("resnet20", "cifar10", "cpu", torch.float32, None, 8)


def _check_bf16(cuda, ref):
    lr, gr = ref
    lg, gg = _grads("resnet20", "cifar10", cuda, torch.bfloat16, None, 8)
    assert abs(lg - lr) < 0.02 * max(1.0, abs(lr)), (lg, lr)
    cos = {k: _cos(gg[k], r) for k, r in gr.items() if r.norm() > 0}
    vals = sorted(cos.values())
    worst = sorted(cos.items(), key=lambda kv: kv[1])[:4]
    assert vals[0] > 0.85 and vals[len(vals) // 2] > 0.95, (vals[0], vals[len(vals) // 2], worst)


@pytest.mark.parametrize("knob", ["_WGRAD_SIDE", "_AUTOTUNE", "_AUTOTUNE_WGRAD", "both"],
                         ids=["wgrad_stream_off", "igemm_autotune_off", "wgrad_autotune_off",
                              "conv_autotune_off"])
def test_stream_and_autotune_knobs_keep_the_gradients(cuda, monkeypatch, knob):
    """KFB_WGRAD_STREAM=0 (weight gradients inline on the compute stream) and
    KFB_CONV_AUTOTUNE=0 (default kernels, no timing): the bf16 network
    gradients still match the fp32 reference as closely as the default
    path's do (test_network_grads_bf16's bounds)."""
    from kf_benchmarks_amd.ops import conv_hip
    ref = _bf16_vs_fp32(cuda)
    for k in (("_AUTOTUNE", "_AUTOTUNE_WGRAD") if knob == "both" else (knob,)):
        monkeypatch.setattr(conv_hip, k, False)
    monkeypatch.setattr(conv_hip, "_ig_tuned", {})
    monkeypatch.setattr(conv_hip, "_wgrad_tuned", {})
    _check_bf16(cuda, ref)


@pytest.mark.parametrize("algo", ["glds", "classic", "onebuf", "glds_n64", "gshort64",
                                  "tall256", "small", "gmulti64"])
def test_forced_conv_kernel_in_network_keeps_the_gradients(cuda, monkeypatch, algo):
    """Every conv of a network (fwd and dgrad with their fused BN epilogues)
    on one forced igemm kernel: the autotune may pick any offered kernel on
    any layer, so each must give the network's gradients, not only pass the
    single-layer epilogue tests (bf16 vs the fp32 reference)."""
    from kf_benchmarks_amd.ops import conv_hip
    ref = _bf16_vs_fp32(cuda)
    monkeypatch.setattr(conv_hip, "_IG_FORCE", conv_hip.IG_ALGOS[algo])
    _check_bf16(cuda, ref)
