#!/usr/bin/env python3
"""Diagnostic: after every conv that ran the in-kernel BN finalize, compare
its outputs (mean / invstd) with the same finalize computed on the host from
the statistics slots the conv accumulated; prints the mismatching convs with
their geometry and kernel choice."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd import params as P  # noqa: E402
from kf_benchmarks_amd.benchmark import BenchmarkCNN  # noqa: E402
from kf_benchmarks_amd.ops import conv_hip  # noqa: E402

orig = conv_hip._igemm_call
bad = []
seen = [0]


def wrapped(algo, x, wmat, y, geo, stats=None, *a, **k):
    fin_on = (stats is not None and getattr(stats, "_kfb_fin", None) is not None
              and len(a) >= 2 and a[1] is None and geo[15] == 1)
    kshift = conv_hip.stats_shift(stats)
    k0 = kshift.clone() if (fin_on and kshift is not None) else None
    orig(algo, x, wmat, y, geo, stats, *a, **k)
    if not fin_on:
        return
    torch.cuda.synchronize()
    seen[0] += 1
    gamma, beta, rm, rv, decay, eps, st, coef = stats._kfb_fin
    C = st.shape[-1]
    s = stats.view(2, 32, C).double().sum(1)
    rows = geo[0] * geo[4] * geo[5]
    kk = k0.double() if k0 is not None else 0.0
    dm = s[0] / rows
    mean = kk + dm
    var = (s[1] / rows - dm * dm).clamp_min(0)
    err_m = (st[0].double() - mean).abs().max().item()
    err_v = (st[1].double() - 1 / torch.sqrt(var + eps)).abs().max().item() / \
        (1 / torch.sqrt(var + eps)).abs().max().item()
    # and the slots vs the conv output itself
    yd = y.double().reshape(-1, C)
    err_y = ((yd.mean(0) - mean).abs().max().item())
    cnt = stats._kfb_counter.view(torch.int32)[0].item()
    if err_m > 1e-4 or err_v > 1e-4 or err_y > 1e-2:
        bad.append((seen[0], conv_hip._ALGO_NAMES.get(algo, algo), geo[:8], err_m, err_v, err_y,
                    cnt))


conv_hip._igemm_call = wrapped


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    p = P.make_params(model=model, batch_size=bs, num_gpus=1, use_bf16=True,
                      optimizer="momentum", data_format="NHWC", variable_update="kungfu",
                      init_learning_rate=0.002, display_every=10 ** 9)
    b = BenchmarkCNN(p)
    b.build()
    if not conv_hip._ALGO_NAMES:
        conv_hip._ALGO_NAMES.update({v: k for k, v in conv_hip.IG_ALGOS.items()})
    for _ in range(2):
        b.train_step(need_loss=True)
    torch.cuda.synchronize()
    print("convs with in-kernel finalize checked: %d, mismatching: %d" % (seen[0], len(bad)))
    for r in bad[:40]:
        print("  #%d algo %s geo %s err_mean %.3g err_invstd %.3g err_vs_y %.3g counter %d" % r)


if __name__ == "__main__":
    main()
