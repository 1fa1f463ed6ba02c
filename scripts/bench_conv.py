#!/usr/bin/env python3
"""Per-layer conv microbenchmark: our HIP implicit-GEMM kernels vs
PyTorch/MIOpen on the ResNet-50 conv shapes (NHWC, bf16, batch 256).

Prints one line per (shape, pass) with us and TFLOP/s for both, plus totals
weighted by how often each shape occurs in ResNet-50 v1.
"""

import argparse
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd.ops import conv_hip  # noqa: E402
from kf_benchmarks_amd.ops import nn as F  # noqa: E402

# (H, Cin, Cout, k, stride, count in resnet50 v1)
RESNET50 = [
    (224, 3, 64, 7, 2, 1),
    (56, 64, 256, 1, 1, 4),   # blk1 shortcut + 3x conv c
    (56, 64, 64, 1, 1, 1),    # blk1 conv a
    (56, 256, 64, 1, 1, 2),
    (56, 64, 64, 3, 1, 3),
    (56, 256, 512, 1, 2, 1),
    (56, 256, 128, 1, 2, 1),
    (28, 128, 128, 3, 1, 4),
    (28, 128, 512, 1, 1, 4),
    (28, 512, 128, 1, 1, 3),
    (28, 512, 1024, 1, 2, 1),
    (28, 512, 256, 1, 2, 1),
    (14, 256, 256, 3, 1, 6),
    (14, 256, 1024, 1, 1, 6),
    (14, 1024, 256, 1, 1, 5),
    (14, 1024, 2048, 1, 2, 1),
    (14, 1024, 512, 1, 2, 1),
    (7, 512, 512, 3, 1, 3),
    (7, 512, 2048, 1, 1, 3),
    (7, 2048, 512, 1, 1, 2),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--json", default=None)
    ap.add_argument("--hip_only", action="store_true", help="skip MIOpen (profiling runs)")
    ap.add_argument("--shapes", default=None, help="comma list of RESNET50 indices")
    ap.add_argument("--sol", action="store_true",
                    help="instead of MIOpen: %% of speed of light = max(bytes / 6 TB/s, "
                         "flops / 2.5 PF/s), and hipBLASLt (torch.matmul) on the 1x1 s1 GEMMs")
    a = ap.parse_args()
    only = {int(i) for i in a.shapes.split(",")} if a.shapes else None
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    tot = {"hip": [0.0, 0.0, 0.0], "miopen": [0.0, 0.0, 0.0], "sol": [0.0, 0.0, 0.0]}
    rows = []
    if a.sol:
        print("%-28s %8s | %9s %7s | %-24s %6s | %s" % ("shape", "pass", "hip_us", "TF/s",
                                                         "sol_us (bound)", "%sol", "blaslt_us"))
    else:
        print("%-28s %8s | %9s %7s | %9s %7s | %s" % ("shape", "pass", "hip_us", "TF/s",
                                                       "miopen_us", "TF/s", "hip/miopen"))
    for si, (H, cin, cout, k, s, cnt) in enumerate(RESNET50):
        if only is not None and si not in only:
            continue
        n = a.batch
        mode = "SAME_RESNET"
        pads = F.resolve_pads(mode, H, H, k, k, s, s)
        x = torch.randn(n, H, H, cin, device=dev, dtype=dt)
        w = torch.randn(cout, k, k, cin, device=dev, dtype=dt) * 0.05
        OH = (H + pads[0] + pads[1] - k) // s + 1
        flops = 2.0 * n * OH * OH * cout * k * k * cin
        dy = torch.randn(n, OH, OH, cout, device=dev, dtype=dt)
        cinp = (cin + 7) // 8 * 8
        xp = torch.nn.functional.pad(x, (0, cinp - cin)) if cinp != cin else x
        wp = torch.nn.functional.pad(w, (0, cinp - cin)).contiguous() if cinp != cin else w
        hip = {
            "fwd": lambda: conv_hip.conv_fwd(xp, wp, (s, s), pads),
            "dgrad": lambda: conv_hip.conv_dgrad(dy, wp, xp.shape, (s, s), pads),
            "wgrad": lambda: conv_hip.conv_wgrad(dy, xp, wp.shape, (s, s), pads),
        }
        if k == 7 and s == 2 and cin <= 4:
            # the stem as the network runs it (ops/conv_hip.py _Conv2d, "pairs"):
            # the padded pixel-pair view and the pair weight are built per call
            # and timed with the conv; no data gradient (the input's)
            def stem_fwd():
                xv = conv_hip.stem_pairs_input(x, w.shape, pads)
                w2 = conv_hip.stem_pairs_weight(w)
                return conv_hip.conv_fwd(xv, w2, (2, 1), (0, 0, 0, 0))

            xv0 = conv_hip.stem_pairs_input(x, w.shape, pads)
            w20 = conv_hip.stem_pairs_weight(w)
            dwo = torch.zeros((cout, k, k, cin), dtype=torch.float32, device=dev)

            def stem_wgrad():
                scratch = torch.zeros((cout, 8, 4, 8), dtype=torch.float32, device=dev)
                conv_hip.conv_wgrad(dy, xv0, w20.shape, (2, 1), (0, 0, 0, 0), out=scratch)
                conv_hip.N.call("kfb_stem_weight_grad", scratch.data_ptr(), dwo.data_ptr(), cout,
                                k, k, cin, conv_hip.N.stream(dev))
                return dwo

            hip = {"fwd": stem_fwd, "wgrad": stem_wgrad}
        xc = x.permute(0, 3, 1, 2)
        wc = w.permute(0, 3, 1, 2)
        dyc = dy.permute(0, 3, 1, 2)
        pt, pb, pl, pr = pads
        xpad = torch.nn.functional.pad(xc, (pl, pr, pt, pb)) if (pt != pb) else xc
        padarg = 0 if pt != pb else pt
        mi = {
            "fwd": lambda: torch.nn.functional.conv2d(xpad, wc, stride=s, padding=padarg),
            "dgrad": lambda: torch.ops.aten.convolution_backward(
                dyc, xpad, wc, None, [s, s], [padarg, padarg], [1, 1], False, [0, 0], 1,
                [True, False, False]),
            "wgrad": lambda: torch.ops.aten.convolution_backward(
                dyc, xpad, wc, None, [s, s], [padarg, padarg], [1, 1], False, [0, 0], 1,
                [False, True, False]),
        }
        if a.sol:
            x2, w2, dy2 = x.view(-1, cin), w.view(cout, -1), dy.view(-1, cout)
            gemm = k == 1 and s == 1
            mi = {"fwd": lambda: x2 @ w2.t(), "dgrad": lambda: dy2 @ w2,
                  "wgrad": lambda: dy2.t() @ x2}
            xb, yb = x.numel() * 2, dy.numel() * 2
            bytes_ = {"fwd": xb + yb, "dgrad": xb + yb, "wgrad": xb + yb + w.numel() * 4}
        for i, pas in enumerate(("fwd", "dgrad", "wgrad")):
            if pas == "dgrad" and cin == 3:
                continue
            th = timeit(hip[pas], a.iters)
            if a.sol:
                sol = max(bytes_[pas] / 6e12, flops / 2.5e15) * 1e6
                tm = timeit(mi[pas], a.iters) if gemm else float("nan")
                name = "%dx%d %d->%d k%d s%d" % (H, H, cin, cout, k, s)
                print("%-28s %8s | %9.1f %7.1f | sol %7.1f us (%s) %5.1f%% | blaslt %9.1f" % (
                    name, pas, th, flops / th / 1e6, sol,
                    "mem" if bytes_[pas] / 6e12 > flops / 2.5e15 else "mfma", 100 * sol / th, tm))
                tot["hip"][i] += th * cnt
                tot["sol"][i] += sol * cnt
                rows.append({"shape": name, "pass": pas, "hip_us": th, "sol_us": sol,
                             "blaslt_us": tm, "count": cnt})
                continue
            tm = timeit(mi[pas], a.iters) if not a.hip_only else float("nan")
            tot["hip"][i] += th * cnt
            tot["miopen"][i] += tm * cnt
            name = "%dx%d %d->%d k%d s%d" % (H, H, cin, cout, k, s)
            print("%-28s %8s | %9.1f %7.1f | %9.1f %7.1f | %5.2f%s" % (
                name, pas, th, flops / th / 1e6, tm, flops / tm / 1e6, th / tm,
                "  MIOPEN FASTER" if tm < th else ""))
            rows.append({"shape": name, "pass": pas, "hip_us": th, "miopen_us": tm,
                         "count": cnt, "tflops_hip": flops / th / 1e6,
                         "tflops_miopen": flops / tm / 1e6})
    for key in (("hip", "sol") if a.sol else ("hip", "miopen")):
        f, d, wg = tot[key]
        print("%-8s ResNet-50 conv time per step: fwd %.2f ms  dgrad %.2f ms  wgrad %.2f ms  "
              "total %.2f ms" % (key, f / 1e3, d / 1e3, wg / 1e3, (f + d + wg) / 1e3))
    if not a.sol and not a.hip_only:
        slower = [r for r in rows if r["miopen_us"] < r["hip_us"]]
        print("layers where MIOpen is faster: %d of %d" % (len(slower), len(rows)))
        for r in slower:
            print("  %-28s %6s hip %8.1f us  miopen %8.1f us  (x%d per step)"
                  % (r["shape"], r["pass"], r["hip_us"], r["miopen_us"], r["count"]))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump({"rows": rows, "totals_us": tot}, fh, indent=1)


if __name__ == "__main__":
    main()
