#!/usr/bin/env python3
"""Backward BN apply with the gradient finalize folded in (bn_bwd_apply_fold_k)
against the finalize launch + apply pass, in isolation, for the ResNet-50
bs256 BN shapes (rows x channels): us per call and TB/s of the apply's bytes
(dy, x read; dx written).

  python scripts/bench_bn_fold.py [--shapes 802816x64,200704x512]"""
import argparse
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd.ops import _native as N  # noqa: E402

SHAPES = "802816x64,802816x256,200704x128,200704x512,50176x256,50176x1024,12544x512,12544x2048"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=SHAPES)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = N.load()
    prev = lib.kfb_bn_get_fold_bwd()
    for sh in a.shapes.split(","):
        rows, C = (int(v) for v in sh.split("x"))
        dy = torch.randn(rows, C, device=dev).to(torch.bfloat16)
        x = torch.randn(rows, C, device=dev).to(torch.bfloat16)
        dx = torch.empty_like(dy)
        parts = torch.randn(2, 32, C, device=dev)
        gamma = torch.rand(C, device=dev) + 0.5
        mean = torch.randn(C, device=dev) * 0.1
        invstd = torch.rand(C, device=dev) + 0.5
        coef = torch.empty(3, C, device=dev)
        dg = torch.zeros(2, C, device=dev)
        res = {}
        for mode in (0, 2, 0, 2):
            lib.kfb_bn_set_fold_bwd(mode)

            def run():
                N.call("kfb_bn_bwd", N.dt(dy), dy.data_ptr(), None, x.data_ptr(), dx.data_ptr(),
                       None, rows, C, gamma.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                       dg[0].data_ptr(), dg[1].data_ptr(), parts[0].data_ptr(),
                       parts[1].data_ptr(), 32, coef[0].data_ptr(), coef[1].data_ptr(),
                       coef[2].data_ptr(), 0, 1, 1, N.stream(dev))
            for _ in range(2):
                run()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                run()
            e.record()
            e.synchronize()
            us = s.elapsed_time(e) * 1e3 / a.iters
            res[mode] = min(res.get(mode, 1e9), us)
        nb = 3 * rows * C * 2
        print("%7d x %4d  launch+apply %8.1f us (%4.2f TB/s)   folded %8.1f us (%4.2f TB/s)"
              % (rows, C, res[0], nb / res[0] / 1e6, res[2], nb / res[2] / 1e6), flush=True)
        del dy, x, dx
    lib.kfb_bn_set_fold_bwd(prev)


if __name__ == "__main__":
    main()
