"""NHWC 2-D convolution: forward, data-gradient and weight-gradient.

Weights are stored [Cout, KH, KW, Cin] so that, in the implicit-GEMM view
(M = N*OH*OW rows, N = Cout columns, K = KH*KW*Cin), both MFMA operands are
K-contiguous: an activation row of K is a run of Cin channels per tap, a
weight column of K is contiguous.

Implementations:
  * GPU: our gfx950 implicit-GEMM kernels - bf16/fp16 in csrc/conv_igemm.hip
    (ops/conv_hip.py, with the fused BN epilogues), fp32 in csrc/conv_f32.hip
    (ops/conv_f32.py).  There is no vendor fallback: a GPU tensor either runs
    one of these kernels or raises.
  * ``impl="torch"`` - PyTorch/MIOpen on channels-last views, reachable only
    from tests as an A/B oracle (the CLI accepts --kernel_impl=hip only).
  * CPU - PyTorch reference (plumbing config and test oracle).
"""

from __future__ import annotations

import os
from typing import Tuple

import torch
import torch.nn.functional as F

from . import _native as N

Pads = Tuple[int, int, int, int]


def out_hw(H, W, kh, kw, stride, pads):
    sh, sw = stride
    pt, pb, pl, pr = pads
    return (H + pt + pb - kh) // sh + 1, (W + pl + pr - kw) // sw + 1


def _torch_conv(x, w, stride, pads):
    """Reference conv through PyTorch on NCHW views (any device)."""
    pt, pb, pl, pr = pads
    xc = x.permute(0, 3, 1, 2)
    wc = w.permute(0, 3, 1, 2)
    if pt == pb and pl == pr:
        y = F.conv2d(xc, wc, stride=stride, padding=(pt, pl))
    else:
        y = F.conv2d(F.pad(xc, (pl, pr, pt, pb)), wc, stride=stride)
    return y.permute(0, 2, 3, 1)


def conv2d_reference(x, w, stride, pads):
    """fp32 reference result (used by tests)."""
    return _torch_conv(x.float(), w.float(), stride, pads).contiguous()


def _hip_supported(x, w, stride, pads) -> bool:
    try:
        from . import conv_hip
    except ImportError:
        return False
    return conv_hip.supported(x, w, stride, pads)


FUSE_BN = os.environ.get("KFB_DISABLE_FUSION", "0") != "1"


def fills_bn_stats(x, cout, impl="hip") -> bool:
    """True when conv2d(..., stats=buf) fills ``buf`` with the BN partial sums
    of its output (HIP implicit-GEMM path)."""
    return (FUSE_BN and x.is_cuda and impl == "hip"
            and x.dtype in (torch.bfloat16, torch.float16) and cout % 8 == 0)


def runs_hip_kernel(x, impl="hip") -> bool:
    """True when conv2d on ``x`` goes through the HIP autograd Function (which
    takes part in the BN-link gradient protocol of ops.nn.BNLink)."""
    return x.is_cuda and impl == "hip" and x.dtype in (torch.bfloat16, torch.float16)


def fuses_bias_act(x, impl="hip") -> bool:
    """True when conv2d(..., bias=, relu=) applies bias + ReLU in the conv's
    own epilogue (the bf16/fp16 HIP kernels)."""
    return FUSE_BN and runs_hip_kernel(x, impl)


def conv2d(x, w, w_lp, stride, pads, impl="hip", stats=None, w_t=None, bias=None, relu=False):
    """NHWC conv.  ``stats``: see fills_bn_stats.  ``w_t``: optional
    dgrad-ready weight copy (ops.conv_hip.DgradWeights).  ``bias`` / ``relu``:
    only where fuses_bias_act(x) (y = act(conv + bias) in the epilogue)."""
    if (bias is not None or relu) and not fuses_bias_act(x, impl):
        raise ValueError("bias/relu epilogue requested on a path without it")
    if not x.is_cuda:
        y = _torch_conv(x.float(), w, stride, pads)
        return y.to(x.dtype).contiguous()
    if impl == "torch":
        # test oracle only: torch/MIOpen on channels-last views; autograd
        # routes the weight gradient through the cast back to the fp32 master
        return _torch_conv(x, w.to(x.dtype), stride, pads).contiguous()
    if x.dtype == torch.float32:
        from . import conv_f32
        return conv_f32.conv2d(x, w, stride, pads)
    if _hip_supported(x, w, stride, pads):
        from . import conv_hip
        return conv_hip.conv2d(x, w, w_lp, stride, pads, stats, w_t, bias, relu)
    raise N.NativeError("no HIP convolution kernel for a %s tensor of shape %s"
                        % (x.dtype, tuple(x.shape)))
