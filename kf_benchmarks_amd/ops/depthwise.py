"""NHWC depthwise convolution (channel multiplier 1) for MobileNet-v2 and
NASNet separable convs (role of slim.separable_conv2d / tf.nn.depthwise_conv2d
in tcb/models/mobilenet_conv_blocks.py and tcb/models/nasnet_utils.py).

Weights are [KH, KW, C] fp32 masters (TF layout [KH, KW, C, 1] on export).
GPU (bf16 / fp16 / fp32): csrc/depthwise.hip (fwd / dgrad / wgrad straight
into the flat gradient sink).  CPU: PyTorch grouped conv on NCHW views.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _native as N

_G = [N.I, N.P, N.P, N.P] + [N.I] * 12 + [N.P]
N.register_optional("kfb_dw_fwd", _G)
N.register_optional("kfb_dw_dgrad", _G)
N.register_optional("kfb_dw_wgrad", _G)


def _torch_dw(x, w, stride, pads):
    pt, pb, pl, pr = pads
    C = x.shape[-1]
    xc = x.permute(0, 3, 1, 2)
    wc = w.permute(2, 0, 1).unsqueeze(1)  # [C, 1, KH, KW]
    if pt == pb and pl == pr:
        y = F.conv2d(xc, wc, stride=stride, padding=(pt, pl), groups=C)
    else:
        y = F.conv2d(F.pad(xc, (pl, pr, pt, pb)), wc, stride=stride, groups=C)
    return y.permute(0, 2, 3, 1)


def depthwise_reference(x, w, stride, pads):
    return _torch_dw(x.float(), w.float(), stride, pads).contiguous()


def _geo(x_shape, w_shape, stride, pads):
    n, H, W, C = x_shape
    KH, KW, _ = w_shape
    sh, sw = stride
    pt, pb, pl, pr = pads
    OH = (H + pt + pb - KH) // sh + 1
    OW = (W + pl + pr - KW) // sw + 1
    return n, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl


class _DepthwiseHip(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, wl, stride, pads):
        x = x.contiguous()
        wl = (w.detach().to(x.dtype) if wl is None or wl.dtype != x.dtype else wl).contiguous()
        g = _geo(x.shape, wl.shape, stride, pads)
        n, H, W, C, OH, OW = g[:6]
        y = torch.empty((n, OH, OW, C), dtype=x.dtype, device=x.device)
        N.call("kfb_dw_fwd", N.dt(x), x.data_ptr(), wl.data_ptr(), y.data_ptr(), *g,
               N.stream(x.device))
        ctx.save_for_backward(x, wl)
        ctx.g = g
        ctx.w = w
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wl = ctx.saved_tensors
        g = ctx.g
        dy = dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            N.call("kfb_dw_dgrad", N.dt(x), dy.data_ptr(), wl.data_ptr(), dx.data_ptr(), *g,
                   N.stream(x.device))
        dw = None
        if ctx.needs_input_grad[1]:
            w = ctx.w
            sink = getattr(w, "_kfb_grad_sink", None)
            out = sink if sink is not None else torch.zeros(w.shape, dtype=torch.float32,
                                                            device=x.device)
            N.call("kfb_dw_wgrad", N.dt(x), dy.data_ptr(), x.data_ptr(), out.data_ptr(), *g,
                   N.stream(x.device))
            if sink is not None:
                cb = getattr(w, "_kfb_ready_cb", None)
                if cb is not None:
                    cb(w)
            else:
                dw = out
        return dx, dw, None, None, None


def depthwise_conv2d(x, w, w_lp, stride, pads, impl="hip"):
    """x [N,H,W,C], w [KH,KW,C] -> [N,OH,OW,C]."""
    if not x.is_cuda:
        return _torch_dw(x.float(), w, stride, pads).to(x.dtype).contiguous()
    if impl == "torch":  # test oracle only
        return _torch_dw(x, w.to(x.dtype), stride, pads).contiguous()
    return _DepthwiseHip.apply(x, w, w_lp, tuple(stride), tuple(pads))
