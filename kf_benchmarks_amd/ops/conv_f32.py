"""fp32 NHWC convolution on the GPU: csrc/conv_f32.hip (implicit GEMM on
v_mfma_f32_16x16x4_f32, exact fp32 products) for forward, data gradient and
weight gradient - the precision of the reference's published runs
(tcb/convnet_builder.py:107-124 with use_fp16=False).  The weight gradient
accumulates straight into the parameter's flat-gradient view when it has one
(as the bf16 kernels do).

Products (``set_products`` / KFB_F32_PRODUCTS):
  exact   v_mfma_f32_16x16x4_f32 (default).
  bf16x3  each product as ah*bh + ah*bl + al*bh over the bf16 split
          x = hi + lo of both operands, on v_mfma_f32_16x16x32_bf16 with fp32
          accumulation: ~2^-16 relative error per product (TF32, which TF
          2.5 uses for fp32 convs on the reference's RTX 3090 by default, has
          2^-11), at 3 x 16 instead of 8 x 32 MFMA cycles per 32 k.  Tensors,
          accumulation and every other op stay fp32."""

from __future__ import annotations

import os

import torch

from . import _native as N

N.register_optional("kfb_conv_f32", [N.I, N.P, N.P, N.P] + [N.I] * 13 + [N.P])

PRODUCTS = ("exact", "bf16x3")
_products = os.environ.get("KFB_F32_PRODUCTS", "exact")
if _products not in PRODUCTS:
    raise ValueError("KFB_F32_PRODUCTS must be one of %s" % (PRODUCTS,))


def set_products(mode: str):
    """Select how the fp32 conv kernels form products (see module doc)."""
    global _products
    if mode not in PRODUCTS:
        raise ValueError("fp32 products must be one of %s, got %r" % (PRODUCTS, mode))
    _products = mode


def products() -> str:
    return _products


def _mode(m):
    return m | (8 if _products == "bf16x3" else 0)


def _geo(x_shape, w_shape, stride, pads):
    n, H, W, C = x_shape
    cout, KH, KW, _ = w_shape
    sh, sw = stride
    pt, pb, pl, pr = pads
    OH = (H + pt + pb - KH) // sh + 1
    OW = (W + pl + pr - KW) // sw + 1
    return (n, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, cout)


class _Conv2dF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pads):
        x = x.contiguous()
        wd = w.detach().contiguous()
        g = _geo(x.shape, wd.shape, stride, pads)
        n, OH, OW, cout = g[0], g[4], g[5], g[12]
        y = torch.empty((n, OH, OW, cout), dtype=torch.float32, device=x.device)
        N.call("kfb_conv_f32", _mode(0), x.data_ptr(), wd.data_ptr(), y.data_ptr(), *g,
               N.stream(x.device))
        ctx.save_for_backward(x, wd)
        ctx.g, ctx.w = g, w
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wd = ctx.saved_tensors
        dy = dy.contiguous()
        g = ctx.g
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            N.call("kfb_conv_f32", _mode(1), dy.data_ptr(), wd.data_ptr(), dx.data_ptr(), *g,
                   N.stream(x.device))
        dw = None
        if ctx.needs_input_grad[1]:
            sink = getattr(ctx.w, "_kfb_grad_sink", None)
            out = sink if sink is not None else torch.zeros_like(wd)
            N.call("kfb_conv_f32", _mode(2), dy.data_ptr(), x.data_ptr(), out.data_ptr(), *g,
                   N.stream(x.device))
            if sink is not None:
                cb = getattr(ctx.w, "_kfb_ready_cb", None)
                if cb is not None:
                    cb(ctx.w)
            else:
                dw = out
        return dx, dw, None, None


def conv2d(x, w, stride, pads):
    """x [N,H,W,C] fp32 (GPU), w [Cout,KH,KW,C] fp32 master."""
    return _Conv2dF32.apply(x, w, tuple(stride), tuple(pads))
