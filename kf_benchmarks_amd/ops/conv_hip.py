"""NHWC convolution autograd Function over the gfx950 implicit-GEMM kernels
(csrc/conv_igemm.hip).

forward : y  = igemm(x, W[Cout][KH*KW*Cin])
dgrad   : 1x1 stride 1  -> igemm(dY, W^T) (plain GEMM)
          1x1 stride s  -> dX = 0; igemm(dY, W^T) scattered to every s-th pixel
          general       -> transposed-gather igemm(dY, W permuted to [Cin][KH][KW][Cout])
wgrad   : split-M MFMA reduction into an fp32 [Cout][KH*KW*Cin] buffer, which
          is exactly the fp32 master weight layout.

Channel counts that are not multiples of 8 (the RGB stem, DenseNet growth
12) are zero-padded to the next multiple of 8 around the kernels.
"""

from __future__ import annotations

import torch

from . import _native as N

_SIG = [N.I, N.P, N.P, N.P] + [N.I] * 17 + [N.I, N.P]
N.register_optional("kfb_conv_igemm", _SIG)
N.register_optional("kfb_conv_wgrad", [N.I, N.P, N.P, N.P] + [N.I] * 12 + [N.I, N.I, N.P])

_WGRAD_TARGET_BLOCKS = 1024


def supported(x, w, stride, pads) -> bool:
    return x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and x.dim() == 4


def _pad8(n):
    return (n + 7) // 8 * 8


def _igemm(x, wmat, y, N_, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, ncol, YH, YW, ys, ldy,
           trans):
    N.call("kfb_conv_igemm", N.dt(x), x.data_ptr(), wmat.data_ptr(), y.data_ptr(), N_, H, W, C,
           OH, OW, KH, KW, sh, sw, pt, pl, ncol, YH, YW, ys, ldy, int(trans), N.stream(x.device))


def conv_fwd(x, wl, stride, pads):
    """x [N,H,W,C] (C%8==0), wl [Cout,KH,KW,C] compute dtype -> y [N,OH,OW,Cout]."""
    n, H, W, C = x.shape
    cout, KH, KW, _ = wl.shape
    sh, sw = stride
    pt, pb, pl, pr = pads
    OH = (H + pt + pb - KH) // sh + 1
    OW = (W + pl + pr - KW) // sw + 1
    y = torch.empty((n, OH, OW, cout), dtype=x.dtype, device=x.device)
    _igemm(x, wl, y, n, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, cout, OH, OW, 1, cout, False)
    return y


def conv_dgrad(dy, wl, x_shape, stride, pads):
    n, H, W, C = x_shape
    cout, KH, KW, _ = wl.shape
    _, OH, OW, _ = dy.shape
    sh, sw = stride
    pt, pb, pl, pr = pads
    if KH == 1 and KW == 1 and pt == 0 and pl == 0:
        wt = wl.reshape(cout, C).t().contiguous()  # [Cin][Cout]
        if sh == 1 and sw == 1 and OH == H and OW == W:
            dx = torch.empty((n, H, W, C), dtype=dy.dtype, device=dy.device)
        else:
            dx = torch.zeros((n, H, W, C), dtype=dy.dtype, device=dy.device)
        # GEMM over dY pixels (1x1, stride 1 in dY space), scattered by ys.
        ys = sh if sh == sw else None
        if ys is None:
            return None
        _igemm(dy, wt, dx, n, OH, OW, cout, OH, OW, 1, 1, 1, 1, 0, 0, C, H, W, ys, C, False)
        return dx
    if sh == 1 and sw == 1 and KH - 1 - pt >= 0 and KH - 1 - pb >= 0 \
            and KW - 1 - pl >= 0 and KW - 1 - pr >= 0:
        # stride-1 transposed conv == forward conv of dY with the spatially
        # flipped, channel-transposed kernel and complementary padding.
        wf = wl.flip(1, 2).permute(3, 1, 2, 0).contiguous()  # [Cin][KH][KW][Cout]
        dx = torch.empty((n, H, W, C), dtype=dy.dtype, device=dy.device)
        _igemm(dy, wf, dx, n, OH, OW, cout, H, W, KH, KW, 1, 1, KH - 1 - pt, KW - 1 - pl, C,
               H, W, 1, C, False)
        return dx
    wd = wl.permute(3, 1, 2, 0).contiguous()  # [Cin][KH][KW][Cout]
    dx = torch.empty((n, H, W, C), dtype=dy.dtype, device=dy.device)
    _igemm(dy, wd, dx, n, OH, OW, cout, H, W, KH, KW, sh, sw, pt, pl, C, H, W, 1, C, True)
    return dx


def conv_wgrad(dy, x, w_shape, stride, pads):
    cout, KH, KW, C = w_shape
    n, H, W, _ = x.shape
    _, OH, OW, _ = dy.shape
    sh, sw = stride
    pt, pb, pl, pr = pads
    dw = torch.zeros((cout, KH, KW, C), dtype=torch.float32, device=x.device)
    N.call("kfb_conv_wgrad", N.dt(x), dy.data_ptr(), x.data_ptr(), dw.data_ptr(), n, H, W, C, OH,
           OW, KH, KW, sh, sw, pt, pl, cout, _WGRAD_TARGET_BLOCKS, N.stream(x.device))
    return dw


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, wl, stride, pads):
        x = x.contiguous()
        if wl is None or wl.dtype != x.dtype:
            wl = w.detach().to(x.dtype)
        cin = x.shape[-1]
        cout = wl.shape[0]
        cin_p, cout_p = _pad8(cin), _pad8(cout)
        xp, wp = x, wl
        if cin_p != cin:
            xp = torch.nn.functional.pad(x, (0, cin_p - cin))
            wp = torch.nn.functional.pad(wp, (0, cin_p - cin))
        if cout_p != cout:
            wp = torch.nn.functional.pad(wp, (0, 0, 0, 0, 0, 0, 0, cout_p - cout))
        wp = wp.contiguous()
        y = conv_fwd(xp, wp, stride, pads)
        if cout_p != cout:
            y = y[..., :cout].contiguous()
        ctx.save_for_backward(xp, wp)
        ctx.meta = (stride, pads, cin, cout, x.shape)
        ctx.x_needs_grad = ctx.needs_input_grad[0]
        return y

    @staticmethod
    def backward(ctx, dy):
        xp, wp = ctx.saved_tensors
        stride, pads, cin, cout, x_shape = ctx.meta
        dy = dy.contiguous()
        cout_p = wp.shape[0]
        if cout_p != cout:
            dy = torch.nn.functional.pad(dy, (0, cout_p - cout))
        dx = None
        if ctx.x_needs_grad:
            dx = conv_dgrad(dy, wp, xp.shape, stride, pads)
            if dx is None:
                raise NotImplementedError("anisotropic strided 1x1 dgrad")
            if dx.shape[-1] != cin:
                dx = dx[..., :cin].contiguous()
        dw = None
        if ctx.needs_input_grad[1]:
            dw = conv_wgrad(dy, xp, wp.shape, stride, pads)
            if dw.shape[0] != cout or dw.shape[-1] != cin:
                dw = dw[:cout, :, :, :cin].contiguous()
        return dx, dw, None, None, None


def conv2d(x, w, wl, stride, pads):
    return _Conv2d.apply(x, w, wl, tuple(stride), tuple(pads))
