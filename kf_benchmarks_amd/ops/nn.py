"""Layer ops on NHWC activations, as autograd Functions.

GPU tensors run our gfx950 kernels (``_native``); CPU tensors run stock
PyTorch ops.  The CPU path is the ``--device=cpu`` plumbing config of the
reference (BASELINE config #1) and the fp32 numerics reference the GPU tests
compare against; it is never a fallback for a GPU tensor.

Layouts:
  activations  [N, H, W, C] contiguous (NHWC), dtype = compute dtype
  conv weight  [Cout, KH, KW, Cin] fp32 master (+ optional low-precision copy)
  affine       [Cin, Cout] fp32 master (TF layout, tcb/convnet_builder.py:331-336)
  BN params    fp32 [C]
"""

from __future__ import annotations

import math
import os
from typing import Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from . import _native as N
from . import conv as _conv

Pads = Tuple[int, int, int, int]  # top, bottom, left, right


def _on_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def _conv_hip():
    from . import conv_hip
    return conv_hip


# ----------------------------------------------------------------- padding math
def same_pads(in_size: int, k: int, s: int) -> Tuple[int, int]:
    """TF 'SAME' padding (begin, end) for one spatial dim."""
    out = (in_size + s - 1) // s
    total = max((out - 1) * s + k - in_size, 0)
    return total // 2, total - total // 2


def conv_out_size(in_size: int, k: int, s: int, pb: int, pe: int) -> int:
    return (in_size + pb + pe - k) // s + 1


def resolve_pads(mode: str, H: int, W: int, kh: int, kw: int, sh: int, sw: int) -> Pads:
    """Padding for 'SAME', 'VALID' and 'SAME_RESNET' (explicit symmetric-ish
    pad then VALID when strided, tcb/convnet_builder.py:159-183)."""
    if mode == "VALID":
        return (0, 0, 0, 0)
    if mode == "SAME" or (mode == "SAME_RESNET" and sh == 1 and sw == 1):
        pt, pb = same_pads(H, kh, sh)
        pl, pr = same_pads(W, kw, sw)
        return (pt, pb, pl, pr)
    if mode == "SAME_RESNET":
        pt = (kh - 1) // 2
        pl = (kw - 1) // 2
        return (pt, kh - 1 - pt, pl, kw - 1 - pl)
    raise ValueError("unknown padding mode %r" % mode)


# ------------------------------------------------------------------------ conv
def conv2d(x, w, w_lp, stride: Tuple[int, int], pads: Pads, impl: str = "hip",
           stats: Optional[torch.Tensor] = None, w_t: Optional[torch.Tensor] = None,
           bias: Optional[torch.Tensor] = None, relu: bool = False):
    """NHWC convolution.  ``w_lp`` is the compute-dtype copy of the fp32
    master ``w`` (None -> cast on the fly).  ``stats`` (GPU): zeroed
    [2*32*Cout] fp32 buffer that receives the BN statistics of the output.
    ``bias`` / ``relu``: fused epilogue where ops.conv.fuses_bias_act(x)."""
    return _conv.conv2d(x, w, w_lp, stride, pads, impl, stats, w_t, bias, relu)


# ------------------------------------------------------------------ batch norm
def _bn_cpu(x, gamma, beta, residual, rm, rv, decay, eps, relu, training):
    xc = x.permute(0, 3, 1, 2)
    g = gamma if gamma is not None else torch.ones_like(beta)
    y = F.batch_norm(xc.float(), rm, rv, g, beta, training=training, momentum=1.0 - decay,
                     eps=eps)
    y = y.permute(0, 2, 3, 1)
    if residual is not None:
        y = y + residual.float()
    if relu == 2:
        y = y.clamp(0.0, 6.0)
    elif relu:
        y = torch.relu(y)
    return y.to(x.dtype).contiguous()


def bn_act_code(activation, x, residual=None) -> int:
    """The ``relu`` code a BN applies itself for ``activation``: 1 ReLU, 2
    ReLU6 (MobileNet-v2) where the GPU apply pass can also write the bit
    mask its consumers' dgrad epilogues gate with (2-byte dtype, C % 8 == 0,
    no residual; csrc/bn.hip act_apply / act_pass), else 0 (the caller
    applies the activation as its own pass)."""
    if activation == "relu":
        return 1
    if activation == "relu6" and residual is None and x.is_cuda and x.element_size() == 2 \
            and x.shape[-1] % 8 == 0 and _RELU_BITS and _conv.FUSE_BN and _RELU6_IN_BN:
        return 2
    return 0


# ReLU6 applied by the BN it follows (bn_act_code); off: a separate act pass
_RELU6_IN_BN = True


# Consumers' dgrad epilogues could recompute a non-residual BN's ReLU mask
# from x_bn instead of reading the BN output: off (the output read is the conv
# input the following wgrad reads anyway, and reading it first leaves it in
# the 256 MB last-level cache; ResNet-50 bs256: 11667 img/s read vs 11567
# recompute)
_MASK_RECOMPUTE = False


class BNLink:
    """Ties a training-mode BN's output y to its consumers so their backward
    kernels can finish the BN's backward work in their epilogues
    (csrc/conv_igemm.hip):

    * every consumer is a conv (input), a BN that adds y as its residual or
      a max / average pool; the ConvNetBuilder counts them (``convs``,
      ``resid``, ``pools``) and marks any other use (``other``), which
      disables the fusion.  A pool contributes like a non-fused conv: it
      deposits its input gradient, or as the last contributor returns it
      summed with the pending one;
    * in backward, all but the last contributor *deposit* their gradient of y
      here (``pending``) and return None to autograd; the last one, if it is a
      conv, adds ``pending`` in its dgrad epilogue, applies y's ReLU mask and
      accumulates the BN backward partial sums (``partials``), so the BN
      backward is only finalize + apply.  A residual-BN last contributor
      returns the summed gradient instead (unfused path).
    """

    __slots__ = ("x_bn", "mean", "relu", "convs", "resid", "pools", "other", "accum", "partials",
                 "pending",
                 "pending_owned", "arrived", "mcoef", "pending_sparse", "pending_event", "mbits",
                 "gfin", "dual", "partials_r")

    def __init__(self, x_bn, mean, relu, mcoef=None):
        self.x_bn, self.mean, self.relu = x_bn, mean, relu
        # [scale | shift] of y = relu(x_bn * scale + shift) when the BN has no
        # residual add: a consumer's dgrad epilogue recomputes the ReLU mask
        # from x_bn instead of reading y
        self.mcoef = mcoef
        # y's ReLU bit mask (uint8 [rows * C / 8], bit k of byte e/8 = y[e+k] > 0)
        # written by the BN apply pass when the mask cannot be recomputed from
        # x_bn (residual add): a consumer's dgrad epilogue reads it instead of y
        self.mbits = None
        self.convs, self.resid, self.pools, self.other = 0, 0, 0, False
        # accumulation-only link (a concat output, no BN behind it): the last
        # conv adds the pending gradient in its dgrad epilogue, nothing else
        self.accum = False
        self.partials, self.pending, self.arrived = None, None, 0
        self.pending_owned = False
        # s when every deposited gradient is zero outside the stride-s pixel
        # grid (strided 1x1 "scatter" dgrads), else None
        self.pending_sparse = None
        # contributors may run on different streams (side branches): the
        # pending gradient is complete once this event has fired
        self.pending_event = None
        # (gamma, st = [mean | invstd], beta) of a plain training BN: the
        # last consumer's dgrad may run the BN's backward finalize in its
        # last workgroup (conv_hip.attach_bn_grad_finalize)
        self.gfin = None
        # (x_r, mean_r) of the second BN of a dual-BN output relu(bn(x) +
        # bn_r(x_r)): a streaming 1x1 last consumer also sums bn_r's backward
        # partial into ``partials_r`` ([STATS_SPREAD][C], with the first half
        # of ``partials`` as its sum of dy'); None: the dual backward's pass
        self.dual = None
        self.partials_r = None

    @property
    def fusable(self):
        return not self.other and self.convs >= 1 and _conv.FUSE_BN

    @property
    def total(self):
        return self.convs + self.resid + self.pools

    def arrive(self) -> bool:
        """Registers one gradient contribution; True if it is the last."""
        self.arrived += 1
        return self.arrived >= self.total

    def deposit(self, g, owned=True, sparse=None):
        """``owned``: g is a fresh buffer nothing else reads, so the last
        contributor may accumulate into it in place.  ``sparse``: g is zero
        outside the stride-``sparse`` pixel grid."""
        if self.pending is None:
            self.pending, self.pending_owned = g, owned
            self.pending_sparse = sparse
        else:
            self.take_pending_stream()
            if g.is_cuda and g.is_contiguous() and self.pending.is_contiguous() \
                    and g.dtype == self.pending.dtype and g.shape == self.pending.shape:
                y = torch.empty_like(g)
                N.call("kfb_add", N.dt(g), self.pending.data_ptr(), g.data_ptr(), y.data_ptr(),
                       g.numel(), 0, N.stream(g.device))
                self.pending = y
            else:
                self.pending = self.pending + g
            self.pending_owned = True
            if sparse != self.pending_sparse:
                self.pending_sparse = None
        if g.is_cuda:
            # the stream that produced it (a recordable wait replaces an event)
            self.pending_event = N.stream(g.device)

    def accumulated(self, g, sparse=None):
        """A contributor computed ``g`` = its gradient + ``pending`` (the
        pending gradient as its dgrad epilogue's addend): g replaces it."""
        if sparse != self.pending_sparse:
            sparse = None
        self.pending, self.pending_owned, self.pending_sparse = g, True, sparse
        if g.is_cuda:
            self.pending_event = N.stream(g.device)

    def take_pending_stream(self):
        """Makes the current stream wait for the pending gradient (written
        on whatever stream its contributors ran on) before using it."""
        if self.pending is not None and self.pending_event is not None:
            cur = N.stream(self.pending.device)
            if cur != self.pending_event:
                N.stream_wait(cur, self.pending_event, device_only=True)
                self.pending.record_stream(torch.cuda.current_stream(self.pending.device))
            self.pending_event = None


def _grad_sink(p):
    """The flat-buffer gradient view of a FlatParams-managed parameter (the
    kernels accumulate straight into it), or None."""
    return getattr(p, "_kfb_grad_sink", None) if p is not None else None


def _grad_ready(p):
    cb = getattr(p, "_kfb_ready_cb", None)
    if cb is not None:
        cb(p)


# off (tests): consumers' dgrad epilogues read the BN output itself for the
# ReLU mask (16x the bytes of the bit mask)
_RELU_BITS = True


def _relu_bits_buffer(x, rows, C):
    """uint8 [rows * C / 8] for the BN apply pass's ReLU bit mask, or None
    (2-byte dtypes with C % 8 == 0 only: one byte per 16-byte vector)."""
    if not _RELU_BITS or x.element_size() != 2 or C % 8 or not _conv.FUSE_BN:
        return None
    return torch.empty((rows * C // 8,), dtype=torch.uint8, device=x.device)


RECOMPUTED = 0  # BN forwards that recomputed their input (tests)


class _BatchNormTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, residual, rm, rv, decay, eps, relu, stats):
        x = x.contiguous()
        C = x.shape[-1]
        rows = x.numel() // C
        dev = x.device
        fin = None
        if stats is not None and getattr(stats, "_kfb_finalized", False):
            # the producing conv's last workgroup already finalized into the
            # BN layer's persistent st / coef (conv_hip.attach_bn_finalize)
            fin = stats._kfb_fin
        if stats is not None:  # partial sums from the producing conv's epilogue
            nslab = stats.numel() // (2 * C)
            psum, psq = stats[:nslab * C], stats[nslab * C:]
            if fin is not None:
                coef = fin[7]
            else:
                ws = torch.empty((4 * C,), dtype=torch.float32, device=dev)
                coef = ws[:2 * C]
        else:
            nslab = N.query("kfb_bn_num_slabs", rows, C)
            ws = torch.empty((2 * nslab * C + 4 * C,), dtype=torch.float32, device=dev)
            psum, psq = ws[:nslab * C], ws[nslab * C:2 * nslab * C]
            coef = ws[2 * nslab * C:2 * nslab * C + 2 * C]
        st = fin[6] if fin is not None else torch.empty((2, C), dtype=torch.float32, device=dev)
        y = torch.empty_like(x)
        res = residual.contiguous() if residual is not None else None
        rec = relu == 1 and residual is None and _MASK_RECOMPUTE
        mbits = _relu_bits_buffer(x, rows, C) if relu and not rec else None
        # x never stored by its producing conv (conv_hip.conv_fwd, statistics
        # only): the apply pass recomputes it from the conv's input and
        # weights and stores it on the way (csrc/conv_s1.hip EPI_APPLY)
        rc = getattr(x, "_kfb_recompute", None) if stats is not None else None
        if rc is not None:
            if relu == 2:
                raise RuntimeError("BN recompute path with ReLU6 is not supported")
            global RECOMPUTED
            RECOMPUTED += 1
            xin, wl = rc
            x._kfb_recompute = None
            n_, h_, w_, cin = xin.shape
            N.call("kfb_bn_fwd_train_recompute", N.dt(x), xin.data_ptr(), wl.data_ptr(),
                   x.data_ptr(), y.data_ptr(), N.ptr(res), n_, h_, w_, cin, C, N.ptr(gamma),
                   N.ptr(beta), float(decay), float(eps), N.ptr(rm), N.ptr(rv),
                   st[0].data_ptr(), st[1].data_ptr(), coef[:C].data_ptr(),
                   coef[C:].data_ptr(), psum.data_ptr(), psq.data_ptr(), nslab,
                   int(fin is not None), N.ptr(_conv_hip().stats_shift(stats)), int(relu),
                   N.ptr(mbits), N.stream(dev))
        else:
            N.call("kfb_bn_fwd_train", N.dt(x), x.data_ptr(), N.ptr(res), y.data_ptr(), rows, C,
                   N.ptr(gamma), N.ptr(beta), float(decay), float(eps), N.ptr(rm), N.ptr(rv),
                   st[0].data_ptr(), st[1].data_ptr(), coef[:C].data_ptr(),
                   coef[C:].data_ptr(), psum.data_ptr(), psq.data_ptr(), nslab, int(relu),
                   2 if fin is not None else int(stats is not None),
                   N.ptr(_conv_hip().stats_shift(stats)), N.ptr(mbits), N.stream(dev))
        ctx.save_for_backward(x, y if relu else None, gamma, st)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.gamma, ctx.beta = gamma, beta
        link = BNLink(x, st[0], relu, coef if rec else None)
        link.mbits = mbits
        if relu == 2 and mbits is None:
            link.other = True  # consumers may only gate ReLU6 with its bit mask
        link.gfin = (gamma, st, beta)
        y._kfb_bn_link = link
        ctx.link = link
        ctx.res_link = getattr(residual, "_kfb_bn_link", None) if residual is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, gamma, st = ctx.saved_tensors
        dx, dgamma, dbeta, dres = _bn_backward(x, y, gamma, st, dy, ctx.relu, ctx.has_res,
                                               ctx.link, ctx.res_link, ctx.gamma, ctx.beta)
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None


def _bn_grad_targets(gamma_p, beta_p, C, dev):
    """Where a BN backward writes dgamma/dbeta: straight into the flat
    gradient buffer (direct) or a fresh [2, C] tensor (dparams)."""
    gsink, bsink = _grad_sink(gamma_p), _grad_sink(beta_p)
    direct = bsink is not None and (gamma_p is None or gsink is not None) and _conv.FUSE_BN
    if direct:
        return True, N.ptr(gsink), bsink.data_ptr(), None
    dparams = torch.empty((2, C), dtype=torch.float32, device=dev)
    return False, dparams[0].data_ptr(), dparams[1].data_ptr(), dparams


def _bn_grad_result(direct, dparams, gamma_p, beta_p):
    if direct:
        _grad_ready(gamma_p)
        _grad_ready(beta_p)
        return None, None
    return (dparams[0] if gamma_p is not None else None), dparams[1]


def _bn_backward(x, y, gamma, st, dy, relu, has_res, link, res_link, gamma_p, beta_p,
                 alias_res=False):
    """BN backward (kfb_bn_bwd): returns (dx, dgamma, dbeta, dres); dgamma and
    dbeta are None when they went straight into the flat gradient buffer.
    ``alias_res``: the caller only reads dres, so it may be dy itself."""
    dy = dy.contiguous()
    C = x.shape[-1]
    rows = x.numel() // C
    dev = x.device
    pre = link is not None and link.partials is not None
    gdone = None
    if pre:
        parts = link.partials
        nslab = parts.numel() // (2 * C)
        pdy, pdyx = parts[:nslab * C], parts[nslab * C:]
        if getattr(parts, "_kfb_gfinalized", False):
            # the dgrad that filled the partials finalized in its last
            # workgroup (dgamma / dbeta and the apply coefficients)
            gdone = parts._kfb_gfin_out
            coef = gdone[0]
        else:
            coef = torch.empty((3 * C,), dtype=torch.float32, device=dev)
        link.partials = None
    else:
        nslab = N.query("kfb_bn_num_slabs", rows, C)
        ws = torch.empty((2 * nslab * C + 3 * C,), dtype=torch.float32, device=dev)
        pdy, pdyx = ws[:nslab * C], ws[nslab * C:2 * nslab * C]
        coef = ws[2 * nslab * C:]
    if gdone is not None:
        direct, dgp, dbp, dparams = gdone[1]
    else:
        direct, dgp, dbp, dparams = _bn_grad_targets(gamma_p, beta_p, C, dev)
    dx = torch.empty_like(x)
    rl = res_link
    res_fused = has_res and rl is not None and rl.fusable
    # the residual's gradient is dy' (masked dy): with a pre-masked dy it
    # is dy itself, no kernel write needed
    dres = torch.empty_like(x) if has_res and not (pre and (res_fused or alias_res)) else None
    N.call("kfb_bn_bwd", N.dt(x), dy.data_ptr(), N.ptr(y), x.data_ptr(), dx.data_ptr(),
           N.ptr(dres), rows, C, N.ptr(gamma), st[0].data_ptr(), st[1].data_ptr(),
           dgp, dbp, pdy.data_ptr(), pdyx.data_ptr(),
           nslab, coef[:C].data_ptr(), coef[C:2 * C].data_ptr(), coef[2 * C:].data_ptr(),
           int(relu), int(direct), 2 if gdone is not None else int(pre), N.stream(dev))
    if has_res and dres is None:
        dres = dy
    if res_fused:
        if rl.arrive():
            if rl.pending is not None:
                rl.take_pending_stream()
                dres = dres + rl.pending
                rl.pending = None
        else:
            rl.deposit(dres, owned=dres is not dy)
            dres = None
    dgamma, dbeta = _bn_grad_result(direct, dparams, gamma_p, beta_p)
    return dx, dgamma, dbeta, dres


class DeferredBN:
    """A training-mode BN (no ReLU, no residual) not applied yet: its raw
    input ``x`` (a conv output whose epilogue accumulated ``stats``) and the
    BN's parameters.  As the ``residual`` of another BN it is applied inside
    that BN's apply pass (:func:`batch_norm_dual`), so its output is never
    materialized; any other use calls :meth:`materialize`."""

    __slots__ = ("x", "gamma", "beta", "rm", "rv", "decay", "eps", "stats")

    def __init__(self, x, gamma, beta, rm, rv, decay, eps, stats):
        self.x, self.gamma, self.beta, self.rm, self.rv = x, gamma, beta, rm, rv
        self.decay, self.eps, self.stats = decay, eps, stats

    def materialize(self):
        return _BatchNormTrain.apply(self.x, self.gamma, self.beta, None, self.rm, self.rv,
                                     self.decay, self.eps, False, self.stats)


# the dual BN backward hands a pre-masked dy to bn_r as is (no copy)
_DUAL_ALIAS_RES = True
# ... and takes bn_r's backward partials from its last consumer's streaming
# 1x1 dgrad epilogue (kfb_conv_s1_dgrad_dual) instead of a pass over dy and
# xr (off: that pass)
_S1_DUAL = True
# ... and with a pre-masked dy runs both BN backwards with one apply pass
# (kfb_bn_bwd_dual; off: two separate BN backwards)
_DUAL_BWD_FUSE = True


class _BatchNormTrainDual(torch.autograd.Function):
    """y = relu?(bn(x) + bn_r(xr)), both BNs in training mode with conv-epilogue
    statistics (kfb_bn_fwd_train_dual: one apply pass over x and xr).  The
    backward is that of the two separate BNs: bn_r's output gradient is the
    ReLU-masked dy, which the first BN backward writes as its residual
    gradient."""

    @staticmethod
    def forward(ctx, x, gamma, beta, xr, gamma_r, beta_r, rm, rv, rm_r, rv_r, decay, eps,
                decay_r, eps_r, relu, stats, stats_r):
        x, xr = x.contiguous(), xr.contiguous()
        C = x.shape[-1]
        rows = x.numel() // C
        dev = x.device
        nslab, nslab_r = stats.numel() // (2 * C), stats_r.numel() // (2 * C)
        ws = torch.empty((2, 4, C), dtype=torch.float32, device=dev)  # [bn][mean|invstd|scale|shift]
        y = torch.empty_like(x)
        mbits = _relu_bits_buffer(x, rows, C) if relu else None
        N.call("kfb_bn_fwd_train_dual", N.dt(x), x.data_ptr(), xr.data_ptr(), y.data_ptr(),
               rows, C, N.ptr(gamma), N.ptr(beta), float(decay), float(eps), N.ptr(rm),
               N.ptr(rv), ws[0, 0].data_ptr(), ws[0, 1].data_ptr(), ws[0, 2].data_ptr(),
               ws[0, 3].data_ptr(), stats[:nslab * C].data_ptr(), stats[nslab * C:].data_ptr(),
               nslab, N.ptr(gamma_r), N.ptr(beta_r), float(decay_r), float(eps_r), N.ptr(rm_r),
               N.ptr(rv_r), ws[1, 0].data_ptr(), ws[1, 1].data_ptr(), ws[1, 2].data_ptr(),
               ws[1, 3].data_ptr(), stats_r[:nslab_r * C].data_ptr(),
               stats_r[nslab_r * C:].data_ptr(), nslab_r, int(relu),
               N.ptr(_conv_hip().stats_shift(stats)), N.ptr(_conv_hip().stats_shift(stats_r)),
               N.ptr(mbits), N.stream(dev))
        st, st_r = ws[0, :2], ws[1, :2]
        ctx.save_for_backward(x, y if relu else None, gamma, st, xr, gamma_r, st_r)
        ctx.relu = relu
        ctx.params = (gamma, beta, gamma_r, beta_r)
        link = BNLink(x, st[0], relu)
        link.mbits = mbits
        if _S1_DUAL and _DUAL_BWD_FUSE and relu and mbits is not None:
            link.dual = (xr, st_r[0])
        y._kfb_bn_link = link
        ctx.link = link
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, gamma, st, xr, gamma_r, st_r = ctx.saved_tensors
        gp, bp, gp_r, bp_r = ctx.params
        link = ctx.link
        if _DUAL_BWD_FUSE and link is not None and link.partials is not None:
            dy = dy.contiguous()
            C = x.shape[-1]
            rows = x.numel() // C
            dev = x.device
            parts = link.partials
            link.partials = None
            nslab = parts.numel() // (2 * C)
            pr_ready = link.partials_r is not None
            if pr_ready:
                # bn_r's partials from the dgrad epilogue: sum dy' (shared) | sum dy'(xr - mean_r)
                nslab_r = nslab
                pdy_r, pdyx_r = parts[:nslab * C].data_ptr(), link.partials_r.data_ptr()
                link.partials_r = None
                coef = torch.empty((6, C), dtype=torch.float32, device=dev)
            else:
                nslab_r = N.query("kfb_bn_num_slabs", rows, C)
                ws = torch.empty((2 * nslab_r * C + 6 * C,), dtype=torch.float32, device=dev)
                pr = ws[:2 * nslab_r * C]
                pdy_r, pdyx_r = pr[:nslab_r * C].data_ptr(), pr[nslab_r * C:].data_ptr()
                coef = ws[2 * nslab_r * C:].view(6, C)
            t, tr = _bn_grad_targets(gp, bp, C, dev), _bn_grad_targets(gp_r, bp_r, C, dev)
            dx, dxr = torch.empty_like(x), torch.empty_like(xr)
            N.call("kfb_bn_bwd_dual", N.dt(x), dy.data_ptr(), x.data_ptr(), xr.data_ptr(),
                   dx.data_ptr(), dxr.data_ptr(), rows, C, N.ptr(gamma), st[0].data_ptr(),
                   st[1].data_ptr(), t[1], t[2], parts[:nslab * C].data_ptr(),
                   parts[nslab * C:].data_ptr(), nslab, coef[0].data_ptr(),
                   coef[1].data_ptr(), coef[2].data_ptr(), int(t[0]), N.ptr(gamma_r),
                   st_r[0].data_ptr(), st_r[1].data_ptr(), tr[1], tr[2], pdy_r, pdyx_r, nslab_r,
                   coef[3].data_ptr(), coef[4].data_ptr(), coef[5].data_ptr(), int(tr[0]),
                   int(pr_ready), N.stream(dev))
            dg, db = _bn_grad_result(t[0], t[3], gp, bp)
            dg_r, db_r = _bn_grad_result(tr[0], tr[3], gp_r, bp_r)
            return (dx, dg, db, dxr, dg_r, db_r) + (None,) * 11
        dx, dg, db, g = _bn_backward(x, y, gamma, st, dy, ctx.relu, True, ctx.link, None, gp, bp,
                                     alias_res=_DUAL_ALIAS_RES)
        dxr, dg_r, db_r, _ = _bn_backward(xr, None, gamma_r, st_r, g, False, False, None, None,
                                          gp_r, bp_r)
        return (dx, dg, db, dxr, dg_r, db_r) + (None,) * 11


def batch_norm_dual(x, gamma, beta, running_mean, running_var, decay, eps, relu, stats,
                    r: "DeferredBN"):
    """relu?(bn(x) + r) for a deferred BN ``r`` (training mode, GPU, both
    inputs with conv-epilogue statistics); otherwise r is materialized first."""
    if stats is None or r.stats is None or not _on_gpu(x) or x.shape != r.x.shape:
        return batch_norm(x, gamma, beta, running_mean, running_var, decay, eps, True, relu,
                          r.materialize(), stats=stats)
    return _BatchNormTrainDual.apply(x, gamma, beta, r.x, r.gamma, r.beta, running_mean,
                                     running_var, r.rm, r.rv, decay, eps, r.decay, r.eps, relu,
                                     stats, r.stats)


def batch_norm(x, gamma: Optional[torch.Tensor], beta: torch.Tensor,
               running_mean: torch.Tensor, running_var: torch.Tensor, decay: float, eps: float,
               training: bool, relu: bool = False, residual: Optional[torch.Tensor] = None,
               stats: Optional[torch.Tensor] = None):
    """y = relu?(bn(x) + residual?).  ``gamma=None`` means scale=False
    (constant 1, tcb/convnet_builder.py:437-438 default).  ``stats``: the
    [2][32][C] partial sums the producing conv kernel already accumulated."""
    if not _on_gpu(x):
        return _bn_cpu(x, gamma, beta, residual, running_mean, running_var, decay, eps, relu,
                       training)
    if training:
        return _BatchNormTrain.apply(x, gamma, beta, residual, running_mean, running_var,
                                     decay, eps, relu, stats)
    return _bn_infer_gpu(x, gamma, beta, residual, running_mean, running_var, eps, relu)


def _bn_infer_gpu(x, gamma, beta, residual, rm, rv, eps, relu):
    x = x.contiguous()
    C = x.shape[-1]
    rows = x.numel() // C
    coef = torch.empty((2, C), dtype=torch.float32, device=x.device)
    y = torch.empty_like(x)
    res = residual.contiguous() if residual is not None else None
    N.call("kfb_bn_fwd_infer", N.dt(x), x.data_ptr(), N.ptr(res), y.data_ptr(), rows, C,
           N.ptr(gamma), N.ptr(beta), rm.data_ptr(), rv.data_ptr(), float(eps),
           coef[0].data_ptr(), coef[1].data_ptr(), int(relu), N.stream(x.device))
    return y


# -------------------------------------------------------------- bias + relu
class _BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b, relu):
        x = x.contiguous()
        C = x.shape[-1]
        rows = x.numel() // C
        y = torch.empty_like(x)
        N.call("kfb_bias_act", N.dt(x), x.data_ptr(), N.ptr(b), y.data_ptr(), rows, C, int(relu),
               N.stream(x.device))
        ctx.save_for_backward(y if relu else None)
        ctx.relu, ctx.has_b, ctx.C = relu, b is not None, C
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.contiguous()
        C = ctx.C
        rows = dy.numel() // C
        dx = torch.empty_like(dy) if ctx.relu else dy
        db = None
        pb = None
        nslab = 1
        if ctx.has_b:
            nslab = N.query("kfb_colsum_num_slabs", rows, C)
            pb = torch.empty((nslab * C,), dtype=torch.float32, device=dy.device)
            db = torch.empty((C,), dtype=torch.float32, device=dy.device)
        if ctx.relu or ctx.has_b:
            N.call("kfb_act_bwd_bias", N.dt(dy), dy.data_ptr(), N.ptr(y), dx.data_ptr(), rows, C,
                   int(ctx.relu), N.ptr(pb), nslab, N.ptr(db), 0, N.stream(dy.device))
        return dx, db, None


def bias_act(x, b: Optional[torch.Tensor], relu: bool):
    if b is None and not relu:
        return x
    if not _on_gpu(x):
        y = x.float() + b if b is not None else x.float()
        if relu:
            y = torch.relu(y)
        return y.to(x.dtype)
    return _BiasAct.apply(x, b, relu)


def relu(x):
    return bias_act(x, None, True)


N.register_optional("kfb_act_fwd", [N.I, N.P, N.P, N.L, N.I, N.P])
N.register_optional("kfb_act_bwd", [N.I, N.P, N.P, N.P, N.L, N.I, N.P])
_ACT_KINDS = {"relu6": 1, "tanh": 2}


class _Act(torch.autograd.Function):
    """relu6 / tanh on the GPU (csrc/elementwise.hip act_fwd_k / act_bwd_k;
    the backward reads the output)."""

    @staticmethod
    def forward(ctx, x, kind):
        x = x.contiguous()
        y = torch.empty_like(x)
        N.call("kfb_act_fwd", N.dt(x), x.data_ptr(), y.data_ptr(), x.numel(), kind,
               N.stream(x.device))
        ctx.save_for_backward(y)
        ctx.kind = kind
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        N.call("kfb_act_bwd", N.dt(dy), dy.data_ptr(), y.data_ptr(), dx.data_ptr(), dy.numel(),
               ctx.kind, N.stream(dy.device))
        return dx, None


def activation(x, kind: Optional[str]):
    if kind in (None, "linear"):
        return x
    if kind == "relu":
        return relu(x)
    if kind in _ACT_KINDS and _on_gpu(x) and x.numel() > 0:
        return _Act.apply(x, _ACT_KINDS[kind])
    if kind == "tanh":
        return torch.tanh(x)
    if kind == "relu6":
        return torch.clamp(x, 0.0, 6.0)
    raise KeyError("Invalid activation type '%s'" % kind)


class _Add(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, relu):
        a, b = a.contiguous(), b.contiguous()
        y = torch.empty_like(a)
        N.call("kfb_add", N.dt(a), a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(),
               int(relu), N.stream(a.device))
        ctx.save_for_backward(y if relu else None)
        ctx.relu = relu
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        if ctx.relu:
            dy = dy.contiguous()
            C = dy.shape[-1]
            dx = torch.empty_like(dy)
            N.call("kfb_act_bwd_bias", N.dt(dy), dy.data_ptr(), y.data_ptr(), dx.data_ptr(),
                   dy.numel() // C, C, 1, None, 1, None, 0, N.stream(dy.device))
            return dx, dx, None
        return dy, dy, None


class _FanOut(torch.autograd.Function):
    """One tensor read by k branches: k aliases whose gradients are summed by
    native adds in the backward (autograd would sum them with torch kernels,
    which a launch tape cannot record)."""

    @staticmethod
    def forward(ctx, x, k):
        ctx.k = k
        return tuple(x.view_as(x) for _ in range(k))

    @staticmethod
    def backward(ctx, *grads):
        gs = [g for g in grads if g is not None]
        if not gs:
            return None, None
        acc = gs[0].contiguous()
        for g in gs[1:]:
            g = g.contiguous()
            y = torch.empty_like(acc)
            N.call("kfb_add", N.dt(acc), acc.data_ptr(), g.data_ptr(), y.data_ptr(), acc.numel(),
                   0, N.stream(acc.device))
            acc = y
        return acc, None


def fanout(x, k: int, force: bool = False):
    """``k`` aliases of ``x`` for ``k`` consumers (GPU: native gradient sum).
    A BN output keeps its link (its conv consumers finish the BN backward)
    unless ``force``: then the aliases carry no link, the BN backward runs
    unfused, and the gradient sum is still native (a consumer that is not a
    conv, e.g. a residual add, makes the link unfusable anyway)."""
    if k <= 1 or not _on_gpu(x) or not x.requires_grad or \
            (getattr(x, "_kfb_bn_link", None) is not None and not force):
        return [x] * k
    return list(_FanOut.apply(x, k))


class _Mul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        y = torch.empty_like(a)
        N.call("kfb_mul", N.dt(a), a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(),
               N.stream(a.device))
        ctx.save_for_backward(a, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        a, b = ctx.saved_tensors
        dy = dy.contiguous()
        da, db = torch.empty_like(a), torch.empty_like(b)
        N.call("kfb_mul_bwd", N.dt(a), a.data_ptr(), b.data_ptr(), dy.data_ptr(), da.data_ptr(),
               db.data_ptr(), a.numel(), N.stream(a.device))
        return da, db


def mul(a, b):
    """Elementwise a * b of one shape and dtype (GPU: native forward and
    backward, so a launch tape can record it)."""
    if not _on_gpu(a):
        return a * b
    if a.shape != b.shape or a.dtype != b.dtype:
        raise ValueError("mul: operands must have one shape and dtype")
    return _Mul.apply(a, b)


def add(a, b, relu: bool = False):
    if not _on_gpu(a):
        y = a + b
        return torch.relu(y) if relu else y
    return _Add.apply(a, b, relu)


# --------------------------------------------------------------------- pooling
def pool_geometry(x_shape, kh, kw, sh, sw, mode):
    n, H, W, C = x_shape
    pt, pb, pl, pr = resolve_pads(mode, H, W, kh, kw, sh, sw)
    OH = conv_out_size(H, kh, sh, pt, pb)
    OW = conv_out_size(W, kw, sw, pl, pr)
    return (pt, pb, pl, pr), OH, OW


def _pool_cpu(x, kh, kw, sh, sw, pads, kind):
    pt, pb, pl, pr = pads
    xc = x.permute(0, 3, 1, 2).float()
    if kind == "max":
        xp = F.pad(xc, (pl, pr, pt, pb), value=-math.inf)
        y = F.max_pool2d(xp, (kh, kw), (sh, sw))
    else:
        xp = F.pad(xc, (pl, pr, pt, pb))
        ones = F.pad(torch.ones_like(xc[:1, :1]), (pl, pr, pt, pb))
        s = F.avg_pool2d(xp, (kh, kw), (sh, sw)) * (kh * kw)
        cnt = F.avg_pool2d(ones, (kh, kw), (sh, sw)) * (kh * kw)
        y = s / cnt
    return y.permute(0, 2, 3, 1).to(x.dtype).contiguous()


def _pool_link_grad(link, dx):
    """A pool's input gradient under the BNLink protocol: deposited (None to
    autograd) unless this pool is the link's last contributor, which returns
    it summed with the pending gradient."""
    if link is None or not link.fusable:
        return dx
    if not link.arrive():
        link.deposit(dx)
        return None
    if link.pending is not None:
        link.take_pending_stream()
        p = link.pending
        if dx.is_cuda and dx.is_contiguous() and p.is_contiguous() and p.dtype == dx.dtype \
                and p.shape == dx.shape:
            # native in-place sum into the fresh pool gradient (recordable by a
            # launch tape, unlike a torch add)
            N.call("kfb_add", N.dt(dx), p.data_ptr(), dx.data_ptr(), dx.data_ptr(), dx.numel(), 0,
                   N.stream(dx.device))
        elif link.pending_owned:
            dx = p.add_(dx)
        else:
            dx = dx.add_(p)
        link.pending = None
    return dx


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kh, kw, sh, sw, pads, OH, OW):
        ctx.link = getattr(x, "_kfb_bn_link", None)
        x = x.contiguous()
        n, H, W, C = x.shape
        y = torch.empty((n, OH, OW, C), dtype=x.dtype, device=x.device)
        idx = torch.empty((n, OH, OW, C), dtype=torch.uint8, device=x.device)
        geo = (n, H, W, C, OH, OW, kh, kw, sh, sw, pads[0], pads[2])
        N.call("kfb_maxpool_fwd", N.dt(x), x.data_ptr(), y.data_ptr(), idx.data_ptr(), *geo,
               N.stream(x.device))
        ctx.save_for_backward(idx)
        ctx.geo = geo
        ctx.dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        dy = dy.contiguous()
        n, H, W, C = ctx.geo[:4]
        dx = torch.empty((n, H, W, C), dtype=dy.dtype, device=dy.device)
        N.call("kfb_maxpool_bwd", N.dt(dy), dy.data_ptr(), idx.data_ptr(), dx.data_ptr(),
               *ctx.geo, N.stream(dy.device))
        return _pool_link_grad(ctx.link, dx), None, None, None, None, None, None, None


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kh, kw, sh, sw, pads, OH, OW):
        ctx.link = getattr(x, "_kfb_bn_link", None)
        x = x.contiguous()
        n, H, W, C = x.shape
        y = torch.empty((n, OH, OW, C), dtype=x.dtype, device=x.device)
        geo = (n, H, W, C, OH, OW, kh, kw, sh, sw, pads[0], pads[2])
        N.call("kfb_avgpool_fwd", N.dt(x), x.data_ptr(), y.data_ptr(), *geo, N.stream(x.device))
        ctx.geo = geo
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        n, H, W, C = ctx.geo[:4]
        dx = torch.empty((n, H, W, C), dtype=dy.dtype, device=dy.device)
        N.call("kfb_avgpool_bwd", N.dt(dy), dy.data_ptr(), dx.data_ptr(), *ctx.geo,
               N.stream(dy.device))
        return _pool_link_grad(ctx.link, dx), None, None, None, None, None, None, None


N.register_optional("kfb_bn_relu_maxpool_fwd", [N.I, N.P, N.P, N.P] + [N.I] * 12 +
                    [N.P, N.P, N.F, N.F] + [N.P] * 8 + [N.I, N.P, N.P])
N.register_optional("kfb_bn_pool_num_slabs", [N.I] * 8, N.c_int)
N.register_optional("kfb_bn_relu_maxpool_bwd", [N.I, N.P, N.P, N.P, N.P, N.P] + [N.I] * 12 +
                    [N.P] * 7 + [N.I] + [N.P] * 3 + [N.I, N.I, N.P])

# The stem BN+ReLU+max-pool backward takes its BN partials from its
# consumers' dgrad epilogue (sum dz', sum dz' (z - beta), rescaled by
# 1 / (gamma * invstd)) instead of its own pass over x.  Default since round
# 4: 18.93 / 18.75 / 18.72 vs 19.09 / 19.06 / 18.82 ms/step interleaved
# (gpurun_out/r10t, profiles/r10_round4_ab.txt); tests/test_model_gpu.py compares
# it with the link off.
_POOL_LINK = True


# Called once at the top of the stem BN+ReLU+max-pool backward (the point
# where every gradient but the stem's is complete or enqueued): the engine
# starts the optimizer on those variables there, beside the stem's backward
# (BenchmarkCNN._early_update)
_BACKWARD_TAIL_HOOK = None


class _BNReluMaxPool(torch.autograd.Function):
    """maxpool(relu(bn_train(x))) with the BN statistics already summed by
    the producing conv (the ResNet stem tail, csrc/bn.hip): neither the BN
    output nor the max-pool input gradient is ever materialized."""

    @staticmethod
    def forward(ctx, x, gamma, beta, rm, rv, decay, eps, stats, kh, kw, sh, sw, pads, OH, OW):
        x = x.contiguous()
        n, H, W, C = x.shape
        dev = x.device
        nslab = stats.numel() // (2 * C)
        st = torch.empty((4, C), dtype=torch.float32, device=dev)  # mean, invstd, scale, shift
        z = torch.empty((n, OH, OW, C), dtype=x.dtype, device=dev)
        idx = torch.empty((n, OH, OW, C), dtype=torch.uint8, device=dev)
        geo = (n, H, W, C, OH, OW, kh, kw, sh, sw, pads[0], pads[2])
        N.call("kfb_bn_relu_maxpool_fwd", N.dt(x), x.data_ptr(), z.data_ptr(), idx.data_ptr(),
               *geo, N.ptr(gamma), N.ptr(beta), float(decay), float(eps), N.ptr(rm), N.ptr(rv),
               st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr(), st[3].data_ptr(),
               stats[:nslab * C].data_ptr(), stats[nslab * C:].data_ptr(), nslab,
               N.ptr(_conv_hip().stats_shift(stats)), N.stream(dev))
        ctx.save_for_backward(x, z, idx, gamma, st)
        ctx.geo = geo
        ctx.gamma, ctx.beta = gamma, beta
        ctx.out_link = None
        if _POOL_LINK and _conv.FUSE_BN:
            # z's consumers (conv1 and the projection shortcut) sum their data
            # gradients in the last one's dgrad epilogue, which also masks them
            # with z > 0 (z * 1 + 0) and accumulates sum(dz') and
            # sum(dz' (z - beta)): the BN partials of this backward
            coef = _conv_hip()._act_link_consts(C, True, dev)[1]
            mu = (beta.detach().float().contiguous() if beta is not None
                  else torch.zeros(C, dtype=torch.float32, device=dev))
            link = BNLink(None, mu, True, coef)
            z._kfb_bn_link = link
            ctx.out_link = link
        return z

    @staticmethod
    def backward(ctx, dz):
        global _BACKWARD_TAIL_HOOK
        hook, _BACKWARD_TAIL_HOOK = _BACKWARD_TAIL_HOOK, None
        if hook is not None:
            hook(ctx.gamma, ctx.beta)
        x, z, idx, gamma, st = ctx.saved_tensors
        dz = dz.contiguous()
        n, H, W, C = ctx.geo[:4]
        dev = x.device
        link = ctx.out_link
        parts = link.partials if link is not None else None
        if link is not None:
            link.partials = None
        if parts is not None:
            nslab = parts.numel() // (2 * C)
            ws = torch.empty((3 * C,), dtype=torch.float32, device=dev)
            pdy, pdyx, o = parts[:nslab * C], parts[nslab * C:], 0
        else:
            nslab = N.query("kfb_bn_pool_num_slabs", n, H, W, C, *ctx.geo[6:10])
            ws = torch.empty((2 * nslab * C + 3 * C,), dtype=torch.float32, device=dev)
            pdy, pdyx, o = ws[:nslab * C], ws[nslab * C:2 * nslab * C], 2 * nslab * C
        gsink, bsink = _grad_sink(ctx.gamma), _grad_sink(ctx.beta)
        direct = bsink is not None and (ctx.gamma is None or gsink is not None) and \
            _conv.FUSE_BN
        if direct:
            dgp, dbp = N.ptr(gsink), bsink.data_ptr()
        else:
            dparams = torch.empty((2, C), dtype=torch.float32, device=dev)
            dgp, dbp = dparams[0].data_ptr(), dparams[1].data_ptr()
        dx = torch.empty_like(x)
        N.call("kfb_bn_relu_maxpool_bwd", N.dt(x), dz.data_ptr(), z.data_ptr(), idx.data_ptr(),
               x.data_ptr(), dx.data_ptr(), *ctx.geo, N.ptr(gamma), st[0].data_ptr(),
               st[1].data_ptr(), dgp, dbp, pdy.data_ptr(), pdyx.data_ptr(), nslab,
               ws[o:o + C].data_ptr(), ws[o + C:o + 2 * C].data_ptr(), ws[o + 2 * C:].data_ptr(),
               int(direct), int(parts is not None), N.stream(dev))
        nones = (None,) * 12
        if direct:
            _grad_ready(ctx.gamma)
            _grad_ready(ctx.beta)
            return (dx, None, None) + nones
        dgamma = dparams[0] if ctx.gamma is not None else None
        return (dx, dgamma, dparams[1]) + nones


def bn_relu_max_pool_fusable(x, stats, training) -> bool:
    return (training and stats is not None and _on_gpu(x) and x.shape[-1] % 8 == 0
            and _conv.FUSE_BN and hasattr(N.load(), "kfb_bn_relu_maxpool_fwd"))


def bn_relu_max_pool(x, gamma, beta, running_mean, running_var, decay, eps, stats,
                     kh, kw, sh, sw, mode="VALID"):
    """maxpool(relu(batch_norm_train(x))) - see _BNReluMaxPool; the caller
    checks bn_relu_max_pool_fusable first."""
    pads, OH, OW = pool_geometry(x.shape, kh, kw, sh, sw, mode)
    return _BNReluMaxPool.apply(x, gamma, beta, running_mean, running_var, decay, eps, stats,
                                kh, kw, sh, sw, pads, OH, OW)


def pool_takes_link(x, kh, kw, sh, sw, mode, kind):
    """True if max_pool / avg_pool of x runs the pool autograd Function
    (which follows the BNLink protocol) rather than a CPU or subsample path."""
    # (the 1x1 subsample's native window op follows the protocol too)
    return _on_gpu(x)


def max_pool(x, kh, kw, sh, sw, mode="VALID"):
    pads, OH, OW = pool_geometry(x.shape, kh, kw, sh, sw, mode)
    if not _on_gpu(x):
        return _pool_cpu(x, kh, kw, sh, sw, pads, "max")
    return _MaxPool.apply(x, kh, kw, sh, sw, pads, OH, OW)


N.register_optional("kfb_window", [N.I, N.P, N.P] + [N.I] * 11 + [N.P])


class _Window(torch.autograd.Function):
    """y[n, oh, ow] = x[n, oh*sh + oh0, ow*sw + ow0] (zero outside x), one
    native kernel each way (csrc/elementwise.hip window_k); its input
    gradient follows the BNLink protocol like a pool's."""

    @staticmethod
    def forward(ctx, x, sh, sw, oh0, ow0, OH, OW):
        x = x.contiguous()
        n, H, W, C = x.shape
        y = torch.empty((n, OH, OW, C), dtype=x.dtype, device=x.device)
        N.call("kfb_window", N.dt(x), x.data_ptr(), y.data_ptr(), n, H, W, C, OH, OW, sh, sw,
               oh0, ow0, 0, N.stream(x.device))
        ctx.geo = (n, H, W, C, OH, OW, sh, sw, oh0, ow0)
        ctx.link = getattr(x, "_kfb_bn_link", None)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, H, W, C, OH, OW, sh, sw, oh0, ow0 = ctx.geo
        dy = dy.contiguous()
        dx = torch.empty((n, H, W, C), dtype=dy.dtype, device=dy.device)
        N.call("kfb_window", N.dt(dy), dy.data_ptr(), dx.data_ptr(), n, H, W, C, OH, OW, sh, sw,
               oh0, ow0, 1, N.stream(dy.device))
        return _pool_link_grad(ctx.link, dx), None, None, None, None, None, None


def window(x, sh, sw, oh0, ow0, OH, OW):
    """Strided / shifted window of an NHWC tensor (see _Window)."""
    if not _on_gpu(x):
        n, H, W, C = x.shape
        xp = torch.nn.functional.pad(x, (0, 0, 0, max(0, (OW - 1) * sw + ow0 + 1 - W),
                                         0, max(0, (OH - 1) * sh + oh0 + 1 - H)))
        return xp[:, oh0:oh0 + (OH - 1) * sh + 1:sh, ow0:ow0 + (OW - 1) * sw + 1:sw, :] \
            .contiguous()
    return _Window.apply(x, sh, sw, oh0, ow0, OH, OW)


def avg_pool(x, kh, kw, sh, sw, mode="VALID"):
    pads, OH, OW = pool_geometry(x.shape, kh, kw, sh, sw, mode)
    if not _on_gpu(x):
        return _pool_cpu(x, kh, kw, sh, sw, pads, "avg")
    if kh == 1 and kw == 1 and pads == (0, 0, 0, 0):
        # 1x1 average pool == strided subsample (ResNet v1 shortcut)
        return window(x, sh, sw, 0, 0, OH, OW)
    return _AvgPool.apply(x, kh, kw, sh, sw, pads, OH, OW)


class _GlobalAvg(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        n, H, W, C = x.shape
        y = torch.empty((n, C), dtype=x.dtype, device=x.device)
        N.call("kfb_gap_fwd", N.dt(x), x.data_ptr(), y.data_ptr(), n, H * W, C,
               N.stream(x.device))
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        n, H, W, C = ctx.shape
        dx = torch.empty(ctx.shape, dtype=dy.dtype, device=dy.device)
        N.call("kfb_gap_bwd", N.dt(dy), dy.data_ptr(), dx.data_ptr(), n, H * W, C,
               N.stream(dy.device))
        return dx


def spatial_mean(x, keep_dims=False):
    if not _on_gpu(x):
        y = x.float().mean(dim=(1, 2), keepdim=keep_dims).to(x.dtype)
        return y
    y = _GlobalAvg.apply(x)
    return y.view(y.shape[0], 1, 1, y.shape[1]) if keep_dims else y


# ---------------------------------------------------------------------- affine
_GEMM_FWD, _GEMM_DGRAD, _GEMM_WGRAD = 0, 1, 2


def _at(t, elems):
    """A view of ``t``'s storage starting ``elems`` elements further on
    (the GEMM entry point only reads the base pointer)."""
    return t.as_strided((1,), (1,), t.storage_offset() + elems)


# off: affine weight gradients never split the batch reduction
_SPLIT_WGRAD = True


def _gemm(mode, p, ldp, q, ldq, rows, cols, red, out, ldc, bias=None, relu=False,
          accumulate=False):
    """csrc/gemm.hip, out [rows][cols]: mode 0 out = p . q (q [red][cols]),
    mode 1 out = p . q^T (q [cols][red]), mode 2 out (+)= p^T . q
    (p [red][rows], q [red][cols], fp32 out).  Operands of 2 GiB or more
    (the kernel's buffer-descriptor range) are cut into row / reduction
    chunks (DeepSpeech2's fp32 [T*B, 8H] gate tensors)."""
    esz = p.element_size()
    lim = (1 << 31) - (1 << 20)
    if mode == _GEMM_WGRAD and (red * ldp * esz >= lim or red * ldq * esz >= lim):
        step = max(1, lim // (max(ldp, ldq) * esz))
        for r0 in range(0, red, step):
            r1 = min(red, r0 + step)
            _gemm(mode, _at(p, r0 * ldp), ldp, _at(q, r0 * ldq), ldq, rows, cols, r1 - r0, out, ldc,
                  accumulate=accumulate or r0 > 0)
        return
    if mode != _GEMM_WGRAD and rows * ldp * esz >= lim:
        step = max(1, lim // (ldp * esz))
        for r0 in range(0, rows, step):
            r1 = min(rows, r0 + step)
            _gemm(mode, _at(p, r0 * ldp), ldp, q, ldq, r1 - r0, cols, red, _at(out, r0 * ldc), ldc,
                  bias=bias, relu=relu, accumulate=accumulate)
        return
    dev = p.device
    nsplit, slab = 1, None
    if mode != _GEMM_WGRAD or _SPLIT_WGRAD:
        nsplit = N.query("kfb_gemm_splits", N.dt(p), rows, cols, red)
        if nsplit > 1:
            slab = torch.empty((nsplit * rows * ((cols + 3) // 4 * 4),), dtype=torch.float32,
                               device=dev)
    N.call("kfb_gemm", N.dt(p), mode, p.data_ptr(), ldp, q.data_ptr(), ldq, rows, cols, red,
           out.data_ptr(), ldc, N.ptr(bias), int(relu), int(accumulate), N.ptr(slab),
           slab.numel() if slab is not None else 0, nsplit, N.stream(dev))


# off: affine weight gradients on the compute stream
_LINEAR_WGRAD_SIDE = True


class _Linear(torch.autograd.Function):
    """y = act(x @ W + b) with W the fp32 master [Cin, Cout] (TF layout) and
    W_lp its compute copy, on the MFMA GEMM (csrc/gemm.hip): the forward
    reads W as is (K-strided operand), the input gradient is dy . W^T
    (K-contiguous W), and the weight gradient x^T . dy is written in fp32
    straight into the flat gradient buffer; bias and ReLU ride in the
    forward's epilogue and one fused ReLU-backward + bias-column-sum pass
    (tcb/convnet_builder.py:311-345)."""

    @staticmethod
    def forward(ctx, x, w, b, w_lp, relu):
        x = x.contiguous()
        wl = (w_lp if w_lp is not None else w.to(x.dtype)).contiguous()
        M, K = x.shape
        Nout = wl.shape[1]
        y = torch.empty((M, Nout), dtype=x.dtype, device=x.device)
        _gemm(_GEMM_FWD, x, K, wl, Nout, M, Nout, K, y, Nout, bias=b, relu=relu)
        ctx.save_for_backward(x, wl, y if relu else None)
        ctx.relu, ctx.has_b = relu, b is not None
        ctx.w, ctx.b = w, b
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wl, y = ctx.saved_tensors
        dy = dy.contiguous()
        M, K = x.shape
        Nout = wl.shape[1]
        dev = dy.device
        db = None
        if ctx.relu or ctx.has_b:
            g = torch.empty_like(dy) if ctx.relu else dy
            pb = dbuf = None
            nslab = 1
            if ctx.has_b:
                nslab = N.query("kfb_colsum_num_slabs", M, Nout)
                pb = torch.empty((nslab * Nout,), dtype=torch.float32, device=dev)
                bsink = _grad_sink(ctx.b)
                dbuf = bsink if bsink is not None else torch.empty(
                    (Nout,), dtype=torch.float32, device=dev)
            N.call("kfb_act_bwd_bias", N.dt(dy), dy.data_ptr(), N.ptr(y), g.data_ptr(), M, Nout,
                   int(ctx.relu), N.ptr(pb), nslab, N.ptr(dbuf),
                   int(ctx.has_b and _grad_sink(ctx.b) is not None), N.stream(dev))
            if ctx.has_b:
                if _grad_sink(ctx.b) is not None:
                    _grad_ready(ctx.b)
                else:
                    db = dbuf
            dy = g
        dx = None
        if ctx.needs_input_grad[0]:
            # (the first affine of a net on raw images needs no input gradient)
            dx = torch.empty((M, K), dtype=dy.dtype, device=dev)
            _gemm(_GEMM_DGRAD, dy, Nout, wl, Nout, M, K, Nout, dx, K)
        wsink = _grad_sink(ctx.w)
        dw = None
        if wsink is not None:
            ch = _conv_hip()
            side = ch.wgrad_stream(dev) if _LINEAR_WGRAD_SIDE else None
            if side is not None:
                # like the conv weight gradients: off the dgrad chain, on the
                # side stream (the classifier's wgrad is a small latency-bound
                # GEMM at the head of the backward critical path)
                N.stream_wait(side.cuda_stream, N.stream(dev), device_only=True)
                ch._queue_join(dev)
                with torch.cuda.stream(side):
                    _gemm(_GEMM_WGRAD, x, K, dy, Nout, K, Nout, M, wsink, Nout, accumulate=True)
                    x.record_stream(side)
                    dy.record_stream(side)
                    _grad_ready(ctx.w)
                return dx, None, db, None, None
            _gemm(_GEMM_WGRAD, x, K, dy, Nout, K, Nout, M, wsink, Nout, accumulate=True)
            _grad_ready(ctx.w)
        else:
            dw = torch.empty((K, Nout), dtype=torch.float32, device=dev)
            _gemm(_GEMM_WGRAD, x, K, dy, Nout, K, Nout, M, dw, Nout)
        return dx, dw, db, None, None


def linear(x, w, b, w_lp=None, relu=False):
    if not _on_gpu(x):
        y = x.float() @ w
        if b is not None:
            y = y + b
        if relu:
            y = torch.relu(y)
        return y.to(x.dtype)
    return _Linear.apply(x, w, b, w_lp, relu)


# --------------------------------------------------------------------- dropout
class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, keep, seed, key):
        x = x.contiguous()
        y = torch.empty_like(x)
        N.call("kfb_dropout", N.dt(x), x.data_ptr(), y.data_ptr(), x.numel(), float(keep),
               N.dyn(key, int(seed) & 0xFFFFFFFF) if key else int(seed) & 0xFFFFFFFF,
               N.stream(x.device))
        ctx.keep, ctx.seed, ctx.key = keep, seed, key
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        seed = int(ctx.seed) & 0xFFFFFFFF
        N.call("kfb_dropout", N.dt(dy), dy.data_ptr(), dx.data_ptr(), dy.numel(),
               float(ctx.keep), N.dyn(ctx.key, seed) if ctx.key else seed, N.stream(dy.device))
        return dx, None, None, None


def dropout(x, keep_prob: float, training: bool, seed: int, key=None):
    """``key``: name of the seed as a per-step launch-tape argument."""
    if not training or keep_prob >= 1.0:
        return x
    if not _on_gpu(x):
        return F.dropout(x, p=1.0 - keep_prob, training=True)
    return _Dropout.apply(x, keep_prob, seed, key)


# ------------------------------------------------------------------- drop path
N.register_optional("kfb_drop_path", [N.I, N.P, N.P, N.L, N.L, N.c_float, N.c_uint32, N.P])


class _DropPath(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kp, seed, kp_key, seed_key):
        x = x.contiguous()
        y = torch.empty_like(x)
        ctx.args = (kp, seed, kp_key, seed_key, x.numel() // x.shape[0])
        _DropPath._call(x, y, *ctx.args)
        return y

    @staticmethod
    def _call(x, y, kp, seed, kp_key, seed_key, per):
        seed = int(seed) & 0xFFFFFFFF
        N.call("kfb_drop_path", N.dt(x), x.data_ptr(), y.data_ptr(), x.numel(), per,
               N.dyn(kp_key, float(kp)) if kp_key else float(kp),
               N.dyn(seed_key, seed) if seed_key else seed, N.stream(x.device))

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        _DropPath._call(dy, dx, *ctx.args)
        return dx, None, None, None, None


def drop_path(x, kp: float, seed: int, kp_key=None, seed_key=None):
    """Per-sample drop path: y = x * floor(kp + u_n) / kp.  On the GPU one
    native kernel whose keep probability and seed are per-step launch-tape
    arguments (``kp_key`` / ``seed_key``), so a taped step follows the
    step-dependent schedule; kp = 1 is the identity."""
    if not _on_gpu(x):
        g = torch.Generator().manual_seed(int(seed) & 0x7FFFFFFF)
        u = torch.rand((x.shape[0],) + (1,) * (x.dim() - 1), generator=g).to(x.device)
        return x * (torch.floor(kp + u) / kp).to(x.dtype)
    return _DropPath.apply(x, kp, seed, kp_key, seed_key)


# ------------------------------------------------------------------------- LRN
class _LRN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, depth_radius, bias, alpha, beta):
        x = x.contiguous()
        C = x.shape[-1]
        y = torch.empty_like(x)
        N.call("kfb_lrn_fwd", N.dt(x), x.data_ptr(), y.data_ptr(), x.numel() // C, C,
               int(depth_radius), float(bias), float(alpha), float(beta), N.stream(x.device))
        ctx.save_for_backward(x)
        ctx.args = (int(depth_radius), float(bias), float(alpha), float(beta))
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous()
        C = x.shape[-1]
        dx = torch.empty_like(x)
        r, bias, alpha, beta = ctx.args
        N.call("kfb_lrn_bwd", N.dt(x), x.data_ptr(), dy.data_ptr(), dx.data_ptr(),
               x.numel() // C, C, r, bias, alpha, beta, N.stream(x.device))
        return dx, None, None, None, None


def lrn(x, depth_radius, bias, alpha, beta):
    """tf.nn.lrn over the channel dim of NHWC x (sum over 2r+1 channels;
    tcb/convnet_builder.py:463-469).  GPU: csrc/lrn.hip."""
    if _on_gpu(x):
        return _LRN.apply(x, depth_radius, bias, alpha, beta)
    xf = x.float()
    sq = (xf * xf).permute(0, 3, 1, 2).unsqueeze(1)  # N,1,C,H,W
    k = 2 * depth_radius + 1
    s = F.avg_pool3d(F.pad(sq, (0, 0, 0, 0, depth_radius, depth_radius)), (k, 1, 1),
                     stride=1) * k
    s = s.squeeze(1).permute(0, 2, 3, 1)
    return (xf / (bias + alpha * s).pow(beta)).to(x.dtype)


# ------------------------------------------------------------------------ loss
class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        logits = logits.contiguous()
        labels = labels.to(torch.int32).contiguous()
        n, k = logits.shape
        loss = torch.empty((n,), dtype=torch.float32, device=logits.device)
        lse = torch.empty((n,), dtype=torch.float32, device=logits.device)
        N.call("kfb_xent_fwd", N.dt(logits), logits.data_ptr(), labels.data_ptr(), n, k,
               loss.data_ptr(), lse.data_ptr(), N.stream(logits.device))
        ctx.save_for_backward(logits, labels, lse)
        mean = torch.empty((), dtype=torch.float32, device=logits.device)
        N.call("kfb_mean_f32", loss.data_ptr(), n, mean.data_ptr(), N.stream(logits.device))
        return mean

    @staticmethod
    def backward(ctx, g):
        logits, labels, lse = ctx.saved_tensors
        n, k = logits.shape
        g = g.float().reshape(1).contiguous()
        dl = torch.empty_like(logits)
        N.call("kfb_xent_bwd", N.dt(logits), logits.data_ptr(), labels.data_ptr(),
               lse.data_ptr(), g.data_ptr(), 1.0 / n, n, k, dl.data_ptr(),
               N.stream(logits.device))
        return dl, None


def softmax_cross_entropy(logits, labels):
    """Mean sparse softmax cross-entropy (fp32 result)."""
    if not _on_gpu(logits):
        return F.cross_entropy(logits.float(), labels.long())
    return _SoftmaxXent.apply(logits, labels)


def ssd_loss_reference(logits, gt_loc, gt_label, num_matched, negs_per_pos=3):
    """Tensor form of the SSD300 loss (tcb/models/ssd_model.py loss_function:
    softmax cross-entropy with hard-negative mining + smooth-L1 box loss).

    logits [B, A, 4 + C]; gt_loc [B, A, 4]; gt_label [B, A] or [B, A, 1]
    (float class ids, truncated); num_matched [B].  Hard negatives are the
    k = min(negs_per_pos * floor(n_b), A) negatives with the largest
    cross-entropy, equal values taken in anchor order (stable sort) -- the
    exact selection rule of the fused kernel."""
    B, A, R = logits.shape
    C = R - 4
    lf = logits.float()
    lab = gt_label.reshape(B, A).float().long()
    pos = lab > 0
    ce = F.cross_entropy(lf[..., 4:].reshape(-1, C), lab.clamp(0, C - 1).reshape(-1),
                         reduction="none").reshape(B, A)
    nm = num_matched.float()
    k = torch.clamp(nm.long() * negs_per_pos, 0, A)
    key = torch.where(pos, torch.zeros_like(ce), ce.clamp(min=0))
    order = torch.sort(key, dim=1, descending=True, stable=True).indices
    rank = torch.empty_like(order)
    rank.scatter_(1, order, torch.arange(A, device=order.device).expand(B, A).contiguous())
    neg = (rank < k[:, None]) & ~pos
    cls = (ce * (pos | neg).float()).sum(1)
    sl1 = F.smooth_l1_loss(lf[..., :4], gt_loc.float(), reduction="none", beta=1.0).sum(2)
    loc = (sl1 * pos.float()).sum(1)
    return ((cls + loc) / nm).mean()


class _SSDLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, gt_loc, gt_label, num_matched, negs_per_pos):
        logits = logits.contiguous()
        B, A, R = logits.shape
        if A > 8960:
            raise N.NativeError("ssd_loss: %d anchors exceed the kernel's LDS rows" % A)
        gt_loc = gt_loc.float().contiguous()
        gt_label = gt_label.float().reshape(B, A).contiguous()
        num_matched = num_matched.float().reshape(B).contiguous()
        if gt_loc.shape != (B, A, 4):
            raise ValueError("ssd_loss: gt_loc %s != %s" % (tuple(gt_loc.shape), (B, A, 4)))
        work = torch.empty((B + 3 * B * A,), dtype=torch.float32, device=logits.device)
        out = torch.empty((1,), dtype=torch.float32, device=logits.device)
        N.call("kfb_ssd_loss_fwd", N.dt(logits), logits.data_ptr(), gt_loc.data_ptr(),
               gt_label.data_ptr(), num_matched.data_ptr(), B, A, R - 4, int(negs_per_pos),
               work.data_ptr(), out.data_ptr(), N.stream(logits.device))
        ctx.save_for_backward(logits, gt_loc, gt_label, num_matched, work)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        logits, gt_loc, gt_label, num_matched, work = ctx.saved_tensors
        B, A, R = logits.shape
        g = g.float().reshape(1).contiguous()
        dl = torch.empty_like(logits)
        N.call("kfb_ssd_loss_bwd", N.dt(logits), logits.data_ptr(), gt_loc.data_ptr(),
               gt_label.data_ptr(), num_matched.data_ptr(), work.data_ptr(), g.data_ptr(), B, A,
               R - 4, dl.data_ptr(), N.stream(logits.device))
        return dl, None, None, None, None


class _SSDHeads(torch.autograd.Function):
    """Anchor-major SSD logits [B, sum(nd*H*W), 4 + classes] from the NHWC
    loc / conf head outputs (kfb_ssd_heads: one launch per head, its
    backward the same walk gathering the head gradients)."""

    @staticmethod
    def forward(ctx, nds, ncls, *heads):
        k = len(heads) // 2
        locs, confs = heads[:k], heads[k:]
        B = locs[0].shape[0]
        rows = sum(nd * l.shape[1] * l.shape[2] for nd, l in zip(nds, locs))
        ld = 4 + ncls
        out = torch.empty((B, rows, ld), dtype=locs[0].dtype, device=locs[0].device)
        st = N.stream(out.device)
        row0 = 0
        geo = []
        for nd, l, c in zip(nds, locs, confs):
            A = l.shape[1] * l.shape[2]
            for t, col0, R in ((l, 0, 4), (c, 4, ncls)):
                t = t.contiguous()
                N.call("kfb_ssd_heads", N.dt(t), t.data_ptr(), out.data_ptr(), B, A, nd, R,
                       row0, col0, rows * ld, ld, 0, st)
            geo.append((tuple(l.shape), tuple(c.shape), A, nd, row0))
            row0 += nd * A
        ctx.geo, ctx.ncls, ctx.ld, ctx.rows = geo, ncls, ld, rows
        return out

    @staticmethod
    def backward(ctx, dout):
        dout = dout.contiguous()
        B = dout.shape[0]
        st = N.stream(dout.device)
        dl, dc = [], []
        for lshape, cshape, A, nd, row0 in ctx.geo:
            for shape, col0, R, lst in ((lshape, 0, 4, dl), (cshape, 4, ctx.ncls, dc)):
                g = torch.empty(shape, dtype=dout.dtype, device=dout.device)
                N.call("kfb_ssd_heads", N.dt(g), dout.data_ptr(), g.data_ptr(), B, A, nd, R,
                       row0, col0, ctx.rows * ctx.ld, ctx.ld, 1, st)
                lst.append(g)
        return (None, None) + tuple(dl) + tuple(dc)


def ssd_heads(locs, confs, nds, ncls):
    """[B, sum(nd*H*W), 4 + ncls] logits (anchor-major rows) from NHWC heads
    l [B, H, W, nd*4], c [B, H, W, nd*ncls]."""
    if not _on_gpu(locs[0]):
        B = locs[0].shape[0]
        ls = [l.reshape(B, l.shape[1], l.shape[2], nd, 4).permute(0, 3, 1, 2, 4).reshape(B, -1, 4)
              for nd, l in zip(nds, locs)]
        cs = [c.reshape(B, c.shape[1], c.shape[2], nd, ncls).permute(0, 3, 1, 2, 4)
              .reshape(B, -1, ncls) for nd, c in zip(nds, confs)]
        return torch.cat([torch.cat(ls, 1), torch.cat(cs, 1)], dim=2)
    return _SSDHeads.apply(tuple(nds), ncls, *locs, *confs)


def ssd_loss(logits, gt_loc, gt_label, num_matched, negs_per_pos=3):
    """SSD300 training loss (fp32 scalar); fused HIP kernels on the GPU
    (csrc/ssd_loss.hip), :func:`ssd_loss_reference` on the CPU."""
    if not _on_gpu(logits):
        return ssd_loss_reference(logits, gt_loc, gt_label, num_matched, negs_per_pos)
    return _SSDLoss.apply(logits, gt_loc, gt_label, num_matched, negs_per_pos)


def in_top_k(logits, labels):
    """(#top-1 correct, #top-5 correct) as fp32 device scalars."""
    if not _on_gpu(logits):
        lf = logits.float()
        t = lf.gather(1, labels.long().view(-1, 1))
        cnt = (lf > t).sum(1)
        fin = torch.isfinite(t.view(-1))
        return ((cnt < 1) & fin).float().sum(), ((cnt < 5) & fin).float().sum()
    logits = logits.contiguous()
    labels = labels.to(torch.int32).contiguous()
    n, k = logits.shape
    out = torch.empty((2, n), dtype=torch.float32, device=logits.device)
    N.call("kfb_in_top_k", N.dt(logits), logits.data_ptr(), labels.data_ptr(), n, k,
           out[0].data_ptr(), out[1].data_ptr(), N.stream(logits.device))
    s = out.sum(1)
    return s[0], s[1]


# ------------------------------------------------------------------- synthetic
def synthetic_images(shape, dtype, device, seed: int, mean=127.0, std=60.0):
    if torch.device(device).type != "cuda":
        g = torch.Generator().manual_seed(seed)
        x = torch.randn(shape, generator=g).clamp_(-2, 2) * std + mean
        return x.to(dtype)
    x = torch.empty(shape, dtype=dtype, device=device)
    N.call("kfb_synthetic_images", N.dt(x), x.data_ptr(), x.numel(), float(mean), float(std),
           N.dyn("input_seed", seed & 0xFFFFFFFF), N.stream(x.device))
    return x


def augment_u8(images, params, dtype):
    """Device half of the train preprocessing (csrc/augment.hip): uint8
    [N, H, W, 3] pixels + [N, 8] float32 parameters (flip, brightness,
    saturation, hue, contrast, order, distort) -> [N, H, W, 3] in [-1, 1],
    ``dtype``.  CPU tensors take the numpy reference."""
    if images.device.type != "cuda":
        from ..data.preprocessing import augment_reference
        out = augment_reference(images.numpy(), params.numpy())
        return torch.from_numpy(out).to(dtype)
    n, h, w, c = images.shape
    if c != 3 or params.shape != (n, 8) or images.dtype != torch.uint8:
        raise ValueError("augment_u8 takes uint8 [N,H,W,3] and float32 [N,8]")
    images = images.contiguous()
    params = params.to(torch.float32).contiguous()
    part = torch.empty((n * N.query("kfb_augment_blocks") * 3,), dtype=torch.float32,
                       device=images.device)
    out = torch.empty((n, h, w, 3), dtype=dtype, device=images.device)
    N.call("kfb_augment", N.dt(out), images.data_ptr(), params.data_ptr(), part.data_ptr(), n, h,
           w, out.data_ptr(), N.stream(images.device))
    return out


def synthetic_uniform(shape, dtype, device, seed: int, salt: int, lo=0.0, hi=1.0):
    """U[lo, hi) of ``shape`` made on the device (csrc/elementwise.hip): one
    launch, the per-step seed a launch-tape argument, ``salt`` a per-tensor
    constant.  CPU: torch's generator seeded with seed + salt."""
    if torch.device(device).type != "cuda":
        g = torch.Generator().manual_seed(seed + salt)
        return (torch.rand(shape, generator=g) * (hi - lo) + lo).to(dtype)
    x = torch.empty(shape, dtype=dtype, device=device)
    N.call("kfb_synthetic_uniform", N.dt(x), x.data_ptr(), x.numel(), float(lo),
           float(hi - lo), N.dyn("input_seed", seed & 0xFFFFFFFF), int(salt) & 0xFFFFFFFF,
           N.stream(x.device))
    return x


def synthetic_ints(n, maxval, device, seed: int, salt: int):
    """int32 uniform in [0, maxval) made on the device; the per-step seed is a
    launch-tape argument, ``salt`` a per-tensor constant."""
    if torch.device(device).type != "cuda":
        g = torch.Generator().manual_seed(seed + salt)
        return torch.randint(0, maxval, (n,), generator=g, dtype=torch.int32)
    if not 0 < maxval <= 1 << 24:
        raise ValueError("synthetic_ints: maxval must be in (0, 2^24]")
    y = torch.empty((n,), dtype=torch.int32, device=device)
    N.call("kfb_synthetic_ints", y.data_ptr(), n, int(maxval),
           N.dyn("input_seed", seed & 0xFFFFFFFF), int(salt) & 0xFFFFFFFF, N.stream(device))
    return y


def synthetic_labels(n, nclass, device, seed: int):
    # Reference: uniform in [0, nclass-1) (tcb/models/model.py:232-236).
    maxval = max(nclass - 1, 1)
    if torch.device(device).type != "cuda":
        g = torch.Generator().manual_seed(seed + 1)
        return torch.randint(0, maxval, (n,), generator=g, dtype=torch.int32)
    y = torch.empty((n,), dtype=torch.int32, device=device)
    N.call("kfb_synthetic_labels", y.data_ptr(), n, maxval,
           N.dyn("input_seed_labels", (seed + 1) & 0xFFFFFFFF), N.stream(device))
    return y


class _Concat(torch.autograd.Function):
    """Channel (last-dim) concat on the GPU (csrc/gather.hip): one launch
    for all inputs; the backward splits the gradient in one launch."""

    @staticmethod
    def forward(ctx, *xs):
        import ctypes
        xs = [x.contiguous() for x in xs]
        widths = [x.shape[-1] for x in xs]
        offs = [0]
        for w in widths:
            offs.append(offs[-1] + w)
        rows = xs[0].numel() // widths[0]
        out = torch.empty(xs[0].shape[:-1] + (offs[-1],), dtype=xs[0].dtype, device=xs[0].device)
        ctx.meta = (widths, offs, rows)
        _concat_call(out, xs, offs, rows, split=False)
        return out

    @staticmethod
    def backward(ctx, dy):
        widths, offs, rows = ctx.meta
        dy = dy.contiguous()
        dxs = [torch.empty(dy.shape[:-1] + (w,), dtype=dy.dtype, device=dy.device)
               for w in widths]
        _concat_call(dy, dxs, offs, rows, split=True)
        return tuple(dxs)


def _concat_call(out, parts, offs, rows, split):
    import ctypes
    k = len(parts)
    esz = out.element_size()
    epv = 16 // esz
    vec = all(w % epv == 0 for w in (offs[j + 1] - offs[j] for j in range(k))) and \
        all(t.data_ptr() % 16 == 0 for t in list(parts) + [out] if t is not None)
    ptrs = (ctypes.c_void_p * k)(*[t.data_ptr() if t is not None else None for t in parts])
    offa = (ctypes.c_int * (k + 1))(*offs)
    N.call("kfb_concat", N.dt(out), out.data_ptr(), ptrs, offa, k, rows, offs[-1], int(vec),
           int(split), N.stream(out.device))


_CAT_MAX = 16


class _ChannelPad(torch.autograd.Function):
    """Zero channels before / after the last dim (one concat launch with
    null parts; the backward is the split of the middle block)."""

    @staticmethod
    def forward(ctx, x, before, after):
        x = x.contiguous()
        C = x.shape[-1]
        offs = [0, before, before + C, before + C + after]
        rows = x.numel() // C
        out = torch.empty(x.shape[:-1] + (offs[-1],), dtype=x.dtype, device=x.device)
        _concat_call(out, [None, x, None], offs, rows, split=False)
        ctx.meta = (C, offs, rows)
        return out

    @staticmethod
    def backward(ctx, dy):
        C, offs, rows = ctx.meta
        dy = dy.contiguous()
        dx = torch.empty(dy.shape[:-1] + (C,), dtype=dy.dtype, device=dy.device)
        _concat_call(dy, [None, dx, None], offs, rows, split=True)
        return dx, None, None


def channel_pad(x, before: int, after: int):
    """[..., C] -> [..., before + C + after] with zero channels around x."""
    if not _on_gpu(x):
        return F.pad(x, (before, after)).contiguous()
    return _ChannelPad.apply(x, before, after)


def concat_channels(xs: Sequence[torch.Tensor]):
    xs = list(xs)
    if len(xs) == 1:
        return xs[0]
    if not xs[0].is_cuda:
        return torch.cat(xs, dim=-1)
    if any(x.shape[:-1] != xs[0].shape[:-1] for x in xs):
        raise N.NativeError("concat inputs differ outside the channel dim: %s"
                            % [tuple(x.shape) for x in xs])
    dt = xs[0].dtype
    for x in xs[1:]:
        dt = torch.promote_types(dt, x.dtype)
    xs = [x if x.dtype == dt else x.to(dt) for x in xs]
    if len(xs) > _CAT_MAX:
        # the kernel takes up to _CAT_MAX inputs per launch: concat groups,
        # then the groups (one extra pass over the output's bytes)
        xs = [concat_channels(xs[i:i + _CAT_MAX]) for i in range(0, len(xs), _CAT_MAX)]
        return concat_channels(xs)
    return _Concat.apply(*xs)


# ------------------------------------------------------------------ embedding
class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, table):
        idx = idx.to(torch.int32).contiguous()
        rows, dim = table.shape
        out = torch.empty((idx.numel(), dim), dtype=table.dtype, device=table.device)
        N.call("kfb_embedding_fwd", N.dt(table), table.data_ptr(), rows, idx.data_ptr(),
               out.data_ptr(), idx.numel(), dim, N.stream(table.device))
        ctx.save_for_backward(idx)
        ctx.table, ctx.shape = table, tuple(table.shape)
        return out.view(tuple(idx.shape) + (dim,))

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        rows, dim = ctx.shape
        dy = dy.contiguous()
        sink = _grad_sink(ctx.table)
        grad = sink if sink is not None else torch.zeros(ctx.shape, dtype=torch.float32,
                                                         device=dy.device)
        N.call("kfb_embedding_bwd", N.dt(dy), dy.data_ptr(), idx.data_ptr(), grad.data_ptr(),
               rows, idx.numel(), dim, N.stream(dy.device))
        if sink is not None:
            _grad_ready(ctx.table)
            return None, None
        return None, grad


def embedding(idx, table):
    """tf.nn.embedding_lookup: rows of ``table`` [rows, dim] at ``idx``.  GPU:
    csrc/gather.hip (gradient scatter-added into the flat-gradient view)."""
    if table.is_cuda:
        return _Embedding.apply(idx, table)
    return F.embedding(idx.long(), table)
