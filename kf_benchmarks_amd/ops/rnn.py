"""Recurrent layers and CTC loss for DeepSpeech2 on our HIP kernels
(csrc/rnn.hip, csrc/ctc.hip).

Reference: tcb/models/experimental/deepspeech.py:121-125 (cells), :231-270
(bidirectional dynamic_rnn), :360-395 (ctc_loss).  Everything is time-major
([T, B, ...]): the whole recurrent stack, its batch norms and the logits
layer run on [T*B, features] rows, which is the order both the per-step
kernels and the CTC recursion walk.

  * ``rnn_layer`` - one (bi)directional LSTM / tanh-RNN layer: the input
    projection of all steps as one affine GEMM (ops.nn.linear), then the
    recurrence (one fused MFMA + cell kernel per step, both directions per
    launch); backward mirrors it and ends with one dWh GEMM per direction.
  * ``ctc_loss`` - per-sequence CTC loss (blank = last class) with the
    gradient computed in the same kernel pass, as TF's op does.

On CPU tensors the same math runs as plain PyTorch autograd (the numerics
oracle of the GPU tests).
"""

from __future__ import annotations

import torch

from . import _native as N
from . import nn as F_ops

LSTM, TANH, GRU = 0, 1, 2
_KIND = {"lstm": LSTM, "rnn": TANH, "gru": GRU}
GATES = {LSTM: 4, TANH: 1, GRU: 3}


# ------------------------------------------------------------------ permute
class _Permute01(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        A, Bd = x.shape[0], x.shape[1]
        R = x[0, 0].numel()
        x = x.contiguous()
        y = torch.empty((Bd, A) + tuple(x.shape[2:]), dtype=x.dtype, device=x.device)
        N.call("kfb_permute01", N.dt(x), x.data_ptr(), y.data_ptr(), A, Bd, R, N.stream(x.device))
        return y

    @staticmethod
    def backward(ctx, dy):
        return _Permute01.apply(dy)


def permute01(x):
    """Swap the two leading dims (materialized): [A, B, ...] -> [B, A, ...]."""
    if not x.is_cuda:
        return x.transpose(0, 1).contiguous()
    return _Permute01.apply(x)


# --------------------------------------------------------------- recurrence
def recurrence_reference(gx, wh, kind, dirs, H):
    """Plain-PyTorch fp32 recurrence (the GPU kernels' numerics oracle).
    gx [T, B, dirs*G*H], wh [dirs, H, G*H] -> out [T, B, dirs*H]."""
    T, B = gx.shape[0], gx.shape[1]
    G = GATES[kind]
    gx = gx.float()
    outs = []
    for d in range(dirs):
        h = gx.new_zeros((B, H))
        c = gx.new_zeros((B, H))
        seq = [None] * T
        order = range(T - 1, -1, -1) if d else range(T)
        for t in order:
            gxt = gx[t, :, d * G * H:(d + 1) * G * H]
            if kind == GRU:  # TF GRUCell: the candidate sees r * h
                whd = wh[d].float()
                r, u = torch.sigmoid(gxt[:, :2 * H] + h @ whd[:, :2 * H]).split(H, dim=1)
                c = torch.tanh(gxt[:, 2 * H:] + (r * h) @ whd[:, 2 * H:])
                h = u * h + (1 - u) * c
                seq[t] = h
                continue
            pre = gxt + h @ wh[d].float()
            if kind == LSTM:
                i, j, f, o = pre.split(H, dim=1)
                c = c * torch.sigmoid(f + 1.0) + torch.sigmoid(i) * torch.tanh(j)
                h = torch.tanh(c) * torch.sigmoid(o)
            else:
                h = torch.tanh(pre)
            seq[t] = h
        outs.append(torch.stack(seq, 0))
    return torch.cat(outs, dim=2)


class _Recurrence(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gx, wh, kind, dirs, H):
        T, B = gx.shape[0], gx.shape[1]
        G = GATES[kind]
        dev, dt = gx.device, gx.dtype
        gx = gx.contiguous()
        whT = torch.empty((dirs, G * H, H), dtype=dt, device=dev)
        N.call("kfb_transpose_cast", N.dt(gx), wh.data_ptr(), whT.data_ptr(), dirs, H, G * H,
               N.stream(dev))
        out = torch.empty((T, B, dirs * H), dtype=dt, device=dev)
        hp = torch.empty((dirs, T, B, H), dtype=dt, device=dev)
        act = torch.empty((dirs, T, B, G * H), dtype=torch.float32, device=dev)
        cell = (torch.empty((dirs, T, B, H), dtype=torch.float32, device=dev)
                if kind == LSTM else None)
        rh = torch.empty((dirs, T, B, H), dtype=dt, device=dev) if kind == GRU else None
        N.call("kfb_rnn_fwd", N.dt(gx), kind, gx.data_ptr(), whT.data_ptr(), out.data_ptr(),
               hp.data_ptr(), act.data_ptr(), N.ptr(cell), N.ptr(rh), T, B, H, dirs,
               N.stream(dev))
        ctx.save_for_backward(hp, act, cell, rh)
        ctx.wh, ctx.kind, ctx.dirs, ctx.H = wh, kind, dirs, H
        return out

    @staticmethod
    def backward(ctx, dout):
        hp, act, cell, rh = ctx.saved_tensors
        wh, kind, dirs, H = ctx.wh, ctx.kind, ctx.dirs, ctx.H
        G = GATES[kind]
        T, B = hp.shape[1], hp.shape[2]
        dev, dt = hp.device, hp.dtype
        dout = dout.contiguous()
        if dt == torch.float32:
            wl = wh.contiguous()
        else:
            wl = torch.empty(wh.shape, dtype=dt, device=dev)
            N.call("kfb_cast_f32", wh.data_ptr(), wl.data_ptr(), N.dt(wl), wh.numel(),
                   N.stream(dev))
        dgx = torch.empty((T, B, dirs * G * H), dtype=dt, device=dev)
        ws = torch.empty((3, 2, dirs, B, H), dtype=torch.float32, device=dev)
        N.call("kfb_rnn_bwd", N.dt(dout), kind, dout.data_ptr(), wl.data_ptr(), act.data_ptr(),
               N.ptr(cell), hp.data_ptr(), dgx.data_ptr(), ws[0].data_ptr(), ws[1].data_ptr(),
               ws[2].data_ptr(), T, B, H, dirs, N.stream(dev))
        # dWh[d] = sum_{t,b} hp[d,t,b,:]^T dG[t,b,d,:]   (one GEMM per direction;
        # GRU: the candidate block's operand is r*h instead of h)
        sink = F_ops._grad_sink(wh)
        dw = None
        target = sink.view(dirs, H, G * H) if sink is not None else torch.empty(
            (dirs, H, G * H), dtype=torch.float32, device=dev)
        ldg = dirs * G * H
        acc = sink is not None
        for d in range(dirs):
            q = dgx.view(T * B, ldg)[:, d * G * H:]
            if kind == GRU:
                F_ops._gemm(F_ops._GEMM_WGRAD, hp[d], H, q, ldg, H, 2 * H, T * B, target[d],
                            G * H, accumulate=acc)
                F_ops._gemm(F_ops._GEMM_WGRAD, rh[d], H, F_ops._at(q, 2 * H), ldg, H, H, T * B,
                            F_ops._at(target[d], 2 * H), G * H, accumulate=acc)
            else:
                F_ops._gemm(F_ops._GEMM_WGRAD, hp[d], H, q, ldg, H, G * H, T * B, target[d],
                            G * H, accumulate=acc)
        if sink is not None:
            F_ops._grad_ready(wh)
        else:
            dw = target
        return dgx, dw, None, None, None


def recurrence(gx, wh, kind, dirs, H):
    if not gx.is_cuda:
        return recurrence_reference(gx, wh, kind, dirs, H).to(gx.dtype)
    if H % 16:
        raise N.NativeError("rnn kernels need hidden size % 16 == 0 (got %d)" % H)
    return _Recurrence.apply(gx, wh, kind, dirs, H)


def rnn_layer(x, wx, bx, wh, kind, dirs, H, wx_lp=None):
    """x [T, B, din] -> [T, B, dirs*H].  wx [din, dirs*G*H] (TF layout),
    bx [dirs*G*H], wh [dirs, H, G*H]."""
    T, B, din = x.shape
    gx = F_ops.linear(x.reshape(T * B, din), wx, bx, w_lp=wx_lp)
    return recurrence(gx.view(T, B, -1), wh, kind, dirs, H)


# ---------------------------------------------------------------------- CTC
def ctc_loss_reference(logits, labels, ilen, llen):
    """Per-sequence CTC loss (blank = last class) in plain PyTorch on
    log_softmax(logits); logits [B, T, C] (any strides)."""
    lp = torch.log_softmax(logits.float(), dim=-1).transpose(0, 1)
    blank = logits.shape[-1] - 1
    return torch.nn.functional.ctc_loss(lp, labels.long(), ilen.long(), llen.long(), blank=blank,
                                        reduction="none", zero_infinity=True)


class _CTC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ilen, llen):
        B, T, C = logits.shape
        dev = logits.device
        Lmax = labels.shape[1]
        smax = 2 * Lmax + 1
        if smax > N.query("kfb_ctc_max_states"):
            raise N.NativeError("CTC label length %d exceeds the kernel's state buffer" % Lmax)
        sb, st, sc = logits.stride()
        if sc != 1:
            logits = logits.contiguous()
            sb, st, sc = logits.stride()
        labels = labels.to(torch.int32).contiguous()
        ilen = ilen.reshape(-1).to(torch.int32).contiguous()
        llen = llen.reshape(-1).to(torch.int32).contiguous()
        lp = torch.empty((T * B * C,), dtype=torch.float32, device=dev)
        alpha = torch.empty((B * T * smax,), dtype=torch.float32, device=dev)
        loss = torch.empty((B,), dtype=torch.float32, device=dev)
        grad = torch.empty_strided(logits.shape, logits.stride(), dtype=torch.float32,
                                   device=dev)
        N.call("kfb_ctc_loss", N.dt(logits), logits.data_ptr(), st, sb, labels.data_ptr(),
               ilen.data_ptr(), llen.data_ptr(), T, B, C, Lmax, lp.data_ptr(), alpha.data_ptr(),
               smax, loss.data_ptr(), grad.data_ptr(), N.stream(dev))
        ctx.save_for_backward(grad)
        ctx.dtype = logits.dtype
        return loss

    @staticmethod
    def backward(ctx, gloss):
        (grad,) = ctx.saved_tensors
        B, T, C = grad.shape
        sb, st, _ = grad.stride()
        gloss = gloss.float().contiguous()
        dz = torch.empty_strided(grad.shape, grad.stride(), dtype=ctx.dtype, device=grad.device)
        N.call("kfb_ctc_grad_scale", N.dt(dz), grad.data_ptr(), gloss.data_ptr(), dz.data_ptr(),
               st, sb, T, B, C, N.stream(grad.device))
        return dz, None, None, None


N.register_optional("kfb_ctc_grad_scale_mean", [N.I, N.P, N.P, N.P, N.L, N.L, N.I, N.I, N.I,
                                                N.F, N.P])
N.register_optional("kfb_ctc_scale_lengths", [N.P, N.P, N.I, N.I, N.I, N.P])


class _CTCMean(torch.autograd.Function):
    """mean_b CTC(logits_b) with the input lengths scaled to the logits' time
    axis (ilen * len_num // len_den, the reference's length arithmetic,
    tcb/models/experimental/deepspeech.py:407-414) - every piece a native
    call: the length scaling, the loss + gradient kernel, the batch mean and
    the mean's backward, so the step that holds it can be taped."""

    @staticmethod
    def forward(ctx, logits, labels, ilen, llen, len_num, len_den):
        B, T, C = logits.shape
        dev = logits.device
        Lmax = labels.shape[1]
        smax = 2 * Lmax + 1
        if smax > N.query("kfb_ctc_max_states"):
            raise N.NativeError("CTC label length %d exceeds the kernel's state buffer" % Lmax)
        if logits.stride(2) != 1:
            logits = logits.contiguous()
        sb, st, _ = logits.stride()
        for t in (labels, ilen, llen):
            if t.dtype != torch.int32 or not t.is_contiguous():
                raise N.NativeError("ctc_loss_mean takes contiguous int32 labels / lengths")
        sl = torch.empty((B,), dtype=torch.int32, device=dev)
        N.call("kfb_ctc_scale_lengths", ilen.data_ptr(), sl.data_ptr(), B, int(len_num),
               int(len_den), N.stream(dev))
        lp = torch.empty((T * B * C,), dtype=torch.float32, device=dev)
        alpha = torch.empty((B * T * smax,), dtype=torch.float32, device=dev)
        loss = torch.empty((B,), dtype=torch.float32, device=dev)
        grad = torch.empty_strided(logits.shape, logits.stride(), dtype=torch.float32,
                                   device=dev)
        N.call("kfb_ctc_loss", N.dt(logits), logits.data_ptr(), st, sb, labels.data_ptr(),
               sl.data_ptr(), llen.data_ptr(), T, B, C, Lmax, lp.data_ptr(), alpha.data_ptr(),
               smax, loss.data_ptr(), grad.data_ptr(), N.stream(dev))
        mean = torch.empty((), dtype=torch.float32, device=dev)
        N.call("kfb_mean_f32", loss.data_ptr(), B, mean.data_ptr(), N.stream(dev))
        ctx.save_for_backward(grad)
        ctx.dtype = logits.dtype
        return mean

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        B, T, C = grad.shape
        sb, st, _ = grad.stride()
        if g.dtype != torch.float32 or not g.is_contiguous():
            raise N.NativeError("ctc_loss_mean: fp32 loss gradient expected")
        dz = torch.empty_strided(grad.shape, grad.stride(), dtype=ctx.dtype, device=grad.device)
        N.call("kfb_ctc_grad_scale_mean", N.dt(dz), grad.data_ptr(), g.data_ptr(),
               dz.data_ptr(), st, sb, T, B, C, 1.0 / B, N.stream(grad.device))
        return dz, None, None, None, None, None


def ctc_loss_mean(logits, labels, ilen, llen, len_num=1, len_den=1):
    """Batch-mean CTC loss (fp32 scalar) of logits [B, T, C] (blank = C-1)
    with input lengths ilen * len_num // len_den; infeasible sequences give
    0.  On the GPU every op is native (recordable in a launch tape)."""
    if not logits.is_cuda:
        ilen_s = (ilen.reshape(-1).long() * len_num) // len_den
        return ctc_loss_reference(logits, labels, ilen_s, llen.reshape(-1)).mean()
    return _CTCMean.apply(logits, labels.contiguous(), ilen.reshape(-1).contiguous(),
                          llen.reshape(-1).contiguous(), len_num, len_den)


def ctc_loss(logits, labels, ilen, llen):
    """Per-sequence CTC losses [B] of logits [B, T, C] (blank = C-1);
    infeasible sequences (label longer than the input allows) give 0."""
    if not logits.is_cuda:
        return ctc_loss_reference(logits, labels, ilen, llen)
    return _CTC.apply(logits, labels, ilen, llen)
