"""Flat parameter storage, fused optimizers and learning-rate schedules.

* :class:`FlatParams` re-homes every trainable variable of a Network into ONE
  contiguous fp32 buffer (ordered by reverse creation order, i.e. the order
  gradients become ready in backward), with a matching flat gradient buffer
  and an optional bf16/fp16 shadow of the weights for the kernels.  Gradient
  buckets for all-reduce are then plain contiguous slices - no pack/unpack.
* :class:`FusedOptimizer` implements tf.train GradientDescent / Momentum
  (Nesterov, as tcb/benchmark_cnn.py:1174-1176) / RMSProp / Adam as one
  launch over the flat buffer (csrc/optim.hip), folding in loss-scale
  unscale, weight-decay gradient and clip-by-value.
* ``get_learning_rate`` / ``get_piecewise_learning_rate``: the schedules of
  tcb/benchmark_cnn.py:1067-1169, evaluated on the host per step.
"""

from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch

from .ops import _native as N

ALIGN = 64  # elements; keeps every view 256-byte aligned


class FlatParams:
    def __init__(self, net, lp_dtype: Optional[torch.dtype] = None, reverse: bool = True):
        self.net = net
        named = net.trainable_variables()
        if reverse:
            named = list(reversed(named))
        self.names: List[str] = [n for n, _ in named]
        self.params: List[torch.nn.Parameter] = [p for _, p in named]
        dev = self.params[0].device
        self.device = dev
        offs, total = [], 0
        for p in self.params:
            offs.append(total)
            total += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.offsets = offs
        self.numel = total
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev)
        for p, o in zip(self.params, offs):
            n = p.numel()
            self.flat[o:o + n].copy_(p.detach().reshape(-1))
            p.data = self.flat[o:o + n].view(p.shape)
            p.grad = self.grad[o:o + n].view(p.shape)
            # GPU kernels (conv wgrad, BN dgamma/dbeta) accumulate straight into
            # this view and skip autograd's AccumulateGrad (see ops/conv_hip.py).
            p._kfb_grad_sink = p.grad
        self.lp_dtype = lp_dtype if lp_dtype not in (None, torch.float32) else None
        self.lp = None
        if self.lp_dtype is not None:
            self.lp = self.flat.to(self.lp_dtype)
            self._attach_lp_views()
        # --staged_vars: the optimizer updates ``master``; the layers read
        # ``flat`` (and its low-precision shadow), which is refreshed from the
        # master just BEFORE each update, so step t's forward/backward reads
        # the variables as they were one update earlier (the StagingArea
        # reads of tcb/variable_mgr_util.py:236-393, VariableMgrLocalFetch-
        # FromStagedPS tcb/variable_mgr.py:246-274)
        self.master: Optional[torch.Tensor] = None

    def _attach_lp_views(self):
        index = {id(p): (o, p) for p, o in zip(self.params, self.offsets)}
        # every parameter knows its compute copy (module models pass it to
        # the ops instead of casting the fp32 master every step)
        for p, o in zip(self.params, self.offsets):
            p._kfb_lp = self.lp[o:o + p.numel()].view(p.shape)
        for layer in self.net.ordered_layers():
            for attr, lp_attr in (("weight", "weight_lp"), ("weights", "weights_lp")):
                p = getattr(layer, attr, None)
                if p is not None and id(p) in index:
                    o, _ = index[id(p)]
                    setattr(layer, lp_attr, self.lp[o:o + p.numel()].view(p.shape))

    def enable_staging(self):
        self.master = self.flat.clone()

    @property
    def update_target(self) -> torch.Tensor:
        """The fp32 buffer the optimizer updates."""
        return self.master if self.master is not None else self.flat

    def stage_reads(self):
        """Staged mode: publish the current master as the values the next
        step reads (called right before the update)."""
        self.flat.copy_(self.master)
        if self.lp is not None:
            self.lp.copy_(self.master)

    def refresh_lp(self):
        """Re-derive the low-precision shadow from the fp32 master (after a
        checkpoint restore or a model broadcast)."""
        if self.master is not None:
            self.master.copy_(self.flat)
        if self.lp is not None:
            self.lp.copy_(self.flat)
        self.after_update()

    def real_values(self):
        """Context manager: the layer-visible buffer holds the real (master)
        variables inside (checkpoint save of a staged run)."""
        import contextlib

        @contextlib.contextmanager
        def swap():
            if self.master is None:
                yield
                return
            keep = self.flat.clone()
            self.flat.copy_(self.master)
            try:
                yield
            finally:
                self.flat.copy_(keep)
        return swap()

    def add_update_hook(self, fn):
        """fn() runs after every write of the weights (optimizer step, restore)."""
        self._hooks = getattr(self, "_hooks", [])
        self._hooks.append(fn)

    def after_update(self):
        for fn in getattr(self, "_hooks", []):
            fn()

    def zero_grad(self):
        if self.grad.is_cuda:
            N.zero_(self.grad)  # a native call: part of a recorded launch tape
        else:
            self.grad.zero_()

    def segments(self):
        """[(name, param, offset, numel)] in flat order."""
        return [(n, p, o, p.numel()) for n, p, o in zip(self.names, self.params, self.offsets)]


_KINDS = {"sgd": 0, "momentum": 1, "rmsprop": 2, "adam": 3}


class FusedOptimizer:
    def __init__(self, flat: FlatParams, kind: str, momentum=0.9, rmsprop_decay=0.9,
                 rmsprop_momentum=0.9, rmsprop_epsilon=1.0, adam_beta1=0.9, adam_beta2=0.999,
                 adam_epsilon=1e-8, nesterov=True):
        if kind not in _KINDS:
            raise ValueError('Optimizer "%s" was not recognized' % kind)
        self.flat = flat
        self.kind = kind
        self.momentum = momentum
        self.rmsprop = (rmsprop_decay, rmsprop_momentum, rmsprop_epsilon)
        self.adam = (adam_beta1, adam_beta2, adam_epsilon)
        self.nesterov = nesterov
        self.t = 0
        # uint8 per flat element: weight decay applies only where it is
        # nonzero (a model's L2 subset, e.g. SSD without batch-norm variables)
        self.decay_mask = None
        dev, n = flat.device, flat.numel
        self.s1 = torch.zeros(n, dtype=torch.float32, device=dev) if kind != "sgd" else None
        self.s2 = None
        if kind == "rmsprop":
            # TF RMSProp initializes the mean-square slot to ones.
            self.s2 = torch.ones(n, dtype=torch.float32, device=dev)
        elif kind == "adam":
            self.s2 = torch.zeros(n, dtype=torch.float32, device=dev)

    def slot_tensors(self):
        out = {}
        if self.s1 is not None:
            out["s1"] = self.s1
        if self.s2 is not None:
            out["s2"] = self.s2
        return out

    def step(self, lr: float, grad_scale: float = 1.0, weight_decay: float = 0.0,
             clip: Optional[float] = None, grad: Optional[torch.Tensor] = None,
             mix=None, wout: Optional[torch.Tensor] = None, lo: int = 0,
             hi: Optional[int] = None, advance: bool = True):
        """One update of every variable. ``grad`` overrides the flat gradient
        buffer (e.g. an all-reduced copy).  ``mix = (src, a, b, ok)`` first
        sets w <- a*w + b*src (model averaging; skipped when the device flag
        ``ok`` (nullable) is 0); ``wout`` receives a copy of the updated
        weights.  Both ride the same single pass over the model.
        ``lo`` / ``hi``: only flat elements [lo, hi) (GPU); ``advance=False``:
        an early part of this step's update (the step counter and the
        after-update hooks wait for the call that finishes the step)."""
        if lo or hi is not None:
            if self.flat.device.type != "cuda" or mix is not None or wout is not None \
                    or grad is not None or self.flat.master is not None:
                raise ValueError("ranged updates: plain GPU updates only")
        if not advance:
            t_saved = self.t
            try:
                self.t += 1
                return self._step(lr, grad_scale, weight_decay, clip, grad, mix, wout, lo, hi,
                                  False)
            finally:
                self.t = t_saved
        self.t += 1
        return self._step(lr, grad_scale, weight_decay, clip, grad, mix, wout, lo, hi, True)

    def _step(self, lr, grad_scale, weight_decay, clip, grad, mix, wout, lo, hi, finish):
        f = self.flat
        g = f.grad if grad is None else grad
        b1, b2, eps, lr_t, mom = 0.0, 0.0, 0.0, 0.0, self.momentum
        if self.kind == "rmsprop":
            b1, mom, eps = self.rmsprop
        elif self.kind == "adam":
            b1, b2, eps = self.adam
            lr_t = lr * math.sqrt(1 - b2 ** self.t) / (1 - b1 ** self.t)
        clipv = float(clip) if clip else 0.0
        staged = f.master is not None
        if staged:
            f.stage_reads()
        w = f.update_target
        lp = None if staged else f.lp
        msrc, ma, mb, mok = mix if mix is not None else (None, 1.0, 0.0, None)
        for t in (msrc, wout):
            if t is not None and (t.numel() != f.numel or t.dtype != torch.float32
                                  or not t.is_contiguous()):
                raise ValueError("mix / wout must be contiguous fp32 of the flat size")
        if f.device.type == "cuda":
            hi_ = f.numel if hi is None else hi

            def at(t):  # pointer to element lo of a flat-sized tensor (or None)
                return None if t is None else t.data_ptr() + lo * t.element_size()
            if hi_ > lo:
                N.call("kfb_opt_step", _KINDS[self.kind], at(w), at(g),
                       at(self.s1), at(self.s2), at(lp),
                       N.dt(lp) if lp is not None else 0, at(self.decay_mask), hi_ - lo, N.dyn("lr", float(lr)),
                       float(grad_scale), float(weight_decay), clipv, float(mom), float(b1),
                       float(b2), float(eps), N.dyn("lr_t", float(lr_t)), int(self.nesterov),
                       N.ptr(msrc),
                       float(ma), float(mb), N.ptr(mok),
                       # (launch tape: the publish slot may change per step)
                       N.dyn("wout", wout.data_ptr()) if wout is not None else None,
                       N.stream(f.device))
            if finish:
                f.after_update()
            return
        w_pre = None
        if msrc is not None and (mok is None or int(mok.reshape(-1)[0]) != 0):
            with torch.no_grad():
                if weight_decay:
                    # (the L2 gradient is of the forward's weights, pre-average)
                    w_pre = w.clone()
                w.mul_(ma).add_(msrc, alpha=mb)
        self._step_torch(g, lr, grad_scale, weight_decay, clipv, mom, b1, b2, eps, lr_t, w_pre)
        if wout is not None:
            wout.copy_(w)
        f.after_update()

    def tape_values(self, lr: float):
        """Per-step arguments of a replayed step's update (launch tape): the
        step counter advances as step() advances it."""
        self.t += 1
        lr_t = 0.0
        if self.kind == "adam":
            b1, b2, _ = self.adam
            lr_t = lr * math.sqrt(1 - b2 ** self.t) / (1 - b1 ** self.t)
        return {"lr_t": lr_t}

    @torch.no_grad()
    def _step_torch(self, g, lr, grad_scale, wd, clip, mom, b1, b2, eps, lr_t, w_decay=None):
        w = self.flat.update_target
        gk = g * grad_scale
        if wd:
            wd_src = w if w_decay is None else w_decay
            dm = self.decay_mask
            gk = gk + (wd * wd_src if dm is None else wd * wd_src * dm.to(w.device, w.dtype))
        if clip > 0:
            gk = gk.clamp(-clip, clip)
        if self.kind == "sgd":
            w.sub_(lr * gk)
        elif self.kind == "momentum":
            self.s1.mul_(mom).add_(gk)
            if self.nesterov:
                w.sub_(lr * (gk + mom * self.s1))
            else:
                w.sub_(lr * self.s1)
        elif self.kind == "rmsprop":
            self.s2.add_((gk * gk - self.s2) * (1 - b1))
            self.s1.mul_(mom).add_(lr * gk * torch.rsqrt(self.s2 + eps))
            w.sub_(self.s1)
        else:
            self.s1.add_((gk - self.s1) * (1 - b1))
            self.s2.add_((gk * gk - self.s2) * (1 - b2))
            w.sub_(lr_t * self.s1 / (self.s2.sqrt() + eps))
        if self.flat.lp is not None and self.flat.master is None:
            self.flat.lp.copy_(w)


# --------------------------------------------------------------- LR schedules
def get_piecewise_learning_rate(schedule: str, global_step: int, num_batches_per_epoch: float):
    """'lr0;e1;lr1;...;eN;lrN' -> lr_i for epochs in (e_i, e_{i+1}]
    (boundaries in steps = int(num_batches_per_epoch * e_i))."""
    pieces = schedule.split(";")
    if len(pieces) % 2 == 0:
        raise ValueError("--piecewise_learning_rate_schedule must have an odd number of "
                         "components")
    values, boundaries = [], []
    for i, piece in enumerate(pieces):
        if i % 2 == 0:
            try:
                values.append(float(piece))
            except ValueError:
                raise ValueError("Invalid learning rate: " + piece)
        else:
            try:
                b = int(int(piece) * num_batches_per_epoch) - 1
            except ValueError:
                raise ValueError("Invalid epoch: " + piece)
            boundaries.append(b)
    for a, b in zip(boundaries, boundaries[1:]):
        if not a < b:
            raise ValueError("Epoch boundaries must be increasing")
    for b, v in zip(boundaries, values):
        if global_step <= b:
            return v
    return values[-1]


def validate_lr_params(params):
    if params.piecewise_learning_rate_schedule and (
            params.init_learning_rate is not None or params.learning_rate_decay_factor or
            params.minimum_learning_rate or params.num_epochs_per_decay):
        raise ValueError("No other learning rate-related flags can be specified if "
                         "--piecewise_learning_rate_schedule is specified")


def get_learning_rate(params, global_step: int, num_examples_per_epoch: int, model,
                      batch_size: int) -> float:
    num_batches_per_epoch = float(num_examples_per_epoch) / batch_size
    if params.piecewise_learning_rate_schedule:
        validate_lr_params(params)
        lr = get_piecewise_learning_rate(params.piecewise_learning_rate_schedule, global_step,
                                         num_batches_per_epoch)
    elif params.init_learning_rate is not None:
        lr = params.init_learning_rate
        if params.num_epochs_per_decay > 0 and params.learning_rate_decay_factor > 0:
            decay_steps = int(num_batches_per_epoch * params.num_epochs_per_decay)
            lr = params.init_learning_rate * (
                params.learning_rate_decay_factor ** (global_step // max(decay_steps, 1)))
            if params.minimum_learning_rate != 0.0:
                lr = max(lr, params.minimum_learning_rate)
    else:
        lr = model.get_learning_rate(global_step, batch_size)
    if params.num_learning_rate_warmup_epochs > 0 and (
            params.init_learning_rate is not None or params.piecewise_learning_rate_schedule):
        warmup_steps = int(num_batches_per_epoch * params.num_learning_rate_warmup_epochs)
        init_lr = params.init_learning_rate
        if init_lr is None:
            init_lr = float(params.piecewise_learning_rate_schedule.split(";")[0])
        if global_step < warmup_steps:
            lr = init_lr * float(global_step) / float(warmup_steps)
    return float(lr)
