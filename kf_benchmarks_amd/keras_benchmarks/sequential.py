"""Minimal Keras-like Sequential model and ``fit`` on our ops (NHWC images).

Layers: Dense, Dropout, Conv2D ('same'/'valid'), MaxPooling2D, Flatten,
LSTM (last output).  Every layer runs through :mod:`kf_benchmarks_amd.ops`
(affine GEMM, implicit-GEMM conv + bias/ReLU, max-pool, dropout, the LSTM
recurrence of ops/rnn.py), so on a GPU these micro-benchmarks time our HIP
kernels like the rest of the framework; on CPU the same ops run as PyTorch.
Loss: categorical cross-entropy of the final softmax layer, computed as the
fused softmax cross-entropy of its logits (csrc/loss.hip).  Optimizer: Keras
RMSprop (rho 0.9, eps 1e-7, zero-initialized accumulator, optional time
decay) on the fused flat-buffer optimizer (csrc/optim.hip; eps sits inside
the square root there, as in TF's RMSProp - parity with Keras unpinned).
Multi-GPU (``gpus > 1``): run under kfb-run, one process per GPU; each
process trains on its slice of every batch and the flat gradient is averaged
with one all-reduce (the data-parallel role of keras.utils.multi_gpu_model).
"""

from __future__ import annotations

import math
import time
from typing import List

import numpy as np
import torch
from torch import nn

from .. import optim
from ..ops import nn as F_ops
from ..ops import rnn as rnn_ops


def _glorot(shape, fan_in, fan_out, gen):
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return (torch.rand(shape, generator=gen) * 2 - 1) * lim


class Layer:
    params: List = []

    def build(self, in_shape, device, gen):
        raise NotImplementedError

    def _param(self, name, t, device):
        p = nn.Parameter(t.to(device))
        self.params = list(self.params) + [(name, p)]
        return p


class Dense(Layer):
    def __init__(self, units, activation=None, input_shape=None):
        self.units, self.activation, self.input_shape = units, activation, input_shape

    def build(self, in_shape, device, gen):
        cin = in_shape[-1]
        self.w = self._param("dense/kernel", _glorot((cin, self.units), cin, self.units, gen),
                             device)  # TF layout [in, out]
        self.b = self._param("dense/bias", torch.zeros(self.units), device)
        return in_shape[:-1] + (self.units,)

    def __call__(self, x, training, logits=False):
        y = F_ops.linear(x, self.w, self.b, relu=self.activation == "relu")
        if self.activation == "softmax" and not logits:
            return torch.softmax(y.float(), dim=-1)
        if self.activation not in (None, "linear", "relu", "softmax"):
            raise ValueError("unknown activation %s" % self.activation)
        return y


class Dropout(Layer):
    def __init__(self, rate):
        self.rate = rate
        self.calls = 0

    def build(self, in_shape, device, gen):
        return in_shape

    def __call__(self, x, training):
        self.calls += 1
        return F_ops.dropout(x, 1.0 - self.rate, training, seed=self.calls)


class Conv2D(Layer):
    def __init__(self, filters, kernel_size, padding="valid", activation=None, input_shape=None):
        self.filters, self.k, self.padding = filters, kernel_size, padding
        self.activation, self.input_shape = activation, input_shape

    def build(self, in_shape, device, gen):
        h, w, c = in_shape
        kh, kw = self.k
        self.w = self._param("conv2d/kernel",
                             _glorot((self.filters, kh, kw, c), kh * kw * c, kh * kw * self.filters,
                                     gen), device)  # [Cout, KH, KW, Cin]
        self.b = self._param("conv2d/bias", torch.zeros(self.filters), device)
        self.pads = (F_ops.resolve_pads("SAME", h, w, kh, kw, 1, 1) if self.padding == "same"
                     else (0, 0, 0, 0))
        if self.padding == "same":
            return (h, w, self.filters)
        return (h - kh + 1, w - kw + 1, self.filters)

    def __call__(self, x, training):  # NHWC in/out
        y = F_ops.conv2d(x, self.w, None, (1, 1), self.pads)
        return F_ops.bias_act(y, self.b, self.activation == "relu")


class MaxPooling2D(Layer):
    def __init__(self, pool_size=(2, 2)):
        self.pool = pool_size

    def build(self, in_shape, device, gen):
        h, w, c = in_shape
        return (h // self.pool[0], w // self.pool[1], c)

    def __call__(self, x, training):
        ph, pw = self.pool
        return F_ops.max_pool(x, ph, pw, ph, pw, "VALID")


class Flatten(Layer):
    def build(self, in_shape, device, gen):
        return (int(np.prod(in_shape)),)

    def __call__(self, x, training):
        return x.reshape(x.shape[0], -1)


class LSTM(Layer):
    """Keras LSTM (tanh / sigmoid, unit_forget_bias): our recurrence kernel's
    forget-gate +1 with a zero bias is the same cell as Keras's forget bias
    initialized to 1."""

    def __init__(self, units, input_shape=None):
        self.units, self.input_shape = units, input_shape

    def build(self, in_shape, device, gen):
        H, F = self.units, in_shape[-1]
        self.wx = self._param("lstm/kernel", _glorot((F, 4 * H), F, 4 * H, gen), device)
        wh = torch.empty(H, 4 * H)
        nn.init.orthogonal_(wh, generator=gen)
        self.wh = self._param("lstm/recurrent_kernel", wh.view(1, H, 4 * H), device)
        self.bx = self._param("lstm/bias", torch.zeros(4 * H), device)
        return (H,)

    def __call__(self, x, training):  # [B, T, F] -> last output [B, H]
        out = rnn_ops.rnn_layer(rnn_ops.permute01(x), self.wx, self.bx, self.wh, rnn_ops.LSTM,
                                1, self.units)
        return out[-1]


class RMSprop:
    def __init__(self, lr=0.001, rho=0.9, epsilon=1e-7, decay=0.0):
        self.lr, self.rho, self.eps, self.decay = lr, rho, epsilon, decay


class TimeHistory:
    """Per-epoch wall times (role of keras_benchmarks/models/timehistory.py)."""

    def on_train_begin(self):
        self.times: List[float] = []

    def on_epoch_begin(self, epoch):
        self.epoch_time_start = time.time()

    def on_epoch_end(self, epoch):
        self.times.append(time.time() - self.epoch_time_start)


class _ParamSet:
    """The FlatParams view of a Sequential's parameters."""

    def __init__(self, named):
        self._named = named

    def trainable_variables(self):
        return self._named

    def ordered_layers(self):
        return []


class Sequential:
    def __init__(self, device=None, seed=0):
        self.layers: List[Layer] = []
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.seed = seed

    def add(self, layer, activation=None):
        if activation is not None and hasattr(layer, "activation"):
            layer.activation = activation
        self.layers.append(layer)

    def compile(self, loss="categorical_crossentropy", optimizer=None, metrics=()):
        if loss != "categorical_crossentropy":
            raise ValueError("only categorical_crossentropy is supported")
        last = self.layers[-1]
        if not (isinstance(last, Dense) and last.activation == "softmax"):
            raise ValueError("the last layer must be Dense(..., activation='softmax')")
        gen = torch.Generator().manual_seed(self.seed)
        shape = tuple(self.layers[0].input_shape)
        named = []
        for i, l in enumerate(self.layers):
            shape = l.build(shape, self.device, gen)
            named += [("layer%d/%s" % (i, n), p) for n, p in getattr(l, "params", [])]
        self.flat = optim.FlatParams(_ParamSet(named), reverse=False)
        opt = optimizer or RMSprop()
        self.opt = optim.FusedOptimizer(self.flat, "rmsprop", rmsprop_decay=opt.rho,
                                        rmsprop_momentum=0.0, rmsprop_epsilon=opt.eps)
        self.opt.s2.zero_()  # Keras' accumulator starts at zero (TF's RMSProp: ones)
        self.decay = opt.decay
        self.base_lr = opt.lr
        self.metrics = metrics

    def __call__(self, x, training=False, logits=False):
        for l in self.layers[:-1]:
            x = l(x, training)
        return self.layers[-1](x, training, logits=logits)

    def fit(self, x, y, batch_size=32, epochs=1, shuffle=False, verbose=0, callbacks=()):
        from ..parallel import comm
        world = comm.init_world(self.device.type)
        for cb in callbacks:
            cb.on_train_begin()
        n = x.shape[0]
        xt = torch.as_tensor(np.asarray(x, np.float32))
        # one-hot targets -> class ids (the fused softmax cross-entropy's labels)
        lt = torch.as_tensor(np.asarray(y)).argmax(1).to(torch.int32)
        rng = np.random.default_rng(0)
        it = 0
        history = []
        for epoch in range(epochs):
            for cb in callbacks:
                cb.on_epoch_begin(epoch)
            order = rng.permutation(n) if shuffle else np.arange(n)
            total = 0.0
            for s in range(0, n, batch_size):
                idx = order[s:s + batch_size]
                # data parallel: each rank takes its slice of the batch
                idx = idx[world.rank::world.size] if world.size > 1 else idx
                xb = xt[idx].to(self.device, non_blocking=True)
                lb = lt[idx].to(self.device, non_blocking=True)
                loss = F_ops.softmax_cross_entropy(self(xb, training=True, logits=True), lb)
                self.flat.zero_grad()
                loss.backward()
                if world.size > 1:
                    comm.all_reduce(self.flat.grad)
                lr = self.base_lr / (1.0 + self.decay * it) if self.decay else self.base_lr
                self.opt.step(lr, grad_scale=1.0 / world.size)
                it += 1
                total += float(loss.detach()) if verbose else 0.0
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            for cb in callbacks:
                cb.on_epoch_end(epoch)
            history.append(total)
        return history
