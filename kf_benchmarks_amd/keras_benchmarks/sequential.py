"""Minimal Keras-like Sequential model and ``fit`` on torch (NHWC images).

Layers: Dense, Dropout, Conv2D ('same'/'valid'), MaxPooling2D, Flatten,
LSTM (last output).  Optimizer: RMSprop (Keras defaults rho 0.9, eps 1e-7,
optional time decay).  Loss: categorical cross-entropy on softmax outputs.
Multi-GPU (``gpus > 1``): run under kfb-run, one process per GPU; each
process trains on its slice of every batch and gradients are averaged with
an all-reduce (the data-parallel role of keras.utils.multi_gpu_model).
"""

from __future__ import annotations

import time
from typing import List, Optional

import numpy as np
import torch
from torch import nn


class Layer:
    def build(self, in_shape, device):
        raise NotImplementedError


class Dense(Layer):
    def __init__(self, units, activation=None, input_shape=None):
        self.units, self.activation, self.input_shape = units, activation, input_shape

    def build(self, in_shape, device):
        self.mod = nn.Linear(in_shape[-1], self.units, device=device)
        nn.init.xavier_uniform_(self.mod.weight)
        nn.init.zeros_(self.mod.bias)
        return in_shape[:-1] + (self.units,)

    def __call__(self, x, training):
        y = self.mod(x)
        return _act(y, self.activation)


class Dropout(Layer):
    def __init__(self, rate):
        self.rate = rate

    def build(self, in_shape, device):
        self.mod = None
        return in_shape

    def __call__(self, x, training):
        return torch.nn.functional.dropout(x, self.rate, training)


class Conv2D(Layer):
    def __init__(self, filters, kernel_size, padding="valid", activation=None, input_shape=None):
        self.filters, self.k, self.padding = filters, kernel_size, padding
        self.activation, self.input_shape = activation, input_shape

    def build(self, in_shape, device):
        h, w, c = in_shape
        kh, kw = self.k
        self.mod = nn.Conv2d(c, self.filters, self.k,
                             padding=(kh // 2, kw // 2) if self.padding == "same" else 0,
                             device=device)
        nn.init.xavier_uniform_(self.mod.weight)
        nn.init.zeros_(self.mod.bias)
        if self.padding == "same":
            return (h, w, self.filters)
        return (h - kh + 1, w - kw + 1, self.filters)

    def __call__(self, x, training):  # NHWC in/out
        y = self.mod(x.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
        return _act(y, self.activation)


class MaxPooling2D(Layer):
    def __init__(self, pool_size=(2, 2)):
        self.pool = pool_size

    def build(self, in_shape, device):
        self.mod = None
        h, w, c = in_shape
        return (h // self.pool[0], w // self.pool[1], c)

    def __call__(self, x, training):
        y = torch.nn.functional.max_pool2d(x.permute(0, 3, 1, 2), self.pool)
        return y.permute(0, 2, 3, 1)


class Flatten(Layer):
    def build(self, in_shape, device):
        self.mod = None
        return (int(np.prod(in_shape)),)

    def __call__(self, x, training):
        return x.reshape(x.shape[0], -1)


class LSTM(Layer):
    def __init__(self, units, input_shape=None):
        self.units, self.input_shape = units, input_shape

    def build(self, in_shape, device):
        self.mod = nn.LSTM(in_shape[-1], self.units, batch_first=True, device=device)
        return (self.units,)

    def __call__(self, x, training):
        out, _ = self.mod(x)
        return out[:, -1]


def _act(y, kind):
    if kind in (None, "linear"):
        return y
    if kind == "relu":
        return torch.relu(y)
    if kind == "softmax":
        return torch.softmax(y, dim=-1)
    raise ValueError("unknown activation %s" % kind)


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


class Sequential:
    def __init__(self, device=None):
        self.layers: List[Layer] = []
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.world = None

    def add(self, layer, activation=None):
        if activation is not None and hasattr(layer, "activation"):
            layer.activation = activation
        self.layers.append(layer)

    def compile(self, loss="categorical_crossentropy", optimizer=None, metrics=()):
        if loss != "categorical_crossentropy":
            raise ValueError("only categorical_crossentropy is supported")
        shape = tuple(self.layers[0].input_shape)
        for l in self.layers:
            shape = l.build(shape, self.device)
        self.params = [p for l in self.layers if getattr(l, "mod", None) is not None
                       for p in l.mod.parameters()]
        opt = optimizer or RMSprop()
        self.opt = torch.optim.RMSprop(self.params, lr=opt.lr, alpha=opt.rho, eps=opt.eps)
        self.decay = opt.decay
        self.base_lr = opt.lr
        self.metrics = metrics

    def __call__(self, x, training=False):
        for l in self.layers:
            x = l(x, training)
        return x

    def fit(self, x, y, batch_size=32, epochs=1, shuffle=False, verbose=0, callbacks=()):
        from ..parallel import comm
        world = comm.init_world(self.device.type)
        for cb in callbacks:
            cb.on_train_begin()
        n = x.shape[0]
        xt = torch.as_tensor(np.asarray(x, np.float32))
        yt = torch.as_tensor(np.asarray(y, np.float32))
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
                yb = yt[idx].to(self.device, non_blocking=True)
                probs = self(xb, training=True)
                loss = -(yb * torch.log(probs.clamp_min(1e-7))).sum(1).mean()
                self.opt.zero_grad(set_to_none=False)
                loss.backward()
                if world.size > 1:
                    for p in self.params:
                        comm.all_reduce(p.grad)
                        p.grad.mul_(1.0 / world.size)
                if self.decay:
                    for g in self.opt.param_groups:
                        g["lr"] = self.base_lr / (1.0 + self.decay * it)
                self.opt.step()
                it += 1
                total += float(loss.detach()) if verbose else 0.0
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            for cb in callbacks:
                cb.on_epoch_end(epoch)
            history.append(total)
        return history
