"""Parameter-holding layer modules created by the ConvNetBuilder.

Each layer records the TF variable scope it corresponds to (e.g.
``resnet_v10/conv1``) so checkpoints keep the reference naming
(``v0/cg/<scope>/conv2d/kernel``, ``.../batchnorm3/gamma``, ...; see
tcb/convnet_builder.py:107-124, 311-345, 408-461).
"""

from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch
from torch import nn


def truncated_normal_(t: torch.Tensor, std: float, gen: torch.Generator):
    """TF truncated_normal initializer: N(0, std) resampled outside 2 std."""
    with torch.no_grad():
        v = torch.randn(t.shape, generator=gen)
        for _ in range(8):
            bad = v.abs() > 2
            if not bad.any():
                break
            v[bad] = torch.randn(int(bad.sum()), generator=gen)
        v.clamp_(-2, 2)
        t.copy_(v * std)
    return t


def glorot_uniform_(t: torch.Tensor, fan_in: int, fan_out: int, gen: torch.Generator):
    limit = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        t.copy_(torch.rand(t.shape, generator=gen) * (2 * limit) - limit)
    return t


class Layer(nn.Module):
    tf_scope: str = ""

    def tf_variables(self) -> Dict[str, torch.Tensor]:
        """{tf variable name (relative to the layer scope): tensor in TF layout}."""
        raise NotImplementedError

    def load_tf_variable(self, name: str, value: np.ndarray) -> None:
        raise NotImplementedError


class ConvLayer(Layer):
    """Weight stored [Cout, KH, KW, Cin] (kernel layout); TF layout is
    [KH, KW, Cin, Cout] and is produced on checkpoint export."""

    def __init__(self, scope, cin, cout, kh, kw, use_bias, bias_init, stddev, gen, device,
                 kernel_initializer=None):
        super().__init__()
        self.tf_scope = scope
        self.cin, self.cout, self.kh, self.kw = cin, cout, kh, kw
        w = torch.empty((cout, kh, kw, cin), dtype=torch.float32)
        if kernel_initializer is not None:
            if callable(kernel_initializer):
                kernel_initializer(w)
            else:
                w.fill_(float(kernel_initializer))
        elif stddev is not None:
            truncated_normal_(w, stddev, gen)
        else:  # tf.layers default kernel initializer
            glorot_uniform_(w, cin * kh * kw, cout * kh * kw, gen)
        self.weight = nn.Parameter(w.to(device))
        self.bias = None
        if use_bias:
            self.bias = nn.Parameter(torch.full((cout,), float(bias_init), device=device))
        self.weight_lp: Optional[torch.Tensor] = None
        self.weight_t: Optional[torch.Tensor] = None  # dgrad layout (ops.conv_hip.DgradWeights)
        self.stride = None

    def tf_variables(self):
        out = {"conv2d/kernel": self.weight.detach().permute(1, 2, 3, 0)}
        if self.bias is not None:
            out["biases"] = self.bias.detach()
        return out

    def load_tf_variable(self, name, value):
        t = torch.as_tensor(value, dtype=torch.float32)
        with torch.no_grad():
            if name == "conv2d/kernel":
                self.weight.copy_(t.permute(3, 0, 1, 2))
            elif name == "biases":
                self.bias.copy_(t)
            else:
                raise KeyError(name)


class DepthwiseConvLayer(Layer):
    """Depthwise filter [KH, KW, C] (channel multiplier 1); TF layout
    [KH, KW, C, 1] (slim.separable_conv2d ``depthwise_weights``)."""

    def __init__(self, scope, channels, kh, kw, stddev, gen, device):
        super().__init__()
        self.tf_scope = scope
        self.cin = self.cout = channels
        self.kh, self.kw = kh, kw
        w = torch.empty((kh, kw, channels), dtype=torch.float32)
        if stddev is not None:
            truncated_normal_(w, stddev, gen)
        else:  # xavier over the depthwise fan (slim's default initializer)
            glorot_uniform_(w, kh * kw, kh * kw, gen)
        self.weight = nn.Parameter(w.to(device))
        self.weight_lp: Optional[torch.Tensor] = None

    def tf_variables(self):
        return {"depthwise_weights": self.weight.detach().unsqueeze(-1)}

    def load_tf_variable(self, name, value):
        if name != "depthwise_weights":
            raise KeyError(name)
        with torch.no_grad():
            self.weight.copy_(torch.as_tensor(value, dtype=torch.float32).reshape(
                self.weight.shape))


class BatchNormLayer(Layer):
    def __init__(self, scope, channels, scale, decay, eps, device):
        super().__init__()
        self.tf_scope = scope
        self.decay, self.eps = float(decay), float(eps)
        self.gamma = nn.Parameter(torch.ones(channels, device=device)) if scale else None
        self.beta = nn.Parameter(torch.zeros(channels, device=device))
        self.register_buffer("moving_mean", torch.zeros(channels, device=device))
        self.register_buffer("moving_variance", torch.ones(channels, device=device))
        # shift of the training-mode statistics partials (the previous step's
        # batch mean; csrc/bn.hip bn_finalize_stats_k) - not a TF variable
        self.register_buffer("stat_shift", torch.zeros(channels, device=device),
                             persistent=False)
        # the training-mode finalize's outputs (mean | invstd, scale | shift)
        # when the producing conv's last workgroup computes them
        # (ops/conv_hip.attach_bn_finalize): persistent, so a launch tape
        # replays stable addresses
        self.register_buffer("fin_st", torch.zeros(2, channels, device=device), persistent=False)
        self.register_buffer("fin_coef", torch.zeros(2 * channels, device=device),
                             persistent=False)

    def tf_variables(self):
        out = {"beta": self.beta.detach(), "moving_mean": self.moving_mean,
               "moving_variance": self.moving_variance}
        if self.gamma is not None:
            out["gamma"] = self.gamma.detach()
        return out

    def load_tf_variable(self, name, value):
        t = torch.as_tensor(value, dtype=torch.float32)
        with torch.no_grad():
            getattr(self, name).copy_(t)


class AffineLayer(Layer):
    """weights [Cin, Cout] (TF layout, used as the GEMM's B operand)."""

    def __init__(self, scope, cin, cout, bias_init, stddev, gen, device):
        super().__init__()
        self.tf_scope = scope
        w = torch.empty((cin, cout), dtype=torch.float32)
        truncated_normal_(w, stddev, gen)
        self.weights = nn.Parameter(w.to(device))
        self.biases = nn.Parameter(torch.full((cout,), float(bias_init), device=device))
        self.weights_lp: Optional[torch.Tensor] = None

    def tf_variables(self):
        return {"weights": self.weights.detach(), "biases": self.biases.detach()}

    def load_tf_variable(self, name, value):
        t = torch.as_tensor(value, dtype=torch.float32)
        with torch.no_grad():
            getattr(self, name).copy_(t)
