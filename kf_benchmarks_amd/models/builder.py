"""ConvNetBuilder: the layer DSL the model zoo is written in.

Same vocabulary and naming as tcb/convnet_builder.py:29-469 (conv with
SAME/VALID/SAME_RESNET, mpool, apool, reshape, affine, inception_module,
spatial_mean, dropout, batch_norm, lrn, aux head), but eager: each call runs
the op immediately on NHWC tensors through :mod:`kf_benchmarks_amd.ops`.

Variables live in a :class:`Network` and are looked up by scope name, which
plays the role of TF's variable scopes with reuse: the first (materializing)
forward creates a layer, every later forward finds it under the same name.
Two additions over the reference DSL, both pure fusions with identical
semantics: ``conv(..., residual=t)`` computes relu(bn(conv(x)) + t) in the BN
epilogue (the ResNet block tail), and ``add(a, b, relu)``.
"""

from __future__ import annotations

import collections
import contextlib
import math
import os
from typing import Optional

import numpy as np
import torch

from .. import ops
from ..ops import _native as N
from ..ops import conv as conv_ops
from ..ops import nn as F
from .layers import AffineLayer, BatchNormLayer, ConvLayer, DepthwiseConvLayer


# Independent branches (ResNet projection shortcuts) on a side stream: off
# (interleaved A/B on ResNet-50 bs256 measured 12150 (off) vs 12115 img/s (on)
# - the four projection branches are short next to the stream
# synchronization they add).
_SIDE_BRANCHES = False
# conv(defer_bn=True) returns the BN unapplied (tests/test_model_gpu.py
# compares it against always applying)
_DEFER_BN = True
# a pool consuming a BN output keeps that BN's fused backward (pool links)
_POOL_LINKS = True
# Concat outputs with an accumulation-only link (their consumers' gradients
# summed in the last conv's dgrad epilogue): off.  Inception-v3 drops 112 of
# 124 adds per 4 steps (-0.45 ms/step GPU time) but the Python link
# bookkeeping (events, stream waits) costs host time in these host-bound
# models: wall time unchanged on Inception-v3, -2% on GoogLeNet
# (profiles/r4_concat_links_ab.txt)
_CONCAT_LINKS = False
_BRANCH_STREAMS = {}


def _branch_stream(device):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _BRANCH_STREAMS.get(idx)
    if st is None:
        st = _BRANCH_STREAMS[idx] = torch.cuda.Stream(device=idx)
    return st


class ConvNetBuilder:
    def __init__(self, net, input_op, input_nchan, phase_train, dtype):
        self.net = net
        self.top_layer = input_op
        self.top_size = input_nchan
        self.phase_train = phase_train
        self.dtype = dtype
        self.counts = collections.defaultdict(int)
        self.use_batch_norm = False
        self.batch_norm_config = {}
        self.aux_top_layer = None
        self.aux_top_size = 0
        self._scopes = []
        self.meta = input_op.device.type == "meta"
        self.impl = net.kernel_impl

    # ---------------------------------------------------------------- scopes
    @contextlib.contextmanager
    def scope(self, name):
        self._scopes.append(name)
        try:
            yield
        finally:
            self._scopes.pop()

    def _scoped(self, name):
        return "/".join(self._scopes + [name])

    def _p(self, t):
        if t is None or not self.meta:
            return t
        return t.detach().to("meta")

    def _layer(self, scope, factory):
        return self.net.get_or_create(scope, factory)

    @staticmethod
    def _use(t, conv=False, resid=False, pool=False):
        """Count a consumer of a BN output (see ops.nn.BNLink): the fused BN
        backward needs every consumer to be a conv or a residual-adding BN."""
        link = getattr(t, "_kfb_bn_link", None) if t is not None else None
        if link is not None:
            if conv:
                link.convs += 1
            elif resid:
                link.resid += 1
            elif pool:
                link.pools += 1
            else:
                link.other = True

    @contextlib.contextmanager
    def side_branch(self, x):
        """Runs the enclosed layers (an independent branch reading ``x``, e.g.
        a projection shortcut) on a side HIP stream, concurrently with the
        main branch that follows.  The branch output must be passed through
        :meth:`join_branch` before the main stream uses it; autograd runs the
        branch's backward on the same side stream.  No-op off the GPU."""
        if (self.meta or not x.is_cuda or not _SIDE_BRANCHES):
            yield
            return
        main = torch.cuda.current_stream(x.device)
        side = _branch_stream(x.device)
        N.stream_wait(side.cuda_stream, main.cuda_stream, device_only=True)  # recordable
        with torch.cuda.stream(side):
            yield

    @staticmethod
    def join_branch(t):
        """Makes the current stream wait for the side branch that produced
        ``t`` (and keeps ``t``'s memory alive for it)."""
        x = t.x if isinstance(t, F.DeferredBN) else t
        if x is None or not x.is_cuda or not _SIDE_BRANCHES:
            return t
        side = _BRANCH_STREAMS.get(x.device.index)
        cur = torch.cuda.current_stream(x.device)
        if side is not None and side != cur:
            N.stream_wait(cur.cuda_stream, side.cuda_stream, device_only=True)
            x.record_stream(cur)
        return t

    @contextlib.contextmanager
    def switch_to_aux_top_layer(self):
        if self.aux_top_layer is None:
            raise RuntimeError("Empty auxiliary top layer in the network.")
        saved = (self.top_layer, self.top_size)
        self.top_layer, self.top_size = self.aux_top_layer, self.aux_top_size
        try:
            yield
        finally:
            self.aux_top_layer, self.aux_top_size = self.top_layer, self.top_size
            self.top_layer, self.top_size = saved

    # ------------------------------------------------------------------ conv
    def conv(self, num_out_channels, k_height, k_width, d_height=1, d_width=1, mode="SAME",
             input_layer=None, num_channels_in=None, use_batch_norm=None, stddev=None,
             activation="relu", bias=0.0, kernel_initializer=None, residual=None, pool=None,
             defer_bn=False):
        """``pool`` = (k_h, k_w, d_h, d_w, mode): a max-pool applied to the
        (BN + ReLU) output, i.e. conv(...) then mpool(*pool); with BN in
        training on the GPU the BN apply, ReLU and pool run as one fused op.

        ``defer_bn``: for a conv + BN with no activation whose only consumer
        is the ``residual`` of a later conv + BN (ResNet v1 projection
        shortcut): in training on the GPU the BN is returned unapplied (an
        ``ops.nn.DeferredBN``) and applied inside that later BN's apply pass;
        top_layer is left unchanged.  Otherwise a normal tensor is returned."""
        x = self.top_layer if input_layer is None else input_layer
        cin = self.top_size if num_channels_in is None else num_channels_in
        name = "conv%d" % self.counts["conv"]
        self.counts["conv"] += 1
        if use_batch_norm is None:
            use_batch_norm = self.use_batch_norm
        scope = self._scoped(name)
        use_bias = (not use_batch_norm) and bias is not None
        layer = self._layer(scope, lambda: ConvLayer(
            scope, cin, num_out_channels, k_height, k_width, use_bias, bias or 0.0, stddev,
            self.net.init_gen, self.net.param_device, kernel_initializer))
        self._use(x, conv=conv_ops.runs_hip_kernel(x, self.impl))
        if residual is not None and not use_batch_norm:
            self._use(residual)
        _, H, W, _ = x.shape
        pads = F.resolve_pads(mode, H, W, k_height, k_width, d_height, d_width)
        w = self._p(layer.weight)
        stats = None
        if use_batch_norm and self.phase_train and not self.meta and \
                conv_ops.fills_bn_stats(x, num_out_channels, self.impl):
            from ..ops import conv_hip
            # partials centered on the BN's previous batch mean (the BN this
            # conv feeds is created under the same scope right below)
            bnl = self._peek_bn_layer(name, num_out_channels)
            stats = conv_hip.stats_buffer(num_out_channels, x.device, shift=bnl.stat_shift)
            # a conv whose output only this residual BN reads (ResNet block
            # output): the conv may leave it unstored and the BN's apply pass
            # recompute it (conv_hip.conv_fwd / nn._BatchNormTrain)
            stats._kfb_defer = (residual is not None and pool is None
                                and not isinstance(residual, F.DeferredBN))
            # the plain BN forward (not the dual / fused-pool forms, which
            # finalize on their own) takes the conv's in-kernel finalize
            if not (defer_bn and activation is None and residual is None and pool is None) \
                    and pool is None and not isinstance(residual, F.DeferredBN):
                conv_hip.attach_bn_finalize(stats, bnl.gamma, bnl.beta, bnl.moving_mean,
                                            bnl.moving_variance, bnl.decay, bnl.eps,
                                            bnl.fin_st, bnl.fin_coef)
        layer.stride = (d_height, d_width)
        relu = activation == "relu"
        # conv + bias (+ ReLU) without BN: applied in the conv's epilogue
        fuse_bact = (not use_batch_norm and residual is None and not self.meta
                     and activation in ("relu", None, "linear")
                     and conv_ops.fuses_bias_act(x, self.impl))
        y = F.conv2d(x, w, None if self.meta else layer.weight_lp, (d_height, d_width), pads,
                     self.impl, stats, None if self.meta else layer.weight_t,
                     bias=self._p(layer.bias) if fuse_bact else None,
                     relu=relu and fuse_bact)
        if defer_bn and _DEFER_BN and use_batch_norm and activation is None and \
                residual is None and pool is None and stats is not None and y.is_cuda:
            with self.scope(name):
                cfg = self.batch_norm_config
                layer = self._bn_layer(num_out_channels, cfg.get("scale", False),
                                       cfg.get("decay", 0.999), cfg.get("epsilon", 0.001))
            return F.DeferredBN(y, layer.gamma, layer.beta, layer.moving_mean,
                                layer.moving_variance, layer.decay, layer.eps, stats)
        if pool is not None:
            if use_batch_norm and relu and residual is None and not self.meta and \
                    F.bn_relu_max_pool_fusable(y, stats, self.phase_train):
                with self.scope(name):
                    self.top_layer, self.top_size = y, num_out_channels
                    y = self._bn_relu_max_pool(y, stats, pool, **self.batch_norm_config)
                # the stem's pooled output feeds conv1 and the projection
                # shortcut: their data gradients sum in the last one's epilogue
                y = self._accum_link(y, always=True)
                self.top_layer, self.top_size = y, num_out_channels
                return y
        if use_batch_norm:
            act = 0 if self.meta else F.bn_act_code(activation, y, residual)
            with self.scope(name):
                self.top_layer, self.top_size = y, num_out_channels
                y = self._batch_norm(y, relu=act if act else relu, residual=residual,
                                     stats=stats, **self.batch_norm_config)
            if activation not in ("relu", None, "linear") and act != 2:
                y = F.activation(y, activation)
        else:
            if not fuse_bact:
                y = F.bias_act(y, self._p(layer.bias), relu)
            if residual is not None:
                y = F.add(y, residual)
            if activation not in ("relu", None, "linear"):
                y = F.activation(y, activation)
        self.top_layer, self.top_size = y, num_out_channels
        if pool is not None:
            return self.mpool(*pool)
        return y

    def depthwise_conv(self, k_height, k_width, d_height=1, d_width=1, mode="SAME",
                       input_layer=None, use_batch_norm=None, stddev=None, activation="relu",
                       name=None):
        """Depthwise conv (channel multiplier 1) + optional BN + activation
        (slim.separable_conv2d with num_outputs=None)."""
        from ..ops import depthwise as dw_ops
        x = self.top_layer if input_layer is None else input_layer
        C = x.shape[-1]
        name = name or "depthwise%d" % self.counts["depthwise"]
        self.counts["depthwise"] += 1
        if use_batch_norm is None:
            use_batch_norm = self.use_batch_norm
        scope = self._scoped(name)
        layer = self._layer(scope, lambda: DepthwiseConvLayer(
            scope, C, k_height, k_width, stddev, self.net.init_gen, self.net.param_device))
        self._use(x)
        _, H, W, _ = x.shape
        pads = F.resolve_pads(mode, H, W, k_height, k_width, d_height, d_width)
        y = dw_ops.depthwise_conv2d(x, self._p(layer.weight),
                                    None if self.meta else layer.weight_lp,
                                    (d_height, d_width), pads, self.impl)
        if use_batch_norm:
            act = 0 if self.meta else F.bn_act_code(activation, y)
            with self.scope(name):
                y = self._batch_norm(y, relu=act if act else activation == "relu",
                                     **self.batch_norm_config)
            if activation not in ("relu", None, "linear") and act != 2:
                y = F.activation(y, activation)
        elif activation not in (None, "linear"):
            y = F.activation(y, activation)
        self.top_layer, self.top_size = y, C
        return y

    def separable_conv(self, num_out_channels, k_height, k_width, d_height=1, d_width=1,
                       mode="SAME", input_layer=None, use_batch_norm=None, stddev=None,
                       activation="relu"):
        """Depthwise k x k then pointwise 1x1 (slim.separable_conv2d)."""
        x = self.top_layer if input_layer is None else input_layer
        name = "separable%d" % self.counts["separable"]
        self.counts["separable"] += 1
        with self.scope(name):
            self.depthwise_conv(k_height, k_width, d_height, d_width, mode, input_layer=x,
                                use_batch_norm=False, stddev=stddev, activation=None)
            return self.conv(num_out_channels, 1, 1, use_batch_norm=use_batch_norm,
                             stddev=stddev, activation=activation)

    # --------------------------------------------------------------- pooling
    def _pool(self, pool_name, k_height, k_width, d_height, d_width, mode, input_layer,
              num_channels_in):
        if input_layer is None:
            input_layer = self.top_layer
        else:
            self.top_size = num_channels_in
        kind = "max" if pool_name == "mpool" else "avg"
        self._use(input_layer, pool=_POOL_LINKS and F.pool_takes_link(
            input_layer, k_height, k_width, d_height, d_width, mode, kind))
        self.counts[pool_name] += 1
        fn = F.max_pool if pool_name == "mpool" else F.avg_pool
        y = fn(input_layer, k_height, k_width, d_height, d_width, mode)
        self.top_layer = y
        return y

    def mpool(self, k_height, k_width, d_height=2, d_width=2, mode="VALID", input_layer=None,
              num_channels_in=None):
        return self._pool("mpool", k_height, k_width, d_height, d_width, mode, input_layer,
                          num_channels_in)

    def apool(self, k_height, k_width, d_height=2, d_width=2, mode="VALID", input_layer=None,
              num_channels_in=None):
        return self._pool("apool", k_height, k_width, d_height, d_width, mode, input_layer,
                          num_channels_in)

    # ----------------------------------------------------------------- shape
    def reshape(self, shape, input_layer=None):
        x = self.top_layer if input_layer is None else input_layer
        self._use(x)
        self.top_layer = x.reshape(shape)
        self.top_size = shape[-1]
        return self.top_layer

    def flatten(self):
        """Flatten NHWC to [N, H*W*C] (the reference reshapes NCHW tensors;
        element order therefore differs but the layer is equivalent)."""
        x = self.top_layer
        self._use(x)
        n = x.shape[0]
        size = int(np.prod(x.shape[1:]))
        self.top_layer = x.reshape(n, size)
        self.top_size = size
        return self.top_layer

    # ---------------------------------------------------------------- affine
    def affine(self, num_out_channels, input_layer=None, num_channels_in=None, bias=0.0,
               stddev=None, activation="relu"):
        x = self.top_layer if input_layer is None else input_layer
        self._use(x)
        cin = self.top_size if num_channels_in is None else num_channels_in
        name = "affine%d" % self.counts["affine"]
        self.counts["affine"] += 1
        scope = self._scoped(name)
        init_factor = 2.0 if activation == "relu" else 1.0
        std = stddev or math.sqrt(init_factor / cin)
        layer = self._layer(scope, lambda: AffineLayer(
            scope, cin, num_out_channels, bias, std, self.net.init_gen, self.net.param_device))
        y = F.linear(x, self._p(layer.weights), self._p(layer.biases),
                     None if self.meta else layer.weights_lp, relu=activation == "relu")
        if activation not in ("relu", None, "linear"):
            raise KeyError("Invalid activation type '%s'" % activation)
        self.top_layer, self.top_size = y, num_out_channels
        return y

    # ------------------------------------------------------------- inception
    def inception_module(self, name, cols, input_layer=None, in_size=None):
        x = self.top_layer if input_layer is None else input_layer
        cin = self.top_size if in_size is None else in_size
        name = name + str(self.counts[name])
        self.counts[name] += 1
        with self.scope(name):
            col_layers, col_sizes = [], []
            # every column reads x: their input gradients sum natively
            heads = [c for c, col in enumerate(cols) if col and col[0][0] != "share"]
            xs = dict(zip(heads, F.fanout(x, len(heads)))) if not self.meta else {}
            for c, col in enumerate(cols):
                col_layers.append([])
                col_sizes.append([])
                for li, layer in enumerate(col):
                    ltype, args = layer[0], layer[1:]
                    kwargs = ({"input_layer": xs.get(c, x), "num_channels_in": cin}
                              if li == 0 else {})
                    if ltype == "conv":
                        self.conv(*args, **kwargs)
                    elif ltype == "mpool":
                        self.mpool(*args, **kwargs)
                    elif ltype == "apool":
                        self.apool(*args, **kwargs)
                    elif ltype == "share":
                        self.top_layer = col_layers[c - 1][li]
                        self.top_size = col_sizes[c - 1][li]
                    else:
                        raise KeyError("Invalid layer type for inception module: '%s'" % ltype)
                    col_layers[c].append(self.top_layer)
                    col_sizes[c].append(self.top_size)
            for l in col_layers:
                self._use(l[-1])
            self.top_layer = self._accum_link(F.concat_channels([l[-1] for l in col_layers]))
            self.top_size = sum(s[-1] for s in col_sizes)
        return self.top_layer

    @staticmethod
    def _accum_link(y, always=False):
        """A tensor read by several branches (a concat output; the fused stem
        BN+ReLU+max-pool output): an accumulation-only BNLink, so its
        consumers' gradients sum in the last conv's dgrad epilogue instead of
        autograd's separate adds.  Concat outputs only with _CONCAT_LINKS
        (measured neutral there); ``always`` for the stem (one 103 MB add per
        ResNet step)."""
        if (_CONCAT_LINKS or always) and y.is_cuda and getattr(y, "_kfb_bn_link", None) is None:
            # (a tensor that already carries a link keeps it: the fused stem
            # pool's BN-partials link, ops/nn.py _BNReluMaxPool)
            if conv_ops.FUSE_BN:
                link = F.BNLink(None, None, False)
                link.accum = True
                y._kfb_bn_link = link
        return y

    # ----------------------------------------------------------------- misc
    def spatial_mean(self, keep_dims=False):
        self._use(self.top_layer)
        self.counts["spatial_mean"] += 1
        self.top_layer = F.spatial_mean(self.top_layer, keep_dims)
        return self.top_layer

    def dropout(self, keep_prob=0.5, input_layer=None):
        x = self.top_layer if input_layer is None else input_layer
        self._use(x)
        if input_layer is not None:
            self.top_size = None
        self.counts["dropout"] += 1
        seed, key = self.net.next_dropout_seed(with_key=True)
        self.top_layer = F.dropout(x, keep_prob, self.phase_train and not self.meta, seed, key)
        return self.top_layer

    def batch_norm(self, input_layer=None, decay=0.999, scale=False, epsilon=0.001, relu=False,
                   residual=None):
        x = self.top_layer if input_layer is None else input_layer
        return self._batch_norm(x, decay=decay, scale=scale, epsilon=epsilon, relu=relu,
                                residual=residual)

    def _peek_bn_layer(self, name, C):
        """The BN layer the next _bn_layer call under scope ``name`` returns
        (created now if new; the batchnorm counter is not advanced)."""
        cfg = self.batch_norm_config
        with self.scope(name):
            scope = self._scoped("batchnorm%d" % self.counts["batchnorm"])
        return self._layer(scope, lambda: BatchNormLayer(
            scope, C, cfg.get("scale", False), cfg.get("decay", 0.999), cfg.get("epsilon", 0.001),
            self.net.param_device))

    def _bn_layer(self, C, scale, decay, epsilon):
        name = "batchnorm%d" % self.counts["batchnorm"]
        self.counts["batchnorm"] += 1
        scope = self._scoped(name)
        return self._layer(scope, lambda: BatchNormLayer(scope, C, scale, decay, epsilon,
                                                         self.net.param_device))

    def _bn_relu_max_pool(self, x, stats, pool, decay=0.999, scale=False, epsilon=0.001):
        """relu(batch_norm(x)) then mpool(*pool), fused (training, GPU); the
        layer names and counts are those of _batch_norm + mpool."""
        self._use(x)
        layer = self._bn_layer(x.shape[-1], scale, decay, epsilon)
        kh, kw, sh, sw, mode = (tuple(pool) + ("VALID",))[:5]
        self.counts["mpool"] += 1
        return F.bn_relu_max_pool(x, layer.gamma, layer.beta, layer.moving_mean,
                                  layer.moving_variance, layer.decay, layer.eps, stats,
                                  kh, kw, sh, sw, mode)

    def _batch_norm(self, x, decay=0.999, scale=False, epsilon=0.001, relu=False,
                    residual=None, stats=None):
        self._use(x)
        deferred = isinstance(residual, F.DeferredBN)
        self._use(None if deferred else residual, resid=True)
        C = x.shape[-1]
        layer = self._bn_layer(C, scale, decay, epsilon)
        training = self.phase_train and not self.meta
        if deferred:
            y = F.batch_norm_dual(x, layer.gamma, layer.beta, layer.moving_mean,
                                  layer.moving_variance, layer.decay, layer.eps, relu,
                                  stats if training else None, residual)
            self.top_layer, self.top_size = y, C
            return y
        if self.meta:
            y = F.batch_norm(x, self._p(layer.gamma), self._p(layer.beta),
                             self._p(layer.moving_mean), self._p(layer.moving_variance),
                             layer.decay, layer.eps, False, relu, residual)
        else:
            y = F.batch_norm(x, layer.gamma, layer.beta, layer.moving_mean,
                             layer.moving_variance, layer.decay, layer.eps, training, relu,
                             residual, stats=stats if training else None)
        self.top_layer, self.top_size = y, C
        return y

    def relu(self, x=None):
        x = self.top_layer if x is None else x
        self._use(x)
        self.top_layer = F.relu(x)
        return self.top_layer

    def add(self, a, b, relu=False):
        self._use(a)
        self._use(b)
        y = F.add(a, b, relu)
        self.top_layer = y
        return y

    def concat(self, xs):
        for t in xs:
            self._use(t)
        self.top_layer = self._accum_link(F.concat_channels(xs))
        self.top_size = self.top_layer.shape[-1]
        return self.top_layer

    def lrn(self, depth_radius, bias, alpha, beta):
        self._use(self.top_layer)
        self.counts["lrn"] += 1
        self.top_layer = F.lrn(self.top_layer, depth_radius, bias, alpha, beta)
        return self.top_layer
