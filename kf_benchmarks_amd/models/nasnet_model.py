"""NASNet-A (mobile / large / CIFAR) (role of tcb/models/nasnet_model.py and
tcb/models/nasnet_utils.py, which build it with tf.contrib.slim).

Same cells as the reference (arXiv:1707.07012):
* normal cell  ops  [sep5x5, sep3x3, sep5x5, sep3x3, avg3x3, none, avg3x3,
  avg3x3, sep3x3, none], inputs [0,1, 1,1, 0,1, 1,1, 0,0], hidden states
  1..6 concatenated;
* reduction cell ops [sep5x5, sep7x7, max3x3, sep7x7, avg3x3, sep5x5, none,
  avg3x3, sep3x3, max3x3], inputs [0,1, 0,1, 0,1, 3,2, 2,0], states 3..6
  concatenated;
* every cell starts with relu -> 1x1 conv -> BN of its input and a
  "reduce previous layer" path (factorized reduction when the spatial size
  differs, relu -> 1x1 -> BN when only the depth differs);
* separable ops are two stacked (relu -> depthwise kxk -> pointwise 1x1 ->
  BN), the stride on the first one; drop-path v3 (scaled by cell depth and
  training progress) on every non-identity op output.

Configs (tcb/models/nasnet_model.py: _mobile/_large_imagenet/_cifar_config):
mobile 12 cells x 44 filters, stem multiplier 1; large 18 x 168, stem 3,
skip_reduction_layer_input; CIFAR 18 x 32, 3x3 stem conv.  The reference
calls the builders with num_classes=None, so no aux head / dropout / logits:
the pooled features feed the CNNModel's final affine layer.
"""

from __future__ import annotations

import math

import torch

from . import model

NORMAL = (["separable_5x5_2", "separable_3x3_2", "separable_5x5_2", "separable_3x3_2",
           "avg_pool_3x3", "none", "avg_pool_3x3", "avg_pool_3x3", "separable_3x3_2", "none"],
          [1, 0, 0, 0, 0, 0, 0], [0, 1, 1, 1, 0, 1, 1, 1, 0, 0])
REDUCTION = (["separable_5x5_2", "separable_7x7_2", "max_pool_3x3", "separable_7x7_2",
              "avg_pool_3x3", "separable_5x5_2", "none", "avg_pool_3x3", "separable_3x3_2",
              "max_pool_3x3"],
             [1, 1, 1, 0, 0, 0, 0], [0, 1, 0, 1, 0, 1, 3, 2, 2, 0])

CONFIGS = {
    "mobile": dict(stem_multiplier=1.0, num_cells=12, num_conv_filters=44,
                   drop_path_keep_prob=1.0, skip_reduction_layer_input=0, stem="imagenet",
                   total_training_steps=250000, bn=(0.9997, 1e-3)),
    "large": dict(stem_multiplier=3.0, num_cells=18, num_conv_filters=168,
                  drop_path_keep_prob=0.7, skip_reduction_layer_input=1, stem="imagenet",
                  total_training_steps=250000, bn=(0.9997, 1e-3)),
    "cifar": dict(stem_multiplier=3.0, num_cells=18, num_conv_filters=32,
                  drop_path_keep_prob=0.6, skip_reduction_layer_input=0, stem="cifar",
                  total_training_steps=937500, bn=(0.9, 1e-5)),
}


def calc_reduction_layers(num_cells, num_reduction_layers):
    return [int(float(p) / (num_reduction_layers + 1) * num_cells)
            for p in range(1, num_reduction_layers + 1)]


def _std(k, cout):
    # variance_scaling_initializer(factor=2, mode=FAN_OUT), truncated normal
    return math.sqrt(1.3 * 2.0 / (k * k * cout))


class _Builder:
    """NASNet ops on top of the ConvNetBuilder."""

    def __init__(self, cnn, cfg, total_cells):
        self.cnn = cnn
        self.cfg = cfg
        self.total_cells = total_cells
        self.net = cnn.net

    # ---- primitives
    def relu(self, x):
        return self.cnn.relu(x)

    def conv_bn(self, x, filters, k=1, stride=1, mode="SAME"):
        return self.cnn.conv(filters, k, k, stride, stride, mode=mode, input_layer=x,
                             num_channels_in=x.shape[-1], use_batch_norm=True,
                             stddev=_std(k, filters), activation=None)

    def factorized_reduction(self, x, filters, stride):
        assert filters % 2 == 0, "Need even number of filters for factorized reduction."
        cnn = self.cnn
        if stride == 1:
            return self.conv_bn(x, filters)
        p1 = cnn.apool(1, 1, stride, stride, input_layer=x, num_channels_in=x.shape[-1])
        p1 = cnn.conv(filters // 2, 1, 1, input_layer=p1, num_channels_in=x.shape[-1],
                      use_batch_norm=False, bias=None, activation=None,
                      stddev=_std(1, filters // 2))
        # shift by one pixel (pad bottom/right, drop the first row/col)
        cnn._use(x)
        from ..ops import nn as F
        x2 = F.window(x, 1, 1, 1, 1, x.shape[1], x.shape[2])  # pad bottom/right, drop row/col 0
        p2 = cnn.apool(1, 1, stride, stride, input_layer=x2, num_channels_in=x.shape[-1])
        p2 = cnn.conv(filters // 2, 1, 1, input_layer=p2, num_channels_in=x.shape[-1],
                      use_batch_norm=False, bias=None, activation=None,
                      stddev=_std(1, filters // 2))
        y = cnn.concat([p1, p2])
        return cnn.batch_norm(y, **cnn.batch_norm_config)

    def separable(self, x, filters, k, stride, layers):
        cnn = self.cnn
        for i in range(layers):
            x = self.relu(x)
            cnn.depthwise_conv(k, k, stride, stride, input_layer=x, use_batch_norm=False,
                               stddev=_std(k, x.shape[-1]), activation=None)
            x = cnn.conv(filters, 1, 1, use_batch_norm=True, stddev=_std(1, filters),
                         activation=None)
            stride = 1
        return x

    def pool(self, x, kind, k, stride):
        fn = self.cnn.apool if kind == "avg" else self.cnn.mpool
        return fn(k, k, stride, stride, mode="SAME", input_layer=x, num_channels_in=x.shape[-1])

    def drop_path(self, x, cell_num):
        """tcb/models/nasnet_model.py _apply_drop_path: the keep probability
        falls linearly with the cell index and ramps in over the first
        total_training_steps steps.  The GPU form always runs (kp = 1 is the
        identity), with kp and the seed as per-step launch-tape arguments:
        a taped step follows the schedule (Network.tape_dropout_values)."""
        base = self.cfg["drop_path_keep_prob"]
        if base >= 1.0 or not self.cnn.phase_train or self.cnn.meta:
            return x
        layer_ratio = (cell_num + 1) / float(self.total_cells)
        kp = self.net.drop_path_kp(base, layer_ratio, self.cfg["total_training_steps"])
        if kp >= 1.0 and not x.is_cuda:
            return x
        seed, key = self.net.next_dropout_seed(with_key=True)
        kp_key = self.net.drop_path_key(base, layer_ratio, self.cfg["total_training_steps"])
        from ..ops import nn as F
        return F.drop_path(x, kp, seed, kp_key, key)

    # ---- cell
    def cell(self, spec, net, filters, stride, prev, cell_num):
        ops, used, idx = spec
        cnn = self.cnn
        # reduce previous layer to the current shape
        if prev is not None:
            if prev.shape[1] != net.shape[1]:
                prev = self.factorized_reduction(self.relu(prev), filters, 2)
            elif prev.shape[-1] != filters:
                prev = self.conv_bn(self.relu(prev), filters)
        h0 = self.conv_bn(self.relu(net), filters)
        states = [h0, prev if prev is not None else net]
        i = 0
        for it in range(5):
            with cnn.scope("comb_iter_%d" % it):
                outs = []
                for side in ("left", "right"):
                    j = idx[i]
                    h = states[j]
                    op = ops[i]
                    s = stride if j < 2 else 1
                    with cnn.scope(side):
                        h = self.apply_op(h, op, s, filters, cell_num)
                    outs.append(h)
                    i += 1
                states.append(cnn.add(outs[0], outs[1]))
        # concatenate unused states, reducing mismatched ones first
        final_h, final_c = states[-1].shape[1], states[-1].shape[-1]
        with cnn.scope("cell_output"):
            for k, u in enumerate(used):
                s = states[k]
                if not u and (s.shape[1] != final_h or s.shape[-1] != final_c):
                    with cnn.scope("reduction_%d" % k):
                        states[k] = self.factorized_reduction(
                            s, final_c, 2 if s.shape[1] != final_h else 1)
            return cnn.concat([s for s, u in zip(states, used) if not u])

    def apply_op(self, x, op, stride, filters, cell_num):
        cin = x.shape[-1]
        if op.startswith("separable"):
            layers = int(op.split("_")[-1])
            k = int(op.split("_")[1].split("x")[0])
            x = self.separable(x, filters, k, stride, layers)
        elif op == "none":
            if stride > 1 or cin != filters:
                x = self.conv_bn(self.relu(x), filters, 1, stride)
        elif "pool" in op:
            kind = op.split("_")[0]
            k = int(op.split("_")[-1].split("x")[0])
            x = self.pool(x, kind, k, stride)
            if cin != filters:
                x = self.conv_bn(x, filters)
        else:
            raise ValueError("Unimplemented operation", op)
        if op != "none":
            x = self.drop_path(x, cell_num)
        return x


def build_nasnet(cnn, cfg_name):
    cfg = CONFIGS[cfg_name]
    bn_decay, bn_eps = cfg["bn"]
    cnn.use_batch_norm = True
    cnn.batch_norm_config = {"decay": bn_decay, "epsilon": bn_eps, "scale": True}
    num_cells = cfg["num_cells"]
    nf = cfg["num_conv_filters"]
    total_cells = num_cells + 2 + (2 if cfg["stem"] == "imagenet" else 0)
    b = _Builder(cnn, cfg, total_cells)
    reduction_indices = calc_reduction_layers(num_cells, 2)
    x = cnn.top_layer
    if cfg["stem"] == "imagenet":
        stem_f = int(32 * cfg["stem_multiplier"])
        net = b.conv_bn(x, stem_f, 3, 2, mode="VALID")
        outputs = [None, net]
        scaling = 1.0 / (2.0 ** 2)
        for c in range(2):
            with cnn.scope("cell_stem_%d" % c):
                net = b.cell(REDUCTION, net, int(nf * scaling), 2, outputs[-2], c)
            outputs.append(net)
            scaling *= 2.0
        true_cell = 2
    else:
        net = b.conv_bn(x, int(nf * cfg["stem_multiplier"]), 3, 1)
        outputs = [None, net]
        true_cell = 0
    scaling = 1.0
    prev = None
    for c in range(num_cells):
        if cfg["skip_reduction_layer_input"]:
            prev = outputs[-2]
        if c in reduction_indices:
            scaling *= 2.0
            with cnn.scope("reduction_cell_%d" % reduction_indices.index(c)):
                net = b.cell(REDUCTION, net, int(nf * scaling), 2, outputs[-2], true_cell)
            true_cell += 1
            outputs.append(net)
        if not cfg["skip_reduction_layer_input"]:
            prev = outputs[-2]
        with cnn.scope("cell_%d" % c):
            net = b.cell(NORMAL, net, int(nf * scaling), 1, prev, true_cell)
        true_cell += 1
        outputs.append(net)
    with cnn.scope("final_layer"):
        cnn.relu(net)
        cnn.spatial_mean()
    cnn.top_size = cnn.top_layer.shape[-1]


class NasnetModel(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("nasnet", 224, 32, 0.005, params=params)

    def add_inference(self, cnn):
        build_nasnet(cnn, "mobile")


class NasnetLargeModel(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("nasnet", 331, 16, 0.005, params=params)

    def add_inference(self, cnn):
        build_nasnet(cnn, "large")


class NasnetCifarModel(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("nasnet", 32, 32, 0.025, params=params)

    def add_inference(self, cnn):
        build_nasnet(cnn, "cifar")
