"""ResNet v1 / v1.5 / v2 (ImageNet, 50/101/152) and CIFAR-10 ResNets.

Block structure follows the intended (pre-fork) definition
(tcb/models/resnet_model_legacy.py:42-198 / tcb/models/resnet_model.py:41-276):
v1 puts the stride on the first 1x1 conv, v1.5 on the 3x3, v2 uses
pre-activation.  The v1/v1.5 block tail relu(shortcut + bn(conv3)) runs as a
single fused BN epilogue (``residual=`` on the last conv).
Learning-rate defaults: 0.128 per 256 images, /num_gpus in replicated mode,
5-epoch warmup, decay x0.1 at epochs 30/60/80/90 (tcb/models/resnet_model.py:330-361).
"""

from __future__ import annotations

from .. import datasets
from . import model as model_lib


def bottleneck_block_v1(cnn, depth, depth_bottleneck, stride):
    input_layer, in_size = cnn.top_layer, cnn.top_size
    name = "resnet_v1%d" % cnn.counts["resnet_v1"]
    cnn.counts["resnet_v1"] += 1
    with cnn.scope(name):
        if depth == in_size:
            shortcut = input_layer if stride == 1 else cnn.apool(
                1, 1, stride, stride, input_layer=input_layer, num_channels_in=in_size)
        else:
            # projection shortcut: independent of the a/b convs until the tail
            # (its BN is applied inside the block-output BN: defer_bn)
            with cnn.side_branch(input_layer):
                shortcut = cnn.conv(depth, 1, 1, stride, stride, activation=None,
                                    use_batch_norm=True, input_layer=input_layer,
                                    num_channels_in=in_size, bias=None, defer_bn=True)
        cnn.conv(depth_bottleneck, 1, 1, stride, stride, input_layer=input_layer,
                 num_channels_in=in_size, use_batch_norm=True, bias=None)
        cnn.conv(depth_bottleneck, 3, 3, 1, 1, mode="SAME_RESNET", use_batch_norm=True,
                 bias=None)
        cnn.conv(depth, 1, 1, 1, 1, activation="relu", use_batch_norm=True, bias=None,
                 residual=cnn.join_branch(shortcut))
        cnn.top_size = depth


def bottleneck_block_v1_5(cnn, depth, depth_bottleneck, stride):
    input_layer, in_size = cnn.top_layer, cnn.top_size
    name = "resnet_v1.5%d" % cnn.counts["resnet_v1.5"]
    cnn.counts["resnet_v1.5"] += 1
    with cnn.scope(name):
        if depth == in_size:
            shortcut = input_layer if stride == 1 else cnn.apool(
                1, 1, stride, stride, input_layer=input_layer, num_channels_in=in_size)
        else:
            shortcut = cnn.conv(depth, 1, 1, stride, stride, activation=None,
                                use_batch_norm=True, input_layer=input_layer,
                                num_channels_in=in_size, bias=None)
        cnn.conv(depth_bottleneck, 1, 1, 1, 1, input_layer=input_layer,
                 num_channels_in=in_size, use_batch_norm=True, bias=None)
        cnn.conv(depth_bottleneck, 3, 3, stride, stride, mode="SAME_RESNET",
                 use_batch_norm=True, bias=None)
        cnn.conv(depth, 1, 1, 1, 1, activation="relu", use_batch_norm=True, bias=None,
                 residual=shortcut)
        cnn.top_size = depth


def bottleneck_block_v2(cnn, depth, depth_bottleneck, stride):
    input_layer, in_size = cnn.top_layer, cnn.top_size
    name = "resnet_v2%d" % cnn.counts["resnet_v2"]
    cnn.counts["resnet_v2"] += 1
    if depth == in_size and not cnn.meta:
        # the block input feeds the pre-activation BN and the identity
        # shortcut (or its strided average pool): two aliases whose gradients
        # a native add sums (autograd's own sum is a torch kernel a launch
        # tape cannot replay)
        from ..ops import nn as F
        cnn.top_layer, input_layer = F.fanout(input_layer, 2)
    preact = cnn.batch_norm(relu=True)
    with cnn.scope(name):
        if depth == in_size:
            shortcut = input_layer if stride == 1 else cnn.apool(
                1, 1, stride, stride, input_layer=input_layer, num_channels_in=in_size)
        else:
            shortcut = cnn.conv(depth, 1, 1, stride, stride, activation=None,
                                use_batch_norm=False, input_layer=preact,
                                num_channels_in=in_size, bias=None)
        cnn.conv(depth_bottleneck, 1, 1, stride, stride, input_layer=preact,
                 num_channels_in=in_size, use_batch_norm=True, bias=None)
        cnn.conv(depth_bottleneck, 3, 3, 1, 1, mode="SAME_RESNET", use_batch_norm=True,
                 bias=None)
        res = cnn.conv(depth, 1, 1, 1, 1, activation=None, use_batch_norm=False, bias=None)
        cnn.add(shortcut, res)
        cnn.top_size = depth


def bottleneck_block(cnn, depth, depth_bottleneck, stride, version):
    if version == "v2":
        bottleneck_block_v2(cnn, depth, depth_bottleneck, stride)
    elif version == "v1.5":
        bottleneck_block_v1_5(cnn, depth, depth_bottleneck, stride)
    else:
        bottleneck_block_v1(cnn, depth, depth_bottleneck, stride)


def residual_block(cnn, depth, stride, version, projection_shortcut=False):
    """CIFAR basic block (two 3x3 convs)."""
    pre_activation = version == "v2"
    input_layer, in_size = cnn.top_layer, cnn.top_size
    if projection_shortcut:
        shortcut = cnn.conv(depth, 1, 1, stride, stride, activation=None, use_batch_norm=True,
                            input_layer=input_layer, num_channels_in=in_size, bias=None)
    elif in_size != depth:
        shortcut = cnn.apool(1, 1, stride, stride, input_layer=input_layer,
                             num_channels_in=in_size)
        pad = (depth - in_size) // 2
        from ..ops import nn as F_ops
        shortcut = F_ops.channel_pad(shortcut, pad, pad)
    else:
        shortcut = input_layer
    if pre_activation:
        res = cnn.batch_norm(input_layer, relu=True)
    else:
        res = input_layer
    cnn.conv(depth, 3, 3, stride, stride, input_layer=res, num_channels_in=in_size,
             use_batch_norm=True, bias=None)
    if pre_activation:
        res = cnn.conv(depth, 3, 3, 1, 1, activation=None, use_batch_norm=False, bias=None)
        cnn.add(shortcut, res)
    else:
        cnn.conv(depth, 3, 3, 1, 1, activation="relu", use_batch_norm=True, bias=None,
                 residual=shortcut)
    cnn.top_size = depth


class ResnetModel(model_lib.CNNModel):
    DEFAULT_BATCH = {"resnet50": 64, "resnet101": 32, "resnet152": 32, "resnet50_v1.5": 64,
                     "resnet101_v1.5": 32, "resnet152_v1.5": 32, "resnet50_v2": 64,
                     "resnet101_v2": 32, "resnet152_v2": 32}

    def __init__(self, model, layer_counts, params=None):
        batch_size = self.DEFAULT_BATCH.get(model, 32)
        self.base_lr_batch_size = 256
        super().__init__(model, 224, batch_size, 0.128, layer_counts, params=params)
        if "v2" in model:
            self.version = "v2"
        elif "v1.5" in model:
            self.version = "v1.5"
        else:
            self.version = "v1"

    def add_inference(self, cnn):
        if self.layer_counts is None:
            raise ValueError("Layer counts not specified for %s" % self.get_model_name())
        cnn.use_batch_norm = True
        cnn.batch_norm_config = {"decay": 0.9, "epsilon": 1e-5, "scale": True}
        # conv -> BN -> ReLU -> 3x3/2 max-pool (fused on the GPU in training)
        cnn.conv(64, 7, 7, 2, 2, mode="SAME_RESNET", use_batch_norm=True,
                 pool=(3, 3, 2, 2, "SAME"))
        for _ in range(self.layer_counts[0]):
            bottleneck_block(cnn, 256, 64, 1, self.version)
        for i in range(self.layer_counts[1]):
            bottleneck_block(cnn, 512, 128, 2 if i == 0 else 1, self.version)
        for i in range(self.layer_counts[2]):
            bottleneck_block(cnn, 1024, 256, 2 if i == 0 else 1, self.version)
        for i in range(self.layer_counts[3]):
            bottleneck_block(cnn, 2048, 512, 2 if i == 0 else 1, self.version)
        if self.version == "v2":
            cnn.batch_norm(relu=True)
        cnn.spatial_mean()

    def get_scaled_base_learning_rate(self, batch_size):
        base_lr = self.learning_rate
        if self.params is not None and self.params.variable_update == "replicated":
            base_lr = self.learning_rate / self.params.num_gpus
        return base_lr * (batch_size / self.base_lr_batch_size)

    def get_learning_rate(self, global_step, batch_size):
        rescaled = self.get_scaled_base_learning_rate(batch_size)
        per_epoch = float(datasets.IMAGENET_NUM_TRAIN_IMAGES) / batch_size
        boundaries = [int(per_epoch * e) for e in (30, 60, 80, 90)]
        values = [rescaled * v for v in (1, 0.1, 0.01, 0.001, 0.0001)]
        warmup_steps = int(per_epoch * 5)
        if global_step < warmup_steps:
            return rescaled * float(global_step) / float(warmup_steps)
        return piecewise_constant(global_step, boundaries, values)


def piecewise_constant(step, boundaries, values):
    """tf.train.piecewise_constant: values[i] for boundaries[i-1] < step <= boundaries[i]."""
    for b, v in zip(boundaries, values):
        if step <= b:
            return v
    return values[-1]


def create_resnet50_model(params):
    return ResnetModel("resnet50", (3, 4, 6, 3), params=params)


def create_resnet50_v1_5_model(params):
    return ResnetModel("resnet50_v1.5", (3, 4, 6, 3), params=params)


def create_resnet50_v2_model(params):
    return ResnetModel("resnet50_v2", (3, 4, 6, 3), params=params)


def create_resnet101_model(params):
    return ResnetModel("resnet101", (3, 4, 23, 3), params=params)


def create_resnet101_v2_model(params):
    return ResnetModel("resnet101_v2", (3, 4, 23, 3), params=params)


def create_resnet152_model(params):
    return ResnetModel("resnet152", (3, 8, 36, 3), params=params)


def create_resnet152_v2_model(params):
    return ResnetModel("resnet152_v2", (3, 8, 36, 3), params=params)


class ResnetCifar10Model(model_lib.CNNModel):
    def __init__(self, model, layer_counts, params=None):
        self.version = "v2" if "v2" in model else "v1"
        super().__init__(model, 32, 128, 0.1, layer_counts, params=params)

    def add_inference(self, cnn):
        if self.layer_counts is None:
            raise ValueError("Layer counts not specified for %s" % self.get_model_name())
        cnn.use_batch_norm = True
        cnn.batch_norm_config = {"decay": 0.9, "epsilon": 1e-5, "scale": True}
        if self.version == "v2":
            cnn.conv(16, 3, 3, 1, 1, use_batch_norm=True)
        else:
            cnn.conv(16, 3, 3, 1, 1, activation=None, use_batch_norm=True)
        for _ in range(self.layer_counts[0]):
            residual_block(cnn, 16, 1, self.version)
        for i in range(self.layer_counts[1]):
            residual_block(cnn, 32, 2 if i == 0 else 1, self.version)
        for i in range(self.layer_counts[2]):
            residual_block(cnn, 64, 2 if i == 0 else 1, self.version)
        if self.version == "v2":
            cnn.batch_norm(relu=True)
        cnn.spatial_mean()

    def get_learning_rate(self, global_step, batch_size):
        per_epoch = int(50000 / batch_size)
        boundaries = [per_epoch * e for e in (82, 123, 300)]
        return piecewise_constant(global_step, boundaries, [0.1, 0.01, 0.001, 0.0002])


def _cifar(name, counts):
    return lambda params: ResnetCifar10Model(name, counts, params=params)


create_resnet20_cifar_model = _cifar("resnet20", (3, 3, 3))
create_resnet20_v2_cifar_model = _cifar("resnet20_v2", (3, 3, 3))
create_resnet32_cifar_model = _cifar("resnet32", (5, 5, 5))
create_resnet32_v2_cifar_model = _cifar("resnet32_v2", (5, 5, 5))
create_resnet44_cifar_model = _cifar("resnet44", (7, 7, 7))
create_resnet44_v2_cifar_model = _cifar("resnet44_v2", (7, 7, 7))
create_resnet56_cifar_model = _cifar("resnet56", (9, 9, 9))
create_resnet56_v2_cifar_model = _cifar("resnet56_v2", (9, 9, 9))
create_resnet110_cifar_model = _cifar("resnet110", (18, 18, 18))
create_resnet110_v2_cifar_model = _cifar("resnet110_v2", (18, 18, 18))
