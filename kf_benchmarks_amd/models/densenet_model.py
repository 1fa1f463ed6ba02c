"""DenseNet-BC-less CIFAR-10 models 40-k12, 100-k12, 100-k24
(tcb/models/densenet_model.py:27-95)."""

import math

from . import model as model_lib
from .resnet_model import piecewise_constant


class DensenetCifar10Model(model_lib.CNNModel):
    def __init__(self, model, layer_counts, growth_rate, params=None):
        self.growth_rate = growth_rate
        super().__init__(model, 32, 64, 0.1, layer_counts=layer_counts, params=params)
        self.batch_norm_config = {"decay": 0.9, "epsilon": 1e-5, "scale": True}

    def dense_block(self, cnn, growth_rate):
        input_layer = cnn.top_layer
        c = cnn.batch_norm(input_layer, relu=True, **self.batch_norm_config)
        c = cnn.conv(growth_rate, 3, 3, 1, 1, stddev=math.sqrt(2.0 / 9 / growth_rate),
                     activation=None, input_layer=c)
        size = cnn.top_size
        cnn.concat([input_layer, c])
        cnn.top_size = input_layer.shape[-1] + growth_rate
        del size

    def transition_layer(self, cnn):
        in_size = cnn.top_size
        cnn.batch_norm(relu=True, **self.batch_norm_config)
        cnn.conv(in_size, 1, 1, 1, 1, stddev=math.sqrt(2.0 / 9 / in_size))
        cnn.apool(2, 2, 2, 2)

    def add_inference(self, cnn):
        if self.layer_counts is None:
            raise ValueError("Layer counts not specified for %s" % self.get_model_name())
        if self.growth_rate is None:
            raise ValueError("Growth rate not specified for %s" % self.get_model_name())
        cnn.conv(16, 3, 3, 1, 1, activation=None)
        for _ in range(self.layer_counts[0]):
            self.dense_block(cnn, self.growth_rate)
        self.transition_layer(cnn)
        for _ in range(self.layer_counts[1]):
            self.dense_block(cnn, self.growth_rate)
        self.transition_layer(cnn)
        for _ in range(self.layer_counts[2]):
            self.dense_block(cnn, self.growth_rate)
        cnn.batch_norm(relu=True, **self.batch_norm_config)
        cnn.top_size = cnn.top_layer.shape[-1]
        cnn.spatial_mean()

    def get_learning_rate(self, global_step, batch_size):
        per_epoch = int(50000 / batch_size)
        boundaries = [per_epoch * e for e in (150, 225, 300)]
        return piecewise_constant(global_step, boundaries, [0.1, 0.01, 0.001, 0.0001])


def create_densenet40_k12_model(params=None):
    return DensenetCifar10Model("densenet40_k12", (12, 12, 12), 12, params=params)


def create_densenet100_k12_model(params=None):
    return DensenetCifar10Model("densenet100_k12", (32, 32, 32), 12, params=params)


def create_densenet100_k24_model(params=None):
    return DensenetCifar10Model("densenet100_k24", (32, 32, 32), 24, params=params)
