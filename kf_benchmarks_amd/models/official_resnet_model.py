"""The tensorflow/models "official" ImageNet ResNets (role of
tcb/models/official_resnet_model.py, which wraps
official.resnet.imagenet_main.ImagenetModel; that package is not a
dependency here, so the architecture is written with the ConvNetBuilder).

ResNet-18/34 use two-3x3 building blocks, 50/101/152/200 bottlenecks
(stride on the 3x3 conv, "v1.5" placement); v1 is post-activation, v2
pre-activation with a final BN+ReLU.  Explicit "fixed" padding for strided
convs (SAME_RESNET), BN decay 0.997 / epsilon 1e-5, he-normal conv init.
Default batch 128 for ResNet-50 and 32 otherwise, LR 0.0125 per 32 images,
x0.1 at epochs 30/60/80/90 (tcb/models/official_resnet_model.py:26-77).
"""

from __future__ import annotations

import math

from .. import datasets
from . import model as model_lib

_BLOCKS = {18: ("building", [2, 2, 2, 2]), 34: ("building", [3, 4, 6, 3]),
           50: ("bottleneck", [3, 4, 6, 3]), 101: ("bottleneck", [3, 4, 23, 3]),
           152: ("bottleneck", [3, 8, 36, 3]), 200: ("bottleneck", [3, 24, 36, 3])}


def _he(cin, k):
    return math.sqrt(2.0 / (cin * k * k))


class ImagenetResnetModel(model_lib.CNNModel):
    def __init__(self, resnet_size, version=2, params=None):
        if resnet_size not in _BLOCKS:
            raise ValueError("Not a valid resnet_size: %d" % resnet_size)
        batch_size = {50: 128, 101: 32, 152: 32}.get(resnet_size, 32)
        super().__init__("official_resnet_%d_v%d" % (resnet_size, version), 224, batch_size,
                         0.0125 * batch_size / 32, params=params)
        self.resnet_size = resnet_size
        self.version = version

    def get_learning_rate(self, global_step, batch_size):
        per_epoch = float(datasets.IMAGENET_NUM_TRAIN_IMAGES) / batch_size
        boundaries = [int(per_epoch * e) for e in (30, 60, 80, 90)]
        adjusted = self.learning_rate / self.default_batch_size * batch_size
        values = [v * adjusted for v in (1, 0.1, 0.01, 0.001, 0.0001)]
        for b, v in zip(boundaries, values):
            if global_step < b:
                return v
        return values[-1]

    # --------------------------------------------------------------- blocks
    def _conv(self, cnn, filters, k, stride, bn, relu, input_layer=None, cin=None,
              residual=None, pool=None):
        cin = cnn.top_size if cin is None else cin
        return cnn.conv(filters, k, k, stride, stride, mode="SAME_RESNET", input_layer=input_layer,
                        num_channels_in=cin, use_batch_norm=bn, bias=None,
                        stddev=_he(cin, k), activation="relu" if relu else None,
                        residual=residual, pool=pool)

    def _block_v1(self, cnn, filters, stride, project, bottleneck):
        x, cin = cnn.top_layer, cnn.top_size
        out = filters * 4 if bottleneck else filters
        shortcut = x
        if project:
            shortcut = self._conv(cnn, out, 1, stride, True, False, x, cin)
        if bottleneck:
            self._conv(cnn, filters, 1, 1, True, True, x, cin)
            self._conv(cnn, filters, 3, stride, True, True)
            self._conv(cnn, out, 1, 1, True, True, residual=shortcut)
        else:
            self._conv(cnn, filters, 3, stride, True, True, x, cin)
            self._conv(cnn, out, 3, 1, True, True, residual=shortcut)
        cnn.top_size = out

    def _block_v2(self, cnn, filters, stride, project, bottleneck):
        x, cin = cnn.top_layer, cnn.top_size
        out = filters * 4 if bottleneck else filters
        pre = cnn.batch_norm(x, relu=True, **cnn.batch_norm_config)
        shortcut = x
        if project:
            shortcut = self._conv(cnn, out, 1, stride, False, False, pre, cin)
        if bottleneck:
            self._conv(cnn, filters, 1, 1, True, True, pre, cin)
            self._conv(cnn, filters, 3, stride, True, True)
            res = self._conv(cnn, out, 1, 1, False, False)
        else:
            self._conv(cnn, filters, 3, stride, True, True, pre, cin)
            res = self._conv(cnn, out, 3, 1, False, False)
        cnn.add(shortcut, res)
        cnn.top_size = out

    def add_inference(self, cnn):
        kind, layers = _BLOCKS[self.resnet_size]
        bottleneck = kind == "bottleneck"
        cnn.use_batch_norm = True
        cnn.batch_norm_config = {"decay": 0.997, "epsilon": 1e-5, "scale": True}
        v1 = self.version == 1
        with cnn.scope("resnet_model"):
            self._conv(cnn, 64, 7, 2, v1, v1, pool=(3, 3, 2, 2, "SAME"))
            filters = 64
            for li, n in enumerate(layers):
                stride = 1 if li == 0 else 2
                with cnn.scope("block_layer%d" % (li + 1)):
                    for b in range(n):
                        with cnn.scope("block%d" % b):
                            project = b == 0
                            if v1:
                                self._block_v1(cnn, filters, stride if b == 0 else 1, project,
                                               bottleneck)
                            else:
                                self._block_v2(cnn, filters, stride if b == 0 else 1, project,
                                               bottleneck)
                filters *= 2
            if not v1:
                cnn.batch_norm(relu=True, **cnn.batch_norm_config)
            cnn.spatial_mean()


def _factory(size, version):
    def make(params=None):
        return ImagenetResnetModel(size, version=version, params=params)
    make.__name__ = "official_v%d_%d" % (version, size)
    return make


for _s in _BLOCKS:
    globals()["official_v1_%d" % _s] = _factory(_s, 1)
    globals()["official_v2_%d" % _s] = _factory(_s, 2)
