"""VGG 11/16/19 (tcb/models/vgg_model.py:30-79): 3x3 SAME convs with bias+ReLU,
2x2 max pools, 4096-4096 FC with dropout.  224 input, bs 64, lr 0.005."""

from . import model


def _construct_vgg(cnn, num_conv_layers):
    assert len(num_conv_layers) == 5
    for width, n in zip((64, 128, 256, 512, 512), num_conv_layers):
        for _ in range(n):
            cnn.conv(width, 3, 3)
        cnn.mpool(2, 2)
    cnn.reshape([-1, 512 * 7 * 7])
    cnn.affine(4096)
    cnn.dropout()
    cnn.affine(4096)
    cnn.dropout()


class Vgg11Model(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("vgg11", 224, 64, 0.005, params=params)

    def add_inference(self, cnn):
        _construct_vgg(cnn, [1, 1, 2, 2, 2])


class Vgg16Model(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("vgg16", 224, 64, 0.005, params=params)

    def add_inference(self, cnn):
        _construct_vgg(cnn, [2, 2, 3, 3, 3])


class Vgg19Model(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("vgg19", 224, 64, 0.005, params=params)

    def add_inference(self, cnn):
        _construct_vgg(cnn, [2, 2, 4, 4, 4])
