"""AlexNet (ImageNet, 227 input) and the CIFAR-10 tutorial variant with LRN
(tcb/models/alexnet_model.py:27-89)."""

from . import model


class AlexnetModel(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("alexnet", 224 + 3, 512, 0.005, params=params)

    def add_inference(self, cnn):
        cnn.conv(64, 11, 11, 4, 4, "VALID")
        cnn.mpool(3, 3, 2, 2)
        cnn.conv(192, 5, 5)
        cnn.mpool(3, 3, 2, 2)
        cnn.conv(384, 3, 3)
        cnn.conv(384, 3, 3)
        cnn.conv(256, 3, 3)
        cnn.mpool(3, 3, 2, 2)
        cnn.reshape([-1, 256 * 6 * 6])
        cnn.affine(4096)
        cnn.dropout()
        cnn.affine(4096)
        cnn.dropout()


class AlexnetCifar10Model(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("alexnet", 32, 128, 0.1, params=params)

    def add_inference(self, cnn):
        cnn.conv(64, 5, 5, 1, 1, "SAME", stddev=5e-2)
        cnn.mpool(3, 3, 2, 2, mode="SAME")
        cnn.lrn(depth_radius=4, bias=1.0, alpha=0.001 / 9.0, beta=0.75)
        cnn.conv(64, 5, 5, 1, 1, "SAME", bias=0.1, stddev=5e-2)
        cnn.lrn(depth_radius=4, bias=1.0, alpha=0.001 / 9.0, beta=0.75)
        cnn.mpool(3, 3, 2, 2, mode="SAME")
        cnn.flatten()
        cnn.affine(384, stddev=0.04, bias=0.1)
        cnn.affine(192, stddev=0.04, bias=0.1)

    def get_learning_rate(self, global_step, batch_size):
        decay_steps = int(100 * 50000 / batch_size)
        return self.learning_rate * (0.1 ** (global_step // decay_steps))
