"""LeNet-5 (tcb/models/lenet_model.py:27-40), 28x28 input."""

from . import model


class Lenet5Model(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("lenet5", 28, 32, 0.005, params=params)

    def add_inference(self, cnn):
        cnn.conv(32, 5, 5)
        cnn.mpool(2, 2)
        cnn.conv(64, 5, 5)
        cnn.mpool(2, 2)
        cnn.reshape([-1, 64 * 7 * 7])
        cnn.affine(512)
