"""OverFeat (tcb/models/overfeat_model.py:28-49), 231 input."""

from . import model


class OverfeatModel(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("overfeat", 231, 32, 0.005, params=params)

    def add_inference(self, cnn):
        cnn.conv(96, 11, 11, 4, 4, mode="VALID")
        cnn.mpool(2, 2)
        cnn.conv(256, 5, 5, 1, 1, mode="VALID")
        cnn.mpool(2, 2)
        cnn.conv(512, 3, 3)
        cnn.conv(1024, 3, 3)
        cnn.conv(1024, 3, 3)
        cnn.mpool(2, 2)
        cnn.reshape([-1, 1024 * 6 * 6])
        cnn.affine(3072)
        cnn.dropout()
        cnn.affine(4096)
        cnn.dropout()
