"""Trivial model (tcb/models/trivial_model.py:20-43): flatten -> affine(1) ->
affine(4096); the reference's default --model."""

from . import model


class TrivialModel(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("trivial", 224 + 3, 32, 0.005, params=params)

    def add_inference(self, cnn):
        cnn.reshape([-1, 227 * 227 * 3])
        cnn.affine(1)
        cnn.affine(4096)


class TrivialCifar10Model(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("trivial", 32, 32, 0.005, params=params)

    def add_inference(self, cnn):
        cnn.reshape([-1, 32 * 32 * 3])
        cnn.affine(1)
        cnn.affine(4096)
