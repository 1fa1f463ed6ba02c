"""Inception v3 (optional auxiliary head) and Inception v4
(tcb/models/inception_model.py:44-209).  299 input, batch-norm on every conv
with the builder defaults (decay 0.999, eps 1e-3, no scale)."""

from . import model


class Inceptionv3Model(model.CNNModel):
    def __init__(self, params=None, auxiliary=False):
        self._auxiliary = auxiliary
        super().__init__("inception3", 299, 32, 0.005, params=params)

    def add_inference(self, cnn):
        def inception_v3_a(cnn, n):
            cols = [[("conv", 64, 1, 1)], [("conv", 48, 1, 1), ("conv", 64, 5, 5)],
                    [("conv", 64, 1, 1), ("conv", 96, 3, 3), ("conv", 96, 3, 3)],
                    [("apool", 3, 3, 1, 1, "SAME"), ("conv", n, 1, 1)]]
            cnn.inception_module("incept_v3_a", cols)

        def inception_v3_b(cnn):
            cols = [[("conv", 384, 3, 3, 2, 2, "VALID")],
                    [("conv", 64, 1, 1), ("conv", 96, 3, 3), ("conv", 96, 3, 3, 2, 2, "VALID")],
                    [("mpool", 3, 3, 2, 2, "VALID")]]
            cnn.inception_module("incept_v3_b", cols)

        def inception_v3_c(cnn, n):
            cols = [[("conv", 192, 1, 1)],
                    [("conv", n, 1, 1), ("conv", n, 1, 7), ("conv", 192, 7, 1)],
                    [("conv", n, 1, 1), ("conv", n, 7, 1), ("conv", n, 1, 7),
                     ("conv", n, 7, 1), ("conv", 192, 1, 7)],
                    [("apool", 3, 3, 1, 1, "SAME"), ("conv", 192, 1, 1)]]
            cnn.inception_module("incept_v3_c", cols)

        def inception_v3_d(cnn):
            cols = [[("conv", 192, 1, 1), ("conv", 320, 3, 3, 2, 2, "VALID")],
                    [("conv", 192, 1, 1), ("conv", 192, 1, 7), ("conv", 192, 7, 1),
                     ("conv", 192, 3, 3, 2, 2, "VALID")],
                    [("mpool", 3, 3, 2, 2, "VALID")]]
            cnn.inception_module("incept_v3_d", cols)

        def inception_v3_e(cnn, pooltype):
            cols = [[("conv", 320, 1, 1)], [("conv", 384, 1, 1), ("conv", 384, 1, 3)],
                    [("share",), ("conv", 384, 3, 1)],
                    [("conv", 448, 1, 1), ("conv", 384, 3, 3), ("conv", 384, 1, 3)],
                    [("share",), ("share",), ("conv", 384, 3, 1)],
                    [("mpool" if pooltype == "max" else "apool", 3, 3, 1, 1, "SAME"),
                     ("conv", 192, 1, 1)]]
            cnn.inception_module("incept_v3_e", cols)

        def incept_v3_aux(cnn):
            assert cnn.aux_top_layer is None
            cnn.aux_top_layer = cnn.top_layer
            cnn.aux_top_size = cnn.top_size
            with cnn.switch_to_aux_top_layer():
                cnn.apool(5, 5, 3, 3, mode="VALID")
                cnn.conv(128, 1, 1, mode="SAME")
                cnn.conv(768, 5, 5, mode="VALID", stddev=0.01)
                cnn.reshape([-1, 768])

        cnn.use_batch_norm = True
        cnn.conv(32, 3, 3, 2, 2, mode="VALID")
        cnn.conv(32, 3, 3, 1, 1, mode="VALID")
        cnn.conv(64, 3, 3, 1, 1, mode="SAME")
        cnn.mpool(3, 3, 2, 2, mode="VALID")
        cnn.conv(80, 1, 1, 1, 1, mode="VALID")
        cnn.conv(192, 3, 3, 1, 1, mode="VALID")
        cnn.mpool(3, 3, 2, 2, "VALID")
        inception_v3_a(cnn, 32)
        inception_v3_a(cnn, 64)
        inception_v3_a(cnn, 64)
        inception_v3_b(cnn)
        inception_v3_c(cnn, 128)
        inception_v3_c(cnn, 160)
        inception_v3_c(cnn, 160)
        inception_v3_c(cnn, 192)
        if self._auxiliary:
            incept_v3_aux(cnn)
        inception_v3_d(cnn)
        inception_v3_e(cnn, "avg")
        inception_v3_e(cnn, "max")
        cnn.apool(8, 8, 1, 1, "VALID")
        cnn.reshape([-1, 2048])


def inception_v4_sa(cnn):
    cnn.inception_module("incept_v4_sa", [[("mpool", 3, 3, 2, 2, "VALID")],
                                          [("conv", 96, 3, 3, 2, 2, "VALID")]])


def inception_v4_sb(cnn):
    cols = [[("conv", 64, 1, 1), ("conv", 96, 3, 3, 1, 1, "VALID")],
            [("conv", 64, 1, 1), ("conv", 64, 7, 1), ("conv", 64, 1, 7),
             ("conv", 96, 3, 3, 1, 1, "VALID")]]
    cnn.inception_module("incept_v4_sb", cols)


def inception_v4_sc(cnn):
    cnn.inception_module("incept_v4_sc", [[("conv", 192, 3, 3, 2, 2, "VALID")],
                                          [("mpool", 3, 3, 2, 2, "VALID")]])


def inception_v4_ra(cnn, k, l, m, n):
    cols = [[("mpool", 3, 3, 2, 2, "VALID")], [("conv", n, 3, 3, 2, 2, "VALID")],
            [("conv", k, 1, 1), ("conv", l, 3, 3), ("conv", m, 3, 3, 2, 2, "VALID")]]
    cnn.inception_module("incept_v4_ra", cols)


def inception_v4_rb(cnn):
    cols = [[("mpool", 3, 3, 2, 2, "VALID")],
            [("conv", 192, 1, 1), ("conv", 192, 3, 3, 2, 2, "VALID")],
            [("conv", 256, 1, 1), ("conv", 256, 1, 7), ("conv", 320, 7, 1),
             ("conv", 320, 3, 3, 2, 2, "VALID")]]
    cnn.inception_module("incept_v4_rb", cols)


class Inceptionv4Model(model.CNNModel):
    def __init__(self, params=None):
        super().__init__("inception4", 299, 32, 0.005, params=params)

    def add_inference(self, cnn):
        def inception_v4_a(cnn):
            cols = [[("apool", 3, 3, 1, 1, "SAME"), ("conv", 96, 1, 1)],
                    [("conv", 96, 1, 1)], [("conv", 64, 1, 1), ("conv", 96, 3, 3)],
                    [("conv", 64, 1, 1), ("conv", 96, 3, 3), ("conv", 96, 3, 3)]]
            cnn.inception_module("incept_v4_a", cols)

        def inception_v4_b(cnn):
            cols = [[("apool", 3, 3, 1, 1, "SAME"), ("conv", 128, 1, 1)],
                    [("conv", 384, 1, 1)],
                    [("conv", 192, 1, 1), ("conv", 224, 1, 7), ("conv", 256, 7, 1)],
                    [("conv", 192, 1, 1), ("conv", 192, 1, 7), ("conv", 224, 7, 1),
                     ("conv", 224, 1, 7), ("conv", 256, 7, 1)]]
            cnn.inception_module("incept_v4_b", cols)

        def inception_v4_c(cnn):
            cols = [[("apool", 3, 3, 1, 1, "SAME"), ("conv", 256, 1, 1)],
                    [("conv", 256, 1, 1)], [("conv", 384, 1, 1), ("conv", 256, 1, 3)],
                    [("share",), ("conv", 256, 3, 1)],
                    [("conv", 384, 1, 1), ("conv", 448, 1, 3), ("conv", 512, 3, 1),
                     ("conv", 256, 3, 1)],
                    [("share",), ("share",), ("share",), ("conv", 256, 1, 3)]]
            cnn.inception_module("incept_v4_c", cols)

        cnn.use_batch_norm = True
        cnn.conv(32, 3, 3, 2, 2, mode="VALID")
        cnn.conv(32, 3, 3, 1, 1, mode="VALID")
        cnn.conv(64, 3, 3)
        inception_v4_sa(cnn)
        inception_v4_sb(cnn)
        inception_v4_sc(cnn)
        for _ in range(4):
            inception_v4_a(cnn)
        inception_v4_ra(cnn, 192, 224, 256, 384)
        for _ in range(7):
            inception_v4_b(cnn)
        inception_v4_rb(cnn)
        for _ in range(3):
            inception_v4_c(cnn)
        cnn.spatial_mean()
        cnn.dropout(0.8)
