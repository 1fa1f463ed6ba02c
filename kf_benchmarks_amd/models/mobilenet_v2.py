"""MobileNet-v2 (role of tcb/models/mobilenet_v2.py, mobilenet.py and
mobilenet_conv_blocks.py, which build it with tf.contrib.slim).

Architecture (arXiv:1801.04381, the slim V2_DEF of tcb/models/mobilenet_v2.py:39-83):
3x3/2 conv 32 -> 17 inverted-residual blocks (expansion 1x1 conv to 6x the
input depth rounded to a multiple of 8, 3x3 depthwise conv, linear 1x1
projection; identity shortcut when stride 1 and depth unchanged) -> 1x1
conv 1280 -> global average pool -> dropout(0.8) -> 1x1 logits conv (1001,
biased).  Every conv except the projection and the logits is conv + BN +
ReLU6; BN decay 0.997, epsilon 0.001; truncated-normal(0.09) conv init.
As in the reference, the CNNModel then adds the final affine layer on the
1001-way logits.

Depthwise convs run on csrc/depthwise.hip; the 1x1 convs on the MFMA
implicit-GEMM kernels.
"""

from . import model

# (expansion factor, output depth, stride) of the 17 expanded_conv blocks
V2_BLOCKS = [(1, 16, 1),
             (6, 24, 2), (6, 24, 1),
             (6, 32, 2), (6, 32, 1), (6, 32, 1),
             (6, 64, 2), (6, 64, 1), (6, 64, 1), (6, 64, 1),
             (6, 96, 1), (6, 96, 1), (6, 96, 1),
             (6, 160, 2), (6, 160, 1), (6, 160, 1),
             (6, 320, 1)]


def make_divisible(v, divisor=8, min_value=None):
    """Channel rounding of tcb/models/mobilenet.py (_make_divisible)."""
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return int(new_v)


class MobilenetModel(model.CNNModel):
    """Mobilenet model configuration (tcb/models/mobilenet_v2.py:188-198)."""

    STDDEV = 0.09

    def __init__(self, params=None, depth_multiplier=1.0):
        super().__init__("mobilenet", 224, 32, 0.005, params=params)
        self.depth_multiplier = depth_multiplier

    def _depth(self, d):
        return make_divisible(d * self.depth_multiplier)

    def add_inference(self, cnn):
        cnn.use_batch_norm = True
        cnn.batch_norm_config = {"decay": 0.997, "epsilon": 0.001, "scale": True}
        std = self.STDDEV
        with cnn.scope("MobilenetV2"):
            cnn.conv(self._depth(32), 3, 3, 2, 2, stddev=std, activation="relu6")
            for i, (t, c, s) in enumerate(V2_BLOCKS):
                with cnn.scope("expanded_conv%s" % ("" if i == 0 else "_%d" % i)):
                    self._expanded_conv(cnn, t, self._depth(c), s, std)
            cnn.conv(self._depth(1280) if self.depth_multiplier > 1 else 1280, 1, 1,
                     stddev=std, activation="relu6")
            cnn.spatial_mean(keep_dims=True)
            cnn.dropout(0.8)
            cnn.conv(1001, 1, 1, use_batch_norm=False, stddev=std, activation=None, bias=0.0)
            cnn.reshape([-1, 1001])

    @staticmethod
    def _expanded_conv(cnn, t, out_depth, stride, std):
        x = cnn.top_layer
        in_depth = cnn.top_size
        if stride == 1 and in_depth == out_depth and not cnn.meta:
            # the block input feeds the expansion and the residual add: two
            # aliases whose gradients a native add sums (autograd's own sum
            # is a torch kernel a launch tape cannot replay)
            from ..ops import nn as F
            cnn.top_layer, x = F.fanout(x, 2, force=True)
        inner = make_divisible(in_depth * t) if t != 1 else in_depth
        if inner > in_depth:
            with cnn.scope("expand"):
                cnn.conv(inner, 1, 1, stddev=std, activation="relu6")
        with cnn.scope("depthwise"):
            cnn.depthwise_conv(3, 3, stride, stride, stddev=std, activation="relu6")
        with cnn.scope("project"):
            cnn.conv(out_depth, 1, 1, stddev=std, activation=None)
        if stride == 1 and in_depth == out_depth:
            cnn.add(cnn.top_layer, x)
            cnn.top_size = out_depth
