"""DeepSpeech2 (role of tcb/models/experimental/deepspeech.py).

Spectrogram [B, 3494, 161, 1] -> two conv+ReLU6+BN layers (41x11/2x2 pad
20x5, 21x11/2x1 pad 10x5, 32 filters) -> 5 bidirectional LSTM(800) layers
with BN on the inputs of layers 2..5 -> BN -> dense(29) -> CTC loss (blank =
class 28) over length-scaled inputs (tcb/models/experimental/
deepspeech.py:121-389).  Batch 128, LR 0.0005.  The recurrent layers and
the CTC loss run on our HIP kernels (ops/rnn.py: csrc/rnn.hip, csrc/ctc.hip);
the greedy decoder and CER/WER (edit distance implemented here, no nltk)
report eval quality like the reference's postprocess.
"""

from __future__ import annotations

import itertools
from typing import List, Sequence

import numpy as np
import torch
from torch import nn

from .. import cnn_util
from ..ops import nn as F_ops
from ..ops import rnn as rnn_ops
from . import model as model_lib

SPEECH_LABELS = " abcdefghijklmnopqrstuvwxyz'-"


def edit_distance(a: Sequence, b: Sequence) -> int:
    """Levenshtein distance."""
    prev = list(range(len(b) + 1))
    for i, ca in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, cb in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ca != cb))
        prev = cur
    return prev[-1]


class DeepSpeechDecoder:
    """Greedy CTC decoder with CER / WER."""

    def __init__(self, labels=SPEECH_LABELS, blank_index=28):
        self.labels = labels
        self.blank_index = blank_index
        self.int_to_char = dict(enumerate(labels))

    def convert_to_string(self, sequence):
        return "".join(self.int_to_char[int(i)] for i in sequence)

    def wer(self, decode, target):
        words = set(decode.split() + target.split())
        w2c = dict(zip(words, range(len(words))))
        return edit_distance([w2c[w] for w in decode.split()], [w2c[w] for w in target.split()])

    def cer(self, decode, target):
        return edit_distance(decode, target)

    def decode(self, char_indexes):
        merged = [k for k, _ in itertools.groupby(char_indexes)]
        return self.convert_to_string([k for k in merged if k != self.blank_index])

    def decode_logits(self, logits):
        return self.decode(list(np.argmax(logits, axis=1)))


class _BN(nn.Module):
    """Batch norm over the last (channel) dim of an NHWC-style tensor on our
    kernels (ops.nn.batch_norm); decay / epsilon of the reference."""

    def __init__(self, c, device, decay=0.997, eps=1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(c, device=device))
        self.bias = nn.Parameter(torch.zeros(c, device=device))
        self.register_buffer("running_mean", torch.zeros(c, device=device))
        self.register_buffer("running_var", torch.ones(c, device=device))
        self.decay, self.eps = decay, eps

    def forward(self, x):
        shape = x.shape
        y = F_ops.batch_norm(x.reshape(-1, 1, 1, shape[-1]), self.weight, self.bias,
                             self.running_mean, self.running_var, self.decay, self.eps,
                             self.training)
        return y.reshape(shape)


class _ConvBN(nn.Module):
    """conv (NHWC, our implicit-GEMM kernels) -> relu6 -> BN, as the reference
    (tcb/models/experimental/deepspeech.py:155-170)."""

    def __init__(self, cin, cout, k, stride, pad, gen, device):
        super().__init__()
        self.pad = pad
        self.stride = stride
        fan_in, fan_out = cin * k[0] * k[1], cout * k[0] * k[1]
        lim = (6.0 / (fan_in + fan_out)) ** 0.5
        w = (torch.rand((cout, k[0], k[1], cin), generator=gen) * 2 - 1) * lim
        self.weight = nn.Parameter(w.to(device))  # [Cout, KH, KW, Cin]
        self.bn = _BN(cout, device)

    def forward(self, x):  # x NHWC [B, T, F, C]
        ph, pw = self.pad
        y = F_ops.conv2d(x, self.weight, getattr(self, "weight_lp", None), self.stride,
                         (ph, ph, pw, pw))
        y = F_ops.activation(y, "relu6")  # relu6 before BN, as the reference
        return self.bn(y)


class _RNNLayer(nn.Module):
    """One (bi)directional recurrent layer (TF BasicLSTMCell with forget bias
    1.0, GRUCell, or the basic tanh cell) on ops.rnn: the [x, h] . W kernel of the
    reference split into an input part wx [din, dirs*G*H] (one GEMM over all
    steps) and a recurrent part wh [dirs, H, G*H]; glorot-uniform over the
    reference's [din+H, G*H] fan, zero bias."""

    def __init__(self, din, hidden, kind, dirs, gen, device):
        super().__init__()
        self.kind, self.dirs, self.hidden = kind, dirs, hidden
        G = rnn_ops.GATES[kind]
        lim = (6.0 / (din + hidden + G * hidden)) ** 0.5
        wx = (torch.rand((din, dirs * G * hidden), generator=gen) * 2 - 1) * lim
        wh = (torch.rand((dirs, hidden, G * hidden), generator=gen) * 2 - 1) * lim
        self.wx = nn.Parameter(wx.to(device))
        bx = torch.zeros(dirs, G, hidden)
        if kind == rnn_ops.GRU:
            bx[:, :2] = 1.0  # TF GRUCell's gate bias initializer
        self.bx = nn.Parameter(bx.reshape(-1).to(device))
        self.wh = nn.Parameter(wh.to(device))

    def forward(self, x):  # [T, B, din] -> [T, B, dirs*H]
        return rnn_ops.rnn_layer(x, self.wx, self.bx, self.wh, self.kind, self.dirs, self.hidden,
                                 wx_lp=getattr(self.wx, "_kfb_lp", None))


class DeepSpeech2(nn.Module):
    def __init__(self, nclass, num_rnn_layers, rnn_type, bidirectional, hidden, use_bias,
                 feature_bins, gen, device):
        super().__init__()
        self.conv1 = _ConvBN(1, 32, (41, 11), (2, 2), (20, 5), gen, device)
        self.conv2 = _ConvBN(32, 32, (21, 11), (2, 1), (10, 5), gen, device)
        f = (feature_bins + 10 - 11) // 2 + 1
        f = (f + 10 - 11) // 1 + 1
        kind = rnn_ops._KIND[rnn_type]
        dirs = 2 if bidirectional else 1
        self.rnns = nn.ModuleList()
        self.bns = nn.ModuleList()
        din = f * 32
        for i in range(num_rnn_layers):
            self.bns.append(_BN(din, device) if i > 0 else nn.Identity())
            self.rnns.append(_RNNLayer(din, hidden, kind, dirs, gen, device))
            din = hidden * dirs
        self.final_bn = _BN(din, device)
        # dense logits in the TF [in, out] layout, on the affine GEMM
        self.fc_weight = nn.Parameter(
            (torch.randn((din, nclass), generator=gen) / din ** 0.5).to(device))
        self.fc_bias = nn.Parameter(torch.zeros(nclass, device=device)) if use_bias else None

    def forward(self, inputs, phase_train=True):
        self.train(phase_train)
        x = inputs[0]  # [B, T, F, 1] (NHWC)
        x = self.conv2(self.conv1(x))
        B, T, F, C = x.shape
        # the reference flattens [F, C] per time step (channels-last); the
        # recurrent stack runs time-major
        x = rnn_ops.permute01(x.reshape(B, T, F * C))  # [T, B, F*C]
        for bn, rnn in zip(self.bns, self.rnns):
            x = rnn(bn(x))
        x = self.final_bn(x)
        logits = F_ops.linear(x.reshape(T * B, -1), self.fc_weight, self.fc_bias,
                              w_lp=getattr(self.fc_weight, "_kfb_lp", None))
        # [B, T, C] view of the time-major logits
        return model_lib.BuildNetworkResult(logits=logits.view(T, B, -1).transpose(0, 1),
                                            extra_info=None)


class DeepSpeech2Model(model_lib.ModuleModel):
    SUPPORTED_RNNS = ("lstm", "rnn", "gru")
    BATCH_NORM_EPSILON = 1e-5
    BATCH_NORM_DECAY = 0.997
    CONV_FILTERS = 32

    def __init__(self, num_rnn_layers=5, rnn_type="lstm", is_bidirectional=True,
                 rnn_hidden_size=800, use_bias=True, params=None):
        super().__init__("deepspeech2", batch_size=128, learning_rate=0.0005,
                         fp16_loss_scale=128, params=params)
        if rnn_type not in self.SUPPORTED_RNNS:
            raise ValueError("rnn_type must be one of %s" % (self.SUPPORTED_RNNS,))
        self.num_rnn_layers = num_rnn_layers
        self.rnn_type = rnn_type
        self.is_bidirectional = is_bidirectional
        self.rnn_hidden_size = rnn_hidden_size
        self.use_bias = use_bias
        self.num_feature_bins = 161
        self.max_time_steps = 3494
        self.max_label_length = 576

    def make_module(self, nclass, device, dtype, gen):
        return DeepSpeech2(nclass, self.num_rnn_layers, self.rnn_type, self.is_bidirectional,
                           self.rnn_hidden_size, self.use_bias, self.num_feature_bins, gen,
                           device)

    def get_input_data_types(self, subset):
        del subset
        return [self.data_type, torch.int32, torch.int32, torch.int32]

    def get_input_shapes(self, subset):
        del subset
        return [[self.batch_size, self.max_time_steps, self.num_feature_bins, 1],
                [self.batch_size, self.max_label_length], [self.batch_size, 1],
                [self.batch_size, 1]]

    def get_synthetic_inputs(self, input_name, nclass, device="cpu", seed=0):
        shapes = self.get_input_shapes("train")
        if torch.device(device).type == "cuda":
            # drawn on the device (one launch each, the seed a launch-tape
            # argument, so a replayed step re-samples them); the constant
            # sequence lengths are persistent tensors (no fill per step)
            B, L = shapes[1]
            feats = F_ops.synthetic_uniform(tuple(shapes[0]), self.data_type, device, seed, 31)
            labels = F_ops.synthetic_ints(B * L, 28, device, seed, 32).view(B, L)
            key = (str(device), B)
            lens = getattr(self, "_lens", None)
            if lens is None or lens[0] != key:
                lens = self._lens = (key, torch.full(shapes[2], self.max_time_steps,
                                                     dtype=torch.int32, device=device),
                                     torch.full(shapes[3], self.max_label_length,
                                                dtype=torch.int32, device=device))
            return feats, labels, lens[1], lens[2]
        g = torch.Generator(device="cpu").manual_seed(seed)
        feats = torch.rand(shapes[0], generator=g).to(device, self.data_type)
        labels = torch.randint(0, 28, shapes[1], generator=g, dtype=torch.int32).to(device)
        ilen = torch.full(shapes[2], self.max_time_steps, dtype=torch.int32, device=device)
        llen = torch.full(shapes[3], self.max_label_length, dtype=torch.int32, device=device)
        return feats, labels, ilen, llen

    def loss_function(self, inputs, build_network_result):
        logits = build_network_result.logits  # [B, T', nclass] (time-major storage)
        T = logits.shape[1]
        # sequence lengths scaled to the logits' time axis, as the reference
        # (on the device, inside the native loss)
        return rnn_ops.ctc_loss_mean(logits, inputs[1], inputs[2], inputs[3], T,
                                     self.max_time_steps)

    def accuracy_function(self, inputs, logits):
        return {"probs": torch.softmax(logits.float(), dim=-1), "labels": inputs[1]}

    def postprocess(self, results):
        probs = np.asarray(results["probs"])
        targets = np.asarray(results["labels"])
        dec = DeepSpeechDecoder()
        total_wer = total_cer = 0.0
        n = probs.shape[0]
        for i in range(n):
            pred = dec.decode_logits(probs[i])
            exp = dec.decode(list(targets[i]))
            total_cer += dec.cer(pred, exp) / float(max(len(exp), 1))
            total_wer += dec.wer(pred, exp) / float(max(len(exp.split()), 1))
        total_cer /= n
        total_wer /= n
        cnn_util.log_fn("total CER: {:f}; total WER: {:f}; total example: {:d}.".format(
            total_cer, total_wer, n))
        return {"top_1_accuracy": 1.0 - total_cer, "top_5_accuracy": 1.0 - total_wer,
                "cer": total_cer, "wer": total_wer}
