"""NCF / NeuMF recommendation model (role of
tcb/models/experimental/official_ncf_model.py, which wraps the
tensorflow/models official.recommendation.neumf_model).

NeuMF on MovieLens-20M sizes (138,493 users, 26,744 items): a GMF branch
(64-d user and item embeddings, elementwise product) and an MLP branch
(128-d user / item embeddings concatenated -> dense 256 -> 128 -> 64, ReLU),
concatenated into one linear logit.  As in the reference, the loss is a
2-way softmax cross-entropy over [1, logit] (tcb/models/experimental/
official_ncf_model.py:86-97); synthetic users/items/labels are uniform
(:99-122).  Default batch 2048, LR 0.0005; fp32 only, like the reference.

    python tf_cnn_benchmarks.py --optimizer=adam --model=ncf --batch_size=65536 \\
        --weight_decay=0
"""

from __future__ import annotations

import math

import torch
from torch import nn

from ..ops import nn as F_ops
from . import model as model_lib

NUM_USERS_20M = 138493
NUM_ITEMS_20M = 26744


class _Dense(nn.Module):
    """Dense layer with the TF variable layout: kernel [in, out], bias [out]."""

    def __init__(self, fan_in, fan_out, device):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(fan_in, fan_out, device=device))
        self.bias = nn.Parameter(torch.zeros(fan_out, device=device))


class NeuMF(nn.Module):
    def __init__(self, num_users, num_items, mf_dim=64, layers=(256, 256, 128, 64),
                 gen=None, device="cpu"):
        super().__init__()
        half = layers[0] // 2
        self.mf_user = nn.Embedding(num_users, mf_dim, device=device)
        self.mf_item = nn.Embedding(num_items, mf_dim, device=device)
        self.mlp_user = nn.Embedding(num_users, half, device=device)
        self.mlp_item = nn.Embedding(num_items, half, device=device)
        dims = [layers[0]] + list(layers[1:])
        self.mlp = nn.ModuleList(_Dense(a, b, device) for a, b in zip(dims[:-1], dims[1:]))
        self.predict = _Dense(mf_dim + dims[-1], 1, device)
        with torch.no_grad():
            for emb in (self.mf_user, self.mf_item, self.mlp_user, self.mlp_item):
                emb.weight.copy_(torch.randn(emb.weight.shape, generator=gen) * 0.01)
            for lin in list(self.mlp) + [self.predict]:
                # glorot uniform for the hidden layers, lecun uniform for the logit
                fan_in, fan_out = lin.weight.shape
                lim = (math.sqrt(3.0 / fan_in) if lin is self.predict
                       else math.sqrt(6.0 / (fan_in + fan_out)))
                lin.weight.copy_((torch.rand(lin.weight.shape, generator=gen) * 2 - 1) * lim)
                lin.bias.zero_()

    def forward(self, inputs, phase_train=True):
        # embedding lookups, GMF product, dense layers and concats on our
        # kernels (ops.nn); the tables are [rows, dim] like the official model
        users, items = inputs[0], inputs[1]
        emb = F_ops.embedding
        gmf = F_ops.mul(emb(users, self.mf_user.weight), emb(items, self.mf_item.weight))
        h = F_ops.concat_channels([emb(users, self.mlp_user.weight),
                                   emb(items, self.mlp_item.weight)])
        for lin in self.mlp:
            h = F_ops.linear(h, lin.weight, lin.bias, relu=True)
        logits = F_ops.linear(F_ops.concat_channels([gmf, h]), self.predict.weight,
                              self.predict.bias)
        return model_lib.BuildNetworkResult(logits=logits, extra_info=None)


class NcfModel(model_lib.ModuleModel):
    def __init__(self, params=None):
        super().__init__("official_ncf", batch_size=2048, learning_rate=0.0005,
                         fp16_loss_scale=128, params=params)
        if self.data_type != torch.float32:
            raise ValueError("NCF model only supports float32 for now.")

    def make_module(self, nclass, device, dtype, gen):
        del nclass, dtype
        return NeuMF(NUM_USERS_20M, NUM_ITEMS_20M, gen=gen, device=device)

    def get_input_shapes(self, subset):
        del subset
        return [[self.batch_size], [self.batch_size], [self.batch_size]]

    def get_input_data_types(self, subset):
        del subset
        return [torch.int32, torch.int32, torch.int32]

    def get_synthetic_inputs(self, input_name, nclass, device="cpu", seed=0):
        # drawn on the device (one launch each; a launch tape re-samples them)
        bs, ints = self.batch_size, F_ops.synthetic_ints
        return (ints(bs, NUM_USERS_20M, device, seed, 21), ints(bs, NUM_ITEMS_20M, device, seed, 22),
                ints(bs, 2, device, seed, 23))

    def loss_function(self, inputs, build_network_result):
        logits = build_network_result.logits.float()
        # softmax over [1, logit] (kept as the official model does); the ones
        # column is a persistent tensor (no fill kernel inside the step)
        ones = getattr(self, "_ones", None)
        if ones is None or ones.shape != logits.shape or ones.device != logits.device \
                or ones.dtype != logits.dtype:
            ones = self._ones = torch.ones_like(logits)
        logits = F_ops.concat_channels([ones, logits])
        return F_ops.softmax_cross_entropy(logits, inputs[2])

    def accuracy_function(self, inputs, logits):
        pred = (logits.float().reshape(-1) > 1.0).to(torch.int32)
        correct = (pred == inputs[2]).sum().float()
        return {"top_1_accuracy": correct, "top_5_accuracy": correct}
