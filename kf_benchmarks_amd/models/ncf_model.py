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

from . import model as model_lib

NUM_USERS_20M = 138493
NUM_ITEMS_20M = 26744


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
        self.mlp = nn.ModuleList(nn.Linear(a, b, device=device) for a, b in zip(dims[:-1], dims[1:]))
        self.predict = nn.Linear(mf_dim + dims[-1], 1, device=device)
        with torch.no_grad():
            for emb in (self.mf_user, self.mf_item, self.mlp_user, self.mlp_item):
                emb.weight.copy_(torch.randn(emb.weight.shape, generator=gen) * 0.01)
            for lin in list(self.mlp) + [self.predict]:
                # glorot uniform for the hidden layers, lecun uniform for the logit
                fan_in, fan_out = lin.weight.shape[1], lin.weight.shape[0]
                lim = (math.sqrt(3.0 / fan_in) if lin is self.predict
                       else math.sqrt(6.0 / (fan_in + fan_out)))
                lin.weight.copy_((torch.rand(lin.weight.shape, generator=gen) * 2 - 1) * lim)
                lin.bias.zero_()

    def forward(self, inputs, phase_train=True):
        users, items = inputs[0].long(), inputs[1].long()
        gmf = self.mf_user(users) * self.mf_item(items)
        h = torch.cat([self.mlp_user(users), self.mlp_item(items)], dim=1)
        for lin in self.mlp:
            h = torch.relu(lin(h))
        logits = self.predict(torch.cat([gmf, h], dim=1))
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
        g = torch.Generator(device="cpu").manual_seed(seed)
        bs = self.batch_size
        users = torch.randint(0, NUM_USERS_20M, (bs,), generator=g, dtype=torch.int32)
        items = torch.randint(0, NUM_ITEMS_20M, (bs,), generator=g, dtype=torch.int32)
        labels = torch.randint(0, 2, (bs,), generator=g, dtype=torch.int32)
        return users.to(device), items.to(device), labels.to(device)

    def loss_function(self, inputs, build_network_result):
        logits = build_network_result.logits.float()
        # softmax over [1, logit] (kept as the official model does)
        logits = torch.cat([torch.ones_like(logits), logits], dim=1)
        return torch.nn.functional.cross_entropy(logits, inputs[2].long())

    def accuracy_function(self, inputs, logits):
        pred = (logits.float().reshape(-1) > 1.0).to(torch.int32)
        correct = (pred == inputs[2]).sum().float()
        return {"top_1_accuracy": correct, "top_5_accuracy": correct}
