"""Checkpoint save / restore (placeholder; replaced by the TF-bundle writer)."""

from __future__ import annotations

import glob
import os
import re

import torch

from .. import cnn_util


class Saver:
    def __init__(self, bench, max_to_keep=5):
        self.bench = bench
        self.max_to_keep = max_to_keep

    def save(self, train_dir, global_step):
        os.makedirs(train_dir, exist_ok=True)
        path = os.path.join(train_dir, "model.ckpt-%d.pt" % global_step)
        state = {k: v.detach().cpu() for k, v in self.bench.net.tf_variables().items()}
        torch.save(state, path)
        return path

    def restore_latest(self, train_dir):
        files = glob.glob(os.path.join(train_dir, "model.ckpt-*.pt"))
        if not files:
            return None
        step = max(int(re.search(r"ckpt-(\d+)", f).group(1)) for f in files)
        state = torch.load(os.path.join(train_dir, "model.ckpt-%d.pt" % step), weights_only=True)
        self.bench.net.load_tf_variables(state)
        self.bench.flat.refresh_lp()
        self.bench.global_step = step
        return step

    def restore_partial(self, path):
        pass
