"""SSD300 with a ResNet-34 backbone (role of tcb/models/ssd_model.py, the
MLPerf single-stage detector).

Backbone: ResNet-34 v1 stem + conv2_x (3 blocks, 64) + conv3_x (4, 128,
stride 2) + conv4_x (6, 256) whose blocks all run at stride 1 (the
reference's block loop reuses the last stride of conv3_x, i.e. 1), giving a
38x38 feature map.  Extra layers 1x1/3x3 pairs down to 19/10/5/3/1; 3x3
location (4 per anchor) and class (81 per anchor) heads on the six maps,
flattened in (anchor, row, col) order to 8732 anchors.  Loss: smooth-L1 on
positive anchors + softmax cross-entropy with 3:1 hard-negative mining,
both normalized by the matched-anchor count (tcb/models/ssd_model.py:
190-260).  L2 weight decay excludes batch-norm variables (custom_l2_loss).
Batch 32, LR 1e-3 per 32 images, x0.1 at 160k/200k (scaled), 5-epoch warmup.
"""

from __future__ import annotations

import numpy as np
import torch

from .. import cnn_util, datasets
from ..ops import nn as F_ops
from . import model as model_lib
from . import resnet_model
from . import ssd_dataloader as sd

BACKBONE_MODEL_SCOPE_NAME = "resnet34_backbone"


def _xavier(cin, k, cout):
    lim = (6.0 / (cin * k * k + cout * k * k)) ** 0.5

    def init(w):
        with torch.no_grad():
            w.uniform_(-lim, lim)
    return init


class SSD300Model(model_lib.CNNModel):
    def __init__(self, label_num=sd.NUM_CLASSES, batch_size=32, learning_rate=1e-3,
                 backbone="resnet34", params=None):
        super().__init__("ssd300", 300, batch_size, learning_rate, params=params)
        if backbone != "resnet34":
            raise ValueError("Invalid backbone model %s for SSD." % backbone)
        self.label_num = label_num
        self.out_chan = [256, 512, 512, 256, 256, 256]
        self.num_dboxes = [4, 6, 6, 6, 4, 4]
        self.base_lr_batch_size = 32
        self.predictions = {}
        self.eval_global_step = 0

    def skip_final_affine_layer(self):
        return True

    def l2_param_filter(self, scope_name):
        return "batchnorm" not in scope_name

    # ----------------------------------------------------------- network
    def add_backbone_model(self, cnn):
        cnn.conv(64, 7, 7, 2, 2, mode="SAME_RESNET", use_batch_norm=True)
        cnn.mpool(3, 3, 2, 2, mode="SAME")
        for _ in range(3):
            resnet_model.residual_block(cnn, 64, 1, "v1")
        for i in range(4):
            resnet_model.residual_block(cnn, 128, 2 if i == 0 else 1, "v1", i == 0)
        for i in range(6):
            resnet_model.residual_block(cnn, 256, 1, "v1", i == 0)

    def add_inference(self, cnn):
        cnn.use_batch_norm = True
        cnn.batch_norm_config = {"decay": sd.BATCH_NORM_DECAY, "epsilon": sd.BATCH_NORM_EPSILON,
                                 "scale": True}
        with cnn.scope(BACKBONE_MODEL_SCOPE_NAME):
            self.add_backbone_model(cnn)

        def ssd_layer(depth, k, stride, mode):
            return cnn.conv(depth, k, k, stride, stride, mode=mode, use_batch_norm=False,
                            kernel_initializer=_xavier(cnn.top_size, k, depth))

        acts = [cnn.top_layer]
        for mid, out, stride, mode in ((256, 512, 2, "SAME"), (256, 512, 2, "SAME"),
                                       (128, 256, 2, "SAME"), (128, 256, 1, "VALID"),
                                       (128, 256, 1, "VALID")):
            ssd_layer(mid, 1, 1, "VALID")
            acts.append(ssd_layer(out, 3, stride, mode))
        locs, confs = [], []
        for nd, ac, oc in zip(self.num_dboxes, acts, self.out_chan):
            l = cnn.conv(nd * 4, 3, 3, 1, 1, input_layer=ac, num_channels_in=oc,
                         activation=None, use_batch_norm=False,
                         kernel_initializer=_xavier(oc, 3, nd * 4))
            c = cnn.conv(nd * self.label_num, 3, 3, 1, 1, input_layer=ac, num_channels_in=oc,
                         activation=None, use_batch_norm=False,
                         kernel_initializer=_xavier(oc, 3, nd * self.label_num))
            locs.append(l)
            confs.append(c)
        # NHWC [B,H,W,nd*k] heads -> [B, sum nd*H*W, 4 + classes] in (anchor, row, col)
        # order (one kernel per head on the GPU)
        logits = F_ops.ssd_heads(locs, confs, list(self.num_dboxes), self.label_num)
        cnn.top_layer = logits
        cnn.top_size = 4 + self.label_num
        return logits

    # ------------------------------------------------------------ inputs
    def get_input_data_types(self, subset):
        if subset == "validation":
            return [self.data_type, torch.float32, torch.float32, torch.float32, torch.int32]
        return [self.data_type, torch.float32, torch.float32, torch.float32]

    def get_input_shapes(self, subset):
        bs, s = self.batch_size, self.image_size
        if subset == "validation":
            return [[bs, s, s, self.depth], [bs, sd.MAX_NUM_EVAL_BOXES, 4],
                    [bs, sd.MAX_NUM_EVAL_BOXES, 1], [bs], [bs, 3]]
        return [[bs, s, s, self.depth], [bs, sd.NUM_SSD_BOXES, 4], [bs, sd.NUM_SSD_BOXES, 1],
                [bs]]

    def get_synthetic_inputs(self, input_name, nclass, device="cpu", seed=0):
        """Uniform images, boxes and class ids, 1..10 boxes per image, drawn on
        the device (one launch each, re-sampled per step inside a launch tape)."""
        shapes = self.get_input_shapes("train")
        u = F_ops.synthetic_uniform
        images = u(shapes[0], self.data_type, device, seed, 11)
        boxes = u(shapes[1], torch.float32, device, seed, 12)
        classes = u(shapes[2], torch.float32, device, seed, 13)
        nboxes = u(shapes[3], torch.float32, device, seed, 14, 1.0, 10.0)
        return images, boxes, classes, nboxes

    # -------------------------------------------------------------- loss
    def get_learning_rate(self, global_step, batch_size):
        base = self.learning_rate
        if self.params is not None and self.params.variable_update == "replicated":
            base = base / self.params.num_gpus
        lr = base * (batch_size / self.base_lr_batch_size)
        boundaries = [b * self.base_lr_batch_size // batch_size for b in (160000, 200000)]
        warmup = int(datasets.COCO_NUM_TRAIN_IMAGES / batch_size * 5)
        if global_step < warmup:
            return lr * global_step / warmup
        for b, d in zip(boundaries, (1, 0.1)):
            if global_step < b:
                return lr * d
        return lr * 0.01

    def loss_function(self, inputs, build_network_result):
        """Classification (softmax xent + 3:1 hard-negative mining) plus
        smooth-L1 box loss, each normalised by the matched-box count and
        averaged over the batch (tcb/models/ssd_model.py loss_function).  On
        the GPU this is the fused kernel trio of csrc/ssd_loss.hip reading
        the bf16 logits directly; ops.ssd_loss_reference is the tensor form."""
        _, gt_loc, gt_label, num_gt = inputs[:4]
        return F_ops.ssd_loss(build_network_result.logits, gt_loc, gt_label, num_gt,
                              sd.NEGS_PER_POSITIVE)

    # -------------------------------------------------------------- eval
    def accuracy_function(self, inputs, logits):
        logits = logits.float()
        anchors = torch.as_tensor(sd.default_boxes()("xywh"), device=logits.device)
        boxes = sd.decode_boxes(logits[..., :4], anchors)
        scores = torch.softmax(logits[..., 4:], dim=2)
        out = {"pred_boxes": boxes, "pred_scores": scores}
        if len(inputs) >= 5:
            out.update(gt_boxes=inputs[1], gt_classes=inputs[2], source_id=inputs[3],
                       raw_shape=inputs[4])
        return out

    def postprocess(self, results):
        from . import coco_metric
        gstep = results.get("global_step", 0)
        if gstep > self.eval_global_step:
            self.eval_global_step = gstep
            self.predictions.clear()
        n = results["pred_boxes"].shape[0]
        for i in range(n):
            sid = int(results["source_id"][i]) if "source_id" in results else len(
                self.predictions)
            self.predictions[sid] = {k: results[k][i] for k in results if k != "global_step"}
        needed = min(sd.COCO_NUM_VAL_IMAGES, getattr(self, "num_eval_images", 1 << 30))
        if len(self.predictions) >= needed:
            cnn_util.log_fn("Got results for all {:d} eval examples. Calculate mAP...".format(
                len(self.predictions)))
            metrics = coco_metric.compute_map(list(self.predictions.values()))
            self.predictions.clear()
            out = {"top_1_accuracy": metrics["AP"], "top_5_accuracy": metrics["AP50"]}
            out.update(metrics)
            return out
        cnn_util.log_fn("Got {:d} out of {:d} eval examples. Waiting for the remaining to "
                        "calculate mAP...".format(len(self.predictions), needed))
        return {"top_1_accuracy": 0.0, "top_5_accuracy": 0.0}
