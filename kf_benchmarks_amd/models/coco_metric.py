"""COCO-style detection mAP for SSD300 evaluation (role of tcb/coco_metric.py).

The reference converts predictions to COCO json and calls pycocotools
against the annotation file; pycocotools is not available here, so this
module implements the same pipeline on the ground truth carried in the eval
batches: per-class NMS at IoU 0.5 keeping the top 200 boxes with score >
0.05 (decode_single), then COCO average precision over IoU thresholds
0.50:0.05:0.95 with 101-point interpolated precision and at most 100
detections per image (AP, AP50, AP75).  Parity with pycocotools is unpinned
(no fixture in the reference covers it); crowd/area breakdowns are omitted.
"""

from __future__ import annotations

from typing import Dict, List

import numpy as np

from . import ssd_dataloader as sd


def calc_iou(target, candidates):
    """IoU of one box against [N, 4] boxes (ltrb)."""
    lt = np.maximum(target[:2], candidates[:, :2])
    rb = np.minimum(target[2:], candidates[:, 2:])
    inter = np.prod(np.clip(rb - lt, 0, None), axis=1)
    a = np.prod(target[2:] - target[:2])
    b = np.prod(candidates[:, 2:] - candidates[:, :2], axis=1)
    return inter / np.maximum(a + b - inter, 1e-12)


def decode_single(bboxes_in, scores_in, criteria=sd.OVERLAP_CRITERIA, max_output=100,
                  max_num=sd.MAX_NUM_EVAL_BOXES):
    """Per-class greedy NMS.  -> [[box(4), score, class], ...] best first."""
    out = []
    for c in range(1, scores_in.shape[1]):  # skip background
        sc = scores_in[:, c]
        keep = sc > sd.MIN_SCORE
        if not keep.any():
            continue
        boxes, sc = bboxes_in[keep], sc[keep]
        order = np.argsort(-sc)[:max_num]
        chosen = []
        while order.size:
            i = order[0]
            chosen.append(i)
            if order.size == 1:
                break
            ious = calc_iou(boxes[i], boxes[order[1:]])
            order = order[1:][ious < criteria]
        for i in chosen:
            out.append((boxes[i], float(sc[i]), c))
    out.sort(key=lambda t: -t[1])
    return out[:max_output]


def compute_map(predictions: List[Dict[str, np.ndarray]]) -> Dict[str, float]:
    """predictions: dicts with pred_boxes [A,4], pred_scores [A,C] and the
    eval batch's gt_boxes [200,4] / gt_classes [200,1] (zero-padded)."""
    thresholds = np.linspace(0.5, 0.95, 10)
    recall_pts = np.linspace(0, 1, 101)
    dets_by_class: Dict[int, list] = {}
    gts_by_class: Dict[int, Dict[int, np.ndarray]] = {}
    for img, p in enumerate(predictions):
        gt_c = np.asarray(p["gt_classes"]).reshape(-1).astype(np.int64)
        gt_b = np.asarray(p["gt_boxes"]).reshape(-1, 4)
        valid = gt_c > 0
        for c in np.unique(gt_c[valid]):
            gts_by_class.setdefault(int(c), {})[img] = gt_b[valid & (gt_c == c)]
        for box, score, c in decode_single(np.asarray(p["pred_boxes"]),
                                           np.asarray(p["pred_scores"])):
            dets_by_class.setdefault(int(c), []).append((score, img, box))
    aps = np.full((len(thresholds), max(len(gts_by_class), 1)), np.nan)
    for ci, (c, gts) in enumerate(sorted(gts_by_class.items())):
        n_gt = sum(len(v) for v in gts.values())
        dets = sorted(dets_by_class.get(c, []), key=lambda t: -t[0])
        for ti, thr in enumerate(thresholds):
            used = {img: np.zeros(len(b), bool) for img, b in gts.items()}
            tp = np.zeros(len(dets))
            for di, (_, img, box) in enumerate(dets):
                if img not in gts:
                    continue
                ious = calc_iou(box, gts[img])
                ious[used[img]] = -1
                j = int(np.argmax(ious)) if ious.size else -1
                if j >= 0 and ious[j] >= thr:
                    used[img][j] = True
                    tp[di] = 1
            ctp = np.cumsum(tp)
            recall = ctp / max(n_gt, 1)
            precision = ctp / np.arange(1, len(dets) + 1) if len(dets) else np.zeros(0)
            # monotone precision envelope, sampled at 101 recall points
            for k in range(len(precision) - 2, -1, -1):
                precision[k] = max(precision[k], precision[k + 1])
            idx = np.searchsorted(recall, recall_pts, side="left")
            samp = np.array([precision[i] if i < len(precision) else 0.0 for i in idx])
            aps[ti, ci] = samp.mean()
    ap = float(np.nanmean(aps)) if np.isfinite(aps).any() else 0.0
    return {"AP": ap, "AP50": float(np.nanmean(aps[0])) if np.isfinite(aps[0]).any() else 0.0,
            "AP75": float(np.nanmean(aps[5])) if np.isfinite(aps[5]).any() else 0.0}
