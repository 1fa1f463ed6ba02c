"""SSD300 constants, default boxes, target encoding and COCO input
processing (roles of tcb/ssd_constants.py and tcb/ssd_dataloader.py; the
reference relies on the TF object-detection API for matching and box
coding, here they are numpy).

* default boxes: 8732 anchors over feature maps 38/19/10/5/3/1 with
  scales 21..315 px and aspect ratios {2} or {2, 3}, ordered
  (anchor size, row, col) per level - the head's output order;
* target assignment: IoU arg-max matching at 0.5 with a forced match for
  every ground-truth box, Faster-RCNN box coding with scales (10, 10, 5, 5);
* train augmentation: IoU-biased random crop (50 proposals per pass, min IoU
  drawn from {0, .1, .3, .5, .7, .9} or no crop), horizontal flip, colour
  jitter (brightness .125, contrast/saturation .5, hue .05), ImageNet
  mean/std normalization; eval: resize to 300 + normalization, ground truth
  padded to 200 boxes.
"""

from __future__ import annotations

import io
import itertools
import math
from concurrent.futures import ThreadPoolExecutor
from typing import Dict

import numpy as np

IMAGE_SIZE = 300
NUM_CLASSES = 81  # 80 COCO classes + background
NUM_SSD_BOXES = 8732
FEATURE_SIZES = (38, 19, 10, 5, 3, 1)
STEPS = (8, 16, 32, 64, 100, 300)
SCALES = (21, 45, 99, 153, 207, 261, 315)
ASPECT_RATIOS = ((2,), (2, 3), (2, 3), (2, 3), (2,), (2,))
NUM_DEFAULTS = (4, 6, 6, 6, 4, 4)
SCALE_XY, SCALE_HW = 0.1, 0.2
BOX_CODER_SCALES = (1 / SCALE_XY, 1 / SCALE_XY, 1 / SCALE_HW, 1 / SCALE_HW)
MATCH_THRESHOLD = 0.5
NORMALIZATION_MEAN = (0.485, 0.456, 0.406)
NORMALIZATION_STD = (0.229, 0.224, 0.225)
NUM_CROP_PASSES = 50
CROP_MIN_IOU_CHOICES = (0, 0.1, 0.3, 0.5, 0.7, 0.9)
P_NO_CROP_PER_PASS = 1 / (len(CROP_MIN_IOU_CHOICES) + 1)
NEGS_PER_POSITIVE = 3
BATCH_NORM_DECAY = 0.997
BATCH_NORM_EPSILON = 1e-4
MAX_NUM_EVAL_BOXES = 200
OVERLAP_CRITERIA = 0.5
MIN_SCORE = 0.05
COCO_NUM_VAL_IMAGES = 4952
# COCO category id (1..90, with gaps) of each of the 80 used classes (+ 0)
CLASS_INV_MAP = (0,) + tuple(i for i in range(1, 91) if i not in
                             (12, 26, 29, 30, 45, 66, 68, 69, 71, 83))
CLASS_MAP = tuple({j: i for i, j in enumerate(CLASS_INV_MAP)}.get(i, -1)
                  for i in range(max(CLASS_INV_MAP) + 1))


class DefaultBoxes:
    """8732 anchors; ``__call__('ltrb')`` -> [ymin, xmin, ymax, xmax],
    ``('xywh')`` -> [cy, cx, h, w], both clipped to [0, 1] centers/sizes."""

    def __init__(self):
        fk = IMAGE_SIZE / np.array(STEPS, dtype=np.float64)
        boxes = []
        for idx, fs in enumerate(FEATURE_SIZES):
            sk1 = SCALES[idx] / IMAGE_SIZE
            sk2 = SCALES[idx + 1] / IMAGE_SIZE
            sizes = [(sk1, sk1), (math.sqrt(sk1 * sk2),) * 2]
            for alpha in ASPECT_RATIOS[idx]:
                w, h = sk1 * math.sqrt(alpha), sk1 / math.sqrt(alpha)
                sizes += [(w, h), (h, w)]
            assert len(sizes) == NUM_DEFAULTS[idx]
            for w, h in sizes:
                for i, j in itertools.product(range(fs), repeat=2):
                    cx, cy = (j + 0.5) / fk[idx], (i + 0.5) / fk[idx]
                    boxes.append([min(max(v, 0.0), 1.0) for v in (cy, cx, h, w)])
        self.xywh = np.asarray(boxes, dtype=np.float32)
        assert self.xywh.shape[0] == NUM_SSD_BOXES
        cy, cx, h, w = self.xywh.T
        self.ltrb = np.stack([cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2], axis=1)

    def __call__(self, order="ltrb"):
        return self.ltrb if order == "ltrb" else self.xywh


_DEFAULT = None


def default_boxes() -> DefaultBoxes:
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = DefaultBoxes()
    return _DEFAULT


def calc_iou(box1: np.ndarray, box2: np.ndarray) -> np.ndarray:
    """IoU [N, M] of corner boxes (any consistent corner order)."""
    lt = np.maximum(box1[:, None, :2], box2[None, :, :2])
    rb = np.minimum(box1[:, None, 2:], box2[None, :, 2:])
    inter = np.prod(np.clip(rb - lt, 0, None), axis=2)
    a1 = np.prod(box1[:, 2:] - box1[:, :2], axis=1)
    a2 = np.prod(box2[:, 2:] - box2[:, :2], axis=1)
    return inter / np.maximum(a1[:, None] + a2[None, :] - inter, 1e-12)


def encode_boxes(boxes_ltrb: np.ndarray, anchors_xywh: np.ndarray) -> np.ndarray:
    """Faster-RCNN coding [ty, tx, th, tw] * (10, 10, 5, 5)."""
    ymin, xmin, ymax, xmax = boxes_ltrb.T
    h = np.maximum(ymax - ymin, 1e-8)
    w = np.maximum(xmax - xmin, 1e-8)
    cy, cx = ymin + h / 2, xmin + w / 2
    acy, acx, ah, aw = anchors_xywh.T
    return np.stack([(cy - acy) / ah * BOX_CODER_SCALES[0], (cx - acx) / aw * BOX_CODER_SCALES[1],
                     np.log(h / ah) * BOX_CODER_SCALES[2], np.log(w / aw) * BOX_CODER_SCALES[3]],
                    axis=1).astype(np.float32)


def decode_boxes(codes, anchors_xywh):
    """Inverse of encode_boxes (numpy or torch arrays) -> ltrb."""
    lib = np
    try:
        import torch
        if isinstance(codes, torch.Tensor):
            lib = torch
            anchors_xywh = torch.as_tensor(anchors_xywh, device=codes.device)
    except ImportError:  # pragma: no cover
        pass
    ty, tx, th, tw = (codes[..., i] / BOX_CODER_SCALES[i] for i in range(4))
    acy, acx, ah, aw = (anchors_xywh[..., i] for i in range(4))
    cy, cx = ty * ah + acy, tx * aw + acx
    h, w = lib.exp(th) * ah, lib.exp(tw) * aw
    return lib.stack([cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2], -1)


def encode_labels(gt_boxes: np.ndarray, gt_labels: np.ndarray):
    """-> (classes [8732, 1] float, boxes [8732, 4], num_matched)."""
    db = default_boxes()
    n_anchor = NUM_SSD_BOXES
    classes = np.zeros((n_anchor, 1), np.float32)
    boxes = np.zeros((n_anchor, 4), np.float32)
    if gt_boxes.shape[0] == 0:
        return classes, boxes, np.float32(0)
    iou = calc_iou(gt_boxes.astype(np.float32), db("ltrb"))  # [G, A]
    match = iou.argmax(axis=0)
    best = iou.max(axis=0)
    match = np.where(best >= MATCH_THRESHOLD, match, -1)
    # force-match every ground-truth box to its best anchor
    force = iou.argmax(axis=1)
    match[force] = np.arange(gt_boxes.shape[0])
    pos = match >= 0
    classes[pos, 0] = gt_labels.reshape(-1)[match[pos]]
    boxes[pos] = encode_boxes(gt_boxes[match[pos]], db("xywh")[pos])
    return classes, boxes, np.float32(pos.sum())


def ssd_crop(image: np.ndarray, boxes: np.ndarray, classes: np.ndarray,
             rng: np.random.Generator):
    """IoU-biased random crop; image float HWC in [0, 1], boxes ltrb."""
    while True:
        if rng.random() < P_NO_CROP_PER_PASS or boxes.shape[0] == 0:
            return _resize(image), boxes, classes
        wh = rng.uniform(0.3, 1.0, size=(NUM_CROP_PASSES, 2))
        lt = rng.uniform(0, 1, size=(NUM_CROP_PASSES, 2)) * (1 - wh)
        left, top = lt[:, 0], lt[:, 1]
        right, bottom = left + wh[:, 0], top + wh[:, 1]
        ltrb = np.stack([left, top, right, bottom], axis=1)
        min_iou = rng.choice(CROP_MIN_IOU_CHOICES)
        # boxes are (ymin, xmin, ymax, xmax); compare in the same order
        crop_yx = np.stack([top, left, bottom, right], axis=1)
        ious = calc_iou(crop_yx, boxes)
        yc = 0.5 * (boxes[:, 0] + boxes[:, 2])
        xc = 0.5 * (boxes[:, 1] + boxes[:, 3])
        masks = ((xc[None] > left[:, None]) & (xc[None] < right[:, None]) &
                 (yc[None] > top[:, None]) & (yc[None] < bottom[:, None]))
        valid = ((wh[:, 1] / wh[:, 0]) < 2) & (ious > min_iou).all(1) & masks.any(1)
        if not valid.any():
            continue
        k = int(np.nonzero(valid)[0][-1])
        m = masks[k]
        t, l_, b, r = crop_yx[k]
        fb = boxes[m]
        fb = np.stack([np.maximum(fb[:, 0], t), np.maximum(fb[:, 1], l_),
                       np.minimum(fb[:, 2], b), np.minimum(fb[:, 3], r)], axis=1)
        hh, ww = b - t, r - l_
        fb = np.stack([(fb[:, 0] - t) / hh, (fb[:, 1] - l_) / ww, (fb[:, 2] - t) / hh,
                       (fb[:, 3] - l_) / ww], axis=1)
        H, W = image.shape[:2]
        y0, y1 = int(t * H), max(int(math.ceil(b * H)), int(t * H) + 1)
        x0, x1 = int(l_ * W), max(int(math.ceil(r * W)), int(l_ * W) + 1)
        return _resize(image[y0:y1, x0:x1]), fb.astype(np.float32), classes[m]


def _resize(image: np.ndarray, size=IMAGE_SIZE) -> np.ndarray:
    from PIL import Image
    u8 = np.clip(image * 255.0, 0, 255).astype(np.uint8)
    out = Image.fromarray(u8).resize((size, size), Image.BILINEAR)
    return np.asarray(out, dtype=np.float32) / 255.0


def color_jitter(image, rng, brightness=0.125, contrast=0.5, saturation=0.5, hue=0.05):
    from ..data import preprocessing as pre
    img = pre.adjust_brightness(image, rng.uniform(-brightness, brightness))
    img = pre.adjust_contrast(img, rng.uniform(1 - contrast, 1 + contrast))
    img = pre.adjust_saturation(np.clip(img, 0, 1), rng.uniform(1 - saturation, 1 + saturation))
    img = pre.adjust_hue(img, rng.uniform(-hue, hue))
    return np.clip(img, 0.0, 1.0)


def normalize_image(image):
    return ((image - np.asarray(NORMALIZATION_MEAN, np.float32)) /
            np.asarray(NORMALIZATION_STD, np.float32)).astype(np.float32)


def decode_coco_example(record: bytes) -> Dict[str, np.ndarray]:
    """tf.Example in the object-detection layout -> dict of arrays."""
    from PIL import Image
    from .. import runtime
    f = runtime.parse_example(record)
    img = np.asarray(Image.open(io.BytesIO(f["image/encoded"][0])).convert("RGB"),
                     dtype=np.float32) / 255.0
    coords = [np.asarray(f.get("image/object/bbox/" + k, []), np.float32)
              for k in ("ymin", "xmin", "ymax", "xmax")]
    boxes = np.stack(coords, axis=1) if coords[0].size else np.zeros((0, 4), np.float32)
    labels = np.asarray(f.get("image/object/class/label", []), np.int64)
    labels = np.asarray([CLASS_MAP[int(x)] if 0 <= int(x) < len(CLASS_MAP) else -1
                         for x in labels], np.float32).reshape(-1, 1)
    sid = f.get("image/source_id", [b"0"])[0]
    return {"image": img, "boxes": boxes, "classes": labels,
            "source_id": int(sid) if sid.strip() else 0,
            "raw_shape": np.asarray(img.shape, np.int32)}


def preprocess(data, train: bool, rng: np.random.Generator):
    image, boxes, classes = data["image"], data["boxes"], data["classes"]
    keep = classes.reshape(-1) >= 0
    boxes, classes = boxes[keep], classes[keep]
    if train:
        image, boxes, classes = ssd_crop(image, boxes, classes, rng)
        if rng.random() < 0.5:
            image = image[:, ::-1]
            boxes = np.stack([boxes[:, 0], 1 - boxes[:, 3], boxes[:, 2], 1 - boxes[:, 1]], 1) \
                if boxes.shape[0] else boxes
        image = normalize_image(color_jitter(image, rng))
        enc_classes, enc_boxes, n = encode_labels(boxes, classes)
        return image, enc_boxes, enc_classes, n
    image = normalize_image(_resize(image))
    b = np.zeros((MAX_NUM_EVAL_BOXES, 4), np.float32)
    c = np.zeros((MAX_NUM_EVAL_BOXES, 1), np.float32)
    k = min(boxes.shape[0], MAX_NUM_EVAL_BOXES)
    b[:k], c[:k] = boxes[:k], classes[:k]
    return image, b, c, np.int32(data["source_id"]), data["raw_shape"]


def batched(pre, records, threads: int, train: bool):
    """Batches of (image, boxes, classes, num_matched) for training or
    (image, gt boxes, gt classes, source_id, raw_shape) for eval; records
    without boxes are skipped (as the reference's dataset filter)."""
    bs = pre.batch_size
    pool = ThreadPoolExecutor(max_workers=threads, thread_name_prefix="kfb-ssd")
    seeds = np.random.SeedSequence(pre.seed)
    try:
        while True:
            items = []
            while len(items) < bs:
                recs = [next(records) for _ in range(bs - len(items))]
                ss = seeds.spawn(1)[0].generate_state(len(recs))
                datas = list(pool.map(decode_coco_example, recs))
                datas = [d for d in datas if d["boxes"].shape[0] > 0]
                items += list(pool.map(
                    lambda a: preprocess(a[0], train, np.random.default_rng(int(a[1]))),
                    zip(datas, ss)))
            cols = list(zip(*items[:bs]))
            yield tuple(np.stack([np.asarray(x) for x in col]) for col in cols)
    finally:
        pool.shutdown(wait=False)
