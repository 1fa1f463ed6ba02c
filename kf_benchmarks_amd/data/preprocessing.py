"""Host-side input preprocessing for real data (role of tcb/preprocessing.py).

The reference builds tf.data graphs; here the pipeline is a pool of host
threads (JPEG decode, crop, resize and colour work in PIL/numpy release the
GIL) that fills whole NHWC batches, which :class:`..input_pipeline.
PrefetchInput` copies to the GPU one batch ahead on a side stream.

Batches leave the host either as ``uint8`` pixels (eval / no colour
distortion: 4x less PCIe traffic, the ``x/127.5-1`` normalization runs on the
GPU) or as normalized ``float32`` (colour-distorted or mean-subtracted data).

Semantics kept from the reference:

* ``parse_example_proto`` - tf.Example keys ``image/encoded``,
  ``image/class/label``, ``image/object/bbox/{ymin,xmin,ymax,xmax}``
  (tcb/preprocessing.py:27-72).
* ``train_image`` - distorted bounding-box crop (min_object_covered 0.1,
  aspect [0.75, 1.33], area [0.05, 1], 100 attempts), random left-right flip,
  resize, optional colour distortion in one of two orders chosen by batch
  position (tcb/preprocessing.py:192-307).
* ``eval_image`` - resize so the short side covers the target x1.15, then
  central crop (tcb/preprocessing.py:137-189).
* ``round_robin`` resize cycles nearest/bilinear/bicubic/area by batch
  position (tcb/preprocessing.py:83-113).
* ``normalized_image`` - ``x / 127.5 - 1`` (tcb/preprocessing.py:130-134).
* CIFAR-10: pad 4 + random crop + flip for training, centre crop for eval
  (tcb/preprocessing.py:653-737).
* ``TestImagePreprocessor`` - fixed fake batches rolled by ``shift_ratio``
  (tcb/preprocessing.py:896-974).
* LibriSpeech SequenceExample parsing + padded batches
  (tcb/preprocessing.py:977-1113).
* the ``official_models_imagenet`` preprocessor reproduces the
  tensorflow/models ResNet preprocessing (bbox crop / aspect-preserving resize
  to 256 + central crop, channel-mean subtraction), which the reference
  imports from the model garden (tcb/preprocessing.py:635-650).
"""

from __future__ import annotations

import glob
import itertools
import io
import math
import os
import random
from concurrent.futures import ThreadPoolExecutor
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np

from .. import cnn_util
from .. import runtime

try:  # PIL is the host JPEG codec (no TF); gate it so synthetic runs never need it
    from PIL import Image
except ImportError:  # pragma: no cover
    Image = None

# ------------------------------------------------------------------ parsing


def parse_example_proto(record: bytes):
    """-> (jpeg bytes, label int, bbox float32 [num_boxes, 4] (ymin, xmin,
    ymax, xmax), class text)."""
    f = runtime.parse_example(record)
    buf = f.get("image/encoded", [b""])
    label = f.get("image/class/label", [-1])
    text = f.get("image/class/text", [b""])
    coords = [f.get("image/object/bbox/" + k, []) for k in ("ymin", "xmin", "ymax", "xmax")]
    n = min(len(c) for c in coords)
    bbox = np.array([c[:n] for c in coords], dtype=np.float32).T.reshape(n, 4)
    return (buf[0] if buf else b""), int(label[0]), bbox, (text[0] if text else b"")


# ------------------------------------------------------------- image ops
_RESIZE_NAMES = ("nearest", "bilinear", "bicubic", "area")


def _pil_filter(name):
    return {"nearest": Image.NEAREST, "bilinear": Image.BILINEAR, "bicubic": Image.BICUBIC,
            "area": Image.BOX}[name]


def get_image_resize_method(resize_method: str, batch_position: int = 0) -> str:
    """Resize method name; ``round_robin`` picks by batch position."""
    if resize_method == "round_robin":
        return _RESIZE_NAMES[batch_position % len(_RESIZE_NAMES)]
    if resize_method not in _RESIZE_NAMES:
        raise ValueError("Unknown resize method %s" % resize_method)
    return resize_method


def jpeg_shape(buf: bytes) -> Tuple[int, int, int]:
    """(height, width, 3) from the JPEG header only."""
    with Image.open(io.BytesIO(buf)) as im:
        return im.size[1], im.size[0], 3


def decode_jpeg(buf: bytes, crop: Optional[Tuple[int, int, int, int]] = None) -> np.ndarray:
    """RGB uint8 [H, W, 3]. ``crop`` = (y, x, h, w) decodes only that window
    (``fuse_decode_and_crop``): PIL decodes at reduced DCT scale when the
    window is far smaller than the image, then crops."""
    im = Image.open(io.BytesIO(buf))
    if crop is not None:
        y, x, h, w = crop
        im = im.convert("RGB").crop((x, y, x + w, y + h))
    else:
        im = im.convert("RGB")
    return np.asarray(im, dtype=np.uint8)


def resize(image: np.ndarray, height: int, width: int, method: str) -> np.ndarray:
    if image.shape[0] == height and image.shape[1] == width:
        return image
    im = Image.fromarray(image)
    return np.asarray(im.resize((width, height), _pil_filter(method)), dtype=np.uint8)


def normalized_image(images):
    """[0, 255] -> [-1, 1]."""
    return images * (1.0 / 127.5) - 1.0


def sample_distorted_bounding_box(image_shape, bboxes, rng: np.random.Generator,
                                  min_object_covered=0.1, aspect_ratio_range=(0.75, 1.33),
                                  area_range=(0.05, 1.0), max_attempts=100):
    """(y, x, h, w) of a random crop covering at least ``min_object_covered``
    of one of ``bboxes`` (normalized ymin, xmin, ymax, xmax); the whole image
    if there are no boxes or no attempt succeeds (tf.image.
    sample_distorted_bounding_box with use_image_if_no_bounding_boxes)."""
    H, W = int(image_shape[0]), int(image_shape[1])
    boxes = np.asarray(bboxes, dtype=np.float32).reshape(-1, 4)
    if boxes.shape[0] == 0:
        boxes = np.array([[0.0, 0.0, 1.0, 1.0]], dtype=np.float32)
    min_area, max_area = area_range[0] * H * W, area_range[1] * H * W
    for _ in range(max_attempts):
        b = boxes[rng.integers(boxes.shape[0])]
        by0, bx0, by1, bx1 = b[0] * H, b[1] * W, b[2] * H, b[3] * W
        ar = rng.uniform(aspect_ratio_range[0], aspect_ratio_range[1])
        max_h = int(round(math.sqrt(max_area / ar)))
        if round(max_h * ar) > W:
            max_h = int((W + 0.5 - 1e-7) / ar)
        max_h = min(max_h, H)
        min_h = min(int(round(math.sqrt(min_area / ar))), max_h)
        if max_h < 1:
            continue
        h = int(rng.integers(max(min_h, 1), max_h + 1))
        w = int(round(h * ar))
        if w < 1 or w > W or h * w < min_area or h * w > max_area:
            continue
        y = int(rng.integers(0, H - h + 1))
        x = int(rng.integers(0, W - w + 1))
        iy = max(0.0, min(by1, y + h) - max(by0, y))
        ix = max(0.0, min(bx1, x + w) - max(bx0, x))
        barea = max((by1 - by0) * (bx1 - bx0), 1e-12)
        if iy * ix / barea < min_object_covered:
            continue
        return y, x, h, w
    return 0, 0, H, W


def _rgb_to_hsv(img):
    r, g, b = img[..., 0], img[..., 1], img[..., 2]
    mx = np.max(img, axis=-1)
    mn = np.min(img, axis=-1)
    d = mx - mn
    v = mx
    s = np.where(mx > 0, d / np.maximum(mx, 1e-12), 0.0)
    dd = np.maximum(d, 1e-12)
    h = np.where(mx == r, (g - b) / dd, np.where(mx == g, 2.0 + (b - r) / dd, 4.0 + (r - g) / dd))
    h = np.where(d > 0, (h / 6.0) % 1.0, 0.0)
    return h, s, v


def _hsv_to_rgb(h, s, v):
    h6 = (h % 1.0) * 6.0
    i = np.floor(h6).astype(np.int32) % 6
    f = h6 - np.floor(h6)
    p = v * (1 - s)
    q = v * (1 - s * f)
    t = v * (1 - s * (1 - f))
    r = np.choose(i, [v, q, p, p, t, v])
    g = np.choose(i, [t, v, v, q, p, p])
    b = np.choose(i, [p, p, t, v, v, q])
    return np.stack([r, g, b], axis=-1)


def adjust_brightness(img, delta):
    return img + delta


def adjust_contrast(img, factor):
    mean = img.mean(axis=(0, 1), keepdims=True)
    return (img - mean) * factor + mean


def adjust_saturation(img, factor):
    h, s, v = _rgb_to_hsv(img)
    return _hsv_to_rgb(h, np.clip(s * factor, 0.0, 1.0), v)


def adjust_hue(img, delta):
    h, s, v = _rgb_to_hsv(img)
    return _hsv_to_rgb((h + delta) % 1.0, s, v)


_NATIVE_COLOR = True  # (False: the numpy colour distortion, the tests' reference)


def distort_color(image, batch_position, rng: np.random.Generator, distort_color_in_yiq=False):
    """float image in [0, 1] -> colour-distorted, clipped to [0, 1].  Even
    batch positions: brightness, saturation/hue, contrast; odd: brightness,
    contrast, saturation/hue (hue first when ``distort_color_in_yiq``)."""
    img = adjust_brightness(image, rng.uniform(-32. / 255., 32. / 255.))

    def sat_hue(x):
        # saturation and hue act on independent HSV components, so one native
        # RGB->HSV->RGB pass applies both (the draw order stays the reference's)
        if distort_color_in_yiq:
            hue = rng.uniform(-0.2, 0.2)
            sat = rng.uniform(0.5, 1.5)
        else:
            sat = rng.uniform(0.5, 1.5)
            hue = rng.uniform(-0.2, 0.2)
        if _NATIVE_COLOR:
            from .. import runtime
            return runtime.adjust_saturation_hue(np.ascontiguousarray(x, dtype=np.float32),
                                                 sat, hue)
        return adjust_hue(adjust_saturation(x, sat), hue)

    if batch_position % 2 == 0:
        img = sat_hue(img)
        img = adjust_contrast(img, rng.uniform(0.5, 1.5))
    else:
        img = adjust_contrast(img, rng.uniform(0.5, 1.5))
        img = sat_hue(img)
    return np.clip(img, 0.0, 1.0)


def train_image(image_buffer, height, width, bbox, batch_position, resize_method, distortions,
                rng, distort_color_in_yiq=False, fuse_decode_and_crop=False):
    """-> uint8 [h, w, 3] (no distortions) or float32 [0, 255]."""
    shape = jpeg_shape(image_buffer)
    y, x, h, w = sample_distorted_bounding_box(shape, bbox, rng)
    if fuse_decode_and_crop:
        image = decode_jpeg(image_buffer, crop=(y, x, h, w))
    else:
        image = decode_jpeg(image_buffer)[y:y + h, x:x + w]
    if rng.random() < 0.5:
        image = image[:, ::-1]
    image = resize(np.ascontiguousarray(image), height, width,
                   get_image_resize_method(resize_method, batch_position))
    if distortions:
        f = image.astype(np.float32) / 255.0
        f = distort_color(f, batch_position, rng, distort_color_in_yiq)
        return (f * 255.0).astype(np.float32)
    return image


# False: decode every JPEG at full size (the DCT-domain 1/2-1/8 scaling below
# changes the pixels slightly; the crop keeps >= the output size)
_JPEG_DRAFT = True
AUG_PARAMS = 8  # per-image parameter row of the device augmentation (csrc/augment.hip)


def train_image_u8(image_buffer, height, width, bbox, batch_position, resize_method, distortions,
                   rng, distort_color_in_yiq=False, draft=None):
    """Host half of the train preprocessing when the colour distortions run on
    the device (csrc/augment.hip): decode + bbox crop + resize to uint8
    [height, width, 3], and the image's augmentation parameters
    (flip, brightness, saturation, hue, contrast, order, distort, 0), drawn
    from ``rng`` in train_image's order so both paths see the same randoms.
    The JPEG is opened once; with ``draft`` (default _JPEG_DRAFT) libjpeg
    decodes at the largest 1/2^k scale that keeps the crop >= the output."""
    im = Image.open(io.BytesIO(image_buffer))
    W0, H0 = im.size
    y, x, h, w = sample_distorted_bounding_box((H0, W0, 3), bbox, rng)
    flip = rng.random() < 0.5
    if _JPEG_DRAFT if draft is None else draft:
        scale = min(w / float(width), h / float(height))
        if scale >= 2.0:
            im.draft("RGB", (int(math.ceil(W0 / scale)), int(math.ceil(H0 / scale))))
            W1, H1 = im.size
            if (W1, H1) != (W0, H0):
                fx, fy = W1 / float(W0), H1 / float(H0)
                x, w = int(x * fx), max(1, int(round(w * fx)))
                y, h = int(y * fy), max(1, int(round(h * fy)))
    im = im.convert("RGB").crop((x, y, x + w, y + h))
    if (w, h) != (width, height):
        im = im.resize((width, height), _pil_filter(get_image_resize_method(resize_method,
                                                                           batch_position)))
    image = np.asarray(im, dtype=np.uint8)
    prm = np.zeros(AUG_PARAMS, dtype=np.float32)
    prm[0] = 1.0 if flip else 0.0
    if distortions:
        prm[1] = rng.uniform(-32. / 255., 32. / 255.)
        order = batch_position % 2
        if order == 0:
            if distort_color_in_yiq:
                prm[3], prm[2] = rng.uniform(-0.2, 0.2), rng.uniform(0.5, 1.5)
            else:
                prm[2], prm[3] = rng.uniform(0.5, 1.5), rng.uniform(-0.2, 0.2)
            prm[4] = rng.uniform(0.5, 1.5)
        else:
            prm[4] = rng.uniform(0.5, 1.5)
            if distort_color_in_yiq:
                prm[3], prm[2] = rng.uniform(-0.2, 0.2), rng.uniform(0.5, 1.5)
            else:
                prm[2], prm[3] = rng.uniform(0.5, 1.5), rng.uniform(-0.2, 0.2)
        prm[5] = float(order)
        prm[6] = 1.0
    return image, prm


def augment_reference(images_u8, params):
    """numpy reference of csrc/augment.hip: uint8 [N,H,W,3] + [N,8] params ->
    float32 [N,H,W,3] in [-1, 1] (the train_image + normalized_image result)."""
    out = []
    for img, p in zip(images_u8, params):
        f = img.astype(np.float32) / 255.0
        if p[0]:
            f = f[:, ::-1]
        if p[6]:
            f = f + p[1]

            def sat_hue(z):
                return adjust_hue(adjust_saturation(z, p[2]), p[3])
            if p[5] == 0:
                f = adjust_contrast(sat_hue(f), p[4])
            else:
                f = sat_hue(adjust_contrast(f, p[4]))
            f = np.clip(f, 0.0, 1.0)
        out.append(normalized_image(f * 255.0))
    return np.stack(out).astype(np.float32)


def eval_image(image, height, width, batch_position, resize_method):
    """Resize so both sides cover the target x1.15, then central crop."""
    ih, iw = image.shape[0], image.shape[1]
    ratio = max(height / float(ih), width / float(iw))
    rh, rw = int(ih * ratio * 1.15), int(iw * ratio * 1.15)
    image = resize(image, rh, rw, get_image_resize_method(resize_method, batch_position))
    top, left = (rh - height) // 2, (rw - width) // 2
    return image[top:top + height, left:left + width]


# --------------------------------------------------------- record sources
class RecordSource:
    """Endless stream of serialized records from TFRecord shards.

    Files are visited in an interleaved order (``cycle_length`` files open
    at once, one record from each in turn), starting ``shift_ratio`` of the
    way through the file list so that workers read different data first
    (RecordInput's shift_ratio).  Training adds a shuffle buffer.
    ``repeat_cached_sample`` repeats the first record forever (memory-speed
    IO emulation); ``use_caching`` keeps every record after the first epoch.
    """

    def __init__(self, files: Sequence[str], train: bool, shift_ratio: float = 0.0,
                 seed: int = 301, cycle_length: Optional[int] = None,
                 shuffle_buffer: int = 10000, repeat_cached_sample: bool = False,
                 use_caching: bool = False):
        if not files:
            raise ValueError("Found no files in --data_dir")
        files = list(files)
        k = int(len(files) * shift_ratio) % len(files)
        self.files = files[k:] + files[:k]
        self.train = train
        self.rng = random.Random(seed)
        self.cycle = max(1, cycle_length or 10)
        self.shuffle_buffer = shuffle_buffer if train else 0
        self.repeat_cached = repeat_cached_sample
        self.use_caching = use_caching
        self._cache: Optional[List[bytes]] = None

    def _one_epoch(self) -> Iterator[bytes]:
        if self._cache is not None:
            yield from self._cache
            return
        cache = [] if self.use_caching else None
        pending = list(self.files)
        active = []
        while pending or active:
            while pending and len(active) < self.cycle:
                active.append(runtime.tf_record_iterator(pending.pop(0)))
            nxt = []
            for it in active:
                rec = next(it, None)
                if rec is None:
                    continue
                nxt.append(it)
                if cache is not None:
                    cache.append(rec)
                yield rec
            active = nxt
        if cache is not None:
            self._cache = cache

    def __iter__(self) -> Iterator[bytes]:
        if self.repeat_cached:
            first = next(iter(self._one_epoch()))
            while True:
                yield first
        buf: List[bytes] = []
        while True:
            got = False
            for rec in self._one_epoch():
                got = True
                if not self.shuffle_buffer:
                    yield rec
                    continue
                if len(buf) < self.shuffle_buffer:
                    buf.append(rec)
                    continue
                i = self.rng.randrange(len(buf))
                out, buf[i] = buf[i], rec
                yield out
            if not got:
                raise ValueError("TFRecord files contain no records")
            if not self.train:
                continue
            # drain part of the buffer between epochs so small datasets move
            self.rng.shuffle(buf)


# -------------------------------------------------------------- preprocessors
def _default_threads():
    return max(1, min(16, (os.cpu_count() or 2) - 1))


class InputPreprocessor:
    """Base class: ``minibatch(dataset, subset, params, shift_ratio)``
    returns an iterator of host batches ``(images, labels)``."""

    def __init__(self, batch_size, output_shapes):
        self.batch_size = batch_size
        self.output_shapes = output_shapes

    def supports_datasets(self):
        return False

    def minibatch(self, dataset, subset, params, shift_ratio=-1):
        raise NotImplementedError("Must be implemented by subclass.")

    def parse_and_preprocess(self, value, batch_position):
        raise NotImplementedError("Must be implemented by subclass.")


class BaseImagePreprocessor(InputPreprocessor):
    def __init__(self, batch_size, output_shapes, num_splits=1, dtype=np.float32, train=True,
                 distortions=False, resize_method="bilinear", shift_ratio=-1,
                 summary_verbosity=0, distort_color_in_yiq=True, fuse_decode_and_crop=True):
        super().__init__(batch_size, output_shapes)
        image_shape = output_shapes[0]
        self.height, self.width, self.depth = image_shape[1], image_shape[2], image_shape[3]
        self.num_splits = num_splits
        self.dtype = dtype
        self.train = train
        self.resize_method = resize_method
        self.shift_ratio = shift_ratio
        self.distortions = distortions
        self.distort_color_in_yiq = distort_color_in_yiq
        self.fuse_decode_and_crop = fuse_decode_and_crop
        if self.batch_size % self.num_splits != 0:
            raise ValueError(("batch_size must be a multiple of num_splits: "
                              "batch_size %d, num_splits: %d") % (self.batch_size,
                                                                  self.num_splits))
        self.batch_size_per_split = self.batch_size // self.num_splits
        self.summary_verbosity = summary_verbosity
        self.seed = 301

    def supports_datasets(self):
        return True

    def parse_and_preprocess(self, value, batch_position, rng=None):
        image_buffer, label, bbox, _ = parse_example_proto(value)
        rng = rng if rng is not None else np.random.default_rng()
        return self.preprocess(image_buffer, bbox, batch_position, rng), label

    def preprocess(self, image_buffer, bbox, batch_position, rng):
        raise NotImplementedError("Must be implemented by subclass.")

    # ---- host batching
    def record_source(self, dataset, subset, params, shift_ratio):
        files = sorted(glob.glob(dataset.tf_record_pattern(subset)))
        if not files:
            raise ValueError("Found no files in --data_dir matching: %s"
                             % dataset.tf_record_pattern(subset))
        return RecordSource(
            files, self.train, max(shift_ratio, 0.0), seed=self.seed,
            cycle_length=getattr(params, "datasets_parallel_interleave_cycle_length", None),
            repeat_cached_sample=getattr(params, "datasets_repeat_cached_sample", False),
            use_caching=getattr(params, "datasets_use_caching", False))

    def minibatch(self, dataset, subset, params, shift_ratio=-1):
        if shift_ratio < 0:
            shift_ratio = self.shift_ratio
        src = iter(self.record_source(dataset, subset, params, shift_ratio))
        threads = getattr(params, "datasets_num_private_threads", None) or _default_threads()
        return _batched(self, src, threads)


class JpegBatch:
    """One train batch in GPU-reconstruction form (ops/jpeg.decode): the
    packed coefficient blocks of every crop plus descriptors, the images the
    host decoded itself, augmentation parameters and labels - views of one
    pinned ring slot, which the consumer marks with ``slot.ev`` once its
    device copies are enqueued (the producer waits for that before refilling
    the slot)."""
    __slots__ = ("slot", "n", "nblocks", "hosted", "height", "width", "crop_pixels")

    def __init__(self, slot, n, nblocks, hosted, height, width, crop_pixels=-1):
        self.slot, self.n, self.nblocks, self.hosted = slot, n, nblocks, hosted
        self.height, self.width, self.crop_pixels = height, width, crop_pixels


class _JpegSlot:
    # arena blocks per image of the batch (shared: large crops borrow from
    # small ones; an image that does not fit is decoded on the host)
    BLOCKS_PER_IMAGE = 4096

    def __init__(self, n, height, width):
        import threading
        import torch
        from .. import runtime
        pin = torch.cuda.is_available()

        def buf(shape, dtype):
            t = torch.empty(shape, dtype=dtype)
            return t.pin_memory() if pin else t
        self.descs = buf((n * runtime.jpeg_desc_bytes(),), torch.uint8)
        self.blocks = buf((n * self.BLOCKS_PER_IMAGE, 64), torch.int16)
        self.images = buf((n, height, width, 3), torch.uint8)
        self.params = buf((n, 8), torch.float32)
        self.labels = buf((n,), torch.int32)
        self.ev = None
        # set while no yielded batch lives in the slot: a batch waiting in a
        # prefetch queue (no copy enqueued yet) keeps it cleared, so the
        # producer can never refill a slot whose batch is still queued
        self._free = threading.Event()
        self._free.set()

    def claim(self):
        self._free.clear()

    def release(self, ev=None):
        """The consumer enqueued its device copies of this slot (``ev`` fires
        when they are done), or dropped the batch (ev None)."""
        self.ev = ev
        self._free.set()

    def wait_free(self):
        self._free.wait()
        if self.ev is not None:
            self.ev.synchronize()
            self.ev = None


# pinned ring slots by default; make_batch_iterator sizes the ring from the
# consumer's real lookahead (prefetch queue + ImageProducer groups)
_JPEG_RING = 6


def jpeg_ring_slots(prefetch_depth: int, batch_group_size: int) -> int:
    """Slots so the producer is never blocked by the ring before it is by the
    queue: every batch the queue (depth) or an ImageProducer (up to 3G-1
    ahead) can hold, plus the one being copied and the one being filled."""
    g = max(int(batch_group_size or 1), 1)
    ahead = max(int(prefetch_depth), 1) + (3 * g if g > 1 else 0)
    return max(_JPEG_RING, ahead + 2)


def _batched(pre, records: Iterator[bytes], threads: int):
    """Yields (images [bs,h,w,3] uint8|float32, labels int32 [bs]) using a
    thread pool; the per-image RNG depends only on (batch, position) so the
    output is deterministic regardless of thread scheduling."""
    bs = pre.batch_size
    base = np.random.SeedSequence(pre.seed)
    if getattr(pre, "gpu_jpeg", False) and _NATIVE_PIPE and runtime.coef_pipeline_available():
        # host threads entropy-decode only; reconstruction on the GPU
        pipe = runtime.ImagePipe(threads, pre.height, pre.width, pre.distortions,
                                 pre.distort_color_in_yiq)
        ring = [_JpegSlot(bs, pre.height, pre.width)
                for _ in range(getattr(pre, "jpeg_ring", _JPEG_RING))]
        try:
            for k in itertools.count():
                recs = [next(records) for _ in range(bs)]
                seeds = base.spawn(1)[0].generate_state(bs, dtype=np.uint64)
                slot = ring[k % len(ring)]
                slot.wait_free()
                slot.claim()
                nblocks, hosted, bad = pipe.run_coef(recs, seeds, slot)
                if bad > 0:
                    raise ValueError("%d of %d image records in this batch could not be "
                                     "decoded (corrupt TFRecord / JPEG data)" % (bad, bs))
                yield JpegBatch(slot, bs, nblocks, hosted, pre.height, pre.width,
                                pipe.crop_pixels)
        finally:
            pipe.close()
    if getattr(pre, "device_augment", False) and _NATIVE_PIPE and runtime.ImagePipe.available():
        # every per-image step in native threads (csrc/runtime/kfb_images.cpp)
        pipe = runtime.ImagePipe(threads, pre.height, pre.width, pre.distortions,
                                 pre.distort_color_in_yiq)
        try:
            while True:
                recs = [next(records) for _ in range(bs)]
                seeds = base.spawn(1)[0].generate_state(bs, dtype=np.uint64)
                imgs, prms, labels, bad = pipe.run(recs, seeds)
                if bad > 0:
                    # the native decoder substitutes a grey image with label -1
                    # for a record it cannot parse; the PIL path raises on the
                    # same record, and a -1 label would poison the loss
                    raise ValueError("%d of %d image records in this batch could not be "
                                     "decoded (corrupt TFRecord / JPEG data)" % (bad, bs))
                yield imgs, labels, prms
        finally:
            pipe.close()
    pool = ThreadPoolExecutor(max_workers=threads, thread_name_prefix="kfb-input")
    try:
        while True:
            recs = [next(records) for _ in range(bs)]
            seeds = base.spawn(1)[0].generate_state(bs)
            results = list(pool.map(
                lambda i: pre.parse_and_preprocess(recs[i], i, np.random.default_rng(int(seeds[i]))),
                range(bs)))
            if getattr(pre, "device_augment", False):
                # (uint8 images, params) per image: colour work on the device
                imgs = np.stack([r[0][0] for r in results])
                prms = np.stack([r[0][1] for r in results])
                labels = np.asarray([r[1] for r in results], dtype=np.int32)
                yield imgs, labels, prms
                continue
            imgs = [r[0] for r in results]
            floaty = any(im.dtype != np.uint8 for im in imgs)
            out = np.stack([im.astype(np.float32) if floaty else im for im in imgs])
            if floaty and not getattr(pre, "normalized_output", False):
                out = normalized_image(out).astype(np.float32)
            labels = np.asarray([r[1] for r in results], dtype=np.int32)
            yield out, labels
    finally:
        pool.shutdown(wait=False)


class RecordInputImagePreprocessor(BaseImagePreprocessor):
    """The default ImageNet-style pipeline (tcb/preprocessing.py:551-632)."""

    # set by make_batch_iterator for GPU consumers: train batches come out as
    # (uint8 images, labels, augmentation params) and csrc/augment.hip does
    # the flip, colour distortions and scaling after the copy
    device_augment = False

    def preprocess(self, image_buffer, bbox, batch_position, rng):
        if self.train and self.device_augment:
            return train_image_u8(image_buffer, self.height, self.width, bbox, batch_position,
                                  self.resize_method, self.distortions, rng,
                                  self.distort_color_in_yiq)
        if self.train:
            return train_image(image_buffer, self.height, self.width, bbox, batch_position,
                               self.resize_method, self.distortions, rng,
                               self.distort_color_in_yiq, self.fuse_decode_and_crop)
        image = decode_jpeg(image_buffer)
        return eval_image(image, self.height, self.width, batch_position, self.resize_method)


_CHANNEL_MEANS = np.array([123.68, 116.78, 103.94], dtype=np.float32)
_RESIZE_MIN = 256


class ImagenetPreprocessor(RecordInputImagePreprocessor):
    """tensorflow/models ResNet ImageNet preprocessing: train = bbox crop +
    flip + bilinear resize; eval = aspect-preserving resize of the short side
    to 256 + central crop; both subtract the channel means (no scaling)."""

    normalized_output = True

    def preprocess(self, image_buffer, bbox, batch_position, rng):
        if self.train:
            shape = jpeg_shape(image_buffer)
            y, x, h, w = sample_distorted_bounding_box(shape, bbox, rng)
            image = decode_jpeg(image_buffer, crop=(y, x, h, w))
            if rng.random() < 0.5:
                image = image[:, ::-1]
            image = resize(np.ascontiguousarray(image), self.height, self.width, "bilinear")
        else:
            image = decode_jpeg(image_buffer)
            ih, iw = image.shape[:2]
            scale = _RESIZE_MIN / float(min(ih, iw))
            image = resize(image, int(round(ih * scale)), int(round(iw * scale)), "bilinear")
            top = (image.shape[0] - self.height) // 2
            left = (image.shape[1] - self.width) // 2
            image = image[top:top + self.height, left:left + self.width]
        return image.astype(np.float32) - _CHANNEL_MEANS


class Cifar10ImagePreprocessor(BaseImagePreprocessor):
    """In-memory CIFAR-10: shuffled batches; training distortion = zero-pad
    to 40x40, random 32x32 crop, random flip."""

    def _distort_image(self, image, rng):
        h, w = self.height, self.width
        padded = np.zeros((h + 8, w + 8, image.shape[2]), dtype=image.dtype)
        padded[4:4 + h, 4:4 + w] = image
        y = int(rng.integers(0, 9))
        x = int(rng.integers(0, 9))
        out = padded[y:y + h, x:x + w]
        if rng.random() < 0.5:
            out = out[:, ::-1]
        return out

    def _eval_image(self, image):
        return image[:self.height, :self.width]

    def preprocess(self, raw_image, rng=None):
        rng = rng if rng is not None else np.random.default_rng()
        if self.train and self.distortions:
            image = self._distort_image(raw_image, rng)
        else:
            image = self._eval_image(raw_image)
        return normalized_image(image.astype(np.float32))

    def minibatch(self, dataset, subset, params, shift_ratio=-1):
        del shift_ratio
        images, labels = dataset.read_data_files(subset)
        images = images.reshape(-1, dataset.depth, dataset.height, dataset.width)
        images = images.transpose(0, 2, 3, 1)  # NHWC
        rng = np.random.default_rng(self.seed)
        n = images.shape[0]
        bs = self.batch_size

        def gen():
            order = rng.permutation(n)
            pos = 0
            while True:
                if pos + bs > n:
                    order = rng.permutation(n)
                    pos = 0
                idx = order[pos:pos + bs]
                pos += bs
                out = np.stack([self.preprocess(images[i], rng) for i in idx])
                yield out.astype(np.float32), labels[idx].astype(np.int32)
        return gen()


class TestImagePreprocessor(BaseImagePreprocessor):
    """Serves fixed fake data (``set_fake_data``) in order, rolled by
    ``shift_ratio`` so each worker starts at a different batch."""

    def __init__(self, batch_size, output_shapes, num_splits=1, dtype=np.float32, train=None,
                 distortions=None, resize_method=None, shift_ratio=0, summary_verbosity=0,
                 distort_color_in_yiq=False, fuse_decode_and_crop=False):
        super().__init__(batch_size, output_shapes, num_splits, dtype, train, distortions,
                         resize_method, shift_ratio, summary_verbosity=summary_verbosity,
                         distort_color_in_yiq=distort_color_in_yiq,
                         fuse_decode_and_crop=fuse_decode_and_crop)
        self.expected_subset = None

    def set_fake_data(self, fake_images, fake_labels):
        assert len(fake_images.shape) == 4
        assert len(fake_labels.shape) == 1
        assert fake_images.shape[0] == fake_labels.shape[0]
        assert fake_images.shape[0] % self.batch_size == 0
        self.fake_images = fake_images
        self.fake_labels = fake_labels

    def minibatch(self, dataset, subset, params, shift_ratio=0):
        del dataset, params
        if not hasattr(self, "fake_images") or not hasattr(self, "fake_labels"):
            raise ValueError("Must call set_fake_data() before calling minibatch "
                             "on TestImagePreprocessor")
        if self.expected_subset is not None:
            assert subset == self.expected_subset
        shift_ratio = shift_ratio or self.shift_ratio
        imgs = cnn_util.roll_numpy_batches(self.fake_images, self.batch_size, shift_ratio)
        labs = cnn_util.roll_numpy_batches(self.fake_labels, self.batch_size, shift_ratio)
        bs = self.batch_size

        def gen():
            n = imgs.shape[0] // bs
            i = 0
            while True:
                k = i % n
                i += 1
                yield (normalized_image(imgs[k * bs:(k + 1) * bs].astype(np.float32)),
                       labs[k * bs:(k + 1) * bs].astype(np.int32))
        return gen()


class COCOPreprocessor(BaseImagePreprocessor):
    """SSD300 inputs from COCO TFRecords (object-detection Example layout):
    train = SSD random crop + flip + colour jitter + normalize + box encoding
    against the default boxes; eval = resize to 300 + normalize + padded
    ground truth (see models/ssd_dataloader.py)."""

    normalized_output = True

    def parse_and_preprocess(self, value, batch_position, rng=None):
        from ..models import ssd_dataloader as sd
        rng = rng if rng is not None else np.random.default_rng()
        data = sd.decode_coco_example(value)
        return sd.preprocess(data, self.train, rng)

    def minibatch(self, dataset, subset, params, shift_ratio=-1):
        from ..models import ssd_dataloader as sd
        src = iter(self.record_source(dataset, subset, params, max(shift_ratio, 0)))
        threads = getattr(params, "datasets_num_private_threads", None) or _default_threads()
        return sd.batched(self, src, threads, self.train)


class LibrispeechPreprocessor(InputPreprocessor):
    """DeepSpeech2 inputs: SequenceExample with context ``labels`` (int64
    list), ``input_length``, ``label_length`` and a feature list
    ``features`` of 161-float frames; padded to the model's input shapes."""

    def __init__(self, batch_size, output_shapes, num_splits=1, dtype=np.float32, train=True,
                 **kwargs):
        del kwargs
        super().__init__(batch_size, output_shapes)
        self.num_splits = num_splits
        self.dtype = dtype
        self.is_train = train
        if self.batch_size % self.num_splits != 0:
            raise ValueError(("batch_size must be a multiple of num_splits: "
                              "batch_size %d, num_splits: %d") % (self.batch_size,
                                                                  self.num_splits))
        self.batch_size_per_split = self.batch_size // self.num_splits

    def supports_datasets(self):
        return True

    def parse_and_preprocess(self, value, batch_position=0):
        ctx, lists = runtime.parse_sequence_example(value)
        frames = lists.get("features", [])
        feats = np.asarray(frames, dtype=np.float32).reshape(len(frames), -1, 1)
        labels = np.asarray(ctx.get("labels", []), dtype=np.int32)
        return (feats, labels, np.array([ctx.get("input_length", [len(frames)])[0]], np.int32),
                np.array([ctx.get("label_length", [len(labels)])[0]], np.int32))

    def minibatch(self, dataset, subset, params, shift_ratio=-1):
        files = sorted(glob.glob(dataset.tf_record_pattern(subset)))
        src = iter(RecordSource(files, self.is_train, max(shift_ratio, 0.0),
                                repeat_cached_sample=params.datasets_repeat_cached_sample))
        shapes = self.output_shapes
        bs = self.batch_size

        def gen():
            while True:
                items = [self.parse_and_preprocess(next(src)) for _ in range(bs)]
                feats = np.zeros([bs] + list(shapes[0][1:]), dtype=np.float32)
                labels = np.zeros([bs] + list(shapes[1][1:]), dtype=np.int32)
                for i, (f, l, _, _) in enumerate(items):
                    n = min(f.shape[0], feats.shape[1])
                    feats[i, :n] = f[:n].reshape(n, *feats.shape[2:])
                    m = min(l.shape[0], labels.shape[1])
                    labels[i, :m] = l[:m]
                ilen = np.concatenate([it[2] for it in items])
                llen = np.concatenate([it[3] for it in items])
                yield feats, labels, ilen, llen
        return gen()


SUPPORTED_INPUT_PREPROCESSORS = {
    "imagenet": {
        "default": RecordInputImagePreprocessor,
        "official_models_imagenet": ImagenetPreprocessor,
    },
    "cifar10": {"default": Cifar10ImagePreprocessor},
    "librispeech": {"default": LibrispeechPreprocessor},
    "coco": {"default": COCOPreprocessor},
}


def get_preprocessor(bench, subset):
    """Instantiates the dataset's preprocessor for one worker / device."""
    params = bench.params
    dataset = bench.dataset
    cls = dataset.get_input_preprocessor(params.input_preprocessor or "default")
    train = subset == "train"
    shapes = bench.model.get_input_shapes(subset)
    shift = bench.task_index / float(max(bench.num_replicas, 1))
    bs = bench.local_batch_size
    if cls is LibrispeechPreprocessor:
        return cls(bs, shapes, 1, np.float32, train)
    return cls(bs, shapes, 1, np.float32, train, params.distortions,
               params.resize_method, shift_ratio=shift,
               summary_verbosity=params.summary_verbosity,
               distort_color_in_yiq=params.distort_color_in_yiq,
               fuse_decode_and_crop=params.fuse_decode_and_crop)


# False: with device augmentation, decode/crop/resize on Python threads over
# PIL instead of the native pipeline
_NATIVE_PIPE = True
# False: the whole train preprocessing on the host threads
_DEVICE_AUGMENT = True


def make_batch_iterator(bench, subset="train"):
    pre = get_preprocessor(bench, subset)
    if (type(pre) is RecordInputImagePreprocessor and pre.train and _DEVICE_AUGMENT
            and getattr(bench, "device", None) is not None and bench.device.type == "cuda"):
        pre.device_augment = True
        # host threads entropy-decode only, reconstruction on the GPU
        # (csrc/jpeg.hip); KFB_GPU_JPEG=0: they decode the whole JPEG
        pre.gpu_jpeg = os.environ.get("KFB_GPU_JPEG", "1") != "0"
        pre.jpeg_ring = jpeg_ring_slots(max(bench.params.datasets_prefetch_buffer_size, 1) + 1,
                                        bench.params.batch_group_size)
    shift = bench.task_index / float(max(bench.num_replicas, 1))
    return pre.minibatch(bench.dataset, subset, bench.params, shift_ratio=shift)
