"""Black/white JPEG TFRecord fixtures (role of
tcb/test_data/tfrecord_image_generator.py).

Training images are black and validation images white, each of random size
in [30, 299]^2, one bounding box (0.1, 0.1, 0.9, 0.9), label = index %
num_classes, written as ``<subset>-%05d-of-%05d`` shards of tf.Example
records with the ImageNet key layout.
"""

from __future__ import annotations

import io
import os
import random

import numpy as np

from .. import runtime


def encode_jpeg(image: np.ndarray, quality: int = 100) -> bytes:
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(image).save(buf, format="JPEG", quality=quality)
    return buf.getvalue()


def image_example(filename, image_buffer, label, synset, human, bbox, height, width) -> bytes:
    """tf.Example with the ImageNet TFRecord keys; bbox boxes are
    [xmin, ymin, xmax, ymax]."""
    xmin = [float(b[0]) for b in bbox]
    ymin = [float(b[1]) for b in bbox]
    xmax = [float(b[2]) for b in bbox]
    ymax = [float(b[3]) for b in bbox]
    return runtime.make_example({
        "image/height": [height], "image/width": [width],
        "image/colorspace": [b"RGB"], "image/channels": [3],
        "image/class/label": [label], "image/class/synset": [synset.encode()],
        "image/class/text": [human.encode()],
        "image/object/bbox/xmin": xmin, "image/object/bbox/xmax": xmax,
        "image/object/bbox/ymin": ymin, "image/object/bbox/ymax": ymax,
        "image/object/bbox/label": [label] * len(xmin),
        "image/format": [b"JPEG"], "image/filename": [os.path.basename(filename).encode()],
        "image/encoded": [image_buffer],
    })


def _process_dataset(output_directory, num_classes, name, num_images, num_shards, rng):
    per_shard = num_images // num_shards
    value = 0 if name == "train" else 255
    for shard in range(num_shards):
        path = os.path.join(output_directory, "%s-%.5d-of-%.5d" % (name, shard, num_shards))
        with runtime.TFRecordWriter(path) as w:
            for i in range(per_shard):
                index = shard * per_shard + i
                h, w_ = rng.randint(30, 299), rng.randint(30, 299)
                jpeg = encode_jpeg(np.full((h, w_, 3), value, np.uint8))
                w.write(image_example("%s_%d_%d" % (name, shard, i), jpeg, index % num_classes,
                                      str(index), name, [[0.1, 0.1, 0.9, 0.9]], h, w_))


def write_black_and_white_tfrecord_data(output_directory, num_classes, num_train_images=512,
                                        num_validation_images=128, train_shards=8,
                                        validation_shards=2, seed=0):
    os.makedirs(output_directory, exist_ok=True)
    rng = random.Random(seed)
    _process_dataset(output_directory, num_classes, "validation", num_validation_images,
                     validation_shards, rng)
    _process_dataset(output_directory, num_classes, "train", num_train_images, train_shards, rng)
