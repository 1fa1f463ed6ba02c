#!/usr/bin/env python3
"""ImageNet-like TFRecords for the real-data input benchmark: JPEGs of
ImageNet's typical size (300-600 px a side, quality 90, ~50-150 KB each)
with smooth content plus noise (so the encoded size and the decode cost are
realistic, unlike the tiny black/white test fixtures), one bounding box per
image, 1001 classes, ``train-%05d-of-%05d`` shards.
usage: make_imagenet_like.py <outdir> [num_images] [shards]"""
import os
import random
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from kf_benchmarks_amd import runtime  # noqa: E402
from kf_benchmarks_amd.data.test_data import encode_jpeg, image_example  # noqa: E402


def main():
    out = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    shards = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    os.makedirs(out, exist_ok=True)
    rng = random.Random(0)
    nrng = np.random.default_rng(0)
    total = 0
    per = n // shards
    for s in range(shards):
        path = os.path.join(out, "train-%05d-of-%05d" % (s, shards))
        with runtime.TFRecordWriter(path) as w:
            for i in range(per):
                h, wd = rng.randint(300, 600), rng.randint(300, 600)
                yy, xx = np.mgrid[0:h, 0:wd].astype(np.float32)
                img = np.stack([127 + 100 * np.sin(xx / rng.uniform(8, 40) + c) *
                                np.cos(yy / rng.uniform(8, 40)) for c in range(3)], -1)
                img += nrng.normal(0, 12, img.shape)
                jpeg = encode_jpeg(np.clip(img, 0, 255).astype(np.uint8), quality=90)
                total += len(jpeg)
                idx = s * per + i
                w.write(image_example("img_%d" % idx, jpeg, idx % 1000 + 1, "n%08d" % idx, "x",
                                      [[0.05, 0.05, 0.95, 0.95]], h, wd))
    print("wrote %d images, %.1f KB average JPEG" % (per * shards, total / 1024.0 / (per * shards)))


if __name__ == "__main__":
    main()
