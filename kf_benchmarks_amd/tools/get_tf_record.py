"""Convert an image-folder dataset (``<dir>/<class>/<image>``, e.g.
tiny-imagenet) into sharded ImageNet-layout TFRecords
``<prefix>-%05d-of-%05d`` (role of tcb/get_tf_record.py).  Labels are the
sorted class-directory index; records carry ``image/encoded``,
``image/format``, ``image/class/label``, ``image/height``, ``image/width``.

usage: python -m kf_benchmarks_amd.tools.get_tf_record --train_dir D
       --val_dir D --output_dir O [--num_shards 1024] [--seed 0]
"""

from __future__ import annotations

import argparse
import os
import random
from typing import List, Tuple

from .. import runtime


def list_images(image_dir: str) -> List[Tuple[str, int]]:
    classes = sorted(d for d in os.listdir(image_dir)
                     if os.path.isdir(os.path.join(image_dir, d)))
    label = {c: i for i, c in enumerate(classes)}
    out = []
    for c in classes:
        for root, _, files in os.walk(os.path.join(image_dir, c)):
            for f in sorted(files):
                if f.lower().endswith((".jpg", ".jpeg", ".png")):
                    out.append((os.path.join(root, f), label[c]))
    return out


def image_record(path: str, label: int) -> bytes:
    from PIL import Image
    with open(path, "rb") as fh:
        data = fh.read()
    with Image.open(path) as im:
        width, height = im.size
        fmt = (im.format or "JPEG").lower().encode()
    return runtime.make_example({"image/encoded": [data], "image/format": [fmt],
                                 "image/class/label": [label], "image/height": [height],
                                 "image/width": [width]})


def convert_dataset(image_dir: str, output_path: str, num_shards: int = 1024, seed: int = 0):
    items = list_images(image_dir)
    random.Random(seed).shuffle(items)
    n = len(items)
    num_shards = max(1, min(num_shards, n)) if n else 1
    per = n // num_shards
    written = []
    for shard in range(num_shards):
        name = "%s-%05d-of-%05d" % (output_path, shard, num_shards)
        lo = shard * per
        hi = n if shard == num_shards - 1 else (shard + 1) * per
        with runtime.TFRecordWriter(name) as w:
            for path, label in items[lo:hi]:
                w.write(image_record(path, label))
        written.append(name)
    return written


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--train_dir")
    ap.add_argument("--val_dir")
    ap.add_argument("--output_dir", required=True)
    ap.add_argument("--num_shards", type=int, default=1024)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    os.makedirs(a.output_dir, exist_ok=True)
    for d, name in ((a.train_dir, "train"), (a.val_dir, "validation")):
        if d:
            for f in convert_dataset(d, os.path.join(a.output_dir, name), a.num_shards, a.seed):
                print("Finished writing %s" % f)


if __name__ == "__main__":
    main()
