"""Probe a local ImageNet copy (role of tcb/get_imagenet.py, which loads a
tfds ImageNet subset to check that the data is reachable).

There is no dataset download here: the tool inspects ``--data_dir`` in the
layout ``--data_dir`` consumers expect (datasets.ImagenetDataset):
TFRecord shards ``train-%05d-of-%05d`` / ``validation-%05d-of-%05d``, or an
image-folder tree ``<dir>/<class>/<image>`` (convertible with
tools.get_tf_record).  It reports the shard and class counts, counts the
records of up to ``--sample_shards`` shards through the native TFRecord
reader (CRC-checked) and decodes the first example of each.

usage: python -m kf_benchmarks_amd.tools.get_imagenet --data_dir D [--sample_shards 2]
"""

from __future__ import annotations

import argparse
import glob
import os
import sys

from .. import runtime


def probe(data_dir: str, sample_shards: int = 2) -> dict:
    out = {"data_dir": data_dir, "subsets": {}}
    for subset in ("train", "validation"):
        shards = sorted(glob.glob(os.path.join(data_dir, "%s-*-of-*" % subset)))
        info = {"shards": len(shards), "sampled_records": 0, "first_example": None}
        for path in shards[:sample_shards]:
            for i, rec in enumerate(runtime.tf_record_iterator(path)):
                if info["first_example"] is None:
                    ex = runtime.parse_example(rec)
                    info["first_example"] = {
                        k: (len(v[0]) if k == "image/encoded" else v[:1])
                        for k, v in ex.items() if k.startswith("image/")}
                info["sampled_records"] += 1
        out["subsets"][subset] = info
    classes = [d for d in os.listdir(data_dir) if os.path.isdir(os.path.join(data_dir, d))]
    out["image_folder_classes"] = len(classes)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--data_dir", required=True)
    ap.add_argument("--sample_shards", type=int, default=2)
    a = ap.parse_args(argv)
    if not os.path.isdir(a.data_dir):
        print("no such directory: %s" % a.data_dir, file=sys.stderr)
        return 1
    res = probe(a.data_dir, a.sample_shards)
    for subset, info in res["subsets"].items():
        print("%-10s shards: %d  records in first %d shard(s): %d  first example: %s"
              % (subset, info["shards"], min(a.sample_shards, info["shards"]),
                 info["sampled_records"], info["first_example"]))
    print("image-folder classes: %d" % res["image_folder_classes"])
    ok = any(i["shards"] for i in res["subsets"].values()) or res["image_folder_classes"]
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
