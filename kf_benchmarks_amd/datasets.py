"""Dataset descriptors (role of tcb/datasets.py:41-251).

Synthetic data is used iff ``data_dir`` is unset (``use_synthetic_gpu_inputs``).
Real data: TFRecord shards ``<subset>-*-of-*`` of tf.Example records
(ImageNet/COCO), CIFAR-10 binary batches, LibriSpeech TFRecords.
"""

from __future__ import annotations

import glob
import os

import numpy as np

IMAGENET_NUM_TRAIN_IMAGES = 1281167
IMAGENET_NUM_VAL_IMAGES = 50000
COCO_NUM_TRAIN_IMAGES = 118287
COCO_NUM_VAL_IMAGES = 4952


class Dataset:
    def __init__(self, name, data_dir=None, queue_runner_required=False, num_classes=None):
        self.name = name
        self.data_dir = data_dir
        self._queue_runner_required = queue_runner_required
        self._num_classes = num_classes

    def tf_record_pattern(self, subset):
        return os.path.join(self.data_dir, "%s-*-of-*" % subset)

    def tf_record_files(self, subset):
        return sorted(glob.glob(self.tf_record_pattern(subset)))

    @property
    def num_classes(self):
        return self._num_classes

    @num_classes.setter
    def num_classes(self, val):
        self._num_classes = val

    def num_examples_per_epoch(self, subset="train"):
        raise NotImplementedError

    def __str__(self):
        return self.name

    def get_input_preprocessor(self, input_preprocessor="default"):
        assert not self.use_synthetic_gpu_inputs()
        from .data import preprocessing
        return preprocessing.SUPPORTED_INPUT_PREPROCESSORS[self.name][input_preprocessor]

    def queue_runner_required(self):
        return self._queue_runner_required

    def use_synthetic_gpu_inputs(self):
        return not self.data_dir


class LibrispeechDataset(Dataset):
    def __init__(self, data_dir=None):
        super().__init__("librispeech", data_dir, num_classes=29)

    def tf_record_pattern(self, subset):
        if subset == "train":
            return os.path.join(self.data_dir, "train-clean-*.tfrecords")
        if subset == "validation":
            return os.path.join(self.data_dir, "test-clean.tfrecords")
        return ""

    def num_examples_per_epoch(self, subset="train"):
        return 2


class ImageDataset(Dataset):
    def __init__(self, name, height, width, depth=None, data_dir=None,
                 queue_runner_required=False, num_classes=1001):
        super().__init__(name, data_dir, queue_runner_required, num_classes)
        self.height, self.width, self.depth = height, width, depth or 3


class ImagenetDataset(ImageDataset):
    def __init__(self, data_dir=None):
        super().__init__("imagenet", 300, 300, data_dir=data_dir)

    def num_examples_per_epoch(self, subset="train"):
        if subset == "train":
            return IMAGENET_NUM_TRAIN_IMAGES
        if subset == "validation":
            return IMAGENET_NUM_VAL_IMAGES
        raise ValueError('Invalid data subset "%s"' % subset)


class Cifar10Dataset(ImageDataset):
    """CIFAR-10, held in memory.  Reads the *binary* release
    (``data_batch_{1..5}.bin`` / ``test_batch.bin``: 1 label byte + 3072 CHW
    pixel bytes per record) or an ``.npz`` with ``images``/``labels``; the
    python-pickle release is not read (no unpickling of data files)."""

    RECORD = 1 + 32 * 32 * 3

    def __init__(self, data_dir=None):
        super().__init__("cifar10", 32, 32, data_dir=data_dir, queue_runner_required=True,
                         num_classes=11)

    def read_data_files(self, subset="train"):
        assert self.data_dir, "Cannot call `read_data_files` when using synthetic data"
        npz = os.path.join(self.data_dir, "%s.npz" % subset)
        if os.path.exists(npz):
            with np.load(npz, allow_pickle=False) as z:
                return z["images"].astype(np.float32), z["labels"].astype(np.int64)
        if subset == "train":
            names = ["data_batch_%d.bin" % i for i in range(1, 6)]
        elif subset == "validation":
            names = ["test_batch.bin"]
        else:
            raise ValueError('Invalid data subset "%s"' % subset)
        recs = []
        for n in names:
            raw = np.fromfile(os.path.join(self.data_dir, n), dtype=np.uint8)
            recs.append(raw.reshape(-1, self.RECORD))
        allr = np.concatenate(recs)
        labels = allr[:, 0].astype(np.int64)
        images = allr[:, 1:].astype(np.float32)  # [n, 3072] CHW order
        return images, labels

    def num_examples_per_epoch(self, subset="train"):
        if subset == "train":
            return 50000
        if subset == "validation":
            return 10000
        raise ValueError('Invalid data subset "%s"' % subset)


class COCODataset(ImageDataset):
    def __init__(self, data_dir=None, image_size=300):
        super().__init__("coco", image_size, image_size, data_dir=data_dir, num_classes=81)

    def num_examples_per_epoch(self, subset="train"):
        if subset == "train":
            return COCO_NUM_TRAIN_IMAGES
        if subset == "validation":
            return COCO_NUM_VAL_IMAGES
        raise ValueError('Invalid data subset "%s"' % subset)


SUPPORTED_DATASETS = {
    "imagenet": ImagenetDataset,
    "cifar10": Cifar10Dataset,
    "librispeech": LibrispeechDataset,
    "coco": COCODataset,
}


def create_dataset(data_dir, data_name):
    if not data_dir and not data_name:
        data_name = "imagenet"
    if data_name is None:
        for name in SUPPORTED_DATASETS:
            if name in data_dir:
                data_name = name
                break
        else:
            raise ValueError("Could not identify name of dataset. "
                             "Please specify with --data_name option.")
    if data_name not in SUPPORTED_DATASETS:
        raise ValueError("Unknown dataset. Must be one of %s"
                         % ", ".join(sorted(SUPPORTED_DATASETS)))
    return SUPPORTED_DATASETS[data_name](data_dir)
