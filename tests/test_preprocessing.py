"""Input preprocessing and TFRecord plumbing (tcb/benchmark_cnn_test.py:817-886,
tcb/test_data/) on the host."""

import os

import numpy as np
import pytest

from kf_benchmarks_amd import params as P, runtime
from kf_benchmarks_amd.data import preprocessing as pre
from kf_benchmarks_amd.data import test_data

REF_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")  # vendored (data/README.md)


def _jpeg(value, h=20, w=30):
    return test_data.encode_jpeg(np.full((h, w, 3), value, np.uint8))


@pytest.mark.parametrize("ih,iw,oh,ow", [(10, 10, 4, 4), (4, 4, 10, 10), (1, 100, 100, 1),
                                         (100, 1, 1, 100), (1, 100, 1, 100)])
def test_eval_image_constant(ih, iw, oh, ow):
    img = np.full((ih, iw, 3), 128, np.uint8)
    out = pre.eval_image(img, oh, ow, 0, "bilinear")
    np.testing.assert_array_equal(out, np.full((oh, ow, 3), 128, np.uint8))


def _buffers():
    if os.path.isdir(os.path.join(REF_DATA, "images")):
        out = []
        for name, color in (("white_image.jpg", 255), ("black_image.jpg", 0)):
            with open(os.path.join(REF_DATA, "images", name), "rb") as f:
                out.append((f.read(), color))
        return out
    return [(_jpeg(255), 255), (_jpeg(0), 0)]


@pytest.mark.parametrize("oh,ow,method", [(100, 100, "round_robin"), (150, 10, "bilinear"),
                                          (10, 150, "nearest")])
@pytest.mark.parametrize("distortions", [True, False])
@pytest.mark.parametrize("fuse", [True, False])
def test_train_image_constant(oh, ow, method, distortions, fuse):
    bbox = np.zeros((0, 4), np.float32)
    rng = np.random.default_rng(0)
    for buf, color in _buffers():
        out = pre.train_image(buf, oh, ow, bbox, 0, method, distortions, rng,
                              fuse_decode_and_crop=fuse)
        assert out.shape == (oh, ow, 3)
        np.testing.assert_allclose(out.astype(np.float32), np.full((oh, ow, 3), color, np.float32),
                                   atol=50.0, rtol=0)


def test_distorted_bbox_respects_ranges():
    rng = np.random.default_rng(1)
    for _ in range(200):
        y, x, h, w = pre.sample_distorted_bounding_box((240, 320), [[0.1, 0.1, 0.9, 0.9]], rng)
        assert 0 <= y and y + h <= 240 and 0 <= x and x + w <= 320
        if (h, w) != (240, 320):
            assert 0.05 * 240 * 320 - 1 <= h * w <= 240 * 320
            assert 0.7 <= w / h <= 1.4


def test_round_robin_resize_cycles():
    assert [pre.get_image_resize_method("round_robin", i) for i in range(5)] == [
        "nearest", "bilinear", "bicubic", "area", "nearest"]
    with pytest.raises(ValueError):
        pre.get_image_resize_method("lanczos")


def test_color_distortion_identity_and_clip():
    img = np.random.default_rng(0).random((8, 8, 3)).astype(np.float32)
    h, s, v = pre._rgb_to_hsv(img)
    np.testing.assert_allclose(pre._hsv_to_rgb(h, s, v), img, atol=1e-5)
    np.testing.assert_allclose(pre.adjust_contrast(img, 1.0), img, atol=1e-6)
    out = pre.distort_color(img, 1, np.random.default_rng(2))
    assert out.min() >= 0 and out.max() <= 1


def test_reference_fake_tfrecords_parse():
    """The reference's checked-in fixture shards read through our TFRecord +
    Example parser: 10 classes, each image a flat gray of level
    label * 255 / 10 (JPEG), 0 or 1 normalized boxes."""
    d = os.path.join(REF_DATA, "fake_tf_record_data")
    n = 0
    for name in sorted(os.listdir(d)):
        for rec in runtime.tf_record_iterator(os.path.join(d, name)):
            buf, label, bbox, text = pre.parse_example_proto(rec)
            assert 0 <= label < 10
            assert bbox.shape[1] == 4 and (bbox >= 0).all() and (bbox <= 1).all()
            assert (bbox[:, 0] <= bbox[:, 2]).all() and (bbox[:, 1] <= bbox[:, 3]).all()
            img = pre.decode_jpeg(buf)
            assert 30 <= img.shape[0] <= 299 and 30 <= img.shape[1] <= 299
            assert abs(float(img.mean()) - label * 25.5) < 3
            n += 1
    assert n == 64 + 64  # one train + one validation shard


def test_generated_fixture_and_batches(tmp_path):
    test_data.write_black_and_white_tfrecord_data(str(tmp_path), 10, 64, 16, 4, 2)
    assert len(list(tmp_path.glob("train-*-of-00004"))) == 4

    class Bench:
        pass
    from kf_benchmarks_amd import datasets
    from kf_benchmarks_amd.models import model_config
    b = Bench()
    b.params = P.make_params(model="trivial", data_dir=str(tmp_path), distortions=False)
    b.dataset = datasets.create_dataset(str(tmp_path), "imagenet")
    b.model = model_config.get_model_config("trivial", b.dataset, b.params)
    b.batch_size = 8
    b.model.set_batch_size(8)
    b.task_index, b.num_workers, b.num_replicas, b.local_batch_size = 0, 1, 1, 8
    it = pre.make_batch_iterator(b, "train")
    imgs, labels = next(it)
    assert imgs.shape == (8, 227, 227, 3) and imgs.dtype == np.uint8
    assert imgs.max() < 20 and labels.dtype == np.int32
    it = pre.make_batch_iterator(b, "validation")
    imgs, _ = next(it)
    assert imgs.min() > 235
    b.params = b.params._replace(distortions=True)
    imgs, _ = next(pre.make_batch_iterator(b, "train"))
    assert imgs.dtype == np.float32 and -1.01 <= imgs.min() and imgs.max() <= 1.01


def test_record_source_shift_and_repeat(tmp_path):
    files = []
    for k in range(3):
        p = str(tmp_path / ("f%d" % k))
        with runtime.TFRecordWriter(p) as w:
            for i in range(2):
                w.write(b"%d-%d" % (k, i))
        files.append(p)
    src = iter(pre.RecordSource(files, train=False, shift_ratio=1 / 3.0, cycle_length=1))
    got = [next(src) for _ in range(7)]
    assert got[:6] == [b"1-0", b"1-1", b"2-0", b"2-1", b"0-0", b"0-1"] and got[6] == b"1-0"
    src = iter(pre.RecordSource(files, train=True, repeat_cached_sample=True))
    assert len({next(src) for _ in range(5)}) == 1


def test_sequence_example_roundtrip():
    rec = runtime.make_sequence_example(
        {"labels": [3, 1, 2], "input_length": [2], "label_length": [3]},
        {"features": [[0.5] * 161, [1.5] * 161]})
    feats, labels, ilen, llen = pre.LibrispeechPreprocessor(
        2, [[2, 4, 161, 1], [2, 5], [2], [2]]).parse_and_preprocess(rec)
    assert feats.shape == (2, 161, 1) and list(labels) == [3, 1, 2]
    assert ilen[0] == 2 and llen[0] == 3


def test_cifar10_preprocessing_shapes():
    p = pre.Cifar10ImagePreprocessor(4, [[4, 32, 32, 3], [4]], train=True, distortions=True)
    img = np.full((32, 32, 3), 255, np.float32)
    out = p.preprocess(img, np.random.default_rng(0))
    assert out.shape == (32, 32, 3) and out.max() <= 1.0 and out.min() >= -1.0


def test_engine_trains_and_evals_on_tfrecords(tmp_path):
    """train -> checkpoint -> eval through the real-data pipeline (TFRecord
    shards -> host decode/crop/resize -> batches) on the CPU path."""
    import kfb_test_util as tu
    from kf_benchmarks_amd import benchmark
    data = tmp_path / "data"
    test_data.write_black_and_white_tfrecord_data(str(data), 2, 32, 16, 2, 1)
    base = dict(model="trivial", data_name="imagenet", data_dir=str(data), batch_size=4,
                num_warmup_batches=0, device="cpu", data_format="NHWC", optimizer="sgd",
                init_learning_rate=0.005, train_dir=str(tmp_path / "train"), num_batches=6,
                distortions=False)
    with tu.capture_logs() as logs:
        stats = benchmark.BenchmarkCNN(benchmark.make_params(**base)).run()
    assert stats["num_steps"] == 6
    assert any("total images/sec" in line for line in logs)
    base.update(eval=True, num_eval_batches=2)
    with tu.capture_logs() as logs:
        benchmark.BenchmarkCNN(benchmark.make_params(**base)).run()
    assert any("Accuracy @ 1" in line for line in logs)


def test_get_imagenet_probe(tmp_path):
    """tools.get_imagenet (role of tcb/get_imagenet.py) finds the shards of
    an ImageNet-layout directory and decodes their records natively."""
    from kf_benchmarks_amd.tools import get_imagenet
    test_data.write_black_and_white_tfrecord_data(str(tmp_path), 11, num_train_images=16,
                                                  num_validation_images=8, train_shards=2,
                                                  validation_shards=1)
    res = get_imagenet.probe(str(tmp_path), sample_shards=2)
    assert res["subsets"]["train"]["shards"] == 2
    assert res["subsets"]["train"]["sampled_records"] == 16
    assert res["subsets"]["validation"]["sampled_records"] == 8
    assert res["subsets"]["train"]["first_example"]["image/encoded"] > 0
    assert get_imagenet.main(["--data_dir", str(tmp_path)]) == 0


def test_native_saturation_hue_matches_numpy():
    """runtime.adjust_saturation_hue (one native HSV round trip) equals the
    numpy adjust_saturation then adjust_hue of the colour distortion."""
    from kf_benchmarks_amd import runtime
    from kf_benchmarks_amd.data import preprocessing as pp
    rng = np.random.default_rng(7)
    img = rng.random((37, 41, 3), dtype=np.float32)
    img[0, 0] = [0.5, 0.5, 0.5]   # grey: no hue
    img[0, 1] = [0.0, 0.0, 0.0]   # black
    img[0, 2] = [1.0, 0.0, 1.0]   # magenta: max shared by r and b
    for sat, hue in [(0.5, 0.0), (1.5, 0.2), (1.0, -0.2), (0.73, 0.11)]:
        ref = pp.adjust_hue(pp.adjust_saturation(img, sat), hue)
        out = runtime.adjust_saturation_hue(img.copy(), sat, hue)
        np.testing.assert_allclose(out, ref, rtol=1e-5, atol=2e-6)


def test_batch_group_size_stages_groups(tmp_path):
    """--batch_group_size=3 on the real-data path: batches are staged by the
    ImageProducer in groups of 3, at most two groups ahead of the consumer
    (tcb/cnn_util.py:118-198), and training consumes them all."""
    import kfb_test_util as tu
    from kf_benchmarks_amd import benchmark
    from kf_benchmarks_amd.data import input_pipeline
    data = tmp_path / "data"
    test_data.write_black_and_white_tfrecord_data(str(data), 2, 48, 16, 2, 1)
    params = benchmark.make_params(model="trivial", data_name="imagenet", data_dir=str(data),
                                   batch_size=4, num_warmup_batches=0, device="cpu",
                                   data_format="NHWC", optimizer="sgd", num_batches=6,
                                   distortions=False, batch_group_size=3)
    seen = []
    orig = input_pipeline.PrefetchInput.__init__

    def init(self, *a, **k):
        orig(self, *a, **k)
        seen.append(self)
    input_pipeline.PrefetchInput.__init__ = init
    try:
        with tu.capture_logs() as logs:
            b = benchmark.BenchmarkCNN(params)
            b.print_info()
            stats = b.run()
    finally:
        input_pipeline.PrefetchInput.__init__ = orig
    assert stats["num_steps"] == 6
    assert any("3 batches per prepocessing group" in line for line in logs)
    prod = seen[0].producer
    assert prod is not None and prod.batch_group_size == 3
    assert prod._consumed >= 6 and prod._produced % 3 == 0
    assert prod._produced - prod._consumed <= 2 * 3 + 3


def test_u8_host_path_plus_augment_reference_matches_host_path():
    """The device-augmentation split (host: decode/crop/resize to uint8 +
    parameter draws; device: flip, colour, scaling) reproduces the all-host
    train_image + normalized_image result for the same randoms."""
    img = np.clip(np.random.default_rng(0).normal(120, 50, (90, 120, 3)), 0, 255).astype(np.uint8)
    buf = test_data.encode_jpeg(img)
    bbox = np.array([[0.1, 0.1, 0.9, 0.8]], np.float32)
    for pos in range(4):
        for distort in (False, True):
            a = pre.train_image(buf, 64, 48, bbox, pos, "bilinear", distort,
                                np.random.default_rng(pos), False, True)
            u8, prm = pre.train_image_u8(buf, 64, 48, bbox, pos, "bilinear", distort,
                                         np.random.default_rng(pos), False, draft=False)
            assert u8.dtype == np.uint8 and u8.shape == (64, 48, 3) and prm.shape == (8,)
            b = pre.augment_reference(u8[None], prm[None])[0]
            ref = pre.normalized_image(a.astype(np.float32))
            np.testing.assert_allclose(b, ref, atol=2e-5)


def test_native_image_pipe_on_reference_fixtures():
    """csrc/runtime/kfb_images.cpp on the reference's fixture shards (flat
    gray JPEGs of level label * 25.5): crops stay flat at that level, labels
    agree with the Python parser, and the augmentation parameters are in the
    reference's ranges and batch-position order."""
    if not runtime.ImagePipe.available():
        pytest.skip("libjpeg not loadable")
    d = os.path.join(REF_DATA, "fake_tf_record_data")
    recs = []
    for name in sorted(os.listdir(d)):
        recs += list(runtime.tf_record_iterator(os.path.join(d, name)))
    recs = recs[:48]
    pipe = runtime.ImagePipe(3, 40, 56, True, False)
    try:
        imgs, prm, labels, bad = pipe.run(recs, np.arange(len(recs), dtype=np.uint64) + 5)
        imgs2, prm2, _, _ = pipe.run(recs, np.arange(len(recs), dtype=np.uint64) + 5)
    finally:
        pipe.close()
    assert bad == 0 and imgs.shape == (48, 40, 56, 3) and imgs.dtype == np.uint8
    assert np.array_equal(imgs, imgs2) and np.array_equal(prm, prm2)  # seeded, deterministic
    for i, rec in enumerate(recs):
        _, label, _, _ = pre.parse_example_proto(rec)
        assert labels[i] == label
        assert abs(float(imgs[i].mean()) - label * 25.5) < 4
    assert set(np.unique(prm[:, 0])) <= {0.0, 1.0}
    assert (np.abs(prm[:, 1]) <= 32 / 255 + 1e-6).all()
    assert ((prm[:, 2] >= 0.5) & (prm[:, 2] <= 1.5)).all()
    assert (np.abs(prm[:, 3]) <= 0.2 + 1e-6).all()
    assert ((prm[:, 4] >= 0.5) & (prm[:, 4] <= 1.5)).all()
    assert np.array_equal(prm[:, 5], np.arange(48) % 2) and (prm[:, 6] == 1).all()


def test_device_augment_batches_on_host(tmp_path):
    """With device augmentation the train batches are (uint8 images, labels,
    params); the CPU form of the device op turns them into the [-1, 1] images."""
    import torch
    from kf_benchmarks_amd.ops import nn as F
    test_data.write_black_and_white_tfrecord_data(str(tmp_path), 10, 32, 8, 2, 1)

    class Bench:
        pass
    from kf_benchmarks_amd import datasets
    from kf_benchmarks_amd.models import model_config
    b = Bench()
    b.params = P.make_params(model="trivial", data_dir=str(tmp_path), distortions=True)
    b.dataset = datasets.create_dataset(str(tmp_path), "imagenet")
    b.model = model_config.get_model_config("trivial", b.dataset, b.params)
    b.model.set_batch_size(8)
    b.task_index, b.num_workers, b.num_replicas, b.local_batch_size = 0, 1, 1, 8
    p = pre.get_preprocessor(b, "train")
    p.device_augment = True
    imgs, labels, prm = next(p.minibatch(b.dataset, "train", b.params))
    assert imgs.dtype == np.uint8 and imgs.shape == (8, 227, 227, 3)
    assert prm.shape == (8, 8) and labels.dtype == np.int32
    out = F.augment_u8(torch.from_numpy(imgs), torch.from_numpy(prm), torch.float32)
    assert out.shape == (8, 227, 227, 3) and out.min() >= -1.0 and out.max() <= 1.0


def test_jpeg_ring_slot_is_held_while_its_batch_is_queued():
    """A yielded GPU-JPEG batch keeps its pinned ring slot until the consumer
    enqueued its copies (or dropped it): the producer cannot refill a slot
    whose batch still waits in a prefetch queue, however deep the queue."""
    import threading
    import time
    slot = pre._JpegSlot(2, 8, 8)
    slot.wait_free()  # a fresh slot is free
    slot.claim()
    done = threading.Event()
    th = threading.Thread(target=lambda: (slot.wait_free(), done.set()), daemon=True)
    th.start()
    time.sleep(0.2)
    assert not done.is_set()  # queued, not yet copied: refilling must wait
    slot.release(None)
    assert done.wait(5)
    th.join(5)


def test_jpeg_ring_follows_the_lookahead():
    assert pre.jpeg_ring_slots(2, 1) == pre._JPEG_RING
    assert pre.jpeg_ring_slots(9, 1) == 11  # queue of 9 + copying + filling
    assert pre.jpeg_ring_slots(3, 3) == 3 + 9 + 2  # ImageProducer keeps <= 3G-1 ahead
