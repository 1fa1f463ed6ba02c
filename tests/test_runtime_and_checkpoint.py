"""Native runtime (CRC32C, TFRecord, tf.Example, SSTable) and TF-bundle
checkpoints.  TFRecord parity is pinned against the reference's own test
fixtures (TF-written files in tcb/test_data/fake_tf_record_data)."""

import glob
import os

import numpy as np
import pytest
import torch

from kf_benchmarks_amd import runtime as rt
from kf_benchmarks_amd.utils import checkpoint as ck
from kf_benchmarks_amd.utils import summary as sm

REF_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data",
                        "fake_tf_record_data")  # vendored reference fixture (data/README.md)


def test_crc32c_known_vectors():
    assert rt.crc32c(b"123456789") == 0xE3069283
    assert rt.crc32c(b"") == 0
    assert rt.crc32c(b"\x00" * 32) == 0x8A9136AA
    data = os.urandom(1000)
    assert rt.crc32c(data[500:], rt.crc32c(data[:500])) == rt.crc32c(data)


def test_tfrecord_roundtrip(tmp_path):
    p = str(tmp_path / "x.tfrecord")
    recs = [os.urandom(n) for n in (0, 1, 100, 70000)]
    with rt.TFRecordWriter(p) as w:
        for r in recs:
            w.write(r)
    assert list(rt.tf_record_iterator(p)) == recs
    raw = bytearray(open(p, "rb").read())
    raw[20] ^= 0xFF
    open(p, "wb").write(bytes(raw))
    with pytest.raises(rt.TFRecordCorrupt):
        list(rt.tf_record_iterator(p))


def test_reads_reference_tf_written_records():
    n = 0
    labels = set()
    for f in sorted(glob.glob(os.path.join(REF_DATA, "*"))):
        for r in rt.tf_record_iterator(f):
            ex = rt.parse_example(r)
            assert ex["image/format"] == [b"JPEG"]
            assert ex["image/encoded"][0][:2] == b"\xff\xd8"  # JPEG SOI
            labels.add(ex["image/class/label"][0])
            n += 1
    assert n > 0 and labels


def test_example_roundtrip():
    ex = {"image/encoded": [b"\x01\x02"], "image/class/label": [7, -3],
          "image/object/bbox/xmin": [0.25, 0.5]}
    out = rt.parse_example(rt.make_example(ex))
    assert out["image/encoded"] == [b"\x01\x02"]
    assert out["image/class/label"] == [7, -3]
    assert out["image/object/bbox/xmin"] == pytest.approx([0.25, 0.5])


def test_table_roundtrip(tmp_path):
    items = [(b"", b"header")] + [(("v0/cg/conv%03d" % i).encode(), os.urandom(i * 37))
                                  for i in range(300)]
    p = str(tmp_path / "t.index")
    rt.table_write(p, items)
    assert rt.table_read(p) == sorted(items)


def test_bundle_roundtrip(tmp_path):
    prefix = str(tmp_path / "model.ckpt-12")
    tensors = {"v0/cg/conv0/conv2d/kernel": np.random.randn(3, 3, 4, 8).astype(np.float32),
               "global_step": np.array(12, dtype=np.int64),
               "v0/cg/affine0/biases": torch.randn(5),
               "half": np.arange(6, dtype=np.float16).reshape(2, 3)}
    ck.write_bundle(prefix, tensors)
    back = ck.read_bundle(prefix)
    assert set(back) == set(tensors)
    np.testing.assert_array_equal(back["v0/cg/conv0/conv2d/kernel"],
                                  tensors["v0/cg/conv0/conv2d/kernel"])
    assert int(back["global_step"]) == 12
    np.testing.assert_array_equal(back["v0/cg/affine0/biases"], tensors["v0/cg/affine0/biases"].numpy())
    assert back["half"].dtype == np.float16


def test_checkpoint_path_resolution(tmp_path):
    assert ck.get_checkpoint_to_load("/foo/bar/model.ckpt-189") == "/foo/bar/model.ckpt-189"
    with pytest.raises(ck.CheckpointNotFoundException):
        ck.get_checkpoint_to_load(str(tmp_path))
    ck.write_checkpoint_state(str(tmp_path), "model.ckpt-1243", ["model.ckpt-1243"])
    assert ck.get_checkpoint_to_load(str(tmp_path)) == str(tmp_path / "model.ckpt-1243")
    assert ck.step_from_path("/path/to/checkpoints/model.ckpt-1243") == 1243


def test_summary_events(tmp_path):
    w = sm.SummaryWriter(str(tmp_path))
    w.add_scalars({"learning_rate": 0.5, "total_loss": 2.0}, 3)
    w.add_histograms({"log_gradients": np.random.randn(100)}, 3)
    w.close()
    ev = sm.read_events(w.path)
    assert ev[1] == (3, {"learning_rate": 0.5, "total_loss": 2.0})
    assert ev[2][1]["log_gradients"] == "histogram"
