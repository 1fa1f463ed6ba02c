"""Keras-style micro-benchmarks (reference keras_benchmarks has no tests;
these check the runner contract: three records with the BigQuery fields)."""

import json

import pytest

from kf_benchmarks_amd.keras_benchmarks import data_generator as dg
from kf_benchmarks_amd.keras_benchmarks import run_benchmark


def test_data_generators():
    x, y = dg.generate_img_input_data((10, 3, 4, 4), 5)
    assert x.shape == (10, 3, 4, 4) and y.max() < 5 and x.max() < 255
    x, y = dg.generate_text_input_data((6, 4, 7))
    assert x.dtype == bool and y.shape == (6, 7)
    assert dg.to_categorical([1, 0], 3).tolist() == [[0, 1, 0], [1, 0, 0]]


def test_runner_writes_records(tmp_path):
    out = tmp_path / "kb.jsonl"
    assert run_benchmark.main(["--mode", "cpu_config", "--output", str(out)]) == 0
    recs = [json.loads(l) for l in out.read_text().splitlines()]
    assert [r["test_name"] for r in recs] == ["mnist_mlp", "cifar10_cnn", "lstm"]
    for r in recs:
        assert r["epochs"] == 2 and r["total_time"] > 0 and r["gpu_count"] == 0


def _learns(device):
    """A Sequential MLP + CNN + LSTM on our ops fits a small fixed problem."""
    import numpy as np
    from kf_benchmarks_amd.keras_benchmarks import sequential as S
    rng = np.random.default_rng(0)
    out = {}
    x = rng.random((64, 8, 8, 3), dtype=np.float32)
    y = dg.to_categorical(rng.integers(0, 4, 64), 4)
    m = S.Sequential(device)
    m.add(S.Conv2D(8, (3, 3), padding="same", input_shape=(8, 8, 3), activation="relu"))
    m.add(S.MaxPooling2D((2, 2)))
    m.add(S.Flatten())
    m.add(S.Dense(32, activation="relu"))
    m.add(S.Dense(4, activation="softmax"))
    m.compile(optimizer=S.RMSprop(lr=0.01))
    out["cnn"] = m.fit(x, y, batch_size=16, epochs=15, verbose=1)
    xs = (rng.random((64, 6, 5)) > 0.5).astype(np.float32)
    m = S.Sequential(device)
    m.add(S.LSTM(16, input_shape=(6, 5)))
    m.add(S.Dense(4), activation="softmax")
    m.compile(optimizer=S.RMSprop(lr=0.01))
    out["lstm"] = m.fit(xs, y, batch_size=16, epochs=15, verbose=1)
    return out


_FACTOR = {"cnn": 0.5, "lstm": 0.8}  # loss-sum drop over 15 epochs (the LSTM fits slower)


def test_sequential_learns_cpu():
    for name, hist in _learns("cpu").items():
        assert hist[-1] < _FACTOR[name] * hist[0], (name, hist)


@pytest.mark.gpu
def test_sequential_learns_gpu(cuda):
    for name, hist in _learns(cuda).items():
        assert all(h == h for h in hist), (name, hist)
        assert hist[-1] < _FACTOR[name] * hist[0], (name, hist)


@pytest.mark.gpu
def test_runner_gpu(cuda, tmp_path):
    out = tmp_path / "kb.jsonl"
    assert run_benchmark.main(["--mode", "gpu_config", "--output", str(out)]) == 0
    recs = [json.loads(l) for l in out.read_text().splitlines()]
    assert [r["test_name"] for r in recs] == ["mnist_mlp", "cifar10_cnn", "lstm"]
    assert all(r["total_time"] > 0 for r in recs)
