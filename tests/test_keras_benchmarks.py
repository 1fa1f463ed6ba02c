"""Keras-style micro-benchmarks (reference keras_benchmarks has no tests;
these check the runner contract: three records with the BigQuery fields)."""

import json

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
