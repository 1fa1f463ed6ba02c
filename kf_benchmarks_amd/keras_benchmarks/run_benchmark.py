"""Entry point (role of keras_benchmarks/run_benchmark.py +
upload_benchmarks_bq.py): runs the three micro-benchmarks with the
``--mode`` hardware config and appends one JSON record per benchmark to
``--output`` (the reference uploads the same fields to BigQuery).

    python -m kf_benchmarks_amd.keras_benchmarks.run_benchmark --mode gpu_config
    python -m kf_benchmarks_amd.parallel.launcher -np 8 \\
        python -m kf_benchmarks_amd.keras_benchmarks.run_benchmark --mode multi_gpu_config
"""

from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import uuid

import torch

from .models.benchmarks import Cifar10CnnBenchmark, LstmBenchmark, MnistMlpBenchmark

HERE = os.path.dirname(os.path.abspath(__file__))


def metrics_record(model, config, backend_version):
    """The fields of upload_benchmarks_bq.upload_metrics_to_bq."""
    return {
        "test_id": str(uuid.uuid4()), "test_name": model.test_name,
        "recorded_at": datetime.datetime.utcnow().isoformat() + "Z",
        "total_time": model.total_time, "epochs": model.epochs,
        "batch_size": model.batch_size, "backend_type": "torch-rocm",
        "backend_version": backend_version, "cpu_num_cores": config["cpu_num_cores"],
        "cpu_memory": config["cpu_memory"], "cpu_memory_info": config["cpu_memory_info"],
        "gpu_count": config["gpus"], "gpu_platform": config["gpu_platform"],
        "platform_type": config["platform_type"],
        "platform_machine_type": config["platform_machine_type"],
        "keras_version": "kf_benchmarks_amd", "sample_type": model.sample_type,
    }


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="gpu_config",
                    help="cpu_config | gpu_config | multi_gpu_config (config.json)")
    ap.add_argument("--config", default=os.path.join(HERE, "config.json"))
    ap.add_argument("--output", default="keras_benchmarks.jsonl")
    ap.add_argument("--only", default=None, help="comma list of test names")
    a = ap.parse_args(argv)
    with open(a.config) as f:
        config = json.load(f)[a.mode]
    device = "cpu" if config["gpus"] == 0 or not torch.cuda.is_available() else None
    if device is None and "LOCAL_RANK" in os.environ:
        device = "cuda:%d" % int(os.environ["LOCAL_RANK"])
    version = torch.__version__ + (" / HIP %s" % torch.version.hip
                                   if getattr(torch.version, "hip", None) else "")
    rank = int(os.environ.get("RANK", "0"))
    for cls in (MnistMlpBenchmark, Cifar10CnnBenchmark, LstmBenchmark):
        model = cls()
        if a.only and model.test_name not in a.only.split(","):
            continue
        model.run_benchmark(gpus=config["gpus"], device=device)
        print("%s: total_time %.4f s (%d epochs, batch %d)"
              % (model.test_name, model.total_time, model.epochs, model.batch_size))
        if rank == 0:
            with open(a.output, "a") as f:
                f.write(json.dumps(metrics_record(model, config, version)) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
