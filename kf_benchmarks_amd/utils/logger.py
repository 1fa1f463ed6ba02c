"""Benchmark JSON logger (role of the model-garden BenchmarkFileLogger used at
tcb/benchmark_cnn.py:1594-1724): run info, metrics and eval results as JSON
lines under --benchmark_log_dir."""

from __future__ import annotations

import datetime
import json
import os
import platform


class BenchmarkFileLogger:
    def __init__(self, log_dir: str, test_id=None):
        os.makedirs(log_dir, exist_ok=True)
        self.log_dir = log_dir
        self.test_id = test_id
        self._metric = os.path.join(log_dir, "metric.log")

    def _stamp(self):
        return datetime.datetime.utcnow().strftime("%Y-%m-%dT%H:%M:%S.%fZ")

    def log_metric(self, name, value, unit=None, global_step=None, extras=None):
        rec = {"name": name, "value": float(value), "unit": unit, "global_step": global_step,
               "timestamp": self._stamp(), "extras": extras or []}
        with open(self._metric, "a") as f:
            f.write(json.dumps(rec) + "\n")

    def log_evaluation_result(self, eval_results):
        step = eval_results.get("global_step")
        for k, v in eval_results.items():
            if k != "global_step":
                self.log_metric(k, v, global_step=step)

    def log_run_info(self, model_name, dataset_name, run_params):
        info = {"model_name": model_name, "dataset": {"name": dataset_name},
                "machine_config": {"platform": platform.platform()},
                "test_id": self.test_id, "run_date": self._stamp(),
                "run_parameters": [{"name": k, "string_value": str(v)}
                                   for k, v in sorted(run_params.items())]}
        with open(os.path.join(self.log_dir, "benchmark_run.log"), "w") as f:
            f.write(json.dumps(info, indent=2))
