"""Step tracing / profiling hooks (--trace_file, --tfprof_file, --graph_file).

Role of tcb/benchmark_cnn.py:801-883 and 1208-1228: one full trace of the
second-to-last warmup step (local step -2) written as a Chrome trace (via
torch.profiler, which records the HIP kernels through roctracer), and a
"tfprof" table of the top ops by device time over steps 0-9.
"""

from __future__ import annotations

import os

import torch

from .. import cnn_util

_NUM_STEPS_TO_PROFILE = 10


def _activities(device):
    acts = [torch.profiler.ProfilerActivity.CPU]
    if device.type == "cuda":
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    return acts


class StepTracer:
    def __init__(self, bench):
        self.bench = bench
        p = bench.params
        self.trace_file = p.trace_file
        self.chrome = p.use_chrome_trace_format
        self.tfprof_file = p.tfprof_file
        self.device = bench.device
        self._prof = None
        self._tfprof = None
        if p.graph_file and bench.world.is_chief:
            self._write_graph(p.graph_file)

    def _write_graph(self, path):
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            f.write(str(self.bench.net))
            f.write("\n")
            for name, p in self.bench.net.trainable_variables():
                f.write("%s %s\n" % (name, tuple(p.shape)))
        cnn_util.log_fn("Writing model description to %s" % path)

    def begin(self, step):
        if self.trace_file and step == -2:
            self._prof = torch.profiler.profile(activities=_activities(self.device),
                                                profile_memory=True, record_shapes=True)
            self._prof.__enter__()
        if self.tfprof_file and step == 0:
            self._tfprof = torch.profiler.profile(activities=_activities(self.device))
            self._tfprof.__enter__()

    def end(self, step):
        if self._prof is not None and step == -2:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self._prof.__exit__(None, None, None)
            cnn_util.log_fn("Dumping trace to %s" % self.trace_file)
            d = os.path.dirname(self.trace_file)
            if d:
                os.makedirs(d, exist_ok=True)
            if self.chrome:
                self._prof.export_chrome_trace(self.trace_file)
            else:
                with open(self.trace_file, "w") as f:
                    f.write(self._prof.key_averages().table(row_limit=-1))
            self._prof = None
        if self._tfprof is not None and step == _NUM_STEPS_TO_PROFILE - 1:
            self._finish_tfprof()

    def _finish_tfprof(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self._tfprof.__exit__(None, None, None)
        key = "self_cuda_time_total" if self.device.type == "cuda" else "self_cpu_time_total"
        table = self._tfprof.key_averages().table(sort_by=key, row_limit=20)
        d = os.path.dirname(self.tfprof_file)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(self.tfprof_file, "w") as f:
            f.write(table)
        cnn_util.log_fn("Top ops by accelerator time:\n%s" % table)
        self._tfprof = None

    def finish(self):
        if self._tfprof is not None:
            self._finish_tfprof()
