"""BenchmarkCNN: the training / eval / forward-only benchmark engine.

Role of tcb/benchmark_cnn.py (C6-C18 in SURVEY §2.1), re-designed for an
eager PyTorch-ROCm process per GPU:

  params -> dataset + model -> Network (variables) -> FlatParams (one flat
  fp32 buffer + grads + bf16 shadow) -> Strategy (RCCL aggregation per
  --variable_update) -> FusedOptimizer -> hot loop.

The hot loop never synchronizes the host per step: each step records a HIP
event and step times are read back at display steps (the reference's
per-step ``sess.run`` wall time, tcb/benchmark_cnn.py:786-884, without the
host round trip).  Log lines keep the reference's format verbatim
(Appendix B of SURVEY.md); tests parse them.
"""

from __future__ import annotations

import json
import math
import os
import sys
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from . import cnn_util, datasets, flags, optim, params as params_lib
from .constants import BenchmarkMode
from .models import model_config
from .models.model import make_network
from .ops import _native
from .parallel import comm
from .parallel import watchdog
from .parallel.variable_mgr import make_strategy

log_fn = cnn_util.log_fn

_DEFAULT_NUM_BATCHES = 100
LOSS_AND_ACCURACY_DIGITS_TO_SHOW = 3
_NUM_STEPS_TO_PROFILE = 10

IGNORED_TF_FLAGS = ("xla", "xla_compile", "winograd_nonfused", "batchnorm_persistent", "mkl",
                    "enable_optimizations", "rewriter_config", "trt_mode", "use_unified_memory",
                    "force_gpu_compatible", "allow_growth", "use_resource_vars",
                    "freeze_when_forward_only", "debugger", "gpu_thread_mode")


class CheckpointNotFoundException(Exception):
    pass


def get_mode_from_params(params):
    if params.eval:
        return BenchmarkMode.EVAL
    if params.forward_only:
        return BenchmarkMode.FORWARD_ONLY
    if (params.eval_during_training_every_n_steps or params.eval_during_training_every_n_epochs
            or params.eval_during_training_at_specified_steps
            or params.eval_during_training_at_specified_epochs):
        return BenchmarkMode.TRAIN_AND_EVAL
    return BenchmarkMode.TRAIN


def get_num_batches_and_epochs(params, batch_size, num_examples_per_epoch):
    if params.num_batches and params.num_epochs:
        raise ValueError("At most one of --num_batches and --num_epochs may be specified.")
    if params.num_epochs:
        num_batches = int(float(params.num_epochs) * num_examples_per_epoch / batch_size)
    else:
        num_batches = params.num_batches or _DEFAULT_NUM_BATCHES
    num_epochs = num_batches * batch_size / float(num_examples_per_epoch)
    return num_batches, num_epochs


def get_perf_timing(batch_size, step_train_times, scale=1):
    times = np.array(step_train_times)
    speeds = batch_size / times
    speed_mean = scale * batch_size / np.mean(times)
    speed_uncertainty = np.std(speeds) / np.sqrt(float(len(speeds)))
    speed_jitter = 1.4826 * np.median(np.abs(speeds - np.median(speeds)))
    return speed_mean, speed_uncertainty, speed_jitter


def get_perf_timing_str(speed_mean, speed_uncertainty, speed_jitter, scale=1):
    if scale == 1:
        return "images/sec: %.1f +/- %.1f (jitter = %.1f)" % (speed_mean, speed_uncertainty,
                                                             speed_jitter)
    return "images/sec: %.1f" % speed_mean


def validate_params_combinations(params):
    """Cross-flag checks of tcb/benchmark_cnn.py:1268-1352 (those meaningful
    on this stack)."""
    p = params
    if p.device.lower() == "cpu" and p.data_format == "NCHW" and not p.mkl:
        raise ValueError("device=cpu requires that data_format=NHWC")
    if ((p.num_epochs_per_decay or p.learning_rate_decay_factor) and
            not (p.init_learning_rate is not None and p.num_epochs_per_decay
                 and p.learning_rate_decay_factor)):
        raise ValueError("If one of num_epochs_per_decay or learning_rate_decay_factor is set, "
                         "both must be set and learning_rate must be set")
    if (p.minimum_learning_rate and
            not (p.init_learning_rate is not None and p.num_epochs_per_decay
                 and p.learning_rate_decay_factor)):
        raise ValueError("minimum_learning_rate requires learning_rate, num_epochs_per_decay, "
                         "and learning_rate_decay_factor to be set")
    if p.use_fp16 and p.fp16_vars and "replicated" in p.variable_update \
            and p.all_reduce_spec and "nccl" in p.all_reduce_spec:
        raise ValueError("fp16 variables are not supported with NCCL")
    if p.use_fp16 and p.fp16_vars and p.gradient_repacking:
        raise ValueError("--fp16_vars cannot be used with --gradient_repacking")
    if p.use_fp16 and p.use_bf16:
        raise ValueError("At most one of --use_fp16 and --use_bf16 may be set")
    if p.variable_update == "horovod" and p.num_gpus > 1:
        raise ValueError("Horovod benchmarks require num_gpus=1 on each worker")
    if p.variable_update == "horovod" and p.job_name:
        raise ValueError("job_name should not be specified for Horovod.")
    if p.variable_update == "kungfu" and p.num_gpus > 1:
        raise ValueError("KungFu benchmarks require num_gpus=1 on each worker")
    if p.variable_update == "kungfu" and p.job_name:
        raise ValueError("job_name should not be specified for KungFu.")
    if p.use_fp16 and p.fp16_enable_auto_loss_scale:
        if p.all_reduce_spec and "nccl" in p.all_reduce_spec:
            raise ValueError("Automatic loss scaling is not supported with NCCL.")
        if p.variable_update not in ("parameter_server", "replicated", "independent"):
            raise ValueError("Automatic loss scaling is not supported with variable_update=%s."
                             % p.variable_update)
        if p.staged_vars:
            raise ValueError("Automatic loss scaling is not supported with staged_vars.")
    if p.debugger is not None and p.debugger != "cli" and ":" not in p.debugger:
        raise ValueError('--debugger must be "cli" or in the form host:port')
    if p.hierarchical_copy and p.num_gpus <= 1 and comm.env_world_size() <= 1 \
            and not comm.force_pg():
        # (one process per GPU: the ranks of the world are the devices; a
        # forced 1-rank group is the GPU tests' stand-in)
        raise ValueError("--hierarchical_copy requires --num_gpus to be greater than 1")
    if p.save_model_secs and p.save_model_steps:
        raise ValueError("At most one of --save_model_secs and --save_model_steps can be "
                         "specified")
    evf = [bool(p.eval_during_training_every_n_steps),
           bool(p.eval_during_training_every_n_epochs),
           bool(p.eval_during_training_at_specified_steps),
           bool(p.eval_during_training_at_specified_epochs)]
    if evf.count(True) > 1:
        raise ValueError("At most one flag with --eval_during_training_* prefix must be "
                         "specified.")
    if any(evf):
        if p.eval:
            raise ValueError("At most one of --eval and --eval_during_training_* must be "
                             "specified")
        if p.forward_only:
            raise ValueError("At most one of --forward_only and --eval_during_training_* must "
                             "be specified")
        if p.job_name:
            raise ValueError("--eval_during_training_* is not yet supported in distributed "
                             "mode.")
        if p.staged_vars:
            raise ValueError("--eval_during_training_* is not currently compatible with "
                             "staged_vars")
    if p.stop_at_top_1_accuracy and not any(evf):
        raise ValueError("--stop_at_top_1_accuracy is only supported with "
                         "--eval_during_training_*")
    if p.forward_only and p.freeze_when_forward_only:
        if p.train_dir is not None:
            raise ValueError("In forward_only mode, when --freeze_when_forward_only is True, "
                             "--train_dir should not be specified")
    elif p.trt_mode:
        raise ValueError("--trt_mode should not be specified if one of --forward_only and "
                         "--freeze_when_forward_only is set to False")
    if p.staged_vars and p.variable_update != "parameter_server":
        raise ValueError("staged_vars for enqueue/dequeue only support variable update "
                         "parameter_server")
    if p.eval and p.forward_only:
        raise ValueError("Only one of --eval and --forward_only may be specified")
    if p.variable_consistency == "relaxed" and p.variable_update != "replicated":
        raise ValueError("variable_consistency=relaxed requires variable_update=replicated")
    if p.kernel_impl not in ("hip", "torch"):
        # torch: the convolutions on stock PyTorch / MIOpen, everything else
        # on our kernels - the same-node reference bar, never a headline
        raise ValueError("--kernel_impl must be hip or torch")


class _EventTimer:
    """Per-step device timing without a per-step host sync."""

    def __init__(self, device):
        self.cuda = device.type == "cuda"
        self.device = device
        self._last = None
        self._pending: List = []

    def mark(self):
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            if self._last is not None:
                self._pending.append((self._last, ev))
            self._last = ev
        else:
            now = time.perf_counter()
            if self._last is not None:
                self._pending.append((self._last, now))
            self._last = now

    def reset(self):
        self._last = None
        self._pending = []

    def collect(self) -> List[float]:
        """Seconds per step since the last collect (blocks on the device)."""
        out = []
        if self.cuda and self._pending:
            self._pending[-1][1].synchronize()
            out = [a.elapsed_time(b) / 1e3 for a, b in self._pending]
        elif self._pending:
            out = [b - a for a, b in self._pending]
        self._pending = []
        return out


class BenchmarkCNN:
    """Class for benchmarking a cnn network."""

    def __init__(self, params, dataset=None, model=None):
        self.params = params
        validate_params_combinations(params)
        self._doing_eval = params.eval
        self.dataset = dataset or datasets.create_dataset(params.data_dir, params.data_name)
        self.model = model or model_config.get_model_config(params.model, self.dataset, params)
        autotune_threshold = params.autotune_threshold or 1
        min_autotune_warmup = 5 * autotune_threshold * autotune_threshold
        self.num_warmup_batches = (params.num_warmup_batches
                                   if params.num_warmup_batches is not None
                                   else max(10, min_autotune_warmup))
        self.trace_filename = params.trace_file
        self.num_gpus = params.num_gpus
        if params.gpu_indices:
            self.gpu_indices = [int(x) for x in params.gpu_indices.split(",")]
        else:
            self.gpu_indices = list(range(self.num_gpus))
        if params.batch_size > 0:
            self.model.set_batch_size(params.batch_size)
        per_device_batch = self.model.get_batch_size()
        self.batch_size = per_device_batch * self.num_gpus
        self.batch_group_size = params.batch_group_size
        self.enable_auto_loss_scale = params.use_fp16 and params.fp16_enable_auto_loss_scale
        self.mode = get_mode_from_params(params)
        self.job_name = params.job_name

        # ---- world & devices: one process per GPU.  --num_gpus=N in one
        # command is run as N "tower" processes (cli.py relaunches through
        # kfb-run with KFB_TOWER_GROUP=1): each tower is a rank, but the job
        # reports as ONE worker with an N-device global batch, as the
        # reference's in-process towers do (tcb/benchmark_cnn.py:1355-1357).
        self.device_type = "cuda" if params.device.lower() == "gpu" else "cpu"
        if self.device_type == "cuda" and not torch.cuda.is_available():
            raise RuntimeError("--device=gpu but no GPU is visible; use --device=cpu "
                               "--data_format=NHWC for the plumbing config")
        self.cluster_manager = None
        if params.job_name:
            from .platforms import util as platforms_util
            self.cluster_manager = platforms_util.get_cluster_manager(params)
            if params.job_name in ("ps", "controller"):
                # stateless roles: no world, no device (see join_server)
                self.world = comm.World()
                self.num_workers = self.cluster_manager.num_workers()
                self.num_replicas, self.task_index = self.num_workers, params.task_index
                self.tower_mode = False
                self.local_batch_size = self.batch_size
                self.device = torch.device("cpu")
                self.devices = ["/job:%s/task:%d/cpu:0" % (params.job_name, params.task_index)]
                self.num_batches, self.num_epochs = get_num_batches_and_epochs(
                    params, self.batch_size * self.num_workers,
                    self.dataset.num_examples_per_epoch("train"))
                self.compute_dtype = self.model.data_type
                self.ignored_flags = []
                self._built = False
                self.global_step = 0
                self.loss_scale = None
                self.benchmark_logger = None
                return
            self.cluster_manager.setup_worker_env()
        # the compute GPU and the RCCL communicator's GPU come from ONE
        # function (comm.select_device_index), decided before the world exists
        env_size = comm.env_world_size()
        # (KFB_FORCE_PG=1 with one rank: the GPU tests' single-tower stand-in
        # for the mode, over a real 1-rank RCCL group)
        self.tower_mode = (os.environ.get("KFB_TOWER_GROUP") == "1" and self.num_gpus > 1
                           and (env_size == self.num_gpus or (env_size == 1 and comm.force_pg())))
        dev_index = None
        if self.device_type == "cuda":
            dev_index = comm.select_device_index(self.gpu_indices, self.num_gpus, self.tower_mode,
                                                 comm.env_local_rank(), env_size,
                                                 torch.cuda.device_count())
        self.world = comm.init_world(self.device_type, params.all_reduce_spec,
                                     channels=params.rccl_channels, device_index=dev_index)
        self.task_index = self.world.rank
        self.num_replicas = self.world.size  # data shards / gradient contributors
        if self.tower_mode:
            self.num_workers = 1
            self.local_batch_size = per_device_batch
        else:
            self.num_workers = self.world.size
            self.local_batch_size = self.batch_size
            if self.num_gpus > 1:
                # no launcher: the towers' batches run as one batch on one
                # device (tower-mean gradient; see Strategy.tower_factor)
                self.model.set_batch_size(self.batch_size)
        if self.device_type == "cuda":
            torch.cuda.set_device(dev_index)
            self.device = torch.device("cuda", dev_index)
            _native.load()  # fail loudly now if the kernels are missing
        else:
            self.device = torch.device("cpu")
        if params.variable_update == "kungfu":
            self.devices = ["kungfu/gpu:%d" % i for i in range(self.num_gpus)]
        elif self.device_type == "cuda":
            self.devices = ["/gpu:%d" % i for i in self.gpu_indices[:self.num_gpus]]
        else:
            self.devices = ["/cpu:0"]
        if self.num_workers > 1 and params.all_reduce_spec == "nccl":
            raise ValueError("--all_reduce_spec=nccl is invalid in a multi-worker job")
        self.num_batches, self.num_epochs = get_num_batches_and_epochs(
            params, self.batch_size * self.num_workers,
            self.dataset.num_examples_per_epoch("train"))
        if params.eval:
            nb = params.num_eval_batches
            ne = params.num_eval_epochs
            self.num_batches, self.num_epochs = get_num_batches_and_epochs(
                params_lib.Params(**{**params._asdict(), "num_batches": nb, "num_epochs": ne}),
                self.batch_size * self.num_workers,
                self.dataset.num_examples_per_epoch("validation"))
        self.compute_dtype = self.model.data_type
        self.loss_scale = None
        if params.use_fp16:
            self.loss_scale = (params.fp16_loss_scale if params.fp16_loss_scale is not None
                               else self.model.get_fp16_loss_scale())
        self.loss_scale_normal_steps = 0
        self.benchmark_logger = None
        if params.benchmark_log_dir:
            from .utils.logger import BenchmarkFileLogger
            self.benchmark_logger = BenchmarkFileLogger(params.benchmark_log_dir,
                                                        params.benchmark_test_id)
        self.ignored_flags = [f for f in IGNORED_TF_FLAGS
                              if getattr(params, f) != flags.param_specs[f].default_value]
        self._built = False
        self.global_step = 0

    # ------------------------------------------------------------------ info
    def _get_params_info(self):
        if self.params.variable_update == "kungfu":
            return "kungfu/" + ",".join(self.devices)
        return str(self.devices)

    def print_info(self):
        p = self.params
        log_fn("Model:       %s" % self.model.get_model_name())
        ds = str(self.dataset)
        if self.dataset.use_synthetic_gpu_inputs():
            ds += " (synthetic)"
        log_fn("Dataset:     %s" % ds)
        log_fn("Mode:        %s" % self.mode)
        log_fn("SingleSess:  %s" % False)
        log_fn("Batch size:  %s global" % (self.batch_size * self.num_workers))
        log_fn("             %s per device" % (self.batch_size / len(self.devices)))
        if self.batch_group_size > 1:
            log_fn("             %d batches per prepocessing group" % self.batch_group_size)
        log_fn("Num batches: %d" % self.num_batches)
        log_fn("Num epochs:  %.2f" % self.num_epochs)
        log_fn("Devices:     %s" % self.devices)
        log_fn("NUMA bind:   %s" % False)
        log_fn("Data format: %s" % p.data_format)
        if self.device_type == "cuda":
            log_fn("Compute:     %s on %s (NHWC, %s kernels)"
                   % (str(self.compute_dtype).replace("torch.", ""),
                      torch.cuda.get_device_name(self.device), p.kernel_impl))
        log_fn("Optimizer:   %s" % p.optimizer)
        log_fn("Variables:   %s" % p.variable_update)
        if p.variable_update in ("replicated", "distributed_all_reduce",
                                 "collective_all_reduce"):
            log_fn("AllReduce:   %s" % p.all_reduce_spec)
        if self.job_name:
            log_fn("Sync:        %s" % p.cross_replica_sync)
        if p.staged_vars:
            log_fn("Staged vars: %s" % p.staged_vars)
        if p.variable_update == "kungfu":
            log_fn("KungFu option:  %s" % p.kungfu_option)
        if self.ignored_flags:
            log_fn("Ignored TF-only flags: %s" % ", ".join(self.ignored_flags))
        log_fn("==========")

    # ----------------------------------------------------------------- build
    def build(self):
        if self._built:
            return
        p = self.params
        log_fn("Generating training model")
        seed = p.tf_random_seed
        torch.manual_seed(seed + self.task_index)
        np.random.seed(4321 + self.task_index)
        nclass = self.dataset.num_classes
        self.net = make_network(self.model, nclass, self.device, self.compute_dtype,
                           kernel_impl=p.kernel_impl, seed=seed)
        lp = self.compute_dtype if self.compute_dtype != torch.float32 else None
        self.flat = optim.FlatParams(self.net, lp)
        if p.staged_vars:
            self.flat.enable_staging()
        if self.device_type == "cuda" and lp is not None and p.kernel_impl == "hip":
            from .ops.conv_hip import DgradWeights
            dgw = DgradWeights(self.net, self.flat)
            self.flat.add_update_hook(dgw.run)
        self.optimizer = optim.FusedOptimizer(
            self.flat, p.optimizer, momentum=p.momentum, rmsprop_decay=p.rmsprop_decay,
            rmsprop_momentum=p.rmsprop_momentum, rmsprop_epsilon=p.rmsprop_epsilon,
            adam_beta1=p.adam_beta1, adam_beta2=p.adam_beta2, adam_epsilon=p.adam_epsilon)
        self.strategy = make_strategy(p, self.world, self.flat, self.tower_mode, self.num_gpus)
        keep = [bool(self.model.l2_param_filter(n)) for n in self.flat.names]
        self.l2_mask = None
        if not all(keep):
            mask = torch.zeros(self.flat.numel, dtype=torch.float32, device=self.device)
            for k, (_, _, off, n) in zip(keep, self.flat.segments()):
                if k:
                    mask[off:off + n] = 1.0
            self.l2_mask = mask
            if self.device_type == "cuda" and self.flat.master is None:
                # the update kernel applies the decay on the masked elements
                # itself (no torch op in the step: the launch tape can record it)
                self.optimizer.decay_mask = mask.to(torch.uint8)
        self.comm_selftest = self._validate_comm()
        self.input = self._make_input()
        self._tape = None
        self._tape_warm = 0
        self._tape_reason = self.tape_eligible() if p.launch_tape else "off"
        if p.launch_tape and self._tape_reason is not None:
            log_fn("launch tape: not used (%s)" % self._tape_reason)
        self._built = True

    def _validate_comm(self):
        p = self.params
        """Multi-rank runs on the native communicator: check it bitwise
        against torch's host group on this job's collective buffer sizes and
        dtypes (gradient buckets and their wire dtype, the whole model) before
        any step runs; KFB_NATIVE_COMM=auto falls back to torch's
        ProcessGroupNCCL (and so to eager steps) if it fails."""
        if self.world.native is None or not self.world.communicates:
            return None
        sizes = {1, self.flat.numel}
        dtypes = [torch.float32]
        r = getattr(self.strategy, "reducer", None)
        groups = []
        hier = getattr(r, "hierarchical", None) if r is not None else None
        if r is not None:
            sizes.update(e - s for s, e in r.buckets)
            if r.wire_dtype is not None:
                dtypes.append(r.wire_dtype)
            if hier is not None and hier.native is not None:
                # the two-level reduction's own native communicators
                g, lead = hier.native
                groups.append(("hier", g, g.rank, g.size))
                if lead is not None:
                    groups.append(("leaders", lead, lead.rank, lead.size))
        st = comm.validate_native(sorted(sizes), tuple(dtypes), groups=groups)
        if st is not None and st.get("fallback") and hier is not None \
                and hier.native is not None:
            # the strategy's reducer was built on native subgroups: rebuild
            # it on torch groups like the world's collectives (collective:
            # every rank shares the verdict)
            self.strategy.close()
            r.remove()
            self.strategy = make_strategy(p, self.world, self.flat, self.tower_mode,
                                          self.num_gpus)
            st["rebuilt_strategy"] = True
        if st is not None:
            log_fn("Native RCCL self-test: %s (%d checks%s)"
                   % ("passed" if st["ok"] else "FAILED", st["checked"],
                      "" if st["ok"] else "; " + ", ".join(st["failed"])))
        return st

    def _make_input(self):
        from .data.input_pipeline import make_input_source
        return make_input_source(self, subset="validation" if self._doing_eval else "train")

    def set_fake_data(self, images, labels):
        """Feed these NHWC numpy images/labels instead of synthetic or real
        data (tests; role of TestImagePreprocessor.set_fake_data)."""
        self.fake_data = (images, labels)

    # ------------------------------------------------------------------ step
    def l2_loss_value(self):
        """sum(w^2)/2 over the L2-regularized trainable variables (device scalar)."""
        w = self.flat.flat
        if self.l2_mask is not None:
            return 0.5 * (w * w * self.l2_mask).sum()
        if w.is_cuda:
            out = torch.zeros(1, dtype=torch.float32, device=w.device)
            _native.call("kfb_half_sumsq", w.data_ptr(), w.numel(), out.data_ptr(),
                         _native.stream(w.device))
            return out[0]
        return 0.5 * (w.double() ** 2).sum().float()

    def learning_rate(self, step=None):
        step = self.global_step if step is None else step
        ex = self.dataset.num_examples_per_epoch("train")
        return optim.get_learning_rate(self.params, step, ex, self.model,
                                       self.batch_size * self.num_workers)

    def forward_backward(self, inputs, need_accuracy=False):
        res = self.net.forward_inputs(inputs, phase_train=True)
        loss = self.model.loss_function(inputs, res)
        if loss.is_cuda:
            # the backward is seeded with the (static) loss scale: d(s*L) = s*dL,
            # from a persistent tensor (no fill or multiply kernel in the step)
            seed = getattr(self, "_loss_seed", None)
            val = float(self.loss_scale or 1.0)
            if seed is None or seed.device != loss.device or seed.dtype != loss.dtype \
                    or seed.shape != loss.shape or self._loss_seed_val != val:
                # (re)made only when the loss scale changes (dynamic loss scaling)
                seed = self._loss_seed = torch.full(loss.shape, val, dtype=loss.dtype,
                                                    device=loss.device)
                self._loss_seed_val = val
            loss.backward(seed)
        else:
            scaled = loss * self.loss_scale if self.loss_scale else loss
            scaled.backward()
        if self.device_type == "cuda":
            from .ops.conv_hip import join_wgrad_stream
            join_wgrad_stream(self.device)
        acc = None
        if need_accuracy:
            acc = self.model.accuracy_function(inputs, res.logits.detach())
        return loss.detach(), acc

    # ------------------------------------------------------------ launch tape
    def tape_eligible(self):
        """Why the step cannot be taped (None: it can).  The tape replays the
        native launches of one step; host logic that must run every step
        (collectives issued from Python, host-side data, loss-scale checks,
        global-step-dependent graphs) keeps a configuration eager."""
        p = self.params
        if self.device_type != "cuda" or p.kernel_impl != "hip":
            return "not a HIP device run"
        if self.world.communicates:
            if self.world.native is None and self.strategy.steps_use_collectives():
                return "device collectives go through torch.distributed (not recordable)"
            why = self.strategy.tape_blocker()
            if why is not None:
                return why
        if getattr(self, "fake_data", None):
            return "host-side input pipeline"
        if not self.dataset.use_synthetic_gpu_inputs():
            from .data.input_pipeline import PrefetchInput
            if not (isinstance(self.input, PrefetchInput) and self.input.tape_capable()):
                return "host-side input pipeline"
        if self.enable_auto_loss_scale:
            return "dynamic loss scaling reads the gradients on the host"
        if p.staged_vars or (self.l2_mask is not None and self.optimizer.decay_mask is None):
            return "staged variables / masked L2 use torch ops in the update"
        return None

    def _tape_values(self, step):
        vals = self.strategy.tape_pre(step)
        vals["lr"] = self.learning_rate(step)
        vals.update(self.optimizer.tape_values(vals["lr"]))
        vals.update(self.input.tape_values())
        vals.update(self.net.tape_dropout_values())
        return vals

    def _tape_step(self, need_loss, need_accuracy):
        """Replays (or records) the step; None = run it eagerly."""
        if need_accuracy:
            return None
        t = getattr(self, "_tape", None)
        phase = self.strategy.tape_phase(self.global_step)
        if t is not None and phase != self._tape_phase:
            # (e.g. ada_sgd's switch from model averaging to S-SGD): the
            # step's launch sequence changed, record it again
            t.close()
            t = self._tape = None
            log_fn("launch tape: strategy phase changed at step %d, re-recording"
                   % self.global_step)
        if t is None:
            if self._tape_warm < 2:  # autotune / arena sizing settle first
                self._tape_warm += 1
                return None
            why = self.strategy.tape_blocker()  # (state created after build)
            if why is not None:
                self._tape_reason = why
                log_fn("launch tape: not used (%s)" % why)
                return None
            self._tape_phase = phase
            from .ops.tape import StepTape, TapeError
            p = self.params
            l2 = None
            if need_loss and p.loss_type_to_report == "total_loss" and p.weight_decay:
                l2 = self.l2_loss_value()  # of the weights this step's forward reads
            self.net.tape_begin_recording()
            t = StepTape(self.device)
            try:
                try:
                    loss, acc = t.record(lambda: self._eager_train_step(False, False))
                finally:
                    self.net.tape_end_recording()
                if l2 is not None:
                    loss = loss + len(self.devices) * p.weight_decay * l2
            except TapeError as e:
                # the step itself ran to completion eagerly; stay eager from now on
                self._tape_reason = "recording failed: %s" % e
                log_fn("launch tape: not used (%s)" % self._tape_reason)
                t.close()
                if os.environ.get("KFB_TAPE_STRICT") == "1" or e.outputs is None:
                    raise
                return e.outputs
            self._tape = t
            self._tape_loss = t.outputs[0]
            self.input.tape_post()
            log_fn("launch tape: recorded %d native calls (per-step arguments: %s)"
                   % (len(t.recorder), ", ".join(t.recorder.keys()) or "none"))
            if need_loss and self.tower_mode:
                loss = self._tower_mean(loss)
            return loss, acc
        p = self.params
        step = self.global_step
        l2 = None
        if need_loss and p.loss_type_to_report == "total_loss" and p.weight_decay:
            l2 = self.l2_loss_value()  # of the weights this step's forward reads
        self.input.tape_advance()
        self.net.global_step = step  # NASNet drop-path schedule (tape_dropout_values)
        vals = self._tape_values(step)
        t.replay(vals)
        self.strategy.tape_post(step)
        self.input.tape_post()
        self.global_step += 1
        loss = self._tape_loss
        if l2 is not None:
            loss = loss + len(self.devices) * p.weight_decay * l2
        if need_loss and self.tower_mode:
            loss = self._tower_mean(loss)
        return loss, None

    def _tower_mean(self, loss):
        """The reported loss of one worker is the mean over its towers (the
        tower processes): a one-element all-reduce outside the recorded step,
        issued by every tower at the same steps (the display schedule)."""
        lt = loss.detach().reshape(1).float().clone()
        comm.all_reduce(lt)
        return lt[0] / self.world.size

    def train_step(self, need_loss=False, need_accuracy=False):
        """One full training step; returns (loss_tensor, accuracy_dict)."""
        # multi-rank runs: the step must come back within KFB_COMM_TIMEOUT_S
        # (first steps: autotuning and tape recording get longer)
        watchdog.beat("step", self.global_step, startup=self.global_step < 4)
        if self.params.launch_tape and self._tape_reason is None:
            r = self._tape_step(need_loss, need_accuracy)
            if r is not None:
                return r
        return self._eager_train_step(need_loss, need_accuracy)

    def _eager_train_step(self, need_loss=False, need_accuracy=False):
        p = self.params
        inputs = tuple(self.input.next())
        self.net.global_step = self.global_step  # NASNet drop-path schedule
        self.flat.zero_grad()
        step = self.global_step
        self.strategy.before_backward(step)
        self._early_hi = 0
        early_args = self._early_update_args(step)
        if early_args is not None:
            from .ops import nn as F
            F._BACKWARD_TAIL_HOOK = lambda g, b: self._early_update(early_args, g, b)
        loss, acc = self.forward_backward(inputs, need_accuracy)
        if early_args is not None:
            from .ops import nn as F
            F._BACKWARD_TAIL_HOOK = None
        self.strategy.after_backward(step)
        if need_loss and p.loss_type_to_report == "total_loss" and p.weight_decay:
            # the reported total loss uses the weights of this step's forward
            loss = loss + len(self.devices) * p.weight_decay * self.l2_loss_value()
        if need_loss and self.tower_mode:
            loss = self._tower_mean(loss)
        grad_scale = self.strategy.grad_scale
        if self.loss_scale:
            grad_scale /= self.loss_scale
        skip = False
        if self.enable_auto_loss_scale:
            skip = self._auto_loss_scale_check()
        if not skip:
            self.strategy.before_update(step)
            try:
                wd = (p.weight_decay or 0.0) * self._l2_multiplier()
                if self.strategy.update_is_empty:
                    wd = 0.0
                if wd and self.l2_mask is not None and self.optimizer.decay_mask is None:
                    # model-specific L2 subset (custom_l2_loss, e.g. SSD without
                    # batch-norm variables): add wd * w on the masked elements
                    # before the gradient scale the optimizer applies
                    self.flat.grad.addcmul_(self.l2_mask, self.flat.flat, value=wd / grad_scale)
                    wd = 0.0
                elif wd and self.flat.master is not None:
                    # staged_vars: the L2 loss is over the staged (read) values,
                    # so its gradient uses them, not the master being updated
                    self.flat.grad.add_(self.flat.flat, alpha=wd / grad_scale)
                    wd = 0.0
                mix, wout = self.strategy.fused_update()
                self.optimizer.step(self.learning_rate(step), grad_scale=grad_scale,
                                    weight_decay=wd, clip=p.gradient_clip, mix=mix, wout=wout,
                                    lo=self._early_hi)
            except BaseException:
                self.strategy.abort_update(step)
                raise
            self.strategy.after_update(step)
        self.global_step += 1
        return loss, acc

    # The update of all but the stem's variables on the weight-gradient stream
    # beside the stem's backward: off.  Both are HBM-bound (the update moves
    # ~560 MB on ResNet-50), so the overlap saves nothing and the split costs
    # 0.08 ms/step (profiles/r8_early_update_ab.txt)
    _EARLY_UPDATE = False

    def _early_update_args(self, step):
        """The optimizer arguments of this step's update if part of it may run
        early (one GPU, a plain synchronous strategy, no host-side gradient
        logic), else None."""
        from .parallel.variable_mgr import (IndependentStrategy, KungFuSyncSGD,
                                            SumAllReduceStrategy)
        p = self.params
        s = self.strategy
        if not self._EARLY_UPDATE or self.device_type != "cuda" or self.tower_mode \
                or type(s) not in (KungFuSyncSGD, SumAllReduceStrategy, IndependentStrategy) \
                or s.reducer is not None or self.world.communicates \
                or self.enable_auto_loss_scale or self.loss_scale \
                or self.l2_mask is not None or self.flat.master is not None:
            return None
        wd = (p.weight_decay or 0.0) * self._l2_multiplier()
        return dict(lr=self.learning_rate(step), grad_scale=s.grad_scale, weight_decay=wd,
                    clip=p.gradient_clip)

    def _early_update(self, args, gamma, beta):
        """Runs the update of every variable before the stem's in flat order
        (their gradients are final: they come earlier in the backward) on the
        weight-gradient stream, beside the stem's backward; the update after
        the backward then covers the stem's variables only."""
        from .ops import conv_hip
        f = self.flat
        offs = {id(q): o for q, o in zip(f.params, f.offsets)}
        tail = [offs.get(id(t)) for t in (gamma, beta) if t is not None]
        if not tail or None in tail:
            return
        hi = min(tail)
        if sum(1 for o in f.offsets if o >= hi) > 3:  # stem BN gamma/beta + stem conv only
            return
        side = conv_hip.wgrad_stream(self.device)
        if side is None:
            return
        # gradients of the range written on the compute stream are enqueued
        # before this point; the side stream's own wgrads precede it in order
        _native.stream_wait(side.cuda_stream, _native.stream(self.device), device_only=True)
        conv_hip._queue_join(self.device)
        with torch.cuda.stream(side):
            self.optimizer.step(args["lr"], grad_scale=args["grad_scale"],
                                weight_decay=args["weight_decay"], clip=args["clip"],
                                lo=0, hi=hi, advance=False)
        self._early_hi = hi

    def _l2_multiplier(self) -> float:
        """Copies of wd * w in the applied gradient.  The reference adds the
        L2 loss (x num_devices) on the last tower only and aggregates tower /
        worker gradients before applying (tcb/benchmark_cnn.py:3070-3099); the
        fused optimizer adds wd * w after grad_scale, so the multiplier is
        grad_scale x (L2 copies summed by the aggregation)."""
        s = self.strategy.grad_scale
        if self.tower_mode:
            return s * self.num_gpus
        if self.num_gpus > 1:
            return s
        return s * (self.world.size if self.strategy.aggregates_gradients else 1)

    def _auto_loss_scale_check(self) -> bool:
        """Dynamic loss scaling (tcb/variable_mgr_util.py:51-139): halve the
        scale and skip the update on inf/nan, double it after
        fp16_inc_loss_scale_every_n finite steps."""
        g = self.flat.grad
        if g.is_cuda:
            flag = torch.zeros(1, dtype=torch.int32, device=g.device)
            _native.call("kfb_nonfinite", g.data_ptr(), g.numel(), flag.data_ptr(),
                         _native.stream(g.device))
            bad = bool(flag.item())
        else:
            bad = not bool(torch.isfinite(g).all())
        if bad:
            self.loss_scale = max(self.loss_scale / 2.0, 1.0)
            self.loss_scale_normal_steps = 0
            return True
        self.loss_scale_normal_steps += 1
        if self.loss_scale_normal_steps >= self.params.fp16_inc_loss_scale_every_n:
            self.loss_scale *= 2.0
            self.loss_scale_normal_steps = 0
        return False

    def forward_only_step(self):
        watchdog.beat("forward", self.global_step, startup=self.global_step < 4)
        inputs = tuple(self.input.next())
        with torch.no_grad():
            res = self.net.forward_inputs(inputs, phase_train=False)
        return res

    # ------------------------------------------------------------------- run
    def run(self):
        # (a high-priority compute stream, dispatching ahead of the
        # weight-gradient side stream, measured neutral and is not used)
        return self._run()

    def _run(self):
        if self.params.job_name in ("ps", "controller"):
            log_fn("Running %s %d: waiting for the workers to finish"
                   % (self.params.job_name, self.params.task_index))
            self.cluster_manager.join_server()
            return {}
        if self._doing_eval:
            from .eval import run_eval
            return run_eval(self)
        return self._benchmark_train()

    def _benchmark_train(self):
        p = self.params
        self.build()
        log_fn("Initializing graph")
        from .utils import checkpoint as ckpt_lib
        self.saver = ckpt_lib.Saver(self, max_to_keep=p.max_ckpts_to_keep)
        if p.train_dir and os.path.isdir(p.train_dir):
            restored = self.saver.restore_latest(p.train_dir)
            if restored is not None:
                log_fn("Restored checkpoint at global step %d" % restored)
        if p.backbone_model_path:
            self.saver.restore_partial(p.backbone_model_path)
        self.strategy.broadcast_initial_model(self.optimizer.slot_tensors().values())
        init_global_step = self.global_step
        eval_hook = None
        if self.mode == BenchmarkMode.TRAIN_AND_EVAL:
            from .eval import EvalDuringTraining
            eval_hook = EvalDuringTraining(self)
        from .utils.tracing import StepTracer
        tracer = StepTracer(self)
        self.summary_writer = None
        if (p.summary_verbosity > 0 and p.save_summaries_steps > 0 and p.train_dir
                and self.world.is_chief):
            from .utils.summary import SummaryWriter
            self.summary_writer = SummaryWriter(p.train_dir)
        timer = _EventTimer(self.device)
        # asynchronous PS: the run is timed by the shared global step
        watcher = None
        if getattr(self.strategy, "state", None) is not None and \
                p.variable_update == "parameter_server" and not p.cross_replica_sync:
            from .parallel.async_ps import GlobalStepWatcher
            watcher = GlobalStepWatcher(self.strategy.state)
        step_train_times: List[float] = []
        forward_only = p.forward_only
        num_warmup = self.num_warmup_batches
        if self.batch_group_size > 1:
            num_warmup = (num_warmup + self.batch_group_size - 1) // self.batch_group_size * \
                self.batch_group_size
        total_steps = self.num_batches - (init_global_step if init_global_step else 0)
        if init_global_step and total_steps < 0:
            total_steps = 0
        log_fn("Running warm up")
        local_step = -1 * num_warmup
        done = False
        last_loss = None
        loop_start = None
        last_ckpt_time = time.time()
        header_printed = False
        while not done:
            if local_step == 0:
                log_fn("Done warm up")
                if not header_printed:
                    header = "Step\tImg/sec\t" + p.loss_type_to_report.replace("/", " ")
                    if p.print_training_accuracy:
                        header += "\ttop_1_accuracy\ttop_5_accuracy"
                    log_fn(header)
                    header_printed = True
                if self.device_type == "cuda":
                    torch.cuda.synchronize(self.device)
                self.world.barrier(self.device if self.device_type == "cuda" else None)
                loop_start = time.perf_counter()
                if watcher is not None:
                    watcher.start()
                step_train_times = []
                timer.reset()
                timer.mark()
            display = local_step >= 0 and (local_step == 0 or
                                           (local_step + 1) % p.display_every == 0)
            tracer.begin(local_step)
            if forward_only:
                self.forward_only_step()
                loss, acc = None, None
            else:
                want_sum = (p.summary_verbosity > 0 and p.save_summaries_steps > 0 and
                            (local_step + 1) % p.save_summaries_steps == 0)
                loss, acc = self.train_step(need_loss=display or want_sum or
                                            local_step >= total_steps - 1,
                                            need_accuracy=display and p.print_training_accuracy)
            tracer.end(local_step)
            if local_step >= 0:
                timer.mark()
            if (self.summary_writer is not None and local_step >= 0
                    and (local_step + 1) % p.save_summaries_steps == 0 and loss is not None):
                self._write_summaries(loss)
            if display:
                step_train_times.extend(timer.collect())
                if step_train_times:
                    lossval = float(loss) if loss is not None else 0.0
                    last_loss = lossval
                    self._log_step(local_step, step_train_times, lossval, acc)
            if local_step >= 0 and not forward_only:
                self._maybe_checkpoint(local_step, last_ckpt_time)
                if p.save_model_secs and time.time() - last_ckpt_time >= p.save_model_secs:
                    last_ckpt_time = time.time()
            if eval_hook is not None and local_step >= 0:
                watchdog.beat("eval", self.global_step, startup=True)
                if eval_hook.maybe_eval(self.global_step):
                    done = True
            local_step += 1
            if local_step >= total_steps:
                done = True
        watchdog.beat("final_sync", self.global_step)
        step_train_times.extend(timer.collect())
        if self.device_type == "cuda":
            torch.cuda.synchronize(self.device)
        elapsed = time.perf_counter() - (loop_start or time.perf_counter())
        num_steps = local_step
        images_per_sec = (self.num_workers * num_steps * self.batch_size / elapsed
                          if elapsed > 0 else 0.0)
        if watcher is not None and watcher.start_step is not None:
            watcher.stop()
            images_per_sec = watcher.steps_per_second() * self.batch_size
        log_fn("-" * 64)
        log_fn("total images/sec: %.2f" % images_per_sec)
        log_fn("-" * 64)
        if self.benchmark_logger:
            self.benchmark_logger.log_metric("average_examples_per_sec", images_per_sec,
                                             global_step=num_steps)
        watchdog.beat("finish", self.global_step, startup=True)
        if p.train_dir and self.world.is_chief and not forward_only:
            self.saver.save(p.train_dir, self.global_step)
        tracer.finish()
        self.strategy.close()
        if getattr(self, "input", None) is not None:
            self.input.close()
        if self.cluster_manager is not None:
            self.world.barrier(self.device if self.device_type == "cuda" else None)
            if self.world.is_chief:
                self.cluster_manager.mark_done()
        if self.summary_writer is not None:
            self.summary_writer.close()
        if p.variable_update == "kungfu" or p.sync_on_finish:
            self.world.barrier(self.device if self.device_type == "cuda" else None)
        if last_loss is None and loss is not None:
            last_loss = float(loss)
        watchdog.pause()  # no collective after this point
        stats = {"num_workers": self.num_workers, "num_steps": num_steps,
                 "average_wall_time": elapsed / num_steps if num_steps > 0 else 0,
                 "images_per_sec": images_per_sec}
        if last_loss is not None:
            stats["last_average_loss"] = last_loss
        if watcher is not None and watcher.end_step is not None:
            stats["ps_global_step"] = watcher.end_step
        if eval_hook is not None:
            stats.update(eval_hook.stats())
        if p.print_json_result and self.world.is_chief:
            print(json.dumps(stats))
        return stats

    def _write_summaries(self, loss):
        """Scalars (verbosity>=1), log|grad| histogram (>=2), per-variable and
        per-gradient histograms (>=3), as tcb/benchmark_cnn.py:2811-2846."""
        p = self.params
        step = self.global_step
        scalars = {"learning_rate": self.learning_rate(step - 1),
                   p.loss_type_to_report: float(loss)}
        if self.loss_scale is not None:
            scalars["loss_scale"] = float(self.loss_scale)
        if self.loss_scale_normal_steps:
            scalars["loss_scale_normal_steps"] = float(self.loss_scale_normal_steps)
        self.summary_writer.add_scalars(scalars, step)
        if p.summary_verbosity >= 2:
            g = self.flat.grad.detach().abs()
            g = g[g != 0].float().log().cpu().numpy()
            self.summary_writer.add_histograms({"log_gradients": g}, step)
        if p.summary_verbosity >= 3:
            hists = {}
            for name, param, off, n in self.flat.segments():
                hists[name + "/gradients"] = self.flat.grad[off:off + n].detach().cpu().numpy()
                hists[name] = param.detach().cpu().numpy()
            self.summary_writer.add_histograms(hists, step)

    def _log_step(self, local_step, step_train_times, lossval, acc):
        p = self.params
        speed_mean, speed_unc, speed_jit = get_perf_timing(self.batch_size, step_train_times)
        log_str = "%i\t%s\t%.*f" % (local_step + 1,
                                    get_perf_timing_str(speed_mean, speed_unc, speed_jit),
                                    LOSS_AND_ACCURACY_DIGITS_TO_SHOW, lossval)
        if acc is not None:
            n = float(self.batch_size)
            log_str += "\t%.*f\t%.*f" % (LOSS_AND_ACCURACY_DIGITS_TO_SHOW,
                                         float(acc["top_1_accuracy"]) / n,
                                         LOSS_AND_ACCURACY_DIGITS_TO_SHOW,
                                         float(acc["top_5_accuracy"]) / n)
        log_fn(log_str)
        if self.benchmark_logger:
            self.benchmark_logger.log_metric("current_examples_per_sec", speed_mean,
                                             global_step=local_step + 1)

    def _maybe_checkpoint(self, local_step, last_ckpt_time):
        p = self.params
        if not p.train_dir or not self.world.is_chief:
            return
        if p.save_model_steps and self.global_step % p.save_model_steps == 0:
            self.saver.save(p.train_dir, self.global_step)
        elif p.save_model_secs and time.time() - last_ckpt_time >= p.save_model_secs:
            self.saver.save(p.train_dir, self.global_step)


def setup(params):
    """Process-level setup (tcb/benchmark_cnn.py:3356-3395): thread counts and
    environment.  No session to create on this stack."""
    if params.num_intra_threads:
        torch.set_num_threads(params.num_intra_threads)
    if params.num_inter_threads:
        try:
            torch.set_num_interop_threads(params.num_inter_threads)
        except RuntimeError:
            pass
    if params.mkl:
        os.environ["KMP_BLOCKTIME"] = str(params.kmp_blocktime)
        os.environ["KMP_SETTINGS"] = str(params.kmp_settings)
        os.environ["KMP_AFFINITY"] = params.kmp_affinity
    return params


def make_params(**kwargs):
    return params_lib.make_params(**kwargs)


def make_params_from_flags(argv=None):
    return params_lib.make_params_from_flags(argv)
