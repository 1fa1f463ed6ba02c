"""The benchmark's full flag surface and the immutable ``Params`` tuple.

Every flag of ``tcb/benchmark_cnn.py:114-634`` is declared here with the same
name, type, default and enum values (129 flags), plus a short block of
MI355X-specific flags at the end (bucket sizing, bf16, hipGraph capture, ...).
TF-only knobs (xla, trt_mode, winograd_nonfused, mkl, ...) are accepted for CLI
compatibility and reported as ignored by the engine.

``make_params`` / ``make_params_from_flags`` / ``validate_params`` /
``remove_param_fields`` mirror ``tcb/benchmark_cnn.py:953-1034``.
"""

from __future__ import annotations

import collections
import sys
from typing import Any, Dict, Optional, Sequence

from . import flags
from .constants import NetworkTopology

D = flags

# --------------------------------------------------------------------------
# Model / mode
D.DEFINE_string("model", "trivial", "Model to run; see models/model_config.py for the list.")
D.DEFINE_boolean("eval", False, "Evaluate a saved checkpoint instead of training.")
D.DEFINE_integer("eval_interval_secs", 0,
                 "Seconds between evaluations of new checkpoints; 0 evaluates once.")
D.DEFINE_integer("eval_during_training_every_n_steps", None,
                 "Pause training every n steps to run evaluation.", lower_bound=1)
D.DEFINE_float("eval_during_training_every_n_epochs", None,
               "Pause training every n epochs to run evaluation.")
D.DEFINE_list("eval_during_training_at_specified_steps", [],
              "Global steps at which to run evaluation during training.")
D.DEFINE_list("eval_during_training_at_specified_epochs", [],
              "Epochs at which to run evaluation during training.")
D.DEFINE_boolean("forward_only", False, "Benchmark only the forward pass.")
D.DEFINE_boolean("freeze_when_forward_only", False,
                 "Freeze the model before forward-only benchmarking (no-op on this stack).")
D.DEFINE_boolean("print_training_accuracy", False,
                 "Report top-1/top-5 training accuracy on each display step.")
# Batching
D.DEFINE_integer("batch_size", 0, "Per-device batch size; 0 uses the model's default.")
D.DEFINE_integer("batch_group_size", 1, "Batches staged together by the input producer.")
D.DEFINE_integer("num_batches", None, "Number of timed batches (default 100).")
D.DEFINE_integer("num_eval_batches", None, "Number of eval batches.")
D.DEFINE_float("num_epochs", None, "Epochs to run (exclusive with --num_batches).")
D.DEFINE_float("num_eval_epochs", None, "Eval epochs to run.")
D.DEFINE_float("stop_at_top_1_accuracy", None,
               "Stop training once eval top-1 accuracy reaches this value.")
D.DEFINE_integer("num_warmup_batches", None, "Untimed warmup batches.")
D.DEFINE_integer("autotune_threshold", None, "Kernel autotune threshold.")
D.DEFINE_integer("num_gpus", 1, "Devices (towers) driven by this process.")
D.DEFINE_string("gpu_indices", "", "Comma list of device indices to use (ring order).")
D.DEFINE_integer("display_every", 10, "Print a step line every n steps.")
# Data
D.DEFINE_string("data_dir", None, "Directory of TFRecord shards; synthetic data if unset.")
D.DEFINE_string("data_name", None, "Dataset name (imagenet, cifar10, coco, librispeech).")
D.DEFINE_string("resize_method", "bilinear",
                "Resize method: crop, nearest, bilinear, bicubic, area, round_robin.")
D.DEFINE_boolean("distortions", True, "Apply random training distortions.")
D.DEFINE_boolean("use_datasets", True, "Use the dataset pipeline for real input.")
D.DEFINE_string("input_preprocessor", "default", "Name of the input preprocessor.")
D.DEFINE_string("gpu_thread_mode", "gpu_private", "GPU thread mode (TF knob; ignored).")
D.DEFINE_integer("per_gpu_thread_count", 0, "Threads per GPU (TF knob; ignored).")
D.DEFINE_boolean("hierarchical_copy", False,
                 "Two-level reduce for --variable_update=replicated.")
D.DEFINE_enum("network_topology", NetworkTopology.DGX1,
              (NetworkTopology.DGX1, NetworkTopology.GCP_V100, NetworkTopology.XGMI_MESH),
              "Topology used by --hierarchical_copy.")
D.DEFINE_integer("gradient_repacking", 0,
                 "Concat all grads and re-split into this many packs before all-reduce.",
                 lower_bound=0)
D.DEFINE_boolean("compact_gradient_transfer", True,
                 "Send repacked gradients at half precision.")
D.DEFINE_enum("variable_consistency", "strong", ("strong", "relaxed"),
              "relaxed applies gradients one step late (overlapped all-reduce).")
D.DEFINE_boolean("datasets_repeat_cached_sample", False,
                 "Repeat one cached sample forever (input-pipeline benchmark).")
D.DEFINE_enum("local_parameter_device", "gpu", ("cpu", "gpu", "CPU", "GPU"),
              "Device holding the shared parameters in parameter_server mode.")
D.DEFINE_enum("device", "gpu", ("cpu", "gpu", "CPU", "GPU"), "Compute device.")
D.DEFINE_enum("data_format", "NCHW", ("NHWC", "NCHW"),
              "Requested layout; kernels always run NHWC internally.")
D.DEFINE_integer("num_intra_threads", None, "Host intra-op threads.")
D.DEFINE_integer("num_inter_threads", 0, "Host inter-op threads.")
D.DEFINE_string("trace_file", "", "Write a Chrome trace of one warmup step here.")
D.DEFINE_boolean("use_chrome_trace_format", True, "Chrome JSON trace (else raw event list).")
D.DEFINE_string("tfprof_file", None, "Profile the first steps and write a top-ops table.")
D.DEFINE_string("graph_file", None, "Write a textual model description here.")
D.DEFINE_string("partitioned_graph_file_prefix", None,
                "Write per-device model descriptions with this prefix.")
# Optimizer / LR
D.DEFINE_enum("optimizer", "sgd", ("momentum", "sgd", "rmsprop", "adam"), "Optimizer.")
D.DEFINE_float("init_learning_rate", None, "Initial learning rate.")
D.DEFINE_string("piecewise_learning_rate_schedule", None,
                "'lr0;epoch1;lr1;...;epochN;lrN' piecewise-constant schedule.")
D.DEFINE_float("num_epochs_per_decay", 0, "Epochs between exponential decays.")
D.DEFINE_float("learning_rate_decay_factor", 0, "Exponential decay factor.")
D.DEFINE_float("num_learning_rate_warmup_epochs", 0, "Linear LR warmup epochs.")
D.DEFINE_float("minimum_learning_rate", 0, "Floor for the decayed learning rate.")
D.DEFINE_float("momentum", 0.9, "Momentum for momentum/rmsprop.")
D.DEFINE_float("rmsprop_decay", 0.9, "RMSProp decay.")
D.DEFINE_float("rmsprop_momentum", 0.9, "RMSProp momentum.")
D.DEFINE_float("rmsprop_epsilon", 1.0, "RMSProp epsilon.")
D.DEFINE_float("adam_beta1", 0.9, "Adam beta1.")
D.DEFINE_float("adam_beta2", 0.999, "Adam beta2.")
D.DEFINE_float("adam_epsilon", 1e-8, "Adam epsilon.")
D.DEFINE_float("gradient_clip", None, "Clip gradients to [-x, x].")
D.DEFINE_float("weight_decay", 0.00004, "L2 weight decay.")
D.DEFINE_float("gpu_memory_frac_for_testing", 0,
               "Cap device memory for tests (0 = no cap).", lower_bound=0.0, upper_bound=1.0)
D.DEFINE_boolean("use_unified_memory", False, "Unified memory (ignored).")
D.DEFINE_boolean("use_tf_layers", True, "Layer-library flag (kept for compatibility).")
D.DEFINE_integer("tf_random_seed", 1234, "Random seed (offset by the worker rank).")
D.DEFINE_string("debugger", None, "Debugger hook (ignored on this stack).")
D.DEFINE_boolean("use_python32_barrier", False, "Python barrier implementation knob.")
D.DEFINE_boolean("datasets_use_prefetch", True, "Prefetch input batches.")
D.DEFINE_integer("datasets_prefetch_buffer_size", 1, "Batches to prefetch per device.")
D.DEFINE_integer("datasets_num_private_threads", None, "Decoder threads for the input pipeline.")
D.DEFINE_boolean("datasets_use_caching", False, "Cache decoded records in memory.")
D.DEFINE_integer("datasets_parallel_interleave_cycle_length", None,
                 "Shards read concurrently.")
D.DEFINE_boolean("datasets_sloppy_parallel_interleave", False,
                 "Allow out-of-order shard interleave.")
D.DEFINE_integer("datasets_parallel_interleave_prefetch", None,
                 "Records prefetched per interleaved shard.")
D.DEFINE_boolean("use_multi_device_iterator", True, "One iterator feeding all towers.")
D.DEFINE_integer("multi_device_iterator_max_buffer_size", 1, "Per-device buffer size.")
D.DEFINE_boolean("winograd_nonfused", True, "cuDNN knob (ignored).")
D.DEFINE_boolean("batchnorm_persistent", True, "cuDNN knob (ignored).")
D.DEFINE_boolean("sync_on_finish", False, "Synchronize all workers at the end.")
D.DEFINE_boolean("staged_vars", False, "Pipeline parameter reads one step ahead (PS mode).")
D.DEFINE_boolean("force_gpu_compatible", False, "Pinned host buffers (ignored).")
D.DEFINE_boolean("allow_growth", None, "Grow device memory on demand (ignored).")
D.DEFINE_boolean("xla", False, "XLA auto-jit (ignored).")
D.DEFINE_boolean("xla_compile", False, "XLA compile (ignored).")
D.DEFINE_boolean("fuse_decode_and_crop", True, "Decode only the crop window.")
D.DEFINE_boolean("distort_color_in_yiq", True, "Color distortion in YIQ space.")
D.DEFINE_boolean("enable_optimizations", True, "Graph optimizations (ignored).")
D.DEFINE_string("rewriter_config", None, "Grappler config (ignored).")
D.DEFINE_enum("loss_type_to_report", "total_loss", ("base_loss", "total_loss"),
              "Which loss is printed.")
D.DEFINE_boolean("single_l2_loss_op", False, "Compute the L2 loss over one concatenated vector.")
D.DEFINE_boolean("use_resource_vars", False, "Resource variables (ignored).")
D.DEFINE_boolean("compute_lr_on_cpu", False, "Compute the learning rate on the host.")
D.DEFINE_boolean("sparse_to_dense_grads", False, "Densify sparse gradients.")
D.DEFINE_boolean("mkl", False, "MKL knob (ignored).")
D.DEFINE_integer("kmp_blocktime", 0, "OpenMP knob.")
D.DEFINE_string("kmp_affinity", "granularity=fine,verbose,compact,1,0", "OpenMP knob.")
D.DEFINE_integer("kmp_settings", 1, "OpenMP knob.")
# Precision
D.DEFINE_boolean("use_fp16", False, "Compute in float16 (fp32 master weights).")
D.DEFINE_float("fp16_loss_scale", None, "Static loss scale for fp16 (model default if unset).")
D.DEFINE_boolean("fp16_vars", False, "Keep the variables themselves in fp16.")
D.DEFINE_boolean("fp16_enable_auto_loss_scale", False, "Dynamic loss scaling.")
D.DEFINE_integer("fp16_inc_loss_scale_every_n", 1000,
                 "Double the loss scale after this many finite steps.")
# Distribution
D.DEFINE_enum("variable_update", "parameter_server",
              ("parameter_server", "replicated", "distributed_replicated", "independent",
               "distributed_all_reduce", "collective_all_reduce", "horovod", "kungfu"),
              "Gradient aggregation / variable placement strategy.")
D.DEFINE_enum("kungfu_option", "sync_sgd", ("async_sgd", "sync_sgd", "ada_sgd", "sma"),
              "KungFu distributed optimizer.")
D.DEFINE_string("all_reduce_spec", None,
                "All-reduce spec 'alg#shards:limit:alg...' (nccl, xring, pscpu, psgpu, collective).")
D.DEFINE_integer("agg_small_grads_max_bytes", 0, "Pack tensors smaller than this.")
D.DEFINE_integer("agg_small_grads_max_group", 10, "Max tensors per small-grad pack.")
D.DEFINE_integer("allreduce_merge_scope", 1, "Grads merged per all-reduce scope.")
D.DEFINE_enum("job_name", "", ("ps", "worker", "controller", ""), "Distributed job role.")
D.DEFINE_string("ps_hosts", "", "Comma list of parameter-server host:port.")
D.DEFINE_string("worker_hosts", "", "Comma list of worker host:port.")
D.DEFINE_string("controller_host", None, "Controller host:port.")
D.DEFINE_integer("task_index", 0, "Index of this task within its job.")
D.DEFINE_string("server_protocol", "grpc", "Transport (tcp rendezvous on this stack).")
D.DEFINE_boolean("cross_replica_sync", True, "Synchronous updates across workers.")
D.DEFINE_string("horovod_device", "", "Device for horovod all-reduce.")
# Checkpoint / summaries
D.DEFINE_integer("summary_verbosity", 0, "0: none, 1: scalars, 2: +grad hist, 3: +all hist.")
D.DEFINE_integer("save_summaries_steps", 0, "Write summaries every n steps.")
D.DEFINE_integer("save_model_secs", 0, "Checkpoint every n seconds.")
D.DEFINE_integer("save_model_steps", None, "Checkpoint every n steps.")
D.DEFINE_integer("max_ckpts_to_keep", 5, "Checkpoints retained.")
D.DEFINE_string("train_dir", None, "Checkpoint / summary directory.")
D.DEFINE_string("eval_dir", "/tmp/tf_cnn_benchmarks/eval", "Eval summary directory.")
D.DEFINE_string("backbone_model_path", None, "Partially restore from this checkpoint.")
D.DEFINE_enum("trt_mode", "", ["", "FP32", "FP16", "INT8"], "TensorRT mode (ignored).")
D.DEFINE_integer("trt_max_workspace_size_bytes", 4 << 30, "TensorRT workspace (ignored).")
D.DEFINE_string("benchmark_log_dir", None, "Write JSON benchmark logs here.")
D.DEFINE_string("benchmark_test_id", None, "Test id recorded in the benchmark log.")

# --------------------------------------------------------------------------
# Flags that only exist on this stack (MI355X-specific). Kept after the 129
# reference flags so the reference surface is a prefix of ours.
D.DEFINE_boolean("use_bf16", False, "Compute in bfloat16 (fp32 master weights). MI355X native.")
D.DEFINE_float("bucket_size_mb", 25.0,
               "Gradient bucket size for overlapped all-reduce (MB of fp32 gradient). "
               "Small enough that the last bucket (launched after backward, not "
               "overlapped) is short on an 8-GPU xGMI ring; large enough that each "
               "RCCL launch moves MBs.")
D.DEFINE_boolean("overlap_gradient_allreduce", True,
                 "Launch bucket all-reduces from backward hooks (overlap with compute).")
D.DEFINE_enum("gradient_wire_dtype", "auto", ("auto", "fp32", "bf16", "fp16"),
              "Dtype gradients travel in over RCCL; auto = fp16 under "
              "--compact_gradient_transfer with repacking, else fp32.")
D.DEFINE_integer("rccl_channels", 0,
                 "Pin the RCCL channel count (NCCL_MIN/MAX_NCHANNELS); 0 = RCCL's choice. "
                 "Each channel is one ring over the xGMI links.", lower_bound=0)
D.DEFINE_float("kungfu_sma_alpha", 0.1, "SMA: pull factor toward the model average.")
D.DEFINE_integer("kungfu_ada_switch_step", 100, "ada_sgd: step at which SMA switches to S-SGD.")
D.DEFINE_integer("kungfu_peer_seed", 0, "Seed for PairAveraging peer selection.")
D.DEFINE_boolean("launch_tape", False,
                 "Record one training step's native launches after warmup and replay them "
                 "from C++ every step (ops/tape.py): one Python call per step instead of one "
                 "per kernel. Single-process synthetic-data runs; other configurations "
                 "run eagerly.")
D.DEFINE_boolean("kungfu_pair_prefetch", True,
                 "PairAveraging: pull the peer model at the start of the step, overlapping "
                 "forward/backward (the averaged model is one step older than KungFu's); "
                 "false pulls it at update time, as KungFu's apply_gradients does.")
D.DEFINE_boolean("kungfu_pair_lockstep", False,
                 "PairAveraging, deterministic mode (tests/oracles): pull at update time, "
                 "every worker finishes its pull before any publishes, and every publish "
                 "commits before the next step, so the averaged peer model is exactly the "
                 "peer's model of the same step (costs two barriers per step).")
D.DEFINE_boolean("synthetic_resample", True,
                 "Re-sample the synthetic batch on device every step, inside the timed step "
                 "(as the fork's graph does; --nosynthetic_resample reuses one batch like "
                 "the original tf_cnn_benchmarks' gpu_cached_images).")
D.DEFINE_string("kernel_impl", "hip",
                "Compute-op implementation on GPU: 'hip' (our kernels) or 'torch' "
                "(stock PyTorch ops, for A/B comparison only).")
D.DEFINE_boolean("print_json_result", False, "Print the final stats dict as one JSON line.")

Params = collections.namedtuple("Params", list(flags.param_specs.keys()))

REFERENCE_FLAG_COUNT = 129


def validate_params(params) -> None:
    """Checks bounds and enum membership; raises ValueError."""
    for name, value in params._asdict().items():
        spec = flags.param_specs[name]
        if spec.flag_type in ("integer", "float") and value is not None:
            lo, hi = spec.kwargs.get("lower_bound"), spec.kwargs.get("upper_bound")
            if lo is not None and value < lo:
                raise ValueError("Param %s value of %s is lower than the lower bound of %s"
                                 % (name, value, lo))
            if hi is not None and hi < value:
                raise ValueError("Param %s value of %s is higher than the upper bound of %s"
                                 % (name, value, hi))
        elif spec.flag_type == "enum" and value is not None \
                and value not in spec.kwargs["enum_values"]:
            raise ValueError("Param %s of value %s is not in %s"
                             % (name, value, spec.kwargs["enum_values"]))


def default_values() -> Dict[str, Any]:
    return {n: s.default_value for n, s in flags.param_specs.items()}


def make_params(**kwargs) -> Params:
    """Params with defaults, overridden by kwargs; validated."""
    unknown = set(kwargs) - set(flags.param_specs)
    if unknown:
        raise ValueError("Unknown params: %s" % sorted(unknown))
    p = Params(**default_values())._replace(**kwargs)
    validate_params(p)
    return p


def make_params_from_flags(argv: Optional[Sequence[str]] = None) -> Params:
    """Parses argv (default ``sys.argv[1:]``) into a validated Params."""
    argv = sys.argv[1:] if argv is None else argv
    values = flags.parse_flags(argv)
    return make_params(**values)


def remove_param_fields(params, fields_to_remove):
    d = params._asdict()
    for f in fields_to_remove:
        assert f in d, "Invalid Params field: " + f
    d = {k: v for k, v in d.items() if k not in fields_to_remove}
    return collections.namedtuple("Params", d.keys())(**d)


def params_to_argv(params) -> list:
    return flags.to_argv(params._asdict())
