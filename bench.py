#!/usr/bin/env python3
"""Headline benchmark: whole-job ResNet-50 synthetic training images/sec.

Driver contract (one rank per GPU, launched by torch.distributed.run for
N > 1):  W untimed warmup steps, then EXACTLY K timed steps bracketed by a
barrier + device synchronize on both sides; the max elapsed over ranks is
used; rank 0 prints ONE JSON line.

Config (BASELINE.json): ResNet-50 v1 (with its final FC, 1001 classes),
bf16 compute with fp32 master weights, 256 images per GPU (weak scaling),
Nesterov momentum SGD, --variable_update=kungfu --kungfu_option=sync_sgd
(bucketed RCCL all-reduce overlapped with backward), synthetic ImageNet-shaped
data (224x224x3) and random-init weights.  Each timed step is a complete
training step: forward, backward, gradient all-reduce and optimizer update.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

# Reference numbers (fork's ResNet-50, fp32, RTX 3090; 4/8-GPU
# values are the linear extrapolation BASELINE.md derives from the 2-GPU run).
BASELINE_IMG_PER_SEC = {1: 416.43, 2: 713.23, 4: 1412.0, 8: 2825.0}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch_size", type=int, default=256, help="per GPU")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--kernel_impl", default="hip")
    ap.add_argument("--optimizer", default="momentum")
    ap.add_argument("--bucket_size_mb", type=float, default=25.0)
    ap.add_argument("--wire_dtype", default="fp32")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--fp32_products", default=None, choices=["exact", "bf16x3"],
                    help="--dtype fp32 conv products: exact fp32 MFMA, or three bf16 MFMAs on "
                         "the operands' bf16 splits (ops/conv_f32.py); default KFB_F32_PRODUCTS "
                         "or exact")
    ap.add_argument("--variable_update", default="kungfu",
                    help="kungfu (headline) | replicated | horovod | parameter_server | ...")
    ap.add_argument("--kungfu_option", default="sync_sgd",
                    help="sync_sgd (headline) | async_sgd (PairAveraging) | sma | ada_sgd")
    ap.add_argument("--data_name", default=None, help="dataset (coco for ssd300, ...)")
    ap.add_argument("--reuse_synthetic", action="store_true",
                    help="generate the synthetic batch once (tf_cnn_benchmarks' gpu_cached_images) "
                         "instead of re-sampling it inside every timed step")
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu"],
                    help="cpu: plumbing rehearsal of the same step over gloo (tests)")
    ap.add_argument("--rccl_channels", type=int, default=0,
                    help="pin the RCCL channel count (0: RCCL's choice)")
    ap.add_argument("--all_reduce_spec", default=None,
                    help="tf_cnn_benchmarks --all_reduce_spec (e.g. pscpu, nccl#2, xring)")
    ap.add_argument("--hierarchical_copy", action="store_true",
                    help="two-level (intra-group then leaders) gradient reduction")
    ap.add_argument("--data_dir", default=None,
                    help="real TFRecord ImageNet-format data (train preprocessing: distorted bbox "
                         "crop, flip, resize) instead of synthetic batches")
    ap.add_argument("--input_threads", type=int, default=0,
                    help="host preprocessing threads with --data_dir (0: the default)")
    ap.add_argument("--launch_tape", type=int, default=-1,
                    help="1: record one step's native launches after warmup and replay them "
                         "from C++ (ops/tape.py); falls back to eager where not eligible (at "
                         "N > 1 it needs the native RCCL communicator, which a startup "
                         "self-test validates against torch's group; see comm.selftest in the "
                         "JSON).  -1 (default): on for GPU runs")
    ap.add_argument("--job_timeout", type=float, default=1800.0,
                    help="self-launched N > 1 runs: kfb-run stops the whole job after this many "
                         "seconds (0: no limit); a stuck collective is caught earlier by the "
                         "per-rank watchdog (KFB_COMM_TIMEOUT_S)")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)

    from kf_benchmarks_amd.parallel import comm

    world_env = comm.env_world_size()
    if a.gpus > 1 and world_env == 1 and os.environ.get("KFB_BENCH_NO_SELF_LAUNCH") != "1":
        # no external launcher: start the N ranks ourselves (children, before
        # anything touches the GPU in this process) and forward rank 0's line
        return _self_launch(a, argv)
    if world_env != a.gpus:
        print("bench.py: --gpus=%d but the launcher started %d ranks" % (a.gpus, world_env),
              file=sys.stderr)
        return 2
    try:
        return _run(a)
    except Exception as e:  # noqa: BLE001 - one diagnosable line, then a non-zero exit
        if world_env > 1:
            rank = comm.env_rank()
            line = json.dumps({"status": "error", "rank": rank, "n_gpus": a.gpus,
                               "reason": "%s: %s" % (type(e).__name__, str(e)[:500])})
            print(line, file=sys.stdout if rank == 0 else sys.stderr)
            sys.stdout.flush()
        raise


def _run(a):
    from kf_benchmarks_amd.parallel import comm
    import torch
    from kf_benchmarks_amd import params as P
    from kf_benchmarks_amd.benchmark import BenchmarkCNN

    cuda = a.device == "gpu"
    from kf_benchmarks_amd.ops import conv_f32
    if a.fp32_products:
        conv_f32.set_products(a.fp32_products)
    if cuda:
        # ranks on this node need a GPU each: either every rank sees the
        # whole node (device_count >= local ranks), or the launcher gave each
        # rank its own device through a *_VISIBLE_DEVICES list
        local_ranks = int(os.environ.get("LOCAL_WORLD_SIZE", a.gpus))
        per_rank = any(os.environ.get(v) not in (None, "") for v in
                       ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"))
        have = torch.cuda.device_count()
        if have < 1 or (have < local_ranks and not (per_rank and have == 1)):
            print("bench.py: --gpus=%d but only %d GPU(s) visible" % (a.gpus, have),
                  file=sys.stderr)
            return 2
    data_name = a.data_name or {"ssd300": "coco", "deepspeech2": "librispeech"}.get(a.model) \
        or ("imagenet" if a.data_dir else None)
    p = P.make_params(model=a.model, batch_size=a.batch_size, num_gpus=1, data_name=data_name,
                      variable_update=a.variable_update, kungfu_option=a.kungfu_option,
                      optimizer=a.optimizer, use_bf16=a.dtype == "bf16",
                      use_fp16=a.dtype == "fp16", data_format="NHWC", device=a.device,
                      rccl_channels=a.rccl_channels,
                      kernel_impl=a.kernel_impl, bucket_size_mb=a.bucket_size_mb,
                      gradient_wire_dtype=a.wire_dtype, display_every=10**9,
                      all_reduce_spec=a.all_reduce_spec, hierarchical_copy=a.hierarchical_copy,
                      launch_tape=(bool(a.launch_tape) if a.launch_tape >= 0 else cuda),
                      data_dir=a.data_dir,
                      datasets_num_private_threads=a.input_threads or None,
                      datasets_repeat_cached_sample=bool(a.data_dir),
                      synthetic_resample=not a.reuse_synthetic)
    bench = BenchmarkCNN(p)
    bench.build()
    world = comm.get_world()
    if world.size != a.gpus:
        print("bench.py: --gpus=%d but the world has %d ranks" % (a.gpus, world.size),
              file=sys.stderr)
        return 2
    dev = bench.device

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)

    bench.strategy.broadcast_initial_model(bench.optimizer.slot_tensors().values())

    from kf_benchmarks_amd.parallel import watchdog
    stall = _stall_point()
    t0 = time.time()
    for i in range(a.warmup):
        loss, _ = bench.train_step(need_loss=(i == a.warmup - 1))
    watchdog.beat("warmup_sync", startup=True)
    sync()
    warm_loss = float(loss) if a.warmup > 0 else float("nan")
    if a.verbose and world.is_chief:
        print("warmup done in %.1fs, loss %.4f" % (time.time() - t0, warm_loss),
              file=sys.stderr)

    reducer = getattr(bench.strategy, "reducer", None)
    if reducer is not None and cuda:
        reducer.pop_exposed_ms()
        reducer.timing = True  # two timing events per step (exposed all-reduce)
    launches0 = reducer.launch_count if reducer is not None else 0

    bdev = dev if cuda else None
    world.barrier(bdev)
    sync()
    start = time.perf_counter()
    host = 0.0
    for i in range(a.steps):
        if stall is not None and stall == (world.rank, i):
            _stall(world.rank, i)
        h0 = time.perf_counter()
        loss, _ = bench.train_step()
        host += time.perf_counter() - h0
    watchdog.beat("final_sync")
    sync()
    world.barrier(bdev)
    sync()
    elapsed = time.perf_counter() - start
    final_loss = float(loss)

    tp = getattr(bench, "_tape", None)
    if os.environ.get("KFB_TAPE_PROFILE") and tp is not None and tp.replays > 0 \
            and world.is_chief:
        print(tp.recorder.host_profile(tp.replays), file=sys.stderr)

    # replica consistency (outside the timed region): every rank's fp32
    # master-weight checksum; synchronous strategies must agree bit for bit
    watchdog.beat("consistency")
    w = bench.strategy.flat.flat
    mine = tuple(float(v) for v in torch.stack([w.double().sum(),
                                                 w.double().square().sum()]).cpu())
    sums = comm.all_gather_object(mine)
    in_sync = all(x == sums[0] for x in sums)
    # how far the replicas drifted apart (0 for synchronous strategies; the
    # model-averaging ones keep it small): spread of the weight sums
    spread = max(x[0] for x in sums) - min(x[0] for x in sums)

    exposed = []
    if reducer is not None:
        reducer.timing = False
        exposed = reducer.pop_exposed_ms()
    t = torch.tensor([elapsed, (sum(exposed) / len(exposed)) if exposed else 0.0],
                     dtype=torch.float64, device=dev)
    watchdog.beat("report")
    comm.all_reduce(t, op="max")
    elapsed = float(t[0].item())
    exposed_ms = float(t[1].item())
    taped_steps = getattr(getattr(bench, "_tape", None), "replays", 0) > 0
    if taped_steps and reducer is not None:
        # a replayed step re-issues the recorded collectives: count them there
        per_step = sum(1 for nm in bench._tape.recorder.names if nm in _COLLECTIVES)
    elif reducer is not None:
        per_step = (reducer.launch_count - launches0) / a.steps
    else:
        per_step = 0
    comm_info = {
        "backend": world.device_backend,
        # native-communicator startup check (None: no native communicator)
        "selftest": getattr(bench, "comm_selftest", None),
        # RCCL communicators of our own still alive (world + subgroups)
        "native_comms_live": _native_comms_live(),
        "buckets": reducer.num_buckets if reducer is not None else 0,
        "collectives_per_step": per_step,
        "wire_dtype": a.wire_dtype,
        "bucket_size_mb": a.bucket_size_mb,
        "rccl_channels": os.environ.get("NCCL_MAX_NCHANNELS", "auto"),
        "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
        # all-reduce time per step that backward did not hide (max over
        # ranks; native timing events inside the step, taped or eager)
        "exposed_allreduce_ms": (round(exposed_ms, 3) if (reducer is not None and cuda
                                                          and exposed) else None),
    }
    n = world.size
    images = a.batch_size * n * a.steps
    value = images / elapsed
    if world.is_chief:
        headline = a.model == "resnet50" and not a.data_dir and a.kernel_impl == "hip"
        base = BASELINE_IMG_PER_SEC.get(n) if headline else None
        out = {
            "metric": ("images/sec (whole node) ResNet-50 synthetic at 1/2/4/8 MI355X"
                       if headline else "images/sec (whole node) %s %s%s"
                       % (a.model, "real data" if a.data_dir else "synthetic",
                          "" if a.kernel_impl == "hip"
                          else " (convs on PyTorch/MIOpen: reference bar only)")),
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * elapsed / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / base, 3) if base else None,
            "dtype": a.dtype,
            "ranks": world.size,
            "backend": world.device_backend,
            "data": ("real TFRecords from %s (train preprocessing on %s host threads, "
                     "repeat-cached records)" % (a.data_dir, a.input_threads or "default")
                     if a.data_dir else
                     "synthetic (%dx%dx3 ImageNet-shaped images %s, random-init weights)"
                     % (bench.model.image_size, bench.model.image_size,
                        "generated once" if a.reuse_synthetic
                        else "re-sampled on device every step")
                     if hasattr(bench.model, "image_size")
                     else "synthetic inputs of the model's shape, random-init weights"),
            "config": {"model": a.model, "global_batch": a.batch_size * n, "seq_len": None,
                       "per_gpu_batch": a.batch_size, "parallelism": "dp%d" % n,
                       "variable_update": (a.variable_update + "/" + a.kungfu_option
                                           if a.variable_update == "kungfu"
                                           else a.variable_update),
                       "all_reduce_spec": a.all_reduce_spec,
                       "launch_tape": (getattr(bench, "_tape", None) is not None
                                       and bench._tape.replays > 0),
                       "launch_tape_off_reason": (None if taped_steps else
                                                  getattr(bench, "_tape_reason", None)),
                       "hierarchical_copy": a.hierarchical_copy,
                       "optimizer": a.optimizer,
                       "kernel_impl": a.kernel_impl, "loss_first": warm_loss,
                       "fp32_products": conv_f32.products() if a.dtype == "fp32" else None,
                       "loss_last": final_loss},
            "comm": comm_info,
            # host time spent issuing a step (rank 0; the step is host-bound
            # when this approaches ms_per_step)
            "host_ms_per_step": round(1000.0 * host / a.steps, 3),
            "weights_in_sync": in_sync,
            "replica_spread": spread,
        }
        print(json.dumps(out))
        sys.stdout.flush()
    # the result line is out: no second JSON line may follow it (a launcher
    # tearing down a peer that fails after this point is not this job's
    # failure); shutdown hangs are bounded by the launcher's own timeout
    watchdog.stop()
    bench.strategy.close()  # collective: model stores / peers released on every rank
    close_input = getattr(getattr(bench, "input", None), "close", None)
    if close_input is not None:
        close_input()  # input producer threads stopped before interpreter exit
    world.shutdown()
    return 0


# native entry points that issue one device collective each
_COLLECTIVES = ("kfb_rccl_all_reduce", "kfb_rccl_reduce", "kfb_rccl_broadcast",
                "kfb_rccl_all_gather", "kfb_rccl_reduce_scatter", "kfb_rccl_send",
                "kfb_rccl_recv")


def _native_comms_live():
    from kf_benchmarks_amd.parallel import rccl
    return rccl.live_count()


def _stall_point():
    """KFB_TEST_STALL=<rank>:<step> (failure-handling tests): that rank stops
    making progress before that timed step, as a hung peer would."""
    v = os.environ.get("KFB_TEST_STALL")
    if not v:
        return None
    r, s = v.split(":")
    return int(r), int(s)


def _stall(rank, step):
    print("bench.py: rank %d stalls before timed step %d (KFB_TEST_STALL)" % (rank, step),
          file=sys.stderr)
    sys.stderr.flush()
    time.sleep(3600)


def _self_launch(a, argv) -> int:
    """``bench.py --gpus N`` without a launcher: N ranks through kfb-run
    (one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* exported);
    rank 0's output is echoed, the others go to per-rank logs."""
    import subprocess
    import tempfile
    if a.device == "gpu":
        # counted without any HIP call in this (launching) process
        from kf_benchmarks_amd.parallel import comm
        n = comm.visible_gpu_count()
        if n < a.gpus:
            print("bench.py: --gpus=%d but only %d GPU(s) visible" % (a.gpus, n), file=sys.stderr)
            return 2
    from kf_benchmarks_amd.parallel import launcher
    root = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    logdir = tempfile.mkdtemp(prefix="kfb_bench_")
    args = list(sys.argv[1:] if argv is None else argv)
    cmd = [launcher.launcher_binary(), "-np", str(a.gpus), "-chief-only", "-logdir", logdir]
    if a.job_timeout and a.job_timeout > 0:
        cmd += ["-timeout", "%g" % a.job_timeout]
    cmd += ["--", sys.executable, os.path.abspath(__file__)] + args
    return subprocess.call(cmd, env=env)


if __name__ == "__main__":
    sys.exit(main())
