"""Process world and collectives: one process per GPU over RCCL (xGMI).

``torch.distributed`` with the ``nccl`` backend is RCCL on ROCm; CPU runs
(tests, the plumbing config) use ``gloo``.  Rank/size come from the standard
launcher variables (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR /
MASTER_PORT), which both ``torch.distributed.run`` and our KungFu-compatible
launcher (:mod:`kf_benchmarks_amd.parallel.launcher`) export.  This replaces
the reference's gRPC cluster / Horovod MPI / KungFu Go runtimes
(tcb/cnn_util.py:201-251, tcb/benchmark_cnn.py:1378-1413, 3356-3395).
"""

from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


class World:
    def __init__(self, rank=0, size=1, local_rank=0, backend=None, initialized_here=False,
                 has_pg=None):
        self.rank = rank
        self.size = size
        self.local_rank = local_rank
        self.backend = backend
        self.initialized_here = initialized_here
        # a process group exists (always for size > 1; at size 1 only with
        # KFB_FORCE_PG=1, so the 1-GPU run exercises the real RCCL path)
        self.has_pg = (size > 1) if has_pg is None else bool(has_pg)
        self.device_index = None  # the rank's GPU (select_device_index), cuda worlds only
        # device collectives: the native RCCL communicator (parallel/rccl.py),
        # else a torch NCCL group (device_group), else the default group
        self.native = None
        self.device_group = None

    @property
    def distributed(self) -> bool:
        return self.size > 1

    @property
    def communicates(self) -> bool:
        """Collectives are issued (size > 1, or a forced 1-rank group)."""
        return self.has_pg

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    def barrier(self, device=None):
        """All ranks block until all arrive (kungfu.run_barrier,
        tcb/tf_cnn_benchmarks.py:58-60).  On RCCL this is a 1-element
        all-reduce on the device, then a host wait."""
        if not self.has_pg:
            return
        from . import watchdog
        watchdog.beat("barrier")
        if self.native is not None and device is not None:
            self.native.barrier()
            return
        if self.backend == "nccl" and device is not None:
            t = torch.zeros(1, device=device)
            dist.all_reduce(t)
            torch.cuda.synchronize(device)
        else:
            dist.barrier()

    @property
    def device_backend(self) -> str:
        """What device collectives run on: rccl (native communicator), nccl
        (torch's ProcessGroupNCCL = RCCL), gloo (CPU tests) or none."""
        if self.native is not None:
            return "rccl"
        if self.device_group is not None:
            return "nccl"
        return self.backend or "none"

    def fall_back_to_torch(self, reason: str):
        """Collective: drop the native communicator and carry the device
        collectives on a torch ProcessGroupNCCL (created here, every rank)."""
        import warnings
        warnings.warn("native RCCL communicator disabled (%s); device collectives on torch's "
                      "ProcessGroupNCCL" % reason)
        if self.native is not None:
            self.native.close(abort=True)
            self.native = None
        if self.device_group is None and self.backend != "nccl" and torch.cuda.is_available():
            self.device_group = dist.new_group(list(range(self.size)), backend="nccl")

    def shutdown(self):
        from . import watchdog
        watchdog.stop()
        if self.native is not None:
            self.native.close()
            self.native = None
        if self.initialized_here and dist.is_initialized():
            dist.destroy_process_group()


_WORLD: Optional[World] = None


def _env_int(names, default):
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            return int(v)
    return default


def env_world_size() -> int:
    """WORLD_SIZE (torch.distributed.run / kfb-run), else the OpenMPI
    variables that ``mpirun -np N`` exports (Horovod launch,
    tcb/run_hv.sh:15-18, tcb/README.md:107-115)."""
    return _env_int(("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE"), 1)


def env_rank() -> int:
    return _env_int(("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK"), 0)


def env_local_rank() -> int:
    return _env_int(("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID"), env_rank())


def force_pg() -> bool:
    return os.environ.get("KFB_FORCE_PG") == "1"


def _pg_options(backend: str):
    """RCCL communicator options: the collective stream gets high priority
    so bucket all-reduces are scheduled ahead of the compute kernels queued
    beside them."""
    if backend != "nccl":
        return None
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        return opts
    except (AttributeError, RuntimeError):
        return None


def rccl_channel_env(channels: Optional[int]) -> dict:
    """``--rccl_channels`` / KFB_RCCL_NCHANNELS: pin the RCCL channel count
    (each channel is one ring over the xGMI links)."""
    if not channels:
        v = os.environ.get("KFB_RCCL_NCHANNELS")
        channels = int(v) if v else 0
    if not channels:
        return {}
    return {"NCCL_MIN_NCHANNELS": str(channels), "NCCL_MAX_NCHANNELS": str(channels)}


def merge_rccl_env(channel_env: dict, spec_env: dict) -> dict:
    """Combine the ``--rccl_channels`` pin with the ``--all_reduce_spec``
    settings: the spec's ``#shards`` raises the channel floor, and the
    ceiling is never left below the floor (RCCL would otherwise clamp one of
    the two settings silently)."""
    env = dict(channel_env)
    for k, v in spec_env.items():
        if k != "NCCL_MIN_NCHANNELS":
            env[k] = v
    lo = max(int(channel_env.get("NCCL_MIN_NCHANNELS", 0)),
             int(spec_env.get("NCCL_MIN_NCHANNELS", 0)))
    if lo:
        env["NCCL_MIN_NCHANNELS"] = str(lo)
        if "NCCL_MAX_NCHANNELS" in env:
            env["NCCL_MAX_NCHANNELS"] = str(max(int(env["NCCL_MAX_NCHANNELS"]), lo))
    return env


def _count_device_list(v: str) -> int:
    return len([d for d in v.split(",") if d.strip() != ""])


def visible_gpu_count() -> int:
    """GPUs this process may use, WITHOUT a HIP call in this process (a
    launcher parent must not initialise the runtime before it starts its
    ranks).  HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES
    when set; otherwise a child interpreter asks the runtime."""
    for name in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        v = os.environ.get(name)
        if v is not None:
            return _count_device_list(v)
    import subprocess
    import sys
    try:
        out = subprocess.run([sys.executable, "-c",
                              "import torch; print(torch.cuda.device_count())"],
                             capture_output=True, text=True, timeout=300)
        return int(out.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError, OSError):
        return 0


def select_device_index(gpu_indices, num_gpus: int, tower_mode: bool, local_rank: int,
                        world_size: int, device_count: int) -> int:
    """The ONE place a rank's GPU is chosen: the compute device and the RCCL
    communicator's device both come from here.  ``device_count`` is what
    this process sees, so a launcher that gives every rank its own
    HIP_VISIBLE_DEVICES (1 visible device) maps every rank to device 0,
    and one that exposes the whole node maps local rank r to GPU r
    (shifted by ``--gpu_indices``)."""
    gpu_indices = list(gpu_indices) or [0]
    local = local_rank if world_size > 1 else 0
    if num_gpus == 1:
        idx = gpu_indices[0] + local
    elif tower_mode:
        idx = gpu_indices[local % len(gpu_indices)]
    else:
        idx = gpu_indices[0]
    return idx % max(int(device_count), 1)


def init_world(device_type: str = "cuda", all_reduce_spec: Optional[str] = None,
               timeout_s: int = 1800, channels: Optional[int] = None,
               device_index: Optional[int] = None) -> World:
    """Initializes the default process group once (idempotent).
    ``all_reduce_spec`` picks RCCL's algorithm / channel count before the
    communicator exists (parallel/allreduce.py:rccl_env_for_spec).  At world
    size 1 no group is created unless KFB_FORCE_PG=1.  ``device_index`` is
    the rank's compute GPU (:func:`select_device_index`); the communicator
    is bound to the same device."""
    global _WORLD
    if _WORLD is not None:
        return _WORLD
    size = env_world_size()
    rank = env_rank()
    local_rank = env_local_rank()
    if size <= 1 and not force_pg():
        _WORLD = World(0, 1, local_rank, None)
        _WORLD.device_index = device_index
        return _WORLD
    if size <= 1:
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
    # KFB_DIST_BACKEND=gloo: ranks that share one GPU (RCCL refuses two ranks
    # on one device) - the 2-rank GPU rehearsal on a 1-GPU box
    forced = os.environ.get("KFB_DIST_BACKEND")
    backend = forced or ("nccl" if device_type == "cuda" else "gloo")
    from . import rccl as _rccl
    native = backend == "nccl" and not forced and _rccl.enabled() and _rccl.available()
    if native or backend == "nccl":
        spec_env = {}
        if all_reduce_spec:
            from .allreduce import rccl_env_for_spec
            spec_env = rccl_env_for_spec(all_reduce_spec)
        for k, v in merge_rccl_env(rccl_channel_env(channels), spec_env).items():
            os.environ.setdefault(k, v)
    here = False
    if device_index is None and device_type == "cuda":
        device_index = select_device_index([0], 1, False, local_rank, size,
                                           torch.cuda.device_count())
    if backend == "nccl":
        _reserve_compute_streams(device_index)
    if native:
        # host-side traffic (object gathers, CPU barriers, the TCP store) on
        # gloo; device collectives on the native communicator created below
        backend = "gloo"
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kwargs = dict(backend=backend, init_method="env://", rank=rank, world_size=size,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kwargs["device_id"] = torch.device("cuda", device_index)
            opts = _pg_options(backend)
            if opts is not None:
                kwargs["pg_options"] = opts
        dist.init_process_group(**kwargs)
        here = True
    world = World(rank, size, local_rank, dist.get_backend(), here, has_pg=True)
    world.device_index = device_index
    if size > 1:
        # from here on a stuck collective ends the job with a diagnosis
        # (parallel/watchdog.py; KFB_COMM_TIMEOUT_S=0 turns it off)
        from . import watchdog
        if watchdog.start(rank):
            watchdog.beat("startup", startup=True)
    if native:
        try:
            store = dist.distributed_c10d._get_default_store()
            world.native = _rccl.NativeComm(rank, size, device_index, store)
        except Exception as e:  # noqa: BLE001 - fall back to torch's RCCL group
            import warnings
            warnings.warn("native RCCL communicator unavailable (%s); using torch's "
                          "ProcessGroupNCCL for device collectives" % e)
            world.device_group = dist.new_group(list(range(size)), backend="nccl")
    _WORLD = world
    return _WORLD


def _reserve_compute_streams(device_index: int):
    """Create the compute side streams (weight-gradient stream) BEFORE the
    RCCL communicator: HIP maps streams onto a few hardware queues
    (GPU_MAX_HW_QUEUES, 4 by default) in creation order, and a side stream
    created after RCCL's streams can land on the compute stream's queue,
    serializing the weight gradients behind the dgrad chain (measured: the
    1-rank RCCL run lost the side-stream overlap, 22.5 vs 21.0 ms/step)."""
    try:
        torch.cuda.set_device(device_index)
        from ..ops import conv_hip
        conv_hip.wgrad_stream(torch.device("cuda", device_index))
    except Exception:  # noqa: BLE001 - best effort; the streams are created lazily anyway
        pass


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def get_world() -> World:
    return _WORLD if _WORLD is not None else World()


def reset_world():
    """Test helper: forget the cached world (does not destroy the group)."""
    global _WORLD
    _WORLD = None


# KFB_SELFTEST_INJECT=1 (tests): rank 0's check sees a wrong sum, so the
# fallback branch runs on a real communicator
_SELFTEST_INJECT = os.environ.get("KFB_SELFTEST_INJECT") == "1"

# largest buffer a self-test check moves (bigger job buffers are checked at
# this size: the startup cost must not grow with the model).  Host buffers
# (CPU rehearsals, where the candidate is a stand-in over gloo and the
# pattern arithmetic runs on one core per rank) use the smaller cap.
SELFTEST_CAP_BYTES = 64 << 20
SELFTEST_CAP_BYTES_HOST = 8 << 20


def _selftest_cap(device) -> int:
    return SELFTEST_CAP_BYTES if (device is not None and torch.device(device).type == "cuda") \
        else SELFTEST_CAP_BYTES_HOST


_HASH = {}


def _selftest_hash(n: int, seed: int, device):
    """17 bits of an index hash (int32), identical on every rank; one per
    (seed, device), grown to the largest size asked for and sliced."""
    key = (seed, str(device))
    h = _HASH.get(key)
    if h is None or h.numel() < n:
        i = torch.arange(n, device=device, dtype=torch.int64)
        h = (i * 2654435761 + seed * 97) & 0xFFFFFFFF
        h = ((h ^ (h >> 13)) * 1274126177) & 0xFFFFFFFF
        # 16 hash bits and a sign bit, as int32
        h = ((h >> 8) & 0x1FFFF).to(torch.int32)
        _HASH[key] = h
    return h[:n]


def _selftest_base(n: int, lim: int, seed: int, device):
    """(base, sign): an index-hashed integer in [-lim, lim] and a +-1 per
    element (int32), identical on every rank."""
    h = _selftest_hash(n, seed, device)
    # (multiply-shift maps the 16 bits onto [0, 2 lim] without a division)
    return (((h & 0xFFFF) * (2 * lim + 1)) >> 16) - lim, ((h >> 15) & 2) - 1


def _member_weights(members: int, dt) -> Optional[list]:
    """Per-member multipliers of the sign term: member + 1 (distinct
    contributions) while every partial sum stays exact in ``dt``, else 1
    for everyone; None when not even that fits (then the dtype is not
    checked at this group size)."""
    top = _EXACT.get(dt, 1 << 24)
    if members * (members + 1) // 2 <= top:
        return list(range(1, members + 1))
    if members <= top:
        return [1] * members
    return None


_EXACT = {torch.bfloat16: 256, torch.float16: 2048}


def selftest_pattern(n: int, member: int, lim: int, seed: int, device,
                     weights=None) -> torch.Tensor:
    """Member ``member``'s test data: base(i) + sign(i) * w[member].
    Element i differs across the buffer (misplaced data is caught) and
    across members (a missing or doubled contribution is caught), and the
    results of every collective have a closed form each rank evaluates on
    its own device (:func:`selftest_expected`) - no buffer crosses the
    host network."""
    base, sign = _selftest_base(n, lim, seed, device)
    w = weights[member] if weights is not None else member + 1
    return base + sign * w


def selftest_expected(kind: str, n: int, members: int, lim: int, seed: int, device,
                      weights=None):
    weights = weights if weights is not None else list(range(1, members + 1))
    base, sign = _selftest_base(n, lim, seed, device)
    if kind == "broadcast":  # member 0's data
        return base + sign * weights[0]
    if kind == "max":
        return base + torch.where(sign > 0, sign * max(weights), sign * min(weights))
    return base * members + sign * sum(weights)  # sum / reduce


def _selftest_lim(dt, members: int, weights=None) -> int:
    # every partial sum of ``members`` values stays an integer the dtype
    # holds exactly (bf16: |x| <= 256, fp16: <= 2048), in any order
    weights = weights if weights is not None else list(range(1, members + 1))
    top = _EXACT.get(dt)
    if top is None:
        return 1024
    return max(0, (top - sum(weights)) // members)


def selftest_device_collectives(cand, sizes, dtypes=(torch.float32,), device=None,
                                 seed: int = 0, groups=None) -> dict:
    """Checks device communicators bitwise on device-generated data.

    ``groups``: [(name, comm, member_index, members)] - the world
    communicator and e.g. the hierarchical reduction's subgroups; default
    the world's ``cand`` alone.  For every buffer size (capped at
    SELFTEST_CAP_BYTES), dtype and group: broadcast from member 0, sum / max
    all-reduce, and sum reduce to member 0 of integer data from
    :func:`selftest_pattern`.  Each rank computes the expected results
    itself from every member's pattern, so no buffer crosses the host
    network; only the per-rank failure lists are exchanged (one small
    ``all_gather_object``).  A check that raises is recorded as a failure
    and the loop goes on, so every rank issues the same collectives and
    reaches the verdict.  Collective over all ranks; every rank returns the
    same verdict {"ok", "checked", "failed"}."""
    w = get_world()
    dev = device if device is not None else getattr(cand, "device", None)
    if groups is None:
        groups = [("world", cand, w.rank, w.size)]
    failed = []
    checked = 0
    cap = _selftest_cap(dev)
    # the hash once, at the largest size checked (the rest are slices)
    _selftest_hash(max(1, min(max(int(n) for n in sizes), cap // 2)), seed, dev)
    for gname, gc, me, members in groups:
        if gc is None:
            continue
        seen = set()
        for n in sizes:
            for dt in dtypes:
                esz = torch.tensor([], dtype=dt).element_size()
                n_ = max(1, min(int(n), cap // esz))
                if (n_, dt) in seen:
                    continue  # (sizes above the cap collapse into one check)
                seen.add((n_, dt))
                wts = _member_weights(members, dt)
                if wts is None:
                    continue  # (more members than the dtype counts exactly)
                lim = _selftest_lim(dt, members, wts)
                base, sign = _selftest_base(n_, lim, seed, dev)
                mine = (base + sign * wts[me]).to(dt)
                expect = {"broadcast": (base + sign * wts[0]).to(dt),
                          "max": (base + torch.where(sign > 0, sign * max(wts),
                                                     sign * min(wts))).to(dt),
                          "sum": (base * members + sign * sum(wts)).to(dt)}
                expect["reduce"] = expect["sum"]
                for kind in ("broadcast", "sum", "max", "reduce"):
                    tag = "%s%s n=%d %s" % ("" if gname == "world" else gname + ":", kind, n_,
                                            str(dt).replace("torch.", ""))
                    checked += 1
                    try:
                        buf = mine.clone()
                        if kind == "broadcast":
                            work = gc.broadcast(buf, 0)
                        elif kind == "reduce":
                            work = gc.reduce(buf, 0, "sum")
                        else:
                            work = gc.all_reduce(buf, kind)
                        if work is not None:
                            work.wait()
                        if kind == "reduce" and me != 0:
                            continue  # (non-root buffers are unspecified)
                        good = torch.equal(buf, expect[kind])
                        if _SELFTEST_INJECT and kind == "sum" and n_ > 1 and w.rank == 0:
                            good = False  # (test hook: a wrong sum on rank 0)
                    except Exception as e:  # noqa: BLE001 - a raising collective fails the check
                        good = False
                        tag += " (raised %s)" % type(e).__name__
                    if not good:
                        failed.append(tag)
    try:
        cand.barrier()
    except Exception as e:  # noqa: BLE001
        failed.append("barrier (raised %s)" % type(e).__name__)
    _HASH.clear()
    verdicts = all_gather_object(failed)
    bad = sorted({f for fl in verdicts for f in fl})
    return {"ok": not bad, "checked": checked, "failed": bad[:8]}


def validate_native(sizes, dtypes=(torch.float32,), groups=None) -> Optional[dict]:
    """KFB_NATIVE_COMM=auto: self-test the native communicators (the world's
    and ``groups``' subgroups) on the job's buffer sizes and fall back to
    torch's ProcessGroupNCCL if any fails.  Returns the self-test record
    (None: no native communicator)."""
    w = get_world()
    if w.native is None or not w.has_pg:
        return None
    from . import rccl as _rccl
    all_groups = [("world", w.native, w.rank, w.size)] + list(groups or [])
    st = selftest_device_collectives(w.native, sizes, dtypes, groups=all_groups)
    st["mode"] = _rccl.mode()
    if not st["ok"] and _rccl.mode() == "auto":
        w.fall_back_to_torch("self-test failed: %s" % ", ".join(st["failed"]))
        st["fallback"] = "torch ProcessGroupNCCL"
    return st


_ROP = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


def _finish(work, async_op):
    if async_op:
        return work
    work.wait()
    return None


def all_reduce(t: torch.Tensor, op: str = "sum", async_op: bool = False):
    """Device tensors: the native communicator (the returned work's wait()
    orders the caller's stream after it; no host wait); host tensors: the
    default (gloo) group."""
    w = get_world()
    if not w.has_pg:
        return None
    if t.is_cuda and w.native is not None:
        return _finish(w.native.all_reduce(t, op), async_op)
    group = w.device_group if t.is_cuda else None
    return dist.all_reduce(t, op=_ROP[op], async_op=async_op, group=group)


def reduce(t: torch.Tensor, dst: int = 0, op: str = "sum", async_op: bool = False):
    w = get_world()
    if not w.has_pg:
        return None
    if t.is_cuda and w.native is not None:
        return _finish(w.native.reduce(t, dst, op), async_op)
    group = w.device_group if t.is_cuda else None
    return dist.reduce(t, dst=dst, op=_ROP[op], async_op=async_op, group=group)


def broadcast(t: torch.Tensor, src: int = 0, async_op: bool = False):
    w = get_world()
    if not w.has_pg:
        return None
    if t.is_cuda and w.native is not None:
        return _finish(w.native.broadcast(t, src), async_op)
    group = w.device_group if t.is_cuda else None
    return dist.broadcast(t, src=src, async_op=async_op, group=group)


def all_gather_object(obj):
    if not get_world().has_pg:
        return [obj]
    out = [None] * get_world().size
    dist.all_gather_object(out, obj)
    return out
