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
    def __init__(self, rank=0, size=1, local_rank=0, backend=None, initialized_here=False):
        self.rank = rank
        self.size = size
        self.local_rank = local_rank
        self.backend = backend
        self.initialized_here = initialized_here

    @property
    def distributed(self) -> bool:
        return self.size > 1

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    def barrier(self, device=None):
        """All ranks block until all arrive (kungfu.run_barrier,
        tcb/tf_cnn_benchmarks.py:58-60).  On RCCL this is a 1-element
        all-reduce on the device, then a host wait."""
        if not self.distributed:
            return
        if self.backend == "nccl" and device is not None:
            t = torch.zeros(1, device=device)
            dist.all_reduce(t)
            torch.cuda.synchronize(device)
        else:
            dist.barrier()

    def shutdown(self):
        if self.initialized_here and dist.is_initialized():
            dist.destroy_process_group()


_WORLD: Optional[World] = None


def env_world_size() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def init_world(device_type: str = "cuda", all_reduce_spec: Optional[str] = None,
               timeout_s: int = 1800) -> World:
    """Initializes the default process group once (idempotent).
    ``all_reduce_spec`` picks RCCL's algorithm / channel count before the
    communicator exists (parallel/allreduce.py:rccl_env_for_spec)."""
    global _WORLD
    if _WORLD is not None:
        return _WORLD
    size = env_world_size()
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if size <= 1:
        _WORLD = World(0, 1, local_rank, None)
        return _WORLD
    # KFB_DIST_BACKEND=gloo: ranks that share one GPU (RCCL refuses two ranks
    # on one device) - the 2-rank GPU rehearsal on a 1-GPU box
    backend = os.environ.get("KFB_DIST_BACKEND") or ("nccl" if device_type == "cuda" else "gloo")
    if backend == "nccl" and all_reduce_spec:
        from .allreduce import rccl_env_for_spec
        for k, v in rccl_env_for_spec(all_reduce_spec).items():
            os.environ.setdefault(k, v)
    here = False
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kwargs = dict(backend=backend, init_method="env://", rank=rank, world_size=size,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kwargs["device_id"] = torch.device("cuda", local_rank)
        dist.init_process_group(**kwargs)
        here = True
    _WORLD = World(rank, size, local_rank, dist.get_backend(), here)
    return _WORLD


def get_world() -> World:
    return _WORLD if _WORLD is not None else World()


def reset_world():
    """Test helper: forget the cached world (does not destroy the group)."""
    global _WORLD
    _WORLD = None


def all_reduce(t: torch.Tensor, op: str = "sum", async_op: bool = False):
    if get_world().size <= 1:
        return None
    rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
    return dist.all_reduce(t, op=rop, async_op=async_op)


def broadcast(t: torch.Tensor, src: int = 0, async_op: bool = False):
    if get_world().size <= 1:
        return None
    return dist.broadcast(t, src=src, async_op=async_op)


def all_gather_object(obj):
    if get_world().size <= 1:
        return [obj]
    out = [None] * get_world().size
    dist.all_gather_object(out, obj)
    return out
