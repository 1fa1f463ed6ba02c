"""Asynchronous parameter server: ``--variable_update=parameter_server
--cross_replica_sync=False`` in a multi-worker job.

Reference semantics (tcb/benchmark_cnn.py:2220-2229, tcb/variable_mgr.py:628-671):
the variables live on the PS; every worker reads them, computes a gradient
and applies it to the PS copy with the optimizer, without waiting for the
other workers, so gradients are applied to a model that may have moved since
they were computed (staleness).  The run is timed by a GlobalStepWatcher that
polls the shared global step (tcb/benchmark_cnn.py:639-684).

One process per GPU, no separate PS job: rank 0's device memory holds the
shared model and optimizer slots, mapped into every rank through HIP IPC
(dmabuf), or /dev/shm files for CPU ranks.  A worker's update is a
read-modify-write of that shared state under an inter-process lock
(fcntl on a /dev/shm file): pull the current shared weights and slots into
the local buffers, run the fused optimizer with the local (stale) gradient,
copy the result back, bump the shared global step.  Each apply is therefore
atomic (no lost updates, unlike TF's use_locking=False Hogwild), and workers
interleave freely between applies.
"""

from __future__ import annotations

import fcntl
import mmap
import os
import struct
import time
import uuid

import numpy as np
import torch

from . import comm
from .variable_mgr import Strategy


class _SharedState:
    """The shared model/slot buffers (owner: rank 0) plus the lock file and
    the global-step word."""

    def __init__(self, tensors, world: comm.World):
        self.world = world
        job = comm.all_gather_object(uuid.uuid4().hex[:12] if world.rank == 0 else None)[0]
        self.lock_path = "/dev/shm/kfb_ps_lock_%s" % job
        self.step_path = "/dev/shm/kfb_ps_step_%s" % job
        if world.rank == 0:
            with open(self.step_path, "wb") as f:
                f.write(b"\0" * 64)
            open(self.lock_path, "wb").close()
        cuda = tensors[0].is_cuda
        self._opened = []
        if cuda:
            # rank 0's buffers mapped into every other rank's OWN device
            # (parallel/ipc.py: no context on rank 0's GPU)
            from . import ipc
            dev = tensors[0].device
            if world.rank == 0:
                self.shared = [t.detach().clone() for t in tensors]
                torch.cuda.synchronize(dev)
                infos = [ipc.export_slots(t) for t in self.shared]
            else:
                infos = None
            infos = comm.all_gather_object(infos)[0]
            if world.rank != 0:
                mine = ipc.export_view(dev)
                self.shared = []
                for t, info in zip(tensors, infos):
                    base = ipc.open_peer_slots(info, mine)
                    self._opened.append(base)
                    self.shared.append(ipc.wrap(base + info["offset"], t.numel(), t.dtype, dev)
                                       .view(t.shape))
        else:
            paths = ["/dev/shm/kfb_ps_var_%s_%d" % (job, i) for i in range(len(tensors))]
            if world.rank == 0:
                for p, t in zip(paths, tensors):
                    arr = np.memmap(p, dtype=np.float32, mode="w+", shape=(t.numel(),))
                    arr[:] = t.detach().reshape(-1).numpy()
                    arr.flush()
            comm.all_gather_object(True)
            self.shared = [torch.from_numpy(np.memmap(p, dtype=np.float32, mode="r+",
                                                      shape=(t.numel(),)))
                           for p, t in zip(paths, tensors)]
            self._paths = paths
        comm.all_gather_object(True)  # every rank has mapped everything
        self._lock_f = open(self.lock_path, "r+b")
        self._step_f = open(self.step_path, "r+b")
        self._step_m = mmap.mmap(self._step_f.fileno(), 64)

    held = False

    def lock(self):
        fcntl.flock(self._lock_f, fcntl.LOCK_EX)
        self.held = True

    def unlock(self):
        if self.held:
            self.held = False
            fcntl.flock(self._lock_f, fcntl.LOCK_UN)

    @property
    def global_step(self) -> int:
        return struct.unpack_from("<q", self._step_m, 0)[0]

    def bump_step(self):
        struct.pack_into("<q", self._step_m, 0, self.global_step + 1)

    def close(self):
        self.unlock()  # never leave the PS lock to a closed file
        self._step_m.close()
        self._step_f.close()
        self._lock_f.close()
        if self._opened:
            from . import ipc
            torch.cuda.synchronize(self.shared[0].device)
            self.shared = []
            for base in self._opened:
                ipc.close_mapping(base)
            self._opened = []
        comm.all_gather_object(True)  # nobody maps the files / buffers any more
        if self.world.rank == 0:
            for p in [self.lock_path, self.step_path] + list(getattr(self, "_paths", [])):
                try:
                    os.remove(p)
                except OSError:
                    pass


class AsyncParameterServer(Strategy):
    name = "parameter_server (async)"

    def __init__(self, params, world, flat, **kw):
        super().__init__(params, world, flat, **kw)
        self.state = None
        self._local = None

    def broadcast_initial_model(self, slots=()):
        super().broadcast_initial_model(slots)
        if self.world.size > 1:
            self._local = [self.flat.flat] + [s for s in slots]
            self.state = _SharedState(self._local, self.world)

    def before_update(self, step):
        """Take the PS lock and load the current shared weights and slots:
        the optimizer then applies this worker's gradient to them."""
        if self.state is None:
            return
        self.state.lock()
        for dst, src in zip(self._local, self.state.shared):
            dst.view(-1).copy_(src.view(-1))

    def after_update(self, step):
        if self.state is None:
            return
        for dst, src in zip(self.state.shared, self._local):
            dst.view(-1).copy_(src.view(-1))
        if self._local[0].is_cuda:
            torch.cuda.current_stream(self._local[0].device).synchronize()
        self.state.bump_step()
        self.state.unlock()

    def abort_update(self, step):
        """The update failed between before_update and after_update: release
        the PS lock so the other workers do not block forever."""
        if self.state is not None:
            self.state.unlock()

    def close(self):
        if self.state is not None:
            self.state.close()
            self.state = None


class GlobalStepWatcher:
    """Times an asynchronous run by the shared global step
    (tcb/benchmark_cnn.py:639-684): images/sec = batch x global steps
    applied by ALL workers between start() and stop() / wall time."""

    def __init__(self, state: _SharedState):
        self.state = state
        self.start_step = self.start_time = None
        self.end_step = self.end_time = None

    def start(self):
        self.start_step, self.start_time = self.state.global_step, time.perf_counter()

    def stop(self):
        self.end_step, self.end_time = self.state.global_step, time.perf_counter()

    def steps_per_second(self) -> float:
        dt = self.end_time - self.start_time
        return (self.end_step - self.start_step) / dt if dt > 0 else 0.0
