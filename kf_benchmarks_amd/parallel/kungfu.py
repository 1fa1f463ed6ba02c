"""KungFu PairAveraging (``--kungfu_option=async_sgd``) on MI355X.

Semantics (KungFu PairAveragingOptimizer, called at tcb/benchmark_cnn.py:1196-1198;
spec in SURVEY.md Appendix A): every step each worker
  1. picks a random peer != self,
  2. reads that peer's most recently *published* model (one-sided: the
     peer does not participate),
  3. sets w <- (w + w_peer) / 2,
  4. applies its own gradient with the wrapped optimizer,
  5. publishes its updated model for others.
There is no global barrier per step.

Model store: each rank owns a double-buffered model snapshot plus a version
counter.  Publishing writes the slot the readers are NOT pointed at, then
bumps the version (host shared memory, release ordering).  Readers copy the
slot of the version they observed and re-check the version afterwards
(retry on a concurrent double publish), so a pulled model is never torn.

* GPU ranks: the two slots live in device memory and are shared with every
  peer through HIP IPC (torch CUDA-tensor sharing over dmabuf), so a pull is
  a device-to-device copy over xGMI that the owner never sees.
* CPU ranks (tests, plumbing config): the slots live in /dev/shm.
The version words always live in a small /dev/shm file per rank.
"""

from __future__ import annotations

import mmap
import os
import random
import struct
import uuid

import numpy as np
import torch

from . import comm
from .variable_mgr import Strategy


class _Versions:
    """One int64 version word per rank in /dev/shm (mapped by every rank)."""

    def __init__(self, job, rank, size):
        self.paths = ["/dev/shm/kfb_ver_%s_%d" % (job, r) for r in range(size)]
        with open(self.paths[rank], "wb") as f:
            f.write(b"\0" * 64)
        self.rank = rank
        self._maps = {}

    def _map(self, r):
        if r not in self._maps:
            f = open(self.paths[r], "r+b")
            self._maps[r] = (f, mmap.mmap(f.fileno(), 64))
        return self._maps[r][1]

    def get(self, r) -> int:
        return struct.unpack_from("<q", self._map(r), 0)[0]

    def set(self, v: int):
        struct.pack_into("<q", self._map(self.rank), 0, v)

    def close(self):
        for f, m in self._maps.values():
            m.close()
            f.close()
        try:
            os.remove(self.paths[self.rank])
        except OSError:
            pass


class ModelStore:
    def __init__(self, flat: torch.Tensor, world: comm.World):
        self.world = world
        self.rank, self.size = world.rank, world.size
        job = comm.all_gather_object(uuid.uuid4().hex[:12] if world.rank == 0 else None)[0]
        self.versions = _Versions(job, self.rank, self.size)
        n = flat.numel()
        self.n = n
        self.device = flat.device
        if flat.is_cuda:
            self.slots = torch.empty((2, n), dtype=flat.dtype, device=flat.device)
            self.slots[0].copy_(flat)
            self.slots[1].copy_(flat)
            from torch.multiprocessing.reductions import reduce_tensor
            handle = reduce_tensor(self.slots)
            handles = comm.all_gather_object(handle)
            self.peer_slots = {}
            for r, (fn, args) in enumerate(handles):
                if r != self.rank:
                    self.peer_slots[r] = fn(*args)
            self._files = []
        else:
            self.path = "/dev/shm/kfb_model_%s_%d" % (job, self.rank)
            arr = np.memmap(self.path, dtype=np.float32, mode="w+", shape=(2, n))
            arr[0] = flat.numpy()
            arr[1] = flat.numpy()
            arr.flush()
            self.slots = torch.from_numpy(arr)
            self._arr = arr
            comm.all_gather_object(True)  # every rank has created its file
            self.peer_slots = {}
            for r in range(self.size):
                if r != self.rank:
                    p = "/dev/shm/kfb_model_%s_%d" % (job, r)
                    self.peer_slots[r] = torch.from_numpy(
                        np.memmap(p, dtype=np.float32, mode="r", shape=(2, n)))
        self.version = 0
        self.versions.set(0)
        comm.all_gather_object(True)

    def publish(self, flat: torch.Tensor):
        nxt = self.version + 1
        self.slots[nxt % 2].copy_(flat)
        if flat.is_cuda:
            torch.cuda.current_stream(flat.device).synchronize()
        self.version = nxt
        self.versions.set(nxt)

    def pull(self, peer: int, out: torch.Tensor) -> int:
        for _ in range(8):
            v = self.versions.get(peer)
            out.copy_(self.peer_slots[peer][v % 2])
            if out.is_cuda:
                torch.cuda.current_stream(out.device).synchronize()
            if self.versions.get(peer) - v < 2:  # slot v%2 not rewritten meanwhile
                return v
        return v

    def close(self):
        self.versions.close()
        if not self.slots.is_cuda:
            try:
                os.remove(self.path)
            except OSError:
                pass


class PairAveraging(Strategy):
    name = "kungfu/async_sgd"

    def __init__(self, params, world, flat, **kw):
        super().__init__(params, world, flat, **kw)
        self.rng = random.Random(params.kungfu_peer_seed * 7919 + world.rank)
        self.store = None
        self._peer_buf = None

    def broadcast_initial_model(self, slots=()):
        super().broadcast_initial_model(slots)
        if self.world.size > 1:
            self.store = ModelStore(self.flat.flat, self.world)
            self._peer_buf = torch.empty_like(self.flat.flat)

    def before_update(self, step):
        if self.store is None:
            return
        peer = self.rng.randrange(self.world.size - 1)
        if peer >= self.world.rank:
            peer += 1
        self.store.pull(peer, self._peer_buf)
        w = self.flat.flat
        w.add_(self._peer_buf).mul_(0.5)

    def after_update(self, step):
        if self.store is not None:
            self.store.publish(self.flat.flat)

    def close(self):
        if self.store is not None:
            self.store.close()
