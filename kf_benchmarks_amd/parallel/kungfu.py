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

Model store: each rank owns two model slots plus a per-slot seqlock in a
small /dev/shm header ``[seq0, seq1, latest]`` (int64 words, mapped by every
rank).  Publish: pick the slot ``latest`` does NOT point at, make its
sequence word odd (write in progress), copy the model into it, and once the
copy has completed make the word even again and point ``latest`` at it.  A
reader reads ``latest`` and that slot's (even) sequence word, copies the
slot, and accepts the copy only if the word is unchanged afterwards; any
overlap with a rewrite of that slot changes it, so a torn model is never
accepted.  Retries are bounded and exhausting them raises.

* GPU ranks: the two slots live in device memory and are shared with every
  peer through HIP IPC (torch CUDA-tensor sharing over dmabuf), so a pull is
  a device-to-device copy over xGMI that the owner never sees.  Nothing
  blocks the host inside the step:
  - the peer pull is issued on a side stream at the start of the step
    (overlapping forward/backward) and validated ON THE DEVICE: a one-thread
    kernel behind the copy re-reads the peer's sequence word (the /dev/shm
    header, page-locked and mapped for the GPU) and sets a flag; the fused
    optimizer averages with the snapshot only if the flag says untorn (a
    torn snapshot - a rewrite overlapped the copy - skips that step's
    averaging and is counted);
  - the optimizer writes the updated model straight into the publish slot
    (no copy pass); the slot is committed (sequence word made even) once
    the update's event has completed, polled at the next step.  If it has
    not completed by the next publish, that publish rewrites the same
    (still odd, never readable) slot.
  ``--kungfu_pair_prefetch=false`` pulls at update time instead (the peer
  model is then as fresh as KungFu's, whose PairAveragingOptimizer requests
  it in apply_gradients); the default prefetch at the start of the step
  averages with a model one forward/backward older, the price of overlapping
  the pull.
* CPU ranks (tests, plumbing config): the slots live in /dev/shm and the
  seqlock is checked on the host.
"""

from __future__ import annotations

import mmap
import os
import random
import struct
import uuid
import warnings

from typing import Optional

import numpy as np
import torch

from . import comm
from .ipc import close_mapping, export_slots, open_peer_slots
from .variable_mgr import Strategy


class _Header:
    """Per-rank seqlock header ``[seq0, seq1, latest]`` in /dev/shm."""

    WORDS = 3

    def __init__(self, job, rank, size):
        self.paths = ["/dev/shm/kfb_ver_%s_%d" % (job, r) for r in range(size)]
        with open(self.paths[rank], "wb") as f:
            f.write(b"\0" * 64)
        self.rank = rank
        self._maps = {}
        self._dev = {}

    def _map(self, r):
        if r not in self._maps:
            f = open(self.paths[r], "r+b")
            self._maps[r] = (f, mmap.mmap(f.fileno(), 64))
        return self._maps[r][1]

    def read(self, r, word) -> int:
        return struct.unpack_from("<q", self._map(r), 8 * word)[0]

    def write(self, word, v: int):
        # aligned 8-byte stores; x86-64 keeps store order, so a reader that
        # sees the new ``latest`` also sees the sequence word written before it
        struct.pack_into("<q", self._map(self.rank), 8 * word, v)

    def device_word(self, r, word):
        """Device address of peer ``r``'s header word (page-locked host
        memory); None if the mapping cannot be registered."""
        if r not in self._dev:
            import ctypes
            from ..ops import _native as N
            m = self._map(r)
            host = ctypes.addressof(ctypes.c_char.from_buffer(m))
            dev = ctypes.c_void_p()
            try:
                N.call("kfb_host_register", host, 64, ctypes.byref(dev))
                self._dev[r] = (host, dev.value)
            except N.NativeError:
                self._dev[r] = (None, None)
        host, dev = self._dev[r]
        return None if dev is None else dev + 8 * word

    def close(self):
        if self._dev:
            from ..ops import _native as N
            for host, dev in self._dev.values():
                if host is not None:
                    try:
                        N.call("kfb_host_unregister", host)
                    except N.NativeError:
                        pass
            self._dev = {}
        for f, m in self._maps.values():
            m.close()
            f.close()
        self._maps = {}
        try:
            os.remove(self.paths[self.rank])
        except OSError:
            pass


class TornReadError(RuntimeError):
    pass


class ModelStore:
    SEQ0, SEQ1, LATEST = 0, 1, 2
    MAX_TRIES = 64

    def __init__(self, flat: torch.Tensor, world: comm.World):
        self.world = world
        self.rank, self.size = world.rank, world.size
        job = comm.all_gather_object(uuid.uuid4().hex[:12] if world.rank == 0 else None)[0]
        self.hdr = _Header(job, self.rank, self.size)
        n = flat.numel()
        self.n = n
        self.device = flat.device
        self.cuda = flat.is_cuda
        if self.cuda:
            self.slots = torch.empty((2, n), dtype=flat.dtype, device=flat.device)
            self.slots[0].copy_(flat)
            self.slots[1].copy_(flat)
            torch.cuda.synchronize(flat.device)
            # the slots' IPC handle, opened by every peer on ITS OWN device
            # (native hipIpcOpenMemHandle; torch's tensor rebuild would open it
            # on this rank's device index and create a context there)
            info = export_slots(self.slots)
            infos = comm.all_gather_object(info)
            self.peer_slots = {}
            self._opened = []
            for r, pinfo in enumerate(infos):
                if r != self.rank:
                    base = open_peer_slots(pinfo, info)
                    self._opened.append(base)
                    nb = self.slots[0].numel() * self.slots.element_size()
                    self.peer_slots[r] = (base + pinfo["offset"], base + pinfo["offset"] + nb)
            self.pull_stream = torch.cuda.Stream(flat.device)
            # device-side seqlock validation (flag read by the fused
            # optimizer) when every peer header can be mapped for the GPU
            self.ok = torch.ones(1, dtype=torch.int32, device=flat.device)
            self.torn = torch.zeros(1, dtype=torch.int32, device=flat.device)
            self.device_check = all(self.hdr.device_word(r, 0) is not None
                                    for r in range(self.size) if r != self.rank)
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
                    with warnings.catch_warnings():  # read-only map, never written
                        warnings.simplefilter("ignore", UserWarning)
                        self.peer_slots[r] = torch.from_numpy(
                            np.memmap(p, dtype=np.float32, mode="r", shape=(2, n)))
            self.pull_stream = None
            self.device_check = False
        self.seq = [0, 0]
        self.latest = 0
        self.hdr.write(self.SEQ0, 0)
        self.hdr.write(self.SEQ1, 0)
        self.hdr.write(self.LATEST, 0)
        self._pending = None  # (slot, event) of a publish not yet committed
        self._writing = None  # slot the current update writes into
        self._inflight = None  # (peer, slot, seq, event, out) of a prefetch
        self.publishes = 0
        self.retries = 0
        comm.all_gather_object(True)

    # ------------------------------------------------------------ writer
    def _commit(self, wait: bool) -> bool:
        if self._pending is None:
            return True
        slot, ev = self._pending
        if ev is not None:
            if wait:
                ev.synchronize()
            elif not ev.query():
                return False
        self.seq[slot] += 1  # even: slot complete
        self.hdr.write(slot, self.seq[slot])
        self.latest = slot
        self.hdr.write(self.LATEST, slot)
        self._pending = None
        return True

    def poll(self):
        """Commit a completed publish without blocking."""
        self._commit(wait=False)

    def begin_publish(self) -> torch.Tensor:
        """The slot the coming update writes the new model into (the fused
        optimizer's ``wout``); marked in progress (odd) for readers."""
        if self._pending is not None and not self._commit(wait=False):
            slot = self._pending[0]  # still odd: rewrite it, commit later
            self._pending = None
        else:
            slot = 1 - self.latest
            self.seq[slot] += 1  # odd: write in progress on this slot
            self.hdr.write(slot, self.seq[slot])
        self._writing = slot
        return self.slots[slot]

    def end_publish(self):
        """The update writing the slot is enqueued (current stream);
        committed once it has completed."""
        slot, self._writing = self._writing, None
        ev = None
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        self._pending = (slot, ev)
        self.publishes += 1
        if ev is None:
            self._commit(wait=True)

    def abort_publish(self):
        """The update failed: the slot stays odd (never read) until the
        next publish rewrites it."""
        if self._writing is not None:
            self._pending = (self._writing, None)
            self._writing = None

    def publish(self, flat: torch.Tensor):
        """Copy ``flat`` into the next slot and commit it once written."""
        self.begin_publish().copy_(flat)
        self.end_publish()

    def flush(self):
        self._commit(wait=True)

    # ------------------------------------------------------------ reader
    def _snapshot_header(self, peer):
        for _ in range(self.MAX_TRIES):
            slot = self.hdr.read(peer, self.LATEST)
            v = self.hdr.read(peer, slot)
            if v % 2 == 0:
                return slot, v
        raise TornReadError("peer %d's latest slot stayed mid-write" % peer)

    def pull_values(self, peer: int) -> dict:
        """The per-step values of a pull of ``peer``'s latest committed model
        (launch tape: the recorded copy and seqlock check read them)."""
        slot, v = self._snapshot_header(peer)
        return {"pa_src": self.peer_slots[peer][slot],
                "pa_word": self.hdr.device_word(peer, slot) or 0, "pa_seq": v,
                "_pa": (peer, slot)}

    def begin_pull(self, peer: int, out: torch.Tensor, vals: Optional[dict] = None):
        """Start copying ``peer``'s latest committed model into ``out``
        (side stream on the GPU; the owner does not participate).  On the GPU
        every operation is a native call (recordable in a launch tape):
        stream waits, the device copy and the device-side seqlock check."""
        if not self.cuda:
            slot, v = self._snapshot_header(peer)
            out.copy_(self.peer_slots[peer][slot])
            self._inflight = (peer, slot, v, None, out)
            return
        from ..ops import _native as N
        vals = vals or self.pull_values(peer)
        ps = self.pull_stream.cuda_stream
        N.stream_wait(ps, N.stream(out.device))  # ``out`` is free to overwrite
        N.call("kfb_memcpy_d2d", out.data_ptr(), N.dyn("pa_src", vals["pa_src"]),
               out.numel() * out.element_size(), ps)
        if self.device_check:
            N.call("kfb_seqlock_check", N.dyn("pa_word", vals["pa_word"]),
                   N.dyn("pa_seq", vals["pa_seq"]), self.ok.data_ptr(), self.torn.data_ptr(), ps)
        # (finish_pull's host-side wait; the device-validated path orders the
        # consumer with a native stream wait instead)
        ev = torch.cuda.Event()
        ev.record(self.pull_stream)
        peer, slot = vals["_pa"]
        self._inflight = (peer, slot, vals["pa_seq"], ev, out)

    def finish_pull_async(self):
        """Device-validated pull: the current stream waits for the copy and
        its seqlock check; returns the device flag (1 = untorn) the fused
        optimizer gates the averaging on.  The host never blocks."""
        peer, slot, v, ev, out = self._inflight
        self._inflight = None
        from ..ops import _native as N
        N.stream_wait(N.stream(out.device), self.pull_stream.cuda_stream)
        return self.ok

    def finish_pull(self) -> int:
        """Wait for the prefetch, validate it against the seqlock (retrying
        synchronously if the slot was rewritten meanwhile); returns the
        accepted sequence number."""
        peer, slot, v, ev, out = self._inflight
        self._inflight = None
        for _ in range(self.MAX_TRIES):
            if ev is not None:
                ev.synchronize()
            if self.hdr.read(peer, slot) == v:
                if self.cuda:
                    torch.cuda.current_stream(out.device).wait_event(ev)
                return v
            self.retries += 1
            self.begin_pull(peer, out)
            peer, slot, v, ev, out = self._inflight
            self._inflight = None
        raise TornReadError("no untorn snapshot of peer %d after %d tries"
                            % (peer, self.MAX_TRIES))

    def pull(self, peer: int, out: torch.Tensor) -> int:
        self.begin_pull(peer, out)
        return self.finish_pull()

    def torn_count(self) -> int:
        """Snapshots rejected so far (host retries + device-side rejections)."""
        n = self.retries
        if self.cuda:
            n += int(self.torn.item())
        return n

    def close(self):
        if self._inflight is not None and self._inflight[3] is not None:
            self._inflight[3].synchronize()
        self._inflight = None
        if self._writing is not None:
            self.abort_publish()
        self.flush()
        self.hdr.close()
        if self.cuda and self._opened:
            torch.cuda.synchronize(self.device)
            for base in self._opened:
                close_mapping(base)
            self._opened = []
        if not self.cuda:
            try:
                os.remove(self.path)
            except OSError:
                pass


class PairAveraging(Strategy):
    name = "kungfu/async_sgd"

    def __init__(self, params, world, flat, **kw):
        super().__init__(params, world, flat, **kw)
        self.rng = random.Random(params.kungfu_peer_seed * 7919 + world.rank)
        self.lockstep = bool(getattr(params, "kungfu_pair_lockstep", False))
        self.prefetch = bool(getattr(params, "kungfu_pair_prefetch", True)) and not self.lockstep
        self.store = None
        self._peer_buf = None
        self._mix = None
        self._wout = None

    def broadcast_initial_model(self, slots=()):
        super().broadcast_initial_model(slots)
        if self.world.size > 1:
            self.store = ModelStore(self.flat.flat, self.world)
            self._peer_buf = torch.empty_like(self.flat.flat)

    def _pick_peer(self) -> int:
        peer = self.rng.randrange(self.world.size - 1)
        return peer + 1 if peer >= self.world.rank else peer

    def before_backward(self, step):
        super().before_backward(step)
        if self.store is None:
            return
        self.store.poll()
        if self.prefetch:
            # pull a random peer's model while forward/backward run
            self.store.begin_pull(self._pick_peer(), self._peer_buf)

    def before_update(self, step):
        if self.store is None:
            return
        if not self.prefetch:
            self.store.begin_pull(self._pick_peer(), self._peer_buf)
        if self.store.device_check:
            ok = self.store.finish_pull_async()
        else:
            self.store.finish_pull()
            ok = None
        if self.lockstep:
            # every worker holds its peer's step-t model before anyone
            # publishes step t+1's
            w = self.flat.flat
            if w.is_cuda:
                torch.cuda.synchronize(w.device)
            self.world.barrier(w.device if w.is_cuda else None)
        # w <- (w + w_peer) / 2 and the update in ONE pass, written straight
        # into the publish slot
        self._mix = (self._peer_buf, 0.5, 0.5, ok)
        self._wout = self.store.begin_publish()

    def fused_update(self):
        mix, wout = self._mix, self._wout
        self._mix = self._wout = None
        return mix, wout

    def after_update(self, step):
        if self.store is not None:
            self.store.end_publish()
            if self.lockstep:
                self.store.flush()  # committed: the next pulls see it
                w = self.flat.flat
                self.world.barrier(w.device if w.is_cuda else None)

    def abort_update(self, step):
        self._mix = self._wout = None
        if self.store is not None:
            self.store.abort_publish()

    # launch tape: the pull (copy + device seqlock check) and the update into
    # the publish slot are recorded native calls whose peer-slot address,
    # sequence word and publish slot are per-step values; the host halves
    # (peer choice, header snapshot, publish bookkeeping) run around a replay
    def steps_use_collectives(self):
        return False  # one-sided pulls over HIP IPC; no collective per step

    def tape_blocker(self):
        if self.world.size > 1 and not self.flat.flat.is_cuda:
            return "host-memory model store"
        if self.lockstep:
            return "lock-step PairAveraging synchronizes on the host"
        if self.store is not None and not self.store.device_check:
            return "peer headers not mappable for the device seqlock check"
        return None

    def tape_pre(self, step):
        if self.store is None:
            return {}
        self.store.poll()
        vals = self.store.pull_values(self._pick_peer())
        vals.pop("_pa")
        vals["wout"] = self.store.begin_publish().data_ptr()
        return vals

    def tape_post(self, step):
        if self.store is not None:
            self.store.end_publish()

    def close(self):
        """Collective: every rank stops reading before any slot is freed."""
        if self.store is not None:
            self.store.flush()
            w = self.flat.flat
            self.world.barrier(w.device if w.is_cuda else None)
            self.torn_snapshots = self.store.torn_count()
            self.store.close()
            self.store = None
