"""Bucketed gradient all-reduce overlapped with backward.

Gradients live in one flat fp32 buffer ordered by the order they become
ready in backward (:class:`kf_benchmarks_amd.optim.FlatParams`), so a bucket
is a contiguous slice: no pack/unpack kernels (the reference's
pack_small_tensors / gradient_repacking / allreduce_merge_scope machinery,
tcb/allreduce.py:420-588, tcb/batch_allreduce.py:391-481, exists to build
exactly such contiguous buffers).

Each parameter's post-accumulate-grad hook counts its bucket down; a full
bucket is handed to RCCL immediately (async), so communication of the late
layers overlaps the backward of the early ones.  Buckets are always launched
in index order so every rank issues the same collective sequence.

Bucket size: RCCL over xGMI uses a ring per channel across the 7 links of
each MI355X; per-message latency is ~10-30 us, so buckets of tens of MB keep
the links busy while leaving enough buckets (ResNet-50: 102 MB fp32 -> 4 at
25 MB) to overlap with backward.  ``--gradient_wire_dtype=bf16|fp16`` halves
the bytes on the wire (the reference's --compact_gradient_transfer).

``num_buckets`` (``--gradient_repacking=k``) splits the flat gradient into k
equal buckets instead of size-capped ones; ``spec`` (the parsed
``--all_reduce_spec``) picks per bucket size the collective algorithm and
the number of concurrent pieces (``alg#shards``), see
:mod:`kf_benchmarks_amd.parallel.allreduce`; ``relaxed`` (``--variable_consistency=relaxed``) defers the
gradients by one step: step t's reduction runs while step t+1 computes, and
step t applies step t-1's result (zeros at the first step), as the
StagingArea deferral of tcb/batch_allreduce.py:353-389.
"""

from __future__ import annotations

import os
from typing import List, Optional

import torch

from . import allreduce, comm


def _unwire(view, buf):
    """The reduced low-precision wire slice back into the fp32 gradient."""
    if view.is_cuda:
        from ..ops import _native as N
        N.call("kfb_cast_to_f32", buf.data_ptr(), N.dt(buf), view.data_ptr(), view.numel(),
               N.stream(view.device))
    else:
        view.copy_(buf)


class BucketReducer:
    def __init__(self, flat, bucket_mb: float = 25.0, wire_dtype: Optional[torch.dtype] = None,
                 overlap: bool = True, op: str = "sum", group=None, num_buckets: int = 0,
                 relaxed: bool = False, shards: int = 1, spec=None, hierarchical=None,
                 tail_mb: Optional[float] = None):
        self.flat = flat
        if tail_mb is None:
            tail_mb = float(os.environ.get("KFB_BUCKET_TAIL_MB", "2"))
        self.wire_dtype = wire_dtype if wire_dtype not in (None, torch.float32) else None
        self.op = op
        self.group = group
        self.shards = max(int(shards), 1)
        self.spec = spec  # [AllReduceSpecTuple] or None
        self.world_size = comm.get_world().size
        self.hierarchical = hierarchical  # allreduce.Hierarchical or None
        self.relaxed = bool(relaxed)
        self._stash = None
        self._stash_works = None
        self._relaxed_step = 0
        self.deferred_empty = False
        if relaxed:
            overlap = False
        if num_buckets and num_buckets > 0:
            limit = max((flat.numel + num_buckets - 1) // num_buckets, 1)
        else:
            limit = max(int(bucket_mb * (1 << 20) / 4), 1)
        self.buckets: List[List[int]] = []  # [start, end) in elements
        self.param_bucket = {}
        segs = flat.segments()
        # Buckets are cut from the END of the ready order: the last bucket only
        # launches once backward is over, so its all-reduce is exposed.  Caps
        # grow geometrically from ``tail_mb`` (the last bucket) up to the
        # bucket size, so the exposed tail is a few MB (ResNet-50 fp32: 2, 4,
        # 8, 16, 25, 25 MB and a 22 MB head instead of 29/26/26/17 MB).
        tail = int(tail_mb * (1 << 20) / 4) if (tail_mb and not num_buckets) else 0
        span = [(segs[i + 1][2] if i + 1 < len(segs) else flat.numel) - segs[i][2]
                for i in range(len(segs))]
        groups, cur, size, j = [], [], 0, 0
        for i in reversed(range(len(segs))):
            cur.append(i)
            size += span[i]
            cap = min(limit, tail << j) if tail > 0 else limit
            if size >= max(cap, 1):
                groups.append(cur)
                cur, size, j = [], 0, j + 1
        if cur:
            groups.append(cur)
        groups = [sorted(g) for g in reversed(groups)]
        for gi, g in enumerate(groups):
            start = segs[0][2] if gi == 0 else segs[g[0]][2]
            end = segs[groups[gi + 1][0]][2] if gi + 1 < len(groups) else flat.numel
            b = len(self.buckets)
            self.buckets.append([start, end])
            for i in g:
                self.param_bucket[id(segs[i][1])] = b
        self.sizes = [sum(1 for v in self.param_bucket.values() if v == b)
                      for b in range(len(self.buckets))]
        self._pending = list(self.sizes)
        self._ready = [False] * len(self.buckets)
        self._arrived = set()
        self._next = 0
        self._works = []
        self._active = False
        self.overlap = overlap
        # persistent wire-dtype staging (one per in-flight step: relaxed mode
        # has the previous step's reduction outstanding while it launches)
        self._wire = [None, None]
        self.launch_count = 0  # collectives issued (tests, all_reduce_benchmark)
        # exposed-communication probe (bench.py): per step, a native timing
        # event when the backward's kernels are done (both streams) and one
        # when the compute stream may use the reduced gradients; their
        # distance is the all-reduce time backward did not hide.  Both are
        # native calls, so a recorded launch tape replays them (each replay
        # fills the next slot of the timer's ring); two event records per step.
        self.timing = False  # (kept for callers; the probe always runs)
        self.probe = True
        self._timer = None
        self._timing_events = []  # CPU runs: none
        self._handles = []
        if overlap:
            for _, p, _, _ in segs:
                self._handles.append(p.register_post_accumulate_grad_hook(self._hook))
                # kernels that write the flat gradient directly notify through this
                p._kfb_ready_cb = self._hook

    @property
    def num_buckets(self):
        return len(self.buckets)

    def begin(self):
        """Arm the hooks for one backward pass."""
        self._arrived = set()
        self._pending = list(self.sizes)
        self._ready = [False] * len(self.buckets)
        self._next = 0
        self._works = []
        self._active = True

    def _hook(self, p):
        if not self._active:
            return
        b = self.param_bucket.get(id(p))
        if b is None:
            return
        # A parameter whose kernel writes the flat gradient directly reports
        # through _kfb_ready_cb, and autograd then still runs its (empty)
        # AccumulateGrad post-hook: count each parameter once per backward, or
        # a bucket would launch while half its gradients are still unwritten.
        if id(p) in self._arrived:
            return
        self._arrived.add(id(p))
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._ready[b] = True
            while self._next < len(self.buckets) and self._ready[self._next]:
                self._launch(self._next)
                self._next += 1

    def _launch(self, b, src=None):
        g = self.flat.grad if src is None else src
        ctx = None
        if g.is_cuda:
            # A bucket holds gradients written on the compute stream (BN,
            # affine) and on the weight-gradient side stream (convs).  The
            # collective is issued FROM the side stream after it has caught
            # up with the compute stream, so RCCL waits for both while the
            # compute (dgrad) stream itself never waits for the side stream.
            from ..ops.conv_hip import wgrad_stream
            side = wgrad_stream(g.device)
            cur = torch.cuda.current_stream(g.device)
            if side is not None and side != cur:
                from ..ops import _native as N
                N.stream_wait(side.cuda_stream, cur.cuda_stream)  # recordable
                ctx = torch.cuda.stream(side)
        if ctx is None:
            self._launch_on_current(b, g)
        else:
            with ctx:
                self._launch_on_current(b, g)

    def _launch_on_current(self, b, g):
        s, e = self.buckets[b]
        view = g[s:e]
        if self.wire_dtype is not None:
            k = self._relaxed_step % 2 if self.relaxed else 0
            if self._wire[k] is None or self._wire[k].device != g.device:
                self._wire[k] = torch.empty(g.numel(), dtype=self.wire_dtype, device=g.device)
            buf = self._wire[k][s:e]
            if buf.is_cuda:  # native cast: recordable in a launch tape
                from ..ops import _native as N
                N.call("kfb_cast_f32", view.data_ptr(), buf.data_ptr(), N.dt(buf), view.numel(),
                       N.stream(view.device))
            else:
                buf.copy_(view)
        else:
            buf = view
        if self.spec:
            alg = allreduce.algorithm_for(self.spec, e - s)
            name, shards = alg.alg, max(alg.shards, 1)
        else:
            name, shards = "nccl", self.shards
        pieces = torch.tensor_split(buf, shards) if shards > 1 else (buf,)
        for piece in pieces:
            self.launch_count += 1
            works = allreduce.launch_collective(comm, piece, name, b, self.world_size, self.op,
                                                self.hierarchical)
            self._works.append((works, None, None))
        self._works[-1] = (self._works[-1][0], buf, view)

    def _finish_relaxed(self):
        """Apply last step's reduced gradients; start reducing this step's."""
        g = self.flat.grad
        if self._stash is None:
            self._stash = [torch.empty_like(g), torch.empty_like(g)]
        cur = self._stash[self._relaxed_step % 2]
        cur.copy_(g)
        prev_works = self._stash_works
        self._works = []
        for b in range(len(self.buckets)):
            self._launch(b, src=cur)
        self._stash_works = self._works
        self._works = []
        self.deferred_empty = prev_works is None
        if prev_works is None:
            g.zero_()  # first step: nothing reduced yet
        else:
            for works, buf, view in prev_works:
                for work in works:
                    work.wait()
                if buf is not None and buf is not view:
                    _unwire(view, buf)
            g.copy_(self._stash[(self._relaxed_step - 1) % 2])
        self._relaxed_step += 1
        self._active = False

    def close(self):
        """Releases the reducer's own communicators (hierarchical subgroups)
        and the probe's events."""
        if self.hierarchical is not None:
            self.hierarchical.close()
        if self._timer is not None:
            from ..ops import _native as N
            N.load().kfb_event_timer_free(self._timer)
            self._timer = None

    def finish(self):
        """Launch whatever did not fire (unused params, overlap off) and make
        the current stream wait for every bucket."""
        if self.relaxed:
            self._finish_relaxed()
            return
        probe = self.probe and self.flat.grad.is_cuda
        if probe:
            self._mark_backward_done()
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        for works, buf, view in self._works:
            for work in works:
                work.wait()
            if buf is not None and buf is not view:
                _unwire(view, buf)
        if probe:
            from ..ops import _native as N
            dev = self.flat.grad.device
            N.call("kfb_event_timer_mark", self._probe_timer(dev), 1, N.stream(dev))
        self._works = []
        self._active = False

    _PROBE_SLOTS = 4096

    def _probe_timer(self, dev):
        if self._timer is None:
            import ctypes
            from ..ops import _native as N
            h = ctypes.c_void_p()
            err = N.load().kfb_event_timer_new(self._PROBE_SLOTS, ctypes.byref(h))
            if err != 0:
                raise N.NativeError("kfb_event_timer_new failed with hipError %d" % err)
            self._timer = h.value
        return self._timer

    def _mark_backward_done(self):
        """Mark 0: the side stream (weight gradients) catches up with the
        compute stream, then records, so the event completes only once both
        streams' backward kernels have."""
        from ..ops import _native as N
        from ..ops.conv_hip import wgrad_stream
        g = self.flat.grad
        side = wgrad_stream(g.device)
        cur = N.stream(g.device)
        s = cur
        if side is not None and side.cuda_stream != cur:
            N.stream_wait(side.cuda_stream, cur)
            s = side.cuda_stream
        N.call("kfb_event_timer_mark", self._probe_timer(g.device), 0, s)

    def pop_exposed_ms(self) -> List[float]:
        """Exposed all-reduce milliseconds of every step since the last call,
        eager or replayed from a launch tape (synchronizes on the events)."""
        if self._timer is None:
            return []
        import ctypes
        from ..ops import _native as N
        buf = (ctypes.c_float * self._PROBE_SLOTS)()
        n = N.load().kfb_event_timer_read(self._timer, buf, self._PROBE_SLOTS)
        return [float(buf[i]) for i in range(max(n, 0))]

    def reduce_now(self):
        """Synchronous all-reduce of the whole gradient (no backward hooks)."""
        self.begin()
        self.finish()

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []
        for _, p, _, _ in self.flat.segments():
            if getattr(p, "_kfb_ready_cb", None) == self._hook:
                p._kfb_ready_cb = None
