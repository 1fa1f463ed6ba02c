"""Input sources feeding the hot loop.

* :class:`SyntheticInput` - on-device synthetic ImageNet-shaped batches
  (tcb/models/model.py:220-237).  Generated once and reused unless
  ``--synthetic_resample`` (the reference re-samples each step; values of
  synthetic data do not matter for the benchmark, and reuse keeps the RNG
  kernel out of the timed step).
* :class:`PrefetchInput` - real data: host preprocessing workers
  (:mod:`kf_benchmarks_amd.data.preprocessing`) produce NHWC uint8/float
  batches into pinned buffers; a copy stream moves them to the device one
  batch ahead (the StagingArea double buffering of tcb/benchmark_cnn.py:2527-2600).
"""

from __future__ import annotations

import queue
import threading
from typing import Optional

import numpy as np
import torch


def _mix32(*vals) -> int:
    """A 31-bit seed from integers (splitmix64 rounds): the synthetic streams
    of different (seed, rank, step) are independent, where consecutive
    integers would share draws (the label seed of one step used to be the
    image seed of the next, and ranks were 1000 steps apart)."""
    m = (1 << 64) - 1
    x = 0x9E3779B97F4A7C15
    for v in vals:
        x = (x ^ (int(v) & m)) & m
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & m
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & m
        x ^= x >> 31
    return x & 0x7FFFFFFE  # (even: the op draws labels from seed + 1)


class SyntheticInput:
    def __init__(self, bench, subset="train"):
        self.bench = bench
        model = bench.model
        nclass = bench.dataset.num_classes
        self.resample = bench.params.synthetic_resample
        self.base = (bench.params.tf_random_seed, bench.task_index)
        self.step = 0
        self.inputs = tuple(model.get_synthetic_inputs("input", nclass, bench.device,
                                                       self.seed_at(0)))

    def seed_at(self, step: int) -> int:
        """The images' seed of ``step`` (labels: + 1) on this rank."""
        return _mix32(*self.base, step)

    def next(self):
        if self.resample:
            self.step += 1
            model = self.bench.model
            self.inputs = tuple(model.get_synthetic_inputs(
                "input", self.bench.dataset.num_classes, self.bench.device,
                self.seed_at(self.step)))
        return self.inputs

    # launch tape: a replayed step re-samples the batch with the seeds an
    # eager step would use
    def tape_advance(self):
        if self.resample:
            self.step += 1

    def tape_values(self):
        s = self.seed_at(self.step)
        return {"input_seed": s & 0xFFFFFFFF, "input_seed_labels": (s + 1) & 0xFFFFFFFF}

    def tape_post(self):
        pass

    def close(self):
        pass


class FakeDataInput:
    """Cycles through a user-provided numpy batch set (tests; the
    TestImagePreprocessor.set_fake_data of tcb/preprocessing.py:896-974).
    Images are normalized like real data (x / 127.5 - 1); each worker starts
    at shift_ratio = rank / num_workers of the data, as in the reference."""

    def __init__(self, bench, images, labels):
        import numpy as np
        from .. import cnn_util
        self.bench = bench
        bs = bench.local_batch_size
        shift = bench.task_index / float(max(bench.num_replicas, 1))
        imgs = cnn_util.roll_numpy_batches(np.asarray(images, dtype=np.float32), bs, shift)
        labs = cnn_util.roll_numpy_batches(np.asarray(labels), bs, shift)
        self.images = torch.from_numpy(imgs / 127.5 - 1.0).to(bench.device, bench.compute_dtype)
        self.labels = torch.from_numpy(labs.astype("int32")).to(bench.device)
        self.n = imgs.shape[0] // bs
        self.i = 0

    def next(self):
        bs = self.bench.local_batch_size
        k = self.i % self.n
        self.i += 1
        return (self.images[k * bs:(k + 1) * bs].contiguous(),
                self.labels[k * bs:(k + 1) * bs].contiguous())

    def close(self):
        pass


class PrefetchInput:
    """Pulls host batches from a preprocessor generator on a thread, copies
    them to the device on a side stream, one batch ahead.

    ``batch_group_size`` > 1 (--batch_group_size): the host side runs as the
    reference's ImageProducer (tcb/cnn_util.py:118-198, wired at
    tcb/benchmark_cnn.py:2139-2146): batches are staged in groups of that
    many, at most two groups ahead of the consumer, which reports every
    consumed batch."""

    def __init__(self, bench, batch_iter, depth: int = 2, batch_group_size: int = 1):
        self.bench = bench
        self.device = bench.device
        self.dtype = bench.compute_dtype
        self._it = batch_iter
        self._stop = threading.Event()
        self._err: Optional[BaseException] = None
        self._stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._next = None
        self._last = self._tape_bufs = None
        self.producer = None
        if batch_group_size > 1:
            from ..cnn_util import ImageProducer
            self._q: "queue.Queue" = queue.Queue()  # bounded by the producer
            self._ended = False
            self.producer = ImageProducer(self._put_one, batch_group_size)
            self.producer.start()
        else:
            self._q = queue.Queue(maxsize=max(depth, 1))
            self._thread = threading.Thread(target=self._run, daemon=True)
            self._thread.start()

    def _host(self, batch):
        from .preprocessing import JpegBatch
        if isinstance(batch, JpegBatch):
            return batch  # (already in pinned ring buffers)
        ts = [torch.from_numpy(np.ascontiguousarray(x)) for x in batch]
        if self.device.type == "cuda":
            ts = [t.pin_memory() for t in ts]
        return ts

    def _put_one(self):
        """ImageProducer put_fn: stage one batch (or the end marker)."""
        if self._ended:
            self._stop.wait(0.05)
            return
        try:
            self._q.put(self._host(next(self._it)))
        except StopIteration:
            self._ended = True
            self._q.put(None)
        except BaseException as e:
            self._ended = True
            self._err = e
            self._q.put(None)

    def _run(self):
        try:
            for batch in self._it:
                if self._stop.is_set():
                    return
                self._q.put(self._host(batch))
            self._q.put(None)
        except BaseException as e:
            self._err = e
            self._q.put(None)

    def _to_device(self, ts):
        from .preprocessing import JpegBatch
        if isinstance(ts, JpegBatch):
            # coefficient blocks -> JPEG reconstruction + resize on the device
            # (csrc/jpeg.hip), then the flip / colour / scaling pass
            from ..ops import jpeg as J
            from ..ops import nn as F
            s, dev = ts.slot, self.device
            descs = s.descs.to(dev, non_blocking=True)
            blocks = s.blocks[:ts.nblocks].to(dev, non_blocking=True)
            hosted = s.images.to(dev, non_blocking=True) if ts.hosted else None
            prm = s.params.to(dev, non_blocking=True)
            lab = s.labels.to(dev, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            s.release(ev)  # the slot may be refilled once these copies are done
            u8 = J.decode(descs, blocks, hosted, ts.n, ts.height, ts.width, ts.crop_pixels)
            return [F.augment_u8(u8, prm, self.dtype), lab]
        img = ts[0].to(self.device, non_blocking=True)
        if len(ts) == 3 and img.dtype == torch.uint8:
            # (uint8 images, labels, augmentation params): flip, colour
            # distortions and [-1, 1] scaling on the device (csrc/augment.hip)
            from ..ops import nn as F
            prm = ts[2].to(self.device, non_blocking=True)
            lab = ts[1].to(self.device, non_blocking=True)
            return [F.augment_u8(img, prm, self.dtype),
                    lab.to(torch.int32) if lab.dtype == torch.int64 else lab]
        if img.dtype == torch.uint8:
            # raw pixels: normalize on the device (x / 127.5 - 1)
            img = img.to(torch.float32).mul_(1.0 / 127.5).sub_(1.0)
        out = [img.to(self.dtype)]
        for t in ts[1:]:
            t = t.to(self.device, non_blocking=True)
            out.append(t.to(torch.int32) if t.dtype == torch.int64 else t)
        return out

    def _fetch(self):
        item = self._q.get()
        if self.producer is not None and item is not None:
            self.producer.notify_image_consumption()
        if item is None:
            if self._err is not None:
                raise RuntimeError("input pipeline failed") from self._err
            raise StopIteration("input exhausted")
        if self._stream is not None:
            with torch.cuda.stream(self._stream):
                out = self._to_device(item)
                ev = torch.cuda.Event()
                ev.record(self._stream)
            return out, ev
        return self._to_device(item), None

    # ---------------------------------------------------------- launch tape
    # A taped step starts with native copies of the current batch (its device
    # addresses per-step values) into buffers the tape owns, behind a
    # recorded wait on the copy stream; the batch after it is fetched between
    # replays (tape_post), so the recorded wait covers only this batch's
    # copy / decode / augmentation work.
    def tape_capable(self) -> bool:
        return self._stream is not None

    def _tape_next(self):
        from ..ops import _native as N
        if self._next is None:
            self._next = self._fetch()
        out, _ = self._next
        self._next = None
        cur = torch.cuda.current_stream(self.device)
        for t in out:
            t.record_stream(cur)
        self._cur = out
        N.stream_wait(cur.cuda_stream, self._stream.cuda_stream)
        bufs = []
        for i, t in enumerate(out):
            b = torch.empty_like(t)
            N.call("kfb_memcpy_d2d", b.data_ptr(), N.dyn("input_%d" % i, t.data_ptr()),
                   t.numel() * t.element_size(), cur.cuda_stream)
            bufs.append(b)
        self._tape_bufs = self._last = tuple(bufs)
        return tuple(bufs)

    def consumed(self):
        """The device tensors the last step's forward read: the tape-owned
        copies (which every replay refills) once a tape was recorded, the
        fetched batch in an eager step (tests compare their contents)."""
        return self._last

    def tape_advance(self):
        if self._next is None:
            self._next = self._fetch()
        out, _ = self._next
        self._next = None
        cur = torch.cuda.current_stream(self.device)
        for t in out:
            t.record_stream(cur)
        self._cur = out
        self._last = self._tape_bufs

    def tape_values(self):
        return {"input_%d" % i: t.data_ptr() for i, t in enumerate(self._cur)}

    def tape_post(self):
        """Prefetch the next batch (after the taped step was enqueued)."""
        if self._next is None:
            try:
                self._next = self._fetch()
            except StopIteration:
                self._exhausted = True

    def next(self):
        from ..ops import _native as N
        if N.recording() and self._stream is not None:
            return self._tape_next()
        if self._next is None:
            self._next = self._fetch()
        out, ev = self._next
        if ev is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            for t in out:
                t.record_stream(cur)
        self._last = tuple(out)
        try:
            self._next = self._fetch()
        except StopIteration:
            self._next = None
            self._exhausted = True
        return tuple(out)

    def close(self):
        """Stops the producer and closes the batch generator (its native
        worker pool) before the process exits: a producer thread left inside
        a native call or a pinned-memory copy at interpreter shutdown can
        abort the process."""
        self._stop.set()
        if self.producer is not None:
            self.producer.done()
            try:
                while True:
                    _drop(self._q.get_nowait())
            except queue.Empty:
                pass
            return
        t = getattr(self, "_thread", None)
        for _ in range(100):  # unblock a put on a full queue until the producer sees _stop
            if t is None or not t.is_alive():
                break
            try:
                while True:
                    _drop(self._q.get_nowait())
            except queue.Empty:
                pass
            t.join(timeout=0.1)
        if t is None or not t.is_alive():
            close = getattr(self._it, "close", None)
            if close is not None:
                try:
                    close()  # generator finally: the native pipe's threads are joined
                except Exception:  # noqa: BLE001 - best effort at shutdown
                    pass


def _drop(item):
    """A queued batch that will never be copied: its pinned ring slot (GPU
    JPEG path) goes back to the producer."""
    slot = getattr(item, "slot", None)
    if slot is not None:
        slot.release()


def make_input_source(bench, subset="train"):
    fake = getattr(bench, "fake_data", None)
    if fake is not None:
        return FakeDataInput(bench, *fake)
    if bench.dataset.use_synthetic_gpu_inputs():
        return SyntheticInput(bench, subset)
    from . import preprocessing
    it = preprocessing.make_batch_iterator(bench, subset)
    return PrefetchInput(bench, it, depth=max(bench.params.datasets_prefetch_buffer_size, 1) + 1,
                         batch_group_size=max(int(bench.params.batch_group_size or 1), 1))
